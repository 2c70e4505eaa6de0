#!/bin/bash
# Per-kernel VGPR/AGPR/spill/occupancy summary of one HIP source (gfx950).
f=$1; shift
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 $EXTRA -fPIC -std=c++17 -c "$f" -o /tmp/_res.o -Rpass-analysis=kernel-resource-usage 2>&1 \
 | sed -n 's/.*remark: *//p' | sed 's/ \[-Rpass-analysis=kernel-resource-usage\]//' \
 | awk '/^Function Name/{name=$3} /^VGPRs:/{v=$2} /^AGPRs:/{a=$2} /^VGPRs Spill/{sp=$3} /^Occupancy/{o=$3; print o" waves/SIMD  vgpr="v" agpr="a" spill="sp"  "name}' | grep -E "${1:-.}" | c++filt | cut -c1-160
