#!/bin/bash
# Diagnostic library with in-kernel phase stamps (-DML_STAMPS); never the product .so.
set -e
cd "$(dirname "$0")/../madrona-learn_amd"
mkdir -p build_stamps variants
for f in csrc/*.hip; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -DML_STAMPS -w -c $f -o build_stamps/$(basename $f .hip).o &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC build_stamps/*.o -o variants/libmlearn_stamps.so -L/opt/rocm/lib -lrccl
