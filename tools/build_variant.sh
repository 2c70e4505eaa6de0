#!/bin/bash
# Build a library variant with extra -D flags: tools/build_variant.sh <name> <flags...>
# -> madrona-learn_amd/variants/libmlearn_<name>.so (A/B runs via tools/variants.sh)
set -e
name=$1; shift
cd "$(dirname "$0")/../madrona-learn_amd"
mkdir -p build_var_$name variants
for f in csrc/*.hip; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -w "$@" -c $f -o build_var_$name/$(basename $f .hip).o &
done
wait; for f in build_var_$name/*.o; do :; done; [ $(ls build_var_$name/*.o | wc -l) -eq $(ls csrc/*.hip | wc -l) ] || { echo "variant build failed"; exit 1; }
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC build_var_$name/*.o -o variants/libmlearn_$name.so -L/opt/rocm/lib -lrccl
rm -rf build_var_$name
