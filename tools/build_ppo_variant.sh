#!/bin/bash
# Like build_variant.sh, but recompiles only csrc/ppo.hip (the other objects
# from madrona-learn_amd/build, which `make` keeps current):
# tools/build_ppo_variant.sh <name> <flags...> -> variants/libmlearn_<name>.so
set -e
name=$1; shift
cd "$(dirname "$0")/../madrona-learn_amd"
mkdir -p build_var_$name variants
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -w "$@" -c csrc/ppo.hip -o build_var_$name/ppo.o
objs="build_var_$name/ppo.o"
for f in build/*.o; do [ "$(basename $f)" = ppo.o ] || objs="$objs $f"; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $objs -o variants/libmlearn_$name.so -L/opt/rocm/lib -lrccl
rm -rf build_var_$name
