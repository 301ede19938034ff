#!/bin/bash
# Experiment build of the fused loop: recompile denoise.hip with extra -D flags, link it with the main build's other
# objects -> normal-guided-pointcloud-denoiser_amd/libpcd_<name>.so (load with PCD_LIB; tools/ab_bench.sh <name>).
# usage: tools/build_variant.sh <name> "<flags>"
set -e
name=$1; flags=$2
cd "$(dirname "$0")/../normal-guided-pointcloud-denoiser_amd/csrc"
make -s -j4 >/dev/null            # the main build's objects are current
mkdir -p build_$name
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -Wall -Wno-unused-function \
  -I../../include -munsafe-fp-atomics $flags -c denoise.hip -o build_$name/denoise.o
objs=""
for o in build/*.o; do b=$(basename $o); [ "$b" = denoise.o ] && objs="$objs build_$name/denoise.o" || objs="$objs $o"; done
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o ../libpcd_$name.so $objs -L/opt/rocm/lib -lamdhip64 -lrccl -Wl,-rpath,/opt/rocm/lib
echo "built libpcd_$name.so ($flags)"
