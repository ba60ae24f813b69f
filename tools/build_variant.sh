#!/bin/bash
# A/B library variant: recompile ONE source with extra flags and link it with
# the in-tree objects of the others into ab/libpardis_<name>.so (bench it with
# PYPARDIS_LIB / tools/gpu_ab_lib.sh).
#   bash tools/build_variant.sh <name> <source.hip> "<extra hipcc flags>"
set -e
cd "$(dirname "$0")/.."
name=$1; src=$2; flags=$3
obj=pypardis_amd/csrc/_obj
mkdir -p ab /tmp/pd_variant_$name
base=$(basename "$src" .hip)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off -fno-fast-math \
    -Wall -Wno-unused-result -Iinclude $flags -c pypardis_amd/csrc/$base.hip -o /tmp/pd_variant_$name/$base.o
objs=$(ls $obj/*.o | grep -v "/$base.o$")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ab/libpardis_$name.so $objs \
    /tmp/pd_variant_$name/$base.o -L/opt/rocm/lib -lrccl
echo "built ab/libpardis_$name.so"
