#!/bin/bash
# build an A/B variant of libshud_rhs.so with extra -D flags for the packed element kernel:
#   tools/ablib.sh NAME -DFOO=1 ...   ->  shud-up_amd/build/ab/libshud_rhs_NAME.so
set -e
cd "$(dirname "$0")/../shud-up_amd"
name=$1; shift
mkdir -p build/ab/$name
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -I../include -Icsrc"
/opt/rocm/bin/hipcc $F "$@" -c csrc/shud_ele_packed.hip -o build/ab/$name/p.o
others=$(ls build/*.o | grep -v shud_ele_packed.o)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o build/ab/libshud_rhs_$name.so build/ab/$name/p.o $others -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
