#!/bin/bash
# build an A/B variant of libshud_rhs.so with extra -D flags for one translation unit (default: the packed element
# kernel, shud_ele_packed.hip; -tu ode: the integrator kernels, shud_ode_kernels.hip; -tu rhs: the runtime, shud_rhs.cpp; -tu odehost: the integrator controller, shud_ode.cpp):
#   tools/ablib.sh NAME [-tu ode] -DFOO=1 ...   ->  shud-up_amd/build/ab/libshud_rhs_NAME.so
set -e
cd "$(dirname "$0")/../shud-up_amd"
name=$1; shift
src=csrc/shud_ele_packed.hip; obj=shud_ele_packed.o
if [ "$1" = "-tu" ]; then
  case "$2" in
    ode) src=csrc/shud_ode_kernels.hip; obj=shud_ode_kernels.o ;;
    ele) ;;
    rhs) src=csrc/shud_rhs.cpp; obj=shud_rhs.o ;;
    odehost) src=csrc/shud_ode.cpp; obj=shud_ode.o ;;
    *) echo "unknown TU $2"; exit 2 ;;
  esac
  shift 2
fi
mkdir -p build/ab/$name
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -I../include -Icsrc"
/opt/rocm/bin/hipcc $F "$@" -c $src -o build/ab/$name/p.o
others=$(ls build/*.o | grep -v "/$obj")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o build/ab/libshud_rhs_$name.so build/ab/$name/p.o $others -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
