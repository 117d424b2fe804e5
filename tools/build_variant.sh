#!/bin/bash
# tools/build_variant.sh <name> <src.hip> [hipcc -D flags...]: rebuild one source with extra
# flags and link variants/libccsc_<name>.so from the in-tree objects (A/B and ablation runs).
set -e
name=$1; src=$2; shift 2
cd "$(dirname "$0")/.."
mkdir -p ${VARDIR:-variants} build/var
base=$(basename $src)
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function "$@" -c ccsc_code_iccv2017_amd/csrc/$src -o build/var/${base}.${name}.o
objs=$(ls build/obj/*.o | grep -v "/${base}.o$")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o ${VARDIR:-variants}/libccsc_${name}.so $objs build/var/${base}.${name}.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
echo ${VARDIR:-variants}/libccsc_${name}.so
