#!/bin/bash
# tools/build_variant_multi.sh <name> "<src1.hip src2.hip ...>" [hipcc -D flags...]: rebuild several
# sources with extra flags and link abx/libccsc_<name>.so with the other in-tree objects (A/B runs
# of header-level switches that reach more than one translation unit).
set -e
name=$1; srcs=$2; shift 2
cd "$(dirname "$0")/.."
mkdir -p abx build/var/$name
pids=()
for s in $srcs; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function "$@" -c ccsc_code_iccv2017_amd/csrc/$s -o build/var/$name/$s.o &
  pids+=($!)
done
for p in "${pids[@]}"; do wait $p; done
objs=""
for o in build/obj/*.o; do
  b=$(basename $o .o)
  if [[ " $srcs " == *" $b "* ]]; then objs="$objs build/var/$name/$b.o"; else objs="$objs $o"; fi
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o abx/libccsc_$name.so $objs -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
echo abx/libccsc_$name.so
