#!/bin/bash
# tools/build_full_variant.sh <name> [hipcc -D flags...]: every source rebuilt with extra
# flags into variants/libccsc_<name>.so (A/B of build-wide constants such as CCSC_NT).
set -e
name=$1; shift
cd "$(dirname "$0")/.."
mkdir -p variants build/fvar/$name
pids=()
for src in ccsc_code_iccv2017_amd/csrc/*.hip ccsc_code_iccv2017_amd/csrc/*.cpp; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function "$@" \
    -c $src -o build/fvar/$name/$(basename $src).o &
  pids+=($!)
done
for p in "${pids[@]}"; do wait $p; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o variants/libccsc_${name}.so build/fvar/$name/*.o \
  -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
echo variants/libccsc_${name}.so
