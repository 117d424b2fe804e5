#!/bin/bash
# variant A/B at full C2 (one outer iteration): tools/gpu_ab_full.sh v1 v2 ... (abv/libccsc_<v>.so)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/abf
for v in "$@"; do
  cp abv/libccsc_$v.so ccsc_code_iccv2017_amd/libccsc.so
  timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/abf/$v.json 2> gpurun_out/abf/$v.err || { tail -5 gpurun_out/abf/$v.err; exit 1; }
  echo "$v: $(grep per-kernel gpurun_out/abf/$v.err)"
done
