#!/bin/bash
# same-box A/B of whole C2 steps: tools/gpu_ab_step.sh v1 v2 ... (abv/libccsc_<v>.so);
# prints ms per step (2 timed outer iterations after 1 warm-up) and the per-kernel stats
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/abs
for v in "$@"; do
  cp abv/libccsc_$v.so ccsc_code_iccv2017_amd/libccsc.so
  timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/abs/$v.json 2> gpurun_out/abs/$v.err || { tail -5 gpurun_out/abs/$v.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/abs/$v.json')); print('$v', round(d['ms_per_step'],1), 'ms/step', round(d['value']), 'patch-iters/s')"
done
