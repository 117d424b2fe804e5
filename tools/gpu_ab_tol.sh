#!/bin/bash
# same-box A/B of C2 at tol = 1e-3: tools/gpu_ab_tol.sh v1 v2 ... (abv/libccsc_<v>.so)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/abt
for v in "$@"; do
  cp abv/libccsc_$v.so ccsc_code_iccv2017_amd/libccsc.so
  timeout -k 10 300 python bench.py --steps 2 --warmup 1 --tol 1e-3 --no-cpu-baseline > gpurun_out/abt/$v.json 2> gpurun_out/abt/$v.err || { tail -5 gpurun_out/abt/$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/abt/$v.json')); print('$v', round(d['ms_per_step'],1), 'ms/step', round(d['roofline']['avg_launch_ms'],1), 'ms z-step')"
done
