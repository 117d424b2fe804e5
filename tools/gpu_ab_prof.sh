#!/bin/bash
# same-box A/B with rocprofv3 kernel stats at full C2 (one outer iteration):
#   tools/gpu_ab_prof.sh v1 v2 ...  (abv/libccsc_<v>.so)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/abp
for v in "$@"; do
  cp abv/libccsc_$v.so ccsc_code_iccv2017_amd/libccsc.so
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/abp/$v -o $v -- python3 bench.py --steps 2 --warmup 0 --no-cpu-baseline > gpurun_out/abp/$v.log 2>&1 || { tail -5 gpurun_out/abp/$v.log; exit 1; }
  find gpurun_out/abp/$v -name "*kernel_trace.csv" -delete
  python3 tools/kstats.py $(find gpurun_out/abp/$v -name "*kernel_stats.csv") $v
done
