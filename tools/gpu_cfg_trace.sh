#!/bin/bash
# Per-dispatch kernel traces of single configs (one warm-up + one timed outer iteration),
# summarised per kernel and grid size on the box: tools/gpu_cfg_trace.sh <tag> C4 C5 ...
# -> gpurun_out/<tag>/<C>_dispatch.txt ; also runs tools/rate_probe (fp64 pipe rates) when built
set -o pipefail
tag=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/$tag
mkdir -p $out
if [ -x tools/rate_probe ]; then timeout -k 10 60 tools/rate_probe > $out/rate_probe.txt 2>&1 || exit $?; fi
for c in "$@"; do
  timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d $out/tr_$c -o $c -- python3 -u tools/bench_configs.py --configs $c --steps 1 > $out/tr_$c.log 2>&1 || exit $?
  f=$(find $out/tr_$c -name "*kernel_trace.csv" | head -1)
  python3 tools/trace_dispatch.py $f > $out/${c}_dispatch.txt || exit $?
  rm -rf $out/tr_$c
done
echo done
