#!/bin/bash
# Per-config timings (C1, C3, C4, C5; seconds per outer iteration) and rocprofv3 kernel stats
# of C3, C4 and C5: tools/gpu_configs_prof.sh <tag>  -> gpurun_out/<tag>/
set -o pipefail
tag=${1:-cfg}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 600 python3 -u tools/bench_configs.py --configs C1,C3,C4,C5 --steps 2 > $out/configs.jsonl 2> $out/configs.err || exit $?
for c in C3 C4 C5; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $out/prof_$c -o $c -- python3 -u tools/bench_configs.py --configs $c --steps 2 > $out/prof_$c.log 2>&1 || exit $?
  f=$(find $out/prof_$c -name "*kernel_stats.csv" | head -1); cp $f $out/${c}_kernel_stats.csv
  rm -rf $out/prof_$c
done
cat $out/configs.jsonl
