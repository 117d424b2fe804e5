#!/bin/bash
# C1 (1000 patches) with the two-stream z-phase on and off
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/c1s
for f in 1 0 1 0; do
  CCSC_ZSPLIT2=$f timeout -k 10 300 python3 -u tools/bench_configs.py --configs C1 --steps 3 > gpurun_out/c1s/c1_$f.jsonl 2>&1 || exit 1
  echo "split=$f $(grep config gpurun_out/c1s/c1_$f.jsonl | cut -c1-140)"
done
