#!/bin/bash
# GPU iteration: parity tests, short bench, full C2 bench (no CPU baseline).
#   tools/gpu_iter.sh <tag> [quick]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-it}; out=gpurun_out/$tag; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || { tail -40 $out/tests.log; exit 1; }
tail -2 $out/tests.log
timeout -k 10 300 python bench.py --n 1000 --steps 2 --warmup 1 --no-cpu-baseline > $out/b1k.json 2> $out/b1k.err || { tail -20 $out/b1k.err; exit 1; }
grep per-kernel $out/b1k.err
[ "$2" = quick ] && exit 0
timeout -k 10 600 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > $out/bfull.json 2> $out/bfull.err || { tail -20 $out/bfull.err; exit 1; }
grep -E "per-kernel|objective" $out/bfull.err; cat $out/bfull.json
