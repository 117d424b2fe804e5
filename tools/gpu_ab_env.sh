#!/bin/bash
# env A/B on the n=1000 C2 slice: tools/gpu_ab_env.sh VAR val1 val2 ...
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
var=$1; shift
mkdir -p gpurun_out/abenv
for v in "$@"; do
  env $var=$v timeout -k 10 300 python bench.py --n 1000 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/abenv/$var-$v.json 2> gpurun_out/abenv/$var-$v.err || { tail -5 gpurun_out/abenv/$var-$v.err; exit 1; }
  echo "$var=$v: $(grep per-kernel gpurun_out/abenv/$var-$v.err)"
done
