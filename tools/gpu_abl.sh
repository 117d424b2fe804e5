#!/bin/bash
# bench-only A/B of abx/ library variants at n = 1000 (ablation builds fail parity by design):
#   tools/gpu_abl.sh v1 v2 ...   (per-kernel lines -> gpurun_out/ab/summary.txt)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/ab
rm -f gpurun_out/ab/summary.txt
AB_N=${AB_N:-1000} bash tools/ab_bench.sh abx "$@" || exit 1
cut -c1-120 gpurun_out/ab/summary.txt
