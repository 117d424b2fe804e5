#!/bin/bash
# z-step variant A/B on the n = 1000 C2 slice: tools/gpu_ab_zl.sh v1 v2 ... (abv/libccsc_<v>.so)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/ab
bash tools/ab_bench.sh abv "$@" || exit 1
for v in "$@"; do echo "$v: $(grep per-kernel gpurun_out/ab/$v.err | cut -c1-120)"; done
