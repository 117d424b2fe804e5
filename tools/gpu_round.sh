#!/bin/bash
# Round measurement call: the whole -m gpu suite, then the round profile
# (bench + rocprofv3 kernel stats + FETCH/WRITE PMC passes): tools/gpu_round.sh <tag>
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-r02}
mkdir -p gpurun_out/$tag
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > gpurun_out/$tag/pytest_gpu.txt 2>&1 || { tail -60 gpurun_out/$tag/pytest_gpu.txt; exit 1; }
tail -3 gpurun_out/$tag/pytest_gpu.txt
bash tools/round_profile.sh $tag
