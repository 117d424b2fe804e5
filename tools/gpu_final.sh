#!/bin/bash
# round-end evidence: the full GPU suite, then the round profile (bench + rocprofv3 + configs) -> gpurun_out/<tag>
set -o pipefail
tag=${1:-r05f}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/$tag
python tools/check_lib.py || exit 1
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$tag/pytest_gpu.txt 2>&1 || { tail -30 gpurun_out/$tag/pytest_gpu.txt; exit 1; }
tail -2 gpurun_out/$tag/pytest_gpu.txt
bash tools/gpu_profile_round.sh $tag || exit $?
echo final-done
