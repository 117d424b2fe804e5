#!/bin/bash
# the full GPU suite on the current tree -> gpurun_out/<tag>/pytest_gpu.txt
set -o pipefail
tag=${1:-suite}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/$tag
python tools/check_lib.py || exit 1
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$tag/pytest_gpu.txt 2>&1 || { tail -30 gpurun_out/$tag/pytest_gpu.txt; exit 1; }
tail -2 gpurun_out/$tag/pytest_gpu.txt
