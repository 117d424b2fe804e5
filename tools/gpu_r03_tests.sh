#!/bin/bash
# Round-3 GPU test pass: the whole -m gpu suite (one process), log under gpurun_out/<tag>.
set -o pipefail
tag=${1:-r03_tests}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/$tag
mkdir -p $out
sel=${2:-tests}
timeout -k 10 1100 python -u -m pytest $sel -m gpu -v -rsP --timeout 300 --timeout-method thread \
    > $out/pytest_gpu.txt 2>&1
rc=$?
tail -5 $out/pytest_gpu.txt
exit $rc
