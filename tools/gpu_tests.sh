#!/bin/bash
# selected GPU tests on the current tree: tools/gpu_tests.sh <tag> <pytest -k expression> [files...]
# -> gpurun_out/<tag>/pytest.txt
set -o pipefail
tag=$1; expr=$2; shift 2
files=${*:-tests}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/$tag
timeout -k 10 1100 python -u -m pytest $files -m gpu -x -v -k "$expr" --timeout 300 --timeout-method thread > gpurun_out/$tag/pytest.txt 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/$tag/pytest.txt | tail -40
exit $rc
