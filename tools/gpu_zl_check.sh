#!/bin/bash
# z-step change gate: the GPU parity cases, then the n = 1000 A/B of the given abv/ variants
# (tools/gpu_zl_check.sh <tag> v1 v2 ...; the in-tree libccsc.so is what the tests load)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
tag=$1; shift
mkdir -p gpurun_out/$tag
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/$tag/pytest.txt 2>&1
rc=$?
tail -3 gpurun_out/$tag/pytest.txt
[ $rc -ne 0 ] && exit $rc
bash tools/gpu_ab_zl.sh "$@"
