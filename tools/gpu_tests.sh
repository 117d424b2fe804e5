#!/bin/bash
# GPU tests subset: tools/gpu_tests.sh <tag> [pytest args...]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
tag=$1; shift
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -m gpu -x -v --timeout 180 --timeout-method thread "$@" > gpurun_out/tests_$tag.log 2>&1 || { tail -60 gpurun_out/tests_$tag.log; exit 1; }
tail -3 gpurun_out/tests_$tag.log
