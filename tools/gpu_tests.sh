#!/bin/bash
# GPU tests (the whole -m gpu suite, or a selection): tools/gpu_tests.sh <tag> [pytest args...]
# log: gpurun_out/tests_<tag>.log; TESTS_TIMEOUT (s, default 900) bounds the run
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
tag=$1; shift
mkdir -p gpurun_out
timeout -k 10 ${TESTS_TIMEOUT:-900} python -u -m pytest -m gpu -x -v -s --timeout 240 --timeout-method thread "$@" > gpurun_out/tests_$tag.log 2>&1 || { tail -60 gpurun_out/tests_$tag.log; exit 1; }
tail -3 gpurun_out/tests_$tag.log
