#!/bin/bash
# one-off round-2 measurement call: new tol parity tests, gram/chol ablation, SQ pass,
# full round profile
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "tol or zline" -x -v --timeout 120 --timeout-method thread > gpurun_out/tol_tests.log 2>&1 || { tail -40 gpurun_out/tol_tests.log; exit 1; }
tail -3 gpurun_out/tol_tests.log
bash tools/ab_bench.sh abv base nogram nochol || exit 1
cp abv/libccsc_base.so ccsc_code_iccv2017_amd/libccsc.so
grep -h per-kernel gpurun_out/ab/*.err
bash tools/sq_profile.sh zl1 || exit 1
bash tools/round_profile.sh r02a || exit 1
