#!/bin/bash
# 74-point prime pass with pre-formed input pairs: parity of the default build (pre), then
# same-box C4 / C5 A/B of base (plain radix-2 pass), pre, qp4 -> gpurun_out/pfa/
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/pfa
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread -k "fft2d or 4d or 3d or c4 or c5 or woodbury" > gpurun_out/pfa/pytest.txt 2>&1 || { tail -30 gpurun_out/pfa/pytest.txt; exit 1; }
tail -2 gpurun_out/pfa/pytest.txt
bash tools/gpu_cfg_ab.sh C4 base pre qp4 base pre qp4 || exit 1
cp gpurun_out/cfgab/summary.txt gpurun_out/pfa/c4.txt
bash tools/gpu_cfg_ab.sh C5 base pre qp4 base pre qp4 || exit 1
cp gpurun_out/cfgab/summary.txt gpurun_out/pfa/c5.txt
cat gpurun_out/pfa/c4.txt gpurun_out/pfa/c5.txt
