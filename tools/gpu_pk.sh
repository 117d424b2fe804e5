#!/bin/bash
# dense-lane 74-point prime pass (pack) vs pre-formed pairs only (pre): parity of the default build, same-box C4 / C5 A/B -> gpurun_out/pk/
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/pk
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread -k "fft2d or 4d or 3d or c4 or c5 or woodbury" > gpurun_out/pk/pytest.txt 2>&1 || { tail -30 gpurun_out/pk/pytest.txt; exit 1; }
tail -2 gpurun_out/pk/pytest.txt
bash tools/gpu_cfg_ab.sh C4 pre pack pre pack || exit 1
cp gpurun_out/cfgab/summary.txt gpurun_out/pk/c4.txt
bash tools/gpu_cfg_ab.sh C5 pre pack pre pack || exit 1
cp gpurun_out/cfgab/summary.txt gpurun_out/pk/c5.txt
cat gpurun_out/pk/c4.txt gpurun_out/pk/c5.txt
