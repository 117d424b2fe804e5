#!/bin/bash
# 3D plane kernels' dense-lane prime pass with two output pairs per task (q2) vs three (cur):
# parity of q2, same-box C4 A/B -> gpurun_out/q2/
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/q2
cp ccsc_code_iccv2017_amd/libccsc.so /tmp/libccsc_keep0.so && cp abx/libccsc_q2.so ccsc_code_iccv2017_amd/libccsc.so || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread -k "3d or c4" > gpurun_out/q2/pytest.txt 2>&1 || { tail -30 gpurun_out/q2/pytest.txt; exit 1; }
tail -2 gpurun_out/q2/pytest.txt
cp /tmp/libccsc_keep0.so ccsc_code_iccv2017_amd/libccsc.so || exit 1
bash tools/gpu_cfg_ab.sh C4 cur q2 cur q2 || exit 1
cp gpurun_out/cfgab/summary.txt gpurun_out/q2/c4.txt
cat gpurun_out/q2/c4.txt
