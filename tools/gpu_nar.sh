#!/bin/bash
# C4 t-solve on 512-thread TC = 1 workgroups (nar, -DCCSC_TSOLVE_NARROW=1) vs 1024-thread TC = 2
# (wide, default build): parity of nar, same-box C4 A/B -> gpurun_out/nar/
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/nar
cp ccsc_code_iccv2017_amd/libccsc.so /tmp/libccsc_keep0.so && cp abx/libccsc_nar.so ccsc_code_iccv2017_amd/libccsc.so || exit 1
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread -k "3d or c4" > gpurun_out/nar/pytest.txt 2>&1 || { tail -30 gpurun_out/nar/pytest.txt; exit 1; }
tail -2 gpurun_out/nar/pytest.txt
cp /tmp/libccsc_keep0.so ccsc_code_iccv2017_amd/libccsc.so || exit 1
bash tools/gpu_cfg_ab.sh C4 wide nar wide nar || exit 1
cp gpurun_out/cfgab/summary.txt gpurun_out/nar/c4.txt
cat gpurun_out/nar/c4.txt
