set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/gw
cp abx/libccsc_gw.so ccsc_code_iccv2017_amd/libccsc.so
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread -k "4d or 3d or C4 or C5 or c4 or c5 or woodbury" > gpurun_out/gw/pytest.txt 2>&1 || { tail -30 gpurun_out/gw/pytest.txt; exit 1; }
tail -2 gpurun_out/gw/pytest.txt
bash tools/gpu_cfg_ab.sh C5 base gw base gw || exit 1
cp gpurun_out/cfgab/summary.txt gpurun_out/gw/c5.txt
bash tools/gpu_cfg_ab.sh C4 base gw base gw || exit 1
cp gpurun_out/cfgab/summary.txt gpurun_out/gw/c4.txt
cat gpurun_out/gw/c5.txt gpurun_out/gw/c4.txt
