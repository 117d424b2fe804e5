set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r05xt
cp abx/libccsc_xt.so ccsc_code_iccv2017_amd/libccsc.so
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread -k "3d or C4 or c4" > gpurun_out/r05xt/pytest.txt 2>&1 || { tail -30 gpurun_out/r05xt/pytest.txt; exit 1; }
tail -2 gpurun_out/r05xt/pytest.txt
bash tools/gpu_cfg_ab.sh C4 base xt base xt
