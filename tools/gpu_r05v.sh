set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r05v
cp abx/libccsc_hs.so ccsc_code_iccv2017_amd/libccsc.so
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread -k "4d or C5 or c5 or woodbury" > gpurun_out/r05v/pytest.txt 2>&1 || { tail -30 gpurun_out/r05v/pytest.txt; exit 1; }
tail -2 gpurun_out/r05v/pytest.txt
bash tools/gpu_cfg_ab.sh C5 base hs base hs
