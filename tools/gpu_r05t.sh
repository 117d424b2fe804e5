set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r05t
cp abx/libccsc_t48n.so ccsc_code_iccv2017_amd/libccsc.so
timeout -k 10 900 python -u -m pytest tests/test_hs23.py tests/test_gpu_solvers.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r05t/pytest.txt 2>&1 || { tail -30 gpurun_out/r05t/pytest.txt; exit 1; }
tail -2 gpurun_out/r05t/pytest.txt
bash tools/gpu_cfg_ab.sh C3 t44 t48n t44 t48n || exit 1
bash tools/gpu_solv_ab.sh t44 t48n
