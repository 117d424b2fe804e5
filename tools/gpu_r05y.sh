set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r05y
cp abx/libccsc_xc.so ccsc_code_iccv2017_amd/libccsc.so
timeout -k 10 900 python -u -m pytest tests/test_gpu_solvers.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "solve or past_lds or generic_prime" > gpurun_out/r05y/pytest.txt 2>&1 || { tail -30 gpurun_out/r05y/pytest.txt; exit 1; }
tail -2 gpurun_out/r05y/pytest.txt
bash tools/gpu_solv_ab.sh base xc base xc
