set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r05m
timeout -k 10 1000 python -u -m pytest tests/test_gpu_parity.py tests/test_hs23.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r05m/pytest.txt 2>&1 || { tail -40 gpurun_out/r05m/pytest.txt; exit 1; }
tail -3 gpurun_out/r05m/pytest.txt
