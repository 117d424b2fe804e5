set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r05k
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -k "past_lds or generic_prime or test_learn_4d" > gpurun_out/r05k/pytest.txt 2>&1 || { tail -40 gpurun_out/r05k/pytest.txt; exit 1; }
tail -3 gpurun_out/r05k/pytest.txt

