set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r05n
timeout -k 10 1000 python -u -m pytest tests/test_gpu_solvers.py tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -k "solve or past_lds or generic_prime or test_learn_2d_matches_oracle or 4d or woodbury or dsolve_tile" > gpurun_out/r05n/pytest.txt 2>&1 || { tail -40 gpurun_out/r05n/pytest.txt; exit 1; }
tail -3 gpurun_out/r05n/pytest.txt
