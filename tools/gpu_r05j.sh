set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r05j
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 240 --timeout-method thread -k "generic_prime or fft2d" > gpurun_out/r05j/pytest.txt 2>&1 || { tail -30 gpurun_out/r05j/pytest.txt; exit 1; }
tail -2 gpurun_out/r05j/pytest.txt
bash tools/gpu_abl.sh new wl0 wl4 new wl0 wl4
