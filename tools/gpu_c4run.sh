set -e
mkdir -p gpurun_out/c4t
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "3d" tests/test_gpu_configs.py > gpurun_out/c4t/pytest.txt 2>&1
for tc in 2 4; do CCSC_TSOLVE3_TC=$tc timeout -k 10 200 python -u tools/bench_configs.py --configs C4 --steps 2 > gpurun_out/c4t/bench_tc$tc.txt 2>&1; done
