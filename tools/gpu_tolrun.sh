set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/tol
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multirank.py tests/test_gpu_fullsize.py -m gpu -v -k "tol or multi or fullsize or two_ranks or zline" --timeout 300 --timeout-method thread > gpurun_out/tol/pytest.txt 2>&1 || { tail -30 gpurun_out/tol/pytest.txt; exit 1; }
tail -3 gpurun_out/tol/pytest.txt
timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 --tol 1e-3 > gpurun_out/tol/b_tol.json 2> gpurun_out/tol/b_tol.err || exit 1
timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/tol/b_0.json 2> gpurun_out/tol/b_0.err || exit 1
python3 -c "
import json
for f in ('b_tol','b_0'):
    d=json.load(open('gpurun_out/tol/'+f+'.json')); print(f, d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])
"
grep "tol 0.001" gpurun_out/tol/b_tol.err
