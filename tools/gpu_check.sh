set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/t1.log 2>&1 || { tail -30 gpurun_out/t1.log; exit 1; }
tail -3 gpurun_out/t1.log
timeout -k 10 300 python bench.py --n 1000 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/b1.json 2> gpurun_out/b1.err || { tail -20 gpurun_out/b1.err; exit 1; }
cat gpurun_out/b1.json; grep per-kernel gpurun_out/b1.err
