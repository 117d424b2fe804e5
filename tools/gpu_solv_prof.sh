# solver bench + kernel stats of the inpainting and Poisson solvers -> gpurun_out/solv/
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/solv


timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/solv/prof -o run -- python tools/bench_solvers.py --no-cpu-baseline --solvers ${SOLV:-inpaint,poisson} > gpurun_out/solv/prof.log 2>&1 || exit 1
find gpurun_out/solv/prof -name "*kernel_stats.csv" | head -3
