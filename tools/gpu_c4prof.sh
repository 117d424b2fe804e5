# C4 per-kernel profile: rocprofv3 kernel-trace stats of two outer iterations
set -e
mkdir -p gpurun_out/c4p
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/c4p/prof -o c4 -- python3 -u tools/bench_configs.py --configs C4 --steps 2 > gpurun_out/c4p/bench.txt 2>&1
find gpurun_out/c4p/prof -name '*kernel_stats.csv' -exec cp {} gpurun_out/c4p/kernel_stats.csv \;
