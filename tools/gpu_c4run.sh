# 3D/4D parity (incl. the C4/C5 grids) + C4/C5 timing and a C4 kernel trace
set -e
out=gpurun_out/${1:-c4t}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_configs.py -k "3d or 4d or c4 or c5 or fft2d" > $out/pytest.txt 2>&1
timeout -k 10 300 python -u tools/bench_configs.py --configs C4,C5 --steps 2 > $out/bench.txt 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $out/prof -o c4 -- python3 -u tools/bench_configs.py --configs C4 --steps 1 > $out/prof.log 2>&1
f=$(find $out/prof -name "*kernel_stats.csv" | head -1); cp $f $out/kernel_stats.csv
rm -rf $out/prof
