# bench-only A/B (ablation builds fail parity by design): tools/ab_bench.sh v1 v2 ...
set -o pipefail
for v in "$@"; do
  cp variants/libccsc_$v.so ccsc_code_iccv2017_amd/libccsc.so
  timeout -k 10 300 python bench.py --n 1000 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/ab_b_$v.log 2>&1 || exit 1
done
