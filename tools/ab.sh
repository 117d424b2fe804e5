# A/B driver: tools/ab.sh v1 v2 ... (variants/libccsc_<v>.so), parity tests + n=1000 bench each
set -o pipefail
for v in "$@"; do
  cp variants/libccsc_$v.so ccsc_code_iccv2017_amd/libccsc.so
  timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -x -q -m gpu > gpurun_out/ab_t_$v.log 2>&1 || exit 1
  timeout -k 10 300 python bench.py --n 1000 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/ab_b_$v.log 2>&1 || exit 1
done
