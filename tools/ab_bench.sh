# bench-only A/B (ablation builds fail parity by design): tools/ab_bench.sh dir v1 v2 ...
# dir holds libccsc_<v>.so (push it un-ignored); n=1000 C2 slice (AB_N to change), per-kernel
# times on stderr; every run's per-kernel line is appended to gpurun_out/ab/summary.txt
set -o pipefail
source tools/_libswap.sh
d=$1; shift
mkdir -p gpurun_out/ab
for v in "$@"; do
  cp $d/libccsc_$v.so ccsc_code_iccv2017_amd/libccsc.so
  timeout -k 10 300 python bench.py --n ${AB_N:-1000} --steps 2 --warmup 1 --no-cpu-baseline --no-configs > gpurun_out/ab/$v.json 2> gpurun_out/ab/$v.err || exit 1
  echo "$v $(grep per-kernel gpurun_out/ab/$v.err)" >> gpurun_out/ab/summary.txt
done
