#!/bin/bash
# A/B of library variants on every config: tools/ab_cfg.sh dir v1 v2 ...
# dir holds libccsc_<v>.so (push it un-ignored); per variant: tools/bench_configs.py
# (C1, C3, C4, C5, or $CONFIGS) and the n=1000 C2 slice of bench.py (per-kernel times on
# stderr; skipped with SKIP_BENCH=1).
set -o pipefail
source tools/_libswap.sh
d=$1; shift
mkdir -p gpurun_out/ab
for v in "$@"; do
  cp $d/libccsc_$v.so ccsc_code_iccv2017_amd/libccsc.so
  timeout -k 10 300 python -u tools/bench_configs.py --steps 1 --configs ${CONFIGS:-C1,C3,C4,C5} > gpurun_out/ab/$v.cfg.json 2> gpurun_out/ab/$v.cfg.err || exit 1
  [ -n "$SKIP_BENCH" ] || timeout -k 10 300 python bench.py --n 1000 --steps 2 --warmup 1 --no-cpu-baseline --no-configs > gpurun_out/ab/$v.json 2> gpurun_out/ab/$v.err || exit 1
done
