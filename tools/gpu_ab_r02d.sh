#!/bin/bash
# one-off A/B call: z-step L2-state ablation, gram/chol ablations (n = 1000 slice),
# d-solve occupancy knob at full C2 (the second sweep's reuse distance depends on n)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/ab gpurun_out/abenv
bash tools/ab_bench.sh abv base zl_l2 nogram nochol || exit 1
for v in base zl_l2 nogram nochol; do echo "$v: $(grep per-kernel gpurun_out/ab/$v.err)"; done
cp abv/libccsc_base.so ccsc_code_iccv2017_amd/libccsc.so
for kb in 0 40 80; do
  CCSC_DS_LDS_KB=$kb timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/abenv/ds$kb.json 2> gpurun_out/abenv/ds$kb.err || { tail -5 gpurun_out/abenv/ds$kb.err; exit 1; }
  echo "DS_LDS_KB=$kb: $(grep per-kernel gpurun_out/abenv/ds$kb.err)"
done
