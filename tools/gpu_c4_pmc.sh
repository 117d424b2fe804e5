#!/bin/bash
# C4 counter passes: SQ (tools/gpu_cfg_pmc.sh), then HBM bytes (FETCH_SIZE, WRITE_SIZE) and the
# wait/stall split -> gpurun_out/<tag>/
set -o pipefail
tag=${1:-c4pmc}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/$tag
mkdir -p $out
[ -f $out/C4_sq.txt ] || bash tools/gpu_cfg_pmc.sh $tag C4 || exit $?
for c in FETCH_SIZE WRITE_SIZE; do   # separate passes: 3 + 2 TCC counters exceed the 4 of one run
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $c -f csv -d $out/hbm_$c -o hbm -- python3 -u tools/bench_configs.py --configs C4 --steps 1 > $out/hbm_$c.log 2>&1 || exit $?
  f=$(find $out/hbm_$c -name "*counter_collection.csv" | head -1)
  python3 tools/pmc_summary.py $f > $out/C4_$c.txt || exit $?
  rm -rf $out/hbm_$c
done
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM SQ_INSTS_SALU SQ_INSTS_VMEM SQ_ACTIVE_INST_ANY -f csv -d $out/st -o st -- python3 -u tools/bench_configs.py --configs C4 --steps 1 > $out/st.log 2>&1 || exit $?
f=$(find $out/st -name "*counter_collection.csv" | head -1)
python3 tools/pmc_summary.py $f > $out/C4_stall.txt || exit $?
rm -rf $out/st
echo done
