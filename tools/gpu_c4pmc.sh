#!/bin/bash
# C4 (3D) per-kernel counters: FETCH / WRITE / two SQ passes over one outer iteration
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/${1:-c4pmc}
mkdir -p $out
B="python3 tools/bench_configs.py --configs C4 --steps 1"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $out/trace -o trace -- $B > $out/trace.log 2>&1 || exit $?
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc FETCH_SIZE -f csv -d $out/fetch -o fetch -- $B > $out/fetch.log 2>&1 || exit $?
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc WRITE_SIZE -f csv -d $out/write -o write -- $B > $out/write.log 2>&1 || exit $?
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE -f csv -d $out/sq -o sq -- $B > $out/sq.log 2>&1 || exit $?
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE -f csv -d $out/sq2 -o sq2 -- $B > $out/sq2.log 2>&1 || exit $?
python3 tools/pmc_summary.py $out/fetch/fetch_counter_collection.csv $out/write/write_counter_collection.csv $out/sq/sq_counter_collection.csv $out/sq2/sq2_counter_collection.csv > $out/pmc_summary.txt
f=$(find $out/trace -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && cp $f $out/rocprof_kernel_stats.csv
for f in $(find $out -name "*_kernel_trace.csv" -o -name "*_counter_collection.csv"); do
  grep -E "ccsc::|Kernel_Name" $f | gzip > $f.ccsc.gz; rm -f $f
done
echo done
