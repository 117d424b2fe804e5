#!/bin/bash
# Full C2 bench + rocprofv3 evidence for one round: tools/round_profile.sh <tag> [nobench]
#   bench.json            the bench line (incl. the CPU baseline leg)
#   trace/                rocprofv3 --kernel-trace --stats of `bench.py --steps 2 --warmup 1`
#   FETCH / WRITE / SQ    separate --pmc passes (MI355X_MICROARCH.md: one TCC pass cannot hold
#                         both; SQ wait/issue counters + GRBM_GUI_ACTIVE for the clock)
#   pmc_zsplit.json       per-kernel merge of the three passes (tools/pmc_summary.py --json),
#                         read by bench.py for roofline.traffic / roofline.sq
# Raw per-dispatch CSVs are summarised on the box and gzipped so gpurun_out stays small.
set -o pipefail
tag=${1:-r03}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/$tag
mkdir -p $out
B="python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-configs --no-shard-diag"
if [ "$2" != "nobench" ]; then
  timeout -k 10 600 python3 bench.py > $out/bench.json 2> $out/bench.err || exit $?
fi
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $out/trace -o trace -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-configs --no-shard-diag > $out/trace.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -f csv -d $out/fetch -o fetch -- $B > $out/fetch.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -f csv -d $out/write -o write -- $B > $out/write.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE -f csv -d $out/sq -o sq -- $B > $out/sq.log 2>&1 || exit $?
python3 tools/pmc_summary.py $out/fetch/fetch_counter_collection.csv $out/write/write_counter_collection.csv $out/sq/sq_counter_collection.csv > $out/pmc_summary.txt
python3 tools/pmc_summary.py --json $out/pmc_zsplit.json 10000 $out/fetch/fetch_counter_collection.csv $out/write/write_counter_collection.csv $out/sq/sq_counter_collection.csv
f=$(find $out/trace -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && cp $f $out/rocprof_kernel_stats.csv
for f in $(find $out -name "*_kernel_trace.csv" -o -name "*_counter_collection.csv"); do
  grep -E "ccsc::|Kernel_Name" $f | gzip > $f.ccsc.gz; rm -f $f
done
du -sh $out
echo done
