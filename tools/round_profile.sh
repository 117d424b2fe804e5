#!/bin/bash
# Full C2 bench + rocprofv3 evidence for one round: tools/round_profile.sh <tag>
# Raw per-dispatch CSVs are summarised on the box (tools/pmc_summary.py) and
# gzipped/dropped so gpurun_out stays under the copy-back limit.
set -o pipefail
tag=${1:-r01}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 600 python3 bench.py > $out/bench.json 2> $out/bench.err || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d $out/trace -o trace -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $out/trace.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --pmc FETCH_SIZE -f csv -d $out/fetch -o fetch -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > $out/fetch.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --pmc WRITE_SIZE -f csv -d $out/write -o write -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > $out/write.log 2>&1 || exit $?
python3 tools/pmc_summary.py $out/fetch/fetch_counter_collection.csv $out/write/write_counter_collection.csv > $out/pmc_summary.txt
python3 tools/pmc_summary.py --json $out/pmc_zsplit.json 10000 $out/fetch/fetch_counter_collection.csv $out/write/write_counter_collection.csv
for f in $(find $out -name "*_kernel_trace.csv" -o -name "*_counter_collection.csv"); do
  grep -E "ccsc::|Kernel_Name" $f | gzip > $f.ccsc.gz; rm -f $f
done
du -sh $out
echo done
