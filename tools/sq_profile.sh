#!/bin/bash
# SQ counter pass on the C2 slice (n=1000): tools/sq_profile.sh <tag> [counters...]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
tag=$1; shift
ctr=${@:-"SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES"}
out=gpurun_out/sq_$tag
mkdir -p $out
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $ctr -f csv -d $out -o sq -- python3 bench.py --n 1000 --steps 1 --warmup 0 --no-cpu-baseline --no-configs > $out/run.log 2>&1 || exit $?
f=$(find $out -name "sq_counter_collection.csv" | head -1)
python3 tools/pmc_summary.py $f > $out/summary.txt
find $out -name "*.csv" -delete
echo done
