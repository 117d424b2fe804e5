#!/bin/bash
# Round profile without the test suite: the C2 bench + rocprofv3 evidence (tools/round_profile.sh),
# an MFMA-counter pass of the D-precompute, then the C3/C4/C5 kernel stats
# (tools/gpu_configs_prof.sh): tools/gpu_profile_round.sh <tag>
set -o pipefail
tag=${1:-r05p}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/round_profile.sh $tag || exit $?
out=gpurun_out/$tag
B="python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-configs --no-shard-diag"
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU_MFMA_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVES GRBM_GUI_ACTIVE -f csv -d $out/mfma -o mfma -- $B > $out/mfma.log 2>&1 || exit $?
python3 tools/pmc_summary.py $out/mfma/mfma_counter_collection.csv > $out/pmc_mfma.txt
for f in $(find $out/mfma -name "*_kernel_trace.csv" -o -name "*_counter_collection.csv"); do
  grep -E "ccsc::|Kernel_Name" $f | gzip > $f.ccsc.gz; rm -f $f
done
bash tools/gpu_configs_prof.sh ${tag}c || exit $?
echo done
