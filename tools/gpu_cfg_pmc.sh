#!/bin/bash
# SQ counters of one config's kernels (one outer iteration): tools/gpu_cfg_pmc.sh <tag> <C>
# -> gpurun_out/<tag>/<C>_sq.txt (mean per dispatch per kernel)
set -o pipefail
tag=$1; c=$2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/$tag
mkdir -p $out
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE -f csv -d $out/pmc_$c -o $c -- python3 -u tools/bench_configs.py --configs $c --steps 1 > $out/pmc_$c.log 2>&1 || exit $?
f=$(find $out/pmc_$c -name "*counter_collection.csv" | head -1)
python3 tools/pmc_summary.py $f > $out/${c}_sq.txt || exit $?
rm -rf $out/pmc_$c
echo done
