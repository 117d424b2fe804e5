# C5 counter passes (SQ, then TA/TCP) for the Woodbury many-view d-solve -> gpurun_out/c5pmc/
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/c5pmc
mkdir -p $out
bash tools/gpu_cfg_pmc.sh c5pmc C5 || exit $?
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc TA_TA_BUSY_sum TA_FLAT_READ_WAVEFRONTS_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum GRBM_GUI_ACTIVE -f csv -d $out/ta -o ta -- python3 -u tools/bench_configs.py --configs C5 --steps 1 > $out/ta.log 2>&1 || { tail -5 $out/ta.log; exit 1; }
f=$(find $out/ta -name "*counter_collection.csv" | head -1)
python3 tools/pmc_summary.py $f > $out/C5_ta.txt || exit $?
rm -rf $out/ta
grep -E "dsolve_wbv|dual_r2c|c2r_dout|zstep_diag" $out/C5_ta.txt $out/C5_sq.txt | cut -c1-600
