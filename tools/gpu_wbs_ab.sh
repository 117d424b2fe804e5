# staged many-view Woodbury d-solve: 4D parity with abx/libccsc_$1.so, then same-box C5 A/B
# (CCSC_WB_STAGE=0 keeps k_dsolve_wbv) -> gpurun_out/wbs/
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/wbs
cp abx/libccsc_$1.so ccsc_code_iccv2017_amd/libccsc.so
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -v --timeout 300 --timeout-method thread -k "4d or C5 or c5" > gpurun_out/wbs/pytest.txt 2>&1 || { tail -30 gpurun_out/wbs/pytest.txt; exit 1; }
tail -2 gpurun_out/wbs/pytest.txt
rm -f gpurun_out/wbs/summary.txt
for r in 1 2; do
  for s in 0 1; do
    CCSC_WB_STAGE=$s timeout -k 10 300 python tools/bench_configs.py --configs C5 --steps 3 > gpurun_out/wbs/c5_$s.$r.json 2>/dev/null || exit 1
    echo "stage=$s $(cut -c1-400 gpurun_out/wbs/c5_$s.$r.json)" >> gpurun_out/wbs/summary.txt
  done
done
CCSC_WB_STAGE=1 timeout -s KILL 240 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/wbs/prof -o c5 -- python3 tools/bench_configs.py --configs C5 --steps 1 > gpurun_out/wbs/prof.log 2>&1 || exit 1
cat gpurun_out/wbs/summary.txt
