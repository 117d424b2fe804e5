# multi-RHS tile d-solve: L23 + 4D parity, then same-box C3 A/B (CCSC_DS_TILE=0: k_dsolve)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r05o
timeout -k 10 900 python -u -m pytest tests/test_hs23.py tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -k "hs23 or 4d or dsolve_tile or test_learn_2d_matches_oracle" > gpurun_out/r05o/pytest.txt 2>&1 || { tail -30 gpurun_out/r05o/pytest.txt; exit 1; }
tail -2 gpurun_out/r05o/pytest.txt
rm -f gpurun_out/r05o/summary.txt
for r in 1 2; do
  for t in 0 1; do
    CCSC_DS_TILE=$t timeout -k 10 300 python tools/bench_configs.py --configs C3 --steps 3 > gpurun_out/r05o/c3_$t.$r.json 2>/dev/null || exit 1
    echo "tile=$t $(python -c "import json;d=json.load(open('gpurun_out/r05o/c3_$t.$r.json'));print(d['s_per_outer_iteration'], d['timed_iterations'])")" >> gpurun_out/r05o/summary.txt
  done
done
timeout -s KILL 240 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/r05o/prof -o c3 -- python3 tools/bench_configs.py --configs C3 --steps 1 > gpurun_out/r05o/prof.log 2>&1 || exit 1
cat gpurun_out/r05o/summary.txt
