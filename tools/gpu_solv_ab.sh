# same-box A/B of abx/ library variants on the solver bench: tools/gpu_solv_ab.sh v1 v2 ...
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
source tools/_libswap.sh
mkdir -p gpurun_out/solvab
rm -f gpurun_out/solvab/summary.txt
for v in "$@"; do
  cp abx/libccsc_$v.so ccsc_code_iccv2017_amd/libccsc.so
  timeout -k 10 300 python tools/bench_solvers.py --no-cpu-baseline > gpurun_out/solvab/$v.jsonl 2> gpurun_out/solvab/$v.err || exit 1
  echo "$v $(python -c "
import json
print(' '.join('%s=%.3f' % (d['solver'], d['ms_per_iter']) for d in map(json.loads, open('gpurun_out/solvab/$v.jsonl'))))")" >> gpurun_out/solvab/summary.txt
done
cat gpurun_out/solvab/summary.txt
