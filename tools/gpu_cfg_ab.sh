# same-box A/B of abx/ variants on one config: tools/gpu_cfg_ab.sh <C> v1 v2 ... -> gpurun_out/cfgab/
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
source tools/_libswap.sh
mkdir -p gpurun_out/cfgab
c=$1; shift
rm -f gpurun_out/cfgab/summary.txt
for v in "$@"; do
  cp abx/libccsc_$v.so ccsc_code_iccv2017_amd/libccsc.so
  timeout -k 10 300 python tools/bench_configs.py --configs $c --steps 3 > gpurun_out/cfgab/$v.json 2>/dev/null || exit 1
  echo "$v $(python -c "import json;d=json.load(open('gpurun_out/cfgab/$v.json'));print(d['s_per_outer_iteration'], d['timed_iterations'])")" >> gpurun_out/cfgab/summary.txt
done
cat gpurun_out/cfgab/summary.txt
