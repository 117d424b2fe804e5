#!/bin/bash
# clock under k_zline on two libraries (abx/libccsc_<v>.so): GRBM_GUI_ACTIVE per dispatch
# over the dispatch's duration = the shader clock it held -> gpurun_out/clk/<v>/
#   tools/gpu_clock_ab.sh v1 v2 ...
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
source tools/_libswap.sh
mkdir -p gpurun_out/clk
for v in "$@"; do
  cp abx/libccsc_$v.so ccsc_code_iccv2017_amd/libccsc.so
  timeout -s KILL 240 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES --kernel-trace -d gpurun_out/clk/$v -o run --output-format csv -- python bench.py --n 1000 --steps 1 --warmup 1 --no-cpu-baseline --no-configs --no-shard-diag > gpurun_out/clk/$v.log 2>&1 || exit 1
done
python tools/clock_summary.py gpurun_out/clk "$@"
