#!/bin/bash
# z-step change check: the 110-grid parity cases + new tests on abx/libccsc_<new>.so, then a
# same-box A/B of the n=1000 C2 slice alternating <old> <new> <old> <new>:
#   tools/gpu_zl_ab.sh <tag> <old> <new>
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
source tools/_libswap.sh
tag=$1; old=$2; new=$3
mkdir -p gpurun_out/$tag
cp abx/libccsc_$new.so ccsc_code_iccv2017_amd/libccsc.so
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_multirank.py -m gpu -x -v --timeout 240 --timeout-method thread \
  -k "${TESTSEL:-110 or zline or headline or fullsize or rccl_self or production_path or two_ranks}" > gpurun_out/$tag/pytest.txt 2>&1 || { tail -40 gpurun_out/$tag/pytest.txt; exit 1; }
tail -2 gpurun_out/$tag/pytest.txt
for v in $old $new $old $new; do
  cp abx/libccsc_$v.so ccsc_code_iccv2017_amd/libccsc.so
  timeout -k 10 300 python bench.py --n ${AB_N:-1000} --steps 3 --warmup 1 --no-cpu-baseline --no-configs > gpurun_out/$tag/$v.json 2> gpurun_out/$tag/$v.err || exit 1
  echo "$v $(python -c "import json;d=json.load(open('gpurun_out/$tag/$v.json'));print(round(d['ms_per_step'],2), round(d['roofline']['avg_launch_ms'],3))") $(grep per-kernel gpurun_out/$tag/$v.err | cut -c1-300)" | tee -a gpurun_out/$tag/ab.txt
done
