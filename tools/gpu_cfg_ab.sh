#!/bin/bash
# config timing A/B over abv/ variants: tools/gpu_cfg_ab.sh <configs> v1 v2 ...
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
cfg=$1; shift
mkdir -p gpurun_out/cfgab
for v in "$@"; do
  cp abv/libccsc_$v.so ccsc_code_iccv2017_amd/libccsc.so
  timeout -k 10 300 python3 -u tools/bench_configs.py --configs $cfg --steps 2 > gpurun_out/cfgab/$v.jsonl 2>&1 || exit 1
  echo "$v: $(cut -c1-160 gpurun_out/cfgab/$v.jsonl | tr '\n' ' ')"
done
