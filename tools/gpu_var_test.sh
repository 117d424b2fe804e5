#!/bin/bash
# run one pytest selection against several abv/ library variants: tools/gpu_var_test.sh <tag> <selection> v1 v2 ...
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
source tools/_libswap.sh
tag=$1; sel=$2; shift 2
mkdir -p gpurun_out/$tag
for v in "$@"; do
  cp abv/libccsc_$v.so ccsc_code_iccv2017_amd/libccsc.so
  timeout -k 10 400 python -u -m pytest "$sel" -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$tag/$v.txt 2>&1
  echo "$v: $(tail -1 gpurun_out/$tag/$v.txt)"
done
