# Gram/Cholesky variant: parity of the 2D learners (every MFMA factor shape) with variant
# $1 in place, then bench-only A/B of abx/ variants: tools/gpu_gc_ab.sh <testvar> v1 v2 ...
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
source tools/_libswap.sh
mkdir -p gpurun_out/gc
t=$1; shift
cp abx/libccsc_$t.so ccsc_code_iccv2017_amd/libccsc.so
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 240 --timeout-method thread -k "test_learn_2d_matches_oracle or dsolve_tile or woodbury" > gpurun_out/gc/pytest_$t.txt 2>&1 || { tail -30 gpurun_out/gc/pytest_$t.txt; exit 1; }
tail -2 gpurun_out/gc/pytest_$t.txt
bash tools/gpu_abl.sh "$@"
