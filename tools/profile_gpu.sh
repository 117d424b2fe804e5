#!/bin/bash
# Profile the bench workload on the GPU box (run via gpurun from the repo root).
#   tools/profile_gpu.sh <tag> [bench args...]
# Writes gpurun_out/prof_<tag>_{trace,fetch,write,sq}/...  Each rocprofv3 pass
# runs under its own timeout; PMC passes use --kernel-trace only (no sys/runtime
# trace), FETCH_SIZE and WRITE_SIZE in separate passes (TCC slot budget).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-run}; shift
args=${@:-"--n 1000 --steps 1 --warmup 1 --no-cpu-baseline"}
out=gpurun_out/prof_${tag}
mkdir -p $out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $out/trace -o trace -- python3 bench.py $args > $out/trace.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -f csv -d $out/fetch -o fetch -- python3 bench.py $args > $out/fetch.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -f csv -d $out/write -o write -- python3 bench.py $args > $out/write.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY -f csv -d $out/sq -o sq -- python3 bench.py $args > $out/sq.log 2>&1 || exit $?
echo done
