#!/bin/bash
# Full GPU pass: the -m gpu suite then the default bench line; logs under gpurun_out/<tag>.
set -o pipefail
tag=${1:-r03_full}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -v -rsP --timeout 300 --timeout-method thread \
    > $out/pytest_gpu.txt 2>&1
rc=$?
tail -3 $out/pytest_gpu.txt
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 5 --warmup 2 > $out/bench.json 2> $out/bench.err || exit $?
python3 -c "import json;d=json.load(open('$out/bench.json'));print('value',d['value'],'ms/step',d['ms_per_step'],'zstep ms',d['roofline']['avg_launch_ms'])"
