#!/bin/bash
# a test selection, then the default bench line: tools/gpu_check_bench.sh <tag> "<pytest -k>"
# -> gpurun_out/<tag>/{pytest.txt,bench.json,bench.err}
set -o pipefail
tag=$1; sel=$2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/$tag
python tools/check_lib.py || exit 1
if [ -n "$sel" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -k "$sel" --timeout 300 --timeout-method thread > gpurun_out/$tag/pytest.txt 2>&1 || { tail -30 gpurun_out/$tag/pytest.txt; exit 1; }
  tail -2 gpurun_out/$tag/pytest.txt
fi
timeout -k 10 900 python -u bench.py ${BENCH_ARGS:-} > gpurun_out/$tag/bench.json 2> gpurun_out/$tag/bench.err || { tail -20 gpurun_out/$tag/bench.err; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/$tag/bench.json'))
r=d['roofline']; print('value', round(d['value']), 'ms/step', round(d['ms_per_step'],1), 'zstep', round(r['avg_launch_ms'],2), 'frac', round(r['frac'],3), 'copy', r['copy_GBps'], 'foc', r['frac_of_copy'])
print('shard8', json.dumps(d.get('shard8_diag')))
print('configs', {k: round(v['s_per_outer_iteration'],4) for k,v in (d.get('configs') or {}).items()})"
