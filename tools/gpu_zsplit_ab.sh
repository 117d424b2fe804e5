#!/bin/bash
# two-stream z-phase gate: its exactness test + the zline parity cases, then the C2 bench with
# the split on and off (CCSC_ZSPLIT2)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/zsplit
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "zline or headline" \
    --timeout 300 --timeout-method thread > $out/pytest.txt 2>&1 || { tail -5 $out/pytest.txt; exit 1; }
tail -1 $out/pytest.txt
for f in 1 0 1; do
  CCSC_ZSPLIT2=$f timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > $out/bench_$f.json 2> $out/bench_$f.err || exit 1
  python3 -c "import json;d=json.load(open('$out/bench_$f.json'));print('split=$f', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])"
done
