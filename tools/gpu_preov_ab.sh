#!/bin/bash
# Same-box A/B of the D-precompute overlap (CCSC_PRE_OVERLAP=1: block j+1's R2C on a side
# stream beside block j's Gram; 0: in series on the engine stream), full C2, alternating.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/preov
mkdir -p $out
for i in 1 2; do
  for v in 1 0; do
    CCSC_PRE_OVERLAP=$v timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline \
        > $out/ov${v}_$i.json 2> $out/ov${v}_$i.err || exit 1
    echo "overlap=$v run $i: $(python3 -c "import json;d=json.load(open('$out/ov${v}_$i.json'));print(round(d['ms_per_step'],1),'ms/step', round(d['value']))") $(grep -o '"gram_chol": {[^}]*}' $out/ov${v}_$i.err | cut -c1-60)" | tee -a $out/summary.txt
  done
done
