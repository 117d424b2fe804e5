cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in bs1 bs2; do cp abv/libccsc_$v.so ccsc_code_iccv2017_amd/libccsc.so; for L in 40 64; do
  echo "$v lds$L"; CCSC_LINE_LDS_KB=$L timeout -k 10 200 python tools/bench_solvers.py --solvers inpaint,poisson,video --iters 50 --no-cpu-baseline 2>/dev/null | python3 -c "
import json,sys
for l in sys.stdin: d=json.loads(l); print('  ', d['solver'], round(d['value'],1))"
done; done
