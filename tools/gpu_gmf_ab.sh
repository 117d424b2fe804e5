#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/ab_bench.sh abv base mf_NOGRAM mf_NOCHOL mf_NOPOTRF mf_NOTRSM mf_NOTRAIL || exit 1
for v in base mf_NOGRAM mf_NOCHOL mf_NOPOTRF mf_NOTRSM mf_NOTRAIL; do echo "$v $(grep -o '"gram_chol": {[^}]*}' gpurun_out/ab/$v.err)"; done
cp abv/libccsc_base.so ccsc_code_iccv2017_amd/libccsc.so
bash tools/sq_profile.sh gmf SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS || exit 1
grep gram_chol gpurun_out/sq_gmf/summary.txt
