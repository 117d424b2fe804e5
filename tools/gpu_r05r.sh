set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r05r
cp abx/libccsc_nb2.so ccsc_code_iccv2017_amd/libccsc.so
timeout -k 10 900 python -u -m pytest tests/test_hs23.py tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -k "hs23 or 4d or dsolve_tile or test_learn_2d_matches_oracle" > gpurun_out/r05r/pytest.txt 2>&1 || { tail -30 gpurun_out/r05r/pytest.txt; exit 1; }
tail -2 gpurun_out/r05r/pytest.txt
bash tools/gpu_cfg_ab.sh C3 base nb2 nb4 base nb2 nb4 || exit 1
bash tools/gpu_abl.sh base nb2 base nb2
