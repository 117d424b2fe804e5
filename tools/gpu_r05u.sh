set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r05u
cp abx/libccsc_sd.so ccsc_code_iccv2017_amd/libccsc.so
timeout -k 10 900 python -u -m pytest tests/test_hs23.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "hs23 or 4d or 3d or test_learn_2d_matches_oracle or zline or woodbury" > gpurun_out/r05u/pytest.txt 2>&1 || { tail -30 gpurun_out/r05u/pytest.txt; exit 1; }
tail -2 gpurun_out/r05u/pytest.txt
bash tools/gpu_cfg_ab.sh C5 base sd base sd || exit 1
cp gpurun_out/cfgab/summary.txt gpurun_out/r05u/c5.txt
bash tools/gpu_cfg_ab.sh C3 base sd base sd || exit 1
cp gpurun_out/cfgab/summary.txt gpurun_out/r05u/c3.txt
cat gpurun_out/r05u/c5.txt gpurun_out/r05u/c3.txt
bash tools/gpu_cfg_ab.sh C4 base sd base sd || exit 1
cp gpurun_out/cfgab/summary.txt gpurun_out/r05u/c4.txt
cat gpurun_out/r05u/c4.txt
