set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/nb3
cp abx/libccsc_nb3.so ccsc_code_iccv2017_amd/libccsc.so
timeout -k 10 600 python -u -m pytest tests/test_hs23.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "hs23 or tile_dsolve" > gpurun_out/nb3/pytest.txt 2>&1 || { tail -30 gpurun_out/nb3/pytest.txt; exit 1; }
tail -2 gpurun_out/nb3/pytest.txt
bash tools/gpu_cfg_ab.sh C3 nb2 nb3 nb2 nb3
