# A/B of a C4 knob: tools/gpu_c4ab.sh <tag> <ENVVAR> <values...>
set -e
out=gpurun_out/$1; var=$2; shift 2
mkdir -p $out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "3d" > $out/pytest.txt 2>&1
for v in "$@"; do
  env $var=$v timeout -k 10 200 python -u tools/bench_configs.py --configs C4 --steps 2 > $out/bench_$v.txt 2>&1
done
