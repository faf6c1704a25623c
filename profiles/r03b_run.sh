set -o pipefail
D=gpurun_out/r03b; mkdir -p $D
timeout -k 10 400 python -u -m pytest tests/test_abi_gpu.py tests/test_config_sized_gpu.py tests/test_routedb_golden_gpu.py tests/test_engine_parity_gpu.py -x -q --timeout 300 --timeout-method thread > $D/gpu_tests.log 2>&1; rc=$?
tail -3 $D/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
Q="--no-cpu-baseline --no-route-db --no-wan --no-whatif --no-repair --steps 20 --warmup 3"
for v in "1 0 0" "0 0 0" "1 1 0" "1 0 1"; do set -- $v
  OPENR_MS_SELL=$1 OPENR_NL_XCD=$2 OPENR_NL_HELD=$3 timeout -k 10 200 python bench.py $Q > $D/fab_$1$2$3.json 2> $D/fab_$1$2$3.err || exit 7
  python -c "import json;d=json.load(open('$D/fab_$1$2$3.json'));print('sell',$1,'xcd',$2,'held',$3,d['ms_per_step'],d.get('kernels'))" | cut -c1-400
done
