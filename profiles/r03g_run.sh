set -o pipefail
D=gpurun_out/r03g; mkdir -p $D
timeout -k 10 300 python -u -m pytest tests/test_abi_gpu.py tests/test_config_sized_gpu.py -x -q --timeout 200 --timeout-method thread -k "swar or msbfs or config or hop_bound or high_degree" > $D/gpu_tests.log 2>&1; rc=$?
tail -3 $D/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
Q="--no-cpu-baseline --no-route-db --no-wan --no-whatif --no-repair --steps 20 --warmup 3"
for v in "1 1" "0 1" "1 0"; do set -- $v
  OPENR_NL_SWAR=$1 OPENR_MS_WREC=$2 timeout -k 10 200 python bench.py $Q > $D/fab_s$1w$2.json 2> $D/fab_s$1w$2.err || exit 7
  python -c "import json;d=json.load(open('$D/fab_s$1w$2.json'));print('swar',$1,'wrec',$2,d['ms_per_step'],d.get('kernels'))"
done
