set -o pipefail
D=gpurun_out/r03ab; mkdir -p $D
OPENR_NL_NPL=8 timeout -k 10 400 python -u -m pytest tests/test_abi_gpu.py tests/test_config_sized_gpu.py tests/test_zero_metric_plan.py -x -q --timeout 300 --timeout-method thread > $D/gpu_tests_npl8.log 2>&1; rc=$?
tail -2 $D/gpu_tests_npl8.log
[ $rc -eq 0 ] || exit $rc
B="bench.py --no-cpu-baseline --no-route-db --no-whatif --no-wan --steps 30 --warmup 5"
for x in 4 8 4 8; do
  OPENR_NL_NPL=$x timeout -k 10 200 python $B > $D/npl$x.json 2>> $D/err.log || exit 5
  python -c "import json;d=json.load(open('$D/npl$x.json'));print('npl=$x', d['ms_per_step'], d['kernels']['spf_nh_levels_held_kernel'], d['parity_spot_check'])"
done
