set -o pipefail
D=gpurun_out/r03r; mkdir -p $D
timeout -k 10 300 python -u -m pytest tests/test_abi_gpu.py -x -q --timeout 200 --timeout-method thread -k "swar or msbfs or levels" > $D/gpu_tests.log 2>&1; rc=$?
tail -2 $D/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
B="bench.py --no-cpu-baseline --no-route-db --no-whatif --no-wan --steps 30 --warmup 5"
for x in 1 2 3 5 10 1; do
  OPENR_NL_CPB=$x timeout -k 10 200 python $B > $D/cpb$x.json 2>> $D/err.log || exit 5
  python -c "import json;d=json.load(open('$D/cpb$x.json'));print('cpb=$x', d['ms_per_step'], d['kernels']['spf_nh_levels_held_kernel'], d['parity_spot_check'])"
done
