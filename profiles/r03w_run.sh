set -o pipefail
D=gpurun_out/r03w; mkdir -p $D
timeout -k 10 300 python -u -m pytest tests/test_abi_gpu.py tests/test_zero_metric_plan.py -x -q --timeout 200 --timeout-method thread > $D/gpu_tests.log 2>&1; rc=$?
tail -2 $D/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
OPENR_MS_LVL_ONLY=1 timeout -k 10 400 python -u -m pytest tests/test_abi_gpu.py tests/test_config_sized_gpu.py -x -q --timeout 300 --timeout-method thread > $D/gpu_tests_lvl.log 2>&1; rc=$?
tail -2 $D/gpu_tests_lvl.log
[ $rc -eq 0 ] || exit $rc
B="bench.py --no-cpu-baseline --no-route-db --no-whatif --no-wan --steps 30 --warmup 5"
for x in 0 1 0 1; do
  OPENR_MS_LVL_ONLY=$x timeout -k 10 200 python $B > $D/lvl$x.json 2>> $D/err.log || exit 5
  python -c "import json;d=json.load(open('$D/lvl$x.json'));print('lvl_only=$x', d['ms_per_step'], d['kernels'], d['parity_spot_check'])"
done
for x in 512 1024; do
  OPENR_NL_HT=$x timeout -k 10 200 python $B > $D/ht$x.json 2>> $D/err.log || exit 6
  python -c "import json;d=json.load(open('$D/ht$x.json'));print('ht=$x', d['ms_per_step'], d['kernels']['spf_nh_levels_held_kernel'], d['parity_spot_check'])"
done
for w in 1 0; do
  OPENR_NL_WIDE=$w timeout -k 10 300 python $B --num-sws 20000 > $D/f20k_wide$w.json 2>> $D/err.log || exit 7
  python -c "import json;d=json.load(open('$D/f20k_wide$w.json'));print('20k wide=$w', d['ms_per_step'], d['kernels'], d['parity_spot_check'])"
done
