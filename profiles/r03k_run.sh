set -o pipefail
D=gpurun_out/r03k; mkdir -p $D
timeout -k 10 400 python -u -m pytest tests/test_abi_gpu.py tests/test_cluster.py tests/test_config_sized_gpu.py tests/test_allsources.py -x -q --timeout 300 --timeout-method thread -m gpu > $D/gpu_tests.log 2>&1; rc=$?
tail -3 $D/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python profiles/scaling_probe.py > $D/scaling_probe.json 2> $D/scaling_probe.err || exit 5
cat $D/scaling_probe.json | tr -d '\n' | cut -c1-1500; echo
timeout -k 10 200 python bench.py --sharded --no-cpu-baseline --no-route-db --no-wan --no-whatif --no-repair > $D/fab_sharded.json 2> $D/fab_sharded.err || exit 6
python -c "import json;d=json.load(open('$D/fab_sharded.json'));print(d['ms_per_step'],d['value'],d['config'].get('kernel'),d.get('parity_spot_check'))"
