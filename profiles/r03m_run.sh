set -o pipefail
D=gpurun_out/r03m; mkdir -p $D
timeout -k 10 700 python -u -m pytest tests/test_all_sources_table_gpu.py tests/test_route_table.py tests/test_table_repair.py tests/test_allsources.py tests/test_abi_gpu.py -x -q --timeout 300 --timeout-method thread -m gpu > $D/gpu_tests.log 2>&1; rc=$?
tail -3 $D/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --no-cpu-baseline --no-route-db --no-whatif > $D/bench.json 2> $D/bench.err || exit 6
python -c "import json;d=json.load(open('$D/bench.json'));print(d['ms_per_step']);print(json.dumps(d['wan_all_sources'].get('table_repair'))[:2500])"
