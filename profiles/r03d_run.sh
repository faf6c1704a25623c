set -o pipefail
D=gpurun_out/r03d; mkdir -p $D
timeout -k 10 600 python -u -m pytest tests/test_abi_gpu.py tests/test_trace_paths_gpu.py tests/test_engine_parity_gpu.py tests/test_routedb_golden_gpu.py tests/test_config_sized_gpu.py tests/test_golden.py tests/test_cluster.py -x -q --timeout 300 --timeout-method thread > $D/gpu_tests.log 2>&1; rc=$?
tail -5 $D/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --no-cpu-baseline --no-wan --no-whatif --no-repair > $D/bench.json 2> $D/bench.err || exit 6
python -c "import json;d=json.load(open('$D/bench.json'));print(d['ms_per_step'],d.get('kernels'));print(json.dumps(d.get('ksp2_route_db'))[:1700]);print(json.dumps(d.get('route_db_rebuild'))[:300])"
OPENR_NL_SWAR=0 timeout -k 10 200 python bench.py --no-cpu-baseline --no-route-db --no-wan --no-whatif --no-repair > $D/fab_noswar.json 2> $D/fab_noswar.err || exit 7
python -c "import json;d=json.load(open('$D/fab_noswar.json'));print('noswar',d['ms_per_step'],d.get('kernels'))"
