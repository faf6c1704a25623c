set -o pipefail
D=gpurun_out/r03p; mkdir -p $D
timeout -k 10 600 python -u -m pytest tests/test_table_repair.py tests/test_all_sources_table_gpu.py tests/test_allsources.py -x -q --timeout 300 --timeout-method thread > $D/gpu_tests.log 2>&1; rc=$?
tail -3 $D/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --no-cpu-baseline --no-route-db --no-whatif > $D/bench_wan.json 2> $D/bench_wan.err || exit 5
python -c "import json;d=json.load(open('$D/bench_wan.json'));w=d['wan_all_sources'];print(w['ms'], w['kernel']);print(json.dumps(w['table_repair']))"
