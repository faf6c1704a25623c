set -o pipefail
D=gpurun_out/r03u; mkdir -p $D
timeout -k 10 600 python -u -m pytest tests/test_golden.py tests/test_routedb_golden_gpu.py tests/test_route_table.py tests/test_engine_parity_gpu.py -x -q --timeout 300 --timeout-method thread > $D/gpu_tests.log 2>&1; rc=$?
tail -2 $D/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
timeout -k 10 120 python -c "import bench, json; print(json.dumps(bench.grid_route_db(0, iters=40)))" >> $D/grid.json 2>> $D/grid.err || exit 5
done
cat $D/grid.json
