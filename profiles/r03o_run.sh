set -o pipefail
D=gpurun_out/r03o; mkdir -p $D
timeout -k 10 600 python -u -m pytest tests/test_zero_metric_plan.py tests/test_wide_plan.py -x -v --timeout 300 --timeout-method thread > $D/gpu_tests.log 2>&1; rc=$?
tail -5 $D/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import bench, json; print(json.dumps(bench.wide_plan(0)))" > $D/wide_plan.json 2> $D/wide_plan.err || exit 5
cat $D/wide_plan.json
timeout -k 10 900 python bench.py --cpu-full --no-route-db --no-wan --no-whatif --no-repair > $D/cpu_full.json 2> $D/cpu_full.err || exit 6
python -c "import json;d=json.load(open('$D/cpu_full.json'));print(json.dumps(d.get('cpu_baseline'))[:3000])"
