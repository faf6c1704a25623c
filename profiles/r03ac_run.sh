set -o pipefail
D=gpurun_out/r03ac; mkdir -p $D
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $D/smoke.log 2>&1 || exit 4
tail -1 $D/smoke.log
timeout -k 10 300 python -u -m pytest tests/test_abi_gpu.py tests/test_zero_metric_plan.py -x -q --timeout 200 --timeout-method thread > $D/gpu_tests.log 2>&1; rc=$?
tail -2 $D/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py > $D/bench_full.json 2> $D/bench_full.err || exit 5
python -c "import json;d=json.load(open('$D/bench_full.json'));print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['traffic_source'], d['roofline'].get('traffic_over_algorithmic'))"
