set -o pipefail
# round 4: RouteDb parity with the SP_ECMP fast path, then the full bench at HEAD
D=gpurun_out/r04g; mkdir -p $D
timeout -k 10 600 python -u -m pytest tests/test_routedb_golden_gpu.py tests/test_engine_parity_gpu.py -x -q --timeout 300 --timeout-method thread -m gpu > $D/gpu_tests.log 2>&1 || { tail -5 $D/gpu_tests.log; exit 4; }
tail -2 $D/gpu_tests.log
timeout -k 10 900 python bench.py > $D/bench_full.json 2> $D/bench_full.err || exit 5
python - <<'PY'
import json
d=json.load(open('gpurun_out/r04g/bench_full.json'))
print(d['value'], d['ms_per_step'], d['roofline']['frac'])
for k in ('wan_all_sources','ksp2_route_db','route_db_rebuild','whatif_batch'):
    v=d.get(k) or {}
    print(k, {x: v.get(x) for x in ('ms','spf_ms','value','ms_median','build_ms_median','loop_ms_median','parity_check','kernel')})
PY
