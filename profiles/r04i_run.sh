set -o pipefail
# round 4: RouteDb parity with the ECMP + label fast paths; kernel trace of the RouteDb / KSP2 sections
D=gpurun_out/r04i; mkdir -p $D
timeout -k 10 600 python -u -m pytest tests/test_trace_paths_gpu.py tests/test_routedb_golden_gpu.py tests/test_engine_parity_gpu.py tests/test_route_table.py -x -q --timeout 300 --timeout-method thread -m gpu > $D/gpu_tests.log 2>&1 || { tail -5 $D/gpu_tests.log; exit 4; }
tail -2 $D/gpu_tests.log
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T -d $R/$D/trace -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-wan --no-whatif > $R/$D/bench_rdb.json 2> $R/$D/bench_rdb.err || exit 5
cd $R
cp $(find $D/trace -name "*kernel_stats.csv" | head -1) $D/kernel_stats.csv
head -12 $D/kernel_stats.csv
python - <<'PY'
import json
d=json.load(open('gpurun_out/r04i/bench_rdb.json'))
for k in ('ksp2_route_db','route_db_rebuild'):
    v=d.get(k) or {}
    print(k, v.get('ms_median'), v.get('build_ms_median'), v.get('release_ms_median'), v.get('per_build_us') or v.get('per_build'))
PY
