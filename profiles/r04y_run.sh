set -o pipefail
# round 4: MS-BFS with per-query ignore lists (KSP2 second passes) -- parity, then the KSP2 loop
D=gpurun_out/r04y; mkdir -p $D
timeout -k 10 900 python -u -m pytest tests/test_whatif_repair_gpu.py tests/test_abi_gpu.py tests/test_trace_paths_gpu.py tests/test_engine_parity_gpu.py \
  tests/test_routedb_golden_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $D/gpu_tests.log 2>&1; rc=$?
tail -3 $D/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 profiles/route_db_probe.py 6 > $D/route_db_probe.json 2> $D/route_db_probe.err || exit 3
python3 - <<'PY'
import json
d=[json.loads(l) for l in open('gpurun_out/r04y/route_db_probe.json') if l.startswith('{')][-1]
for k in ('route_db_rebuild','ksp2_route_db'):
    v=d[k]; print(k, {x: v.get(x) for x in ('ms_median','build_ms_median','update_ms_median','release_ms_median','parity_check')})
    print('  ', v.get('per_build_us') or v.get('per_build'))
PY
