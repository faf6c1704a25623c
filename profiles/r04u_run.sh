set -o pipefail
# round 4: ignore lists as an LDS hash set in spf_sssp_kernel (KSP2 second passes):
# ignore-list / KSP2 / what-if parity, then the KSP2 + RouteDb loops and the what-if batch
D=gpurun_out/r04u; mkdir -p $D
timeout -k 10 900 python -u -m pytest tests/test_abi_gpu.py tests/test_whatif_repair_gpu.py tests/test_trace_paths_gpu.py \
  tests/test_engine_parity_gpu.py tests/test_routedb_golden_gpu.py tests/test_config_sized_gpu.py -m gpu -x -q \
  --timeout 300 --timeout-method thread > $D/gpu_tests.log 2>&1; rc=$?
tail -3 $D/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 profiles/route_db_probe.py 6 > $D/route_db_probe.json 2> $D/route_db_probe.err || exit 3
python3 - <<'PY'
import json
d=[json.loads(l) for l in open('gpurun_out/r04u/route_db_probe.json') if l.startswith('{')][-1]
for k in ('route_db_rebuild','ksp2_route_db'):
    v=d[k]; print(k, {x: v.get(x) for x in ('ms_median','build_ms_median','update_ms_median','release_ms_median','parity_check')})
    print('  ', v.get('per_build_us') or v.get('per_build'))
PY
timeout -k 10 240 python3 profiles/whatif_probe.py 3 > $D/whatif.log 2>&1 || exit 6
grep '^{' $D/whatif.log | cut -c1-400
