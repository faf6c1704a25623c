set -o pipefail
# round 5: KSP2 device-trace step budget (deep queries traced on the host),
# upload_weights sub-phases of the link-flap rebuild
D=gpurun_out/r05r; mkdir -p $D
timeout -k 10 600 python -u -m pytest tests/test_engine_parity_gpu.py tests/test_trace_paths_gpu.py tests/test_routedb_golden_gpu.py -k "ksp2 or trace or kth" -m gpu -x -q --timeout 300 --timeout-method thread > $D/gpu_tests.log 2>&1 || { tail -30 $D/gpu_tests.log; exit 3; }
tail -1 $D/gpu_tests.log
for b in 4096 1024 100000000; do
OPENR_SPF_TRACE_BUDGET=$b timeout -k 10 300 python3 profiles/route_db_probe.py 6 > $D/rdb.b$b.json 2> $D/rdb.b$b.err || { tail -5 $D/rdb.b$b.err; exit 2; }
python3 -c "
import json; d=json.loads(open('$D/rdb.b$b.json').read().strip().split('\n')[-1])
k=d['ksp2_route_db']; print('budget=$b', 'ksp2', k['ms_median'], k['build_ms_median'], {x: k.get('per_build',{}).get(x) for x in ('kth2_device_trace_us','kth2_trace_us','kth2_device_overflows','ksp2_paths_us','ksp2_nexthops_us')}, k.get('parity_check'))"
done
OPENR_SPF_CREATE_TIMING=1 timeout -k 10 300 python3 profiles/linkflap_probe.py > $D/linkflap.json 2> $D/linkflap.err || { tail -5 $D/linkflap.err; exit 4; }
python3 -c "import json; d=json.load(open('$D/linkflap.json')); print({k: d.get(k) for k in ('ms_median','update_ms_median','build_ms_median','parity_check')})"
grep "spf_graph_update" $D/linkflap.err | tail -13
