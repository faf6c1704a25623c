set -o pipefail
# round 4: KSP2 memo fills on the host pool (parity), then device traces vs waves per CU
D=gpurun_out/r04aa; mkdir -p $D
timeout -k 10 700 python -u -m pytest tests/test_engine_parity_gpu.py tests/test_routedb_golden_gpu.py tests/test_trace_paths_gpu.py tests/test_route_table.py -m gpu -x -q \
  --timeout 300 --timeout-method thread > $D/gpu_tests.log 2>&1; rc=$?
tail -2 $D/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 profiles/ksp2_trace_probe.py 16 8 4 > $D/ksp2_trace.log 2>&1; rc=$?
grep '^{' $D/ksp2_trace.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 bench.py --sharded --no-cpu-baseline --no-route-db --steps 5 --warmup 2 > $D/bench_sharded.json 2> $D/bench_sharded.err || exit 4
python3 -c "import json;d=json.load(open('$D/bench_sharded.json'));print('sharded', d['value'], d['ms_per_step'], d.get('parity_spot_check'), d['wan_all_sources'].get('parity_check'), d['wan_all_sources'].get('ms'), d['whatif_batch'].get('ms'), d['whatif_batch'].get('parity_check'))"
timeout -k 10 200 python3 profiles/route_table_probe.py --breakdown > $D/rt_breakdown.log 2>&1 || exit 6
tail -1 $D/rt_breakdown.log
