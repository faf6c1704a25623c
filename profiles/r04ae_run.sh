set -o pipefail
# round 4: trace store-wait flags out of scratch (macro, not a lambda)
D=gpurun_out/r04ae; mkdir -p $D
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_trace_paths_gpu.py tests/test_engine_parity_gpu.py tests/test_routedb_golden_gpu.py -m gpu > $D/tests.log 2>&1 || { tail -30 $D/tests.log; exit 1; }
tail -3 $D/tests.log
OPENR_SPF_TRACE_STATS=1 timeout -k 10 300 python3 profiles/ksp2_trace_probe.py 16 > $D/ksp2_trace.log 2>&1; rc=$?
grep -E '^\{|trace stats' $D/ksp2_trace.log | tail -4
[ $rc = 0 ] || exit $rc
timeout -k 10 300 python3 profiles/ksp2_trace_probe.py 16 > $D/ksp2_trace_nostats.log 2>&1; rc=$?
grep -E '^\{' $D/ksp2_trace_nostats.log | tail -2
exit $rc
