set -o pipefail
# round 4: batched cursor trace, default build without instrumentation (STATS template)
D=gpurun_out/r04ag; mkdir -p $D
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_trace_paths_gpu.py tests/test_engine_parity_gpu.py -m gpu > $D/tests.log 2>&1 || { tail -30 $D/tests.log; exit 1; }
tail -2 $D/tests.log
for i in 1 2; do
timeout -k 10 300 python3 profiles/ksp2_trace_probe.py 16 > $D/ksp2_trace.$i.log 2>&1 || exit $?
grep -E '^\{' $D/ksp2_trace.$i.log | tail -1
done
OPENR_SPF_TRACE_STATS=1 timeout -k 10 300 python3 profiles/ksp2_trace_probe.py 16 > $D/ksp2_trace_stats.log 2>&1 || exit $?
grep -E '^\{|trace stats' $D/ksp2_trace_stats.log | tail -2
