set -o pipefail
# round 4: trace ignore list as an LDS hash set; register rank for lists <= 64
D=gpurun_out/r04ah; mkdir -p $D
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_trace_paths_gpu.py tests/test_engine_parity_gpu.py tests/test_routedb_golden_gpu.py tests/test_cluster.py -m gpu > $D/tests.log 2>&1 || { tail -30 $D/tests.log; exit 1; }
tail -2 $D/tests.log
for i in 1 2; do
timeout -k 10 300 python3 profiles/ksp2_trace_probe.py 16 > $D/ksp2_trace.$i.log 2>&1 || exit $?
grep -E '^\{' $D/ksp2_trace.$i.log | tail -1
done
OPENR_SPF_TRACE_STATS=1 timeout -k 10 300 python3 profiles/ksp2_trace_probe.py 16 > $D/ksp2_trace_stats.log 2>&1 || exit $?
grep -E '^\{|trace stats' $D/ksp2_trace_stats.log | tail -2
