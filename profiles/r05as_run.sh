set -o pipefail
# KSP2 heavy trace v2 (register frames + LDS batch cache; build only below
# the destination's distance): parity, budget sweep, kernel trace
D=gpurun_out/r05as; mkdir -p $D
R=$(pwd)
timeout -k 10 400 python -u -m pytest tests/test_trace_paths_gpu.py tests/test_engine_parity_gpu.py tests/test_routedb_golden_gpu.py -k "trace or ksp2" -m gpu -x -q --timeout 300 --timeout-method thread > $D/gpu_tests.log 2>&1 || { tail -30 $D/gpu_tests.log; exit 2; }
tail -1 $D/gpu_tests.log
timeout -k 10 400 python3 profiles/ksp2_budget_probe.py "" "OPENR_SPF_TRACE_DYN=0" "OPENR_SPF_TRACE_BUDGET=512" "OPENR_SPF_TRACE_BUDGET=768" "" > $D/sweep.json 2> $D/sweep.err || { tail -5 $D/sweep.err; exit 3; }
cat $D/sweep.json; grep "trace heavy" $D/sweep.err | tail -8
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d $R/$D/trace -o run --output-format csv -- python3 $R/profiles/ksp2_budget_probe.py "" > $R/$D/trace.json 2>&1 || exit 4
cd $R
head -6 $(find $D/trace -name "*kernel_stats.csv" | head -1)
