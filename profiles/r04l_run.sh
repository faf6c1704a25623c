set -o pipefail
# round 4: what-if repair mode -- parity (new repair tests + every ignore-list
# / KSP2 / what-if GPU test), then the what-if batch timing and kernel trace
D=gpurun_out/r04l; mkdir -p $D
timeout -k 10 600 python -u -m pytest tests/test_whatif_repair_gpu.py tests/test_abi_gpu.py tests/test_trace_paths_gpu.py \
  tests/test_engine_parity_gpu.py tests/test_routedb_golden_gpu.py tests/test_config_sized_gpu.py -m gpu -x -q \
  --timeout 300 --timeout-method thread > $D/gpu_tests.log 2>&1; rc=$?
tail -3 $D/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
R=$(pwd); cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -T -d $R/$D/wi_trace -o run --output-format csv -- \
  python3 $R/profiles/whatif_probe.py 5 > $R/$D/wi_trace.log 2>&1 || exit 4
cd $R
grep '"config"' $D/wi_trace.log | cut -c1-1200
cut -d, -f1-5 $(find $D/wi_trace -name "*kernel_stats.csv" | head -1)
timeout -k 10 200 python3 profiles/route_table_probe.py --breakdown > $D/rt_breakdown.log 2>&1 || exit 5
tail -1 $D/rt_breakdown.log
