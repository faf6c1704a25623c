set -o pipefail
# round 4: dlds two-node prefetch sweep + the targeted GPU tests
D=gpurun_out/r04e; mkdir -p $D
timeout -k 10 400 python -u profiles/quick_wan.py 8192 base LPF=0 LG=2 LG=2,LPF=0 LSHIFT=6 LG=2,LSHIFT=6 LG=8 base > $D/quick_wan.log 2>&1 || exit 3
timeout -k 10 800 python -u -m pytest tests/test_dstep_ldsrow_gpu.py tests/test_trace_paths_gpu.py tests/test_all_sources_table_gpu.py tests/test_table_repair.py tests/test_engine_parity_gpu.py -x -q --timeout 300 --timeout-method thread -m gpu > $D/gpu_tests.log 2>&1; rc=$?
tail -5 $D/gpu_tests.log
exit $rc
