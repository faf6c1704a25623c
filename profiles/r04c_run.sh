set -o pipefail
# round 4: LDS-row WAN kernel sweep + byte-granular next-hop masks: new tests first
D=gpurun_out/r04c; mkdir -p $D
timeout -k 10 400 python -u profiles/quick_wan.py 8192 LDSROW=0 base LG=1 LG=2 LG=8 LG=1,LSHIFT=5 LG=1,LSHIFT=7 LG=2,LSHIFT=5 LSHIFT=5 LSHIFT=7 base > $D/quick_wan.log 2>&1 || exit 3
timeout -k 10 600 python -u -m pytest tests/test_dstep_ldsrow_gpu.py tests/test_cluster.py tests/test_abi_gpu.py tests/test_trace_paths_gpu.py tests/test_config_sized_gpu.py -x -q --timeout 300 --timeout-method thread -m gpu > $D/gpu_tests.log 2>&1; rc=$?
tail -5 $D/gpu_tests.log
exit $rc
