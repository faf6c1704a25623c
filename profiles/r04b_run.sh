set -o pipefail
# round 4: pipelined spf_dlds_kernel, lanes per node / bucket width sweep
D=gpurun_out/r04b; mkdir -p $D
timeout -k 10 500 python -u profiles/quick_wan.py 8192 LDSROW=0 base LG=1 LG=2 LG=8 LG=1,LSHIFT=5 LG=1,LSHIFT=7 LG=2,LSHIFT=5 LG=2,LSHIFT=7 LSHIFT=5 LSHIFT=7 base > $D/quick_wan.log 2>&1 || exit 3
timeout -k 10 400 python -u -m pytest tests/test_dstep_ldsrow_gpu.py -x -v --timeout 120 --timeout-method thread > $D/tests.log 2>&1; rc=$?
tail -5 $D/tests.log
exit $rc
