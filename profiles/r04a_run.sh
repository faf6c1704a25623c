set -o pipefail
# round 4: first run of the LDS-resident delta-stepping plan (spf_dlds_kernel)
D=gpurun_out/r04a; mkdir -p $D
timeout -k 10 400 python -u profiles/quick_wan.py 8192 base LDSROW=0 LSHIFT=3 LSHIFT=5 LSHIFT=6 LSHIFT=8 STATS=1 > $D/quick_wan.log 2>&1 || exit 3
timeout -k 10 400 python -u -m pytest tests/test_dstep_ldsrow_gpu.py -x -v --timeout 120 --timeout-method thread > $D/tests.log 2>&1; rc=$?
tail -5 $D/tests.log
exit $rc
