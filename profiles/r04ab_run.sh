set -o pipefail
# round 4: where the KSP2 device-trace time goes (OPENR_SPF_TRACE_STATS)
D=gpurun_out/r04ab; mkdir -p $D
OPENR_SPF_TRACE_STATS=1 timeout -k 10 300 python3 profiles/ksp2_trace_probe.py 16 > $D/ksp2_trace.log 2>&1; rc=$?
grep -E '^\{|trace stats' $D/ksp2_trace.log | tail -6
exit $rc
