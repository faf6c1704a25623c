set -o pipefail
# round 4: trace store waits split vs joined, same box (A/B/A/B); the
# OPENR_SPF_TRACE_JOIN knob was removed after this run (no difference)
D=gpurun_out/r04af; mkdir -p $D
for i in 1 2; do
for j in 0 1; do
OPENR_SPF_TRACE_JOIN=$j timeout -k 10 300 python3 profiles/ksp2_trace_probe.py 16 > $D/ksp2_trace_join$j.$i.log 2>&1 || exit $?
echo "join=$j $(grep -E '^\{' $D/ksp2_trace_join$j.$i.log | tail -1)"
done
done
