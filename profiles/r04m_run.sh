set -o pipefail
# round 4: what-if split probe (baseline plan, repair on/off by K size)
D=gpurun_out/r04m; mkdir -p $D
timeout -k 10 300 python3 profiles/whatif_split_probe.py > $D/split.log 2>&1; rc=$?
cat $D/split.log | grep '^{'
exit $rc
