set -o pipefail
D=gpurun_out/r03v; mkdir -p $D
timeout -k 10 300 python -u profiles/debug/coop_probe.py > $D/coop_probe.jsonl 2> $D/coop_probe.err; rc=$?
cat $D/coop_probe.jsonl
exit $rc
