set -o pipefail
# round 6: patch kernel phase ticks
D=gpurun_out/r06j; mkdir -p $D
OPENR_SPF_WHATIF_STATS=1 timeout -k 10 300 python3 profiles/whatif_probe.py 1 > $D/wi_stats.json 2> $D/wi_stats.err || { tail -20 $D/wi_stats.err; exit 4; }
grep "whatif patch\|whatif stats" $D/wi_stats.err | tail -8
