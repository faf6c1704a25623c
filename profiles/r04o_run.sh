set -o pipefail
# round 4: what-if repair phase split (OPENR_SPF_WHATIF_STATS) + route table build split
D=gpurun_out/r04o; mkdir -p $D
OPENR_SPF_WHATIF_STATS=1 timeout -k 10 200 python3 profiles/whatif_probe.py 1 > $D/wi_stats.log 2>&1 || exit 3
grep -E "whatif stats|\"ms\"" $D/wi_stats.log | cut -c1-400
timeout -k 10 200 python3 profiles/route_table_probe.py --breakdown > $D/rt_breakdown.log 2>&1 || exit 5
tail -1 $D/rt_breakdown.log
