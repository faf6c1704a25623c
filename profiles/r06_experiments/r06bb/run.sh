set -o pipefail
# 16-byte what-if row copies (block_copy_v): repair phase stats, batch time,
# what-if parity tests
D=gpurun_out/r06bb; mkdir -p $D
OPENR_SPF_WHATIF_STATS=1 timeout -k 10 200 python3 profiles/whatif_probe.py 3 > $D/wi_stats.json 2> $D/stats.txt || exit 3
grep "whatif stats" $D/stats.txt | tail -2
for i in 1 2; do timeout -k 10 200 python3 profiles/whatif_probe.py 8 > $D/wi_$i.json 2>/dev/null || exit 4; python3 -c "import json; j=json.load(open('$D/wi_$i.json')); print(j['ms'], j['device_ms'], j['parity_check'])"; done
timeout -k 10 600 python3 -u -m pytest tests/test_whatif_repair_gpu.py tests/test_whatif_firsthop_gpu.py tests/test_abi_gpu.py -x -q --timeout 120 --timeout-method thread -k "whatif or repair or screen or firsthop or source_link" > $D/t.log 2>&1 || { tail -30 $D/t.log; exit 6; }
tail -1 $D/t.log
