set -o pipefail
# adaptive lanes per node (SSSP PUSH/PULL, what-if repair init): what-if
# probes with stats, then the GPU tests that cover spf_sssp_kernel
D=gpurun_out/${TAG:-r06s}; mkdir -p $D
timeout -k 10 200 python profiles/whatif_probe.py 5 > $D/wi.json 2> $D/wi.err || { tail -20 $D/wi.err; exit 3; }
OPENR_SPF_WHATIF_STATS=1 timeout -k 10 200 python profiles/whatif_probe.py 1 > $D/wi_stats.json 2> $D/wi_stats.err || { tail -20 $D/wi_stats.err; exit 4; }
grep "whatif stats" $D/wi_stats.err | tail -2
python3 -c "
import json
d=json.loads(open('$D/wi.json').read().strip().splitlines()[-1]); print('whatif', d['ms'], d['device_ms'], d['value'], d['parity_check'])"
timeout -k 10 200 python profiles/firsthop_probe.py 20 > $D/fh.jsonl 2> $D/fh.err || { tail -20 $D/fh.err; exit 5; }
cat $D/fh.jsonl | cut -c1-200
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ > $D/gpu_tests.log 2>&1 || { tail -40 $D/gpu_tests.log; exit 6; }
tail -2 $D/gpu_tests.log
