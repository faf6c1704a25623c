set -o pipefail
# round 6: wave-per-query what-if patch -- parity, ticks, A/B, trace
R=$(pwd)
D=gpurun_out/r06l; mkdir -p $D
timeout -k 10 900 python -u -m pytest tests/test_whatif_repair_gpu.py tests/test_golden.py -m gpu -x -q --timeout 300 --timeout-method thread > $D/gpu_tests.log 2>&1 || { tail -40 $D/gpu_tests.log; exit 2; }
tail -1 $D/gpu_tests.log
OPENR_SPF_WHATIF_STATS=1 timeout -k 10 300 python3 profiles/whatif_probe.py 1 > $D/wi_stats.json 2> $D/wi_stats.err || { tail -20 $D/wi_stats.err; exit 4; }
grep "whatif patch" $D/wi_stats.err | tail -2
for M in 1 0 1 0; do
  OPENR_SPF_WHATIF_PATCH=$M timeout -k 10 300 python3 profiles/whatif_probe.py 5 > $D/wi_patch$M.json 2> $D/wi_patch$M.err || { tail -20 $D/wi_patch$M.err; exit 3; }
  python3 -c "import json; d=json.loads(open('$D/wi_patch$M.json').read().strip().splitlines()[-1]); print('patch=$M', d['ms'], d['device_ms'], d['value'], d['parity_check'], d['screened_queries'])"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$D/kt -o run --output-format csv -- python3 $R/profiles/whatif_probe.py 5 > $R/$D/kt.log 2>&1 || { tail -20 $R/$D/kt.log; exit 5; }
cd $R
python3 - <<PY
import csv, glob
f = glob.glob("$D/kt/**/*kernel_stats.csv", recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:10]:
    print(r["Name"][:70], r["Calls"], r["AverageNs"], r["TotalDurationNs"])
PY
