set -o pipefail
# round 6: patch kernel without the agent fence (parity + A/B + trace), and
# PMC traffic of the v2 pass with and without the 2-bit neighbour rows
R=$(pwd)
D=gpurun_out/r06i; mkdir -p $D
timeout -k 10 900 python -u -m pytest tests/test_whatif_repair_gpu.py tests/test_golden.py -m gpu -x -q --timeout 300 --timeout-method thread > $D/gpu_tests.log 2>&1 || { tail -40 $D/gpu_tests.log; exit 2; }
tail -1 $D/gpu_tests.log
for M in 1 0 1 0; do
  OPENR_SPF_WHATIF_PATCH=$M timeout -k 10 300 python3 profiles/whatif_probe.py 5 > $D/wi_patch$M.json 2> $D/wi_patch$M.err || { tail -20 $D/wi_patch$M.err; exit 3; }
  python3 -c "import json; d=json.loads(open('$D/wi_patch$M.json').read().strip().splitlines()[-1]); print('patch=$M', d['ms'], d['device_ms'], d['value'], d['parity_check'], d['screened_queries'])"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$D/kt -o run --output-format csv -- python3 $R/profiles/whatif_probe.py 5 > $R/$D/kt.log 2>&1 || { tail -20 $R/$D/kt.log; exit 5; }
for P in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 200 rocprofv3 --pmc $P -T -d $R/$D/trit_$P -o run --output-format csv -- python3 $R/profiles/nl_ab.py 5 1 OPENR_NL_TRIT > $R/$D/trit_$P.log 2>&1 || { tail -20 $R/$D/trit_$P.log; exit 6; }
done
cd $R
python3 - <<PY
import csv, glob
f = glob.glob("$D/kt/**/*kernel_stats.csv", recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:8]:
    print(r["Name"][:70], r["Calls"], r["AverageNs"], r["TotalDurationNs"])
PY
python3 profiles/collect_pmc.py $D/trit_FETCH_SIZE $D/trit_WRITE_SIZE $D/pmc_trit.json || exit 7
python3 -c "
import json
d=json.load(open('$D/pmc_trit.json'))
for k,v in d['kernels'].items():
    if 'v2' in k or 'trit' in k or 'msbfs' in k: print(k[:80], v)
"
