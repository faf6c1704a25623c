set -o pipefail
# round 6: the v2 pass's shallow one-add compare -- parity, A/B, kernel trace
R=$(pwd)
D=gpurun_out/r06d; mkdir -p $D
timeout -k 10 600 python -u -m pytest tests/test_nl_trit_gpu.py tests/test_abi_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $D/gpu_tests.log 2>&1 || { tail -40 $D/gpu_tests.log; exit 2; }
tail -1 $D/gpu_tests.log
timeout -k 10 300 python3 profiles/nl_ab.py 20 4 OPENR_NL_SHALLOW > $D/shallow_ab.json 2> $D/shallow_ab.err || { tail -20 $D/shallow_ab.err; exit 3; }
python3 -c "import json; d=json.load(open('$D/shallow_ab.json')); print({k:v for k,v in d.items() if k!='raw'})"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$D/kt -o run --output-format csv -- python3 $R/profiles/nl_ab.py 10 2 OPENR_NL_SHALLOW > $R/$D/kt.log 2>&1 || { tail -20 $R/$D/kt.log; exit 4; }
cd $R
python3 - <<PY
import csv, glob
f = glob.glob("$D/kt/**/*kernel_trace.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
by = {}
for r in rows:
    n = r["Kernel_Name"]
    if "v2_kernel" in n:
        by.setdefault("v2", []).append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
v = by["v2"]
# launches alternate per block of 10: shallow=1 block then shallow=0 block (warm-up 3 each first)
print("v2 launches", len(v), "first", v[:6])
PY
