#!/bin/bash
# Fabric step: SQ / TCC counter passes for the kernel analysis (one block
# group per pass, each under its own KILL timeout).  Usage from the repo
# root on the GPU box: bash profiles/prof_fabric_sq.sh <tag>
set -e
R=$(pwd)
TAG=${1:-r03}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
B="$R/bench.py --no-cpu-baseline --no-route-db --no-whatif --no-wan --steps 3 --warmup 1"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INSTS_VALU SQ_INSTS_VMEM_WR \
  -T -d $OUT/pmc_sq -o run --output-format csv -- python3 $B > $OUT/pmc_sq.json
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT \
  -T -d $OUT/pmc_tcc -o run --output-format csv -- python3 $B > $OUT/pmc_tcc.json
cd $R
python3 - "$OUT" <<'PY'
import csv, glob, json, os, sys
from collections import defaultdict
out = sys.argv[1]
acc = defaultdict(lambda: defaultdict(list))
for d in ("pmc_sq", "pmc_tcc"):
    for f in glob.glob(os.path.join(out, d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r.get("Kernel_Name", "").split("(")[0].replace("void ", "").split("<")[0].split("::")[-1]
            acc[k][r["Counter_Name"]].append(float(r.get("Counter_Value") or 0))
res = {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in acc.items()
       if k.startswith("spf_")}
json.dump(res, open(os.path.join(out, "sq_counters.json"), "w"), indent=1)
for k, cs in res.items():
    print(k, {c: round(v) for c, v in cs.items()})
PY
