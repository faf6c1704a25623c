#!/bin/bash
# FETCH_SIZE / WRITE_SIZE calibration (profiles/calib/fetch_calib.hip) on the
# GPU box, from the repo root: one PMC pass per counter, then the ratio of
# counted to touched bytes per kernel -> gpurun_out/calib/calib.json
set -e
R=$(pwd)
OUT=$R/gpurun_out/calib
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE -T -d $OUT/fetch -o run --output-format csv -- \
  $R/profiles/calib/fetch_calib > $OUT/fetch.log 2>&1
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE -T -d $OUT/write -o run --output-format csv -- \
  $R/profiles/calib/fetch_calib > $OUT/write.log 2>&1
cd $R
python3 - <<'PY'
import json, sys
sys.path.insert(0, "profiles")
from collect_pmc import per_dispatch
R = "gpurun_out/calib"
B = float(1 << 30)
f = per_dispatch(R + "/fetch", "FETCH_SIZE")
w = per_dispatch(R + "/write", "WRITE_SIZE")
out = {"bytes_touched_per_kernel": int(B), "kernels": {}}
for k in sorted(set(f) | set(w)):
    ent = {}
    if f.get(k):
        ent["FETCH_SIZE_bytes"] = [v * 1024 for v in f[k]]
        ent["fetch_over_touched"] = round(sum(f[k]) / len(f[k]) * 1024 / B, 4)
    if w.get(k):
        ent["WRITE_SIZE_bytes"] = [v * 1024 for v in w[k]]
        ent["write_over_touched"] = round(sum(w[k]) / len(w[k]) * 1024 / B, 4)
    out["kernels"][k] = ent
json.dump(out, open(R + "/calib.json", "w"), indent=1)
print(json.dumps({k: {x: y for x, y in v.items() if "over" in x} for k, v in out["kernels"].items()}))
PY
