"""Parse rocprofv3 PMC passes into profiles/<round>/pmc_traffic.json.

The passes themselves run on the GPU box (one counter group per pass, as the
MI355X guide requires), e.g.:

  cd /tmp && export TMPDIR=/tmp
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -T -d $R/gpurun_out/pmc_fetch \
      -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 \
      --no-route-db --no-cpu-baseline
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -T -d $R/gpurun_out/pmc_write ...
  python $R/profiles/collect_pmc.py $R/gpurun_out/pmc_fetch $R/gpurun_out/pmc_write \
      $R/profiles/r01/pmc_traffic.json

HBM bytes per launch = 2 * FETCH_SIZE + WRITE_SIZE (kB units in rocprofv3;
FETCH_SIZE is doubled: on gfx950 it reports exactly half the bytes of wide
coalesced reads — MI355X_MICROARCH.md, "HBM").  Averaged over the dispatches
of each kernel.
"""

from __future__ import annotations

import csv
import glob
import json
import os
import sys
from collections import defaultdict


def _rows(d):
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            yield from csv.DictReader(fh)


def _short(name):
    n = name.split("(")[0].strip()
    n = n.replace("void ", "").replace("(anonymous namespace)::", "")
    return n.split("<")[0].split("::")[-1]


def per_dispatch(d, counter):
    """{kernel: [value per dispatch, in dispatch order]} (kB)."""
    acc = defaultdict(lambda: defaultdict(float))
    for r in _rows(d):
        if r.get("Counter_Name") != counter:
            continue
        k = _short(r.get("Kernel_Name", ""))
        disp = r.get("Dispatch_Id") or r.get("Correlation_Id") or str(len(acc[k]))
        acc[k][disp] += float(r.get("Counter_Value", 0) or 0)
    return {k: [v[x] for x in sorted(v, key=lambda x: int(x) if str(x).isdigit() else 0)]
            for k, v in acc.items() if v}


def main(fetch_dir, write_dir, out):
    fetch = per_dispatch(fetch_dir, "FETCH_SIZE")
    write = per_dispatch(write_dir, "WRITE_SIZE")
    kernels = {}
    for k in sorted(set(fetch) | set(write)):
        f = fetch.get(k)
        w = write.get(k)
        f_kb = sum(f) / len(f) if f else None
        w_kb = sum(w) / len(w) if w else None
        ent = {"FETCH_SIZE_kB": f_kb, "WRITE_SIZE_kB": w_kb}
        if f_kb is not None and w_kb is not None:
            ent["hbm_bytes_per_launch"] = int(round((2.0 * f_kb + w_kb) * 1024.0))
            # the largest dispatch (kernels launched at several sizes, e.g.
            # a warm-up batch before the measured one)
            ent["hbm_bytes_largest_launch"] = int(round((2.0 * max(f) + max(w)) * 1024.0))
            # and the smallest (a kernel run in two modes, e.g. the route
            # table with and without LFA columns)
            ent["hbm_bytes_smallest_launch"] = int(round((2.0 * min(f) + min(w)) * 1024.0))
            ent["dispatches"] = len(f)
        kernels[k] = ent
    json.dump(
        {
            "what": "per-launch HBM bytes from rocprofv3 PMC passes "
            "(2*FETCH_SIZE + WRITE_SIZE, kB->bytes, gfx950 FETCH_SIZE correction)",
            "kernels": kernels,
        },
        open(out, "w"),
        indent=1,
    )
    print(json.dumps(kernels, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:4])
