"""Per-dispatch means of every PMC counter recorded for one kernel under a
directory of rocprofv3 passes: python profiles/pmc_summary.py <dir> <kernel>"""

import csv
import glob
import json
import os
import sys
from collections import defaultdict


def main(d, kernel):
    acc = defaultdict(lambda: defaultdict(float))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if kernel not in r.get("Kernel_Name", ""):
                continue
            disp = r.get("Dispatch_Id") or r.get("Correlation_Id")
            acc[r["Counter_Name"]][(f, disp)] += float(r.get("Counter_Value", 0) or 0)
    out = {k: {"mean": sum(v.values()) / len(v), "dispatches": len(v)} for k, v in sorted(acc.items())}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
