"""Probe: run only bench.py's what-if batch (BASELINE configs[4]) on one GPU,
so PMC passes over it see the what-if plan's kernels alone.  Prints the
section's JSON; with --batches-out FILE also writes the number of batch runs
(warm-up + timed), which profiles/collect_pmc.py's output needs to turn
summed dispatch bytes into bytes per batch.

  python profiles/whatif_probe.py [STEPS] [--batches-out FILE]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def main():
    args = sys.argv[1:]
    out = None
    if "--batches-out" in args:
        i = args.index("--batches-out")
        out = args[i + 1]
        del args[i:i + 2]
    steps = int(args[0]) if args else 3
    r = bench.whatif_batch(1, 0, 0, None, steps=steps, cpu_lines=False)
    print(json.dumps(r), flush=True)
    if out:
        with open(out, "w") as f:
            json.dump({"batches": steps + 1}, f)


if __name__ == "__main__":
    main()
