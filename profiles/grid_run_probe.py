"""Where the grid RouteDb batch's host time goes: one 13-row query on the
10x10 grid (node 1, its neighbours and theirs, next hops) rerun N times --
run+sync alone, then with the row and mask fetches -- against its device time.

  python profiles/grid_run_probe.py [N]
"""
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: F401,E402

from openr_amd import abi  # noqa: E402
from openr_amd import topologies as TP  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
topo = TP.grid(10)
csr = topo.csr()
g = abi.Graph(csr)
r_, _ = topo.rank()
src = [int(r_[topo.names.index(x)]) for x in ("1", "0", "2", "11")]
q = g.query(src, abi.SPF_F_NEXTHOPS)
q.run()
V = csr.num_nodes
rows = np.zeros(len(src) * V, dtype=np.uint32)
out = {"kernel": q.kernel, "kernels": q.kernels()}


def timed(fn):
    for _ in range(50):
        fn()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    return round((time.perf_counter() - t) / n * 1e6, 2)


out["run_sync_us"] = timed(lambda: q.run())
out["device_us"] = round(q.elapsed_ms() * 1e3, 2)
out["run_nosync_us"] = timed(lambda: (q.run(sync=False), q.sync()))
out["fetch_rows_us"] = timed(lambda: q.fetch_rows(0, len(src), rows.ctypes.data, V * 4, on_device=False))
out["fetch_nexthops_us"] = timed(lambda: q.fetch_nexthops(0, len(src)))
out["run_fetch_us"] = timed(lambda: (q.run(), q.fetch_rows(0, len(src), rows.ctypes.data, V * 4, on_device=False),
                                     q.fetch_nexthops(0, len(src))))
print(json.dumps(out), flush=True)
