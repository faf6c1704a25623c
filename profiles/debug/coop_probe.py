"""Cooperative MS-BFS diagnostics: per (block size, P cap), does the barrier
complete, how long does the block take, and do the rows equal the
one-workgroup-per-batch kernel's."""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.getcwd())
from openr_amd import abi
from openr_amd import topologies as TP

topo = TP.fabric(10000)
csr = topo.csr()
V = csr.num_nodes
g = abi.Graph(csr)
out = []
for N in (8, 4, 2, 1):
    n = (V + N - 1) // N
    first = (N // 2) * n if N > 1 else 0
    srcs = np.arange(first, min(V, first + n), dtype=np.uint32)
    os.environ["OPENR_MS_COOP"] = "0"
    q0 = g.query(srcs, abi.SPF_F_NEXTHOPS).run()
    ref = [(q0.dist(i), q0.nexthops(i)) for i in (0, len(srcs) // 2, len(srcs) - 1)]
    q0.close()
    for pmax in ("2", "4", "8", "16"):
        os.environ["OPENR_MS_COOP"] = "1"
        os.environ["OPENR_MS_COOP_PMAX"] = pmax
        rec = {"N": N, "sources": int(len(srcs)), "pmax": int(pmax)}
        try:
            q = g.query(srcs, abi.SPF_F_NEXTHOPS)
            t0 = time.perf_counter()
            q.run()
            rec["first_run_ms"] = round((time.perf_counter() - t0) * 1e3, 3)
            for _ in range(3):
                q.run()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(20):
                q.run(sync=False)
            q.sync()
            rec["ms"] = round((time.perf_counter() - t0) / 20 * 1e3, 4)
            rec["stage_ms"] = [round(x, 4) for x in q.stage_ms()]
            rec["same"] = all((q.dist(i) == d).all() and (q.nexthops(i) == m).all()
                              for i, (d, m) in zip((0, len(srcs) // 2, len(srcs) - 1), ref))
            q.close()
        except abi.SpfError as e:
            rec["error"] = str(e)
        out.append(rec)
        print(json.dumps(rec), flush=True)
