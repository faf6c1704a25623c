"""What one rank of an N-GPU fabric table computes: a middle block of
ceil(9976/N) sources as one query on one GPU (msbfs+levels with its helper
rows), timed over 20 launches, with the cooperative MS-BFS split
(OPENR_MS_COOP=1, default) and without it.  Emulates the per-rank device work
of bench.py's fabric_sharded at N = 1, 2, 4, 8 on a one-GPU box."""
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
out = {}
for N in (1, 2, 4, 8):
    n = (V + N - 1) // N
    for coop in ("1", "0"):
        os.environ["OPENR_MS_COOP"] = coop
        # a middle block (the first block holds the SSWs)
        first = (N // 2) * n if N > 1 else 0
        srcs = np.arange(first, min(V, first + n), dtype=np.uint32)
        q = g.query(srcs, abi.SPF_F_NEXTHOPS)
        for _ in range(3):
            q.run()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(20):
            q.run(sync=False)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / 20 * 1e3
        out[f"N{N}_coop{coop}"] = {
            "sources": int(len(srcs)), "plan": q.kernel, "kernels": q.kernels(), "ms": round(ms, 4),
            "stage_ms": [round(x, 4) for x in q.stage_ms()]}
        q.close()
print(json.dumps(out, indent=1))
