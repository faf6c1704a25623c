"""A/B of a next-hop-pass switch read at query creation (default
OPENR_NL_TRIT: the 2-bit neighbour rows; OPENR_NL_SHALLOW: the one-add
compare) on the fabric all-sources step, same process, same graph:
alternating timed blocks of each query; per-stage device times from the
engine's HIP events (stage_history: msbfs stage incl. any pack kernel,
next-hop stage = the v2 kernel).

    python profiles/nl_ab.py [steps] [rounds] [ENV_NAME] [MODE,MODE] > gpurun_out/ab.json
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402,F401

import numpy as np  # noqa: E402

from openr_amd import abi  # noqa: E402
from openr_amd import topologies as TP  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 4
env = sys.argv[3] if len(sys.argv) > 3 else "OPENR_NL_TRIT"
modes = sys.argv[4].split(",") if len(sys.argv) > 4 else ["1", "0"]
csr = TP.fabric(10000).csr()
g = abi.Graph(csr, device=0)
st = torch.cuda.Stream()
torch.cuda.set_stream(st)
g.set_stream(st.cuda_stream)
src = np.arange(csr.num_nodes, dtype=np.uint32)
qs = {}
for mode in modes:
    os.environ[env] = mode
    qs[mode] = g.query(src, abi.SPF_F_NEXTHOPS)
out = {k: {"step_ms": [], "dist_ms": [], "nh_ms": []} for k in qs}
for q in qs.values():
    for _ in range(3):
        q.run(sync=False)
torch.cuda.synchronize()
for r in range(rounds):
    for mode, q in qs.items():
        os.environ[env] = mode  # (switches read at launch, e.g. OPENR_NL_TILEW)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            q.run(sync=False)
        torch.cuda.synchronize()
        out[mode]["step_ms"].append((time.perf_counter() - t0) * 1e3 / steps)
        h = q.stage_history(steps)
        out[mode]["dist_ms"].append(sum(x[0] for x in h) / len(h))
        out[mode]["nh_ms"].append(sum(x[1] for x in h) / len(h))
a, b = qs[modes[0]], qs[modes[1]]
os.environ[env] = modes[0]
a.run()
os.environ[env] = modes[1]
b.run()
same = bool((a.fetch_nexthops(0, csr.num_nodes) == b.fetch_nexthops(0, csr.num_nodes)).all())
res = {"env": env}
res.update({env + "=" + k: {kk: round(float(np.median(v)), 4) for kk, v in d.items()} for k, d in out.items()})
res["raw"] = out
res["masks_equal"] = same
res["kernels"] = {k: q.kernels() for k, q in qs.items()}
print(json.dumps(res), flush=True)
