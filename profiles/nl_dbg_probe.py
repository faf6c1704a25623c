"""Where the v2 next-hop pass's time goes (measurement builds of the same
kernel, OPENR_NL_V2_DBG read at query creation; rows are NOT valid for the
dbg modes): 0 = the pass; 4 = everything but the stores; 8 = the stores
alone (same addresses, no loads); 8|16 = mask stores alone; 8|32 =
distance-row stores alone.  Fabric all-sources, same process / graph,
alternating blocks; next-hop stage device time from the engine's events.

    python profiles/nl_dbg_probe.py [steps] [rounds] > gpurun_out/nl_dbg.json
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402,F401

import numpy as np  # noqa: E402

from openr_amd import abi  # noqa: E402
from openr_amd import topologies as TP  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
modes = [0, 4, 8, 8 | 16, 8 | 32]
csr = TP.fabric(10000).csr()
g = abi.Graph(csr, device=0)
st = torch.cuda.Stream()
torch.cuda.set_stream(st)
g.set_stream(st.cuda_stream)
src = np.arange(csr.num_nodes, dtype=np.uint32)
qs = {}
for m in modes:
    os.environ["OPENR_NL_V2_DBG"] = str(m)
    qs[m] = g.query(src, abi.SPF_F_NEXTHOPS)
os.environ.pop("OPENR_NL_V2_DBG")
nh = {m: [] for m in modes}
for q in qs.values():
    for _ in range(3):
        q.run(sync=False)
torch.cuda.synchronize()
for r in range(rounds):
    for m, q in qs.items():
        for _ in range(steps):
            q.run(sync=False)
        torch.cuda.synchronize()
        h = q.stage_history(steps)
        nh[m].append(sum(x[1] for x in h) / len(h))
labels = {0: "full pass", 4: "no stores", 8: "stores only", 24: "mask stores only",
          40: "distance-row stores only"}
print(json.dumps({labels[m]: round(float(np.median(v)), 4) for m, v in nh.items()}), flush=True)
