"""Debug probe: SWAR next-hop pass vs the scalar pass on the hubs graph."""
import os, random, sys
import numpy as np
sys.path.insert(0, os.getcwd())
import torch  # noqa: F401  (bind the HIP runtime first)
from openr_amd import abi
from tests.test_abi_gpu import random_links

rng = random.Random(6)
V = 1300
links = random_links(rng, V, 7000, wmin=1, wmax=1, parallel=0.03)
links += [(7, v, 1, 1) for v in range(100, 260)]
links += [(8, v, 1, 1) for v in range(300, 400)]
ov = np.zeros(V, dtype=np.uint8)
ov[rng.sample(range(V), V // 40)] = 1
csr = abi.Csr.from_links(V, links, overloaded=ov)
g = abi.Graph(csr)
srcs = np.arange(V, dtype=np.uint32)
flags = abi.SPF_F_NEXTHOPS | abi.SPF_F_UNIT_METRIC
res = {}
for swar, held in (("1", "1"), ("0", "1"), ("0", "0")):
    os.environ["OPENR_NL_SWAR"] = swar
    os.environ["OPENR_NL_HELD"] = held
    q = g.query(srcs, flags).run()
    res[(swar, held)] = [q.nexthops(i).copy() for i in range(V)]
    W = [q.nh_words(i) for i in range(V)]
for key in res:
    if key == ("0", "0"):
        continue
    bad = [i for i in range(V) if not (res[key][i] == res[("0", "0")][i]).all()]
    print(key, "differs from scalar/held=0 on", len(bad), "sources", bad[:10],
          "W", [W[i] for i in bad[:10]], "deg", [g.num_nbrs(i) for i in bad[:10]])
    for i in bad[:3]:
        m = res[key][i]; r = res[("0", "0")][i]
        rows = np.flatnonzero((m != r).any(axis=1))
        print("  src", i, "rows", rows[:8].tolist(), "got", [hex(int(x)) for x in m[rows[0]]],
              "want", [hex(int(x)) for x in r[rows[0]]])
