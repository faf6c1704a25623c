"""Debug: in-place link flaps then a drain on a ShardedAllSources table."""
import os, random, sys
import numpy as np
sys.path.insert(0, os.getcwd())
import torch
from openr_amd import abi
from openr_amd import allsources as AS
from tests.test_table_repair import _random_links, _oracle_rows, _full_table

V, L, wmax = 2500, 9000, 30
rng = random.Random(V + L + wmax)
links = _random_links(V, L, rng, wmax=wmax)
ov = np.zeros(V, dtype=np.uint8)
csr = abi.Csr.from_links(V, links, ov)
srcs = np.asarray(sorted(rng.sample(range(V), min(V, 600))), dtype=np.uint32)
torch.cuda.set_device(0)
sas = AS.ShardedAllSources(csr, sources=srcs)
sas.run()
gone = []
for kind in ["down", "down", "up", "metric", "drain"]:
    if kind == "down":
        i = rng.randrange(len(links)); gone.append((i, links.pop(i)))
    elif kind == "up":
        links.insert(*gone.pop())
    elif kind == "metric":
        i = rng.randrange(len(links)); u, v, a, b = links[i]; links[i] = (u, v, a + 1 + rng.randrange(wmax), b)
    elif kind == "drain":
        d = rng.randrange(V); ov[d] ^= 1; print("drain node", d, "now", ov[d])
    csr = abi.Csr.from_links(V, links, ov)
    rep = sas.update(csr)
    got = sas.table.cpu().numpy().view(np.uint32)[: len(srcs)]
    want = _full_table(csr, srcs)
    bad = np.argwhere(got != want)
    # fresh query on the resident (patched) graph
    q = sas.graph.query(srcs, 0).run()
    lay = np.empty((len(srcs), V), dtype=np.uint32)
    q.fetch_rows(0, len(srcs), lay.ctypes.data, V * 4, on_device=False)
    q.close()
    print(kind, "patched", rep.graph_patched, "relaxed", rep.relaxed, "affected", rep.affected,
          "bad cells", len(bad), "fresh-on-layout bad", int((lay != want).sum()))
    if len(bad):
        i, v = bad[0]
        print("  src", srcs[i], "node", v, "got", got[i, v], "want", want[i, v], "layout-fresh", lay[i, v])
        print("  deltas", len(AS.abi.graph_diff(csr, csr)))
        break
