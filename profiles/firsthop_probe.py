"""Probe: the what-if batch "every link of one node fails" (LFA
precomputation for that node) on the 10k fabric, first-hop form vs the pull
kernel (OPENR_SPF_WHATIF_FIRSTHOP=1 / 0).  Prints one JSON line per form:
device ms per batch (spf_query_elapsed_ms median over runs).

  python profiles/firsthop_probe.py [RUNS] [NODE]
"""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from openr_amd import abi  # noqa: E402
from openr_amd import topologies as TP  # noqa: E402


def main():
    runs = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    node = sys.argv[2] if len(sys.argv) > 2 else "2-0-0"
    topo = TP.fabric(9976)
    csr = topo.csr()
    r, _ = topo.rank()
    s = int(r[topo.names.index(node)])
    g = abi.Graph(csr)
    rp = csr.row_ptr
    links = sorted({int(csr.link_id[e]) for e in range(int(rp[s]), int(rp[s + 1]))})
    ign = [[l] for l in links]
    qs = [s] * len(ign)
    base = None
    for form in ("1", "0"):
        os.environ["OPENR_SPF_WHATIF_FIRSTHOP"] = form
        q = g.query(qs, abi.SPF_F_NEXTHOPS, ignore=ign)
        ms = []
        for i in range(runs + 2):
            q.run()
            if i >= 2:
                ms.append(q.elapsed_ms())
        rows = [q.dist(i).copy() for i in range(len(qs))]
        masks = [q.nexthops(i).copy() for i in range(len(qs))]
        same = None
        if base is not None:
            same = all((a == b).all() for a, b in zip(rows, base[0])) and \
                all((a == b).all() for a, b in zip(masks, base[1]))
        else:
            base = (rows, masks)
        print(json.dumps({"form": "firsthop" if form == "1" else "pull", "node": node,
                          "queries": len(qs), "device_ms_median": round(statistics.median(ms), 4),
                          "device_ms_min": round(min(ms), 4), "kernels": q.kernels(),
                          "same_as_firsthop": same}), flush=True)
        q.close()
    g.close()


if __name__ == "__main__":
    main()
