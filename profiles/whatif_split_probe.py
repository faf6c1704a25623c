"""Probe: where the what-if batch's device time goes (configs[4] areas).
Per area: the baseline SPF alone (few-source plan on / off), then the
what-if batch split into the queries whose failed link touches the border
node (their K spans most of the graph) and the rest, with the repair on and
off.  Prints one JSON line per measurement."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402


def timed(q, n=3):
    q.run()
    best = None
    for _ in range(n):
        q.run()
        ms = q.elapsed_ms()
        best = ms if best is None else min(best, ms)
    return round(best, 3)


def main():
    import torch

    torch.cuda.init()
    from openr_amd import abi
    from openr_amd import topologies as TP

    for name, topo, links in TP.whatif_two_area():
        csr = topo.csr()
        r, _ = topo.rank()
        s = int(r[topo.names.index(TP.WHATIF_BORDER)])
        g = abi.Graph(csr)
        for few in ("1", "0"):
            os.environ["OPENR_SPF_FEW_DSTEP"] = few
            q = g.query([s], abi.SPF_F_NEXTHOPS)
            print(json.dumps({"area": name, "what": "baseline", "few_dstep": few, "kernel": q.kernel,
                              "ms": timed(q)}), flush=True)
            q.close()
        os.environ.pop("OPENR_SPF_FEW_DSTEP")
        rp = csr.row_ptr.astype(np.int64)
        adj = set(int(x) for x in csr.link_id[rp[s]:rp[s + 1]])
        near = [int(l) for l in links if int(l) in adj]
        far = [int(l) for l in links if int(l) not in adj]
        for part, ls in (("adjacent-to-source", near), ("rest", far), ("all", [int(l) for l in links])):
            if not ls:
                continue
            for rep in ("1", "0"):
                os.environ["OPENR_SPF_WHATIF_REPAIR"] = rep
                q = g.query(np.full(len(ls), s, dtype=np.uint32), abi.SPF_F_NEXTHOPS, ignore=[[l] for l in ls])
                ms = timed(q)
                print(json.dumps({"area": name, "what": part, "queries": len(ls), "repair": rep,
                                  "screened": q.screened(), "kernel": q.kernel, "ms": ms}), flush=True)
                q.close()
            os.environ.pop("OPENR_SPF_WHATIF_REPAIR")
        g.close()


if __name__ == "__main__":
    main()
