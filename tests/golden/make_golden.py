"""Generate the golden fixtures under tests/golden/ (TEST INFRASTRUCTURE).

Run in the build container:  python tests/golden/make_golden.py

Sources of truth, in order of strength:
  * wan_anchors.json — distance checksums produced by the REFERENCE's own
    LinkState::runSpf (openr/decision/LinkState.cpp:806-880) on the
    SURVEY §8(d) row-3 WAN generator, recorded in SURVEY.md §8(d).  Not
    regenerated here (the reference cannot be built in this image); this
    script only re-checks them with an independent scipy Dijkstra.
  * grid10.json, fabric_sampled.json, whatif_fabric.json — outputs of the
    CPU oracle (oracle/ref_decision.cpp, oracle/spf_py.py), which is itself
    pinned by the reference's known answers (tests/known_answers.py) and by
    wan_anchors.json.  They let the GPU box check the engine at config sizes
    without re-running the (slow) oracle there.
"""

from __future__ import annotations

import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)


def canon(x):
    """Hashable route / SPF structures -> JSON-able canonical form."""
    if isinstance(x, bytes):
        return x.hex()
    if isinstance(x, (frozenset, set)):
        items = [canon(i) for i in x]
        return sorted(items, key=lambda i: json.dumps(i, sort_keys=True))
    if isinstance(x, (list, tuple)):
        return [canon(i) for i in x]
    if isinstance(x, dict):
        items = [[canon(k), canon(v)] for k, v in x.items()]
        return sorted(items, key=lambda i: json.dumps(i[0], sort_keys=True))
    return x


def digest(obj) -> str:
    return hashlib.sha256(json.dumps(canon(obj), sort_keys=True).encode()).hexdigest()


def spf_canon(res):
    """getSpfResult dict -> {node: (metric, sorted next hops)} (pathLinks are
    compared separately where the order matters)."""
    return {n: (int(v[0]), sorted(v[1])) for n, v in res.items()}


def load(M, topo, area="0", fwd_type=0, fwd_algo=0):
    areas = M.AreaLinkStates()
    ls = areas.add(area)
    for db in topo.adj_dbs(area):
        ls.updateAdjacencyDatabase(db)
    ps = M.PrefixState()
    for pdb in topo.prefix_dbs(area, fwd_type, fwd_algo):
        ps.updatePrefixDatabase(pdb)
    return areas, ls, ps


FABRIC_SOURCES = ["2-0-0", "1-0-0", "3-0-0", "1-7-35", "2-172-7", "3-86-47", "3-172-0", "2-100-3"]
KSP2_DESTS = ["3-0-1", "3-1-0", "2-5-5", "1-3-3", "3-172-47", "2-99-1", "1-0-35", "3-50-20"]


def whatif_links(topo, n=6):
    """Deterministic sample of fabric links (by creation index)."""
    step = max(1, len(topo.links) // n)
    return [topo.links[i][:2] for i in range(0, len(topo.links), step)][:n]


def main():
    from oracle import build as OB

    OB.build()
    from oracle import _oracle_ref as O
    from oracle import spf_py
    from openr_amd import topologies as TP
    from openr_amd import thrift as T

    # ---- config 1: 10x10 grid, RouteDb of node "1" (LFA on, SP_ECMP) and
    #      KSP2_ED_ECMP / SR_MPLS variant
    g = TP.grid(10)
    out = {}
    for tag, ft, fa, lfa in (
        ("sp_ecmp_lfa", 0, 0, True),
        ("ksp2_ed_ecmp", T.PrefixForwardingType.SR_MPLS, T.PrefixForwardingAlgorithm.KSP2_ED_ECMP, False),
    ):
        areas, ls, ps = load(O, g, "0", ft, fa)
        s = O.SpfSolver("1", False, lfa)
        db = s.buildRouteDb("1", areas, ps)
        out[tag] = {
            "node": "1",
            "lfa": lfa,
            "num_unicast": len(db["unicast"]),
            "num_mpls": len(db["mpls"]),
            "routes": canon(db),
            "digest": digest(db),
        }
    json.dump(out, open(os.path.join(HERE, "grid10.json"), "w"), indent=0, sort_keys=True)

    # ---- config 2/4: fabric_full, sampled sources + KSP2 paths
    f = TP.fabric(10000)
    areas, ls, ps = load(O, f)
    rows = {}
    for src in FABRIC_SOURCES:
        res = ls.getSpfResult(src, True)
        c = spf_canon(res)
        rows[src] = {
            "reached": len(c),
            "sum_metric": sum(m for m, _ in c.values()),
            "sum_nexthops": sum(len(h) for _, h in c.values()),
            "digest": digest(c),
        }
    ksp = {}
    for d in KSP2_DESTS:
        ksp[d] = {str(k): [[list(l.key()) for l in p] for p in ls.getKthPaths("2-0-0", d, k)] for k in (1, 2)}
    json.dump(
        {"topology": "fabric_full(10000)", "spf": rows, "ksp2_src": "2-0-0", "ksp2": ksp},
        open(os.path.join(HERE, "fabric_sampled.json"), "w"),
        indent=0,
        sort_keys=True,
    )

    # ---- config 5: what-if single-link failures on the fabric (runSpf with
    #      linksToIgnore = {link}, LinkState.cpp:806-880), oracle/spf_py replay
    csr = f.csr()
    r, names_by_rank = f.rank()
    wi = []
    for (a, b) in whatif_links(f):
        # link id in the device CSR = creation index of the link
        lid = next(i for i, l in enumerate(f.links) if l[0] == a and l[1] == b)
        for src in ("2-0-0", f.names[a]):
            sid = int(r[f.names.index(src)])
            res = spf_py.run_spf(csr, sid, True, frozenset([lid]))
            c = {
                names_by_rank[v]: (int(m), sorted(names_by_rank[h] for h in nh))
                for v, (m, nh, _, _) in res.items()
            }
            wi.append({
                "src": src,
                "link": [f.names[a], f.names[b]],
                "reached": len(c),
                "sum_metric": sum(m for m, _ in c.values()),
                "digest": digest(c),
            })
    json.dump({"topology": "fabric_full(10000)", "queries": wi},
              open(os.path.join(HERE, "whatif_fabric.json"), "w"), indent=0, sort_keys=True)
    print("goldens written")


if __name__ == "__main__":
    main()
