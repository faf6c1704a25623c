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
    config_sized(O, f)
    print("goldens written")


def csr_summary(O, csr, sources, ignore=None, want_nh=True, threads=None):
    """oracle/csr_spf.h per-query (reached, sum of distances, (node, next hop)
    pairs, mix) -- see tests/golden/summary.py for the same numbers computed
    from the engine's rows."""
    import numpy as np

    ioff = ign = None
    if ignore is not None:
        ioff = np.zeros(len(ignore) + 1, dtype=np.uint32)
        ioff[1:] = np.cumsum([len(x) for x in ignore])
        ign = np.asarray([int(v) for x in ignore for v in sorted(x)] or [0], dtype=np.uint32)
    return O.csr_spf_summary(csr.row_ptr, csr.col, csr.metric.astype(np.uint64), csr.link_id,
                             csr.overloaded, np.asarray(sources, dtype=np.uint32), ioff, ign,
                             True, want_nh, threads or os.cpu_count())


def config_sized(O, fab):
    """Round-2 goldens for the configs at their real plans:
      fabric_allsources.npz  every one of the 9,976 fabric sources (config 2)
      whatif_two_area.npz    the 8,192 two-area what-if queries (config 5)
      whatif_two_area.json   reference-form digests of sampled what-if queries
                             through the oracle's multi-area LinkState
      wan100k_rows.json      sampled rows of the 100k WAN (config 3)
    The flat summaries come from oracle/csr_spf.h, cross-checked here against
    the reference-style oracle on sampled sources."""
    import numpy as np

    from oracle import spf_py
    from openr_amd import topologies as TP
    from tests.golden.summary import summary_from_spf_result

    # ---- config 2: all fabric sources
    csr = fab.csr()
    V = csr.num_nodes
    S = csr_summary(O, csr, np.arange(V))
    r, names_by_rank = fab.rank()
    areas, ls, _ = load(O, fab)
    for src in FABRIC_SOURCES[:3]:
        sid = names_by_rank.index(src)
        assert tuple(int(x) for x in S[sid]) == summary_from_spf_result(ls.getSpfResult(src, True),
                                                                        names_by_rank), src
    np.savez_compressed(os.path.join(HERE, "fabric_allsources.npz"), summary=S)

    # ---- config 5: two areas, border node 2-0-0, 4,096 link failures each
    meta = {"border": TP.WHATIF_BORDER, "areas": []}
    summ = []
    for area, topo, links in TP.whatif_two_area():
        c = topo.csr()
        rr, nbr = topo.rank()
        sid = int(rr[topo.names.index(TP.WHATIF_BORDER)])
        Sa = csr_summary(O, c, np.full(len(links), sid), [[int(l)] for l in links])
        summ.append(Sa)
        # reference-form digests of sampled queries through the oracle's
        # multi-area LinkState (runSpf with linksToIgnore = {link})
        oareas = O.AreaLinkStates()
        ols = oareas.add(area)
        for db in topo.adj_dbs(area):
            ols.updateAdjacencyDatabase(db)
        sampled = []
        for qi in list(range(0, len(links), len(links) // 12))[:12]:
            a, b = topo.links[int(links[qi])][:2]
            na, nb = topo.names[a], topo.names[b]
            lk = [l for l in ols.linksFromNode(na) if l.getOtherNodeName(na) == nb]
            res = ols.runSpfIgnoring(TP.WHATIF_BORDER, lk, True)
            assert summary_from_spf_result(res, nbr) == tuple(int(x) for x in Sa[qi]), (area, qi)
            sampled.append({"query": qi, "link": [na, nb], "reached": len(res),
                            "digest": digest(spf_canon(res))})
        # one literal DijkstraQ replay per area pins csr_spf on the ignore path
        q0 = sampled[0]["query"]
        rep = spf_py.run_spf(c, sid, True, frozenset([int(links[q0])]))
        assert len(rep) == sampled[0]["reached"]
        meta["areas"].append({"area": area, "links": [int(x) for x in links], "sampled": sampled})
    np.savez_compressed(os.path.join(HERE, "whatif_two_area.npz"), summary=np.concatenate(summ))
    json.dump(meta, open(os.path.join(HERE, "whatif_two_area.json"), "w"), sort_keys=True)

    # ---- config 3: sampled rows of the 100k WAN
    import hashlib

    w = TP.wan(100000, 1000000)
    c = w.csr()
    srcs = [0, 1, 99999] + [int(x) for x in np.random.default_rng(3).choice(100000, 29, replace=False)]
    rows = O.csr_spf_rows(c.row_ptr, c.col, c.metric.astype(np.uint64), c.link_id, c.overloaded,
                          np.asarray(srcs, dtype=np.uint32), True)
    out = []
    for s, row in zip(srcs, rows):
        r32 = np.where(row == np.uint64(2**64 - 1), np.uint64(0xFFFFFFFF), row).astype(np.uint32)
        out.append({"src": s, "sum": int(row[row != np.uint64(2**64 - 1)].sum()),
                    "sha256": hashlib.sha256(r32.tobytes()).hexdigest()})
    json.dump({"topology": "wan(100000, 1000000)", "rows": out},
              open(os.path.join(HERE, "wan100k_rows.json"), "w"), indent=0, sort_keys=True)


if __name__ == "__main__":
    main()
