"""Wide plan (spf_wide_kernel) vs the literal replay it replaced as the
whole-area fall-back (VERDICT r1 "exact-kernel cliff"):

  * fabric(10000) with ONE metric-0 link, all 9,976 sources + next hops;
  * WAN-100k / 1M links with metrics up to 10^6 (maxw * (V-1) >= 2^32),
    distance-only rows for a source sample (per-SPF time, extrapolated to all
    sources), rows checked against scipy's Dijkstra.

Usage (GPU box): python profiles/wide_plan_probe.py [--literal-sample N]
Prints one JSON object.
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402  (initialise torch's HIP runtime first)

import numpy as np  # noqa: E402

from openr_amd import abi  # noqa: E402
from openr_amd import topologies as TP  # noqa: E402
from oracle import spf_py  # noqa: E402


def timed(g, srcs, flags, reps=2):
    q = g.query(srcs, flags)
    best = None
    for _ in range(reps):
        q.run()
        ms = q.elapsed_ms()
        best = ms if best is None else min(best, ms)
    return q, best


def main():
    lit_n = int(sys.argv[sys.argv.index("--literal-sample") + 1]) if "--literal-sample" in sys.argv else 64
    torch.cuda.init()
    out = {}
    # ---- fabric with one metric-0 link
    topo = TP.fabric(10000)
    k = len(topo.links) // 2
    a, b, _, _ = topo.links[k]
    topo.links[k] = (a, b, 0, 0)
    csr = topo.csr()
    g = abi.Graph(csr)
    V = csr.num_nodes
    srcs = np.arange(V, dtype=np.uint32)
    q, ms = timed(g, srcs, abi.SPF_F_NEXTHOPS)
    bad = 0
    for i in (0, a, b, V - 1):
        ref = spf_py.run_spf(csr, int(srcs[i]), True)
        d = q.dist(i)
        sets = q.nexthop_sets(i, int(srcs[i]))
        for v, (m, nhs, _, _) in ref.items():
            bad += int(d[v]) != m or (v != srcs[i] and sets[v] != nhs)
    os.environ["OPENR_SPF_LITERAL"] = "1"
    ql, ms_l = timed(g, srcs[:lit_n], abi.SPF_F_NEXTHOPS, reps=1)
    del os.environ["OPENR_SPF_LITERAL"]
    out["fabric_one_zero_link"] = {
        "nodes": V, "sources": V, "kernel": q.kernel, "ms": round(ms, 2),
        "spf_per_s": round(V / (ms / 1e3), 1),
        "literal_replay": {"sources": lit_n, "kernel": ql.kernel, "ms": round(ms_l, 2),
                           "ms_all_sources_est": round(ms_l * V / lit_n, 1)},
        "parity_vs_replay_rows": 4, "mismatches": bad,
    }
    q.close(); ql.close(); g.close()
    # ---- WAN-100k, metrics up to 10^6
    import scipy.sparse as sp
    import scipy.sparse.csgraph as cg

    topo = TP.wan(100000, 1000000, wmax=1_000_000)
    csr = topo.csr()
    g = abi.Graph(csr)
    V = csr.num_nodes
    S = 2048
    srcs = np.arange(0, V, V // S, dtype=np.uint32)[:S]
    q, ms = timed(g, srcs, 0)
    A = sp.csr_matrix((csr.metric.astype(np.float64), csr.col, csr.row_ptr), shape=(V, V))
    D = cg.dijkstra(A, indices=[int(srcs[0]), int(srcs[-1])])
    bad = 0
    for kk, i in enumerate((0, S - 1)):
        ref = np.where(np.isfinite(D[kk]), D[kk], -1).astype(np.int64)
        got = q.dist(i).astype(np.int64)
        got[q.dist(i) == abi.SPF_UNREACHABLE] = -1
        bad += int((ref != got).sum())
    maxd = int(q.dist(0)[q.dist(0) != abi.SPF_UNREACHABLE].max())
    os.environ["OPENR_SPF_LITERAL"] = "1"
    ql, ms_l = timed(g, srcs[:lit_n], 0, reps=1)
    del os.environ["OPENR_SPF_LITERAL"]
    out["wan100k_metric_1e6"] = {
        "nodes": V, "links": int(csr.num_links), "sources_timed": S, "kernel": q.kernel,
        "ms": round(ms, 2), "ms_per_spf": round(ms / S, 4),
        "all_sources_s_est": round(ms / S * V / 1e3, 2), "max_dist_src0": maxd,
        "literal_replay": {"sources": lit_n, "kernel": ql.kernel, "ms": round(ms_l, 2),
                           "ms_per_spf": round(ms_l / lit_n, 3)},
        "parity_vs_scipy_rows": 2, "mismatches": bad,
    }
    print(json.dumps(out, default=int))


if __name__ == "__main__":
    main()
