"""What-if repair (spf_sssp_kernel repair mode): a what-if query whose
ignored links touch the baseline's shortest-path DAG starts from the baseline
rows of its source and recomputes only K, the nodes downstream of the tight
ignored links (whatif_repair_init).  Parity: every row and
next-hop mask equals the same batch recomputed from scratch
(OPENR_SPF_WHATIF_REPAIR=0) and sampled rows equal the literal DijkstraQ
replay with the same ignore list (oracle/spf_py.py, LinkState.cpp:806-880).

Ignore lists are drawn mostly from the baseline's TIGHT links (so the
repair, not the screen's copy, runs), 1-4 links each, plus links off the DAG,
ids beyond the graph, links of the source (K past V / 4: the
query runs from scratch) and empty lists; drained nodes, parallel links and
asymmetric metrics; the LDS and the global-memory kernels; metric and
hop-count (SPF_F_UNIT_METRIC) queries.
"""

import random

import numpy as np
import pytest

from openr_amd import abi
from openr_amd import topologies as TP
from tests.test_abi_gpu import check_query, random_links

pytestmark = pytest.mark.gpu

INF32 = 0xFFFFFFFF


def _tight_links(csr, s, d, unit):
    """Link ids of the usable tight half-edges of source s's row d."""
    rp, col, w, lid = csr.row_ptr, csr.col, csr.metric, csr.link_id
    ov = csr.overloaded
    out = set()
    for u in range(csr.num_nodes):
        du = int(d[u])
        if du == INF32 or (u != s and ov[u]):
            continue
        for e in range(int(rp[u]), int(rp[u + 1])):
            c = du + (1 if unit else int(w[e]))
            if c == int(d[col[e]]):
                out.add(int(lid[e]))
    return sorted(out)


def _batch(g, csr, rng, srcs, per_src, flags, nlinks):
    unit = bool(flags & abi.SPF_F_UNIT_METRIC)
    base = g.query(srcs, flags & abi.SPF_F_UNIT_METRIC).run()
    qs, ign = [], []
    for i, s in enumerate(srcs):
        d = base.dist(i).astype(np.uint64)
        d = np.where(d == np.uint64(abi.SPF_UNREACHABLE), INF32, d)
        tight = _tight_links(csr, s, d, unit)
        for j in range(per_src):
            k = rng.randint(1, 4)
            if j % 5 == 4 or not tight:
                lst = rng.sample(range(nlinks), k)  # mostly off the DAG
            else:
                lst = rng.sample(tight, min(k, len(tight)))
            if j == 1:
                lst = [nlinks + 2]  # no such link
            if j == 2:
                lst = []
            if j == 3:
                # a link of the source itself: K spans most of the graph and
                # the query runs from scratch instead (the V / 4 rule)
                rp = csr.row_ptr
                lst = [int(csr.link_id[rp[s] + (j % max(1, int(rp[s + 1] - rp[s])))])] \
                    if rp[s + 1] > rp[s] else []
            qs.append(s)
            ign.append(sorted(set(lst)))
    base.close()
    return qs, ign


def _compare(g, csr, qs, ign, flags, monkeypatch, rows):
    # distance-only batches on a uniform metric take the bit-parallel BFS
    # with ignore masks (no screen, test_msbfs_ignore_lists); keep them on
    # the repair path here
    monkeypatch.setenv("OPENR_SPF_MSBFS_IGN", "0")
    q = g.query(qs, flags, ignore=ign).run()
    nscr = q.screened()
    assert nscr is not None and nscr < len(qs)  # the repair ran on the rest
    monkeypatch.setenv("OPENR_SPF_WHATIF_REPAIR", "0")
    r = g.query(qs, flags, ignore=ign).run()
    monkeypatch.delenv("OPENR_SPF_WHATIF_REPAIR")
    assert q.kernel == r.kernel
    for i in range(len(qs)):
        assert (q.dist(i) == r.dist(i)).all(), i
        if flags & abi.SPF_F_NEXTHOPS:
            assert (q.nexthops(i) == r.nexthops(i)).all(), i
    check_query(csr, q, qs, not (flags & abi.SPF_F_UNIT_METRIC), ignore=ign, rows=rows)
    kern = q.kernel
    q.close()
    r.close()
    return kern, nscr


@pytest.mark.parametrize("seed,wmax,unit", [(301, 30, False), (302, 1, False), (303, 40, True)])
def test_repair_random_lds(gpu_ready, seed, wmax, unit, monkeypatch):
    rng = random.Random(seed)
    V = 2500
    links = random_links(rng, V, 8000, wmin=1, wmax=wmax, parallel=0.04)
    ov = np.zeros(V, dtype=np.uint8)
    ov[rng.sample(range(V), 50)] = 1
    csr = abi.Csr.from_links(V, links, overloaded=ov)
    g = abi.Graph(csr)
    drained = int(np.flatnonzero(ov)[0])
    srcs = [0, 17, drained, V - 1]
    flags = abi.SPF_F_NEXTHOPS | (abi.SPF_F_UNIT_METRIC if unit else 0)
    qs, ign = _batch(g, csr, rng, srcs, 120, flags, len(links))
    kern, _ = _compare(g, csr, qs, ign, flags, monkeypatch, rows={0, 3, 125, 250, 379, 400, 479})
    assert kern.startswith("lds")
    # distances only
    _compare(g, csr, qs, ign, 0, monkeypatch, rows={5, 300})
    g.close()


def test_repair_global_memory_kernel(gpu_ready, monkeypatch):
    """A uniform-metric graph too large for the LDS row: the global-memory
    kernel's repair path (dist rows in HBM)."""
    rng = random.Random(304)
    V = 40000
    links = random_links(rng, V, 100000, wmin=1, wmax=1, parallel=0.01, asym=False)
    ov = np.zeros(V, dtype=np.uint8)
    ov[rng.sample(range(V), 200)] = 1
    csr = abi.Csr.from_links(V, links, overloaded=ov)
    g = abi.Graph(csr)
    qs, ign = _batch(g, csr, rng, [3, 999], 60, abi.SPF_F_NEXTHOPS, len(links))
    kern, _ = _compare(g, csr, qs, ign, abi.SPF_F_NEXTHOPS, monkeypatch, rows={0, 61})
    assert kern.startswith("gmem")
    g.close()


def test_repair_fabric_clos(gpu_ready, monkeypatch):
    """A small Clos fabric from a spine and from a rack switch: failures of
    links on the ECMP DAG (most of them), whose K spans whole planes."""
    topo = TP.fabric(1200)
    csr = topo.csr()
    g = abi.Graph(csr)
    r, _ = topo.rank()
    srcs = [int(r[topo.names.index("2-0-0")]), int(r[topo.names.index(sorted(
        n for n in topo.names if n.startswith("3-"))[0])])]
    rng = random.Random(305)
    L = int(csr.link_id.max()) + 1
    qs, ign = _batch(g, csr, rng, srcs, 150, abi.SPF_F_NEXTHOPS, L)
    kern, nscr = _compare(g, csr, qs, ign, abi.SPF_F_NEXTHOPS, monkeypatch, rows={0, 3, 77, 150, 151, 299})
    assert kern.startswith("lds")
    g.close()


@pytest.mark.parametrize("mode", ["firsthop", "pull", "queue"])
@pytest.mark.parametrize("case", ["fabric", "uniform5"])
def test_source_link_failures_heavy_kernel(gpu_ready, case, mode, monkeypatch):
    """What-ifs that fail a link of the source itself on a uniform-metric
    area (K is most of the graph).  Queries whose every ignored link is at
    the source take the first-hop form (spf_whatif_firsthop_kernel over one
    nested batch of the source's neighbour rows, default); the others, and
    all of them with OPENR_SPF_WHATIF_FIRSTHOP=0, run on one 1,024-thread
    workgroup per query: a BFS and a level-by-level next-hop pass, in pull
    form over the sliced ELL (spf_whatif_pull_kernel) or over a BFS queue
    (spf_whatif_heavy_kernel, OPENR_SPF_WHATIF_PULL=0).  Rows and masks
    equal the same batch with none of them (OPENR_SPF_WHATIF_HEAVY=0:
    spf_sssp_kernel from scratch) and the DijkstraQ replay; parallel links
    of the source keep its neighbour bit."""
    monkeypatch.setenv("OPENR_SPF_MSBFS_IGN", "0")
    monkeypatch.setenv("OPENR_SPF_WHATIF_FIRSTHOP", "1" if mode == "firsthop" else "0")
    monkeypatch.setenv("OPENR_SPF_WHATIF_PULL", "0" if mode == "queue" else "1")
    kname = {"firsthop": "spf_whatif_firsthop_kernel", "pull": "spf_whatif_pull_kernel",
             "queue": "spf_whatif_heavy_kernel"}[mode]
    rng = random.Random(306)
    if case == "fabric":
        topo = TP.fabric(1200)
        csr = topo.csr()
        r, _ = topo.rank()
        s = int(r[topo.names.index("2-0-0")])
    else:
        V = 1500
        links = random_links(rng, V, 5000, wmin=5, wmax=5, parallel=0.05, asym=False)
        # a parallel link at the source
        links.append((0, links[0][1] if links[0][0] == 0 else 1, 5, 5))
        ov = np.zeros(V, dtype=np.uint8)
        ov[rng.sample(range(1, V), 30)] = 1
        csr = abi.Csr.from_links(V, links, overloaded=ov)
        s = 0
    g = abi.Graph(csr)
    rp = csr.row_ptr
    src_links = sorted({int(csr.link_id[e]) for e in range(int(rp[s]), int(rp[s + 1]))})
    L = int(csr.link_id.max()) + 1
    ign = [[l] for l in src_links] + [sorted(rng.sample(range(L), 2)) for _ in range(40)]
    qs = [s] * len(ign)
    flags = abi.SPF_F_NEXTHOPS
    q = g.query(qs, flags, ignore=ign).run()
    assert kname in q.kernels()
    monkeypatch.setenv("OPENR_SPF_WHATIF_HEAVY", "0")
    r = g.query(qs, flags, ignore=ign).run()
    monkeypatch.delenv("OPENR_SPF_WHATIF_HEAVY")
    assert kname not in r.kernels()
    assert "spf_whatif_firsthop_kernel" not in r.kernels()
    for i in range(len(qs)):
        assert (q.dist(i) == r.dist(i)).all(), i
        assert (q.nexthops(i) == r.nexthops(i)).all(), i
    check_query(csr, q, qs, True, ignore=ign,
                rows=set(range(0, len(src_links), max(1, len(src_links) // 6))) | {len(qs) - 1})
    q.close()
    r.close()
    g.close()
