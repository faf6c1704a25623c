"""Device k-th path traces (spf_query_trace_paths) against the literal
traceOnePath recursion (LinkState.cpp:398-419, repeated as getKthPaths does,
:776-786) over the DijkstraQ replay's pathLinks (oracle/spf_py.py): seeded
random graphs with drained nodes, parallel links, asymmetric and unit
metrics, and the KSP2 second-pass ignore lists (the first paths' links)."""

import random
import sys

import numpy as np
import pytest

from openr_amd import abi
from oracle import spf_py

pytestmark = pytest.mark.gpu


def random_links(rng, V, L, wmin=1, wmax=20, parallel=0.05):
    links = []
    for v in range(1, V):
        links.append((rng.randrange(v), v, rng.randint(wmin, wmax), rng.randint(wmin, wmax)))
    while len(links) < L:
        u, v = rng.randrange(V), rng.randrange(V)
        if u == v:
            continue
        links.append((u, v, rng.randint(wmin, wmax), rng.randint(wmin, wmax)))
        if rng.random() < parallel:
            links.append((u, v, rng.randint(wmin, wmax), rng.randint(wmin, wmax)))
    rng.shuffle(links)
    return links


def trace_all(csr, ref, src, dst):
    """getKthPaths' loop: traceOnePath until a trace fails (or is empty)."""
    lid = csr.link_id
    visited = set()

    def one(v):
        if v == src:
            return []
        for (e, u) in ref[v][2]:
            l = int(lid[e])
            if l in visited:
                continue
            visited.add(l)
            p = one(u)
            if p is not None:
                p.append(l)
                return p
        return None

    out = []
    if dst not in ref:
        return out
    while True:
        p = one(dst)
        if not p:
            return out
        out.append(p)


@pytest.mark.parametrize("seed,unit", [(1, False), (2, False), (3, True), (4, False)])
def test_trace_paths_random(gpu_ready, seed, unit):
    sys.setrecursionlimit(10000)
    rng = random.Random(seed)
    V = 120
    links = random_links(rng, V, 400, wmax=1 if unit else 6)
    ov = np.zeros(V, dtype=np.uint8)
    ov[rng.sample(range(V), 6)] = 1
    csr = abi.Csr.from_links(V, links, overloaded=ov)
    g = abi.Graph(csr)
    src = rng.randrange(V)
    dsts = [d for d in range(V) if d != src]
    flags = abi.SPF_F_UNIT_METRIC if unit else 0
    # k = 1: the source's own row for every destination
    q1 = g.query([src] * len(dsts), flags).run()
    got1 = q1.trace_paths(dsts)
    ref = spf_py.run_spf(csr, src, not unit)
    first = []
    for d, got in zip(dsts, got1):
        want = trace_all(csr, ref, src, d)
        assert got == want, (d, got, want)
        first.append(sorted({l for p in want for l in p}))
    # k = 2: the first paths' links ignored, one query per destination
    keep = [i for i, f in enumerate(first) if f]
    srcs = [src] * len(keep)
    ign = [first[i] for i in keep]
    q2 = g.query(srcs, flags, ignore=ign).run()
    got2 = q2.trace_paths([dsts[i] for i in keep])
    for j, i in enumerate(keep):
        r2 = spf_py.run_spf(csr, src, not unit, frozenset(ign[j]))
        want = trace_all(csr, r2, src, dsts[i])
        assert got2[j] == want, (dsts[i], got2[j], want)


def test_trace_paths_overflow_and_range(gpu_ready, monkeypatch):
    """A link capacity too small for the paths reports overflow (None) for
    that query only; a sub-range of queries traces the right rows."""
    # ladder 0..9 x 2 rails with rungs: many equal-cost paths
    links = []
    for i in range(9):
        links.append((i, i + 1, 1, 1))
        links.append((10 + i, 10 + i + 1, 1, 1))
    for i in range(10):
        links.append((i, 10 + i, 1, 1))
    csr = abi.Csr.from_links(20, links)
    g = abi.Graph(csr)
    q = g.query([0, 0, 0], abi.SPF_F_UNIT_METRIC).run()
    ref = spf_py.run_spf(csr, 0, False)
    full = q.trace_paths([19, 9, 10])
    assert full == [trace_all(csr, ref, 0, d) for d in (19, 9, 10)]
    monkeypatch.setenv("OPENR_SPF_TRACE_CAP", "4")
    small = q.trace_paths([19, 9, 10])
    monkeypatch.delenv("OPENR_SPF_TRACE_CAP")
    assert small[0] is None  # 19 is 10 hops away
    assert small[2] == [[9 * 2]]  # one rung: 0 - 10 (link id 18)
    sub = q.trace_paths([9, 10], first=1)
    assert sub == full[1:]


@pytest.mark.parametrize("cursor", ["1", "0"])
def test_trace_paths_visited_set_overflow(gpu_ready, cursor, monkeypatch):
    """Two full bipartite middle layers: the traces take more links than the
    round-3 kernel's per-wave visited set holds (OPENR_SPF_TRACE_CURSOR=0), so
    it reports overflow (None) and never a wrong path; the cursor DFS keeps no
    visited set (one pathLinks cursor per node in device scratch) and traces
    both sizes exactly."""
    monkeypatch.setenv("OPENR_SPF_TRACE_CURSOR", cursor)
    sys.setrecursionlimit(10000)
    for m, expect_overflow in ((8, False), (40, cursor == "0")):
        V = 2 + 2 * m
        src, dst = 0, V - 1
        links = [(src, 1 + i, 1, 1) for i in range(m)]
        links += [(1 + i, 1 + m + j, 1, 1) for i in range(m) for j in range(m)]
        links += [(1 + m + j, dst, 1, 1) for j in range(m)]
        csr = abi.Csr.from_links(V, links)
        g = abi.Graph(csr)
        q = g.query([src], abi.SPF_F_UNIT_METRIC).run()
        got = q.trace_paths([dst])[0]
        if expect_overflow:
            assert got is None
        else:
            assert got == trace_all(csr, spf_py.run_spf(csr, src, False), src, dst)


@pytest.mark.parametrize("reach", ["1", "0"])
@pytest.mark.parametrize("seed,unit", [(5, False), (6, True), (7, False)])
def test_trace_paths_heavy_launch(gpu_ready, seed, unit, reach, monkeypatch):
    """Queries past the cursor kernel's step budget are re-traced by the heavy
    launch: spf_trace_heavy_build_kernel pre-builds every node's pathLinks,
    then spf_trace_reach_kernel (reachability counts + greedy walk, the
    default) or spf_trace_heavy_kernel (the DFS with LDS cursors,
    OPENR_SPF_TRACE_REACH=0) traces.  With a budget of one step every query
    takes that path; the traces must equal the recursion's, for the k = 1
    rows and the KSP2 ignore-list rows.  A heavy budget too small reports
    overflow (None), never a wrong path."""
    sys.setrecursionlimit(10000)
    monkeypatch.setenv("OPENR_SPF_TRACE_BUDGET", "1")
    monkeypatch.setenv("OPENR_SPF_TRACE_REACH", reach)
    rng = random.Random(seed)
    V = 150
    links = random_links(rng, V, 520, wmax=1 if unit else 5)
    ov = np.zeros(V, dtype=np.uint8)
    ov[rng.sample(range(V), 5)] = 1
    csr = abi.Csr.from_links(V, links, overloaded=ov)
    g = abi.Graph(csr)
    src = rng.randrange(V)
    dsts = [d for d in range(V) if d != src]
    flags = abi.SPF_F_UNIT_METRIC if unit else 0
    q1 = g.query([src] * len(dsts), flags).run()
    got1 = q1.trace_paths(dsts)
    assert ("spf_trace_reach_kernel" if reach == "1" else "spf_trace_heavy_kernel") in q1.kernels()
    ref = spf_py.run_spf(csr, src, not unit)
    first = []
    for d, got in zip(dsts, got1):
        want = trace_all(csr, ref, src, d)
        assert got == want, (d, got, want)
        first.append(sorted({l for p in want for l in p}))
    keep = [i for i, f in enumerate(first) if f]
    ign = [first[i] for i in keep]
    q2 = g.query([src] * len(keep), flags, ignore=ign).run()
    got2 = q2.trace_paths([dsts[i] for i in keep])
    for j, i in enumerate(keep):
        r2 = spf_py.run_spf(csr, src, not unit, frozenset(ign[j]))
        assert got2[j] == trace_all(csr, r2, src, dsts[i]), dsts[i]
    # the heavy kernel's own budget: a multi-step trace overflows, the rest
    # stay exact
    monkeypatch.setenv("OPENR_SPF_TRACE_HEAVY_BUDGET", "3")
    small = q1.trace_paths(dsts)
    n_over = 0
    for d, got in zip(dsts, small):
        if got is None:
            n_over += 1
        else:
            assert got == trace_all(csr, ref, src, d), d
    assert n_over > 0


@pytest.mark.parametrize("reach", ["1", "0"])
def test_trace_paths_heavy_bipartite(gpu_ready, reach, monkeypatch):
    """The two-layer bipartite case (1,600 middle links) through the heavy
    launch only."""
    monkeypatch.setenv("OPENR_SPF_TRACE_BUDGET", "1")
    monkeypatch.setenv("OPENR_SPF_TRACE_REACH", reach)
    sys.setrecursionlimit(10000)
    m = 40
    V = 2 + 2 * m
    src, dst = 0, V - 1
    links = [(src, 1 + i, 1, 1) for i in range(m)]
    links += [(1 + i, 1 + m + j, 1, 1) for i in range(m) for j in range(m)]
    links += [(1 + m + j, dst, 1, 1) for j in range(m)]
    csr = abi.Csr.from_links(V, links)
    g = abi.Graph(csr)
    q = g.query([src, src], abi.SPF_F_UNIT_METRIC).run()
    got = q.trace_paths([dst, 1 + m])
    ref = spf_py.run_spf(csr, src, False)
    assert got == [trace_all(csr, ref, src, dst), trace_all(csr, ref, src, 1 + m)]
    assert ("spf_trace_reach_kernel" if reach == "1" else "spf_trace_heavy_kernel") in q.kernels()
