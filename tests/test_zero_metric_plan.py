"""GPU parity of the zero-metric plan ("msbfs0+levels"): a uniform metric
plus a few node-disjoint metric-0 links, run as one MS-BFS table per settle
order variant (spf_zvar_kernel) instead of the wide plan.

The reference settles a plateau of equal distance in (metric, name) order
among discovered nodes (LinkState.h:483-535) and hands next hops only from
nodes settled earlier (LinkState.cpp:842-871); the oracle is the literal
DijkstraQ replay (oracle/spf_py.py).  Every row is also compared word for
word with the wide plan (OPENR_SPF_ZERO_MSBFS=0), which the replay pins in
tests/test_wide_plan.py.
"""

import random

import numpy as np
import pytest

from openr_amd import abi
from openr_amd import topologies as TP

from .test_abi_gpu import check_query, random_links

pytestmark = pytest.mark.gpu


def _zero_graph(rng, V, L, c, k, oneway=False, ov_ends=False, ov_frac=0.03):
    """random_links with every metric c, then k metric-0 links between 2k
    distinct nodes (one direction only when `oneway`)."""
    links = random_links(rng, V, L, wmin=c, wmax=c)
    ends = rng.sample(range(V), 2 * k)
    for i in range(k):
        a, b = ends[2 * i], ends[2 * i + 1]
        links.append((a, b, 0, c if (oneway and i % 2 == 0) else 0))
    ov = [1 if rng.random() < ov_frac else 0 for _ in range(V)]
    if ov_ends:
        ov[ends[0]] = 1
    return abi.Csr.from_links(V, links, ov), ends


def _same_as_wide(csr, q, sources, monkeypatch, rows=None):
    g = abi.Graph(csr)
    monkeypatch.setenv("OPENR_SPF_ZERO_MSBFS", "0")
    w = g.query(sources, q.flags).run()
    monkeypatch.delenv("OPENR_SPF_ZERO_MSBFS")
    assert w.kernel == "wide"
    for i in range(len(sources)):
        if rows is not None and i not in rows:
            continue
        assert (q.dist(i) == w.dist(i)).all(), i
        if q.flags & abi.SPF_F_NEXTHOPS:
            assert (q.nexthops(i) == w.nexthops(i)).all(), i
    w.close()
    g.close()


@pytest.mark.parametrize(
    "seed,c,k,oneway,ov_ends",
    [(1, 1, 1, False, False), (2, 1, 2, False, False), (3, 1, 3, True, False),
     (4, 3, 1, True, True), (5, 2, 2, False, True), (6, 1, 3, False, False),
     (7, 5, 1, False, False), (8, 1, 2, True, True)])
def test_zero_plan_random(gpu_ready, monkeypatch, seed, c, k, oneway, ov_ends):
    rng = random.Random(seed)
    V = 260
    csr, ends = _zero_graph(rng, V, 700, c, k, oneway, ov_ends)
    g = abi.Graph(csr)
    assert g.needs_exact
    sources = list(range(V))
    q = g.query(sources, abi.SPF_F_NEXTHOPS).run()
    assert q.kernel == "msbfs0+levels"
    # the replay on every metric-0 end and a sample of the rest
    rows = set(ends) | set(rng.sample(range(V), 40))
    check_query(csr, q, sources, True, rows=rows)
    _same_as_wide(csr, q, sources, monkeypatch)


def test_zero_plan_grid_every_row(gpu_ready, monkeypatch):
    """A 40x40 unit grid with one metric-0 link: every plateau order occurs
    (sources on either side, and both ends discovered at once on the link's
    symmetry line)."""
    n = 40
    links = []
    for r in range(n):
        for col in range(n):
            v = r * n + col
            if col + 1 < n:
                links.append((v, v + 1, 1, 1))
            if r + 1 < n:
                links.append((v, v + n, 1, 1))
    mid = len(links) // 2
    a, b = links[mid][0], links[mid][1]
    links[mid] = (a, b, 0, 0)
    csr = abi.Csr.from_links(n * n, links)
    g = abi.Graph(csr)
    sources = list(range(n * n))
    q = g.query(sources, abi.SPF_F_NEXTHOPS).run()
    assert q.kernel == "msbfs0+levels"
    rng = random.Random(9)
    check_query(csr, q, sources, True, rows={a, b} | set(rng.sample(sources, 30)))
    _same_as_wide(csr, q, sources, monkeypatch)


def test_zero_plan_distances_only(gpu_ready, monkeypatch):
    rng = random.Random(13)
    csr, _ = _zero_graph(rng, 300, 900, 2, 3)
    g = abi.Graph(csr)
    sources = list(range(0, 300, 2))
    q = g.query(sources, 0).run()
    assert q.kernel == "msbfs0"
    check_query(csr, q, sources, True, rows=set(range(0, len(sources), 10)))
    _same_as_wide(csr, q, sources, monkeypatch)


def test_zero_plan_helper_sources(gpu_ready, monkeypatch):
    """A batch whose sources' neighbours lie outside it (helper rows in
    every variant table)."""
    rng = random.Random(17)
    V = 400
    csr, ends = _zero_graph(rng, V, 1200, 1, 2)
    g = abi.Graph(csr)
    sources = sorted(set(rng.sample(range(V), 70)) | {ends[0], ends[3]})
    q = g.query(sources, abi.SPF_F_NEXTHOPS).run()
    assert q.kernel == "msbfs0+levels"
    check_query(csr, q, sources, True, rows=set(range(0, len(sources), 5)) | {
        sources.index(ends[0]), sources.index(ends[3])})
    _same_as_wide(csr, q, sources, monkeypatch)


def test_zero_plan_deep_levels(gpu_ready, monkeypatch):
    """Paths deeper than 254 levels: the next-hop pass takes the 32-bit rows
    of each source's variant table."""
    V = 700
    links = [(v, v + 1, 1, 1) for v in range(V - 1)]
    links += [(v, v + 3, 1, 1) for v in range(0, V - 3, 97)]
    links.append((300, 301, 0, 0))       # on the path itself
    links.append((150, 420, 0, 0))       # a metric-0 shortcut
    csr = abi.Csr.from_links(V, links)
    g = abi.Graph(csr)
    sources = list(range(0, V, 5)) + [150, 301]
    q = g.query(sources, abi.SPF_F_NEXTHOPS).run()
    assert q.kernel == "msbfs0+levels"
    check_query(csr, q, sources, True, rows={0, 1, 30, 60, len(sources) - 2, len(sources) - 1})
    _same_as_wide(csr, q, sources, monkeypatch)


def test_zero_plan_parallel_links(gpu_ready, monkeypatch):
    """A metric-0 link beside a metric-c link between the same two nodes,
    and two parallel metric-0 links between another pair."""
    rng = random.Random(21)
    V = 240
    links = random_links(rng, V, 700, wmin=1, wmax=1)
    links += [(3, 77, 0, 0), (3, 77, 1, 1), (10, 11, 0, 0), (10, 11, 0, 0)]
    csr = abi.Csr.from_links(V, links)
    g = abi.Graph(csr)
    sources = list(range(V))
    q = g.query(sources, abi.SPF_F_NEXTHOPS).run()
    assert q.kernel == "msbfs0+levels"
    check_query(csr, q, sources, True, rows={3, 77, 10, 11} | set(rng.sample(sources, 20)))
    _same_as_wide(csr, q, sources, monkeypatch)


def test_zero_plan_falls_back(gpu_ready):
    """Four zero links, or two sharing a node (a three-node plateau): wide."""
    rng = random.Random(25)
    csr, _ = _zero_graph(rng, 200, 600, 1, 4)
    assert abi.Graph(csr).query(list(range(200)), abi.SPF_F_NEXTHOPS).run().kernel == "wide"
    links = random_links(rng, 200, 600, wmin=1, wmax=1) + [(5, 6, 0, 0), (6, 7, 0, 0)]
    csr = abi.Csr.from_links(200, links)
    q = abi.Graph(csr).query(list(range(200)), abi.SPF_F_NEXTHOPS).run()
    assert q.kernel == "wide"
    check_query(csr, q, list(range(200)), True, rows={5, 6, 7, 100})


def test_zero_plan_fabric(gpu_ready, monkeypatch):
    """The fabric with one metric-0 link (bench.py wide_plan section): every
    source through the zero-metric plan; rows of both link ends and a sample
    against the wide plan, two against the replay."""
    topo = TP.fabric(10000)
    k = len(topo.links) // 2
    a, b, _, _ = topo.links[k]
    topo.links[k] = (a, b, 0, 0)
    csr = topo.csr()
    g = abi.Graph(csr)
    V = csr.num_nodes
    sources = np.arange(V, dtype=np.uint32)
    q = g.query(sources, abi.SPF_F_NEXTHOPS).run()
    assert q.kernel == "msbfs0+levels"
    r, _ = topo.rank()
    ia, ib = int(r[a]), int(r[b])
    rng = random.Random(31)
    rows = {ia, ib} | set(rng.sample(range(V), 24))
    _same_as_wide(csr, q, [int(s) for s in sources], monkeypatch, rows=rows)
    check_query(csr, q, [int(s) for s in sources], True, rows={0, V // 2})
