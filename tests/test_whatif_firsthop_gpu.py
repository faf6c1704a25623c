"""What-if source-link failures in first-hop form (round 6,
spf_whatif_firsthop_kernel; DESIGN.md §3 "What-if batches").

On a uniform metric a query that ignores links of its source s alone has
lvl(v) = 1 + min over the usable first hops n of R_s[n][v] (R_s = BFS levels
from s's neighbours with every link of s ignored: one nested batch), and v's
next hops are the slots of the first hops at that minimum.  Rows and masks
must equal the same batch run from scratch (OPENR_SPF_WHATIF_HEAVY=0:
spf_sssp_kernel) and the literal DijkstraQ replay (oracle/spf_py.py,
LinkState.cpp:806-880), including:
  * drained first hops (they reach only themselves) and a drained source
    (the source is exempt from the transit rule);
  * parallel links at the source with one of them ignored (the neighbour
    keeps its slot) and with both ignored;
  * several source links ignored at once, every source link ignored (only
    the source is reached), a link id past the graph;
  * transit bits flipped between runs of the same query objects, and a source
    link set down in place between runs (spf_graph_set_edges).
"""

import copy
import random

import numpy as np
import pytest

from openr_amd import abi
from tests.test_abi_gpu import check_query, random_links

pytestmark = pytest.mark.gpu

FH = "spf_whatif_firsthop_kernel"


def _source_links(csr, s):
    rp = csr.row_ptr
    return sorted({int(csr.link_id[e]) for e in range(int(rp[s]), int(rp[s + 1]))})


def _lists(rng, csr, s, L):
    sl = _source_links(csr, s)
    out = [[l] for l in sl]
    out += [sorted(rng.sample(sl, min(2, len(sl)))) for _ in range(6)]
    out += [sorted(rng.sample(sl, min(3, len(sl)))) for _ in range(4)]
    out.append(sorted(sl))               # the source cut off
    out.append(sorted([sl[0], L + 7]))   # a link id past the graph
    return out


def _same(q, r, n):
    for i in range(n):
        assert (q.dist(i) == r.dist(i)).all(), i
        if q.flags & abi.SPF_F_NEXTHOPS:
            assert (q.nexthops(i) == r.nexthops(i)).all(), i


def _reference(g, qs, flags, ign, monkeypatch):
    monkeypatch.setenv("OPENR_SPF_WHATIF_HEAVY", "0")
    r = g.query(qs, flags, ignore=ign).run()
    monkeypatch.delenv("OPENR_SPF_WHATIF_HEAVY")
    assert FH not in r.kernels()
    return r


def _uniform_graph(seed, V=1200, w=3):
    rng = random.Random(seed)
    links = random_links(rng, V, 4200, wmin=w, wmax=w, parallel=0.0, asym=False)
    s = 0
    have = sorted({b for (a, b, _, _) in links if a == s} | {a for (a, b, _, _) in links if b == s})
    # parallel links at the source, to two of its neighbours
    links += [(s, have[0], w, w), (s, have[1], w, w), (s, have[1], w, w)]
    ov = np.zeros(V, dtype=np.uint8)
    ov[rng.sample(range(1, V), 40)] = 1
    ov[have[2]] = 1  # drained first hops
    ov[have[3]] = 1
    return rng, links, ov, s


@pytest.mark.parametrize("form", ["blocked", "ign_msbfs", "ign_sssp"])
@pytest.mark.parametrize("unit", [False, True])
@pytest.mark.parametrize("drained_source", [False, True])
def test_firsthop_random_uniform(gpu_ready, unit, drained_source, form, monkeypatch):
    # form: the nested batch -- the plain bit-parallel BFS with the source
    # non-transit in its neighbours' batches (MsBfsArgs::blocked, default,
    # on the side stream), or every link of the source ignored (the BFS with
    # ignore masks, or one SSSP per row)
    monkeypatch.setenv("OPENR_SPF_WHATIF_FIRSTHOP_BLOCKED", "1" if form == "blocked" else "0")
    monkeypatch.setenv("OPENR_SPF_MSBFS_IGN", "0" if form == "ign_sssp" else "1")
    rng, links, ov, s = _uniform_graph(41 + unit)
    ov[s] = 1 if drained_source else 0
    V = len(ov)
    csr = abi.Csr.from_links(V, links, overloaded=ov)
    g = abi.Graph(csr)
    L = int(csr.link_id.max()) + 1
    ign = _lists(rng, csr, s, L)
    # a second source in the same batch (its own neighbour rows)
    s2 = 7
    ign2 = _lists(rng, csr, s2, L)
    qs = [s] * len(ign) + [s2] * len(ign2)
    ign = ign + ign2
    flags = abi.SPF_F_NEXTHOPS | (abi.SPF_F_UNIT_METRIC if unit else 0)
    q = g.query(qs, flags, ignore=ign).run()
    assert FH in q.kernels(), q.kernels()
    assert "spf_whatif_pull_kernel" not in q.kernels()
    r = _reference(g, qs, flags, ign, monkeypatch)
    _same(q, r, len(qs))
    n1 = len(qs) - len(ign2)
    check_query(csr, q, qs, not unit, ignore=ign,
                rows={0, 1, 2, n1 - 2, n1 - 1, n1, len(qs) - 1} | set(range(3, n1, 7)))
    q.close()
    r.close()
    g.close()


def test_firsthop_fabric_transit_flips(gpu_ready, monkeypatch):
    """Fabric: every single-link failure at an FSW (84 first hops), then one
    of its RSWs and one of its SSWs drained, then undrained, rerunning the
    same query objects (both read the transit bits at run time)."""
    from openr_amd import topologies as TP

    topo = TP.fabric(2000)
    csr = topo.csr()
    r_, _ = topo.rank()
    s = int(r_[topo.names.index("2-0-0")])
    g = abi.Graph(csr)
    sl = _source_links(csr, s)
    ign = [[l] for l in sl] + [sorted(sl[:2]), sorted(sl[-3:])]
    qs = [s] * len(ign)
    flags = abi.SPF_F_NEXTHOPS
    q = g.query(qs, flags, ignore=ign)
    q.run()
    assert FH in q.kernels()
    r = _reference(g, qs, flags, ign, monkeypatch)
    _same(q, r, len(qs))
    check_query(csr, q, qs, True, ignore=ign, rows={0, 5, len(qs) - 1})
    r.close()
    rp = csr.row_ptr
    nbrs = sorted({int(csr.col[e]) for e in range(int(rp[s]), int(rp[s + 1]))})
    names = [topo.names[i] for i in np.argsort(r_)]  # CSR id -> name
    pick = [next(n for n in nbrs if names[n].startswith(p)) for p in ("3-", "1-")]
    ov = np.zeros(csr.num_nodes, dtype=np.uint8)
    ov[pick] = 1
    g.set_transit(ov)
    q.run()
    r = _reference(g, qs, flags, ign, monkeypatch)
    _same(q, r, len(qs))
    csr_d = copy.copy(csr)
    csr_d.overloaded = ov
    check_query(csr_d, q, qs, True, ignore=ign, rows={0, 1, len(qs) - 2})
    r.close()
    g.set_transit(np.zeros(csr.num_nodes, dtype=np.uint8))
    q.run()
    r = _reference(g, qs, flags, ign, monkeypatch)
    _same(q, r, len(qs))
    q.close()
    r.close()
    g.close()


def test_firsthop_source_link_set_down_between_runs(gpu_ready, monkeypatch):
    """A source link taken down in place (both halves, spf_graph_set_edges)
    between runs of the same query: its slot is no longer a usable first
    hop; then brought back up.  Each run equals a fresh from-scratch batch
    on the patched graph."""
    rng, links, ov, s = _uniform_graph(77)
    V = len(ov)
    csr = abi.Csr.from_links(V, links, overloaded=ov)
    g = abi.Graph(csr)
    L = int(csr.link_id.max()) + 1
    ign = _lists(rng, csr, s, L)
    qs = [s] * len(ign)
    flags = abi.SPF_F_NEXTHOPS
    q = g.query(qs, flags, ignore=ign)
    q.run()
    assert FH in q.kernels()
    sl = _source_links(csr, s)
    down = sl[len(sl) // 2]
    halves = np.flatnonzero(csr.link_id == down).astype(np.uint32)
    assert len(halves) == 2
    met = csr.metric[halves].astype(np.uint64)
    g.set_edges(halves, np.zeros(2, dtype=np.uint8), met)
    q.run()
    assert FH in q.kernels()
    r = _reference(g, qs, flags, ign, monkeypatch)
    _same(q, r, len(qs))
    r.close()
    g.set_edges(halves, np.ones(2, dtype=np.uint8), met)
    q.run()
    r = _reference(g, qs, flags, ign, monkeypatch)
    _same(q, r, len(qs))
    check_query(csr, q, qs, True, ignore=ign, rows={0, 1, len(qs) - 1})
    q.close()
    r.close()
    g.close()
