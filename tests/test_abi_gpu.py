"""GPU parity of the raw C ABI (spf_query_*) against the literal DijkstraQ
replay in oracle/spf_py.py, on seeded random graphs.

Covers: positive / unit / zero / negative (uint64 wrap) metrics, overloaded
(drained) nodes, parallel links, per-query ignored links, the LDS, global
memory and exact kernels.  Bit-exact distances and next-hop sets.
"""

import os
import random

import numpy as np
import pytest

from openr_amd import abi
from oracle import spf_py

pytestmark = pytest.mark.gpu

UNREACH = np.uint64(abi.SPF_UNREACHABLE)


def random_links(rng, V, L, wmin=1, wmax=20, parallel=0.05, asym=True):
    links = []
    # spanning-ish backbone so most nodes are reachable
    for v in range(1, V):
        u = rng.randrange(v)
        a = rng.randint(wmin, wmax)
        b = rng.randint(wmin, wmax) if asym else a
        links.append((u, v, a, b))
    while len(links) < L:
        u, v = rng.randrange(V), rng.randrange(V)
        if u == v:
            continue
        a = rng.randint(wmin, wmax)
        b = rng.randint(wmin, wmax) if asym else a
        links.append((u, v, a, b))
        if rng.random() < parallel:
            links.append((u, v, rng.randint(wmin, wmax), rng.randint(wmin, wmax)))
    rng.shuffle(links)
    return links


def check_query(csr, q, sources, use_metric, ignore=None, rows=None):
    for i, s in enumerate(sources):
        if rows is not None and i not in rows:
            continue
        ref = spf_py.run_spf(
            csr, s, use_metric, frozenset(ignore[i]) if ignore else frozenset()
        )
        d = q.dist(i)
        for v in range(csr.num_nodes):
            if v in ref:
                assert int(d[v]) == ref[v][0], (s, v)
            else:
                assert d[v] == UNREACH, (s, v)
        if q.flags & abi.SPF_F_NEXTHOPS:
            # unreached nodes: the empty next-hop set
            assert not q.nexthops(i)[d == UNREACH].any(), s
        if q.flags & abi.SPF_F_NEXTHOPS:
            got = q.nexthop_sets(i, s)
            for v, (m, nhs, _, _) in ref.items():
                if v == s:
                    assert got[v] == frozenset()
                else:
                    assert got[v] == nhs, (s, v, got[v], nhs)


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_weighted_random(gpu_ready, seed):
    rng = random.Random(seed)
    V = 300
    links = random_links(rng, V, 1200)
    ov = [1 if rng.random() < 0.03 else 0 for _ in range(V)]
    csr = abi.Csr.from_links(V, links, ov)
    g = abi.Graph(csr)
    assert not g.needs_exact
    sources = list(range(0, V, 7))
    q = g.query(sources, abi.SPF_F_NEXTHOPS).run()
    assert q.kernel == "lds"
    check_query(csr, q, sources, True)
    qu = g.query(sources, abi.SPF_F_NEXTHOPS | abi.SPF_F_UNIT_METRIC).run()
    check_query(csr, qu, sources, False)
    qd = g.query(sources, 0).run()
    check_query(csr, qd, sources, True)


def test_ignore_lists(gpu_ready):
    rng = random.Random(11)
    V = 200
    links = random_links(rng, V, 700)
    csr = abi.Csr.from_links(V, links)
    g = abi.Graph(csr)
    sources = [rng.randrange(V) for _ in range(40)]
    ignore = [rng.sample(range(len(links)), rng.randint(0, 30)) for _ in sources]
    q = g.query(sources, abi.SPF_F_NEXTHOPS, ignore=ignore).run()
    check_query(csr, q, sources, True, ignore)


def test_high_degree_masks(gpu_ready):
    # a hub with 300 neighbours -> 5 mask words (WMAX 16 kernel)
    V = 400
    links = [(0, v, 1, 1) for v in range(1, 301)]
    links += [(v, 300 + (v % 99) + 1, 2, 3) for v in range(1, 301)]
    csr = abi.Csr.from_links(V, links)
    g = abi.Graph(csr)
    q = g.query([0, 5, 350], abi.SPF_F_NEXTHOPS).run()
    assert q.nh_words(0) == 5
    check_query(csr, q, [0, 5, 350], True)


@pytest.mark.parametrize("seed", [4, 5])
def test_zero_metric_exact(gpu_ready, seed):
    rng = random.Random(seed)
    V = 150
    links = random_links(rng, V, 500, wmin=0, wmax=5)
    ov = [1 if rng.random() < 0.05 else 0 for _ in range(V)]
    csr = abi.Csr.from_links(V, links, ov)
    g = abi.Graph(csr)
    assert g.needs_exact
    sources = list(range(0, V, 5))
    q = g.query(sources, abi.SPF_F_NEXTHOPS | abi.SPF_F_ORDER).run()
    assert q.kernel == "wide"
    check_query(csr, q, sources, True)
    for i, s in enumerate(sources):
        ref = spf_py.run_spf(csr, s, True)
        order = q.order(i)
        for v, (_, _, _, rank) in ref.items():
            assert int(order[v]) == rank


def test_zero_metric_triangle_name_order(gpu_ready):
    # SURVEY §8(a) probe: all-zero triangle from "1": nh(2)={2}, nh(3)={2,3}
    # with node ids = name ranks 0:"1", 1:"2", 2:"3"
    csr = abi.Csr.from_links(3, [(0, 1, 0, 0), (0, 2, 0, 0), (1, 2, 0, 0)])
    g = abi.Graph(csr)
    q = g.query([0], abi.SPF_F_NEXTHOPS).run()
    sets = q.nexthop_sets(0, 0)
    assert sets[1] == frozenset({1})
    assert sets[2] == frozenset({1, 2})


def test_negative_metric_wraps(gpu_ready):
    # an i32 metric of -5 is the uint64 2^64-5 (LinkStateMetric)
    m = (1 << 64) - 5
    csr = abi.Csr.from_links(4, [(0, 1, m, 1), (1, 2, 10, 10), (0, 2, 3, 3), (2, 3, 1, 1)])
    g = abi.Graph(csr)
    assert g.needs_exact
    q = g.query([0, 1, 2, 3], abi.SPF_F_NEXTHOPS).run()
    check_query(csr, q, [0, 1, 2, 3], True)


def test_gmem_kernel_large_graph(gpu_ready):
    rng = random.Random(21)
    V = 70000
    links = random_links(rng, V, 150000, wmin=1, wmax=50, parallel=0.0)
    csr = abi.Csr.from_links(V, links)
    g = abi.Graph(csr)
    q = g.query([0, 12345], abi.SPF_F_NEXTHOPS).run()
    assert q.kernel == "dstep"
    check_query(csr, q, [0, 12345], True)


@pytest.mark.parametrize("seed,ldsbkt", [(31, "1"), (32, "1"), (33, "0")])
def test_dstep_vs_frontier_gmem(gpu_ready, seed, ldsbkt, monkeypatch):
    """Delta-stepping (large weighted graphs) against the literal replay
    and against the frontier Bellman-Ford gmem kernel on the same batch:
    drained nodes, parallel links, asymmetric metrics, ignore lists, several
    bucket widths (incl. the saturated last bucket), bucket bytes read from
    the distance row (default) or kept in LDS."""
    monkeypatch.setenv("OPENR_SPF_DSTEP_LDSBKT", ldsbkt)
    rng = random.Random(seed)
    V = 40000
    links = random_links(rng, V, 120000, wmin=1, wmax=300, parallel=0.02)
    ov = np.zeros(V, dtype=np.uint8)
    ov[rng.sample(range(V), 400)] = 1
    csr = abi.Csr.from_links(V, links, overloaded=ov)
    g = abi.Graph(csr)
    srcs = [0, 777, 39999]
    ign = [[], sorted(rng.sample(range(len(links)), 50)), [int(csr.link_id[csr.row_ptr[39999]])]]
    for shift in ("0", "3", "9", "20"):
        monkeypatch.setenv("OPENR_SPF_DSTEP_SHIFT", shift)
        q = g.query(srcs, abi.SPF_F_NEXTHOPS, ignore=ign).run()
        assert q.kernel == "dstep"
        check_query(csr, q, srcs, True, ignore=ign, rows={0, 1, 2} if shift == "3" else {1})
        # distances only: the push / atomicMin variant must give the same rows
        qd = g.query(srcs, 0, ignore=ign).run()
        assert qd.kernel == "dstep"
        for i in range(len(srcs)):
            assert (qd.dist(i) == q.dist(i)).all(), (shift, i)
        if shift == "9":
            monkeypatch.setenv("OPENR_SPF_DSTEP", "0")
            r = g.query(srcs, abi.SPF_F_NEXTHOPS, ignore=ign).run()
            monkeypatch.delenv("OPENR_SPF_DSTEP")
            assert r.kernel == "gmem"
            for i in range(len(srcs)):
                assert (q.dist(i) == r.dist(i)).all()
                if not (q.nexthops(i) == r.nexthops(i)).all():
                    bad = np.flatnonzero((q.nexthops(i) != r.nexthops(i)).any(axis=1))
                    ok_q = ok_r = True
                    try:
                        check_query(csr, q, srcs, True, ignore=ign, rows={i})
                    except AssertionError:
                        ok_q = False
                    try:
                        check_query(csr, r, srcs, True, ignore=ign, rows={i})
                    except AssertionError:
                        ok_r = False
                    raise AssertionError(
                        f"row {i}: {len(bad)} nodes differ (first {bad[:5]}); "
                        f"dstep matches replay: {ok_q}, gmem matches replay: {ok_r}")


@pytest.mark.parametrize("seed", [41, 42])
def test_msdstep_vs_dstep_and_replay(gpu_ready, seed, monkeypatch):
    """Multi-source delta-stepping (32 sources per workgroup, node-major
    slab) against the per-source delta-stepping kernel on every row and the
    literal replay on two rows: drained nodes (also as sources), parallel
    links, duplicate sources, a partial last batch, bucket widths from
    'everything saturates into the last bucket' to 'one bucket', clustered
    and unclustered batches."""
    rng = random.Random(seed)
    V = 70000
    links = random_links(rng, V, 200000, wmin=1, wmax=300, parallel=0.02)
    ov = np.zeros(V, dtype=np.uint8)
    ov[rng.sample(range(V), 700)] = 1
    csr = abi.Csr.from_links(V, links, overloaded=ov)
    g = abi.Graph(csr)
    drained = [int(v) for v in np.flatnonzero(ov)[:3]]
    srcs = [rng.randrange(V) for _ in range(150)] + drained + [5, 5, 77]
    ref = g.query(srcs, 0).run()
    assert ref.kernel == "dstep-ldsrow"  # distance rows in LDS (metrics <= 300)
    monkeypatch.setenv("OPENR_SPF_MSD", "1")
    want = [ref.dist(i) for i in range(len(srcs))]
    for shift, cluster in (("0", "1"), ("4", "0"), (None, "1"), ("30", "1")):
        if shift is None:
            monkeypatch.delenv("OPENR_SPF_MSD_SHIFT", raising=False)
        else:
            monkeypatch.setenv("OPENR_SPF_MSD_SHIFT", shift)
        monkeypatch.setenv("OPENR_SPF_MSD_CLUSTER", cluster)
        q = g.query(srcs, 0).run()
        assert q.kernel == "msdstep"
        for i in range(len(srcs)):
            assert (q.dist(i) == want[i]).all(), (shift, cluster, i)
    check_query(csr, q, srcs, True, rows={0, len(srcs) - 4})


def test_msdstep_wan_anchor(gpu_ready):
    """100k-node WAN (SURVEY §8(d) generator): the row of source 0 from the
    multi-source kernel reproduces the reference runSpf checksum, and 16
    sampled rows equal the per-source kernel's."""
    import json
    import os

    from openr_amd import topologies as TP

    gold = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "wan_anchors.json")))
    a = [x for x in gold["anchors"] if x["V"] == 100000][0]
    topo = TP.wan(a["V"], a["L"])
    csr = topo.csr()
    g = abi.Graph(csr)
    srcs = np.arange(0, a["V"], 397, dtype=np.uint32)[:256]
    assert srcs[0] == 0
    os.environ["OPENR_SPF_MSD"] = "1"
    try:
        q = g.query(srcs, 0).run()
    finally:
        del os.environ["OPENR_SPF_MSD"]
    assert q.kernel == "msdstep"
    d0 = q.dist(0)
    assert (d0 != UNREACH).all()
    assert int(d0.sum()) == a["sum_dist"]
    rows = list(range(0, 256, 16))
    r = g.query(srcs[rows], 0).run()  # 16 sources: per-source kernel
    assert r.kernel == "dstep-ldsrow"
    for k, i in enumerate(rows):
        assert (q.dist(i) == r.dist(k)).all(), i


def test_transit_update(gpu_ready):
    rng = random.Random(8)
    V = 120
    links = random_links(rng, V, 400)
    csr = abi.Csr.from_links(V, links)
    g = abi.Graph(csr)
    ov = np.zeros(V, dtype=np.uint8)
    ov[rng.sample(range(V), 10)] = 1
    g.set_transit(ov)
    csr.overloaded = ov
    q = g.query(list(range(V)), abi.SPF_F_NEXTHOPS).run()
    check_query(csr, q, list(range(V)), True)


# ---- batch plans: distance rows + next hops from rows (neighbour-closed batches)


@pytest.mark.parametrize("seed", [31, 32])
def test_all_sources_rows_plan_weighted(gpu_ready, seed):
    rng = random.Random(seed)
    V = 250
    links = random_links(rng, V, 900)
    ov = [1 if rng.random() < 0.05 else 0 for _ in range(V)]
    csr = abi.Csr.from_links(V, links, ov)
    g = abi.Graph(csr)
    sources = list(range(V))
    q = g.query(sources, abi.SPF_F_NEXTHOPS).run()
    assert q.kernel == "lds+rows"
    check_query(csr, q, sources, True)


@pytest.fixture(params=["0", "32", "64"])
def msbfs(request, monkeypatch):
    monkeypatch.setenv("OPENR_SPF_MSBFS", request.param)
    return request.param


def _bfs_kernel(msbfs, nh=True):
    if msbfs == "0":
        return "bfs+rows" if nh else "bfs"
    return "msbfs+levels" if nh else "msbfs"


@pytest.mark.parametrize("seed", [41, 42])
def test_all_sources_bfs_plan(gpu_ready, seed, msbfs):
    rng = random.Random(seed)
    V = 300
    links = random_links(rng, V, 1000)
    ov = [1 if rng.random() < 0.05 else 0 for _ in range(V)]
    csr = abi.Csr.from_links(V, links, ov)
    g = abi.Graph(csr)
    sources = list(range(V))
    q = g.query(sources, abi.SPF_F_NEXTHOPS | abi.SPF_F_UNIT_METRIC).run()
    assert q.kernel == _bfs_kernel(msbfs)
    check_query(csr, q, sources, False)
    qd = g.query(sources[::3], abi.SPF_F_UNIT_METRIC).run()
    assert qd.kernel == _bfs_kernel(msbfs, nh=False)
    check_query(csr, qd, sources[::3], False)


def test_uniform_metric_scaled_bfs(gpu_ready, msbfs):
    rng = random.Random(5)
    V = 200
    links = [(u, v, 7, 7) for (u, v, _, _) in random_links(rng, V, 600)]
    csr = abi.Csr.from_links(V, links)
    g = abi.Graph(csr)
    sources = list(range(V))
    q = g.query(sources, abi.SPF_F_NEXTHOPS).run()
    assert q.kernel == _bfs_kernel(msbfs)
    check_query(csr, q, sources, True)


def test_deep_graph_many_levels(gpu_ready, msbfs):
    # a 300-node path: BFS depth 299 > 255 exercises the 32-bit fallback of
    # the level rows and long MS-BFS level loops
    V = 300
    links = [(i, i + 1, 1, 1) for i in range(V - 1)]
    csr = abi.Csr.from_links(V, links)
    g = abi.Graph(csr)
    sources = list(range(V))
    q = g.query(sources, abi.SPF_F_NEXTHOPS).run()
    assert q.kernel == _bfs_kernel(msbfs)
    check_query(csr, q, sources, True, rows=set(range(0, V, 37)) | {V - 1})
    # reruns: the MS-BFS "level >= 255" flag alternates between two words
    # per launch (each launch clears the other), so both words are exercised
    for _ in range(2):
        q.run()
        check_query(csr, q, sources, True, rows={0, 150, V - 1})


def test_fabric_all_sources_sampled(gpu_ready, msbfs):
    from openr_amd import topologies as TP

    topo = TP.fabric(2000)  # 29 pods, same structure as the 10k fabric
    rsw = [i for i, n in enumerate(topo.names) if n.startswith("3-")]
    csr = topo.csr(overloaded=[rsw[3], rsw[77]])
    g = abi.Graph(csr)
    sources = list(range(csr.num_nodes))
    q = g.query(sources, abi.SPF_F_NEXTHOPS).run()
    assert q.kernel == _bfs_kernel(msbfs)
    check_query_sample = sources[:: max(1, len(sources) // 25)]
    for i in check_query_sample:
        ref = spf_py.run_spf(csr, i, True)
        d = q.dist(i)
        got = q.nexthop_sets(i, i)
        for v in range(csr.num_nodes):
            if v in ref:
                assert int(d[v]) == ref[v][0]
                if v != i:
                    assert got[v] == ref[v][1], (i, v)
            else:
                assert d[v] == UNREACH


def test_gmem_bfs_plan_large(gpu_ready):
    rng = random.Random(22)
    V = 70000
    links = random_links(rng, V, 140000, wmin=1, wmax=1, parallel=0.0)
    csr = abi.Csr.from_links(V, links)
    g = abi.Graph(csr)
    q = g.query([0, 4321, 69999], abi.SPF_F_UNIT_METRIC).run()
    assert q.kernel == "bfs-gmem"
    check_query(csr, q, [0, 4321, 69999], False)


def test_bulk_fetch_matches_row_reads(gpu_ready):
    """spf_query_fetch_rows (host) / spf_query_fetch_nexthops return exactly
    the per-row spf_query_dist / spf_query_nexthops contents, in order."""
    rng = random.Random(12)
    V = 300
    csr = abi.Csr.from_links(V, random_links(rng, V, 900, parallel=0.05))
    srcs = rng.sample(range(V), 40)
    q = g_query = abi.Graph(csr).query(srcs, abi.SPF_F_NEXTHOPS).run()
    rows = np.zeros((len(srcs), V), dtype=np.uint32)
    q.fetch_rows(0, len(srcs), rows.ctypes.data, V * 4, on_device=False)
    flat = q.fetch_nexthops(0, len(srcs))
    off = 0
    for i in range(len(srcs)):
        d = q.dist(i)
        assert (np.where(d == UNREACH, np.uint64(0xFFFFFFFF), d) == rows[i]).all()
        m = q.nexthops(i).ravel()
        assert (flat[off : off + m.size] == m).all()
        off += m.size
    assert off == flat.size
    # spf_query_fetch_host: both in one call, through the pinned staging
    # buffer (small) and through the two plain calls (staging off), over a
    # sub-range, rows or masks alone
    for stage in ("1", "0"):
        os.environ["OPENR_SPF_FETCH_STAGE"] = stage
        try:
            r2, f2 = q.fetch_host(0, len(srcs))
            assert (r2 == rows).all() and (f2 == flat).all()
            r3, f3 = q.fetch_host(5, 7)
            lo = sum(q.nexthops(i).size for i in range(5))
            assert (r3 == rows[5:12]).all()
            assert (f3 == flat[lo : lo + f3.size]).all()
            assert q.fetch_host(3, 2, masks=False)[1] is None
            lo3 = sum(q.nexthops(i).size for i in range(3))
            n3 = q.nexthops(3).size + q.nexthops(4).size
            assert (q.fetch_host(3, 2, rows=False)[1] == flat[lo3 : lo3 + n3]).all()
        finally:
            os.environ.pop("OPENR_SPF_FETCH_STAGE", None)
    del g_query


@pytest.mark.parametrize("weighted", [False, True])
def test_whatif_screen_matches_full_runs(gpu_ready, weighted, monkeypatch):
    """Single-link-failure batches from repeated sources: queries whose
    failed link is off the baseline shortest-path DAG copy the baseline rows
    (the screen); the result must equal running every query in full, and the
    replay on sampled queries, including drained nodes, parallel links and
    link ids beyond the graph (they match nothing)."""
    rng = random.Random(91 + weighted)
    V = 2000
    links = random_links(rng, V, 6000, wmin=1, wmax=30 if weighted else 1, parallel=0.03)
    ov = np.zeros(V, dtype=np.uint8)
    ov[rng.sample(range(V), 40)] = 1
    csr = abi.Csr.from_links(V, links, overloaded=ov)
    g = abi.Graph(csr)
    srcs = [0] * 300 + [int(np.flatnonzero(ov)[0])] * 100 + [7] * 100
    ign = [[rng.randrange(len(links))] for _ in srcs]
    ign[5] = [len(links) + 3]  # no such link
    ign[6] = []
    q = g.query(srcs, abi.SPF_F_NEXTHOPS, ignore=ign).run()
    monkeypatch.setenv("OPENR_SPF_WHATIF_SCREEN", "0")
    r = g.query(srcs, abi.SPF_F_NEXTHOPS, ignore=ign).run()
    for i in range(len(srcs)):
        assert (q.dist(i) == r.dist(i)).all(), i
        assert (q.nexthops(i) == r.nexthops(i)).all(), i
    check_query(csr, q, srcs, True, ignore=ign, rows={0, 5, 6, 310, 499})


@pytest.mark.parametrize("V,L,wmax", [(300, 1200, 10 ** 8), (20000, 80000, 10 ** 6)])
def test_hop_bound_keeps_32bit_rows(gpu_ready, V, L, wmax, monkeypatch):
    """Large metrics whose coarse bound maxw * (V - 1) passes 2^32 still run
    the 32-bit plans when maxw * (transit hop bound + 1) fits (refresh_exact):
    same rows as the literal replay, drained nodes included; the 64-bit
    plan (OPENR_SPF_HOP_BOUND=0) agrees bit for bit."""
    from openr_amd.allsources import needs_64bit_rows

    rng = random.Random(V)
    links = random_links(rng, V, L, wmin=1, wmax=wmax, parallel=0.01)
    ov = np.zeros(V, dtype=np.uint8)
    ov[rng.sample(range(V), V // 100)] = 1
    csr = abi.Csr.from_links(V, links, overloaded=ov)
    assert wmax * (V - 1) >= 1 << 32
    g = abi.Graph(csr)
    assert not g.needs_exact
    assert not needs_64bit_rows(csr)
    srcs = [0, 1, V - 1] + [rng.randrange(V) for _ in range(5)]
    q = g.query(srcs, abi.SPF_F_NEXTHOPS).run()
    assert q.kernel != "wide"
    rows = set(range(len(srcs))) if V <= 1000 else {0, 2}
    check_query(csr, q, srcs, True, rows=rows)
    monkeypatch.setenv("OPENR_SPF_HOP_BOUND", "0")
    g64 = abi.Graph(csr)
    assert g64.needs_exact
    w = g64.query(srcs, abi.SPF_F_NEXTHOPS).run()
    assert w.kernel == "wide"
    for i in range(len(srcs)):
        assert (w.dist(i) == q.dist(i)).all(), i
        assert w.nexthop_sets(i, srcs[i]) == q.nexthop_sets(i, srcs[i]), i


def test_hop_bound_follows_drains(gpu_ready):
    """A drain that partitions the transit graph withdraws the hop bound
    (spf_graph_set_transit re-runs refresh_exact); undraining restores it."""
    # star 0 - {1..8} plus 9 - 8: hub 0, ecc 2 -> bound 4 hops; 5w fits in
    # 32 bits, the coarse 9w does not
    w = (1 << 32) // 7
    links = [(0, v, w, w) for v in range(1, 9)] + [(8, 9, w, w)]
    csr = abi.Csr.from_links(10, links)
    g = abi.Graph(csr)
    assert not g.needs_exact
    ov = np.zeros(10, dtype=np.uint8)
    ov[8] = 1
    g.set_transit(ov)
    assert g.needs_exact  # the hub no longer reaches 9
    g.set_transit(np.zeros(10, dtype=np.uint8))
    assert not g.needs_exact


@pytest.mark.parametrize("sell,wrec", [("0", "1"), ("1", "1"), ("1", "0")])
def test_msbfs_sliced_ell_matches_csr(gpu_ready, sell, wrec, monkeypatch):
    """MS-BFS over the sliced-ELL copy of the CSR (upload_sell) and over the
    plain CSR, with wave-cooperative or per-lane row stores: identical
    distance and next-hop rows, checked against the literal replay on a few
    sources (irregular degrees, drained nodes, parallel links, a ragged last
    slice)."""
    monkeypatch.setenv("OPENR_MS_SELL", sell)
    monkeypatch.setenv("OPENR_MS_WREC", wrec)
    rng = random.Random(77)
    V = 3001
    links = random_links(rng, V, 9000, wmin=1, wmax=1, parallel=0.05)
    links += [(5, v, 1, 1) for v in range(100, 400)]  # a hub: a wide slice
    ov = np.zeros(V, dtype=np.uint8)
    ov[rng.sample(range(V), 30)] = 1
    csr = abi.Csr.from_links(V, links, overloaded=ov)
    g = abi.Graph(csr)
    srcs = np.arange(V, dtype=np.uint32)
    q = g.query(srcs, abi.SPF_F_NEXTHOPS | abi.SPF_F_UNIT_METRIC).run()
    assert q.kernel == "msbfs+levels"
    check_query(csr, q, [int(s) for s in srcs], False, rows={0, 5, 17, 1500, V - 1})
    monkeypatch.setenv("OPENR_MS_SELL", "1" if sell == "0" else "0")
    monkeypatch.setenv("OPENR_MS_WREC", "1" if wrec == "0" else "0")
    r = g.query(srcs, abi.SPF_F_NEXTHOPS | abi.SPF_F_UNIT_METRIC).run()
    for i in range(0, V, 97):
        assert (q.dist(i) == r.dist(i)).all(), i
        assert (q.nexthops(i) == r.nexthops(i)).all(), i


@pytest.mark.parametrize("case", ["random", "hubs", "wide_hubs", "deep"])
def test_nh_levels_swar_matches_scalar(gpu_ready, case, monkeypatch):
    """The byte-SIMD next-hop pass (spf_nh_levels_held_kernel, its 4-8 word
    instance and spf_nh_levels_swar_kernel) against the per-node pass
    (spf_nh_levels_kernel) on the same MS-BFS rows, and both against the
    literal replay on a few sources: drained neighbours (next hop only to
    themselves), sources with 1-3, 4-8 and more mask words, a ragged last
    chunk, and a BFS deeper than 254 levels (the 32-bit-row branch)."""
    rng = random.Random({"random": 5, "hubs": 6, "wide_hubs": 8, "deep": 7}[case])
    if case == "deep":
        V = 700  # a 600-node chain hanging off a random core: levels > 255
        links = random_links(rng, 100, 400, wmin=1, wmax=1, parallel=0.0)
        links += [(99 + i, 100 + i, 1, 1) for i in range(600)]
    else:
        V = 2500 if case == "random" else 1300
        links = random_links(rng, V, 7000, wmin=1, wmax=1, parallel=0.03)
        if case == "hubs":
            links += [(7, v, 1, 1) for v in range(100, 260)]  # 3 mask words
            links += [(8, v, 1, 1) for v in range(300, 400)]  # 2 mask words
        if case == "wide_hubs":
            links += [(7, v, 1, 1) for v in range(20, 300)]   # 5 mask words
            links += [(8, v, 1, 1) for v in range(300, 800)]  # 8 mask words
            links += [(9, v, 1, 1) for v in range(200, 800)]  # 10 mask words (generic)
    ov = np.zeros(V, dtype=np.uint8)
    ov[rng.sample(range(V), V // 40)] = 1
    csr = abi.Csr.from_links(V, links, overloaded=ov)
    g = abi.Graph(csr)
    srcs = np.arange(V, dtype=np.uint32)
    flags = abi.SPF_F_NEXTHOPS | abi.SPF_F_UNIT_METRIC
    monkeypatch.setenv("OPENR_NL_SWAR", "1")
    a = g.query(srcs, flags).run()
    assert a.kernel == "msbfs+levels"
    monkeypatch.setenv("OPENR_NL_SWAR", "0")
    b = g.query(srcs, flags).run()
    for i in range(V):
        assert a.nh_words(i) == b.nh_words(i)
    ma = a.fetch_nexthops(0, V)
    mb = b.fetch_nexthops(0, V)
    if not (ma == mb).all():
        bad = int(np.flatnonzero(ma != mb)[0])
        pytest.fail(f"mask word {bad} differs: {ma[bad]:#x} vs {mb[bad]:#x}")
    probe = [0, 7, 8, 9, V - 1, V // 2] if case != "deep" else [0, 99, 650, 699]
    check_query(csr, a, [int(s) for s in srcs], False, rows=set(probe))


@pytest.mark.parametrize("case", ["weighted", "uniform", "large"])
def test_sparse_metric_patch_equals_fresh_graph(gpu_ready, case, monkeypatch):
    """spf_graph_patch_metrics' sparse path (a few edges: only their device
    words are scattered, scalars rescanned) gives the same rows and masks as
    a graph created from the patched CSR, and as the full re-upload
    (OPENR_SPF_PATCH_INPLACE=0): weighted / uniform-metric (the patch breaks
    and then restores uniformity, i.e. the MS-BFS plan) / delta-stepping
    graphs, parallel links (cheapest-neighbour metric), drained nodes."""
    rng = random.Random({"weighted": 51, "uniform": 52, "large": 53}[case])
    V = {"weighted": 400, "uniform": 2000, "large": 40000}[case]
    wmax = 1 if case == "uniform" else 30
    links = random_links(rng, V, 4 * V, wmin=1, wmax=wmax, parallel=0.05)
    ov = np.zeros(V, dtype=np.uint8)
    ov[rng.sample(range(V), V // 50)] = 1
    csr = abi.Csr.from_links(V, links, overloaded=ov)
    srcs = [0, 1, V // 2, V - 1] if case != "uniform" else list(range(64))
    flags = abi.SPF_F_NEXTHOPS
    for inplace in ("1", "0"):
        monkeypatch.setenv("OPENR_SPF_PATCH_INPLACE", inplace)
        g = abi.Graph(csr)
        metric = csr.metric.copy()
        for step in range(3):
            E = len(metric)
            k = 6
            e = np.array(rng.sample(range(E), k), dtype=np.uint32)
            if case == "uniform" and step == 2:
                m = np.ones(k, dtype=np.uint64)  # restore: uniform again below
                e = np.flatnonzero(metric != 1).astype(np.uint32)[:64]
                m = np.ones(len(e), dtype=np.uint64)
            else:
                m = np.array([rng.randint(1, 40) for _ in range(k)], dtype=np.uint64)
            g.patch_metrics(e, m)
            metric[e] = m
            fresh_csr = abi.Csr(csr.num_nodes, csr.row_ptr, csr.col, metric.copy(), csr.link_id,
                                csr.rev, csr.overloaded, csr.num_links)
            f = abi.Graph(fresh_csr)
            assert g.needs_exact == f.needs_exact
            a = g.query(srcs, flags).run()
            b = f.query(srcs, flags).run()
            assert a.kernel == b.kernel, (step, a.kernel, b.kernel)
            for i in range(len(srcs)):
                assert (a.dist(i) == b.dist(i)).all(), (inplace, step, i)
                assert (a.nexthops(i) == b.nexthops(i)).all(), (inplace, step, i)
            check_query(fresh_csr, a, srcs, True, rows={0, len(srcs) - 1} if V > 1000 else None)
            a.close()
            b.close()
            f.close()
        g.close()


@pytest.mark.parametrize("block", [(0, 700), (1300, 1900), (2900, 3001)])
def test_msbfs_block_with_helper_sources(gpu_ready, block):
    """One rank's block of an all-sources table (sources whose neighbours lie
    outside the block): the MS-BFS plan computes the missing neighbours' level
    rows as helper sources, so the block keeps msbfs+levels, and its rows and
    masks equal the full batch's rows for the same sources."""
    rng = random.Random(91)
    V = 3001
    links = random_links(rng, V, 9000, wmin=1, wmax=1, parallel=0.03)
    ov = np.zeros(V, dtype=np.uint8)
    ov[rng.sample(range(V), 40)] = 1
    csr = abi.Csr.from_links(V, links, overloaded=ov)
    g = abi.Graph(csr)
    flags = abi.SPF_F_NEXTHOPS | abi.SPF_F_UNIT_METRIC
    full = g.query(np.arange(V, dtype=np.uint32), flags).run()
    lo, hi = block
    srcs = np.arange(lo, hi, dtype=np.uint32)
    q = g.query(srcs, flags).run()
    assert q.kernel == "msbfs+levels"
    n = hi - lo
    got = np.empty((n, V), dtype=np.uint32)
    want = np.empty((n, V), dtype=np.uint32)
    q.fetch_rows(0, n, got.ctypes.data, V * 4, on_device=False)
    full.fetch_rows(lo, n, want.ctypes.data, V * 4, on_device=False)
    assert (got == want).all()
    for i in range(0, n, 37):
        assert (q.nexthops(i) == full.nexthops(lo + i)).all(), i
    check_query(csr, q, [int(s) for s in srcs], False, rows={0, n - 1})


def test_msbfs_20k_nodes_32bit_batches(gpu_ready):
    """Past 16 Ki nodes (fabric(20000): 20,000 nodes) the MS-BFS plan runs
    32-source batches with 20 nodes per thread (the 2 * V * 4-byte frontier
    double buffer still fits 160 KB of LDS): rows and masks against the
    literal replay on sampled sources."""
    rng = random.Random(2020)
    V = 20000
    links = random_links(rng, V, 60000, wmin=1, wmax=1, parallel=0.0)
    ov = np.zeros(V, dtype=np.uint8)
    ov[rng.sample(range(V), 200)] = 1
    csr = abi.Csr.from_links(V, links, overloaded=ov)
    g = abi.Graph(csr)
    srcs = np.arange(0, V, 97, dtype=np.uint32)[:96]
    q = g.query(srcs, abi.SPF_F_NEXTHOPS | abi.SPF_F_UNIT_METRIC).run()
    assert q.kernel == "msbfs+levels"
    check_query(csr, q, [int(s) for s in srcs], False, rows={0, 50, 95})


@pytest.mark.parametrize("seed", [71, 72])
def test_msbfs_ignore_lists(gpu_ready, seed, monkeypatch):
    """Distance-only batches with ignore lists on a uniform metric run the
    bit-parallel BFS with per-batch masks of the ignored half-edges (KSP2
    second passes): rows equal the per-query SSSP (OPENR_SPF_MSBFS_IGN=0)
    and the literal replay, with drained nodes, parallel links (one of two
    parallel links ignored keeps the other), repeated and distinct sources,
    lists from empty to hundreds of links, ids beyond the graph, and a batch
    that is not a multiple of 64."""
    rng = random.Random(seed)
    V = 1500
    links = random_links(rng, V, 5000, wmin=3, wmax=3, parallel=0.05, asym=False)
    ov = np.zeros(V, dtype=np.uint8)
    ov[rng.sample(range(V), 30)] = 1
    csr = abi.Csr.from_links(V, links, overloaded=ov)
    g = abi.Graph(csr)
    srcs = [rng.randrange(V) for _ in range(60)] + [7] * 70
    ign = []
    for i in range(len(srcs)):
        k = rng.choice([0, 1, 3, 20, 200])
        ign.append(rng.sample(range(len(links)), k) + ([len(links) + 5] if i % 9 == 0 else []))
    q = g.query(srcs, 0, ignore=ign).run()
    assert q.kernel == "msbfs"
    monkeypatch.setenv("OPENR_SPF_MSBFS_IGN", "0")
    r = g.query(srcs, 0, ignore=ign).run()
    assert r.kernel != "msbfs"
    for i in range(len(srcs)):
        assert (q.dist(i) == r.dist(i)).all(), i
    check_query(csr, q, srcs, True, ignore=ign, rows={0, 5, 63, 64, 100, 129})
    q.close()
    r.close()
    g.close()
