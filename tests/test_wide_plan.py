"""GPU parity of the wide plan (spf_wide_kernel): 64-bit distances, metric-0
plateaus and next hops for the graphs the 32-bit plans cannot take, against
the literal DijkstraQ replay (oracle/spf_py.py, LinkState.cpp:806-880) and,
at sizes the replay cannot reach, the flat CPU restatement
(oracle/csr_spf.h, positive metrics).

The wide plan replaced the per-area fall-back to one thread per query
(spf_exact_kernel): metric 0 anywhere in an area, or maxw * (V - 1) >= 2^32
(e.g. a 100k-node WAN with metrics up to 10^6).  The literal replay now only
runs for metrics that wrap (negative i32 as uint64).
"""

import random

import numpy as np
import pytest

from openr_amd import abi
from oracle import spf_py

from .test_abi_gpu import check_query, random_links

pytestmark = pytest.mark.gpu


def check_order(csr, q, sources, use_metric=True, ignore=None, rows=None):
    """Settle ranks (spf_query_order) and the (dist, key) comparison
    (spf_query_order_keys) both equal the replay's extraction order, for the
    query rows `rows` (default: all)."""
    for i, s in enumerate(sources):
        if rows is not None and i not in rows:
            continue
        ref = spf_py.run_spf(csr, s, use_metric, frozenset(ignore[i]) if ignore else frozenset())
        order = q.order(i)
        for v, (_, _, _, rank) in ref.items():
            assert int(order[v]) == rank, (s, v)
        keys = q.order_keys(i)
        d = q.dist(i)
        seq = sorted(ref, key=lambda v: (int(d[v]), int(keys[v])))
        assert [ref[v][3] for v in seq] == list(range(len(seq))), s


@pytest.mark.parametrize("seed", [4, 5, 6, 7])
def test_zero_metric_plateaus(gpu_ready, seed):
    rng = random.Random(seed)
    V = 150
    links = random_links(rng, V, 500, wmin=0, wmax=5)
    ov = [1 if rng.random() < 0.05 else 0 for _ in range(V)]
    csr = abi.Csr.from_links(V, links, ov)
    g = abi.Graph(csr)
    assert g.needs_exact
    sources = list(range(V))
    q = g.query(sources, abi.SPF_F_NEXTHOPS | abi.SPF_F_ORDER).run()
    assert q.kernel == "wide"
    check_query(csr, q, sources, True)
    check_order(csr, q, sources, rows=set(range(0, V, 7)))
    # distances only, no order: same rows
    qd = g.query(sources, 0).run()
    assert qd.kernel == "wide"
    for i in range(0, V, 11):
        assert (qd.dist(i) == q.dist(i)).all()


@pytest.mark.parametrize("zero_frac", [0.3, 1.0])
def test_dense_zero_plateaus(gpu_ready, zero_frac):
    """Large plateaus: 30 % and 100 % metric-0 links (one plateau of every
    node: the whole replay is the plateau heap)."""
    rng = random.Random(int(zero_frac * 100))
    V = 120
    links = []
    for u, v, a, b in random_links(rng, V, 420, wmin=1, wmax=4):
        if rng.random() < zero_frac:
            a = 0
        if rng.random() < zero_frac:
            b = 0
        links.append((u, v, a, b))
    ov = [1 if rng.random() < 0.05 else 0 for _ in range(V)]
    csr = abi.Csr.from_links(V, links, ov)
    g = abi.Graph(csr)
    sources = list(range(0, V, 3))
    q = g.query(sources, abi.SPF_F_NEXTHOPS | abi.SPF_F_ORDER).run()
    assert q.kernel == "wide"
    check_query(csr, q, sources, True)
    check_order(csr, q, sources, rows=set(range(0, len(sources), 4)))


def test_zero_metric_ignore_lists(gpu_ready):
    rng = random.Random(17)
    V = 160
    links = random_links(rng, V, 560, wmin=0, wmax=6)
    csr = abi.Csr.from_links(V, links)
    g = abi.Graph(csr)
    sources = [rng.randrange(V) for _ in range(48)]
    ignore = [sorted(rng.sample(range(len(links)), rng.randint(0, 40))) for _ in sources]
    q = g.query(sources, abi.SPF_F_NEXTHOPS | abi.SPF_F_ORDER, ignore=ignore).run()
    assert q.kernel == "wide"
    check_query(csr, q, sources, True, ignore)
    check_order(csr, q, sources, ignore=ignore, rows=set(range(12)))


def test_zero_metric_unit_runs(gpu_ready):
    """useLinkMetric = false on a metric-0 area: every hop costs 1, so the
    fast plans run; with a settle order asked for, the wide plan (no
    plateaus: key = id)."""
    rng = random.Random(23)
    V = 140
    csr = abi.Csr.from_links(V, random_links(rng, V, 480, wmin=0, wmax=3))
    g = abi.Graph(csr)
    sources = list(range(0, V, 2))
    qf = g.query(sources, abi.SPF_F_NEXTHOPS | abi.SPF_F_UNIT_METRIC).run()
    assert qf.kernel != "wide" and qf.kernel != "exact"
    check_query(csr, qf, sources, False)
    qo = g.query(sources, abi.SPF_F_NEXTHOPS | abi.SPF_F_UNIT_METRIC | abi.SPF_F_ORDER).run()
    assert qo.kernel == "wide"
    check_query(csr, qo, sources, False)
    check_order(csr, qo, sources, use_metric=False, rows=set(range(0, len(sources), 5)))


def test_sums_beyond_32_bits(gpu_ready):
    """Metrics up to 2^31 - 1: distances pass 2^32 (uint64 sums, no wrap)."""
    rng = random.Random(29)
    V = 260
    big = (1 << 31) - 1
    links = random_links(rng, V, 900, wmin=big // 3, wmax=big)
    ov = [1 if rng.random() < 0.04 else 0 for _ in range(V)]
    csr = abi.Csr.from_links(V, links, ov)
    g = abi.Graph(csr)
    assert g.needs_exact
    sources = list(range(0, V, 3))
    q = g.query(sources, abi.SPF_F_NEXTHOPS).run()
    assert q.kernel == "wide"
    assert max(int(q.dist(i)[q.dist(i) != abi.SPF_UNREACHABLE].max()) for i in range(4)) > (1 << 32)
    check_query(csr, q, sources, True)


def test_hub_source_beyond_16_mask_words(gpu_ready):
    """A source with 1,100 distinct neighbours (18 mask words) in a batch
    whose rows plan does not apply: the wide plan (was the literal replay)."""
    V = 1300
    links = [(0, v, 1, 1) for v in range(1, 1101)]
    links += [(v, 1100 + (v % 199) + 1, 2, 3) for v in range(1, 1101)]
    csr = abi.Csr.from_links(V, links)
    g = abi.Graph(csr)
    q = g.query([0, 7, 1250], abi.SPF_F_NEXTHOPS).run()
    assert q.nh_words(0) == 18
    assert q.kernel == "wide"
    check_query(csr, q, [0, 7, 1250], True)


def test_negative_metric_keeps_literal_replay(gpu_ready):
    m = (1 << 64) - 5
    csr = abi.Csr.from_links(4, [(0, 1, m, 1), (1, 2, 10, 10), (0, 2, 3, 3), (2, 3, 1, 1)])
    g = abi.Graph(csr)
    q = g.query([0, 1, 2, 3], abi.SPF_F_NEXTHOPS).run()
    assert q.kernel == "exact"
    check_query(csr, q, [0, 1, 2, 3], True)


def _grid_links(n, metric=1):
    links = []
    for r in range(n):
        for c in range(n):
            v = r * n + c
            if c + 1 < n:
                links.append((v, v + 1, metric, metric))
            if r + 1 < n:
                links.append((v, v + n, metric, metric))
    return links


def test_grid_one_zero_link(gpu_ready):
    """A 40x40 unit grid with ONE metric-0 link (the case that used
    to send the whole area to one thread per query): all 1,600 sources with
    next hops, sampled rows against the replay."""
    n = 40
    links = _grid_links(n)
    links[len(links) // 2] = (links[len(links) // 2][0], links[len(links) // 2][1], 0, 0)
    csr = abi.Csr.from_links(n * n, links)
    g = abi.Graph(csr)
    assert g.needs_exact
    sources = np.arange(n * n, dtype=np.uint32)
    q = g.query(sources, abi.SPF_F_NEXTHOPS | abi.SPF_F_ORDER).run()
    assert q.kernel == "wide"
    rng = random.Random(3)
    rows = set(rng.sample(range(n * n), 12)) | {links[len(links) // 2][0]}
    check_query(csr, q, [int(s) for s in sources], True, rows=rows)
    check_order(csr, q, [int(s) for s in sources], rows={0, 1, 2})


def _csr_arrays(csr):
    return (
        np.ascontiguousarray(csr.row_ptr, dtype=np.uint32),
        np.ascontiguousarray(csr.col, dtype=np.uint32),
        np.ascontiguousarray(csr.metric, dtype=np.uint64),
        np.ascontiguousarray(csr.link_id, dtype=np.uint32),
        np.ascontiguousarray(csr.overloaded, dtype=np.uint8),
    )


@pytest.mark.parametrize("hop_bound", ["1", "0"])
def test_wan_large_metrics_vs_flat_oracle(gpu_ready, hop_bound, monkeypatch):
    """A 20k-node WAN-like graph with metrics up to 10^6 (maxw * (V-1) >=
    2^32): distance rows and next-hop summaries of sampled sources against
    the flat CPU restatement (uint64 sums) -- on the 32-bit plans the
    transit hop bound admits (maxw * (hop bound + 1) < 2^32), and on the
    wide plan with the bound disabled."""
    from oracle import build

    build.build()
    from oracle import _oracle_ref as O

    monkeypatch.setenv("OPENR_SPF_HOP_BOUND", hop_bound)
    rng = random.Random(41)
    V = 20000
    links = random_links(rng, V, 100000, wmin=1, wmax=1_000_000, parallel=0.01)
    ov = np.zeros(V, dtype=np.uint8)
    ov[rng.sample(range(V), 100)] = 1
    csr = abi.Csr.from_links(V, links, overloaded=ov)
    g = abi.Graph(csr)
    assert g.needs_exact == (hop_bound == "0")
    srcs = np.array(rng.sample(range(V), 24), dtype=np.uint32)
    q = g.query(srcs, abi.SPF_F_NEXTHOPS).run()
    assert (q.kernel == "wide") == (hop_bound == "0")
    row, col, w, link, ovl = _csr_arrays(csr)
    ref = O.csr_spf_rows(row, col, w, link, ovl, srcs, True, 4)
    for i in range(len(srcs)):
        assert (q.dist(i) == ref[i]).all(), i
    summ = O.csr_spf_summary(row, col, w, link, ovl, srcs, use_metric=True, want_nh=True, threads=4)
    for i, s in enumerate(srcs):
        d = q.dist(i)
        sets = q.nexthop_sets(i, int(s))
        reached = d != abi.SPF_UNREACHABLE
        assert int(reached.sum()) == int(summ[i, 0])
        n_pairs = sum(len(sets[v]) for v in np.flatnonzero(reached) if v != s)
        assert n_pairs == int(summ[i, 2]), i
