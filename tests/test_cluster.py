"""Multi-GPU all-sources tables inside the C ABI (include/openr_spf.h
spf_cluster_* / spf_table_*; SURVEY.md §8(b) "the multi-GPU fan-out happens
inside the call", §8(e) source blocks + RCCL all-gather).

CPU: the host-side layout (spf_table_layout) of the source blocks and of the
gathered next-hop masks, checked against a restatement and an all-gather
simulation.  GPU: a table over one device (local and rank-mode clusters)
equals a plain query bit for bit, rows and masks; the LinkState fan-out
(set_spf_devices) gives the same SpfResults as the single-device path.  The
1/2/4/8-GPU exchange itself runs only on an 8-GPU node (bench.py at N > 1);
this pool's boxes have one GPU.
"""

import numpy as np
import pytest

from openr_amd import abi
from openr_amd import allsources as AS


@pytest.mark.parametrize("n,world", [(10, 3), (9976, 8), (7, 8), (100000, 8), (1, 1), (0, 4)])
def test_table_layout_blocks_match_shard(n, world):
    rng = np.random.default_rng(n + world)
    V = 37
    words = rng.integers(1, 4, size=n).astype(np.uint32)
    bf, mo, cap = abi.table_layout(n, world, V, words)
    for r in range(world):
        first, count = AS.shard(n, world, r)
        assert (int(bf[r]), int(bf[r + 1] - bf[r])) == (first, count)
    assert int(bf[world]) == n
    # mask slots: equal-sized, every source inside its owner's slot, back to back
    size = lambda i: ((V * int(words[i]) + 3) // 4) * 4  # noqa: E731
    for r in range(world):
        off = r * cap
        for i in range(int(bf[r]), int(bf[r + 1])):
            assert int(mo[i]) == off
            off += size(i)
        assert off <= (r + 1) * cap


def test_table_layout_gather_simulation():
    """Rank r's packed masks (query order, each roundup4(V*W) words) placed in
    slot r of an all-gather land where mask_off says."""
    rng = np.random.default_rng(5)
    n, world, V = 23, 4, 11
    words = rng.integers(1, 3, size=n).astype(np.uint32)
    bf, mo, cap = abi.table_layout(n, world, V, words)
    gathered = np.zeros(world * cap, dtype=np.uint64)
    truth = {}
    for r in range(world):
        packed = []
        for i in range(int(bf[r]), int(bf[r + 1])):
            m = rng.integers(0, 2**63, size=V * int(words[i]), dtype=np.uint64)
            truth[i] = m
            pad = (-len(m)) % 4
            packed.append(np.concatenate([m, np.zeros(pad, dtype=np.uint64)]))
        if packed:
            blk = np.concatenate(packed)
            gathered[r * cap : r * cap + len(blk)] = blk  # ncclAllGather slot r
    for i, m in truth.items():
        assert (gathered[int(mo[i]) : int(mo[i]) + len(m)] == m).all()


def _random_csr(V, L, seed, wmax=20):
    rng = np.random.default_rng(seed)
    links = []
    for v in range(1, V):
        u = int(rng.integers(0, v))
        links.append((u, v, int(rng.integers(1, wmax)), int(rng.integers(1, wmax))))
    while len(links) < L:
        a, b = (int(x) for x in rng.integers(0, V, size=2))
        if a != b:
            links.append((a, b, int(rng.integers(1, wmax)), int(rng.integers(1, wmax))))
    ov = (rng.random(V) < 0.05).astype(np.uint8)
    return abi.Csr.from_links(V, links, ov)


def _check_table_equals_query(t, g, csr, sources, flags):
    q = g.query(sources, flags).run()
    n = len(sources)
    rows = np.empty((n, csr.num_nodes), dtype=np.uint32)
    q.fetch_rows(0, n, rows.ctypes.data, csr.num_nodes * 4, on_device=False)
    assert (t.fetch_rows(0, n) == rows).all()
    if flags & abi.SPF_F_NEXTHOPS:
        assert [t.nh_words(i) for i in range(n)] == [q.nh_words(i) for i in range(n)]
        assert (t.fetch_nexthops(0, n) == q.fetch_nexthops(0, n)).all()
    q.close()


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["local", "rank"])
@pytest.mark.parametrize("unit", [False, True])
def test_table_one_device_equals_query(gpu_ready, mode, unit):
    csr = _random_csr(3000, 12000, 11 + unit)
    sources = np.arange(0, 3000, 7, dtype=np.uint32)
    flags = abi.SPF_F_NEXTHOPS | (abi.SPF_F_UNIT_METRIC if unit else 0)
    if mode == "local":
        c = abi.Cluster([0])
    else:
        c = abi.Cluster(world=1, rank=0, uid=abi.cluster_unique_id(), device=0)
    assert (c.world, c.first_rank, c.local_devices) == (1, 0, 1)
    t = abi.Table(c, csr, sources, flags | abi.SPF_T_GATHER_ROWS | abi.SPF_T_GATHER_NEXTHOPS)
    t.run()
    compute, gather = t.elapsed_ms()
    assert compute > 0 and gather >= 0
    assert t.block(0) == (0, len(sources))
    g = abi.Graph(csr)
    _check_table_equals_query(t, g, csr, sources, flags)
    # the gathered device buffers hold the same rows (slot 0 of 1)
    rows_ptr, masks_ptr, cap = t.device_buffers(0)
    assert rows_ptr and masks_ptr and cap > 0
    t.close()
    # no gather flags: rows stay with the owner
    t2 = abi.Table(c, csr, sources, flags).run()
    assert t2.device_buffers(0)[:2] == (None, None)
    _check_table_equals_query(t2, g, csr, sources, flags)
    t2.close()
    g.close()
    c.close()


@pytest.mark.gpu
def test_linkstate_prefetch_fans_out(gpu_ready):
    """LinkState::prefetchSpf over the multi-GPU path (set_spf_devices, here
    one device) equals the CPU oracle's SpfResults."""
    import openr_amd._openr_spf as E
    from oracle import build
    from tests import randomized as RZ

    build.build()
    from oracle import _oracle_ref as O

    names, adj_dbs, prefix_dbs = RZ.random_network(77, n_nodes=120, n_links=300)
    ea, _ = RZ.load(E, adj_dbs, prefix_dbs, 1)
    oa, _ = RZ.load(O, adj_dbs, prefix_dbs, 1)
    E.set_spf_devices([0])
    try:
        E.reset_counters()
        ea["0"].prefetchSpf(names, True)
        assert E.get_counters().get("decision.spf_cluster_batches", 0) == 1
        for node in names[::7]:
            a = ea["0"].getSpfResult(node, True)
            b = oa["0"].getSpfResult(node, True)
            assert a.keys() == b.keys()
            for k in a:
                assert a[k][0] == b[k][0] and a[k][1] == b[k][1], (node, k)
                assert list(a[k][2]) == list(b[k][2]), (node, k)
    finally:
        E.set_spf_devices([])
