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


def test_nh_bytes_rule():
    """Device mask bytes per node (SPF_NH_BYTES): 1 / 2 / 4 bytes up to 8 / 16
    / 32 neighbours (a fabric RSW's 8 neighbours: one byte per node), then
    whole u64 words."""
    want = {0: 1, 1: 1, 8: 1, 9: 2, 16: 2, 17: 4, 32: 4, 33: 8, 64: 8, 65: 16, 173: 24}
    assert {n: abi.nh_bytes_for(n) for n in want} == want


@pytest.mark.parametrize("n,world", [(10, 3), (9976, 8), (7, 8), (100000, 8), (1, 1), (0, 4)])
def test_table_layout_blocks_match_shard(n, world):
    rng = np.random.default_rng(n + world)
    V = 37
    nbytes = rng.choice([1, 2, 4, 8, 16, 24], size=n).astype(np.uint32)
    bf, mo, cap = abi.table_layout(n, world, V, nbytes)
    for r in range(world):
        first, count = AS.shard(n, world, r)
        assert (int(bf[r]), int(bf[r + 1] - bf[r])) == (first, count)
    assert int(bf[world]) == n
    assert cap % 32 == 0
    # mask slots: equal-sized, every source inside its owner's slot, back to back
    size = lambda i: ((V * int(nbytes[i]) + 31) // 32) * 32  # noqa: E731
    for r in range(world):
        off = r * cap
        for i in range(int(bf[r]), int(bf[r + 1])):
            assert int(mo[i]) == off
            off += size(i)
        assert off <= (r + 1) * cap


def test_table_layout_gather_simulation():
    """Rank r's packed masks (query order, each roundup32(V*B) bytes) placed
    in slot r of an all-gather land where mask_off says."""
    rng = np.random.default_rng(5)
    n, world, V = 23, 4, 11
    nbytes = rng.choice([1, 2, 4, 8, 16], size=n).astype(np.uint32)
    bf, mo, cap = abi.table_layout(n, world, V, nbytes)
    gathered = np.zeros(world * cap, dtype=np.uint8)
    truth = {}
    for r in range(world):
        packed = []
        for i in range(int(bf[r]), int(bf[r + 1])):
            m = rng.integers(0, 256, size=V * int(nbytes[i]), dtype=np.uint8)
            truth[i] = m
            pad = (-len(m)) % 32
            packed.append(np.concatenate([m, np.zeros(pad, dtype=np.uint8)]))
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
        assert [t.nh_bytes(i) for i in range(n)] == [q.nh_bytes(i) for i in range(n)]
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


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["local", "rank"])
def test_query_table_ignore_lists_persistent_graph(gpu_ready, mode):
    """spf_table_create_q over a persistent spf_cgraph: per-query ignore
    lists (KSP2 second passes / what-if / LFA batches, LinkState.cpp:776-777,
    842-847) sliced per block give the single-device query's rows and masks
    exactly; the same cgraph serves later tables after in-place transit and
    metric patches (no re-upload)."""
    csr = _random_csr(2500, 9000, 21)
    rng = np.random.default_rng(5)
    n = 300
    sources = rng.integers(0, csr.num_nodes, n).astype(np.uint32)
    ignore = [sorted(set(int(x) for x in rng.integers(0, csr.num_links, int(rng.integers(0, 40)))))
              for _ in range(n)]
    c = abi.Cluster([0]) if mode == "local" else abi.Cluster(
        world=1, rank=0, uid=abi.cluster_unique_id(), device=0)
    cg = abi.ClusterGraph(c, csr)
    g = abi.Graph(csr)
    for step in range(3):
        for flags in (abi.SPF_F_NEXTHOPS, abi.SPF_F_NEXTHOPS | abi.SPF_F_UNIT_METRIC, 0):
            t = cg.table(sources, flags, ignore=ignore).run()
            q = g.query(sources, flags, ignore=ignore).run()
            rows = np.empty((n, csr.num_nodes), dtype=np.uint32)
            q.fetch_rows(0, n, rows.ctypes.data, csr.num_nodes * 4, on_device=False)
            assert (t.fetch_rows(0, n) == rows).all(), (step, flags)
            if flags & abi.SPF_F_NEXTHOPS:
                assert (t.fetch_nexthops(0, n) == q.fetch_nexthops(0, n)).all(), (step, flags)
            q.close()
            t.close()
        # churn on both graphs: drain toggles and metric changes in place
        ov = (rng.random(csr.num_nodes) < 0.05).astype(np.uint8)
        cg.set_transit(ov)
        g.set_transit(ov)
        e = rng.choice(len(csr.col), 50, replace=False).astype(np.uint32)
        m = rng.integers(1, 20, 50).astype(np.uint64)
        cg.patch_metrics(e, m)
        g.patch_metrics(e, m)
    g.close()
    cg.close()
    c.close()


@pytest.mark.gpu
def test_linkstate_batches_fan_out_with_ignore_lists(gpu_ready):
    """The drop-in with setSpfDevices: what-if batches (runSpfBatch), KSP2
    second passes (prefetchKthPaths) and LFA neighbour batches (prefetchSpf)
    all run through the persistent cluster graph -- one upload, patched by
    drain churn -- and every SpfResult / RouteDb equals the oracle's."""
    import copy

    import openr_amd._openr_spf as E
    from oracle import build
    from openr_amd import thrift as T
    from tests import randomized as RZ

    build.build()
    from oracle import _oracle_ref as O

    names, adj_dbs, prefix_dbs = RZ.random_network(91, n_nodes=60, n_links=150)
    for pdb in prefix_dbs:  # SR-MPLS KSP2 for half the prefixes
        for i, e in enumerate(pdb.prefixEntries):
            if i % 2 == 0:
                e.forwardingType = T.PrefixForwardingType.SR_MPLS
                e.forwardingAlgorithm = T.PrefixForwardingAlgorithm.KSP2_ED_ECMP
    ea, ep = RZ.load(E, adj_dbs, prefix_dbs, 1)
    oa, op = RZ.load(O, adj_dbs, prefix_dbs, 1)
    E.set_spf_devices([0])
    E.set_cluster_min_sources(4)
    try:
        E.reset_counters()
        me = names[0]
        links = list(ea["0"].linksFromNode(me))
        by_key = {tuple(l.key()): l for l in oa["0"].linksFromNode(me)}
        olinks = [by_key[tuple(l.key())] for l in links]
        batch = ea["0"].runSpfBatch(me, [[l] for l in links], True)
        for i, ol in enumerate(olinks):
            want = oa["0"].runSpfIgnoring(me, [ol], True)
            got = batch.result(i)
            assert got.keys() == want.keys()
            for k in got:
                assert got[k][0] == want[k][0] and got[k][1] == want[k][1], (i, k)
        for lfa in (False, True):
            es = E.SpfSolver(me, True, lfa)
            os_ = O.SpfSolver(me, True, lfa)
            assert es.buildRouteDb(me, ea, ep) == os_.buildRouteDb(me, oa, op), lfa
        c = E.get_counters()
        assert c.get("decision.spf_cluster_batches", 0) >= 3
        assert c.get("decision.cluster_graph_uploads", 0) == 1
        # drain churn patches the cluster graph in place
        dbs = [copy.deepcopy(d) for d in adj_dbs["0"]]
        for step in range(3):
            db = dbs[(step * 17) % len(dbs)]
            db.isOverloaded = not db.isOverloaded
            ea["0"].updateAdjacencyDatabase(db)
            oa["0"].updateAdjacencyDatabase(db)
            es = E.SpfSolver(me, True, True)
            os_ = O.SpfSolver(me, True, True)
            assert es.buildRouteDb(me, ea, ep) == os_.buildRouteDb(me, oa, op), step
        assert E.get_counters().get("decision.cluster_graph_uploads", 0) == 1
    finally:
        E.set_cluster_min_sources(64)
        E.set_spf_devices([])


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["local", "rank"])
def test_query_table_trace_paths(gpu_ready, mode):
    """spf_table_trace_paths / spf_table_trace_fetch: the KSP2 second-pass
    traces of a query table (one source, per-destination ignore lists = the
    first paths' links) equal the single-device query's traces in table
    order, overflowed entries included."""
    csr = _random_csr(1500, 6000, 31, wmax=4)
    g = abi.Graph(csr)
    src = 7
    dsts = np.arange(0, csr.num_nodes, 3, dtype=np.uint32)
    dsts = dsts[dsts != src]
    first = g.query(np.full(len(dsts), src, dtype=np.uint32), 0).run().trace_paths(dsts)
    keep = [i for i, p in enumerate(first) if p]
    ign = [sorted({l for p in first[i] for l in p}) for i in keep]
    srcs = np.full(len(keep), src, dtype=np.uint32)
    d2 = dsts[keep]
    want = g.query(srcs, 0, ignore=ign).run().trace_paths(d2)
    c = abi.Cluster([0]) if mode == "local" else abi.Cluster(
        world=1, rank=0, uid=abi.cluster_unique_id(), device=0)
    cg = abi.ClusterGraph(c, csr)
    t = cg.table(srcs, 0, ignore=ign).run()
    assert t.trace_paths(d2) == want
    t.close()
    cg.close()
    c.close()
    g.close()
