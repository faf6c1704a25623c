"""Sharded all-sources tables (openr_amd/allsources.py).

CPU ("not gpu"): the source partition / slot arithmetic, and the exchange
step — per-rank row blocks all-gathered in place into the global table —
over torch.distributed gloo at world sizes 2 and 3 (uneven blocks).  The
rows each rank contributes in these tests come from scipy's Dijkstra on a
small weighted graph (a stand-in producer for the gather logic only); the
gathered table must equal the all-pairs matrix row for row.
GPU: the same class with the HIP engine as the producer, at world size 1,
against direct engine queries and the literal DijkstraQ replay.
"""

import os
import random
import socket

import numpy as np
import pytest

from openr_amd import allsources as AS


def test_shard_partition():
    for n in (0, 1, 5, 7, 64, 100, 100000):
        for world in (1, 2, 3, 8):
            blocks = [AS.shard(n, world, r) for r in range(world)]
            assert blocks[0][0] == 0
            for (f0, c0), (f1, _) in zip(blocks, blocks[1:]):
                assert f0 + c0 == f1  # contiguous
            assert sum(c for _, c in blocks) == n
            sizes = [c for _, c in blocks]
            assert max(sizes) - min(sizes) <= 1
            cap = AS.shard_cap(n, world)
            assert max(sizes) == cap or n == 0
            idx = AS.slot_index(n, world)
            assert len(set(idx.tolist())) == n
            for i in range(0, n, max(1, n // 50)):
                assert AS.slot_row(i, n, world) == idx[i]
                r = idx[i] // cap
                f, c = blocks[r]
                assert f <= i < f + c and idx[i] % cap == i - f
    with pytest.raises(ValueError):
        AS.shard(10, 2, 2)
    with pytest.raises(IndexError):
        AS.slot_row(10, 10, 2)


def _graph(V=60, L=180, seed=5):
    rng = random.Random(seed)
    links = [(rng.randrange(v), v, rng.randint(1, 20), rng.randint(1, 20)) for v in range(1, V)]
    while len(links) < L:
        u, v = rng.randrange(V), rng.randrange(V)
        if u != v:
            links.append((u, v, rng.randint(1, 20), rng.randint(1, 20)))
    return V, links


def _dist_matrix(V, links):
    import scipy.sparse as sp
    import scipy.sparse.csgraph as cg

    # directed metrics: u->v advertised by u (parallel links: cheapest)
    W = np.full((V, V), np.inf)
    for (u, v, a, b) in links:
        W[u, v] = min(W[u, v], a)
        W[v, u] = min(W[v, u], b)
    W[~np.isfinite(W)] = 0
    D = cg.dijkstra(sp.csr_matrix(W), directed=True)
    D[~np.isfinite(D)] = AS.UNREACHABLE_U32
    return D.astype(np.int64).astype(np.uint32).view(np.int32)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _gather_worker(rank, world, port, out_q):
    import torch
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        V, links = _graph()
        D = _dist_matrix(V, links)
        n = V
        first, count = AS.shard(n, world, rank)
        cap = AS.shard_cap(n, world)
        table = torch.full((world * cap, V), -1, dtype=torch.int32)
        mine = table[rank * cap : (rank + 1) * cap]
        mine[:count] = torch.from_numpy(D[first : first + count])
        AS.gather_rows(mine, n, out=table)  # in place
        full = table.numpy()[AS.slot_index(n, world)]
        out_q.put((rank, bool((full == D).all())))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gather_rows_gloo(world):
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gather_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    res = dict(q.get(timeout=10) for _ in range(world))
    assert all(res.values()), res


@pytest.mark.gpu
def test_sharded_all_sources_engine(gpu_ready):
    """World size 1 (no process group): the table rows equal direct engine
    queries and the literal replay, on a graph big enough for the
    delta-stepping plan."""
    import torch

    from openr_amd import abi
    from oracle import spf_py

    rng = random.Random(77)
    V = 70000
    links = []
    for v in range(1, V):
        links.append((rng.randrange(v), v, rng.randint(1, 100), rng.randint(1, 100)))
    while len(links) < 180000:
        u, v = rng.randrange(V), rng.randrange(V)
        if u != v:
            links.append((u, v, rng.randint(1, 100), rng.randint(1, 100)))
    csr = abi.Csr.from_links(V, links)
    srcs = np.asarray(rng.sample(range(V), 300), dtype=np.uint32)
    torch.cuda.set_device(0)
    sas = AS.ShardedAllSources(csr, sources=srcs, gather=False)
    assert sas.kernel == "dstep-ldsrow"  # distances fit the 12-bit LDS rows
    run = sas.run()
    assert run.count == 300 and run.spf_ms > 0
    g = abi.Graph(csr)
    q = g.query(srcs[:8], 0).run()
    for i in range(8):
        assert (sas.row(i).astype(np.uint64) == np.where(
            q.dist(i) == np.uint64(abi.SPF_UNREACHABLE), np.uint64(0xFFFFFFFF), q.dist(i))).all()
    for i in (0, 299):
        ref = spf_py.run_spf(csr, int(srcs[i]), True)
        row = sas.row(i)
        for v in range(V):
            assert int(row[v]) == (ref[v][0] if v in ref else 0xFFFFFFFF)
    sas.close()


def test_needs_64bit_rows_matches_engine_rule():
    """ShardedAllSources.update refuses a topology that needs 64-bit rows
    BEFORE touching its table / graph / query: the host rule
    mirrors the engine's upload_weights (metric 0, a wrapping metric, or
    maxw * (V - 1) >= 2^32)."""
    from openr_amd import abi
    from openr_amd.allsources import needs_64bit_rows

    def csr(links, V=4):
        return abi.Csr.from_links(V, links)

    assert not needs_64bit_rows(csr([(0, 1, 1, 1), (1, 2, 5, 7), (2, 3, 9, 9)]))
    assert needs_64bit_rows(csr([(0, 1, 0, 1), (1, 2, 5, 7)]))
    assert needs_64bit_rows(csr([(0, 1, (1 << 64) - 5, 1)]))
    big = (1 << 32) // 3 + 1  # maxw * (V - 1) >= 2^32 at V = 4
    assert needs_64bit_rows(csr([(0, 1, big, 1)]))
    assert not needs_64bit_rows(csr([(0, 1, big - 2, 1)]))


def test_transit_hop_bound_rule():
    """The 32-bit row bound's hop count (spf_device.hip transit_hop_bound):
    2 * eccentricity of the first highest-degree transit node, 0 when a drain
    cuts a node off from it."""
    import numpy as np

    from openr_amd import abi
    from openr_amd.allsources import needs_64bit_rows, transit_hop_bound

    star = [(0, v, 1, 1) for v in range(1, 9)] + [(8, 9, 1, 1)]
    csr = abi.Csr.from_links(10, star)
    assert transit_hop_bound(csr) == 4
    ov = np.zeros(10, dtype=np.uint8)
    ov[8] = 1
    assert transit_hop_bound(abi.Csr.from_links(10, star, overloaded=ov)) == 0
    w = (1 << 32) // 7  # 5w fits, 9w (the coarse V - 1 bound) does not
    big = [(a, b, w, w) for (a, b, _, _) in star]
    assert not needs_64bit_rows(abi.Csr.from_links(10, big))
    assert needs_64bit_rows(abi.Csr.from_links(10, big, overloaded=ov))
