"""Incremental all-sources tables.

The reference drops its whole SPF memo on any topology change
(openr/decision/LinkState.cpp:712-715, driven by updateAdjacencyDatabase
:564-717).  The engine repairs a resident table instead: spf_graph_diff lists
the change as directed edge deltas, spf_table_screen marks the sources whose
shortest-path DAG a delta can touch, and only those are recomputed.

CPU ("not gpu"):
  * spf_graph_diff (host-only C) against a Python restatement;
  * the screen RULE (restated in numpy below, test-only) is exact: on random
    graphs and random churn (link down / up, metric up / down, node
    overload / un-overload, several at once) every source it does NOT flag
    has the same distances AND next-hop sets before and after, by the
    literal DijkstraQ replay (oracle/spf_py.py);
  * exchange_rows (repaired rows to the other ranks) over gloo, world 2 / 3.
  * the in-place repair RULE of spf_table_repair (reset the nodes that lost
    every supporting tight path, relax from the reset boundary and the
    improved edges; restated in Python below) gives the new distances of
    every source exactly.
GPU: ShardedAllSources.update() — diff + screen kernel + in-place repair
kernel (or, forced, recompute of the affected sources + scatter kernel) —
equals a full recompute bit for bit, on the frontier (LDS), delta-stepping
(beyond LDS) and MS-BFS (uniform metric) plans.
"""

import os
import random
import socket

import numpy as np
import pytest

from openr_amd import abi
from openr_amd import allsources as AS

INF = 0xFFFFFFFF


def _random_links(V, L, rng, wmax=20):
    links = [(rng.randrange(v), v, rng.randint(1, wmax), rng.randint(1, wmax)) for v in range(1, V)]
    seen = {(min(u, v), max(u, v)) for (u, v, _, _) in links}
    while len(links) < L:
        u, v = rng.randrange(V), rng.randrange(V)
        if u != v and (min(u, v), max(u, v)) not in seen:
            seen.add((min(u, v), max(u, v)))
            links.append((u, v, rng.randint(1, wmax), rng.randint(1, wmax)))
    return links


def _churn(V, links, ov, rng, kinds, wmax=20):
    """One topology change: returns (links', ov')."""
    links = list(links)
    ov = np.array(ov, dtype=np.uint8)
    for kind in kinds:
        if kind == "down" and links:
            links.pop(rng.randrange(len(links)))
        elif kind == "up":
            u, v = rng.randrange(V), rng.randrange(V)
            if u != v:
                links.append((u, v, rng.randint(1, wmax), rng.randint(1, wmax)))
        elif kind in ("metric_up", "metric_down") and links:
            i = rng.randrange(len(links))
            u, v, a, b = links[i]
            if kind == "metric_up":
                a = a + rng.randint(1, wmax)
            else:
                a = max(1, a - rng.randint(1, wmax))
            links[i] = (u, v, a, b)
        elif kind == "drain":
            ov[rng.randrange(V)] ^= 1
    return links, ov


def _diff_py(a, b):
    """Python restatement of spf_graph_diff (include/openr_spf.h)."""
    out = []
    for u in range(a.num_nodes):
        ea = sorted((int(a.col[e]), int(a.metric[e])) for e in range(a.row_ptr[u], a.row_ptr[u + 1]))
        eb = sorted((int(b.col[e]), int(b.metric[e])) for e in range(b.row_ptr[u], b.row_ptr[u + 1]))
        trA, trB = not a.overloaded[u], not b.overloaded[u]
        ca = {}
        for x in ea:
            ca[x] = ca.get(x, 0) + 1
        cb = {}
        for x in eb:
            cb[x] = cb.get(x, 0) + 1
        for x in sorted(set(ca) | set(cb)):
            na, nb = ca.get(x, 0), cb.get(x, 0)
            common = min(na, nb)
            out += [(u, x[0], x[1], abi.SPF_DELTA_REMOVED, 0 if trA else 1)] * (na - common)
            out += [(u, x[0], x[1], abi.SPF_DELTA_ADDED, 0 if trB else 1)] * (nb - common)
            if trA and not trB:
                out += [(u, x[0], x[1], abi.SPF_DELTA_REMOVED, 2)] * common
            elif trB and not trA:
                out += [(u, x[0], x[1], abi.SPF_DELTA_ADDED, 2)] * common
    return sorted(out)


def _screen_np(D, sources, deltas):
    """Test-only restatement of spf_table_screen_kernel's rule."""
    out = np.zeros(len(sources), dtype=np.uint8)
    for i, s in enumerate(sources):
        for d in deltas:
            u, v, w, kind, scope = int(d["tail"]), int(d["head"]), int(d["metric"]), int(d["kind"]), int(d["scope"])
            if (scope == abi.SPF_SCOPE_TAIL_ONLY and s != u) or (scope == abi.SPF_SCOPE_NOT_TAIL and s == u):
                continue
            du = int(D[i][u])
            if du == INF:
                continue
            dv = int(D[i][v])
            dv = float("inf") if dv == INF else dv
            if (kind == abi.SPF_DELTA_REMOVED and du + w == dv) or (kind == abi.SPF_DELTA_ADDED and du + w <= dv):
                out[i] = 1
                break
    return out


def _rows(csr, srcs):
    from oracle import spf_py

    D = np.full((len(srcs), csr.num_nodes), INF, dtype=np.uint64)
    NH = []
    for i, s in enumerate(srcs):
        r = spf_py.run_spf(csr, int(s), True)
        for v, (m, nh, _, _) in r.items():
            D[i, v] = m
        NH.append({v: nh for v, (m, nh, _, _) in r.items()})
    return D, NH


def test_graph_diff_matches_restatement():
    rng = random.Random(3)
    for trial in range(12):
        V = rng.randint(2, 40)
        links = _random_links(V, min(V * (V - 1) // 2, rng.randint(V - 1, 3 * V)), rng)
        ov = np.array([rng.random() < 0.2 for _ in range(V)], dtype=np.uint8)
        kinds = rng.choices(["down", "up", "metric_up", "metric_down", "drain"], k=rng.randint(0, 5))
        links2, ov2 = _churn(V, links, ov, rng, kinds)
        a = abi.Csr.from_links(V, links, ov)
        b = abi.Csr.from_links(V, links2, ov2)
        got = sorted(tuple(int(x) for x in d) for d in abi.graph_diff(a, b))
        assert got == _diff_py(a, b), (trial, kinds)
    # identical graphs: no deltas; different node counts: refused
    assert len(abi.graph_diff(a, a)) == 0
    with pytest.raises(abi.SpfError):
        abi.graph_diff(a, abi.Csr.from_links(V + 1, links, np.append(ov, 0)))


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_screen_rule_is_exact(seed):
    """Unflagged sources keep distances AND next-hop sets (replay oracle)."""
    rng = random.Random(seed)
    kept = total = 0
    for trial in range(6):
        V = 45
        links = _random_links(V, 110, rng, wmax=6)  # small metrics: many ties
        ov = np.array([rng.random() < 0.1 for _ in range(V)], dtype=np.uint8)
        kinds = [rng.choice(["down", "up", "metric_up", "metric_down", "drain"])
                 for _ in range(rng.choice([1, 1, 2, 4]))]
        links2, ov2 = _churn(V, links, ov, rng, kinds, wmax=6)
        a = abi.Csr.from_links(V, links, ov)
        b = abi.Csr.from_links(V, links2, ov2)
        srcs = list(range(V))
        D0, NH0 = _rows(a, srcs)
        D1, NH1 = _rows(b, srcs)
        flags = _screen_np(D0, srcs, abi.graph_diff(a, b))
        for i in range(V):
            if not flags[i]:
                assert (D0[i] == D1[i]).all(), (trial, kinds, i)
                assert NH0[i] == NH1[i], (trial, kinds, i)
                kept += 1
            total += 1
    assert kept > total // 10  # the screen does skip work


def _repair_py(row, csr, src, deltas):
    """Test-only restatement of spf_table_repair's rule for one row (the
    seeded spf_dstep_kernel with its repair_invalidate prologue): returns
    the repaired row (uint64, INF = unreached)."""
    import heapq

    d = [int(x) for x in row]
    V = csr.num_nodes
    rp, col, met, rev = csr.row_ptr, csr.col, csr.metric, csr.rev
    ov = csr.overloaded

    def usable(u):
        return u == src or not ov[u]

    K = set()
    for x in deltas:
        u, v, w, kind, sc = (int(x[k]) for k in ("tail", "head", "metric", "kind", "scope"))
        if kind != abi.SPF_DELTA_REMOVED:
            continue
        if (sc == abi.SPF_SCOPE_TAIL_ONLY and src != u) or (sc == abi.SPF_SCOPE_NOT_TAIL and src == u):
            continue
        if d[u] != INF and d[v] != INF and d[u] + w == d[v]:
            K.add(v)
    stack = list(K)
    while stack:
        x = stack.pop()
        if not usable(x):
            continue
        for e in range(rp[x], rp[x + 1]):
            z = int(col[e])
            if d[z] != INF and d[x] + int(met[e]) == d[z] and z not in K:
                K.add(z)
                stack.append(z)
    ok = set()
    for x in K:
        for e in range(rp[x], rp[x + 1]):
            y = int(col[e])
            if y not in K and usable(y) and d[y] != INF and d[y] + int(met[rev[e]]) == d[x]:
                ok.add(x)
    stack = list(ok)
    while stack:
        x = stack.pop()
        if not usable(x):
            continue
        for e in range(rp[x], rp[x + 1]):
            z = int(col[e])
            if z in K and z not in ok and d[x] + int(met[e]) == d[z]:
                ok.add(z)
                stack.append(z)
    reset = K - ok
    for x in reset:
        d[x] = INF
    seeds = {int(x["tail"]) for x in deltas if int(x["kind"]) == abi.SPF_DELTA_ADDED}
    for x in reset:
        for e in range(rp[x], rp[x + 1]):
            y = int(col[e])
            if y not in reset:
                seeds.add(y)
    pq = [(d[u], u) for u in seeds if d[u] != INF]
    heapq.heapify(pq)
    while pq:  # label-correcting relaxation from the seeds
        du, u = heapq.heappop(pq)
        if du != d[u] or not usable(u):
            continue
        for e in range(rp[u], rp[u + 1]):
            v = int(col[e])
            c = du + int(met[e])
            if c < d[v]:
                d[v] = c
                heapq.heappush(pq, (c, v))
    return d


@pytest.mark.parametrize("seed", [4, 5])
def test_repair_rule_is_exact(seed):
    """The in-place repair rule reproduces the new distances exactly, for
    every source, under every kind of churn (replay oracle)."""
    rng = random.Random(seed)
    for trial in range(10):
        V = 40
        links = _random_links(V, 90, rng, wmax=5)
        ov = np.array([rng.random() < 0.1 for _ in range(V)], dtype=np.uint8)
        kinds = [rng.choice(["down", "up", "metric_up", "metric_down", "drain"])
                 for _ in range(rng.choice([1, 1, 2, 5]))]
        links2, ov2 = _churn(V, links, ov, rng, kinds, wmax=5)
        a = abi.Csr.from_links(V, links, ov)
        b = abi.Csr.from_links(V, links2, ov2)
        deltas = abi.graph_diff(a, b)
        D0, _ = _rows(a, range(V))
        D1, _ = _rows(b, range(V))
        for s in range(V):
            assert _repair_py(D0[s], b, s, deltas) == [int(x) for x in D1[s]], (trial, kinds, s)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _exchange_worker(rank, world, port, out_q):
    import torch
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        n, V = 23, 17
        cap = AS.shard_cap(n, world)
        g = torch.Generator().manual_seed(5)
        before = torch.randint(0, 1000, (world * cap, V), generator=g, dtype=torch.int32)
        after = before.clone()
        expect = before.clone()
        # rank r rewrites r + 1 rows of its own slot (rank 0 also none-case below)
        for r in range(world):
            first, count = AS.shard(n, world, r)
            k = min(count, r + 1)
            rows = torch.arange(k, dtype=torch.int64) * 2 % max(count, 1) + r * cap
            rows = torch.unique(rows)
            new = torch.full((len(rows), V), 7000 + r, dtype=torch.int32)
            expect[rows] = new
            if r == rank:
                after[rows] = new
                mine = rows
        got = AS.exchange_rows(after, mine, n)
        ok = bool((after == expect).all())
        # nothing repaired anywhere: no traffic, table unchanged
        none = AS.exchange_rows(after, torch.zeros(0, dtype=torch.int64), n)
        out_q.put((rank, ok and got > 0 and none == 0 and bool((after == expect).all())))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_exchange_rows_gloo(world):
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_exchange_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    res = dict(q.get(timeout=10) for _ in range(world))
    assert all(res.values()), res


def _oracle_rows(csr, srcs):
    """uint32 distance rows of the CPU oracle's flat restatement
    (oracle/csr_spf.h; 0xFFFFFFFF = unreached, like the device table)."""
    from oracle import build

    build.build()
    from oracle import _oracle_ref as O

    rows = O.csr_spf_rows(csr.row_ptr, csr.col, csr.metric.astype(np.uint64), csr.link_id,
                          csr.overloaded, np.asarray(srcs, dtype=np.uint32), True, 8)
    return np.where(rows == np.uint64(2**64 - 1), np.uint64(0xFFFFFFFF), rows).astype(np.uint32)


def _full_table(csr, srcs):
    import torch

    g = abi.Graph(csr)
    q = g.query(srcs, 0).run()
    t = torch.full((len(srcs), csr.num_nodes), -1, dtype=torch.int32, device="cuda:0")
    torch.cuda.synchronize()  # the fill runs on torch's stream, the copy on the graph's
    q.fetch_rows(0, len(srcs), t.data_ptr(), csr.num_nodes * 4, on_device=True)
    q.sync()
    out = t.cpu().numpy().view(np.uint32).copy()
    q.close()
    g.close()
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["repair", "recompute"])
@pytest.mark.parametrize(
    "V,L,wmax,nsrc,expect_kernel",
    [(3000, 12000, 50, 3000, None), (40000, 160000, 1000, 400, "dstep-ldsrow"), (2500, 9000, 1, 2500, None)],
)
def test_repair_equals_full_recompute(gpu_ready, V, L, wmax, nsrc, expect_kernel, mode, monkeypatch):
    import torch

    if mode == "recompute":
        monkeypatch.setenv("OPENR_SPF_REPAIR_RECOMPUTE", "1")

    rng = random.Random(V + L)
    links = _random_links(V, L, rng, wmax=wmax)
    ov = np.zeros(V, dtype=np.uint8)
    csr = abi.Csr.from_links(V, links, ov)
    srcs = np.asarray(sorted(rng.sample(range(V), nsrc)), dtype=np.uint32)
    torch.cuda.set_device(0)
    sas = AS.ShardedAllSources(csr, sources=srcs)
    if expect_kernel:
        assert sas.kernel == expect_kernel
    sas.run()
    plan = [["down"], ["up"], ["metric_up"], ["metric_down"], ["drain"], ["drain"],
            ["down", "down", "up", "metric_down", "drain"], []]
    affected, relaxed = [], []
    for kinds in plan:
        links, ov = _churn(V, links, ov, rng, kinds, wmax=wmax)
        csr = abi.Csr.from_links(V, links, ov)
        rep = sas.update(csr)
        affected.append(rep.affected)
        relaxed.append(rep.relaxed)
        got = sas.table.cpu().numpy().view(np.uint32)[: len(srcs)]
        assert (got == _full_table(csr, srcs)).all(), kinds
        # and against the CPU oracle (oracle/csr_spf.h) on sampled rows
        pick = np.asarray(sorted(rng.sample(range(len(srcs)), min(48, len(srcs)))))
        ref = _oracle_rows(csr, srcs[pick])
        assert (got[pick] == ref).all(), kinds
    assert affected[-1] == 0  # no change: nothing recomputed
    assert min(affected[:-1]) < len(srcs)  # the screen skips sources
    # rows repaired in place (spf_table_repair) unless recompute is forced
    assert all(r == (mode == "repair") for r, n in zip(relaxed, affected) if n)
    # a full run after repairs still works (the batch query is rebuilt)
    sas.run()
    assert (sas.table.cpu().numpy().view(np.uint32)[: len(srcs)] == _full_table(csr, srcs)).all()
    sas.close()


@pytest.mark.gpu
@pytest.mark.parametrize("V,L,wmax", [(1500, 5000, 40), (2500, 9000, 1)])
def test_repaired_table_next_hops(gpu_ready, V, L, wmax):
    """SURVEY §8(f) row 2 with next hops: ShardedAllSources(nexthops=True)
    keeps a next-hop mask table beside the distance rows; after each churn
    event the repaired sources' masks are rebuilt from the table rows
    (spf_table_nexthops, the all-sources rows rule) and EVERY source's masks
    equal a fresh engine query's on the new graph, sampled sources the
    literal DijkstraQ replay's next-hop sets."""
    import torch

    from oracle import spf_py

    rng = random.Random(V * 7 + L)
    links = _random_links(V, L, rng, wmax=wmax)
    ov = np.zeros(V, dtype=np.uint8)
    csr = abi.Csr.from_links(V, links, ov)
    torch.cuda.set_device(0)
    sas = AS.ShardedAllSources(csr, nexthops=True)
    sas.run()
    srcs = np.arange(V, dtype=np.uint32)

    def check(csr, tag):
        g = abi.Graph(csr)
        q = g.query(srcs, abi.SPF_F_NEXTHOPS).run()
        for i in range(V):
            assert (sas.nexthop_masks(i) == q.nexthops(i)).all(), (tag, i)
        for i in rng.sample(range(V), 3):
            ref = spf_py.run_spf(csr, i, True)
            nb = g.nbrs(i)
            m = sas.nexthop_masks(i)
            for v, (_, nhs, _, _) in ref.items():
                if v == i:
                    continue
                got = {int(nb[w * 64 + b]) for w in range(m.shape[1]) for b in range(64)
                       if (int(m[v, w]) >> b) & 1}
                assert got == set(nhs), (tag, i, v)
        q.close()
        g.close()

    check(csr, "initial")
    for kinds in (["down"], ["metric_down"], ["drain"], ["metric_up"], ["up", "down"]):
        links, ov = _churn(V, links, ov, rng, kinds, wmax=wmax)
        csr = abi.Csr.from_links(V, links, ov)
        rep = sas.update(csr)
        assert "nexthops_ms" in rep.extra
        check(csr, kinds)
    sas.close()


@pytest.mark.gpu
@pytest.mark.parametrize("V,L,wmax", [(2500, 9000, 30), (2500, 9000, 1), (40000, 160000, 1000)])
def test_link_flaps_patched_in_place(gpu_ready, V, L, wmax, monkeypatch):
    """Link down / back up (and parallel-link churn) on a distance table keep
    the resident device graph: the half-edges stay in place as self-loops
    (spf_graph_set_edges) and the repaired table equals a full recompute and
    the CPU oracle after every event -- flaps, metric changes on the patched
    layout, drains, a brand-new link (that one rebuilds the graph), and the
    same sequence with the in-place path disabled."""
    import torch

    for inplace in ("1", "0"):
        monkeypatch.setenv("OPENR_SPF_LINKS_INPLACE", inplace)
        rng = random.Random(V + L + wmax)
        links = _random_links(V, L, rng, wmax=wmax)
        ov = np.zeros(V, dtype=np.uint8)
        csr = abi.Csr.from_links(V, links, ov)
        srcs = np.asarray(sorted(rng.sample(range(V), min(V, 600))), dtype=np.uint32)
        torch.cuda.set_device(0)
        sas = AS.ShardedAllSources(csr, sources=srcs)
        sas.run()
        gone = []
        steps = ["down", "down", "up", "metric", "drain", "up", "new", "down", "metric"]
        for kind in steps:
            if kind == "down":
                i = rng.randrange(len(links))
                gone.append((i, links.pop(i)))
            elif kind == "up":
                links.insert(*gone.pop())
            elif kind == "metric":
                i = rng.randrange(len(links))
                u, v, a, b = links[i]
                links[i] = (u, v, a + 1 + rng.randrange(wmax), b)
            elif kind == "drain":
                ov[rng.randrange(V)] ^= 1
            elif kind == "new":
                while True:
                    u, v = rng.randrange(V), rng.randrange(V)
                    if u != v:
                        break
                links.append((u, v, rng.randint(1, wmax), rng.randint(1, wmax)))
            csr = abi.Csr.from_links(V, links, ov.copy())  # the old CSR keeps its own bits
            rep = sas.update(csr)
            if inplace == "1" and kind in ("down", "up", "metric", "drain"):
                assert rep.graph_patched, kind
            if kind == "new":
                assert not rep.graph_patched
            got = sas.table.cpu().numpy().view(np.uint32)[: len(srcs)]
            pick = np.asarray(sorted(rng.sample(range(len(srcs)), 32)))
            assert (got[pick] == _oracle_rows(csr, srcs[pick])).all(), (inplace, kind)
            if V <= 3000:
                assert (got == _full_table(csr, srcs)).all(), (inplace, kind)
        sas.run()  # a full pass over the patched layout
        got = sas.table.cpu().numpy().view(np.uint32)[: len(srcs)]
        pick = np.asarray(sorted(rng.sample(range(len(srcs)), 32)))
        assert (got[pick] == _oracle_rows(csr, srcs[pick])).all()
        sas.close()
