"""All-sources SPF tables sharded over the GPUs of one node.

Every SSSP of an all-sources pass is independent given the read-only graph,
so rank r of W solves a contiguous block of sources (`shard`) on its own
MI355X and the one exchange step is an all-gather of the per-source distance
rows over xGMI (torch.distributed "nccl" = RCCL), in place: each rank copies
its rows into its slot of the output table (`spf_query_fetch_rows`, device to
device on the engine stream) and RCCL fills the other slots.

What this replaces.  The reference computes one source at a time and keeps
the results in the string-keyed memo of LinkState::getSpfResult
(openr/decision/LinkState.cpp:791-801, memo LinkState.h:279-282); an
all-sources view (Decision::getDecisionRouteDb for every node,
openr/decision/Decision.cpp:1437-1462, or DecisionTest getRouteMap
DecisionTest.cpp:256-274) fills it with V runSpf calls.  Here the memo of a
whole area is one uint32 table [sources][V] in HBM (0xFFFFFFFF =
unreachable; the uint64 LinkStateMetric sums fit 32 bits whenever the fast
kernels run, i.e. spf_graph_needs_exact == 0).

The gather logic is device-agnostic (any torch.distributed backend, tensors
on any device), so the N>1 path is tested with gloo on the CPU; the row
producer on the GPU is the HIP engine (openr_amd.abi), never a CPU fallback.
"""

from __future__ import annotations

import os
import time
from dataclasses import dataclass, field

UNREACHABLE_U32 = 0xFFFFFFFF


def shard(n: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous block (first, count) of n sources for `rank`.

    Blocks differ in size by at most one; the first n % world ranks take the
    larger ones.  Every rank's slot in the gathered table has
    shard_cap(n, world) rows, so RCCL sees equal-sized contributions.
    """
    if world <= 0 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} of {world}")
    base, extra = divmod(n, world)
    first = rank * base + min(rank, extra)
    return first, base + (1 if rank < extra else 0)


def shard_cap(n: int, world: int) -> int:
    """Rows per rank slot of the gathered table (the largest block)."""
    return (n + world - 1) // world


def slot_row(i: int, n: int, world: int) -> int:
    """Row of global source i in the gathered [world * cap, V] table."""
    if not 0 <= i < n:
        raise IndexError(i)
    base, extra = divmod(n, world)
    big = extra * (base + 1)  # sources held by the ranks with a larger block
    if i < big:
        r, k = divmod(i, base + 1)
    else:
        r, k = divmod(i - big, base)
        r += extra
    return r * shard_cap(n, world) + k


def slot_index(n: int, world: int):
    """numpy int64 [n]: slot_row for every source, in source order."""
    import numpy as np

    cap = shard_cap(n, world)
    out = np.empty(n, dtype=np.int64)
    for r in range(world):
        first, count = shard(n, world, r)
        out[first : first + count] = r * cap + np.arange(count)
    return out


def gather_rows(local, n: int, group=None, out=None):
    """All-gather the per-rank [cap, ...] row blocks into the [world*cap, ...]
    table (rank r's block lands at rows [r*cap, (r+1)*cap)).

    `local` may be this rank's own slot of `out` (in-place gather: no copy).
    """
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group) if dist.is_initialized() else 1
    cap = shard_cap(n, world)
    if local.shape[0] != cap:
        raise ValueError(f"local block has {local.shape[0]} rows, expected {cap}")
    if out is None:
        out = torch.empty((world * cap,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    if out.shape[0] != world * cap or out.shape[1:] != local.shape[1:]:
        raise ValueError("output table has the wrong shape")
    if world == 1:
        if out.data_ptr() != local.data_ptr():
            out.copy_(local)
        return out
    dist.all_gather_into_tensor(out, local.contiguous(), group=group)
    return out


def exchange_rows(table, local_rows, n: int, group=None):
    """Propagate repaired rows to every rank's copy of the gathered table.

    `local_rows` (int64 [k], on the table's device) are rows of `table`
    inside this rank's slot that were just rewritten; after the call every
    rank's table holds them.  Ranks repair different numbers of rows, so the
    counts are all-gathered first, each rank contributes a block padded to
    the largest count (row index -1 = padding), and the received rows are
    copied into place with index_copy_.  Traffic is proportional to the
    repaired rows, not to the table.  Returns the number of rows received.
    """
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group) if dist.is_initialized() else 1
    if world == 1:
        return 0
    dev = table.device
    k = torch.tensor([int(local_rows.numel())], dtype=torch.int64, device=dev)
    counts = torch.empty(world, dtype=torch.int64, device=dev)
    dist.all_gather_into_tensor(counts, k, group=group)
    m = int(counts.max().item())
    if m == 0:
        return 0
    idx = torch.full((m,), -1, dtype=torch.int64, device=dev)
    idx[: local_rows.numel()] = local_rows
    rows = torch.zeros((m,) + tuple(table.shape[1:]), dtype=table.dtype, device=dev)
    if local_rows.numel():
        rows[: local_rows.numel()] = table.index_select(0, local_rows)
    all_idx = torch.empty(world * m, dtype=torch.int64, device=dev)
    all_rows = torch.empty((world * m,) + tuple(table.shape[1:]), dtype=table.dtype, device=dev)
    dist.all_gather_into_tensor(all_idx, idx, group=group)
    dist.all_gather_into_tensor(all_rows, rows, group=group)
    keep = all_idx >= 0
    table.index_copy_(0, all_idx[keep], all_rows[keep])
    return int(keep.sum().item())


def transit_hop_bound(csr) -> int:
    """Host restatement of the engine's transit_hop_bound (spf_device.hip):
    2 * eccentricity of the highest-degree transit node r under the transit
    rule (a node is expanded iff it is r or not overloaded), or 0 when r does
    not reach every node (or no node may be transited)."""
    import numpy as np

    V = int(csr.num_nodes)
    row = np.asarray(csr.row_ptr, dtype=np.int64)
    col = np.asarray(csr.col, dtype=np.int64)
    transit = np.asarray(csr.overloaded, dtype=np.uint8) == 0
    if V == 0 or not transit.any():
        return 0
    deg = np.diff(row)
    cand = np.where(transit)[0]
    r = int(cand[np.argmax(deg[cand])])  # first of the largest degree
    seen = np.zeros(V, dtype=bool)
    seen[r] = True
    cur = np.array([r], dtype=np.int64)
    depth = 0
    while cur.size:
        exp = cur[(cur == r) | transit[cur]]
        if exp.size == 0:
            break
        lo, hi = row[exp], row[exp + 1]
        idx = np.repeat(hi - (hi - lo).cumsum(), hi - lo) + np.arange((hi - lo).sum())
        nb = np.unique(col[idx]) if idx.size else idx
        nb = nb[~seen[nb]]
        if nb.size == 0:
            break
        seen[nb] = True
        depth += 1
        cur = nb
    return 2 * depth if seen.all() else 0


def needs_64bit_rows(csr) -> bool:
    """Host restatement of spf_graph_needs_exact for metric runs (the
    engine's refresh_exact rule): a metric-0 or wrapping (> 2^31 - 1) metric,
    or maxw * (V - 1) >= 2^32 - 1 AND no transit hop bound h with
    maxw * (h + 1) < 2^32 - 1.  Checked BEFORE any state changes."""
    import numpy as np

    m = np.asarray(csr.metric, dtype=np.uint64)
    if m.size == 0:
        return False
    if (m == 0).any() or (m > np.uint64(0x7FFFFFFF)).any():
        return True
    maxw = int(m.max())
    if maxw * max(csr.num_nodes - 1, 0) < 0xFFFFFFFF:
        return False
    h = transit_hop_bound(csr)
    return not (h and maxw * (h + 1) < 0xFFFFFFFF)


@dataclass
class RepairRun:
    """One incremental table update on one rank (ShardedAllSources.update)."""

    deltas: int = 0
    affected: int = 0        # this rank's recomputed sources
    affected_total: int = 0  # over all ranks
    diff_ms: float = 0.0     # host edge diff (spf_graph_diff)
    graph_ms: float = 0.0    # new device graph (host flatten + upload)
    screen_ms: float = 0.0   # spf_table_screen (kernel + transfers)
    spf_ms: float = 0.0      # device time of the affected sources' SSSPs
    exchange_ms: float = 0.0 # repaired rows to the other ranks
    wall_ms: float = 0.0     # barrier to barrier
    graph_patched: bool = False  # device graph patched in place (same links)
    relaxed: bool = False    # rows repaired in place (spf_table_repair), not recomputed
    extra: dict = field(default_factory=dict)


@dataclass
class AllSourcesRun:
    """Timing of one sharded all-sources pass on one rank."""

    first: int = 0
    count: int = 0
    spf_ms: float = 0.0     # HIP-event device time of this rank's SSSP batch
    fetch_ms: float = 0.0   # rows -> table slot (device to device)
    gather_ms: float = 0.0  # RCCL all-gather (wall, after the compute)
    wall_ms: float = 0.0    # barrier to barrier on this rank
    kernel: str = ""
    extra: dict = field(default_factory=dict)


class ShardedAllSources:
    """All-sources distance table of one area over the ranks of `group`.

    Construct once per topology (the device graph and the query of this
    rank's sources stay resident in HBM), then run() per pass.  Rank r's
    rows come from the HIP engine on the rank's current device.  With
    gather=False each rank keeps only its own block (the "no-gather" mode of
    SURVEY §8(e): a RouteDb needs only its own row).
    """

    def __init__(self, csr, sources=None, group=None, device=None, gather=True, nexthops=False):
        import numpy as np
        import torch
        import torch.distributed as dist

        from openr_amd import abi

        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.device = torch.cuda.current_device() if device is None else device
        self.V = csr.num_nodes
        src = np.arange(self.V, dtype=np.uint32) if sources is None else np.asarray(sources, dtype=np.uint32)
        self.n = len(src)
        self.first, self.count = shard(self.n, self.world, self.rank)
        self.cap = shard_cap(self.n, self.world)
        self.graph = abi.Graph(csr, device=self.device)
        self._layout(csr)
        if self.graph.needs_exact:
            raise abi.SpfError("all-sources tables need 32-bit sums (no metric 0 / 64-bit metrics)")
        self.stream = torch.cuda.Stream(device=self.device)
        self.graph.set_stream(self.stream.cuda_stream)
        mine = src[self.first : self.first + self.count]
        self.query = self.graph.query(mine, 0) if self.count else None
        self.kernel = self.query.kernel if self.query else ""
        rows = self.world * self.cap if gather else self.cap
        self.gather = gather
        self.csr = csr
        self.sources = src
        self.table = torch.full((rows, self.V), -1, dtype=torch.int32, device=f"cuda:{self.device}")
        # next-hop masks of every source (spf_table_nexthops from the table
        # rows; one rank: a source's neighbours' rows must all be local)
        self.nexthops = nexthops
        self.masks = None
        if nexthops:
            if self.world > 1 or self.n != self.V:
                raise ValueError("next-hop tables need one rank and every node as a source")
            self._mask_layout()

    def _mask_layout(self):
        import numpy as np
        import torch

        from openr_amd import abi

        self.mask_words, self.mask_off, total = abi.mask_layout(self.graph, self.sources)
        self.masks = torch.zeros(max(total, 1), dtype=torch.int64, device=f"cuda:{self.device}")
        self.row_of = np.full(self.V, -1, dtype=np.int32)
        self.row_of[self.sources] = np.arange(self.n, dtype=np.int32)

    def _refresh_masks(self, idx):
        """Masks of sources[idx] from the current table rows."""
        if len(idx):
            self.graph.table_nexthops(self.table.data_ptr(), self.V, self.row_of,
                                      self.sources[idx], self.masks.data_ptr(), self.mask_off[idx])

    def nexthop_masks(self, i):
        """[V, W] uint64 next-hop masks of source i (host copy)."""
        W = int(self.mask_words[i])
        o = int(self.mask_off[i])
        return self.masks[o : o + self.V * W].cpu().numpy().view("uint64").reshape(self.V, W)

    def local_block(self):
        if not self.gather:
            return self.table
        return self.table[self.rank * self.cap : (self.rank + 1) * self.cap]

    def run(self) -> AllSourcesRun:
        import torch
        import torch.distributed as dist

        if self.query is None and self.count:
            mine = self.sources[self.first : self.first + self.count]
            self.query = self.graph.query(mine, 0)
            self.kernel = self.query.kernel
        out = AllSourcesRun(first=self.first, count=self.count, kernel=self.kernel)
        multi = self.world > 1
        if multi:
            dist.barrier(group=self.group)
        torch.cuda.synchronize(self.device)
        t0 = time.perf_counter()
        with torch.cuda.stream(self.stream):
            ev0 = torch.cuda.Event(enable_timing=True)
            ev1 = torch.cuda.Event(enable_timing=True)
            if self.query:
                self.query.run(sync=False)
                ev0.record(self.stream)
                self.query.fetch_rows(0, self.count, self.local_block().data_ptr(), self.V * 4, on_device=True)
                ev1.record(self.stream)
            self.stream.synchronize()
            t1 = time.perf_counter()
            if self.gather and multi:
                gather_rows(self.local_block(), self.n, group=self.group, out=self.table)
                torch.cuda.synchronize(self.device)
            t2 = time.perf_counter()
            if self.nexthops:
                import numpy as np

                self._refresh_masks(np.arange(self.n))
                out.extra["nexthops_ms"] = (time.perf_counter() - t2) * 1e3
        if multi:
            dist.barrier(group=self.group)
        out.wall_ms = (time.perf_counter() - t0) * 1e3
        out.gather_ms = (t2 - t1) * 1e3
        out.extra["compute_wall_ms"] = (t1 - t0) * 1e3
        if self.query:
            out.spf_ms = self.query.elapsed_ms()
            out.fetch_ms = ev0.elapsed_time(ev1)
        return out

    def _layout(self, csr):
        """Half-edge layout of the resident device graph: heads as created,
        which half-edges are up, their current metrics (spf_graph_set_edges
        keeps down half-edges in place)."""
        import numpy as np

        self._lay_row = np.asarray(csr.row_ptr, dtype=np.int64)
        self._lay_col = np.asarray(csr.col, dtype=np.uint32).copy()
        self._lay_up = np.ones(len(csr.col), dtype=bool)
        self._lay_w = np.asarray(csr.metric, dtype=np.uint64).copy()
        self._lay_rev = np.asarray(csr.rev, dtype=np.int64).copy()  # the other half of each link
        self._lay_is_csr = csr  # the layout is exactly this CSR's (no link set in place)

    def _links_in_place(self, deltas):
        """Map link-set deltas (spf_graph_diff: REMOVED / ADDED half-edges
        (tail, head, metric), multiset per tail) onto the resident layout:
        a removed half-edge is an up slot (tail, head, metric) going down, an
        added one a down slot (tail, head) coming back up with its metric.
        Slots are chosen as LINK PAIRS: the pull kernels read a slot's head
        together with win[e] = metric of its reverse half rev[e], so both
        halves of a link must be up or down together.  An added half-edge
        takes, in order of preference, the slot a removed delta of this same
        update took down (a metric change), a slot whose other half this pass
        already brought up, then any down slot; a layout in which some touched
        slot's halves disagree afterwards (parallel links matched across
        links) is refused.  None when some added half-edge has no down slot (a
        new link: rebuild), the halves cannot be paired, or a metric is 0 /
        past 2^31 - 1 (64-bit graphs rebuild too)."""
        import numpy as np

        from openr_amd import abi

        SCOPE_NOT_TAIL = 2
        up0, w0, rev = self._lay_up, self._lay_w, self._lay_rev
        touched = {}  # slot -> (up, metric), applied once every delta has mapped
        removed_here = set()
        order = sorted((d for d in deltas if int(d["scope"]) != SCOPE_NOT_TAIL),
                       key=lambda d: int(d["kind"]) != abi.SPF_DELTA_REMOVED)

        def state(e):
            t = touched.get(e)
            return (t[0], t[1]) if t is not None else (bool(up0[e]), int(w0[e]))

        for d in order:
            u, v, m, kind = int(d["tail"]), int(d["head"]), int(d["metric"]), int(d["kind"])
            if m == 0 or m > 0x7FFFFFFF:
                return None
            lo, hi = int(self._lay_row[u]), int(self._lay_row[u + 1])
            slots = [lo + int(k) for k in np.nonzero(self._lay_col[lo:hi] == v)[0]]
            removed = kind == abi.SPF_DELTA_REMOVED
            if removed:
                cand = [e for e in slots if state(e)[0] and state(e)[1] == m]
            else:
                down = [e for e in slots if not state(e)[0]]
                cand = ([e for e in down if e in removed_here]
                        + [e for e in down if e not in removed_here and int(rev[e]) in touched
                           and touched[int(rev[e])][0]]
                        + [e for e in down if e not in removed_here])
            if not cand:
                return None
            e = cand[0]
            if removed:
                removed_here.add(e)
                touched[e] = (False, state(e)[1])
            else:
                touched[e] = (True, m)
        for e in list(touched):
            if state(e)[0] != state(int(rev[e]))[0]:
                return None  # the halves of a link disagree: rebuild
        e = np.fromiter(touched.keys(), dtype=np.uint32, count=len(touched))
        new_up = np.fromiter((t[0] for t in touched.values()), dtype=bool, count=len(touched))
        new_w = np.fromiter((t[1] for t in touched.values()), dtype=np.uint64, count=len(touched))
        up0[e] = new_up
        w0[e] = new_w
        return e, new_up.astype(np.uint8), new_w

    def update(self, new_csr) -> RepairRun:
        """Repair the table after a topology change instead of recomputing
        every source (the reference clears its whole SPF
        memo, LinkState.cpp:712-715).

        `new_csr` must keep the node ids (same names, so the same ranks).
        The change is listed as directed edge deltas (spf_graph_diff), the
        screen kernel marks the sources of this rank whose shortest-path DAG
        a delta can touch (spf_table_screen), only those rows are repaired in
        place on the new device graph (spf_table_repair; or recomputed and
        scattered when the repair image does not fit LDS, or with
        OPENR_SPF_REPAIR_RECOMPUTE=1), and the repaired rows are exchanged
        between ranks (exchange_rows).  The result equals a full recompute
        bit for bit (tests/test_table_repair.py)."""
        import numpy as np
        import torch
        import torch.distributed as dist

        from openr_amd import abi

        if new_csr.num_nodes != self.V:
            raise ValueError("node set changed: node ids are not shared, rebuild the table")
        out = RepairRun()
        multi = self.world > 1
        if needs_64bit_rows(new_csr):
            # refused before anything changes: the table, graph and query
            # still describe the old topology and stay usable
            raise abi.SpfError("all-sources tables need 32-bit sums (no metric 0 / 64-bit metrics)")
        if multi:
            dist.barrier(group=self.group)
        torch.cuda.synchronize(self.device)
        t0 = time.perf_counter()
        deltas = abi.graph_diff(self.csr, new_csr)
        t1 = time.perf_counter()
        out.deltas = len(deltas)
        # the full-batch query holds a result block the size of this rank's
        # table slot: release it before the repair allocates
        if self.query is not None:
            tr = time.perf_counter()
            self.query.close()
            self.query = None
            out.extra["release_ms"] = (time.perf_counter() - tr) * 1e3
        old = self.csr

        def same(x, y):  # shared arrays (a metric / drain event) skip the compare
            return x is y or np.array_equal(x, y)

        same_links = (
            len(old.col) == len(new_csr.col)
            and same(old.row_ptr, new_csr.row_ptr)
            and same(old.col, new_csr.col)
            and same(old.link_id, new_csr.link_id)
            and same(old.rev, new_csr.rev)
        )
        # the resident graph's layout is the old CSR's unless links were
        # taken down / up in place before
        layout_is_old = self._lay_is_csr is old or (
            bool(self._lay_up.all()) and len(self._lay_col) == len(old.col)
            and np.array_equal(self._lay_row, old.row_ptr) and np.array_equal(self._lay_col, old.col))
        inplace = None
        if (not (same_links and layout_is_old)
                and os.environ.get("OPENR_SPF_LINKS_INPLACE", "1") != "0"):
            inplace = self._links_in_place(deltas)
        if same_links and layout_is_old:
            # metric / drain churn: patch the resident device graph in place
            ch = np.nonzero(old.metric != new_csr.metric)[0]
            if len(ch):
                self.graph.patch_metrics(ch, new_csr.metric[ch])
            if not np.array_equal(old.overloaded, new_csr.overloaded):
                self.graph.set_transit(new_csr.overloaded)
            self.graph.csr = new_csr
            self._lay_w[ch] = new_csr.metric[ch]
            self._lay_is_csr = new_csr
            out.graph_patched = True
        elif inplace is not None:
            # links down / back up: the half-edges stay at their positions of
            # the resident graph (spf_graph_set_edges), transit bits as above
            e, up, w = inplace
            if len(e):
                self.graph.set_edges(e, up, w)
            self._lay_is_csr = None
            if not np.array_equal(old.overloaded, new_csr.overloaded):
                self.graph.set_transit(new_csr.overloaded)
            out.graph_patched = True
        else:
            graph = abi.Graph(new_csr, device=self.device)
            graph.set_stream(self.stream.cuda_stream)
            self.graph.close()
            self.graph = graph
            self._layout(new_csr)
        self.csr = new_csr
        t2 = time.perf_counter()
        block = self.local_block()
        base = self.rank * self.cap if self.gather else 0
        mine = self.sources[self.first : self.first + self.count]
        hit = np.zeros(0, dtype=np.int64)
        if self.count and len(deltas):
            flags = self.graph.table_screen(block.data_ptr(), self.V, mine, deltas)
            hit = np.nonzero(flags)[0]
        t3 = time.perf_counter()
        out.screen_ms = (t3 - t2) * 1e3
        out.affected = len(hit)
        relaxed = False
        if len(hit) and not os.environ.get("OPENR_SPF_REPAIR_RECOMPUTE"):
            # repair the affected rows in place (reset what lost its support,
            # relax from the boundary and the improved edges) instead of
            # recomputing them from scratch
            t = time.perf_counter()
            relaxed = self.graph.table_repair(block.data_ptr(), self.V, mine[hit],
                                              hit.astype(np.uint32), deltas)
            if relaxed:
                out.relaxed = True
                out.spf_ms = (time.perf_counter() - t) * 1e3
        if len(hit) and not relaxed:
            q = self.graph.query(mine[hit], 0)
            try:
                q.run(sync=False)
                q.scatter_rows(hit.astype(np.uint32), block.data_ptr(), self.V * 4)
                self.stream.synchronize()
                out.spf_ms = q.elapsed_ms()
            finally:
                q.close()
        t4 = time.perf_counter()
        total = len(hit)
        if self.gather and multi:
            rows = torch.from_numpy(hit + base).to(block.device)
            total = exchange_rows(self.table, rows, self.n, group=self.group) or 0
            torch.cuda.synchronize(self.device)
        elif multi:
            t = torch.tensor([len(hit)], dtype=torch.int64, device=block.device)
            dist.all_reduce(t, group=self.group)
            total = int(t.item())
        t5 = time.perf_counter()
        if self.nexthops:
            # next hops of the repaired sources (a source the screen passed
            # keeps them: they are defined by its tight edges alone); a link
            # set change -- rebuilt, or set in place (spf_graph_set_edges
            # rebuilds the distinct-neighbour lists) -- can add / drop a
            # source's neighbours, which moves its mask bits, so then every
            # source is recomputed
            if out.graph_patched and inplace is None:
                self._refresh_masks(hit)
            else:
                self._mask_layout()
                self._refresh_masks(np.arange(self.n))
            out.extra["nexthops_ms"] = (time.perf_counter() - t5) * 1e3
        if multi:
            dist.barrier(group=self.group)
        out.affected_total = total
        out.diff_ms = (t1 - t0) * 1e3
        out.graph_ms = (t2 - t1) * 1e3
        out.exchange_ms = (t5 - t4) * 1e3
        out.wall_ms = (time.perf_counter() - t0) * 1e3
        return out

    def row(self, i: int):
        """Distance row of global source i as host uint32 (needs the gathered
        table, or i in this rank's block)."""
        import numpy as np

        if self.gather:
            r = slot_row(i, self.n, self.world)
        else:
            if not self.first <= i < self.first + self.count:
                raise IndexError(f"source {i} is not in this rank's block")
            r = i - self.first
        return self.table[r].cpu().numpy().view(np.uint32)

    def close(self):
        if self.query:
            self.query.close()
            self.query = None
        self.graph.close()
