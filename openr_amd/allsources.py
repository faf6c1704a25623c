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

    def __init__(self, csr, sources=None, group=None, device=None, gather=True):
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
        if self.graph.needs_exact:
            raise abi.SpfError("all-sources tables need 32-bit sums (no metric 0 / 64-bit metrics)")
        self.stream = torch.cuda.Stream(device=self.device)
        self.graph.set_stream(self.stream.cuda_stream)
        mine = src[self.first : self.first + self.count]
        self.query = self.graph.query(mine, 0) if self.count else None
        self.kernel = self.query.kernel if self.query else ""
        rows = self.world * self.cap if gather else self.cap
        self.gather = gather
        self.table = torch.full((rows, self.V), -1, dtype=torch.int32, device=f"cuda:{self.device}")

    def local_block(self):
        if not self.gather:
            return self.table
        return self.table[self.rank * self.cap : (self.rank + 1) * self.cap]

    def run(self) -> AllSourcesRun:
        import torch
        import torch.distributed as dist

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
        if multi:
            dist.barrier(group=self.group)
        out.wall_ms = (time.perf_counter() - t0) * 1e3
        out.gather_ms = (t2 - t1) * 1e3
        out.extra["compute_wall_ms"] = (t1 - t0) * 1e3
        if self.query:
            out.spf_ms = self.query.elapsed_ms()
            out.fetch_ms = ev0.elapsed_time(ev1)
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
