"""Pure-Python restatement of LinkState::runSpf over the flat CSR model.

TEST INFRASTRUCTURE ONLY (oracle): imported by tests/, __graft_entry__.smoke()
and bench.py's cpu_baseline leg as a checker; never by the product path.

It replays the reference DijkstraQ literally (openr/decision/LinkState.cpp:
806-880 and LinkState.h:483-535):
  * the queue holds DISCOVERED nodes only and extracts the (metric, name)
    minimum (node ids are name ranks, so name order == id order);
  * a settled node is recorded, and expanded only if it is the source or not
    overloaded (LinkState.cpp:829-836);
  * a link relaxes only into unsettled nodes, with `>=` (equal cost appends
    the path link and unions the next hops), a strictly better metric resets
    them (LinkState.cpp:855-871);
  * "directly connected": if the next-hop set is still empty after the union,
    the neighbour itself is the next hop (LinkState.cpp:867-870);
  * metrics are uint64 and sums wrap mod 2^64 (LinkStateMetric, LinkState.h:22).

Small graphs only (pure-Python loops).  The C++ restatement in oracle/ is the
one used for big inputs.
"""

from __future__ import annotations

import heapq

MASK64 = (1 << 64) - 1


def run_spf(csr, src, use_link_metric=True, ignore=frozenset()):
    """Returns {node: (metric, frozenset(nexthop nodes), [(edge, prev)...],
    settle_rank)} for every reached node.

    `csr` is openr_amd.abi.Csr; `ignore` is a set of link ids
    (linksToIgnore).  Path links are edge indices of the half-edge u->v,
    in relaxation order; within one settled node the edges are visited in
    CSR row order (the caller fixes that order to the reference's
    linksFromNode iteration order when it matters).
    """
    row, col, met, lid = csr.row_ptr, csr.col, csr.metric, csr.link_id
    ov = csr.overloaded
    dist = {src: 0}
    nh = {src: set()}
    paths = {src: []}
    settled = {}
    heap = [(0, src)]
    gen = {src: 0}
    while heap:
        d, u = heapq.heappop(heap)
        if u in settled or dist[u] != d:
            continue
        settled[u] = len(settled)
        if u != src and ov[u]:
            continue
        for e in range(int(row[u]), int(row[u + 1])):
            v = int(col[e])
            if v in settled or int(lid[e]) in ignore:
                continue
            w = int(met[e]) if use_link_metric else 1
            c = (d + w) & MASK64
            if v not in dist:
                dist[v] = c
                nh[v] = set()
                paths[v] = []
                heapq.heappush(heap, (c, v))
            if dist[v] >= c:
                if dist[v] > c:
                    dist[v] = c
                    nh[v] = set()
                    paths[v] = []
                    heapq.heappush(heap, (c, v))
                paths[v].append((e, u))
                nh[v] |= nh[u]
                if not nh[v]:
                    nh[v].add(v)
    return {
        v: (dist[v], frozenset(nh[v]), paths[v], settled[v]) for v in settled
    }
