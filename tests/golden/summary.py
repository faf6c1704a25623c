"""Per-query SPF summaries (TEST INFRASTRUCTURE): the same four numbers
oracle/csr_spf.h computes on the CPU, computed here from reference-form
SpfResults or from the engine's flat rows.

  reached   number of reached nodes (the source included)
  sum_dist  sum of their distances
  sum_nh    number of (node, next-hop node) pairs
  mix       sum_v splitmix64((d[v] << 24) ^ v)
            + sum_{(v, n in NH(v))} splitmix64(((v + 1) << 32) | n)   (mod 2^64)

Node ids are name ranks (the device graph's ids).  Order-free, so any
correct engine reproduces them bit-exactly.
"""

from __future__ import annotations

import numpy as np

M64 = (1 << 64) - 1
UNREACHED32 = np.uint32(0xFFFFFFFF)


def splitmix64(x: int) -> int:
    x = (x + 0x9E3779B97F4A7C15) & M64
    x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & M64
    x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & M64
    return x ^ (x >> 31)


def splitmix64_np(x: np.ndarray) -> np.ndarray:
    x = x.astype(np.uint64, copy=True)
    with np.errstate(over="ignore"):
        x += np.uint64(0x9E3779B97F4A7C15)
        x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return x ^ (x >> np.uint64(31))


def summary_from_spf_result(res, names_by_rank):
    """getSpfResult-form dict {name: (metric, next-hop names, pathLinks)}."""
    ids = {n: i for i, n in enumerate(names_by_rank)}
    reached = sum_d = sum_nh = mix = 0
    for name, val in res.items():
        v = ids[name]
        d = int(val[0])
        reached += 1
        sum_d += d
        mix = (mix + splitmix64(((d << 24) & M64) ^ v)) & M64
        for h in val[1]:
            sum_nh += 1
            mix = (mix + splitmix64(((v + 1) << 32) | ids[h])) & M64
    return (reached, sum_d, sum_nh, mix)


_POP8 = np.array([bin(i).count("1") for i in range(256)], dtype=np.uint8)


def summaries_full(rows32, masks, words, nbrs, threads=None):
    """Every query's four numbers (mix included) from the engine's rows,
    computed by the oracle extension's multi-threaded rows_summary (checker
    code, oracle/ref_decision.cpp) -- the pure numpy path below is too slow
    to expand every (node, next hop) pair of a 9,976-source batch."""
    import os

    from oracle import _oracle_ref as O

    Q, V = rows32.shape
    words = np.asarray(words, dtype=np.uint64)
    mask_off = np.zeros(Q + 1, dtype=np.uint64)
    mask_off[1:] = np.cumsum(np.uint64(V) * words)
    nbr_off = np.zeros(Q + 1, dtype=np.uint32)
    nbr_off[1:] = np.cumsum([len(n) for n in nbrs])
    nbr_ids = np.concatenate([np.asarray(n, dtype=np.uint32) for n in nbrs] or [np.zeros(0, np.uint32)])
    if len(nbr_ids) == 0:
        nbr_ids = np.zeros(1, dtype=np.uint32)
    return O.rows_summary(np.ascontiguousarray(rows32, dtype=np.uint32), np.ascontiguousarray(masks),
                          mask_off, nbr_off, nbr_ids, threads or min(16, os.cpu_count() or 1))


def summaries_from_rows(rows32, masks, words, nbrs, mix_rows=()):
    """Engine output of a batch -> uint64 [Q, 4].

    rows32    uint32 [Q, V] distance rows (0xFFFFFFFF = unreached)
    masks     uint64, the queries' next-hop masks back to back (V * words[q])
    words     mask words per query
    nbrs      per query: node id of each mask bit (the source's neighbours)
    mix_rows  query indices whose `mix` is computed (the rest stay 0: the
              pair expansion is the slow part)
    """
    Q, V = rows32.shape
    out = np.zeros((Q, 4), dtype=np.uint64)
    reach = rows32 != UNREACHED32
    out[:, 0] = reach.sum(axis=1)
    out[:, 1] = np.where(reach, rows32, 0).astype(np.uint64).sum(axis=1)
    words = np.asarray(words, dtype=np.int64)
    offs = np.zeros(Q + 1, dtype=np.int64)
    offs[1:] = np.cumsum(V * words)
    # per-query popcount sums over each query's (non-empty) byte range
    pop = _POP8[masks[: offs[-1]].view(np.uint8)]
    out[:, 2] = np.add.reduceat(pop, offs[:-1] * 8, dtype=np.int64).astype(np.uint64)
    vids = np.arange(V, dtype=np.uint64)
    for q in mix_rows:
        r = rows32[q]
        m = reach[q]
        d = r[m].astype(np.uint64)
        mix = splitmix64_np((d << np.uint64(24)) ^ vids[m]).sum(dtype=np.uint64)
        W = int(words[q])
        mk = masks[offs[q] : offs[q + 1]].reshape(V, W)
        bits = np.unpackbits(mk.view(np.uint8).reshape(V, W * 8), axis=1, bitorder="little")
        vv, bb = np.nonzero(bits)
        if len(vv):
            nb = np.asarray(nbrs[q], dtype=np.uint64)[bb]
            key = ((vv.astype(np.uint64) + np.uint64(1)) << np.uint64(32)) | nb
            with np.errstate(over="ignore"):
                mix = mix + splitmix64_np(key).sum(dtype=np.uint64)
        out[q, 3] = mix
    return out


def dist_summaries_torch(rows):
    """(reached, sum_dist, 0, mix) of distance-only rows, computed where the
    rows live: `rows` is an int32 torch tensor [Q, V] (-1 = unreached, the
    uint32 rows reinterpreted), on any device — the checker side of the
    100,000-row WAN golden (tests/golden/wan100k_allsources.npz) without
    copying 40 GB to the host.  uint64 arithmetic is done in int64 (two's
    complement: sums and products wrap mod 2^64 alike, right shifts are
    masked to be logical).  Returns uint64 [Q, 4] numpy."""
    import torch

    def lsr(x, k):
        return (x >> k) & ((1 << (64 - k)) - 1)

    def s64(c):
        return c - (1 << 64) if c >= 1 << 63 else c

    Q, V = rows.shape
    reach = rows != -1
    d = rows.to(torch.int64) & 0xFFFFFFFF
    x = (d << 24) ^ torch.arange(V, device=rows.device, dtype=torch.int64)
    x = x + s64(0x9E3779B97F4A7C15)
    x = (x ^ lsr(x, 30)) * s64(0xBF58476D1CE4E5B9)
    x = (x ^ lsr(x, 27)) * s64(0x94D049BB133111EB)
    x = x ^ lsr(x, 31)
    zero = torch.zeros((), dtype=torch.int64, device=rows.device)
    out = torch.stack([reach.sum(dim=1, dtype=torch.int64),
                       torch.where(reach, d, zero).sum(dim=1),
                       torch.zeros(Q, dtype=torch.int64, device=rows.device),
                       torch.where(reach, x, zero).sum(dim=1)], dim=1)
    return out.cpu().numpy().view(np.uint64)
