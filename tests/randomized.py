"""Seeded random topologies / prefix sets for oracle-vs-engine parity.

Used by tests/test_engine_parity_gpu.py (MI355X engine vs CPU oracle on the
same inputs, bit-exact) and by the CPU suite (oracle self-consistency).
"""

from __future__ import annotations

import random

from openr_amd import thrift as T


def random_network(
    seed,
    n_nodes=30,
    n_links=70,
    metric_range=(1, 20),
    zero_metric_prob=0.0,
    parallel_prob=0.08,
    overload_prob=0.05,
    link_overload_prob=0.03,
    node_labels=True,
    areas=("0",),
    bgp=False,
):
    """Returns (adj_dbs per area, prefix_dbs).  Node names are random-ish
    strings so that name order differs from creation order."""
    rng = random.Random(seed)
    names = [f"n{rng.randrange(10**6):06d}-{i}" for i in range(n_nodes)]
    adjs = {a: {n: [] for n in names} for a in areas}
    ifcount = {}
    for k in range(n_links + n_nodes - 1):
        area = rng.choice(areas)
        if k < n_nodes - 1:
            u, v = names[rng.randrange(k + 1)], names[k + 1]  # backbone
        else:
            u, v = rng.sample(names, 2)
        reps = 2 if rng.random() < parallel_prob else 1
        for _ in range(reps):
            key = (min(u, v), max(u, v))
            i = ifcount.get(key, 0)
            ifcount[key] = i + 1
            ifu, ifv = f"if_{u}_{v}_{i}", f"if_{v}_{u}_{i}"

            def metric():
                if rng.random() < zero_metric_prob:
                    return 0
                return rng.randint(*metric_range)

            au = T.createAdjacency(v, ifu, ifv, f"fe80::{k+1:x}:{i+1:x}", f"10.{k % 250}.{i}.1",
                                   metric(), 50000 + (k * 4 + i) % 9000)
            av = T.createAdjacency(u, ifv, ifu, f"fe80::{k+1:x}:{i+1:x}:2", f"10.{k % 250}.{i}.2",
                                   metric(), 50000 + (k * 4 + i + 7) % 9000)
            au.isOverloaded = rng.random() < link_overload_prob
            adjs[area][u].append(au)
            adjs[area][v].append(av)
    adj_dbs = {}
    for area in areas:
        dbs = []
        for idx, n in enumerate(names):
            if not adjs[area][n] and rng.random() < 0.5:
                continue
            label = (101 + idx) if node_labels else 0
            dbs.append(T.createAdjDb(n, adjs[area][n], label, rng.random() < overload_prob, area))
        adj_dbs[area] = dbs
    prefix_dbs = []
    for idx, n in enumerate(names):
        entries = [T.createPrefixEntry(T.toIpPrefix(f"fc00:{idx:x}::1/128"))]
        r = rng.random()
        if r < 0.15:
            entries.append(T.createPrefixEntry(T.toIpPrefix(f"10.{idx}.0.0/16")))
        elif r < 0.3:
            e = T.createPrefixEntry(
                T.toIpPrefix(f"fd00:{idx:x}::/64"),
                forwardingType=T.PrefixForwardingType.SR_MPLS,
                forwardingAlgorithm=T.PrefixForwardingAlgorithm.KSP2_ED_ECMP,
            )
            entries.append(e)
        if rng.random() < 0.1:  # anycast prefix shared by a few nodes
            entries.append(T.createPrefixEntry(T.toIpPrefix("fc99::1/128")))
        if bgp:
            entries += _bgp_entries(rng, idx)
        for area in areas:
            prefix_dbs.append(T.createPrefixDb(n, entries, area))
    return names, adj_dbs, prefix_dbs


# BGP prefixes shared by random announcers, each with a random MetricVector
# (Lsdb.thrift:183-213): few metric types, small values and random ops so that
# best-path selection (Decision.cpp:715-800, MetricVectorUtils Util.cpp:
# 1051-1228) hits wins, losses, ties, tie-breakers and absent entries
_BGP_PREFIXES = [f"2001:db8:{k:x}::/48" for k in range(6)]


def _bgp_entries(rng, idx):
    out = []
    for k, pfx in enumerate(_BGP_PREFIXES):
        if rng.random() >= 0.25:
            continue
        metrics = []
        for t in rng.sample(range(4), rng.randint(1, 3)):
            metrics.append(T.createMetricEntity(
                t, 10 - t,  # priority fixed per type
                rng.choice([T.CompareType.WIN_IF_PRESENT, T.CompareType.WIN_IF_NOT_PRESENT,
                            T.CompareType.IGNORE_IF_NOT_PRESENT]),
                rng.random() < 0.3,
                [rng.randint(0, 2) for _ in range(rng.randint(1, 2))]))
        e = T.createPrefixEntry(T.toIpPrefix(pfx), T.PrefixType.BGP, f"d{idx}",
                                mv=T.MetricVector(0, metrics))
        if k >= 4:  # SR-MPLS BGP prefixes (selectKsp2 with metric-vector best path)
            e.forwardingType = T.PrefixForwardingType.SR_MPLS
            e.forwardingAlgorithm = rng.choice([T.PrefixForwardingAlgorithm.SP_ECMP,
                                                T.PrefixForwardingAlgorithm.KSP2_ED_ECMP])
        out.append(e)
    return out


def load(M, adj_dbs, prefix_dbs, order_seed=0):
    areas = M.AreaLinkStates()
    rng = random.Random(order_seed)
    for area, dbs in adj_dbs.items():
        ls = areas.add(area)
        order = list(dbs)
        rng.shuffle(order)
        for db in order:
            ls.updateAdjacencyDatabase(db)
    ps = M.PrefixState()
    for pdb in prefix_dbs:
        ps.updatePrefixDatabase(pdb)
    return areas, ps
