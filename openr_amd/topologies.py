"""Synthetic topologies of BASELINE.json's configs.

  grid(n)      DecisionBenchmark.cpp:360-431 (createGrid): names "0".."n²-1",
               metric 1, if-names if_<id>_<nbr>, adj label 100001+nbr,
               prefix fc00:{id>>16:02x}::{id&0xffff:02x}/128.
  fabric(...)  DecisionBenchmark.cpp:438-587 with the SSW bug fixed (every
               SSW reaches one FSW in EVERY pod, the documented intent;
               the reference emplaces one key per pod so only pod 0 sticks).
               Markers 1 = SSW, 2 = FSW, 3 = RSW; names "<marker>-<pod>-<sw>".
  wan(V, L)    SURVEY §8(d) row 3: one std::mt19937_64(12345) draw sequence.

Each generator can emit thrift AdjacencyDatabases (for LinkState /
SpfSolver) or a device CSR directly (node id = name rank, as LinkState's
flattening produces) for the raw-ABI benchmark.
"""

from __future__ import annotations

import numpy as np

from openr_amd import thrift as T


# ---------------------------------------------------------------- helpers


class Topology:
    """Undirected links with per-direction metrics between named nodes."""

    def __init__(self, names, links, ifnames=None, labels=None, node_labels=None):
        self.names = list(names)  # index = creation id
        self.links = links  # list of (a, b, metric_ab, metric_ba) by creation id
        self.ifnames = ifnames  # list of (if_a, if_b) or None -> generated
        self.labels = labels  # list of (adjlabel_a, adjlabel_b) or None
        self.node_labels = node_labels

    @property
    def num_nodes(self):
        return len(self.names)

    def rank(self):
        """creation id -> name rank (node id of the device graph)."""
        order = sorted(range(len(self.names)), key=lambda i: self.names[i])
        r = np.empty(len(self.names), dtype=np.int64)
        r[np.asarray(order, dtype=np.int64)] = np.arange(len(order))
        return r, [self.names[i] for i in order]

    def csr(self, overloaded=None):
        """Device CSR with ids = name ranks (openr_amd.abi.Csr)."""
        from openr_amd.abi import Csr

        r, _ = self.rank()
        V = self.num_nodes
        L = len(self.links)
        a = np.fromiter((l[0] for l in self.links), dtype=np.int64, count=L)
        b = np.fromiter((l[1] for l in self.links), dtype=np.int64, count=L)
        mab = np.fromiter((l[2] for l in self.links), dtype=np.int64, count=L)
        mba = np.fromiter((l[3] for l in self.links), dtype=np.int64, count=L)
        a, b = r[a], r[b]
        src = np.concatenate([a, b])
        dst = np.concatenate([b, a])
        met = np.concatenate([mab, mba]).astype(np.uint64)
        lid = np.concatenate([np.arange(L), np.arange(L)])
        half = np.concatenate([np.zeros(L, np.int64), np.ones(L, np.int64)])
        order = np.lexsort((half, lid, src))
        src, dst, met, lid, half = src[order], dst[order], met[order], lid[order], half[order]
        E = 2 * L
        row = np.zeros(V + 1, dtype=np.int64)
        np.add.at(row, src + 1, 1)
        row = np.cumsum(row)
        # reverse half-edge index
        pos = np.empty((L, 2), dtype=np.int64)
        pos[lid, half] = np.arange(E)
        rev = pos[lid, 1 - half]
        ov = np.zeros(V, dtype=np.uint8)
        if overloaded is not None:
            for i in overloaded:
                ov[r[i]] = 1
        return Csr(
            V,
            row.astype(np.uint32),
            dst.astype(np.uint32),
            met,
            lid.astype(np.uint32),
            rev.astype(np.uint32),
            ov,
            L,
        )

    def adj_dbs(self, area=T.kDefaultArea, overloaded=()):
        """thrift AdjacencyDatabases (one per node, creation order)."""
        per = [[] for _ in self.names]
        for k, (a, b, mab, mba) in enumerate(self.links):
            if self.ifnames:
                ia, ib = self.ifnames[k]
            else:
                ia, ib = f"if_{a}_{b}_{k}", f"if_{b}_{a}_{k}"
            la, lb = self.labels[k] if self.labels else (0, 0)
            na, nb = self.names[a], self.names[b]
            per[a].append(
                T.createThriftAdjacency(
                    nb, ia, _v6(b), _v4(b), int(mab), la, False, 100, 10000, 1, ib
                )
            )
            per[b].append(
                T.createThriftAdjacency(
                    na, ib, _v6(a), _v4(a), int(mba), lb, False, 100, 10000, 1, ia
                )
            )
        ov = set(overloaded)
        return [
            T.createAdjDb(
                n,
                per[i],
                self.node_labels[i] if self.node_labels else 0,
                i in ov,
                area,
            )
            for i, n in enumerate(self.names)
        ]

    def prefix_dbs(self, area=T.kDefaultArea, fwd_type=0, fwd_algo=0):
        out = []
        for i, n in enumerate(self.names):
            p = T.toIpPrefix(f"fc00:{i >> 16:02x}::{i & 0xffff:02x}/128")
            out.append(
                T.createPrefixDb(
                    n,
                    [T.createPrefixEntry(p, forwardingType=fwd_type, forwardingAlgorithm=fwd_algo)],
                    area,
                )
            )
        return out


def _v6(i):
    return f"fe80:{i >> 16:02x}::{i & 0xffff:02x}"


def _v4(i):
    return f"10.{(i >> 16) & 0xff}.{(i >> 8) & 0xff}.{i & 0xff}"


# ------------------------------------------------------------------- grid


def grid(n):
    names = [f"{i}" for i in range(n * n)]
    links, ifn, labels = [], [], []
    for r in range(n):
        for c in range(n):
            a = r * n + c
            for b in ([a + 1] if c + 1 < n else []) + ([a + n] if r + 1 < n else []):
                links.append((a, b, 1, 1))
                ifn.append((f"if_{a}_{b}", f"if_{b}_{a}"))
                labels.append((100001 + b, 100001 + a))
    return Topology(names, links, ifn, labels, node_labels=[0] * (n * n))


# ----------------------------------------------------------------- fabric


def fabric(num_sws=10000, planes=8, ssw_per_plane=36, rsw_per_pod=48):
    """Corrected DecisionBenchmark fabric: V = 9,976, L = 116,256 at 10k."""
    fsw_per_pod = planes
    pods = (num_sws - planes * ssw_per_plane) // (fsw_per_pod + rsw_per_pod)
    names, idx = [], {}

    def node(marker, pod, sw):
        key = (marker, pod, sw)
        if key not in idx:
            idx[key] = len(names)
            names.append(f"{marker}-{pod}-{sw}")
        return idx[key]

    links, ifn, labels = [], [], []

    def link(a, b):
        links.append((a, b, 1, 1))
        ifn.append((f"if_{names[a]}_{names[b]}", f"if_{names[b]}_{names[a]}"))
        labels.append((0, 0))

    for p in range(planes):
        for s in range(ssw_per_plane):
            node(1, p, s)
    for pod in range(pods):
        for f in range(fsw_per_pod):
            node(2, pod, f)
        for r in range(rsw_per_pod):
            node(3, pod, r)
    for p in range(planes):
        for s in range(ssw_per_plane):
            for pod in range(pods):
                link(node(1, p, s), node(2, pod, p))
    for pod in range(pods):
        for f in range(fsw_per_pod):
            for r in range(rsw_per_pod):
                link(node(2, pod, f), node(3, pod, r))
    rank = {n: i for i, n in enumerate(sorted(names))}
    node_labels = [rank[n] + 1 for n in names]  # nodeLabel = rank+1
    return Topology(names, links, ifn, labels, node_labels)


# -------------------------------------------------------------------- WAN


class MT19937_64:
    """std::mt19937_64 (the C++ standard engine, default parameters)."""

    def __init__(self, seed):
        self.mt = [0] * 312
        self.mt[0] = seed & 0xFFFFFFFFFFFFFFFF
        for i in range(1, 312):
            self.mt[i] = (
                6364136223846793005 * (self.mt[i - 1] ^ (self.mt[i - 1] >> 62)) + i
            ) & 0xFFFFFFFFFFFFFFFF
        self.idx = 312

    def _twist(self):
        mt = self.mt
        for i in range(312):
            x = (mt[i] & 0xFFFFFFFF80000000) | (mt[(i + 1) % 312] & 0x7FFFFFFF)
            xa = x >> 1
            if x & 1:
                xa ^= 0xB5026F5AA96619E9
            mt[i] = mt[(i + 156) % 312] ^ xa
        self.idx = 0

    def __call__(self):
        if self.idx >= 312:
            self._twist()
        y = self.mt[self.idx]
        self.idx += 1
        y ^= (y >> 29) & 0x5555555555555555
        y ^= (y << 17) & 0x71D67FFFEDA60000
        y ^= (y << 37) & 0xFFF7EEE000000000
        y ^= y >> 43
        return y & 0xFFFFFFFFFFFFFFFF


def wan(V=100000, L=1000000, seed=12345, wmax=1000):
    """backbone (rng()%i, i), then random pairs until L
    distinct links, then one weight per link in ascending (a, b) order."""
    rng = MT19937_64(seed)
    edges = set()
    for i in range(1, V):
        edges.add((rng() % i, i))
    while len(edges) < L:
        a = rng() % V
        b = rng() % V
        if a == b:
            continue
        edges.add((min(a, b), max(a, b)))
    links = []
    for (a, b) in sorted(edges):
        w = 1 + rng() % wmax
        links.append((a, b, w, w))
    names = [f"n{i}" for i in range(V)]
    ifn = [(f"if_{a}_{b}", f"if_{b}_{a}") for (a, b, _, _) in links]
    return Topology(names, links, ifn, None, None)


# ------------------------------------------------- config 5 (what-if, 2 areas)

WHATIF_BORDER = "2-0-0"


def wan_border(V=10000, L=100000, border=WHATIF_BORDER):
    """The WAN of wan(V, L) with node n0 renamed to the border node, so that
    one node is present in both what-if areas (BASELINE configs[4]: "multi-area
    LinkState", the border-node setup of DecisionTest.cpp:4503-4545)."""
    t = wan(V, L)
    t.names[0] = border
    return t


def whatif_two_area(per_area=4096, seed=7):
    """BASELINE configs[4]: area "A" = fabric(10000), area "B" = WAN-10k (100k
    links) sharing the border node "2-0-0"; `per_area` links of each area
    sampled without replacement (numpy default_rng(seed), area A first).
    Returns [(area, topology, link creation ids)]."""
    rng = np.random.default_rng(seed)
    out = []
    for area, topo in (("A", fabric(10000)), ("B", wan_border(10000, 100000))):
        links = rng.choice(len(topo.links), per_area, replace=False).astype(np.int64)
        out.append((area, topo, links))
    return out
