"""2-bit neighbour rows of the v2 next-hop pass (round 6, DESIGN.md §3
"Next-hop pass v2, 2-bit neighbour rows").

spf_lvl_trit_kernel writes every MS-BFS level row as level mod 3 (3 =
unreached); an item of spf_nh_levels_v2_kernel whose sources are all transit
reads its neighbours' rows in that form.  The masks and distance rows must be
bit-identical to the byte rows' (OPENR_NL_TRIT=0) and to the literal
DijkstraQ replay (oracle/spf_py.py), including:
  * drained sources (their items fall back to byte rows at run time) and
    drained neighbours (next hop only to themselves);
  * shared-neighbour groups with one drained member;
  * the transit bits flipped between runs of the SAME query
    (spf_graph_set_transit: the kernel re-reads them every run);
  * a ragged last chunk, parallel links, BFS levels past 3 (mod 3 wraps).
"""

import random

import numpy as np
import pytest

from openr_amd import abi
from oracle import spf_py
from tests.test_abi_gpu import check_query, random_links

pytestmark = pytest.mark.gpu


def _pair(g, srcs, flags, monkeypatch):
    monkeypatch.setenv("OPENR_NL_TRIT", "1")
    a = g.query(srcs, flags)
    monkeypatch.setenv("OPENR_NL_TRIT", "0")
    b = g.query(srcs, flags)
    return a, b


def _same(a, b, V):
    a.run()
    b.run()
    assert a.kernel == "msbfs+levels" and b.kernel == "msbfs+levels"
    assert "spf_lvl_trit_kernel" in a.kernels(), a.kernels()
    assert "spf_lvl_trit_kernel" not in b.kernels()
    for i in range(V):
        assert (a.dist(i) == b.dist(i)).all(), i
    ma, mb = a.fetch_nexthops(0, V), b.fetch_nexthops(0, V)
    if not (ma == mb).all():
        bad = int(np.flatnonzero(ma != mb)[0])
        pytest.fail(f"mask word {bad} differs: {ma[bad]:#x} vs {mb[bad]:#x}")


@pytest.mark.parametrize("seed", [11, 12])
def test_trit_rows_random_uniform(gpu_ready, seed, monkeypatch):
    rng = random.Random(seed)
    V = 1999  # ragged last chunk
    links = random_links(rng, V, 6000, wmin=1, wmax=1, parallel=0.03)
    ov = np.zeros(V, dtype=np.uint8)
    ov[rng.sample(range(V), V // 30)] = 1
    csr = abi.Csr.from_links(V, links, overloaded=ov)
    g = abi.Graph(csr)
    srcs = np.arange(V, dtype=np.uint32)
    a, b = _pair(g, srcs, abi.SPF_F_NEXTHOPS | abi.SPF_F_UNIT_METRIC, monkeypatch)
    _same(a, b, V)
    drained = [int(x) for x in np.flatnonzero(ov)[:3]]
    check_query(csr, a, [int(s) for s in srcs], False, rows=set([0, 5, V - 1] + drained))


def test_trit_rows_fabric_groups_and_transit_flips(gpu_ready, monkeypatch):
    """Fabric (29 pods): RSW groups share their FSWs; drain an RSW (its group
    falls back), an FSW (a drained neighbour of every group of its pod) and
    an SSW, run, undrain, rerun the same queries."""
    from openr_amd import topologies as TP

    topo = TP.fabric(2000)
    csr = topo.csr()
    V = csr.num_nodes
    g = abi.Graph(csr)
    srcs = np.arange(V, dtype=np.uint32)
    a, b = _pair(g, srcs, abi.SPF_F_NEXTHOPS, monkeypatch)
    _same(a, b, V)
    names = topo.names
    pick = [next(i for i, n in enumerate(names) if n.startswith(p)) for p in ("3-", "2-", "1-")]
    csr_d = topo.csr(overloaded=pick)  # (names-order indices; the CSR's ids are name ranks)
    ids = [int(x) for x in np.flatnonzero(csr_d.overloaded)]
    assert len(ids) == 3
    g.set_transit(csr_d.overloaded)
    _same(a, b, V)
    check_query(csr_d, a, [int(s) for s in srcs], True, rows=set(ids) | {0, V - 1})
    g.set_transit(np.zeros(V, dtype=np.uint8))
    _same(a, b, V)
    check_query(csr, a, [int(s) for s in srcs], True, rows={ids[0], ids[1], V // 2})


def test_trit_rows_deep_levels(gpu_ready, monkeypatch):
    """Levels up to ~200 (the mod-3 code wraps many times), a ring with
    chords: every source's masks equal the byte pass's and the replay's."""
    V = 400
    links = [(i, (i + 1) % V, 1, 1) for i in range(V)]
    links += [(i, (i + 37) % V, 1, 1) for i in range(0, V, 50)]
    csr = abi.Csr.from_links(V, links)
    g = abi.Graph(csr)
    srcs = np.arange(V, dtype=np.uint32)
    a, b = _pair(g, srcs, abi.SPF_F_NEXTHOPS | abi.SPF_F_UNIT_METRIC, monkeypatch)
    _same(a, b, V)
    check_query(csr, a, [int(s) for s in srcs], False, rows={0, 1, 199, 399})


# ---- the shallow one-add compare (round 6, nl_s_cmp8): on by default when
# every level is below 127 (MsBfsArgs::flags bit 1); OPENR_NL_SHALLOW=0 keeps
# the exact zero-byte test.  Masks and rows must be identical either way,
# and a batch with levels in [127, 254] must take the exact test.


def _pair_env(g, srcs, flags, monkeypatch, name):
    monkeypatch.setenv(name, "1")
    a = g.query(srcs, flags)
    monkeypatch.setenv(name, "0")
    b = g.query(srcs, flags)
    monkeypatch.delenv(name)
    return a, b


def _equal_rows(a, b, V):
    a.run()
    b.run()
    for i in range(V):
        assert (a.dist(i) == b.dist(i)).all(), i
    ma, mb = a.fetch_nexthops(0, V), b.fetch_nexthops(0, V)
    if not (ma == mb).all():
        bad = int(np.flatnonzero(ma != mb)[0])
        pytest.fail(f"mask word {bad} differs: {ma[bad]:#x} vs {mb[bad]:#x}")


@pytest.mark.parametrize("seed", [21, 22])
def test_shallow_compare_random_with_drains(gpu_ready, seed, monkeypatch):
    rng = random.Random(seed)
    V = 2111
    links = random_links(rng, V, 7000, wmin=1, wmax=1, parallel=0.03)
    links += [(5, v, 1, 1) for v in range(40, 160)]  # a 2-word source
    ov = np.zeros(V, dtype=np.uint8)
    ov[rng.sample(range(V), V // 25)] = 1
    csr = abi.Csr.from_links(V, links, overloaded=ov)
    g = abi.Graph(csr)
    srcs = np.arange(V, dtype=np.uint32)
    a, b = _pair_env(g, srcs, abi.SPF_F_NEXTHOPS | abi.SPF_F_UNIT_METRIC, monkeypatch,
                     "OPENR_NL_SHALLOW")
    _equal_rows(a, b, V)
    assert "spf_nh_levels_v2_kernel" in a.kernels()
    drained = [int(x) for x in np.flatnonzero(ov)[:3]]
    check_query(csr, a, [int(s) for s in srcs], False, rows=set([0, 5, V - 1] + drained))


def test_shallow_compare_fabric_groups(gpu_ready, monkeypatch):
    """RSW groups and FSW / SSW solo items with a drained FSW and RSW."""
    from openr_amd import topologies as TP

    topo = TP.fabric(2000)
    names = topo.names
    pick = [next(i for i, n in enumerate(names) if n.startswith(p)) for p in ("3-", "2-")]
    csr = topo.csr(overloaded=pick)
    V = csr.num_nodes
    g = abi.Graph(csr)
    srcs = np.arange(V, dtype=np.uint32)
    a, b = _pair_env(g, srcs, abi.SPF_F_NEXTHOPS, monkeypatch, "OPENR_NL_SHALLOW")
    _equal_rows(a, b, V)
    ids = [int(x) for x in np.flatnonzero(csr.overloaded)]
    check_query(csr, a, [int(s) for s in srcs], True, rows=set(ids) | {0, V // 3, V - 1})


def test_levels_127_to_254_take_the_exact_compare(gpu_ready, monkeypatch):
    """A random core with a 180-node chain: levels up to ~190 set the
    kMsShallowLevel flag, so the v2 pass keeps the exact test; rows equal the
    per-node kernel's (OPENR_NL_SWAR=0) and the replay."""
    rng = random.Random(9)
    V = 300
    links = random_links(rng, 120, 400, wmin=1, wmax=1, parallel=0.0)
    links += [(119 + i, 120 + i, 1, 1) for i in range(180)]
    csr = abi.Csr.from_links(V, links)
    g = abi.Graph(csr)
    srcs = np.arange(V, dtype=np.uint32)
    flags = abi.SPF_F_NEXTHOPS | abi.SPF_F_UNIT_METRIC
    a, b = _pair_env(g, srcs, flags, monkeypatch, "OPENR_NL_SWAR")
    a.run()
    assert "spf_nh_levels_v2_kernel" in a.kernels()
    assert max(int(a.dist(0)[v]) for v in range(V)) >= 127
    _equal_rows(a, b, V)
    check_query(csr, a, [int(s) for s in srcs], False, rows={0, 119, 200, 299})
