"""Fib's best-next-hop filters, getBestNextHopsUnicast / getBestNextHopsMpls
(Util.cpp:473-531), pinned by the reference's own known
answers (UtilTest.cpp:26-98 fixtures, :592-660 expectations) on both the
product (openr_amd/csrc/host/Util.h) and the oracle's restatement; then the
two agree on random next-hop lists."""

import random

import pytest

from openr_amd import thrift as T

MAC = T.MplsActionCode


def _nh(addr, ifname, metric, action=None, swap=None):
    act = None if action is None else T.createMplsAction(action, swap)
    return T.createNextHop(T.toBinaryAddress(addr), ifname, metric, act)


# UtilTest.cpp:26-98 (area = the default area, as createNextHop's default)
P121 = _nh("fe80::2", "iface_1_2_1", 1)
P122 = _nh("fe80::2", "iface_1_2_2", 2)
P123 = _nh("fe80::2", "iface_1_2_3", 3)
P131 = _nh("fe80::3", "iface_1_3_1", 1)
P132 = _nh("fe80::3", "iface_1_3_2", 2)
S121 = _nh("fe80::2", "iface_1_2_1", 1, MAC.SWAP, 1)
S122 = _nh("fe80::2", "iface_1_2_2", 2, MAC.SWAP, 1)
S123 = _nh("fe80::2", "iface_1_2_3", 3, MAC.SWAP, 1)
S131 = _nh("fe80::3", "iface_1_3_1", 1, MAC.SWAP, 1)
S132 = _nh("fe80::3", "iface_1_3_2", 2, MAC.SWAP, 1)
H121 = _nh("fe80::2", "iface_1_2_1", 1, MAC.PHP)
H122 = _nh("fe80::2", "iface_1_2_2", 2, MAC.PHP)
H123 = _nh("fe80::2", "iface_1_2_3", 3, MAC.PHP)
H131 = _nh("fe80::3", "iface_1_3_1", 1, MAC.PHP)
H132 = _nh("fe80::3", "iface_1_3_2", 2, MAC.PHP)
POP122 = _nh("fe80::2", "iface_1_2_1", 2, MAC.POP_AND_LOOKUP)


def _updated_122():
    nh = _nh("fe80::2", "iface_1_2_2", 2)
    nh.useNonShortestRoute = True
    return nh


# (function, input, expected) — UtilTest.cpp:592-660
UNICAST = [
    ([P121, P122], [P121]),
    ([P121, P122, P123, P131], [P121, P131]),
    ([P121, _updated_122(), P123, P131], [P121, _updated_122(), P131]),
]
MPLS = [
    ([POP122], [POP122]),
    ([S121, S122, S123, S131, S132], [S121, S131]),
    ([H121, H122, H123, H131, H132], [H121, H131]),
    ([S121, H122, S131, H132], [S121, S131]),
    ([H121, S122, H131, S132], [H121, H131]),
    ([S121, H131], [H131]),
]


@pytest.fixture(scope="module")
def mods():
    from oracle import build

    build.build()
    from oracle import _oracle_ref as O
    import openr_amd._openr_spf as E

    return E, O


@pytest.mark.parametrize("case", range(len(UNICAST)))
def test_best_nexthops_unicast_known_answers(mods, case):
    nhs, want = UNICAST[case]
    for m in mods:
        assert m.getBestNextHopsUnicast(nhs) == [n.key() for n in want]


@pytest.mark.parametrize("case", range(len(MPLS)))
def test_best_nexthops_mpls_known_answers(mods, case):
    nhs, want = MPLS[case]
    for m in mods:
        assert m.getBestNextHopsMpls(nhs) == [n.key() for n in want]


def test_best_nexthops_mpls_rejects_push(mods):
    push = _nh("fe80::4", "iface_1_4_1", 1)
    push.mplsAction = T.createMplsAction(MAC.PUSH, None, [5])
    for m in mods:
        with pytest.raises(Exception):
            m.getBestNextHopsMpls([S121, push])


def test_best_nexthops_random_product_equals_oracle(mods):
    E, O = mods
    rng = random.Random(11)
    for _ in range(300):
        n = rng.randrange(0, 7)
        nhs, mp = [], []
        for i in range(n):
            nh = _nh(f"fe80::{rng.randrange(1, 4)}", f"if_{i}", rng.randrange(1, 4))
            nh.useNonShortestRoute = rng.random() < 0.2
            nhs.append(nh)
            mp.append(_nh(f"fe80::{rng.randrange(1, 4)}", f"if_{i}", rng.randrange(1, 4),
                          rng.choice([MAC.SWAP, MAC.PHP]), 7))
        assert E.getBestNextHopsUnicast(nhs) == O.getBestNextHopsUnicast(nhs)
        assert E.getBestNextHopsMpls(mp) == O.getBestNextHopsMpls(mp)
