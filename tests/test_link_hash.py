"""Link::hash — folly's std::hash<pair<pair<string,string>,pair<string,string>>>
over SpookyHashV2 string hashes (openr_amd/csrc/host/FollyHash.h) — agrees
between the product and the oracle's independent restatement for names of
every length class of SpookyHash (short remainders 0..15, >= 16-byte chunks,
the >= 192-byte long path).  The formula itself is pinned by the reference's
hash-dependent parallel-link goldens (tests/known_answers*.py)."""

import random

import pytest


@pytest.fixture(scope="module")
def mods():
    from oracle import build

    build.build()
    from oracle import _oracle_ref as O
    import openr_amd._openr_spf as E

    return E, O


def test_link_hash_product_equals_oracle(mods):
    E, O = mods
    rng = random.Random(3)
    lengths = list(range(0, 40)) + [63, 64, 65, 95, 96, 97, 191, 192, 193, 287, 288, 300, 500]
    for ln in lengths:
        for _ in range(3):
            mk = lambda n: "".join(chr(rng.randrange(33, 127)) for _ in range(n))  # noqa: E731
            n1, i1, n2, i2 = mk(ln), mk(rng.randrange(0, 12)), mk(rng.randrange(0, 30)), mk(ln)
            e = E.Link("0", n1, i1, n2, i2).hash
            o = O.Link("0", n1, i1, n2, i2).__hash__()
            assert e == o, (ln, n1, i1, n2, i2)
