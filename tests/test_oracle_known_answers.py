"""The CPU oracle reproduces the reference's own known answers
(LinkStateTest.cpp / DecisionTest.cpp, see tests/known_answers.py).
This pins the oracle before it is used to check the MI355X engine."""

import pytest

from tests import known_answers as KA
from tests import known_answers_more as KB

SCENARIOS = [getattr(M, n) for M in (KA, KB) for n in dir(M) if n.startswith("sc_")]


@pytest.fixture(scope="module")
def oracle_mod():
    from oracle import build

    build.build()
    from oracle import _oracle_ref

    return _oracle_ref


@pytest.mark.parametrize("scenario", SCENARIOS, ids=lambda f: f.__name__)
def test_oracle_known_answer(oracle_mod, scenario):
    oracle_mod.reset_counters()
    scenario(oracle_mod)
