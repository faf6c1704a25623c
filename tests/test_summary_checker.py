"""The checker that turns an engine batch into the config-2 golden's four
numbers (oracle rows_summary, tests/golden/summary.py summaries_full) is
itself checked here on the CPU: on rows and masks built from the literal
DijkstraQ replay (oracle/spf_py.py) it must reproduce oracle/csr_spf.h's
summaries exactly, and agree with the pure-numpy path."""

import numpy as np

from tests.golden.summary import summaries_from_rows, summaries_full


def _grid_csr(n, seed):
    from openr_amd import abi

    rng = np.random.default_rng(seed)
    links = []
    for r in range(n):
        for c in range(n):
            v = r * n + c
            if c + 1 < n:
                links.append((v, v + 1, int(rng.integers(1, 4)), int(rng.integers(1, 4))))
            if r + 1 < n:
                links.append((v, v + n, int(rng.integers(1, 4)), int(rng.integers(1, 4))))
    ov = np.zeros(n * n, dtype=np.uint8)
    ov[rng.choice(n * n, 3, replace=False)] = 1
    return abi.Csr.from_links(n * n, links, ov)


def test_rows_summary_matches_csr_spf():
    from oracle import build as OB

    OB.build()
    from oracle import _oracle_ref as O
    from oracle import spf_py

    csr = _grid_csr(7, 3)
    V = csr.num_nodes
    sources = np.arange(V, dtype=np.uint32)
    rows = np.full((V, V), 0xFFFFFFFF, dtype=np.uint32)
    nbrs, words, masks = [], [], []
    for s in range(V):
        nb = sorted(set(int(x) for x in csr.col[csr.row_ptr[s]:csr.row_ptr[s + 1]]))
        bit = {x: i for i, x in enumerate(nb)}
        W = max(1, (len(nb) + 63) // 64)
        m = np.zeros((V, W), dtype=np.uint64)
        for v, (d, nh, _, _) in spf_py.run_spf(csr, s, True).items():
            rows[s, v] = d
            for h in nh:
                m[v, bit[h] // 64] |= np.uint64(1) << np.uint64(bit[h] % 64)
        nbrs.append(nb)
        words.append(W)
        masks.append(m.ravel())
    masks = np.concatenate(masks)
    want = O.csr_spf_summary(csr.row_ptr, csr.col, csr.metric.astype(np.uint64), csr.link_id,
                             csr.overloaded, sources, None, None, True, True, 2)
    full = summaries_full(rows, masks, words, nbrs, threads=3)
    assert (full == want).all()
    slow = summaries_from_rows(rows, masks, words, nbrs, range(V))
    assert (slow == want).all()
