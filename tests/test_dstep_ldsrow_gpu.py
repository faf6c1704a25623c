"""GPU parity of the LDS-resident delta-stepping plan (spf_dlds_kernel, kernel
name "dstep-ldsrow": distance rows held in LDS as 12-bit fields) against the
flat CPU oracle (oracle/csr_spf.h, LinkState.cpp:806-880) and against the
HBM-row delta-stepping kernel (OPENR_SPF_DSTEP_LDSROW=0) on the same batch.

Covers: drained nodes (also as sources), parallel links, asymmetric metrics,
unreachable components, duplicate sources, bucket widths from 1 to 2,048,
sources whose values leave the 12-bit range (flagged by the kernel and
recomputed by the HBM-row pass: a long chain of 1,000-metric links), and the
100k WAN of config 3 (reference checksum of row n0, the 32 golden rows).
"""

import hashlib
import json
import os
import random

import numpy as np
import pytest

from openr_amd import abi

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
UNREACH32 = np.uint32(0xFFFFFFFF)


def _oracle_rows(csr, srcs):
    from oracle import build as OB

    OB.build()
    from oracle import _oracle_ref as O

    rows = O.csr_spf_rows(csr.row_ptr, csr.col, csr.metric.astype(np.uint64), csr.link_id,
                          csr.overloaded, np.asarray(srcs, dtype=np.uint32), True, 8)
    return np.where(rows == np.uint64(2**64 - 1), np.uint64(0xFFFFFFFF), rows).astype(np.uint32)


def _rows(q, n, V):
    out = np.empty((n, V), dtype=np.uint32)
    q.fetch_rows(0, n, out.ctypes.data, V * 4, on_device=False)
    return out


def _graph(seed, V, L, wmax, drained=0.01, parallel=0.02, islands=0):
    rng = random.Random(seed)
    links = []
    core = V - islands
    for v in range(1, core):
        links.append((rng.randrange(v), v, rng.randint(1, wmax), rng.randint(1, wmax)))
    while len(links) < L:
        a, b = rng.randrange(core), rng.randrange(core)
        if a == b:
            continue
        links.append((a, b, rng.randint(1, wmax), rng.randint(1, wmax)))
        if rng.random() < parallel:
            links.append((a, b, rng.randint(1, wmax), rng.randint(1, wmax)))
    # an island of `islands` nodes (a ring) no core node reaches
    for i in range(islands):
        links.append((core + i, core + (i + 1) % islands, rng.randint(1, wmax), rng.randint(1, wmax)))
    ov = np.zeros(V, dtype=np.uint8)
    ov[rng.sample(range(V), int(V * drained))] = 1
    return abi.Csr.from_links(V, links, overloaded=ov), ov


@pytest.mark.parametrize("seed,wmax", [(51, 300), (52, 1000), (53, 4000)])
def test_ldsrow_vs_oracle_and_hbm_rows(gpu_ready, seed, wmax, monkeypatch):
    V = 60000
    csr, ov = _graph(seed, V, 210000, wmax, islands=40)
    g = abi.Graph(csr)
    rng = random.Random(seed)
    drained = [int(v) for v in np.flatnonzero(ov)[:3]]
    srcs = [rng.randrange(V) for _ in range(300)] + drained + [5, 5, V - 1, V - 20]
    want = _oracle_rows(csr, srcs)
    monkeypatch.setenv("OPENR_SPF_DSTEP_LDSROW", "0")
    ref = g.query(srcs, 0).run()
    assert ref.kernel == "dstep"
    assert (_rows(ref, len(srcs), V) == want).all()
    ref.close()
    monkeypatch.delenv("OPENR_SPF_DSTEP_LDSROW")
    for shift in (None, "0", "3", "7", "11"):
        if shift is None:
            monkeypatch.delenv("OPENR_SPF_DSTEP_LSHIFT", raising=False)
        else:
            monkeypatch.setenv("OPENR_SPF_DSTEP_LSHIFT", shift)
        q = g.query(srcs, 0).run()
        # metrics above 4,094 cannot be a 12-bit field: the HBM-row plan
        assert q.kernel == ("dstep-ldsrow" if wmax <= 4094 else "dstep")
        got = _rows(q, len(srcs), V)
        bad = np.flatnonzero((got != want).any(axis=1))
        assert len(bad) == 0, (shift, bad[:5].tolist())
        q.close()
    g.close()


def test_ldsrow_overflow_rows_recomputed(gpu_ready):
    """A core whose distances fit 12 bits plus a chain of 1,000-metric links
    whose far nodes do not: sources that reach the chain are flagged and
    recomputed by the HBM-row pass, the rest stay on the LDS rows."""
    rng = random.Random(61)
    core, chain = 50000, 30
    links = []
    for v in range(1, core):
        links.append((rng.randrange(v), v, rng.randint(1, 50), rng.randint(1, 50)))
    while len(links) < 160000:
        a, b = rng.randrange(core), rng.randrange(core)
        if a != b:
            links.append((a, b, rng.randint(1, 50), rng.randint(1, 50)))
    # chain core+0 .. core+chain-1, hung off node 7: the core reaches it only
    # through node 7's link
    links.append((7, core, 1000, 1000))
    for i in range(chain - 1):
        links.append((core + i, core + i + 1, 1000, 1000))
    V = core + chain
    ov = np.zeros(V, dtype=np.uint8)
    ov[core + chain // 2] = 1  # a drained chain node: the far half is reached only from itself
    csr = abi.Csr.from_links(V, links, overloaded=ov)
    g = abi.Graph(csr)
    srcs = [0, 7, 123, core, core + 5, core + chain // 2, V - 1] + [rng.randrange(core) for _ in range(60)]
    q = g.query(srcs, 0).run()
    assert q.kernel == "dstep-ldsrow"
    want = _oracle_rows(csr, srcs)
    got = _rows(q, len(srcs), V)
    assert (got.astype(np.uint64)[want != UNREACH32] > 4094).any()  # the overflow path ran
    bad = np.flatnonzero((got != want).any(axis=1))
    assert len(bad) == 0, bad[:5].tolist()
    g.close()


def test_ldsrow_wan100k_anchor_and_golden_rows(gpu_ready):
    from openr_amd import topologies as TP

    anchor = [a for a in json.load(open(os.path.join(GOLD, "wan_anchors.json")))["anchors"]
              if a["V"] == 100000 and a["S"] == 1][0]
    gold = json.load(open(os.path.join(GOLD, "wan100k_rows.json")))["rows"]
    csr = TP.wan(100000, 1000000).csr()
    V = csr.num_nodes
    g = abi.Graph(csr)
    srcs = [r["src"] for r in gold]
    assert srcs[0] == 0
    q = g.query(srcs, 0).run()
    assert q.kernel == "dstep-ldsrow"
    got = _rows(q, len(srcs), V)
    assert int(got[0].astype(np.int64).sum()) == anchor["sum_dist"]
    for r, row in zip(gold, got):
        assert hashlib.sha256(row.tobytes()).hexdigest() == r["sha256"], r["src"]
    g.close()
