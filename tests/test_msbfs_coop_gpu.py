"""Cooperative MS-BFS (spf_msbfs_coop_kernel): a batch's 64 sources split
over P workgroups that meet at a counter barrier per BFS level.  It runs when
a query has few batches (a rank's block of a sharded all-sources table,
DESIGN §7); its distance rows and next-hop masks must equal the
one-workgroup kernel's (OPENR_MS_COOP=0) and the DijkstraQ replay's."""

import random

import numpy as np
import pytest

from openr_amd import abi
from openr_amd import topologies as T
from tests.test_abi_gpu import check_query, random_links

pytestmark = pytest.mark.gpu


def _rows(g, sources, monkeypatch, coop):
    monkeypatch.setenv("OPENR_MS_COOP", "1" if coop else "0")
    q = g.query(sources, abi.SPF_F_NEXTHOPS).run()
    ks = q.kernels()
    d = np.stack([q.dist(i) for i in range(len(sources))])
    m = [q.nexthops(i) for i in range(len(sources))]
    q.close()
    return ks, d, m


@pytest.mark.parametrize("case", ["fabric", "random"])
def test_coop_rows_equal_plain(gpu_ready, monkeypatch, case):
    if case == "fabric":
        csr = T.fabric(2300).csr()  # 8 planes, V ~ 2.3k: three 1,024-node slots
        V = csr.num_nodes
        sources = list(range(V // 3, V // 3 + 150))
    else:
        rng = random.Random(11)
        V = 3000
        links = random_links(rng, V, 9000, wmin=1, wmax=1, asym=False)
        ov = [1 if rng.random() < 0.02 else 0 for _ in range(V)]
        csr = abi.Csr.from_links(V, links, ov)
        sources = rng.sample(range(V), 100)
    g = abi.Graph(csr)
    ks1, d1, m1 = _rows(g, sources, monkeypatch, True)
    ks0, d0, m0 = _rows(g, sources, monkeypatch, False)
    assert "spf_msbfs_coop_kernel" in ks1, ks1
    assert "spf_msbfs_coop_kernel" not in ks0, ks0
    assert np.array_equal(d1, d0)
    for a, b in zip(m1, m0):
        assert np.array_equal(a, b)
    # and against the replay, on a sample of rows
    monkeypatch.setenv("OPENR_MS_COOP", "1")
    q = g.query(sources, abi.SPF_F_NEXTHOPS).run()
    check_query(csr, q, sources, True, rows=set(range(0, len(sources), 17)))
    q.close()
    g.close()
