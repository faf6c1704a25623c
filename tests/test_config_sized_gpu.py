"""BASELINE configs 2, 3 and 5 at their real sizes and production plans,
against goldens made on the CPU (tests/golden/make_golden.py: oracle/csr_spf.h,
itself cross-checked there against the reference-style oracle and the literal
DijkstraQ replay) and against size-independent properties.

  config 2  all 9,976 fabric sources in ONE batch (the msbfs+levels plan):
            per-source (reached, sum of distances, next-hop pairs) AND the
            order-free mix of every (node, distance) and (node, next hop) pair
            for EVERY source, the reference-form digest of the 8
            fabric_sampled.json sources.
  config 3  the 100k-node / 1M-link WAN, all 100,000 sources through
            ShardedAllSources (world 1, LDS-resident delta-stepping): the
            reference's own checksum of row n0, EVERY row's (reached, sum,
            mix) against the 100,000-source golden, 32 sampled rows by sha256, and
            for those rows the Bellman conditions (no edge relaxes, every
            reached node has a tight in-edge) plus D[s][t] == D[t][s].
  config 5  8,192 single-link-failure SPFs from the border node 2-0-0 over two
            areas (fabric + WAN-10k): every query's summary through the C ABI,
            and sampled queries' reference-form SpfResults through the
            multi-area LinkState (LinkState::runSpfBatch).
"""

import hashlib
import json
import os

import numpy as np
import pytest

from tests.golden.make_golden import FABRIC_SOURCES, digest, spf_canon
from tests.golden.summary import summaries_from_rows, summaries_full

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _batch_summaries(q, g, sources, mix_rows):
    """mix_rows=None: every query's mix (oracle rows_summary, threaded)."""
    n = len(sources)
    V = g.V
    rows = np.empty((n, V), dtype=np.uint32)
    q.fetch_rows(0, n, rows.ctypes.data, V * 4, on_device=False)
    words = [q.nh_words(i) for i in range(n)]
    masks = q.fetch_nexthops(0, n)
    nbr_cache = {}
    nbrs = []
    for s in sources:
        s = int(s)
        if s not in nbr_cache:
            nbr_cache[s] = g.nbrs(s)
        nbrs.append(nbr_cache[s])
    if mix_rows is None:
        return summaries_full(rows, masks, words, nbrs)
    return summaries_from_rows(rows, masks, words, nbrs, mix_rows)


def _check_summary(got, want, mix_rows, what):
    bad = np.nonzero((got[:, :3] != want[:, :3]).any(axis=1))[0]
    assert len(bad) == 0, f"{what}: {len(bad)} queries differ, first {bad[:5].tolist()}"
    if mix_rows is None:
        mix_rows = range(len(want))
    mr = np.asarray(sorted(mix_rows), dtype=np.int64)
    bad = mr[got[mr, 3] != want[mr, 3]]
    assert len(bad) == 0, f"{what}: mix differs for queries {bad[:5].tolist()}"


def test_config2_fabric_all_sources_msbfs(gpu_ready):
    from openr_amd import abi
    from openr_amd import topologies as TP

    want = np.load(os.path.join(GOLD, "fabric_allsources.npz"))["summary"]
    topo = TP.fabric(10000)
    csr = topo.csr()
    V = csr.num_nodes
    g = abi.Graph(csr)
    sources = np.arange(V, dtype=np.uint32)
    q = g.query(sources, abi.SPF_F_NEXTHOPS)
    assert q.kernel == "msbfs+levels"  # the production plan of config 2
    q.run()
    _, names_by_rank = topo.rank()
    sampled_ids = [names_by_rank.index(s) for s in FABRIC_SOURCES]
    got = _batch_summaries(q, g, sources, None)  # every source's full mix
    _check_summary(got, want, None, "fabric all-sources")
    gold = json.load(open(os.path.join(GOLD, "fabric_sampled.json")))
    for src, sid in zip(FABRIC_SOURCES, sampled_ids):
        d = q.dist(sid)
        nh = q.nexthop_sets(sid, sid)
        c = {names_by_rank[v]: (int(d[v]), sorted(names_by_rank[h] for h in nh[v])) for v in nh}
        assert digest(c) == gold["spf"][src]["digest"], src
    q.close()
    g.close()


def test_config3_wan100k_all_sources_sharded(gpu_ready):
    import torch

    from openr_amd import allsources as AS
    from openr_amd import topologies as TP

    torch.cuda.set_device(0)
    gold = json.load(open(os.path.join(GOLD, "wan100k_rows.json")))["rows"]
    anchor = [a for a in json.load(open(os.path.join(GOLD, "wan_anchors.json")))["anchors"]
              if a["V"] == 100000 and a["S"] == 1][0]
    topo = TP.wan(100000, 1000000)
    csr = topo.csr()
    V = csr.num_nodes
    sas = AS.ShardedAllSources(csr, device=0, gather=False)
    # LDS-resident delta-stepping (12-bit rows), the config-3 plan
    assert sas.kernel == "dstep-ldsrow"
    sas.run()
    # the reference's runSpf checksum of source n0
    assert int(sas.row(0).astype(np.int64).sum()) == anchor["sum_dist"]
    # EVERY row against the 100,000-source golden (oracle/csr_spf.h,
    # tests/golden/make_wan_allsources.py): (reached, sum, mix) per source,
    # summarised on the device in 2,048-row slices
    from tests.golden.summary import dist_summaries_torch

    want = np.load(os.path.join(GOLD, "wan100k_allsources.npz"))["summary"]
    bad = []
    for lo in range(0, V, 2048):
        got = dist_summaries_torch(sas.table[lo:min(V, lo + 2048)])
        bad += (lo + np.flatnonzero((got != want[lo:lo + len(got)]).any(axis=1))).tolist()
    assert not bad, f"{len(bad)} of {V} WAN rows differ from the golden, first {bad[:5]}"
    row = csr.row_ptr.astype(np.int64)
    src_of_edge = np.repeat(np.arange(V, dtype=np.int64), np.diff(row))
    col = csr.col.astype(np.int64)
    w = csr.metric.astype(np.int64)
    rows = {}
    for r in gold:
        d = sas.row(r["src"])
        assert hashlib.sha256(d.tobytes()).hexdigest() == r["sha256"], r["src"]
        rows[r["src"]] = d
        dd = d.astype(np.int64)
        reach = d != np.uint32(0xFFFFFFFF)
        assert reach.all()  # the WAN is connected
        # Bellman: no edge relaxes, and every non-source node has a tight in-edge
        cand = dd[src_of_edge] + w
        assert (cand >= dd[col]).all(), r["src"]
        tight = np.zeros(V, dtype=bool)
        tight[col[cand == dd[col]]] = True
        tight[r["src"]] = True
        assert tight.all() and dd[r["src"]] == 0, r["src"]
    srcs = list(rows)
    for a in srcs:  # symmetric metrics: D[a][b] == D[b][a]
        for b in srcs:
            assert rows[a][b] == rows[b][a], (a, b)
    sas.close()


def test_config3_wan100k_all_sources_spf_table(gpu_ready):
    """Config 3 through the in-ABI multi-GPU path (spf_cluster + spf_cgraph +
    spf_table_create_q, world 1, rows all-gathered into the rank slots):
    the reference's checksum of row n0 and the 32 golden rows."""
    from openr_amd import abi
    from openr_amd import topologies as TP

    gold = json.load(open(os.path.join(GOLD, "wan100k_rows.json")))["rows"]
    anchor = [a for a in json.load(open(os.path.join(GOLD, "wan_anchors.json")))["anchors"]
              if a["V"] == 100000 and a["S"] == 1][0]
    csr = TP.wan(100000, 1000000).csr()
    c = abi.Cluster([0])
    cg = abi.ClusterGraph(c, csr)
    t = cg.table(np.arange(csr.num_nodes, dtype=np.uint32), 0, gather=abi.SPF_T_GATHER_ROWS).run()
    assert t.kernel(0) == "dstep-ldsrow"
    assert int(t.fetch_rows(0, 1)[0].astype(np.int64).sum()) == anchor["sum_dist"]
    for r in gold:
        row = t.fetch_rows(r["src"], 1)[0]
        assert hashlib.sha256(row.tobytes()).hexdigest() == r["sha256"], r["src"]
    t.close()
    cg.close()
    c.close()


def _two_area():
    from openr_amd import topologies as TP

    meta = json.load(open(os.path.join(GOLD, "whatif_two_area.json")))
    want = np.load(os.path.join(GOLD, "whatif_two_area.npz"))["summary"]
    areas = TP.whatif_two_area()
    for (area, _, links), m in zip(areas, meta["areas"]):
        assert m["area"] == area and m["links"] == [int(x) for x in links]
    return meta, want, areas


def test_config5_whatif_batch_c_abi(gpu_ready):
    from openr_amd import abi
    from openr_amd import topologies as TP

    meta, want, areas = _two_area()
    off = 0
    for area, topo, links in areas:
        csr = topo.csr()
        r, _ = topo.rank()
        sid = int(r[topo.names.index(TP.WHATIF_BORDER)])
        n = len(links)
        g = abi.Graph(csr)
        srcs = np.full(n, sid, dtype=np.uint32)
        q = g.query(srcs, abi.SPF_F_NEXTHOPS, ignore=[[int(l)] for l in links]).run()
        got = _batch_summaries(q, g, srcs, None)  # every query's full mix
        _check_summary(got, want[off:off + n], None, f"what-if area {area}")
        off += n
        q.close()
        g.close()
    assert off == len(want) == 8192


@pytest.mark.parametrize("fan_out", [False, True])
def test_config5_whatif_multi_area_linkstate(gpu_ready, fan_out):
    """The same failures through the drop-in: one AreaLinkStates holding both
    areas, LinkState::runSpfBatch(border, {link}) per area, sampled results
    materialised in the reference's SpfResult form; fan_out: through the
    multi-GPU path (setSpfDevices, the cluster graph, ignore lists sliced per
    block)."""
    import openr_amd._openr_spf as E
    from openr_amd import topologies as TP

    E.set_spf_devices([0] if fan_out else [])
    try:
        _config5_linkstate(E, TP, fan_out)
    finally:
        E.set_spf_devices([])


def _config5_linkstate(E, TP, fan_out):
    meta, want, areas = _two_area()
    la = E.AreaLinkStates()
    for area, topo, _ in areas:
        ls = la.add(area)
        for db in topo.adj_dbs(area):
            ls.updateAdjacencyDatabase(db)
    off = 0
    for (area, topo, links), m in zip(areas, meta["areas"]):
        ls = la[area]
        ign = []
        for l in links:
            a, b = topo.links[int(l)][:2]
            na, nb = topo.names[a], topo.names[b]
            ign.append([x for x in ls.linksFromNode(na) if x.getOtherNodeName(na) == nb])
        E.reset_counters()
        batch = ls.runSpfBatch(TP.WHATIF_BORDER, ign, True)
        assert len(batch) == len(links)
        assert E.get_counters()["decision.spf_runs"] == len(links)
        assert (E.get_counters().get("decision.spf_cluster_batches", 0) == 1) == fan_out
        _, names_by_rank = topo.rank()
        for s in m["sampled"]:
            res = batch.result(s["query"])
            assert len(res) == s["reached"]
            assert digest(spf_canon(res)) == s["digest"], (area, s["query"])
        # every query's distance checksum from the flat batch (node ids = ranks)
        for qi in range(0, len(links), 97):
            tot = sum(batch.metric(qi, v) or 0 for v in range(topo.num_nodes))
            assert tot == int(want[off + qi, 1]), (area, qi)
        off += len(links)
