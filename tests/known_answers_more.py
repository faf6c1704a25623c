"""More known answers of the reference's own tests (round 2), restated as
scenarios in the same form as tests/known_answers.py: each `sc_*` function
runs against a module `M` exposing the LinkState / SpfSolver / PrefixState
surface -- the CPU oracle (oracle._oracle_ref) in the "not gpu" suite and the
MI355X engine (openr_amd._openr_spf) in the gpu suite -- and asserts the
reference's expected values.

They pin the branches round 1 left to engine-vs-oracle comparison only:
  * holds          HoldableValueTest / LinkTest       LinkStateTest.cpp:22-137
  * BGP best path  BGPRedistribution                   DecisionTest.cpp:673-1016
                   SimpleRing Ksp2EdEcmpForBGP(123)    DecisionTest.cpp:2140-2453
                   ParallelAdjRing Ksp2EdEcmp(ForBGP)  DecisionTest.cpp:3213-3538
  * multi-area     MultiAreaBestPathCalculation        DecisionTest.cpp:4503-4638
  * SR-MPLS / MPLS SimpleRingMesh Ksp2EdEcmp / SPMPLS  DecisionTest.cpp:1409-1499
                   Ip2MplsRoutes                       DecisionTest.cpp:3558-3844
                   DuplicateMplsRoutes (getRouteDelta) DecisionTest.cpp:1774-1822
  * LFA / overload OverloadLinkTest                    DecisionTest.cpp:2625-2805
                   ParallelAdjRing MultiPathTest       DecisionTest.cpp:3054-3208
                   ParallelLinks, DuplicatePrefixes    DecisionTest.cpp:4882-4982, 5374-5479
  * grid           GridTopologyFixture n = 10..16      DecisionTest.cpp:3920-4010

The DecisionTestFixture cases (Decision on its own thread fed by KvStore
publications, DecisionTest.cpp:4033-4223) are restated through `DecisionSim`:
the publications' AdjacencyDatabase / PrefixDatabase objects are applied to the
per-area LinkState and the PrefixState (processPublication, Decision.cpp:
1631-1763), and dumpRouteDb is getDecisionRouteDb = buildRouteDb of the node
on SpfSolver("1", v4 off, LFA on) (Decision.cpp:1437-1462; the fixture's
Decision is built with computeLfaPaths = true, DecisionTest.cpp:4042-4050).
With `wire=True` (engine only) the same publications go through
PublicationIngest as CompactProtocol blobs instead.
"""

from __future__ import annotations

import copy

from openr_amd import thrift as T
from tests import known_answers as KA
from tests.known_answers import (
    L,
    NH,
    P,
    R,
    addr1,
    addr1V4,
    addr2,
    addr2V4,
    addr3,
    addr3V4,
    addr4,
    addr4V4,
    adj12,
    adj13,
    adj14,
    adj21,
    adj23,
    adj24,
    adj31,
    adj32,
    adj34,
    adj41,
    adj42,
    adj43,
    counters,
    get_route_map,
    kDefaultArea,
    labelPhpAction,
    nh,
    prefixDb1,
    prefixDb2,
    prefixDb3,
    prefixDb4,
    prefixDb1V4,
    prefixDb2V4,
    prefixDb3V4,
    prefixDb4V4,
    push,
    single_area,
    swap,
    validate_adj_label_routes,
    validate_pop_label_route,
)

A = T.MplsActionCode
BGP = T.PrefixType.BGP

# DecisionTest.cpp:100-107
bgpAddr1 = T.toIpPrefix("2401:1::10.1.1.1/32")
bgpAddr2 = T.toIpPrefix("2401:2::10.2.2.2/32")
bgpAddr3 = T.toIpPrefix("2401:3::10.3.3.3/32")
bgpAddr4 = T.toIpPrefix("2401:4::10.4.4.4/32")
bgpAddr1V4 = T.toIpPrefix("10.11.1.1/16")
bgpAddr2V4 = T.toIpPrefix("10.22.2.2/16")
bgpAddr3V4 = T.toIpPrefix("10.33.3.3/16")
bgpAddr4V4 = T.toIpPrefix("10.43.4.4/16")


def _mv(n=5, tie_last=False):
    """The 5-entry MetricVector the BGP tests build: type = priority = i,
    WIN_IF_PRESENT, metric {i} (DecisionTest.cpp:696-706)."""
    return T.MetricVector(
        0,
        [
            T.createMetricEntity(i, i, T.CompareType.WIN_IF_PRESENT, tie_last and i == n - 1, [i])
            for i in range(n)
        ],
    )


def kspf(pdb, prefixType=None, prefix=None, prependLabel=None):
    """DecisionTest.cpp:147-180 createPrefixDbWithKspfAlgo."""
    db = copy.deepcopy(pdb)
    for e in db.prefixEntries:
        e.forwardingType = T.PrefixForwardingType.SR_MPLS
        e.forwardingAlgorithm = T.PrefixForwardingAlgorithm.KSP2_ED_ECMP
        if prefixType == BGP and prefix is None:
            e.type = BGP
            e.mv = T.MetricVector()
    if prefix is not None:
        e = T.PrefixEntry(
            prefix=prefix,
            type=BGP,
            forwardingType=T.PrefixForwardingType.SR_MPLS,
            forwardingAlgorithm=T.PrefixForwardingAlgorithm.KSP2_ED_ECMP,
            mv=T.MetricVector(),
            prependLabel=prependLabel,
        )
        db.prefixEntries.append(e)
    return db


# ------------------------------------------------------- LinkStateTest.cpp


def sc_holdable_value(M):
    """LinkStateTest.cpp:22-83 (HoldableValueTest.BasicOperation)."""
    hv = M.HoldableValueBool(True)
    assert hv.value() is True and not hv.hasHold() and not hv.decrementTtl()
    up, down = 10, 5
    assert not hv.updateValue(False, up, down)
    for _ in range(up - 1):
        assert hv.hasHold() and hv.value() is True and not hv.decrementTtl()
    assert hv.decrementTtl()
    assert not hv.hasHold() and hv.value() is False
    # same value: no hold
    assert not hv.updateValue(False, up, down)
    assert not hv.hasHold() and hv.value() is False
    # bringing down now
    assert not hv.updateValue(True, up, down)
    for _ in range(down - 1):
        assert hv.hasHold() and hv.value() is False and not hv.decrementTtl()
    assert hv.decrementTtl()
    assert not hv.hasHold() and hv.value() is True
    # change twice within the ttl
    assert not hv.updateValue(False, up, down)
    assert hv.hasHold() and hv.value() is True and not hv.decrementTtl()
    assert hv.updateValue(True, up, down)
    assert not hv.hasHold() and hv.value() is True
    # LinkStateMetric
    hm = M.HoldableValueMetric(10)
    assert hm.value() == 10 and not hm.hasHold() and not hm.decrementTtl()
    assert not hm.updateValue(5, up, down)
    for _ in range(up - 1):
        assert hm.hasHold() and hm.value() == 10 and not hm.decrementTtl()
    assert hm.decrementTtl()
    assert not hm.hasHold() and hm.value() == 5


def sc_link_basic(M):
    """LinkStateTest.cpp:85-137 (LinkTest.BasicOperation)."""
    n1, n2, n3 = "node1", "node2", "node3"
    a1 = T.createAdjacency(n1, "if1", "if2", "fe80::2", "10.0.0.2", 1, 1, 1)
    a2 = T.createAdjacency(n2, "if2", "if1", "fe80::1", "10.0.0.1", 1, 2, 1)
    l1 = M.Link.fromAdjacencies(kDefaultArea, n1, a1, n2, a2)
    assert l1.getArea() == kDefaultArea
    assert l1.getOtherNodeName(n1) == n2 and l1.getOtherNodeName(n2) == n1
    for getter in ("getOtherNodeName", "getIfaceFromNode", "getMetricFromNode", "getAdjLabelFromNode"):
        try:
            getattr(l1, getter)(n3)
        except ValueError:  # std::invalid_argument
            pass
        else:
            raise AssertionError(f"{getter}(node3) did not throw")
    assert l1.getIfaceFromNode(n1) == a1.ifName and l1.getIfaceFromNode(n2) == a2.ifName
    assert l1.getMetricFromNode(n1) == a1.metric and l1.getMetricFromNode(n2) == a2.metric
    assert l1.getAdjLabelFromNode(n1) == a1.adjLabel and l1.getAdjLabelFromNode(n2) == a2.adjLabel
    assert not l1.getOverloadFromNode(n1) and not l1.getOverloadFromNode(n2)
    assert l1.isUp()
    assert l1.setMetricFromNode(n1, 2, 0, 0)
    assert l1.getMetricFromNode(n1) == 2
    assert l1.setOverloadFromNode(n2, True, 0, 0)
    assert not l1.getOverloadFromNode(n1) and l1.getOverloadFromNode(n2)
    assert not l1.isUp()
    l2 = M.Link.fromAdjacencies(kDefaultArea, n2, a2, n1, a1)
    assert l1 == l2 and not (l1 < l2) and not (l2 < l1)
    a3 = T.createAdjacency(n2, "if3", "if2", "fe80::3", "10.0.0.3", 1, 1, 1)
    l3 = M.Link.fromAdjacencies(kDefaultArea, n1, a1, n3, a3)
    assert not (l1 == l3)
    assert (l1 < l3) or (l3 < l1)


# ------------------------------------------------- BGPRedistribution


def _bgp_entry(prefix, data, mv, ftype=T.PrefixForwardingType.IP, algo=T.PrefixForwardingAlgorithm.SP_ECMP):
    return T.createPrefixEntry(prefix, BGP, data, ftype, algo, False, mv, None)


def sc_bgp_redistribution_basic(M):
    """DecisionTest.cpp:673-841 (BGPRedistribution.BasicOperation)."""
    s = M.SpfSolver("1", False, False)
    areas, ls = single_area(M)
    ps = M.PrefixState()
    assert not ls.updateAdjacencyDatabase(T.createAdjDb("1", [adj12, adj13], 0))[0]
    assert ls.updateAdjacencyDatabase(T.createAdjDb("2", [adj21], 0))[0]
    assert ls.updateAdjacencyDatabase(T.createAdjDb("3", [adj31], 0))[0]
    db1 = copy.deepcopy(prefixDb1)
    db2 = copy.deepcopy(prefixDb2)
    bgpPrefix1 = addr3
    db1.prefixEntries.append(_bgp_entry(bgpPrefix1, "data1", _mv()))
    assert ps.updatePrefixDatabase(db1)
    assert ps.updatePrefixDatabase(db2)
    route1_nhs = NH(nh(adj21, False, adj21.metric))
    best1 = T.createNextHop(addr1.prefixAddress).key()

    def check_route(db, nhs, best, data):
        e = db["unicast"][bgpPrefix1.key()]
        assert e["nexthops"] == nhs
        assert e["bestNexthop"] == best
        assert e["bestPrefixEntry"][1] == BGP and e["bestPrefixEntry"][2] == data
        assert e["doNotInstall"] is False

    db = s.buildRouteDb("2", areas, ps)
    assert len(db["unicast"]) == 2
    check_route(db, route1_nhs, best1, b"data1")
    # node 2 advertises the same metric vector: no best path, no route
    db2.prefixEntries.append(_bgp_entry(bgpPrefix1, "data2", _mv()))
    assert ps.updatePrefixDatabase(db2)
    assert len(s.buildRouteDb("1", areas, ps)["unicast"]) == 1
    # node 2's last metric one lower: node 1 wins again
    db2.prefixEntries[-1].mv.metrics[4].metric[0] -= 1
    assert ps.updatePrefixDatabase(db2)
    db = s.buildRouteDb("2", areas, ps)
    assert len(db["unicast"]) == 2
    check_route(db, route1_nhs, best1, b"data1")
    # node 2 better
    db2.prefixEntries[-1].mv.metrics[4].metric[0] += 2
    assert ps.updatePrefixDatabase(db2)
    route2_nhs = NH(nh(adj12, False, adj12.metric))
    best2 = T.createNextHop(addr2.prefixAddress).key()
    db = s.buildRouteDb("1", areas, ps)
    assert len(db["unicast"]) == 2
    check_route(db, route2_nhs, best2, b"data2")
    # tie-breaker on the last metric: multipath
    db1.prefixEntries[-1].mv.metrics[4].isBestPathTieBreaker = True
    db2.prefixEntries[-1].mv.metrics[4].isBestPathTieBreaker = True
    assert ps.updatePrefixDatabase(db1)
    assert ps.updatePrefixDatabase(db2)
    assert len(s.buildRouteDb("1", areas, ps)["unicast"]) == 1
    db = s.buildRouteDb("3", areas, ps)
    assert len(db["unicast"]) == 3
    e = db["unicast"][bgpPrefix1.key()]
    assert e["bestPrefixEntry"][2] == b"data2"
    assert e["nexthops"] == NH(nh(adj31, False, 10))
    # disconnect: every node considers its own route best, programs nothing
    assert ls.updateAdjacencyDatabase(T.createAdjDb("1", [], 0))[0]
    for node in ("1", "2"):
        db = s.buildRouteDb(node, areas, ps)
        e = db["unicast"].get(bgpPrefix1.key())
        assert e is None or (e["nexthops"] not in (route1_nhs, route2_nhs))


def sc_bgp_redistribution_igp_metric(M):
    """DecisionTest.cpp:853-1016 (BGPRedistribution.IgpMetric,
    bgpUseIgpMetric = true)."""
    s = M.SpfSolver("1", False, False, False, False, True)
    areas, ls = single_area(M)
    ps = M.PrefixState()
    mv = _mv(tie_last=True)
    bgpPrefix2 = _bgp_entry(addr1, "data1", copy.deepcopy(mv))
    mv.metrics[4].metric = [100]
    bgpPrefix3 = _bgp_entry(addr1, "data1", copy.deepcopy(mv))
    db1 = T.createAdjDb("1", copy.deepcopy([adj12, adj13]), 0)
    assert not ls.updateAdjacencyDatabase(db1)[0]
    assert ls.updateAdjacencyDatabase(T.createAdjDb("2", [adj21], 0))[0]
    assert ls.updateAdjacencyDatabase(T.createAdjDb("3", [adj31], 0))[0]
    assert ps.updatePrefixDatabase(T.createPrefixDb("2", [T.createPrefixEntry(addr2), bgpPrefix2]))
    assert ps.updatePrefixDatabase(T.createPrefixDb("3", [T.createPrefixEntry(addr3), bgpPrefix3]))

    def check(n_routes, *hops):
        db = s.buildRouteDb("1", areas, ps)
        assert len(db["unicast"]) == n_routes
        e = db["unicast"][addr1.key()]
        assert e["bestPrefixEntry"][2] == b"data1"
        assert e["nexthops"] == NH(*[nh(a, False, m) for a, m in hops])

    check(3, (adj12, 10), (adj13, 10))
    db1.adjacencies[1].metric = 20
    assert ls.updateAdjacencyDatabase(db1)[0]
    check(3, (adj12, 10))
    db1.adjacencies[0].isOverloaded = True
    assert ls.updateAdjacencyDatabase(db1)[0]
    check(2, (adj13, 20))
    db1.adjacencies[0].metric = 20
    assert ls.updateAdjacencyDatabase(db1)[0]
    check(2, (adj13, 20))
    db1.adjacencies[0].isOverloaded = False
    assert ls.updateAdjacencyDatabase(db1)[0]
    check(3, (adj12, 20), (adj13, 20))


# ------------------------------------------------------------ SimpleRingMesh


def _ring_pdbs(v4):
    return (prefixDb1V4, prefixDb2V4, prefixDb3V4, prefixDb4V4) if v4 else (
        prefixDb1, prefixDb2, prefixDb3, prefixDb4)


def _bgp_addrs(v4):
    return (bgpAddr1V4, bgpAddr2V4, bgpAddr3V4, bgpAddr4V4) if v4 else (
        bgpAddr1, bgpAddr2, bgpAddr3, bgpAddr4)


def _addrs(v4):
    return (addr1V4, addr2V4, addr3V4, addr4V4) if v4 else (addr1, addr2, addr3, addr4)


def _ring_like_setup(M, adj_lists, v4, lfa, ksp2, prefixType=None, newBgp=False):
    """SimpleRing(Mesh)TopologyFixture::CustomSetUp (DecisionTest.cpp:
    1316-1390 / 1530-1600)."""
    s = M.SpfSolver("1", v4, lfa)
    dbs = {str(i + 1): T.createAdjDb(str(i + 1), copy.deepcopy(adj_lists[i]), i + 1) for i in range(4)}
    areas, ls = single_area(M)
    assert ls.updateAdjacencyDatabase(dbs["1"]) == (False, False, True)
    for n in ("2", "3", "4"):
        assert ls.updateAdjacencyDatabase(dbs[n]) == (True, False, True)
    ps = M.PrefixState()
    pdbs = {}
    for i, pdb in enumerate(_ring_pdbs(v4)):
        if ksp2:
            pdb = kspf(pdb, prefixType, _bgp_addrs(v4)[i] if newBgp else None)
        pdbs[str(i + 1)] = copy.deepcopy(pdb)
        ps.updatePrefixDatabase(pdb)
    return s, areas, ls, ps, dbs, pdbs


MESH = ([adj12, adj13, adj14], [adj21, adj23, adj24], [adj31, adj32, adj34], [adj41, adj42, adj43])
RING = ([adj12, adj13], [adj21, adj24], [adj31, adj34], [adj42, adj43])


def sc_ring_mesh_ksp2(M):
    """DecisionTest.cpp:1409-1467 (SimpleRingMesh Ksp2EdEcmp), the four
    instances (v4 x {none, BGP})."""
    for v4 in (True, False):
        for ptype in (None, BGP):
            s, areas, ls, ps, dbs, _ = _ring_like_setup(M, MESH, v4, False, True, ptype)
            rm = get_route_map(s, ["1"], areas, ps)
            a = _addrs(v4)
            n = lambda adj, m, act=None: nh(adj, v4, m, act, True)  # noqa: E731
            assert R(rm, "1", P(a[3])) == NH(n(adj14, 10), n(adj12, 20, push(4)), n(adj13, 20, push(4))), (v4, ptype)
            assert R(rm, "1", L(4)) == NH(nh(adj14, False, 10, labelPhpAction))
            assert R(rm, "1", P(a[2])) == NH(n(adj13, 10), n(adj12, 20, push(3)), n(adj14, 20, push(3)))
            assert R(rm, "1", P(a[1])) == NH(n(adj12, 10), n(adj13, 20, push(2)), n(adj14, 20, push(2)))
            validate_pop_label_route(rm, "1", 1)
            validate_adj_label_routes(rm, "1", dbs["1"].adjacencies)
            dbs["3"].isOverloaded = True
            assert ls.updateAdjacencyDatabase(dbs["3"])[0]
            rm = get_route_map(s, ["1"], areas, ps)
            assert R(rm, "1", P(a[3])) == NH(n(adj14, 10), n(adj12, 20, push(4)))


def sc_ring_mesh_sp_mpls(M):
    """DecisionTest.cpp:1469-1499 (SimpleRingMesh SPMPLS): SR_MPLS prefixes
    with SP_ECMP go through selectKsp2 with k = 1 only."""
    for v4 in (True, False):
        for ptype in (None, BGP):
            s, areas, ls, ps, dbs, pdbs = _ring_like_setup(M, MESH, v4, False, True, ptype)
            db = pdbs["1"]
            for e in db.prefixEntries:
                e.forwardingAlgorithm = T.PrefixForwardingAlgorithm.SP_ECMP
            ps.updatePrefixDatabase(db)
            a1 = _addrs(v4)[0]
            for node, adj in (("2", adj21), ("3", adj31), ("4", adj41)):
                rm = get_route_map(s, [node], areas, ps)
                assert R(rm, node, P(a1)) == NH(nh(adj, v4, 10, None, True)), (v4, ptype, node)


# ------------------------------------------------------------ SimpleRing


def sc_ring_duplicate_mpls_routes(M):
    """DecisionTest.cpp:1774-1822 (DuplicateMplsRoutes): the smaller node name
    keeps a duplicated node label; getRouteDelta reports it as an update and
    never as a delete; one decision.duplicate_node_label per build."""
    for v4 in (True, False):
        s, areas, ls, ps, dbs, _ = _ring_like_setup(M, RING, v4, False, False)
        M.reset_counters()
        dbs["1"].nodeLabel = 2
        ls.updateAdjacencyDatabase(dbs["1"])
        empty = M.DecisionRouteDb()

        def verify(node, label, comp):
            new = s.buildRouteDbObject(node, areas, ps)
            d = M.getRouteDelta(new, comp)
            assert sum(1 for lab in d["mplsRoutesToUpdate"] if lab == label) == 1, (node, d)
            assert len(d["mplsRoutesToDelete"]) == 0, (node, d)

        for node in ("1", "2", "3"):
            verify(node, 2, empty)
        assert counters(M)["decision.duplicate_node_label"] == 3
        comp = {node: s.buildRouteDbObject(node, areas, ps) for node in ("1", "2", "3")}
        assert counters(M)["decision.duplicate_node_label"] == 6
        dbs["1"].nodeLabel = 1
        ls.updateAdjacencyDatabase(dbs["1"])
        for node in ("1", "2", "3"):
            verify(node, 2, comp[node])
        assert counters(M)["decision.duplicate_node_label"] == 6


def _static_60000(M, s):
    """DecisionTest.cpp:2325-2337: static MPLS route 60000 -> 1.1.1.1 PHP."""
    hop = T.NextHopThrift(address=T.toBinaryAddress("1.1.1.1"), mplsAction=T.createMplsAction(A.PHP))
    s.pushRoutesDeltaUpdates([T.MplsRoute(60000, [hop])], [])
    s.processStaticRouteUpdates()


def sc_ring_ksp2_for_bgp(M):
    """DecisionTest.cpp:2140-2354 (SimpleRing Ksp2EdEcmpForBGP, BGP instances):
    metric-vector best path over KSP2 routes, prependLabel, tie-breaker
    multipath, static MPLS next hops of the prepend label; spf_runs == 6."""
    for v4 in (True, False):
        s, areas, ls, ps, dbs, pdbs = _ring_like_setup(M, RING, v4, True, True, BGP, True)
        M.reset_counters()
        one, two = pdbs["1"], pdbs["2"]
        one.prefixEntries[1].mv = _mv()
        two.prefixEntries.append(copy.deepcopy(one.prefixEntries[1]))
        one.prefixEntries[1].prependLabel = 60000
        ps.updatePrefixDatabase(one)
        ps.updatePrefixDatabase(two)
        rm = get_route_map(s, ["3"], areas, ps)
        assert counters(M)["decision.spf_runs"] == 6
        b1 = _bgp_addrs(v4)[0]
        a = _addrs(v4)
        n = lambda adj, m, act=None: nh(adj, v4, m, act, True)  # noqa: E731
        assert ("3",) + P(b1) not in rm
        two.prefixEntries[-1].mv.metrics[4].metric[0] -= 1
        one.prefixEntries[-1].data = b"123"
        ps.updatePrefixDatabase(two)
        ps.updatePrefixDatabase(one)
        rm = get_route_map(s, ["3"], areas, ps)
        assert R(rm, "3", P(b1)) == NH(n(adj31, 10, push(60000)), n(adj34, 30, push(60000, 1, 2))), v4
        best1 = T.createNextHop(a[0].prefixAddress).key()
        best2 = T.createNextHop(a[1].prefixAddress).key()
        assert s.buildRouteDb("3", areas, ps)["unicast"][b1.key()]["bestNexthop"] == best1
        two.prefixEntries[-1].mv.metrics[4].metric[0] += 2
        ps.updatePrefixDatabase(two)
        rm = get_route_map(s, ["3"], areas, ps)
        assert R(rm, "3", P(b1)) == NH(n(adj31, 20, push(2)), n(adj34, 20, push(2)))
        assert s.buildRouteDb("3", areas, ps)["unicast"][b1.key()]["bestNexthop"] == best2
        two.prefixEntries[-1].mv.metrics[4].isBestPathTieBreaker = True
        one.prefixEntries[-1].mv.metrics[4].isBestPathTieBreaker = True
        ps.updatePrefixDatabase(two)
        ps.updatePrefixDatabase(one)
        rm = get_route_map(s, ["3"], areas, ps)
        assert R(rm, "3", P(b1)) == NH(n(adj31, 20, push(2)), n(adj34, 20, push(2)), n(adj31, 10, push(60000)))
        e = s.buildRouteDb("3", areas, ps)["unicast"][b1.key()]
        assert e["bestNexthop"] in (best1, best2)
        assert e["bestPrefixEntry"][2] == (b"123" if e["bestNexthop"] == best1 else None)
        assert e["bestPrefixEntry"][1] == BGP
        _static_60000(M, s)
        rm = get_route_map(s, ["1"], areas, ps)
        assert R(rm, "1", P(b1)) == NH(
            T.createNextHop(T.toBinaryAddress("1.1.1.1"), None, 0, None, True).key(),
            n(adj13, 30, push(2, 4)),
            n(adj12, 10),
        ), v4


def sc_ring_ksp2_for_bgp123(M):
    """DecisionTest.cpp:2356-2453 (SimpleRing Ksp2EdEcmpForBGP123): static
    next hops count towards nothing but the route; minNexthop 3 drops it."""
    for v4 in (True, False):
        s, areas, ls, ps, dbs, pdbs = _ring_like_setup(M, RING, v4, True, True, BGP, True)
        one, two = pdbs["1"], pdbs["2"]
        one.prefixEntries[1].mv = _mv()
        two.prefixEntries.append(copy.deepcopy(one.prefixEntries[1]))
        one.prefixEntries[1].prependLabel = 60000
        two.prefixEntries[-1].mv.metrics[4].metric[0] += 1
        two.prefixEntries[-1].mv.metrics[4].isBestPathTieBreaker = True
        one.prefixEntries[-1].mv.metrics[4].isBestPathTieBreaker = True
        ps.updatePrefixDatabase(one)
        ps.updatePrefixDatabase(two)
        _static_60000(M, s)
        b1 = _bgp_addrs(v4)[0]
        n = lambda adj, m, act=None: nh(adj, v4, m, act, True)  # noqa: E731
        rm = get_route_map(s, ["1"], areas, ps)
        assert R(rm, "1", P(b1)) == NH(
            T.createNextHop(T.toBinaryAddress("1.1.1.1"), None, 0, None, True).key(),
            n(adj13, 30, push(2, 4)),
            n(adj12, 10),
        ), v4
        one.prefixEntries[1].minNexthop = 3
        ps.updatePrefixDatabase(one)
        rm = get_route_map(s, ["1"], areas, ps)
        assert ("1",) + P(b1) not in rm


def sc_ring_overload_link(M):
    """DecisionTest.cpp:2625-2805 (OverloadLinkTest, LFA on): adj31 then adj34
    overloaded; node 3 ends up disconnected."""
    for v4 in (True, False):
        s, areas, ls, ps, dbs, _ = _ring_like_setup(M, RING, v4, True, False)
        a = _addrs(v4)
        db3 = dbs["3"]
        db3.adjacencies[0].isOverloaded = True
        assert ls.updateAdjacencyDatabase(db3)[0]
        rm = get_route_map(s, ["1", "2", "3", "4"], areas, ps)
        assert len(rm) == 36
        exp = {
            "1": {4: (adj12, 20), 3: (adj12, 30), 2: (adj12, 10)},
            "2": {4: (adj24, 10), 3: (adj24, 20), 1: (adj21, 10)},
            "3": {4: (adj34, 10), 2: (adj34, 20), 1: (adj34, 30)},
            "4": {3: (adj43, 10), 2: (adj42, 10), 1: (adj42, 20)},
        }

        def check(exp):
            for node, dsts in exp.items():
                for d, (adj, m) in dsts.items():
                    assert R(rm, node, P(a[d - 1])) == NH(nh(adj, v4, m)), (v4, node, d)
                    act = labelPhpAction if m == 10 else swap(d)
                    assert R(rm, node, L(d)) == NH(nh(adj, False, m, act)), (v4, node, "label", d)
                validate_pop_label_route(rm, node, int(node))
                validate_adj_label_routes(rm, node, dbs[node].adjacencies)

        check(exp)
        db3.adjacencies[1].isOverloaded = True
        assert ls.updateAdjacencyDatabase(db3)[0]
        rm = get_route_map(s, ["1", "2", "3", "4"], areas, ps)
        assert len(rm) == 24
        check({
            "1": {4: (adj12, 20), 2: (adj12, 10)},
            "2": {4: (adj24, 10), 1: (adj21, 10)},
            "3": {},
            "4": {2: (adj42, 10), 1: (adj42, 20)},
        })


# ------------------------------------------------------------ ParallelAdjRing


def _par(M, lfa, ksp2, ptype=None):
    """ParallelAdjRingTopologyFixture::CustomSetUp (DecisionTest.cpp:
    2830-2914), prefixes through createPrefixDbWithKspfAlgo(db, prefixType)."""
    s = M.SpfSolver("1", False, lfa)
    dbs = {
        "1": T.createAdjDb("1", copy.deepcopy([KA.adj12_1, KA.adj12_2, KA.adj12_3, KA.adj13_1]), 1),
        "2": T.createAdjDb("2", copy.deepcopy([KA.adj21_1, KA.adj21_2, KA.adj21_3, KA.adj24_1]), 2),
        "3": T.createAdjDb("3", copy.deepcopy([KA.adj31_1, KA.adj34_1, KA.adj34_2, KA.adj34_3]), 3),
        "4": T.createAdjDb("4", copy.deepcopy([KA.adj42_1, KA.adj43_1, KA.adj43_2, KA.adj43_3]), 4),
    }
    areas, ls = single_area(M)
    assert not ls.updateAdjacencyDatabase(dbs["1"])[0]
    for n in ("2", "3", "4"):
        assert ls.updateAdjacencyDatabase(dbs[n])[0]
    ps = M.PrefixState()
    pdbs = {}
    for i, pdb in enumerate((prefixDb1, prefixDb2, prefixDb3, prefixDb4)):
        pdb = kspf(pdb, ptype) if ksp2 else copy.deepcopy(pdb)
        pdbs[str(i + 1)] = copy.deepcopy(pdb)
        ps.updatePrefixDatabase(pdb)
    return s, areas, ls, ps, dbs, pdbs


def sc_parallel_ring_multipath(M):
    """DecisionTest.cpp:3054-3208 (ParallelAdjRing MultiPathTest, LFA on):
    44 routes; LFA keeps the parallel 20-metric links."""
    s, areas, ls, ps, dbs, _ = _par(M, True, False)
    rm = get_route_map(s, ["1", "2", "3", "4"], areas, ps)
    assert len(rm) == 44
    k = KA
    exp = {
        ("1", 4): [(k.adj12_1, 22), (k.adj12_2, 22), (k.adj12_3, 31), (k.adj13_1, 22)],
        ("1", 3): [(k.adj13_1, 11)],
        ("1", 2): [(k.adj12_1, 11), (k.adj12_2, 11), (k.adj12_3, 20)],
        ("2", 4): [(k.adj24_1, 11)],
        ("2", 3): [(k.adj21_1, 22), (k.adj21_2, 22), (k.adj21_3, 31), (k.adj24_1, 22)],
        ("2", 1): [(k.adj21_1, 11), (k.adj21_2, 11), (k.adj21_3, 20)],
        ("3", 4): [(k.adj34_1, 11), (k.adj34_2, 20), (k.adj34_3, 20)],
        ("3", 2): [(k.adj31_1, 22), (k.adj34_1, 22), (k.adj34_2, 31), (k.adj34_3, 31)],
        ("3", 1): [(k.adj31_1, 11)],
        ("4", 3): [(k.adj43_1, 11), (k.adj43_2, 20), (k.adj43_3, 20)],
        ("4", 2): [(k.adj42_1, 11)],
        ("4", 1): [(k.adj42_1, 22), (k.adj43_1, 22), (k.adj43_2, 31), (k.adj43_3, 31)],
    }
    addrs = {1: addr1, 2: addr2, 3: addr3, 4: addr4}
    for (node, d), hops in exp.items():
        assert R(rm, node, P(addrs[d])) == NH(*[nh(x, False, m) for x, m in hops]), (node, d)
        # the label action follows the shortest distance to the node (PHP
        # when it is a neighbour)
        act = labelPhpAction if min(m for _, m in hops) == 11 else swap(d)
        assert R(rm, node, L(d)) == NH(*[nh(x, False, m, act) for x, m in hops]), (node, "label", d)
    for node in ("1", "2", "3", "4"):
        validate_pop_label_route(rm, node, int(node))
        validate_adj_label_routes(rm, node, dbs[node].adjacencies)


def sc_parallel_ring_ksp2_bgp_instance(M):
    """DecisionTest.cpp:3213-3385 (ParallelAdjRing Ksp2EdEcmp, the BGP-typed
    instance: every loopback is a BGP entry with an empty metric vector)."""
    s, areas, ls, ps, dbs, pdbs = _par(M, True, True, BGP)
    n = lambda adj, m, act=None: nh(adj, False, m, act, True)  # noqa: E731
    k = KA
    rm = get_route_map(s, ["1"], areas, ps)
    assert R(rm, "1", P(addr2)) == NH(n(k.adj12_1, 11), n(k.adj12_2, 11), n(k.adj12_3, 20))
    four, three = pdbs["4"], pdbs["3"]
    newp = T.createPrefixEntry(
        bgpAddr1, T.PrefixType.LOOPBACK, "", T.PrefixForwardingType.SR_MPLS,
        T.PrefixForwardingAlgorithm.KSP2_ED_ECMP, None, None, 4,
    )
    four.prefixEntries.append(copy.deepcopy(newp))
    ps.updatePrefixDatabase(four)
    rm = get_route_map(s, ["1"], areas, ps)
    assert ("1",) + P(bgpAddr1) not in rm
    four.prefixEntries.pop()
    newp.minNexthop = 2
    four.prefixEntries.append(copy.deepcopy(newp))
    ps.updatePrefixDatabase(four)
    rm = get_route_map(s, ["1"], areas, ps)
    assert R(rm, "1", P(bgpAddr1)) == NH(n(k.adj12_2, 22, push(4)), n(k.adj13_1, 22, push(4)))
    newp.minNexthop = 4
    three.prefixEntries.append(copy.deepcopy(newp))
    ps.updatePrefixDatabase(three)
    rm = get_route_map(s, ["1"], areas, ps)
    assert ("1",) + P(bgpAddr1) not in rm
    four.prefixEntries.pop()
    three.prefixEntries.pop()
    ps.updatePrefixDatabase(four)
    ps.updatePrefixDatabase(three)
    dbs["1"].adjacencies[1].isOverloaded = True
    dbs["3"].adjacencies[2].isOverloaded = True
    assert ls.updateAdjacencyDatabase(dbs["1"])[0]
    assert ls.updateAdjacencyDatabase(dbs["3"])[0]
    rm = get_route_map(s, ["1", "2", "3", "4"], areas, ps)
    assert len(rm) == 44
    exp = {
        ("1", 4): [n(k.adj12_1, 22, push(4)), n(k.adj13_1, 22, push(4))],
        ("1", 3): [n(k.adj13_1, 11), n(k.adj12_1, 33, push(3, 4))],
        ("1", 2): [n(k.adj12_1, 11), n(k.adj12_3, 20)],
        ("2", 4): [n(k.adj24_1, 11), n(k.adj21_1, 33, push(4, 3))],
        ("2", 3): [n(k.adj21_1, 22, push(3)), n(k.adj24_1, 22, push(3))],
        ("2", 1): [n(k.adj21_1, 11), n(k.adj21_3, 20)],
        ("3", 4): [n(k.adj34_1, 11), n(k.adj34_3, 20)],
        ("3", 2): [n(k.adj31_1, 22, push(2)), n(k.adj34_1, 22, push(2))],
        ("3", 1): [n(k.adj31_1, 11), n(k.adj34_1, 33, push(1, 2))],
        ("4", 3): [n(k.adj43_1, 11), n(k.adj43_3, 20)],
        ("4", 2): [n(k.adj42_1, 11), n(k.adj43_1, 33, push(2, 1))],
        ("4", 1): [n(k.adj42_1, 22, push(1)), n(k.adj43_1, 22, push(1))],
    }
    addrs = {1: addr1, 2: addr2, 3: addr3, 4: addr4}
    for (node, d), hops in exp.items():
        assert R(rm, node, P(addrs[d])) == NH(*hops), (node, d)


def sc_parallel_ring_ksp2_for_bgp(M):
    """DecisionTest.cpp:3387-3538 (ParallelAdjRing Ksp2EdEcmpForBGP):
    metric-vector best path with per-announcer minNexthop thresholds."""
    s, areas, ls, ps, dbs, pdbs = _par(M, True, True, BGP)
    n = lambda adj, m, act=None: nh(adj, False, m, act, True)  # noqa: E731
    k = KA
    rm = get_route_map(s, ["1"], areas, ps)
    assert R(rm, "1", P(addr2)) == NH(n(k.adj12_1, 11), n(k.adj12_2, 11), n(k.adj12_3, 20))
    dbs["1"].adjacencies[1].isOverloaded = True
    dbs["3"].adjacencies[2].isOverloaded = True
    assert ls.updateAdjacencyDatabase(dbs["1"])[0]
    assert ls.updateAdjacencyDatabase(dbs["3"])[0]
    one, two = pdbs["1"], pdbs["2"]
    one.prefixEntries[0].mv = _mv()
    two.prefixEntries.append(copy.deepcopy(one.prefixEntries[0]))
    ps.updatePrefixDatabase(one)
    ps.updatePrefixDatabase(two)
    rm = get_route_map(s, ["3"], areas, ps)
    assert ("3",) + P(addr1) not in rm
    two.prefixEntries[-1].mv.metrics[4].metric[0] -= 1
    two.prefixEntries[-1].minNexthop = 4
    one.prefixEntries[-1].minNexthop = 2
    ps.updatePrefixDatabase(two)
    ps.updatePrefixDatabase(one)
    rm = get_route_map(s, ["3"], areas, ps)
    assert R(rm, "3", P(addr1)) == NH(n(k.adj31_1, 11), n(k.adj34_1, 33, push(1, 2)))
    two.prefixEntries[-1].minNexthop = 2
    one.prefixEntries[-1].minNexthop = 4
    ps.updatePrefixDatabase(two)
    ps.updatePrefixDatabase(one)
    rm = get_route_map(s, ["3"], areas, ps)
    assert ("3",) + P(addr1) not in rm
    two.prefixEntries[-1].minNexthop = None
    one.prefixEntries[-1].minNexthop = None
    ps.updatePrefixDatabase(two)
    ps.updatePrefixDatabase(one)
    two.prefixEntries[-1].mv.metrics[4].metric[0] += 2
    ps.updatePrefixDatabase(two)
    rm = get_route_map(s, ["3"], areas, ps)
    assert R(rm, "3", P(addr1)) == NH(n(k.adj31_1, 22, push(2)), n(k.adj34_1, 22, push(2)))
    two.prefixEntries[-1].mv.metrics[4].isBestPathTieBreaker = True
    one.prefixEntries[-1].mv.metrics[4].isBestPathTieBreaker = True
    ps.updatePrefixDatabase(two)
    ps.updatePrefixDatabase(one)
    rm = get_route_map(s, ["3"], areas, ps)
    assert R(rm, "3", P(addr1)) == NH(n(k.adj31_1, 22, push(2)), n(k.adj34_1, 22, push(2)), n(k.adj31_1, 11))


# ------------------------------------------------------------- Ip2MplsRoutes


def sc_ip2mpls_routes(M):
    """DecisionTest.cpp:3558-3844 (DecisionTest.Ip2MplsRoutes, LFA on): SR_MPLS
    prefixes with SP_ECMP (k = 1 edge-disjoint paths), an anycast default
    route from nodes 4 and 5, parallel links 1-2, no adjacency labels."""
    s = M.SpfSolver("1", False, True)
    areas, ls = single_area(M)
    ps = M.PrefixState()
    ca = T.createAdjacency
    adj12_1 = ca("2", "2/1", "1/1", "fe80::2", "192.168.1.2", 10, 0)
    adj12_2 = ca("2", "2/2", "1/2", "fe80::2", "192.168.1.2", 10, 0)
    adj13 = ca("3", "3/1", "1/1", "fe80::3", "192.168.1.3", 10, 0)
    adj21_1 = ca("1", "1/1", "2/1", "fe80::1", "192.168.1.1", 10, 0)
    adj21_2 = ca("1", "1/2", "2/2", "fe80::1", "192.168.1.1", 10, 0)
    adj24 = ca("4", "4/1", "2/1", "fe80::4", "192.168.1.4", 10, 0)
    adj25 = ca("5", "5/1", "2/1", "fe80::5", "192.168.1.5", 10, 0)
    adj31 = ca("1", "1/1", "3/1", "fe80::1", "192.168.1.1", 10, 0)
    adj34 = ca("4", "4/1", "3/1", "fe80::4", "192.168.1.4", 20, 0)
    adj35 = ca("5", "5/1", "3/1", "fe80::5", "192.168.1.5", 10, 0)
    adj42 = ca("2", "2/1", "4/1", "fe80::2", "192.168.1.2", 10, 0)
    adj43 = ca("3", "3/1", "4/1", "fe80::3", "192.168.1.3", 20, 0)
    adj52 = ca("2", "2/1", "5/1", "fe80::2", "192.168.1.2", 10, 0)
    adj53 = ca("3", "3/1", "5/1", "fe80::3", "192.168.1.3", 10, 0)
    dbs = [
        T.createAdjDb("1", [adj12_1, adj12_2, adj13], 1),
        T.createAdjDb("2", [adj21_1, adj21_2, adj24, adj25], 2),
        T.createAdjDb("3", [adj31, adj34, adj35], 3),
        T.createAdjDb("4", [adj42, adj43], 4),
        T.createAdjDb("5", [adj52, adj53], 5),
    ]
    assert not ls.updateAdjacencyDatabase(dbs[0])[0]
    for db in dbs[1:]:
        assert ls.updateAdjacencyDatabase(db)[0]
    dflt = T.toIpPrefix("::/0")
    SR = T.PrefixForwardingType.SR_MPLS
    LO = T.PrefixType.LOOPBACK
    for node, pfx in (("1", addr1), ("2", addr2), ("3", addr3), ("4", dflt), ("5", dflt)):
        assert ps.updatePrefixDatabase(T.createPrefixDb(node, [T.createPrefixEntry(pfx, LO, "", SR)]))
    rm = get_route_map(s, ["1", "2", "3", "4", "5"], areas, ps)
    assert len(rm) == 40
    u = lambda adj, m, act=None: nh(adj, False, m, act, True)  # noqa: E731
    m = lambda adj, mt, act: nh(adj, False, mt, act)  # noqa: E731
    php = labelPhpAction
    for node in "12345":
        validate_pop_label_route(rm, node, int(node))
    D = ("P", dflt.key())
    # router 1
    assert R(rm, "1", P(addr2)) == NH(u(adj12_2, 10), u(adj12_1, 10))
    assert R(rm, "1", P(addr3)) == NH(u(adj13, 10))
    assert R(rm, "1", D) == NH(u(adj13, 20, push(5)), u(adj12_1, 20, push(4)), u(adj12_1, 20, push(5)))
    assert R(rm, "1", L(2)) == NH(m(adj12_1, 10, php), m(adj12_2, 10, php))
    assert R(rm, "1", L(3)) == NH(m(adj13, 10, php))
    assert R(rm, "1", L(4)) == NH(m(adj12_1, 20, swap(4)), m(adj12_2, 20, swap(4)), m(adj13, 30, swap(4)))
    assert R(rm, "1", L(5)) == NH(m(adj12_1, 20, swap(5)), m(adj12_2, 20, swap(5)), m(adj13, 20, swap(5)))
    # router 2
    assert R(rm, "2", P(addr1)) == NH(u(adj21_1, 10), u(adj21_2, 10))
    assert R(rm, "2", P(addr3)) == NH(u(adj21_1, 20, push(3)), u(adj25, 20, push(3)))
    assert R(rm, "2", D) == NH(u(adj24, 10), u(adj25, 10))
    assert R(rm, "2", L(1)) == NH(m(adj21_1, 10, php), m(adj21_2, 10, php))
    assert R(rm, "2", L(3)) == NH(
        m(adj21_1, 20, swap(3)), m(adj21_2, 20, swap(3)), m(adj25, 20, swap(3)), m(adj24, 30, swap(3)))
    assert R(rm, "2", L(4)) == NH(m(adj24, 10, php))
    assert R(rm, "2", L(5)) == NH(m(adj25, 10, php))
    # router 3
    assert R(rm, "3", P(addr1)) == NH(u(adj31, 10))
    assert R(rm, "3", P(addr2)) == NH(u(adj31, 20, push(2)), u(adj35, 20, push(2)))
    assert R(rm, "3", D) == NH(u(adj34, 20), u(adj35, 10))
    assert R(rm, "3", L(1)) == NH(m(adj31, 10, php), m(adj34, 40, swap(1)))
    assert R(rm, "3", L(2)) == NH(m(adj31, 20, swap(2)), m(adj35, 20, swap(2)), m(adj34, 30, swap(2)))
    assert R(rm, "3", L(4)) == NH(m(adj34, 20, php), m(adj31, 30, swap(4)), m(adj35, 30, swap(4)))
    assert R(rm, "3", L(5)) == NH(m(adj35, 10, php), m(adj34, 40, swap(5)))
    # router 4
    assert R(rm, "4", P(addr1)) == NH(u(adj42, 20, push(1)))
    assert R(rm, "4", P(addr2)) == NH(u(adj42, 10))
    assert R(rm, "4", P(addr3)) == NH(u(adj43, 20))
    assert R(rm, "4", L(1)) == NH(m(adj42, 20, swap(1)), m(adj43, 30, swap(1)))
    assert R(rm, "4", L(2)) == NH(m(adj42, 10, php), m(adj43, 40, swap(2)))
    assert R(rm, "4", L(3)) == NH(m(adj43, 20, php), m(adj42, 30, swap(3)))
    assert R(rm, "4", L(5)) == NH(m(adj42, 20, swap(5)), m(adj43, 30, swap(5)))
    # router 5
    assert R(rm, "5", P(addr1)) == NH(u(adj52, 20, push(1)), u(adj53, 20, push(1)))
    assert R(rm, "5", P(addr2)) == NH(u(adj52, 10))
    assert R(rm, "5", P(addr3)) == NH(u(adj53, 10))
    assert R(rm, "5", L(1)) == NH(m(adj52, 20, swap(1)), m(adj53, 20, swap(1)))
    assert R(rm, "5", L(2)) == NH(m(adj52, 10, php))
    assert R(rm, "5", L(3)) == NH(m(adj53, 10, php))
    assert R(rm, "5", L(4)) == NH(m(adj52, 20, swap(4)), m(adj53, 30, swap(4)))


# --------------------------------------------------------------------- Grid


def sc_grid_shortest_path_large(M):
    """DecisionTest.cpp:3920-4010 (GridTopologyFixture) for n = 10..16 (the
    reference range is 2..16 step 2; 2..8 are in tests/known_answers.py):
    route count 2n^4+3n^2-4n and Manhattan metrics corner to corner."""
    import random

    rnd = random.Random(11)
    for n in (10, 12, 14, 16):
        areas, ps, pfx = KA._grid(M, n)
        s = M.SpfSolver("1", False, False)
        nodes = [str(i) for i in range(n * n)]
        rm = get_route_map(s, nodes, areas, ps)
        assert len(rm) == 2 * n**4 + 3 * n**2 - 4 * n, n

        def dist(a, b):
            return abs(a % n - b % n) + abs(a // n - b // n)

        pairs = [(0, n * n - 1), (n - 1, n * (n - 1)), (0, rnd.randrange(1, n * n))]
        pairs += [(rnd.randrange(n * n), rnd.randrange(n * n)) for _ in range(4)]
        for a, b in pairs:
            if a == b:
                continue
            hops = R(rm, str(a), P(pfx(b)))
            assert hops and all(h[4] == dist(a, b) for h in hops), (n, a, b)


# ------------------------------------------------ DecisionTestFixture cases


class DecisionSim:
    """Decision's ingest + getDecisionRouteDb without its event loop (see the
    module docstring).  `wire=True` feeds the engine's PublicationIngest with
    CompactProtocol blobs (Decision.cpp:1631-1763) instead of objects."""

    def __init__(self, M, my="1", lfa=True, wire=False):
        self.M = M
        self.areas = M.AreaLinkStates()
        self.ps = M.PrefixState()
        self.solver = M.SpfSolver(my, False, lfa)
        self.wire = wire
        self.ingest = M.PublicationIngest(my) if wire else None
        self.known = set()

    def publish(self, area=kDefaultArea, adj=(), prefix=()):
        if self.wire:
            kv = {f"adj:{d.thisNodeName}": self.M.compact_encode_adj_db(d) for d in adj}
            kv.update({f"prefix:{p.thisNodeName}": self.M.compact_encode_prefix_db(p) for p in prefix})
            self.ingest.processPublication(self.areas, self.ps, area, kv)
            return
        if area not in self.known:
            self.areas.add(area)
            self.known.add(area)
        for d in adj:
            d = copy.deepcopy(d)
            d.area = area
            self.areas[area].updateAdjacencyDatabase(d)
        for p in prefix:
            p = copy.deepcopy(p)
            p.area = area
            self.ps.updatePrefixDatabase(p)

    def route_db(self, node):
        """getDecisionRouteDb (Decision.cpp:1437-1462): an empty database for a
        node in no area."""
        db = self.solver.buildRouteDbObject(node, self.areas, self.ps)
        return db if db is not None else self.M.DecisionRouteDb()

    def unicast(self, node):
        return self.route_db(node).to_dict()["unicast"]


def _adjv(node, adjs, overloaded=False, nodeId=0):
    """createAdjValue (DecisionTest.cpp:4112-4129) as the database it carries."""
    db = T.createAdjDb(node, copy.deepcopy(list(adjs)), nodeId)
    db.isOverloaded = overloaded
    return db


def _pfxv(node, prefixes, area=kDefaultArea):
    """createPrefixValue (DecisionTest.cpp:4146-4157)."""
    return T.createPrefixDb(node, [T.createPrefixEntry(p) for p in prefixes], area)


def _routes(uni, area_default=kDefaultArea):
    return {k: v["nexthops"] for k, v in uni.items()}


def sc_decision_multi_area_best_path(M, wire=False):
    """DecisionTest.cpp:4503-4638 (MultiAreaBestPathCalculation): area A =
    1-2, 2-4; area B = 1-3, 3-4; per-area next hops and the cross-area ECMP
    once "1" originates addr1 into both areas."""
    d = DecisionSim(M, wire=wire)
    d.publish("A", adj=[_adjv("1", [adj12], False, 1), _adjv("2", [adj21, adj24], False, 2),
                        _adjv("4", [adj42], False, 4)],
              prefix=[_pfxv("1", [addr1], "A"), _pfxv("2", [addr2], "A")])
    d.publish("B", adj=[_adjv("1", [adj13], False, 1), _adjv("3", [adj31, adj34], False, 3),
                        _adjv("4", [adj43], False, 4)],
              prefix=[_pfxv("3", [addr3], "B"), _pfxv("4", [addr4], "B")])
    f = lambda adj, m, area: nh(adj, False, m, None, False, area)  # noqa: E731
    assert _routes(d.unicast("1")) == {
        addr2.key(): NH(f(adj12, 10, "A")),
        addr3.key(): NH(f(adj13, 10, "B")),
        addr4.key(): NH(f(adj13, 20, "B")),
    }
    assert _routes(d.unicast("2")) == {addr1.key(): NH(f(adj21, 10, "A"))}
    assert _routes(d.unicast("3")) == {addr4.key(): NH(f(adj34, 10, "B"))}
    assert _routes(d.unicast("4")) == {
        addr2.key(): NH(f(adj42, 10, "A")),
        addr3.key(): NH(f(adj43, 10, "B")),
        addr1.key(): NH(f(adj42, 20, "A")),
    }
    d.publish("B", prefix=[_pfxv("1", [addr1], "B")])
    assert d.unicast("3")[addr1.key()]["nexthops"] == NH(f(adj31, 10, "B"))
    assert d.unicast("4")[addr1.key()]["nexthops"] == NH(f(adj43, 20, "B"), f(adj42, 20, "A"))


def sc_decision_parallel_links(M, wire=False):
    """DecisionTest.cpp:4882-4982 (ParallelLinks): parallel 1-2 links of
    metric 100 / 800; each publication changes exactly one route of node 1
    and the route delta is getRouteDelta of the dumps before and after."""
    ca = T.createAdjacency
    adj12_1 = ca("2", "1/2-1", "2/1-1", "fe80::2", "192.168.0.2", 100, 0)
    adj12_2 = ca("2", "1/2-2", "2/1-2", "fe80::2", "192.168.0.2", 800, 0)
    adj21_1 = ca("1", "2/1-1", "1/2-1", "fe80::1", "192.168.0.1", 100, 0)
    adj21_2 = ca("1", "2/1-2", "1/2-2", "fe80::1", "192.168.0.1", 800, 0)
    d = DecisionSim(M, wire=wire)

    def step(expect, **pub):
        before = d.route_db("1")
        d.publish(**pub)
        after = d.route_db("1")
        delta = M.getRouteDelta(after, before)
        assert len(delta["unicastRoutesToUpdate"]) == 1, delta
        assert delta["unicastRoutesToDelete"] == []
        assert after.to_dict()["unicast"][addr2.key()]["nexthops"] == NH(*[nh(a, False, m) for a, m in expect])

    step([(adj12_1, 100), (adj12_2, 800)],
         adj=[_adjv("1", [adj12_1, adj12_2]), _adjv("2", [adj21_1, adj21_2])],
         prefix=[_pfxv("1", [addr1]), _pfxv("2", [addr2])])
    step([(adj12_2, 800)], adj=[_adjv("2", [adj21_2])])
    step([(adj12_1, 100), (adj12_2, 800)], adj=[_adjv("2", [adj21_1, adj21_2])])
    ov = copy.deepcopy(adj21_1)
    ov.isOverloaded = True
    step([(adj12_2, 800)], adj=[_adjv("2", [ov, adj21_2])])


def sc_decision_duplicate_prefixes(M, wire=False):
    """DecisionTest.cpp:5374-5479 (DuplicatePrefixes): addr2 anycast from
    nodes 2 and 3; after draining 2 and 4 node 1 routes addr2 via 3 only but
    keeps the unicast route to 4."""
    ca = T.createAdjacency
    a14 = ca("4", "1/4", "4/1", "fe80::4", "192.168.0.4", 5, 0)
    a41 = ca("1", "4/1", "1/4", "fe80::1", "192.168.0.1", 5, 0)
    a12 = ca("2", "1/2", "2/1", "fe80::2", "192.168.0.2", 10, 0)
    a21 = ca("1", "2/1", "1/2", "fe80::1", "192.168.0.1", 10, 0)
    d = DecisionSim(M, wire=wire)
    d.publish(adj=[_adjv("1", [a14, a12, adj13]), _adjv("2", [a21]), _adjv("3", [adj31]),
                   _adjv("4", [a41])],
              prefix=[_pfxv("1", [addr1]), _pfxv("2", [addr2]), _pfxv("3", [addr2]),
                      _pfxv("4", [addr4])])
    u = {n: d.unicast(n) for n in "1234"}
    assert all(len(u[n]) == 2 for n in "1234")
    assert u["1"][addr2.key()]["nexthops"] == NH(nh(a12, False, 10), nh(adj13, False, 10))
    assert u["2"][addr1.key()]["nexthops"] == NH(nh(a21, False, 10))
    assert u["3"][addr1.key()]["nexthops"] == NH(nh(adj31, False, 10))
    assert u["4"][addr2.key()]["nexthops"] == NH(nh(a41, False, 15))
    d.publish(adj=[_adjv("2", [a21], True), _adjv("4", [a41], True)])
    u1 = d.unicast("1")
    assert u1[addr2.key()]["nexthops"] == NH(nh(adj13, False, 10))
    assert u1[addr4.key()]["nexthops"] == NH(nh(a14, False, 5))


def sc_fb303_counter_names(M):
    """The fb303-exported names the reference tests read: DecisionTest.cpp:
    1970 (decision.spf_runs.count == 16 on the KSP2 ring) and :1794
    (decision.duplicate_node_label.count.60).  Engine only (the oracle keeps
    raw keys)."""
    if not hasattr(M, "get_fb303_counters"):
        return
    M.reset_counters()
    s, areas, ls, ps, dbs = KA.ring_setup(M, False, True, True)
    get_route_map(s, ["1", "2", "3", "4"], areas, ps)
    c = M.get_fb303_counters()
    assert c["decision.spf_runs.count"] == 16
    assert c["decision.route_build_runs.count"] == 4
    assert "decision.spf_ms.avg" in c and "decision.route_build_ms.avg.60" in c
    dbs["1"].nodeLabel = 2
    ls.updateAdjacencyDatabase(dbs["1"])
    M.reset_counters()
    s.buildRouteDb("1", areas, ps)
    assert M.get_fb303_counters()["decision.duplicate_node_label.count.60"] == 1
