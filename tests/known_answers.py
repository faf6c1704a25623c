"""Known answers of the reference's own tests, restated as scenarios.

Each `sc_*` function runs against a module `M` that exposes the LinkState /
AreaLinkStates / PrefixState / SpfSolver surface — the CPU oracle
(oracle._oracle_ref) in the "not gpu" suite, and the MI355X engine
(openr_amd._openr_spf) in the gpu suite — and asserts the reference's
expected values.  Fixtures and expectations are transcribed from
openr/decision/tests/DecisionTest.cpp and LinkStateTest.cpp (cited per
scenario; paths relative to the reference repo root).
"""

from __future__ import annotations

from openr_amd import thrift as T

A = T.MplsActionCode
kDefaultArea = T.kDefaultArea

# ------------------------------------------ DecisionTest.cpp:47-137 fixtures
adj12 = T.createAdjacency("2", "1/2", "2/1", "fe80::2", "192.168.0.2", 10, 100002)
adj13 = T.createAdjacency("3", "1/3", "3/1", "fe80::3", "192.168.0.3", 10, 100003)
adj14 = T.createAdjacency("4", "1/4", "4/1", "fe80::4", "192.168.0.4", 10, 100004)
adj12_old_1 = T.createAdjacency("2", "1/2", "2/1", "fe80::2", "192.168.0.2", 10, 1000021)
adj12_old_2 = T.createAdjacency("2", "1/2", "2/1", "fe80::2", "192.168.0.2", 20, 1000022)
adj13_old = T.createAdjacency("3", "1/3", "3/1", "fe80::3", "192.168.0.3", 10, 1000031)
adj21 = T.createAdjacency("1", "2/1", "1/2", "fe80::1", "192.168.0.1", 10, 100001)
adj21_old_1 = T.createAdjacency("1", "2/1", "1/2", "fe80::1", "192.168.0.1", 10, 1000011)
adj23 = T.createAdjacency("3", "2/3", "3/2", "fe80::3", "192.168.0.3", 10, 100003)
adj24 = T.createAdjacency("4", "2/4", "4/2", "fe80::4", "192.168.0.4", 10, 100004)
adj31 = T.createAdjacency("1", "3/1", "1/3", "fe80::1", "192.168.0.1", 10, 100001)
adj31_old = T.createAdjacency("1", "3/1", "1/3", "fe80::1", "192.168.0.1", 10, 1000011)
adj32 = T.createAdjacency("2", "3/2", "2/3", "fe80::2", "192.168.0.2", 10, 100002)
adj34 = T.createAdjacency("4", "3/4", "4/3", "fe80::4", "192.168.0.4", 10, 100004)
adj41 = T.createAdjacency("1", "4/1", "1/4", "fe80::1", "192.168.0.1", 10, 100001)
adj42 = T.createAdjacency("2", "4/2", "2/4", "fe80::2", "192.168.0.2", 10, 100002)
adj43 = T.createAdjacency("3", "4/3", "3/4", "fe80::3", "192.168.0.3", 10, 100003)

addr1 = T.toIpPrefix("::ffff:10.1.1.1/128")
addr2 = T.toIpPrefix("::ffff:10.2.2.2/128")
addr3 = T.toIpPrefix("::ffff:10.3.3.3/128")
addr4 = T.toIpPrefix("::ffff:10.4.4.4/128")
addr1V4 = T.toIpPrefix("10.1.1.1/32")
addr2V4 = T.toIpPrefix("10.2.2.2/32")
addr3V4 = T.toIpPrefix("10.3.3.3/32")
addr4V4 = T.toIpPrefix("10.4.4.4/32")

prefixDb1 = T.createPrefixDb("1", [T.createPrefixEntry(addr1)])
prefixDb2 = T.createPrefixDb("2", [T.createPrefixEntry(addr2)])
prefixDb3 = T.createPrefixDb("3", [T.createPrefixEntry(addr3)])
prefixDb4 = T.createPrefixDb("4", [T.createPrefixEntry(addr4)])
prefixDb1V4 = T.createPrefixDb("1", [T.createPrefixEntry(addr1V4)])
prefixDb2V4 = T.createPrefixDb("2", [T.createPrefixEntry(addr2V4)])
prefixDb3V4 = T.createPrefixDb("3", [T.createPrefixEntry(addr3V4)])
prefixDb4V4 = T.createPrefixDb("4", [T.createPrefixEntry(addr4V4)])

labelPopAction = T.createMplsAction(A.POP_AND_LOOKUP)
labelPhpAction = T.createMplsAction(A.PHP)


def swap(label):
    return T.createMplsAction(A.SWAP, label)


def push(*labels):
    return T.createMplsAction(A.PUSH, None, list(labels))


labelPopNextHop = T.createNextHop(
    T.toBinaryAddress("::"), None, 0, labelPopAction, False, kDefaultArea
)


def nh(adj, isV4, metric, action=None, nonShortest=False, area=kDefaultArea):
    return T.createNextHopFromAdj(adj, isV4, metric, action, nonShortest, area).key()


def NH(*nhs):
    return frozenset(nhs)


# ------------------------------------------------------------- helpers


def P(prefix):
    return ("P", prefix.key())


def L(label):
    return ("L", int(label))


def fill_route_map(node, rm, db):
    """DecisionTest.cpp:205-232 (fillRouteMap)."""
    for pkey, e in db["unicast"].items():
        rm.setdefault((node,) + ("P", pkey), set()).update(e["nexthops"])
    for label, nhs in db["mpls"].items():
        rm.setdefault((node,) + ("L", int(label)), set()).update(nhs)


def get_route_map(solver, nodes, areas, ps):
    """DecisionTest.cpp:256-274 (getRouteMap)."""
    rm = {}
    for n in nodes:
        db = solver.buildRouteDb(n, areas, ps)
        if db is None:
            continue
        fill_route_map(n, rm, db)
    return {k: frozenset(v) for k, v in rm.items()}


def R(rm, node, key):
    return rm.get((node,) + key, frozenset())


def validate_adj_label_routes(rm, node, adjs):
    """DecisionTest.cpp:295-308."""
    for adj in adjs:
        assert R(rm, node, L(adj.adjLabel)) == NH(
            nh(adj, False, adj.metric, labelPhpAction)
        ), (node, adj.adjLabel)


def validate_pop_label_route(rm, node, label):
    """DecisionTest.cpp:310-317."""
    assert R(rm, node, L(label)) == NH(labelPopNextHop.key())


def single_area(M):
    areas = M.AreaLinkStates()
    ls = areas.add(kDefaultArea)
    return areas, ls


def counters(M):
    return M.get_counters()


# ------------------------------------------------------- LinkStateTest.cpp


def sc_linkstate_basic_operation(M):
    """LinkStateTest.cpp:139-200."""
    n1, n2, n3 = "node1", "node2", "node3"
    a12 = T.createAdjacency(n2, "if2", "if1", "fe80::2", "10.0.0.2", 1, 1, 1)
    a13 = T.createAdjacency(n3, "if3", "if1", "fe80::3", "10.0.0.3", 1, 1, 1)
    a21 = T.createAdjacency(n1, "if1", "if2", "fe80::1", "10.0.0.1", 1, 1, 1)
    a23 = T.createAdjacency(n3, "if3", "if2", "fe80::3", "10.0.0.3", 1, 1, 1)
    a31 = T.createAdjacency(n1, "if1", "if3", "fe80::1", "10.0.0.1", 1, 1, 1)
    a32 = T.createAdjacency(n2, "if2", "if3", "fe80::2", "10.0.0.2", 1, 1, 1)
    l1 = tuple(sorted([(n1, "if2"), (n2, "if1")]))
    l2 = tuple(sorted([(n2, "if3"), (n3, "if2")]))
    l3 = tuple(sorted([(n3, "if1"), (n1, "if3")]))
    db1 = T.createAdjDb(n1, [a12, a13], 1)
    db2 = T.createAdjDb(n2, [a21, a23], 2)
    db3 = T.createAdjDb(n3, [a31, a32], 3)
    ls = M.LinkState(kDefaultArea)
    assert ls.getArea() == kDefaultArea
    assert not ls.updateAdjacencyDatabase(db1, 0, 0)[0]
    assert ls.updateAdjacencyDatabase(db2, 0, 0)[0]
    assert ls.updateAdjacencyDatabase(db3, 0, 0)[0]

    def links(n):
        return sorted(l.key() for l in ls.linksFromNode(n))

    assert links(n1) == sorted([l1, l3])
    assert links(n2) == sorted([l1, l2])
    assert links(n3) == sorted([l2, l3])
    assert links("node4") == []
    assert not ls.isNodeOverloaded(n1)
    db1.isOverloaded = True
    assert ls.updateAdjacencyDatabase(db1, 0, 0)[0]
    assert ls.isNodeOverloaded(n1)
    assert not ls.updateAdjacencyDatabase(db1, 0, 0)[0]
    db1.isOverloaded = False
    assert ls.updateAdjacencyDatabase(db1, 0, 0)[0]
    assert not ls.isNodeOverloaded(n1)
    db1 = T.createAdjDb(n1, [a13], 1)
    assert ls.updateAdjacencyDatabase(db1, 0, 0)[0]
    assert links(n1) == [l3]
    assert links(n2) == [l2]
    assert links(n3) == sorted([l2, l3])
    assert ls.deleteAdjacencyDatabase(n1)[0]
    assert links(n1) == []
    assert links(n2) == [l2]
    assert links(n3) == [l2]


def sc_linkstate_path_a_in_path_b(M):
    """LinkStateTest.cpp:202-242."""
    l1 = M.Link(kDefaultArea, "1", "1/2", "2", "2/1")
    l2 = M.Link(kDefaultArea, "2", "2/3", "3", "3/2")
    l3 = M.Link(kDefaultArea, "1", "1/3", "3", "3/1")
    f = M.LinkState.pathAInPathB
    p1, p2 = [], []
    assert f(p1, p2) and f(p2, p1)
    p1.append(l1)
    assert not f(p1, p2) and f(p2, p1)
    p2.append(l1)
    assert f(p1, p2) and f(p2, p1)
    p1.append(l2)
    assert not f(p1, p2) and f(p2, p1)
    p1.append(l3)
    p2.append(l2)
    assert not f(p1, p2) and f(p2, p1)
    p1, p2 = [l3, l2], [l1]
    assert not f(p1, p2) and not f(p2, p1)


def link_state_from_map(M, adj_map):
    """DecisionTestUtils.cpp:16-55 (getLinkState): iterate the std::unordered_map
    in libstdc++ order (oracle helper), parallel adjacencies numbered."""
    from oracle import _oracle_ref as O

    ls = M.LinkState(kDefaultArea)
    for node in O.cxx_unordered_int_order(list(adj_map.keys())):
        adjs = []
        num_par = {}
        for item in adj_map[node]:
            adj, weight = item if isinstance(item, tuple) else (item, 1)
            k = num_par.get(adj, 0)
            num_par[adj] = k + 1
            bottom, top = adj & 0xFF, (adj & 0xFF00) >> 8
            adjs.append(
                T.createAdjacency(
                    f"{adj}",
                    f"{node}/{adj}/{k}",
                    f"{adj}/{node}/{k}",
                    f"fe80::{top:02x}{bottom:02x}",
                    f"192.168.{top}.{bottom}",
                    weight,
                    (node << 16) + adj,
                )
            )
        ls.updateAdjacencyDatabase(T.createAdjDb(f"{node}", adjs, node), 0, 0)
    return ls


def sc_linkstate_kth_paths(M):
    """LinkStateTest.cpp:244-316."""
    ls = link_state_from_map(
        M,
        {
            1: [(2, 10), (3, 5)],
            2: [(1, 10), (4, 15), (4, 35)],
            3: [(1, 5), (4, 20)],
            4: [(2, 15), (3, 20), (2, 35)],
        },
    )
    first = ls.getKthPaths("2", "4", 1)
    assert len(first) == 1 and len(first[0]) == 1
    assert first[0][0].getMetricFromNode("2") == 15
    second = ls.getKthPaths("2", "4", 2)
    assert sorted(len(p) for p in second) == [1, 3]
    for path in second:
        nxt, dist = "2", 0
        for link in path:
            dist += link.getMetricFromNode(nxt)
            nxt = link.getOtherNodeName(nxt)
        assert dist == 35

    ls = link_state_from_map(
        M,
        {
            1: [2, 2, 3, 3, 4, 4],
            2: [1, 1, 3, 3, 4, 4],
            3: [1, 1, 2, 2, 4, 4],
            4: [1, 1, 2, 2, 3, 3],
        },
    )
    first = ls.getKthPaths("2", "4", 1)
    assert len(first) == 2 and all(len(p) == 1 for p in first)
    second = ls.getKthPaths("2", "4", 2)
    assert len(second) == 4 and all(len(p) == 2 for p in second)
    seen = set()
    for path in list(first) + list(second):
        for link in path:
            assert link.key() not in seen
            seen.add(link.key())


def sc_linkstate_hop_counts(M):
    """LinkStateTest.cpp:318-377."""
    ls = link_state_from_map(M, {1: [2, 3], 2: [1, 4], 3: [1, 4], 4: [2, 3]})
    assert ls.getHopsFromAToB("1", "2") == 1
    assert ls.getHopsFromAToB("1", "4") == 2
    assert ls.getMaxHopsToNode("1") == 2
    ls = link_state_from_map(M, {1: [2], 2: [1, 3], 3: [2, 4], 4: [3, 5], 5: [4]})
    assert ls.getHopsFromAToB("1", "2") == 1
    assert ls.getHopsFromAToB("1", "4") == 3
    assert ls.getHopsFromAToB("2", "3") == 1
    assert ls.getMaxHopsToNode("1") == 4
    assert ls.getMaxHopsToNode("2") == 3
    assert ls.getMaxHopsToNode("3") == 2
    ls = link_state_from_map(M, {1: [2], 2: [1, 3], 3: [2, 4], 4: [3], 5: []})
    assert ls.getHopsFromAToB("1", "5") is None
    assert ls.getHopsFromAToB("2", "3") == 1
    assert ls.getMaxHopsToNode("1") == 3
    assert ls.getMaxHopsToNode("5") == 0


# -------------------------------------------------------- DecisionTest.cpp


def sc_unreachable_nodes(M):
    """DecisionTest.cpp:364-398."""
    areas, ls = single_area(M)
    ps = M.PrefixState()
    s = M.SpfSolver("1", False, False)
    assert not ls.updateAdjacencyDatabase(T.createAdjDb("1", [], 0))[0]
    assert not ls.updateAdjacencyDatabase(T.createAdjDb("2", [], 0))[0]
    assert ps.updatePrefixDatabase(prefixDb1)
    assert ps.updatePrefixDatabase(prefixDb2)
    for node in ["1", "2"]:
        db = s.buildRouteDb(node, areas, ps)
        assert db is not None
        assert len(db["unicast"]) == 0 and len(db["mpls"]) == 0


def sc_missing_neighbor_adjdb(M):
    """DecisionTest.cpp:405-430."""
    areas, ls = single_area(M)
    ps = M.PrefixState()
    s = M.SpfSolver("1", False, False)
    assert not ls.updateAdjacencyDatabase(T.createAdjDb("1", [adj12], 0))[0]
    ps.updatePrefixDatabase(prefixDb1)
    ps.updatePrefixDatabase(prefixDb2)
    db = s.buildRouteDb("1", areas, ps)
    assert len(db["unicast"]) == 0 and len(db["mpls"]) == 0


def sc_empty_neighbor_adjdb(M):
    """DecisionTest.cpp:438-466."""
    areas, ls = single_area(M)
    ps = M.PrefixState()
    s = M.SpfSolver("1", False, False)
    assert not ls.updateAdjacencyDatabase(T.createAdjDb("1", [adj12], 0))[0]
    assert not ls.updateAdjacencyDatabase(T.createAdjDb("2", [], 0))[0]
    ps.updatePrefixDatabase(prefixDb1)
    ps.updatePrefixDatabase(prefixDb2)
    assert len(s.buildRouteDb("1", areas, ps)["unicast"]) == 0
    assert len(s.buildRouteDb("2", areas, ps)["unicast"]) == 0


def sc_unknown_node(M):
    """DecisionTest.cpp:471-486."""
    areas, _ = single_area(M)
    ps = M.PrefixState()
    s = M.SpfSolver("1", False, False)
    assert s.buildRouteDb("1", areas, ps) is None
    assert s.buildRouteDb("2", areas, ps) is None


def sc_adjacency_update(M):
    """DecisionTest.cpp:491-622."""
    import copy

    db1 = T.createAdjDb("1", [copy.deepcopy(adj12)], 1)
    db2 = T.createAdjDb("2", [copy.deepcopy(adj21)], 2)
    areas, ls = single_area(M)
    ps = M.PrefixState()
    s = M.SpfSolver("1", False, False)
    r = ls.updateAdjacencyDatabase(db1)
    assert not r[0] and r[2]
    r = ls.updateAdjacencyDatabase(db2)
    assert r[0] and r[2]
    ps.updatePrefixDatabase(prefixDb1)
    ps.updatePrefixDatabase(prefixDb2)

    def check():
        for node in ["1", "2"]:
            db = s.buildRouteDb(node, areas, ps)
            assert len(db["unicast"]) == 1 and len(db["mpls"]) == 3

    check()
    db1.adjacencies[0].nextHopV6 = T.toBinaryAddress("fe80::1234:b00c")
    r = ls.updateAdjacencyDatabase(db1)
    assert not r[0] and r[1]
    check()
    db2.adjacencies[0].nextHopV6 = T.toBinaryAddress("fe80::5678:b00c")
    r = ls.updateAdjacencyDatabase(db2)
    assert not r[0] and r[1]
    check()
    db1.adjacencies[0].adjLabel = 111
    r = ls.updateAdjacencyDatabase(db1)
    assert not r[0] and r[1]
    db2.adjacencies[0].adjLabel = 222
    r = ls.updateAdjacencyDatabase(db2)
    assert not r[0] and r[1]
    db1.nodeLabel = 11
    assert ls.updateAdjacencyDatabase(db1) == (False, False, True)
    db2.nodeLabel = 22
    assert ls.updateAdjacencyDatabase(db2) == (False, False, True)


def sc_mpls_routes_basic(M):
    """DecisionTest.cpp:629-670 (MplsRoutes.BasicTest)."""
    areas, ls = single_area(M)
    ps = M.PrefixState()
    s = M.SpfSolver("1", False, False)
    db1 = T.createAdjDb("1", [adj12], 1)
    db2 = T.createAdjDb("2", [adj23], 0)
    db3 = T.createAdjDb("3", [adj32], 3)
    assert ls.updateAdjacencyDatabase(db1) == (False, False, True)
    assert ls.updateAdjacencyDatabase(db1) == (False, False, False)
    assert ls.updateAdjacencyDatabase(db2) == (False, False, False)
    assert ls.updateAdjacencyDatabase(db3) == (True, False, True)
    rm = get_route_map(s, ["1", "2", "3"], areas, ps)
    assert len(rm) == 5
    validate_pop_label_route(rm, "1", 1)
    validate_adj_label_routes(rm, "2", [adj23])
    validate_pop_label_route(rm, "3", 3)
    validate_adj_label_routes(rm, "3", [adj32])


def sc_connectivity(M):
    """DecisionTest.cpp:1022-1082 (both partitioned and connected)."""
    for partitioned in (True, False):
        db1 = T.createAdjDb("1", [], 1)
        db2 = T.createAdjDb("2", [adj21, adj23], 2)
        db3 = T.createAdjDb("3", [], 3)
        if not partitioned:
            db1 = T.createAdjDb("1", [adj12], 1)
            db3 = T.createAdjDb("3", [adj32], 3)
        areas, ls = single_area(M)
        ps = M.PrefixState()
        s = M.SpfSolver("1", False, False)
        assert ls.updateAdjacencyDatabase(db1) == (False, False, True)
        assert ls.updateAdjacencyDatabase(db2) == (not partitioned, False, True)
        assert ls.updateAdjacencyDatabase(db3) == (not partitioned, False, True)
        for pdb in (prefixDb1, prefixDb2, prefixDb3):
            ps.updatePrefixDatabase(pdb)
        db = s.buildRouteDb("1", areas, ps)
        found_v6 = addr3.key() in db["unicast"]
        found_label = 3 in db["mpls"]
        assert partitioned == (not found_v6)
        assert partitioned == (not found_label)


def sc_overload_node(M):
    """DecisionTest.cpp:1084-1174."""
    areas, ls = single_area(M)
    ps = M.PrefixState()
    s = M.SpfSolver("1", False, False)
    db1 = T.createAdjDb("1", [adj12], 1)
    db2 = T.createAdjDb("2", [adj21, adj23], 2, True)
    db3 = T.createAdjDb("3", [adj32], 3)
    for pdb in (prefixDb1, prefixDb2, prefixDb3):
        ps.updatePrefixDatabase(pdb)
    assert not ls.updateAdjacencyDatabase(db1)[0]
    assert ls.updateAdjacencyDatabase(db2)[0]
    assert ls.updateAdjacencyDatabase(db3)[0]
    rm = get_route_map(s, ["1", "2", "3"], areas, ps)
    assert len(rm) == 15
    assert R(rm, "1", P(addr2)) == NH(nh(adj12, False, 10))
    assert R(rm, "1", L(2)) == NH(nh(adj12, False, adj12.metric, labelPhpAction))
    validate_pop_label_route(rm, "1", 1)
    validate_adj_label_routes(rm, "1", db1.adjacencies)
    assert R(rm, "2", P(addr3)) == NH(nh(adj23, False, 10))
    assert R(rm, "2", P(addr1)) == NH(nh(adj21, False, 10))
    assert R(rm, "2", L(1)) == NH(nh(adj21, False, adj21.metric, labelPhpAction))
    assert R(rm, "2", L(3)) == NH(nh(adj23, False, adj23.metric, labelPhpAction))
    validate_pop_label_route(rm, "2", 2)
    validate_adj_label_routes(rm, "2", db2.adjacencies)
    assert R(rm, "3", P(addr2)) == NH(nh(adj32, False, 10))
    assert R(rm, "3", L(2)) == NH(nh(adj32, False, adj32.metric, labelPhpAction))
    validate_pop_label_route(rm, "3", 3)
    validate_adj_label_routes(rm, "3", db3.adjacencies)


def sc_compatibility_node(M):
    """DecisionTest.cpp:1181-1297."""
    areas, ls = single_area(M)
    ps = M.PrefixState()
    s = M.SpfSolver("1", False, False)
    db1 = T.createAdjDb("1", [adj12_old_1], 1)
    db2 = T.createAdjDb("2", [adj21_old_1, adj23], 2)
    db3 = T.createAdjDb("3", [adj32, adj31_old], 3)
    for pdb in (prefixDb1, prefixDb2, prefixDb3):
        ps.updatePrefixDatabase(pdb)
    assert not ls.updateAdjacencyDatabase(db2)[0]
    assert ls.updateAdjacencyDatabase(db3)[0]
    assert ls.updateAdjacencyDatabase(db1)[0]
    db1 = T.createAdjDb("1", [adj12_old_1, adj13_old], 1)
    assert ls.updateAdjacencyDatabase(db1)[0]
    db1 = T.createAdjDb("1", [adj12_old_2, adj13_old], 1)
    assert ls.updateAdjacencyDatabase(db1)[0]
    rm = get_route_map(s, ["1", "2", "3"], areas, ps)
    assert len(rm) == 21
    assert R(rm, "1", P(addr2)) == NH(
        nh(adj12_old_2, False, 20), nh(adj13_old, False, 20)
    )
    assert R(rm, "1", P(addr3)) == NH(nh(adj13, False, 10))
    assert R(rm, "1", L(2)) == NH(
        nh(adj12_old_2, False, 20, labelPhpAction), nh(adj13_old, False, 20, swap(2))
    )
    assert R(rm, "1", L(3)) == NH(nh(adj13_old, False, adj13_old.metric, labelPhpAction))
    validate_pop_label_route(rm, "1", 1)
    validate_adj_label_routes(rm, "1", db1.adjacencies)
    assert R(rm, "2", P(addr3)) == NH(nh(adj23, False, 10))
    assert R(rm, "2", P(addr1)) == NH(nh(adj21, False, 10))
    assert R(rm, "2", L(1)) == NH(nh(adj21, False, adj21.metric, labelPhpAction))
    assert R(rm, "2", L(3)) == NH(nh(adj23, False, adj23.metric, labelPhpAction))
    validate_pop_label_route(rm, "3", 3)
    validate_adj_label_routes(rm, "3", db3.adjacencies)
    assert R(rm, "3", P(addr2)) == NH(nh(adj32, False, 10))
    assert R(rm, "3", P(addr1)) == NH(nh(adj31, False, 10))
    assert R(rm, "3", L(1)) == NH(nh(adj31, False, adj31.metric, labelPhpAction))
    assert R(rm, "3", L(2)) == NH(nh(adj32, False, adj32.metric, labelPhpAction))
    db1 = T.createAdjDb("1", [adj12_old_2], 0)
    assert ls.updateAdjacencyDatabase(db1)[0]
    db3 = T.createAdjDb("3", [adj32], 0)
    assert not ls.updateAdjacencyDatabase(db3)[0]
    db1 = T.createAdjDb("1", [adj12_old_2, adj13_old], 0)
    assert not ls.updateAdjacencyDatabase(db1)[0]
