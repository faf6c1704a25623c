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


# ------------------------------------------- SimpleRing (DecisionTest.cpp)
#
#   1 --10-- 2
#   |        |
#   10       10
#   |        |
#   3 --10-- 4
#
# DecisionTest.cpp:1522-1640 (SimpleRingTopologyFixture::CustomSetUp)

bgpAddr1 = T.toIpPrefix("2401:1::10.1.1.1/32")  # DecisionTest.cpp:100


def kspf_db(pdb, minNexthop=None):
    """DecisionTest.cpp:147-180 (createPrefixDbWithKspfAlgo, non-BGP)."""
    entries = []
    for e in pdb.prefixEntries:
        entries.append(
            T.createPrefixEntry(
                e.prefix,
                forwardingType=T.PrefixForwardingType.SR_MPLS,
                forwardingAlgorithm=T.PrefixForwardingAlgorithm.KSP2_ED_ECMP,
                minNexthop=minNexthop,
            )
        )
    return T.createPrefixDb(pdb.thisNodeName, entries)


def ring_setup(M, v4, lfa, ksp2):
    s = M.SpfSolver("1", v4, lfa)
    dbs = {
        "1": T.createAdjDb("1", [adj12, adj13], 1),
        "2": T.createAdjDb("2", [adj21, adj24], 2),
        "3": T.createAdjDb("3", [adj31, adj34], 3),
        "4": T.createAdjDb("4", [adj42, adj43], 4),
    }
    areas, ls = single_area(M)
    assert ls.updateAdjacencyDatabase(dbs["1"]) == (False, False, True)
    for n in ("2", "3", "4"):
        assert ls.updateAdjacencyDatabase(dbs[n]) == (True, False, True)
    ps = M.PrefixState()
    pdbs = (
        (prefixDb1V4, prefixDb2V4, prefixDb3V4, prefixDb4V4)
        if v4
        else (prefixDb1, prefixDb2, prefixDb3, prefixDb4)
    )
    for pdb in pdbs:
        ps.updatePrefixDatabase(kspf_db(pdb) if ksp2 else pdb)
    return s, areas, ls, ps, dbs


def _ring_addr(v4, i):
    return P((addr1V4, addr2V4, addr3V4, addr4V4)[i - 1] if v4 else (addr1, addr2, addr3, addr4)[i - 1])


def _check_ring_ecmp(rm, v4, dbs):
    """DecisionTest.cpp:1642-1765 / 1827-1951: expected routes of every node
    (ShortestPathTest and MultiPathTest expect the same sets on this ring)."""
    a = lambda i: _ring_addr(v4, i)  # noqa: E731
    exp = {
        # node: {dst: [(adj, metric)], ...}
        "1": {4: [(adj12, 20), (adj13, 20)], 3: [(adj13, 10)], 2: [(adj12, 10)]},
        "2": {4: [(adj24, 10)], 3: [(adj21, 20), (adj24, 20)], 1: [(adj21, 10)]},
        "3": {4: [(adj34, 10)], 2: [(adj31, 20), (adj34, 20)], 1: [(adj31, 10)]},
        "4": {3: [(adj43, 10)], 2: [(adj42, 10)], 1: [(adj42, 20), (adj43, 20)]},
    }
    for node, dsts in exp.items():
        for d, hops in dsts.items():
            assert R(rm, node, a(d)) == NH(*[nh(x, v4, m) for x, m in hops]), (node, d)
            act = (lambda m: labelPhpAction) if len(hops) == 1 and hops[0][1] == 10 else (
                lambda m: swap(d)
            )
            assert R(rm, node, L(d)) == NH(
                *[nh(x, False, m, act(m)) for x, m in hops]
            ), (node, "label", d)
        validate_pop_label_route(rm, node, int(node))
        validate_adj_label_routes(rm, node, dbs[node].adjacencies)


def sc_ring_shortest_path(M):
    """DecisionTest.cpp:1642-1765 (ShortestPathTest): 36 routes, spf_runs 4."""
    for v4 in (True, False):
        M.reset_counters()
        s, areas, ls, ps, dbs = ring_setup(M, v4, False, False)
        rm = get_route_map(s, ["1", "2", "3", "4"], areas, ps)
        assert len(rm) == 36
        assert counters(M)["decision.spf_runs"] == 4
        _check_ring_ecmp(rm, v4, dbs)


def sc_ring_multipath_lfa(M):
    """DecisionTest.cpp:1827-1951 (MultiPathTest, LFA on): 36 routes."""
    for v4 in (True, False):
        s, areas, ls, ps, dbs = ring_setup(M, v4, True, False)
        rm = get_route_map(s, ["1", "2", "3", "4"], areas, ps)
        assert len(rm) == 36
        _check_ring_ecmp(rm, v4, dbs)


def sc_ring_ksp2_ed_ecmp(M):
    """DecisionTest.cpp:1953-2138 (Ksp2EdEcmp): 36 routes, spf_runs 16,
    second edge-disjoint paths with PUSH label stacks, then overloads."""
    for v4 in (True, False):
        M.reset_counters()
        s, areas, ls, ps, dbs = ring_setup(M, v4, True, True)
        rm = get_route_map(s, ["1", "2", "3", "4"], areas, ps)
        assert len(rm) == 36
        assert counters(M)["decision.spf_runs"] == 16
        a = lambda i: _ring_addr(v4, i)  # noqa: E731
        n = lambda adj, m, act=None: nh(adj, v4, m, act, True)  # noqa: E731
        exp = {
            ("1", 4): [n(adj12, 20, push(4)), n(adj13, 20, push(4))],
            ("1", 3): [n(adj13, 10), n(adj12, 30, push(3, 4))],
            ("1", 2): [n(adj12, 10), n(adj13, 30, push(2, 4))],
            ("2", 4): [n(adj24, 10), n(adj21, 30, push(4, 3))],
            ("2", 3): [n(adj21, 20, push(3)), n(adj24, 20, push(3))],
            ("2", 1): [n(adj21, 10), n(adj24, 30, push(1, 3))],
            ("3", 4): [n(adj34, 10), n(adj31, 30, push(4, 2))],
            ("3", 2): [n(adj31, 20, push(2)), n(adj34, 20, push(2))],
            ("3", 1): [n(adj31, 10), n(adj34, 30, push(1, 2))],
            ("4", 3): [n(adj43, 10), n(adj42, 30, push(3, 1))],
            ("4", 2): [n(adj42, 10), n(adj43, 30, push(2, 1))],
            ("4", 1): [n(adj42, 20, push(1)), n(adj43, 20, push(1))],
        }
        for (node, d), hops in exp.items():
            assert R(rm, node, a(d)) == NH(*hops), (v4, node, d)
        # node-label routes stay shortest-path (DecisionTest.cpp:1996-2008 ...)
        assert R(rm, "1", L(4)) == NH(
            nh(adj12, False, 20, swap(4)), nh(adj13, False, 20, swap(4))
        )
        assert R(rm, "1", L(3)) == NH(nh(adj13, False, 10, labelPhpAction))
        for node in ("1", "2", "3", "4"):
            validate_pop_label_route(rm, node, int(node))
            validate_adj_label_routes(rm, node, dbs[node].adjacencies)
        # overload link 1->2 and node 3 (DecisionTest.cpp:2116-2138)
        db1 = dbs["1"]
        db1.adjacencies[0].isOverloaded = True
        dbs["3"].isOverloaded = True
        assert ls.updateAdjacencyDatabase(db1)[0]
        assert ls.updateAdjacencyDatabase(dbs["3"])[0]
        db1.adjacencies[0].isOverloaded = False  # module-level adj objects are shared
        rm = get_route_map(s, ["1"], areas, ps)
        assert ("1",) + a(4) not in rm
        assert R(rm, "1", a(3)) == NH(n(adj13, 10))
        assert ("1",) + a(2) not in rm


def sc_ring_overload_node(M):
    """DecisionTest.cpp:2510-2623 (OverloadNodeTest): nodes 2 and 3 drained,
    LFA on: 32 routes."""
    for v4 in (True, False):
        s, areas, ls, ps, dbs = ring_setup(M, v4, True, False)
        dbs["2"].isOverloaded = True
        dbs["3"].isOverloaded = True
        assert ls.updateAdjacencyDatabase(dbs["2"])[0]
        assert ls.updateAdjacencyDatabase(dbs["3"])[0]
        rm = get_route_map(s, ["1", "2", "3", "4"], areas, ps)
        assert len(rm) == 32
        a = lambda i: _ring_addr(v4, i)  # noqa: E731
        assert R(rm, "1", a(3)) == NH(nh(adj13, v4, 10))
        assert R(rm, "1", L(3)) == NH(nh(adj13, False, 10, labelPhpAction))
        assert R(rm, "1", a(2)) == NH(nh(adj12, v4, 10))
        assert ("1",) + a(4) not in rm
        assert R(rm, "2", a(4)) == NH(nh(adj24, v4, 10))
        assert R(rm, "2", a(3)) == NH(nh(adj21, v4, 20), nh(adj24, v4, 20))
        assert R(rm, "2", L(3)) == NH(
            nh(adj21, False, 20, swap(3)), nh(adj24, False, 20, swap(3))
        )
        assert R(rm, "2", a(1)) == NH(nh(adj21, v4, 10))
        assert R(rm, "3", a(4)) == NH(nh(adj34, v4, 10))
        assert R(rm, "3", a(2)) == NH(nh(adj31, v4, 20), nh(adj34, v4, 20))
        assert R(rm, "3", a(1)) == NH(nh(adj31, v4, 10))
        assert R(rm, "4", a(3)) == NH(nh(adj43, v4, 10))
        assert R(rm, "4", a(2)) == NH(nh(adj42, v4, 10))
        assert ("4",) + a(1) not in rm
        for node in ("1", "2", "3", "4"):
            validate_pop_label_route(rm, node, int(node))
            validate_adj_label_routes(rm, node, dbs[node].adjacencies)


# ------------------------------------------------ Grid (DecisionTest.cpp)


def _grid(M, n):
    """DecisionTest.cpp:3862-3918 (addAdj / createGrid)."""
    areas, ls = single_area(M)
    ps = M.PrefixState()

    def pfx(node):
        return T.toIpPrefix(f"::ffff:10.1.{node // 256}.{node % 256}/128")

    for i in range(n):
        for j in range(n):
            node = i * n + j
            adjs = []
            for (ii, jj, ifn, oifn) in (
                (i, j + 1, "0/1", "0/3"),
                (i - 1, j, "0/2", "0/4"),
                (i, j - 1, "0/3", "0/1"),
                (i + 1, j, "0/4", "0/2"),
            ):
                if 0 <= ii < n and 0 <= jj < n:
                    nb = ii * n + jj
                    adjs.append(
                        T.createThriftAdjacency(
                            str(nb), ifn, f"fe80::{nb}",
                            f"192.168.{nb // 256}.{nb % 256}",
                            1, 100001 + nb, False, 100, 10000, 1, oifn,
                        )
                    )
            ls.updateAdjacencyDatabase(T.createAdjDb(str(node), adjs, node + 1))
            ps.updatePrefixDatabase(
                T.createPrefixDb(str(node), [T.createPrefixEntry(pfx(node))])
            )
    return areas, ps, pfx


def sc_grid_shortest_path(M):
    """DecisionTest.cpp:3920-4010 (GridTopologyFixture, n = 2..8 of the
    reference's 2..16): route count 2n^4+3n^2-4n and Manhattan metrics."""
    import random

    rnd = random.Random(5)
    for n in (2, 4, 6, 8):
        areas, ps, pfx = _grid(M, n)
        s = M.SpfSolver("1", False, False)
        nodes = [str(i) for i in range(n * n)]
        rm = get_route_map(s, nodes, areas, ps)
        assert len(rm) == 2 * n**4 + 3 * n**2 - 4 * n, n

        def dist(a, b):
            return abs(a % n - b % n) + abs(a // n - b // n)

        pairs = [(0, n * n - 1), (n - 1, n * (n - 1))]
        pairs += [(rnd.randrange(n * n), rnd.randrange(n * n)) for _ in range(6)]
        for a, b in pairs:
            if a == b:
                continue
            hops = R(rm, str(a), P(pfx(b)))
            assert hops and all(h[4] == dist(a, b) for h in hops), (n, a, b)


# ------------------------------------- ParallelAdjRing (DecisionTest.cpp)

adj12_1 = T.createAdjacency("2", "2/1", "1/1", "fe80::2:1", "192.168.2.1", 11, 201)
adj12_2 = T.createAdjacency("2", "2/2", "1/2", "fe80::2:2", "192.168.2.2", 11, 202)
adj12_3 = T.createAdjacency("2", "2/3", "1/3", "fe80::2:3", "192.168.2.3", 20, 203)
adj13_1 = T.createAdjacency("3", "3/1", "1/1", "fe80::3:1", "192.168.3.1", 11, 301)
adj21_1 = T.createAdjacency("1", "1/1", "2/1", "fe80::1:1", "192.168.1.1", 11, 101)
adj21_2 = T.createAdjacency("1", "1/2", "2/2", "fe80::1:2", "192.168.1.2", 11, 102)
adj21_3 = T.createAdjacency("1", "1/3", "2/3", "fe80::1:3", "192.168.1.3", 20, 103)
adj24_1 = T.createAdjacency("4", "4/1", "2/1", "fe80::4:1", "192.168.4.1", 11, 401)
adj31_1 = T.createAdjacency("1", "1/1", "3/1", "fe80::1:1", "192.168.1.1", 11, 101)
adj34_1 = T.createAdjacency("4", "4/1", "3/1", "fe80::4:1", "192.168.4.1", 11, 401)
adj34_2 = T.createAdjacency("4", "4/2", "3/2", "fe80::4:2", "192.168.4.2", 20, 402)
adj34_3 = T.createAdjacency("4", "4/3", "3/3", "fe80::4:3", "192.168.4.3", 20, 403)
adj42_1 = T.createAdjacency("2", "2/1", "4/1", "fe80::2:1", "192.168.2.1", 11, 201)
adj43_1 = T.createAdjacency("3", "3/1", "4/1", "fe80::3:1", "192.168.3.1", 11, 301)
adj43_2 = T.createAdjacency("3", "3/2", "4/2", "fe80::3:2", "192.168.3.2", 20, 302)
adj43_3 = T.createAdjacency("3", "3/3", "4/3", "fe80::3:3", "192.168.3.3", 20, 303)


def par_setup(M, lfa, ksp2):
    """DecisionTest.cpp:2824-2925 (ParallelAdjRingTopologyFixture)."""
    import copy

    s = M.SpfSolver("1", False, lfa)
    dbs = {
        "1": T.createAdjDb("1", copy.deepcopy([adj12_1, adj12_2, adj12_3, adj13_1]), 1),
        "2": T.createAdjDb("2", copy.deepcopy([adj21_1, adj21_2, adj21_3, adj24_1]), 2),
        "3": T.createAdjDb("3", copy.deepcopy([adj31_1, adj34_1, adj34_2, adj34_3]), 3),
        "4": T.createAdjDb("4", copy.deepcopy([adj42_1, adj43_1, adj43_2, adj43_3]), 4),
    }
    areas, ls = single_area(M)
    assert not ls.updateAdjacencyDatabase(dbs["1"])[0]
    for n in ("2", "3", "4"):
        assert ls.updateAdjacencyDatabase(dbs[n])[0]
    ps = M.PrefixState()
    for pdb in (prefixDb1, prefixDb2, prefixDb3, prefixDb4):
        ps.updatePrefixDatabase(kspf_db(pdb) if ksp2 else pdb)
    return s, areas, ls, ps, dbs


def sc_parallel_ring_shortest_path(M):
    """DecisionTest.cpp:2932-3052 (ShortestPathTest): 44 routes, ECMP over
    parallel links."""
    s, areas, ls, ps, dbs = par_setup(M, False, False)
    rm = get_route_map(s, ["1", "2", "3", "4"], areas, ps)
    assert len(rm) == 44
    exp = {
        ("1", 4): [(adj12_2, 22), (adj13_1, 22), (adj12_1, 22)],
        ("1", 3): [(adj13_1, 11)],
        ("1", 2): [(adj12_2, 11), (adj12_1, 11)],
        ("2", 4): [(adj24_1, 11)],
        ("2", 3): [(adj21_2, 22), (adj21_1, 22), (adj24_1, 22)],
        ("2", 1): [(adj21_2, 11), (adj21_1, 11)],
        ("3", 4): [(adj34_1, 11)],
        ("3", 2): [(adj31_1, 22), (adj34_1, 22)],
        ("3", 1): [(adj31_1, 11)],
        ("4", 3): [(adj43_1, 11)],
        ("4", 2): [(adj42_1, 11)],
        ("4", 1): [(adj42_1, 22), (adj43_1, 22)],
    }
    addrs = {1: addr1, 2: addr2, 3: addr3, 4: addr4}
    for (node, d), hops in exp.items():
        assert R(rm, node, P(addrs[d])) == NH(*[nh(x, False, m) for x, m in hops])
        act = labelPhpAction if hops[0][1] == 11 else swap(d)
        assert R(rm, node, L(d)) == NH(*[nh(x, False, m, act) for x, m in hops])
    for node in ("1", "2", "3", "4"):
        validate_pop_label_route(rm, node, int(node))
        validate_adj_label_routes(rm, node, dbs[node].adjacencies)


def sc_parallel_ring_ksp2(M):
    """DecisionTest.cpp:3213-3385 (Ksp2EdEcmp, non-BGP instance): parallel
    links in KSP2 traces, minNexthop thresholds, then link overloads (the
    adj12_1-vs-adj12_2 choice there depends on folly's pair hash)."""
    s, areas, ls, ps, dbs = par_setup(M, True, True)
    rm = get_route_map(s, ["1"], areas, ps)
    n = lambda adj, m, act=None: nh(adj, False, m, act, True)  # noqa: E731
    assert R(rm, "1", P(addr2)) == NH(n(adj12_1, 11), n(adj12_2, 11), n(adj12_3, 20))
    # extra prefix from node 4 with minNexthop 4 -> dropped
    base4 = kspf_db(prefixDb4)

    def with_bgp(db, mnh):
        e = T.createPrefixEntry(
            bgpAddr1, T.PrefixType.LOOPBACK, "", T.PrefixForwardingType.SR_MPLS,
            T.PrefixForwardingAlgorithm.KSP2_ED_ECMP, None, None, mnh,
        )
        return T.createPrefixDb(db.thisNodeName, list(db.prefixEntries) + [e])

    ps.updatePrefixDatabase(with_bgp(base4, 4))
    rm = get_route_map(s, ["1"], areas, ps)
    assert ("1",) + P(bgpAddr1) not in rm
    ps.updatePrefixDatabase(with_bgp(base4, 2))
    rm = get_route_map(s, ["1"], areas, ps)
    assert R(rm, "1", P(bgpAddr1)) == NH(n(adj12_2, 22, push(4)), n(adj13_1, 22, push(4)))
    base3 = kspf_db(prefixDb3)
    ps.updatePrefixDatabase(with_bgp(base3, 4))
    rm = get_route_map(s, ["1"], areas, ps)
    assert ("1",) + P(bgpAddr1) not in rm
    ps.updatePrefixDatabase(base4)
    ps.updatePrefixDatabase(base3)
    # overload adj12_2 and adj34_2 (DecisionTest.cpp:3322-3330)
    dbs["1"].adjacencies[1].isOverloaded = True
    dbs["3"].adjacencies[2].isOverloaded = True
    assert ls.updateAdjacencyDatabase(dbs["1"])[0]
    assert ls.updateAdjacencyDatabase(dbs["3"])[0]
    rm = get_route_map(s, ["1", "2", "3", "4"], areas, ps)
    assert len(rm) == 44
    exp = {
        ("1", 4): [n(adj12_1, 22, push(4)), n(adj13_1, 22, push(4))],
        ("1", 3): [n(adj13_1, 11), n(adj12_1, 33, push(3, 4))],
        ("1", 2): [n(adj12_1, 11), n(adj12_3, 20)],
        ("2", 4): [n(adj24_1, 11), n(adj21_1, 33, push(4, 3))],
        ("2", 3): [n(adj21_1, 22, push(3)), n(adj24_1, 22, push(3))],
        ("2", 1): [n(adj21_1, 11), n(adj21_3, 20)],
        ("3", 4): [n(adj34_1, 11), n(adj34_3, 20)],
        ("3", 2): [n(adj31_1, 22, push(2)), n(adj34_1, 22, push(2))],
        ("3", 1): [n(adj31_1, 11), n(adj34_1, 33, push(1, 2))],
        ("4", 3): [n(adj43_1, 11), n(adj43_3, 20)],
        ("4", 2): [n(adj42_1, 11), n(adj43_1, 33, push(2, 1))],
        ("4", 1): [n(adj42_1, 22, push(1)), n(adj43_1, 22, push(1))],
    }
    addrs = {1: addr1, 2: addr2, 3: addr3, 4: addr4}
    for (node, d), hops in exp.items():
        assert R(rm, node, P(addrs[d])) == NH(*hops), (node, d)


# ------------------------------------------------- LFA (DecisionTest.cpp)


def sc_loop_free_alternates(M):
    """DecisionTest.cpp:5222-5357 (LoopFreeAlternatePaths), run through
    SpfSolver directly with computeLfaPaths=true (the fixture's Decision
    is built with LFA on): triangle 1-2 (10), 1-3 (8), 2-3 (9)."""
    import copy

    a12 = T.createAdjacency("2", "1/2", "2/1", "fe80::2", "192.168.0.2", 10, 0)
    a13 = T.createAdjacency("3", "1/3", "3/1", "fe80::3", "192.168.0.3", 8, 0)
    a21 = T.createAdjacency("1", "2/1", "1/2", "fe80::1", "192.168.0.1", 10, 0)
    a23 = T.createAdjacency("3", "2/3", "3/2", "fe80::3", "192.168.0.3", 9, 0)
    a31 = T.createAdjacency("1", "3/1", "1/3", "fe80::1", "192.168.0.1", 8, 0)
    a32 = T.createAdjacency("2", "3/2", "2/3", "fe80::2", "192.168.0.2", 9, 0)
    areas, ls = single_area(M)
    ps = M.PrefixState()
    ls.updateAdjacencyDatabase(T.createAdjDb("1", [a12, a13], 0))
    ls.updateAdjacencyDatabase(T.createAdjDb("2", [a21, a23], 0))
    ls.updateAdjacencyDatabase(T.createAdjDb("3", [a31, a32], 0))
    for pdb in (prefixDb1, prefixDb2, prefixDb3):
        ps.updatePrefixDatabase(pdb)
    s = M.SpfSolver("1", False, True)
    rm = get_route_map(s, ["1", "2", "3"], areas, ps)
    f = lambda adj, m: nh(adj, False, m)  # noqa: E731
    assert R(rm, "1", P(addr2)) == NH(f(a12, 10), f(a13, 17))
    assert R(rm, "1", P(addr3)) == NH(f(a12, 19), f(a13, 8))
    assert R(rm, "2", P(addr1)) == NH(f(a21, 10), f(a23, 17))
    assert R(rm, "2", P(addr3)) == NH(f(a21, 18), f(a23, 9))
    assert R(rm, "3", P(addr1)) == NH(f(a31, 8), f(a32, 19))
    assert R(rm, "3", P(addr2)) == NH(f(a31, 18), f(a32, 9))
    # raise 1-2 to 100: no LFA from node 3 any more
    a12 = copy.deepcopy(a12)
    a21 = copy.deepcopy(a21)
    a12.metric = 100
    a21.metric = 100
    ls.updateAdjacencyDatabase(T.createAdjDb("1", [a12, a13], 0))
    ls.updateAdjacencyDatabase(T.createAdjDb("2", [a21, a23], 0))
    rm = get_route_map(s, ["1", "2", "3"], areas, ps)
    assert R(rm, "1", P(addr2)) == NH(f(a12, 100), f(a13, 17))
    assert R(rm, "1", P(addr3)) == NH(f(a12, 109), f(a13, 8))
    assert R(rm, "2", P(addr1)) == NH(f(a21, 100), f(a23, 17))
    assert R(rm, "2", P(addr3)) == NH(f(a21, 108), f(a23, 9))
    assert R(rm, "3", P(addr1)) == NH(f(a31, 8))
    assert R(rm, "3", P(addr2)) == NH(f(a32, 9))
