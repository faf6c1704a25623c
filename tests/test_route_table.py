"""All-nodes unicast route table on the device.

AllNodesRouteTable (openr_amd/csrc/host/RouteTable.cpp) runs one all-sources
SPF with next hops over an area and spf_route_table_kernel over every IP /
SP_ECMP prefix: the restatement of SpfSolverImpl::selectEcmpOpenr
(openr/decision/Decision.cpp:668-712 with getBestAnnouncingNodes :544-630,
maybeFilterDrainedNodes :651-666, getNextHopsWithMetric :1093-1179,
getNextHopsThrift :1181-1271).  Parity: for EVERY node, the table's routes
equal the unicast entries of the CPU oracle's buildRouteDb(node) (the
reference-style restatement, pinned by the reference's known answers) for
those prefixes —
seeded random networks with anycast prefixes, drained nodes, overloaded
links, parallel links and v4 / v6 prefixes, and the benchmark fabric.
"""

import pytest

from openr_amd import thrift as T
from tests import randomized as RZ

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def E(gpu_ready):
    import openr_amd._openr_spf as E

    return E


@pytest.fixture(scope="module")
def O():
    from oracle import build

    build.build()
    from oracle import _oracle_ref

    return _oracle_ref


def _ecmp_only(unicast):
    # SR_MPLS prefixes (fd00::/64 in the generator) are not in the table
    return {k: v for k, v in unicast.items() if not bytes(k[0][0] if isinstance(k[0], tuple) else k[0]).startswith(b"\xfd\x00")}


@pytest.mark.parametrize("seed", range(6))
@pytest.mark.parametrize("v4", [True, False])
def test_route_table_matches_build_route_db(E, O, seed, v4):
    """Every node's table routes == the CPU oracle's buildRouteDb (the
    reference-style restatement, pinned by the reference known answers)."""
    names, adj_dbs, prefix_dbs = RZ.random_network(
        700 + seed, n_nodes=40, n_links=90, overload_prob=0.15, link_overload_prob=0.05
    )
    areas, ps = RZ.load(E, adj_dbs, prefix_dbs, seed)
    oareas, ops = RZ.load(O, adj_dbs, prefix_dbs, seed)
    table = E.AllNodesRouteTable(areas, "0", ps, v4)
    assert table.spf_ms > 0 and table.route_ms > 0
    solver = O.SpfSolver(names[0], v4, False)
    checked = 0
    for node in names:
        db = solver.buildRouteDb(node, oareas, ops)
        got = table.routes(node)
        if db is None:
            assert got == {}, node
            continue
        assert got == _ecmp_only(db["unicast"]), node
        checked += len(got)
    assert checked > 0


def test_route_table_fabric(E, O):
    from openr_amd import topologies as TP

    topo = TP.fabric(600)
    dbs = topo.adj_dbs(overloaded=[5, 77])
    built = {}
    for M in (E, O):
        areas = M.AreaLinkStates()
        ls = areas.add("0")
        for db in dbs:
            ls.updateAdjacencyDatabase(db)
        ps = M.PrefixState()
        for pdb in topo.prefix_dbs("0"):
            ps.updatePrefixDatabase(pdb)
        built[M] = (areas, ps)
    table = E.AllNodesRouteTable(built[E][0], "0", built[E][1], True)
    assert table.num_nodes == topo.num_nodes and table.num_prefixes == topo.num_nodes
    solver = O.SpfSolver("2-0-0", False, False)
    for node in sorted(topo.names)[:: max(1, topo.num_nodes // 25)] + ["2-0-0"]:
        db = solver.buildRouteDb(node, *built[O])
        assert table.routes(node) == db["unicast"], node


def _delta_py(new, old):
    """getRouteDelta (Decision.cpp:47-85) over unicast dicts: updates = new
    or changed entries, deletes = prefixes only in old."""
    upd = {k: v for k, v in new.items() if old.get(k) != v}
    dele = sorted(k for k in old if k not in new)
    return upd, dele


@pytest.mark.parametrize("seed", range(4))
def test_route_table_diff_equals_route_delta(E, O, seed):
    """Overload / metric churn (same links): the device diff + delta of every
    node equal getRouteDelta of that node's buildRouteDb before and after."""
    import random

    names, adj_dbs, prefix_dbs = RZ.random_network(
        900 + seed, n_nodes=40, n_links=90, overload_prob=0.1, link_overload_prob=0.0
    )
    areas, ps = RZ.load(E, adj_dbs, prefix_dbs, seed)
    oareas, ops = RZ.load(O, adj_dbs, prefix_dbs, seed)
    osolver = O.SpfSolver(names[0], True, False)
    before = {n: osolver.buildRouteDb(n, oareas, ops) for n in names}
    t0 = E.AllNodesRouteTable(areas, "0", ps, True)
    rng = random.Random(seed)
    for db in rng.sample(adj_dbs["0"], 3):  # drain toggles and metric changes
        db.isOverloaded = not db.isOverloaded
        if db.adjacencies:
            db.adjacencies[0].metric += rng.randint(1, 9)
    # the same load order: same links, same linksFromNode order (CSR layout)
    areas, ps = RZ.load(E, adj_dbs, prefix_dbs, seed)
    oareas, ops = RZ.load(O, adj_dbs, prefix_dbs, seed)
    t1 = E.AllNodesRouteTable(areas, "0", ps, True)
    changed = t1.diff(t0)
    total = 0
    for i, c in enumerate(changed):
        node = t1.node_name(i)
        upd, dele = t1.delta(node)
        uni, lab = t1.changed_split(node)
        assert uni + lab == c, node
        assert len(upd) + len(dele) == uni, node
        # device delta == delta of the table rows == getRouteDelta of the host RouteDbs
        assert (upd, sorted(dele)) == _delta_py(t1.routes(node), t0.routes(node)), node
        after = osolver.buildRouteDb(node, oareas, ops)
        b = _ecmp_only(before[node]["unicast"]) if before.get(node) else {}
        a = _ecmp_only(after["unicast"]) if after else {}
        assert (upd, sorted(dele)) == _delta_py(a, b), node
        total += c
    assert total > 0


def _label_network(seed, n_nodes=40, n_links=90):
    """Random network whose node labels collide (17 distinct values over the
    nodes), one invalid label, adjacency labels that repeat a node label and
    each other (the emplace-first rules of Decision.cpp:483-534)."""
    import random

    names, adj_dbs, prefix_dbs = RZ.random_network(
        1300 + seed, n_nodes=n_nodes, n_links=n_links, overload_prob=0.12, link_overload_prob=0.06
    )
    # no SR_MPLS prefixes: a KSP2 label stack through the node with the
    # invalid label is the reference's fatal CHECK (createMplsAction)
    for pdb in prefix_dbs:
        pdb.prefixEntries = [e for e in pdb.prefixEntries if int(e.forwardingType) == 0]
    rng = random.Random(seed)
    for k, db in enumerate(adj_dbs["0"]):
        db.nodeLabel = 101 + (k % 17)
        if k == 3:
            db.nodeLabel = 1 << 21  # invalid: skipped
        for adj in db.adjacencies:
            r = rng.random()
            if r < 0.05:
                adj.adjLabel = 101 + rng.randrange(17)  # repeats a node label
            elif r < 0.1:
                adj.adjLabel = 60000  # repeated adjacency label
            elif r < 0.13:
                adj.adjLabel = 0  # not SR
    return names, adj_dbs, prefix_dbs


@pytest.mark.parametrize("seed", range(5))
def test_route_table_mpls_matches_build_route_db(E, O, seed):
    """Every node's MPLS routes from the table (node-label columns of the same
    device pass + adjacency labels) == the CPU oracle's buildRouteDb mpls
    entries: POP_AND_LOOKUP / PHP / SWAP, label collisions (smallest-named
    owner the node reaches), invalid labels, adjacency-label precedence."""
    names, adj_dbs, prefix_dbs = _label_network(seed)
    areas, ps = RZ.load(E, adj_dbs, prefix_dbs, seed)
    oareas, ops = RZ.load(O, adj_dbs, prefix_dbs, seed)
    table = E.AllNodesRouteTable(areas, "0", ps, True)
    assert table.num_label_columns > 17
    solver = O.SpfSolver(names[0], True, False)
    checked = 0
    for node in names:
        db = solver.buildRouteDb(node, oareas, ops)
        got = table.mpls_routes(node)
        if db is None:
            assert got == {}, node
            continue
        assert got == db["mpls"], node
        checked += len(got)
    assert checked > 0


def test_route_table_mpls_fabric(E, O):
    from openr_amd import topologies as TP

    topo = TP.fabric(600)
    dbs = topo.adj_dbs(overloaded=[5, 77])
    built = {}
    for M in (E, O):
        areas = M.AreaLinkStates()
        ls = areas.add("0")
        for db in dbs:
            ls.updateAdjacencyDatabase(db)
        ps = M.PrefixState()
        for pdb in topo.prefix_dbs("0"):
            ps.updatePrefixDatabase(pdb)
        built[M] = (areas, ps)
    table = E.AllNodesRouteTable(built[E][0], "0", built[E][1], True)
    assert table.num_label_columns == topo.num_nodes
    solver = O.SpfSolver("2-0-0", False, False)
    for node in sorted(topo.names)[:: max(1, topo.num_nodes // 20)] + ["2-0-0"]:
        db = solver.buildRouteDb(node, *built[O])
        assert table.mpls_routes(node) == db["mpls"], node


@pytest.mark.parametrize("seed", range(3))
def test_route_table_delta_mpls_equals_route_delta(E, O, seed):
    """Overload / metric / adjacency-label churn on the same links: the MPLS
    part of the table delta of every node == getRouteDelta of the oracle's
    RouteDbs before and after."""
    import random

    names, adj_dbs, prefix_dbs = _label_network(seed)
    areas, ps = RZ.load(E, adj_dbs, prefix_dbs, seed)
    oareas, ops = RZ.load(O, adj_dbs, prefix_dbs, seed)
    osolver = O.SpfSolver(names[0], True, False)
    before = {n: osolver.buildRouteDb(n, oareas, ops) for n in names}
    t0 = E.AllNodesRouteTable(areas, "0", ps, True)
    rng = random.Random(seed)
    for db in rng.sample(adj_dbs["0"], 4):
        db.isOverloaded = not db.isOverloaded
        if db.adjacencies:
            db.adjacencies[0].metric += rng.randint(1, 9)
            db.adjacencies[-1].adjLabel = 70000 + rng.randrange(50)
    areas, ps = RZ.load(E, adj_dbs, prefix_dbs, seed)
    oareas, ops = RZ.load(O, adj_dbs, prefix_dbs, seed)
    t1 = E.AllNodesRouteTable(areas, "0", ps, True)
    t1.diff(t0)
    total = 0
    for node in names:
        upd, dele = t1.delta_mpls(node)
        after = osolver.buildRouteDb(node, oareas, ops)
        b = before[node]["mpls"] if before.get(node) else {}
        a = after["mpls"] if after else {}
        want_upd = {k: v for k, v in a.items() if b.get(k) != v}
        want_del = sorted(k for k in b if k not in a)
        assert (upd, sorted(dele)) == (want_upd, want_del), node
        total += len(upd) + len(dele)
    assert total > 0


@pytest.mark.parametrize("seed", range(5))
@pytest.mark.parametrize("v4", [True, False])
def test_route_table_lfa_matches_build_route_db(E, O, seed, v4):
    """computeLfaPaths on (SpfSolver(..., computeLfaPaths=true)): every node's
    unicast AND MPLS routes from the LFA table (shortest-path and
    loop-free-alternate next hops, each with its own metric, RFC 5286
    condition d(n, x) < d(s, x) + d(n, s)) == the CPU oracle's buildRouteDb."""
    names, adj_dbs, prefix_dbs = RZ.random_network(
        1700 + seed, n_nodes=40, n_links=100, overload_prob=0.12, link_overload_prob=0.05
    )
    areas, ps = RZ.load(E, adj_dbs, prefix_dbs, seed)
    oareas, ops = RZ.load(O, adj_dbs, prefix_dbs, seed)
    table = E.AllNodesRouteTable(areas, "0", ps, v4, True)
    solver = O.SpfSolver(names[0], v4, True)
    checked = lfa_hops = 0
    for node in names:
        db = solver.buildRouteDb(node, oareas, ops)
        got, mpls = table.routes(node), table.mpls_routes(node)
        if db is None:
            assert got == {} and mpls == {}, node
            continue
        want = _ecmp_only(db["unicast"])
        assert got == want, node
        assert mpls == db["mpls"], node
        checked += len(got)
    assert checked > 0
    # LFA adds next hops somewhere: the LFA table differs from the plain one
    plain = E.AllNodesRouteTable(areas, "0", ps, v4, False)
    for node in names:
        a, b = table.routes(node), plain.routes(node)
        lfa_hops += sum(1 for k in a if a[k] != b.get(k))
    assert lfa_hops > 0


def test_route_table_lfa_fabric_and_delta(E, O):
    """Fabric LFA table against the oracle on sampled nodes, then an RSW drain:
    the LFA table delta of every node == getRouteDelta of the oracle."""
    from openr_amd import topologies as TP

    topo = TP.fabric(600)
    dbs = topo.adj_dbs(overloaded=[5])

    def load(M, dbs):
        areas = M.AreaLinkStates()
        ls = areas.add("0")
        for db in dbs:
            ls.updateAdjacencyDatabase(db)
        ps = M.PrefixState()
        for pdb in topo.prefix_dbs("0"):
            ps.updatePrefixDatabase(pdb)
        return areas, ps

    ea, eps = load(E, dbs)
    oa, ops = load(O, dbs)
    t0 = E.AllNodesRouteTable(ea, "0", eps, False, True)
    solver = O.SpfSolver("2-0-0", False, True)
    sample = sorted(topo.names)[:: max(1, topo.num_nodes // 12)] + ["2-0-0"]
    before = {}
    for node in sample:
        db = solver.buildRouteDb(node, oa, ops)
        assert t0.routes(node) == db["unicast"], node
        assert t0.mpls_routes(node) == db["mpls"], node
        before[node] = db
    rsw = next(i for i, n in enumerate(topo.names) if n.startswith("3-"))
    dbs2 = topo.adj_dbs(overloaded=[5, rsw])
    ea2, eps2 = load(E, dbs2)
    oa2, ops2 = load(O, dbs2)
    t1 = E.AllNodesRouteTable(ea2, "0", eps2, False, True)
    t1.diff(t0)
    for node in sample:
        after = solver.buildRouteDb(node, oa2, ops2)
        upd, dele = t1.delta(node)
        assert (upd, sorted(dele)) == _delta_py(after["unicast"], before[node]["unicast"]), node
        mu, md = t1.delta_mpls(node)
        want_u = {k: v for k, v in after["mpls"].items() if before[node]["mpls"].get(k) != v}
        assert (mu, sorted(md)) == (want_u, sorted(k for k in before[node]["mpls"] if k not in after["mpls"])), node


def _two_area_network(seed, bgp, n_areas=2):
    """Areas "A", "B" (, "C") with disjoint interior nodes joined by border
    nodes: area k is RZ.random_network(seed + k) with its nodes renamed, and
    its first two nodes renamed to the border nodes shared with area A.
    IP-forwarding entries only (SR-MPLS across areas trips the reference's
    .at() on nodes absent from an area)."""
    from tests import randomized as RZ

    adj_dbs, prefix_dbs, names = {}, [], []
    border = None
    for k, area in enumerate(("A", "B", "C")[:n_areas]):
        nm, adj, pdb = RZ.random_network(seed * 10 + k, n_nodes=16, n_links=34, areas=(area,),
                                         bgp=bgp)
        ren = {n: f"{area.lower()}{i:02d}-{n}" for i, n in enumerate(nm)}
        if border is None:
            border = [ren[nm[0]], ren[nm[1]]]
        else:
            ren[nm[0]], ren[nm[1]] = border
        for db in adj[area]:
            db.thisNodeName = ren[db.thisNodeName]
            for a in db.adjacencies:
                a.otherNodeName = ren[a.otherNodeName]
        for p in pdb:
            p.thisNodeName = ren[p.thisNodeName]
            p.prefixEntries = [e for e in p.prefixEntries
                               if e.forwardingType == T.PrefixForwardingType.IP]
        adj_dbs[area] = adj[area]
        prefix_dbs += pdb
        names += [ren[n] for n in nm if ren[n] not in names]
    return names, adj_dbs, prefix_dbs


@pytest.mark.gpu
@pytest.mark.parametrize("seed,n_areas,bgp", [(0, 1, True), (1, 2, False), (2, 2, True),
                                               (3, 3, True)])
def test_all_areas_route_table_equals_oracle(gpu_ready, seed, n_areas, bgp):
    """AllAreasRouteTable: every node's complete RouteDb (multi-area, BGP
    metric-vector prefixes, SR-MPLS / KSP2 prefixes in one area, MPLS routes)
    equals the oracle's buildRouteDb; interior nodes take their IP / SP_ECMP
    routes from the per-area device tables, border nodes and the other
    prefixes from the host path."""
    from oracle import _oracle_ref as O
    import openr_amd._openr_spf as E
    from tests import randomized as RZ

    if n_areas == 1:
        names, adj_dbs, prefix_dbs = RZ.random_network(4100 + seed, n_nodes=28, n_links=70,
                                                       bgp=bgp)
    else:
        names, adj_dbs, prefix_dbs = _two_area_network(4100 + seed, bgp, n_areas)
    ea, ep = RZ.load(E, adj_dbs, prefix_dbs, seed)
    oa, op = RZ.load(O, adj_dbs, prefix_dbs, seed)
    for lfa in (False, True):
        t = E.AllAreasRouteTable(ea, ep, True, lfa)
        table_routes = host_routes = 0
        for node in names:
            os_ = O.SpfSolver(node, True, lfa)
            want = os_.buildRouteDb(node, oa, op)
            got = t.route_db(node)
            assert got == want, (node, lfa, t.is_border(node))
            table_routes += t.last_table_routes
            host_routes += t.last_host_routes
        assert table_routes > 0  # the device tables served the interior nodes
        if n_areas > 1:
            assert host_routes > 0  # border nodes / multi-area routes on the host


def _bgp_network(seed, n_nodes=40, split=False):
    """One area with BGP prefixes (RZ.random_network's metric-vector
    entries).  split: two components joined by nothing, so BGP prefixes with
    announcers on both sides are unreachable from some nodes."""
    from tests import randomized as RZ

    names, adj_dbs, prefix_dbs = RZ.random_network(seed, n_nodes=n_nodes, n_links=n_nodes * 3,
                                                   bgp=True)
    if split:
        half = set(names[: n_nodes // 2])
        for db in adj_dbs["0"]:
            db.adjacencies = [a for a in db.adjacencies
                              if (a.otherNodeName in half) == (db.thisNodeName in half)]
    return names, adj_dbs, prefix_dbs


@pytest.mark.gpu
@pytest.mark.parametrize("seed,dry,igp,split", [(11, False, False, False), (12, True, False, False),
                                                 (13, False, True, False), (14, False, False, True),
                                                 (15, True, False, True)])
def test_all_areas_route_table_bgp_on_device(gpu_ready, seed, dry, igp, split):
    """BGP prefixes (IP / SP_ECMP) in the device table (round 6): without the
    IGP cost in the metric vector and with every announcer reachable from
    every node, the metric-vector selection (runBestPathSelectionBgp,
    Decision.cpp:714-803) has the same winners at every node, so it runs once
    on the host and the winners are the column's announcers
    (selectEcmpBgp :805-866: no route at a winner, bestPrefixEntry / loopback
    next hop of the selection, doNotInstall = bgpDryRun).  Every node's
    RouteDb equals the oracle's, with bgpDryRun, with bgpUseIgpMetric (BGP
    then stays on the host) and on a split graph (prefixes some node cannot
    reach stay on the host)."""
    from oracle import _oracle_ref as O
    import openr_amd._openr_spf as E
    from tests import randomized as RZ

    names, adj_dbs, prefix_dbs = _bgp_network(5200 + seed, split=split)
    ea, ep = RZ.load(E, adj_dbs, prefix_dbs, seed)
    oa, op = RZ.load(O, adj_dbs, prefix_dbs, seed)
    for lfa in (False, True):
        t = E.AllAreasRouteTable(ea, ep, True, lfa, dry, igp)
        if igp:
            assert t.bgp_device_prefixes == 0
        elif not split:
            assert t.bgp_device_prefixes > 0
        for node in names:
            os_ = O.SpfSolver(node, True, lfa, False, dry, igp)
            want = os_.buildRouteDb(node, oa, op)
            got = t.route_db(node)
            assert got == want, (node, lfa)
        assert t.num_tables == 1
