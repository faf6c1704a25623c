"""MI355X engine (openr_amd._openr_spf, HIP kernels through the C ABI) vs the
CPU oracle (oracle._oracle_ref): the reference known answers, then bit-exact
SpfResult / KSP2 path / RouteDb equality on seeded random networks."""

import copy

import pytest

from openr_amd import thrift as T
from tests import known_answers as KA
from tests import known_answers_more as KB
from tests import randomized as RZ

pytestmark = pytest.mark.gpu

SCENARIOS = [getattr(M, n) for M in (KA, KB) for n in dir(M) if n.startswith("sc_")]
# DecisionTestFixture cases, replayed through PublicationIngest (CompactProtocol)
WIRE_SCENARIOS = [getattr(KB, n) for n in dir(KB) if n.startswith("sc_decision_")]


@pytest.fixture(scope="module")
def mods(gpu_ready):
    from oracle import _oracle_ref
    import openr_amd._openr_spf as E

    return E, _oracle_ref


@pytest.mark.parametrize("scenario", SCENARIOS, ids=lambda f: f.__name__)
def test_engine_known_answer(mods, scenario):
    E, _ = mods
    E.reset_counters()
    scenario(E)


@pytest.mark.parametrize("scenario", WIRE_SCENARIOS, ids=lambda f: f.__name__)
def test_engine_known_answer_via_publication_ingest(mods, scenario):
    E, _ = mods
    scenario(E, wire=True)


def _spf_equal(e_ls, o_ls, node, use_metric=True):
    a = e_ls.getSpfResult(node, use_metric)
    b = o_ls.getSpfResult(node, use_metric)
    assert a.keys() == b.keys(), node
    for k in a:
        assert a[k][0] == b[k][0], (node, k)
        assert a[k][1] == b[k][1], (node, k, a[k][1], b[k][1])
        assert list(a[k][2]) == list(b[k][2]), (node, k)


@pytest.mark.parametrize("seed", range(6))
def test_random_spf_results(mods, seed):
    E, O = mods
    names, adj_dbs, prefix_dbs = RZ.random_network(seed, n_nodes=40, n_links=90)
    ea, _ = RZ.load(E, adj_dbs, prefix_dbs, seed)
    oa, _ = RZ.load(O, adj_dbs, prefix_dbs, seed)
    for node in names[:: max(1, len(names) // 12)]:
        _spf_equal(ea["0"], oa["0"], node, True)
        _spf_equal(ea["0"], oa["0"], node, False)


@pytest.mark.parametrize("seed", range(3))
def test_random_zero_metric_spf(mods, seed):
    E, O = mods
    names, adj_dbs, prefix_dbs = RZ.random_network(
        100 + seed, n_nodes=30, n_links=70, metric_range=(0, 4), zero_metric_prob=0.3
    )
    ea, _ = RZ.load(E, adj_dbs, prefix_dbs, seed)
    oa, _ = RZ.load(O, adj_dbs, prefix_dbs, seed)
    for node in names[::3]:
        _spf_equal(ea["0"], oa["0"], node, True)


def _paths(ls, s, d, k):
    return [[l.key() for l in p] for p in ls.getKthPaths(s, d, k)]


@pytest.mark.parametrize("seed", range(3))
def test_random_kth_paths(mods, seed):
    E, O = mods
    names, adj_dbs, prefix_dbs = RZ.random_network(200 + seed, n_nodes=25, n_links=60)
    ea, _ = RZ.load(E, adj_dbs, prefix_dbs, seed)
    oa, _ = RZ.load(O, adj_dbs, prefix_dbs, seed)
    src = names[0]
    for d in names[1:]:
        for k in (1, 2):
            assert _paths(ea["0"], src, d, k) == _paths(oa["0"], src, d, k), (d, k)


@pytest.mark.parametrize("seed", range(5))
@pytest.mark.parametrize("lfa", [False, True])
def test_random_route_db(mods, seed, lfa):
    E, O = mods
    names, adj_dbs, prefix_dbs = RZ.random_network(300 + seed, n_nodes=30, n_links=70)
    ea, ep = RZ.load(E, adj_dbs, prefix_dbs, seed)
    oa, op = RZ.load(O, adj_dbs, prefix_dbs, seed)
    es = E.SpfSolver(names[0], True, lfa)
    os_ = O.SpfSolver(names[0], True, lfa)
    for node in names:
        a = es.buildRouteDb(node, ea, ep)
        b = os_.buildRouteDb(node, oa, op)
        assert a == b, node


@pytest.mark.parametrize("seed", range(6))
@pytest.mark.parametrize("igp", [False, True])
def test_random_route_db_bgp(mods, seed, igp):
    """BGP prefixes with random metric vectors (runBestPathSelectionBgp /
    selectEcmpBgp, Decision.cpp:715-866; SR-MPLS BGP through selectKsp2):
    every node's RouteDb equals the oracle's (whose BGP rules are pinned by
    the BGPRedistribution / Ksp2EdEcmpForBGP known answers)."""
    E, O = mods
    names, adj_dbs, prefix_dbs = RZ.random_network(600 + seed, n_nodes=24, n_links=50, bgp=True)
    ea, ep = RZ.load(E, adj_dbs, prefix_dbs, seed)
    oa, op = RZ.load(O, adj_dbs, prefix_dbs, seed)
    for lfa in (False, True):
        es = E.SpfSolver(names[0], True, lfa, False, seed % 2 == 1, igp)
        os_ = O.SpfSolver(names[0], True, lfa, False, seed % 2 == 1, igp)
        for node in names:
            assert es.buildRouteDb(node, ea, ep) == os_.buildRouteDb(node, oa, op), (node, lfa)


@pytest.mark.parametrize("seed", range(3))
def test_random_route_db_multi_area(mods, seed):
    E, O = mods
    names, adj_dbs, prefix_dbs = RZ.random_network(
        400 + seed, n_nodes=30, n_links=80, areas=("A", "B")
    )
    # KSP2 across areas needs every node in every area (reference .at()):
    # keep this case SP_ECMP only
    for pdb in prefix_dbs:
        pdb.prefixEntries = [
            e for e in pdb.prefixEntries if e.forwardingType == T.PrefixForwardingType.IP
        ]
    ea, ep = RZ.load(E, adj_dbs, prefix_dbs, seed)
    oa, op = RZ.load(O, adj_dbs, prefix_dbs, seed)
    es = E.SpfSolver(names[0], True, True)
    os_ = O.SpfSolver(names[0], True, True)
    for node in names:
        assert es.buildRouteDb(node, ea, ep) == os_.buildRouteDb(node, oa, op), node


def test_spf_runs_counter_matches_oracle(mods):
    E, O = mods
    names, adj_dbs, prefix_dbs = RZ.random_network(7, n_nodes=20, n_links=40)
    for lfa in (False, True):
        E.reset_counters()
        O.reset_counters()
        ea, ep = RZ.load(E, adj_dbs, prefix_dbs, 1)
        oa, op = RZ.load(O, adj_dbs, prefix_dbs, 1)
        es = E.SpfSolver(names[0], False, lfa)
        os_ = O.SpfSolver(names[0], False, lfa)
        for node in names:
            es.buildRouteDb(node, ea, ep)
            os_.buildRouteDb(node, oa, op)
        assert (
            E.get_counters().get("decision.spf_runs", 0)
            == O.get_counters()["decision.spf_runs"]
        )


@pytest.mark.parametrize("seed", range(4))
def test_incremental_updates(mods, seed):
    """Churn that keeps the set of up links (node drain toggles, metric
    changes of up links) patches the device graph in place instead of
    rebuilding it (LinkState::patchMemo); churn that changes it (link
    overloads) rebuilds.  After every step the engine's SPF rows, KSP2 paths
    and RouteDb equal the oracle's, and the change flags match."""
    import random

    E, O = mods
    names, adj_dbs, prefix_dbs = RZ.random_network(500 + seed, n_nodes=30, n_links=70)
    ea, ep = RZ.load(E, adj_dbs, prefix_dbs, seed)
    oa, op = RZ.load(O, adj_dbs, prefix_dbs, seed)
    es = E.SpfSolver(names[0], True, True)
    os_ = O.SpfSolver(names[0], True, True)
    rng = random.Random(seed)
    dbs = [copy.deepcopy(d) for d in adj_dbs["0"]]
    E.reset_counters()
    for step in range(12):
        db = rng.choice(dbs)
        kind = rng.random()
        if kind < 0.45 or not db.adjacencies:
            db.isOverloaded = not db.isOverloaded
        elif kind < 0.85:
            adj = rng.choice(db.adjacencies)
            adj.metric = rng.randint(1, 20)
        else:
            adj = rng.choice(db.adjacencies)
            adj.isOverloaded = not adj.isOverloaded
        assert ea["0"].updateAdjacencyDatabase(db) == oa["0"].updateAdjacencyDatabase(db)
        node = rng.choice(names)
        if ea["0"].hasNode(node):
            _spf_equal(ea["0"], oa["0"], node, True)
            _spf_equal(ea["0"], oa["0"], node, False)
        me = names[step % len(names)]
        assert es.buildRouteDb(me, ea, ep) == os_.buildRouteDb(me, oa, op), (step, me)
    assert E.get_counters().get("decision.graph_patches", 0) > 0


@pytest.mark.parametrize("seed", range(4))
def test_link_flaps_in_place(mods, seed):
    """Link flaps in the product LinkState (LinkState::patchStructure): an
    adjacency withdrawn (the link goes down), restored, or a link overload
    toggled splices the affected CSR rows in place (link ids of the other
    links kept, freed ids reused) instead of flattening the LinkState again.
    After every flap every node's metric and hop-count SpfResult (distances,
    next hops, pathLinks order), k = 2 paths and a RouteDb equal the
    oracle's; the in-place path ran and no full rebuild happened."""
    import random

    E, O = mods
    names, adj_dbs, prefix_dbs = RZ.random_network(3100 + seed, n_nodes=32, n_links=90)
    ea, ep = RZ.load(E, adj_dbs, prefix_dbs, seed)
    oa, op = RZ.load(O, adj_dbs, prefix_dbs, seed)
    es = E.SpfSolver(names[0], True, False)
    os_ = O.SpfSolver(names[0], True, False)
    rng = random.Random(seed)
    dbs = [copy.deepcopy(d) for d in adj_dbs["0"]]
    withdrawn = {}  # node index -> withdrawn adjacencies
    es.buildRouteDb(names[0], ea, ep)  # builds the engine
    E.reset_counters()
    for step in range(24):
        i = rng.randrange(len(dbs))
        db = dbs[i]
        kind = rng.random()
        if withdrawn.get(i) and kind < 0.4:
            db.adjacencies = db.adjacencies + [withdrawn[i].pop()]
        elif db.adjacencies and kind < 0.8:
            k = rng.randrange(len(db.adjacencies))
            withdrawn.setdefault(i, []).append(db.adjacencies[k])
            db.adjacencies = db.adjacencies[:k] + db.adjacencies[k + 1:]
        elif db.adjacencies:
            adj = rng.choice(db.adjacencies)
            adj.isOverloaded = not adj.isOverloaded
        assert ea["0"].updateAdjacencyDatabase(db) == oa["0"].updateAdjacencyDatabase(db)
        for node in names[step % 4::4]:
            if ea["0"].hasNode(node):
                _spf_equal(ea["0"], oa["0"], node, True)
                _spf_equal(ea["0"], oa["0"], node, False)
        a, b = names[step % len(names)], names[(7 * step + 3) % len(names)]
        if a != b and ea["0"].hasNode(a) and ea["0"].hasNode(b):
            assert _paths(ea["0"], a, b, 2) == _paths(oa["0"], a, b, 2), (step, a, b)
        me = names[step % len(names)]
        assert es.buildRouteDb(me, ea, ep) == os_.buildRouteDb(me, oa, op), (step, me)
    c = E.get_counters()
    assert c.get("decision.graph_inplace_link_patches", 0) > 0
    assert c.get("decision.graph_build_us", 0) == 0  # never flattened again


@pytest.mark.parametrize("seed", range(4))
def test_link_flap_with_metric_raise_in_one_update(mods, seed):
    """one adjacency update that withdraws an adjacency AND
    raises the metric of another (tight) link of the same node.  The node's
    CSR row is rebuilt from linkMap_ after Link::setMetricFromNode ran, so the
    memo screen must take the REMOVED delta's metric from the retired arrays;
    with the new metric it kept memoized views whose shortest paths used the
    old, cheaper link.  Every node's metric SpfResult is memoized before each
    update and must equal the oracle's after it (no full rebuild)."""
    import random

    E, O = mods
    names, adj_dbs, prefix_dbs = RZ.random_network(4100 + seed, n_nodes=30, n_links=80)
    ea, ep = RZ.load(E, adj_dbs, prefix_dbs, seed)
    oa, op = RZ.load(O, adj_dbs, prefix_dbs, seed)
    es = E.SpfSolver(names[0], True, False)
    os_ = O.SpfSolver(names[0], True, False)
    rng = random.Random(seed)
    dbs = [copy.deepcopy(d) for d in adj_dbs["0"]]
    es.buildRouteDb(names[0], ea, ep)
    E.reset_counters()
    steps = 0
    for _ in range(40):
        if steps == 8:
            break
        i = rng.randrange(len(dbs))
        db = dbs[i]
        if len(db.adjacencies) < 3:
            continue
        for node in names:  # warm the whole memo
            if ea["0"].hasNode(node):
                ea["0"].getSpfResult(node, True)
        k = rng.randrange(len(db.adjacencies))
        rest = db.adjacencies[:k] + db.adjacencies[k + 1:]
        # raise one kept link (or every one) of the same node in the same update
        bump = rest if steps % 2 else [rng.choice(rest)]
        for adj in bump:
            adj.metric = adj.metric + rng.randint(1, 6)
        db.adjacencies = rest
        assert ea["0"].updateAdjacencyDatabase(db) == oa["0"].updateAdjacencyDatabase(db)
        for node in names:
            if ea["0"].hasNode(node):
                _spf_equal(ea["0"], oa["0"], node, True)
        me = names[steps % len(names)]
        assert es.buildRouteDb(me, ea, ep) == os_.buildRouteDb(me, oa, op), (steps, me)
        steps += 1
    assert steps == 8
    c = E.get_counters()
    assert c.get("decision.graph_inplace_link_patches", 0) > 0
    assert c.get("decision.graph_build_us", 0) == 0
    assert c.get("decision.spf_memo_dropped", 0) > 0


@pytest.mark.parametrize("seed", range(4))
def test_selective_memo_invalidation(mods, seed):
    """SURVEY §8(f) row 2 in LinkState: a topology change keeps the memoized
    SPF views whose shortest-path DAG no edge delta touches (the table screen
    rule on the host rows) instead of dropping the whole memo
    (LinkState.cpp:712-715).  Every node's metric AND hop-count SpfResult is
    memoized, then drain toggles, metric changes, link overloads (the CSR
    changes: the retired engine's views are screened against spf_graph_diff)
    and link additions are applied; after each, EVERY node's SpfResult
    (distances, next hops, pathLinks order) and a RouteDb equal the oracle's,
    and views were both kept and dropped."""
    import random

    E, O = mods
    names, adj_dbs, prefix_dbs = RZ.random_network(
        2100 + seed, n_nodes=36, n_links=80, overload_prob=0.05, link_overload_prob=0.02
    )
    ea, ep = RZ.load(E, adj_dbs, prefix_dbs, seed)
    oa, op = RZ.load(O, adj_dbs, prefix_dbs, seed)
    es = E.SpfSolver(names[0], True, False)
    os_ = O.SpfSolver(names[0], True, False)
    rng = random.Random(seed)
    dbs = [copy.deepcopy(d) for d in adj_dbs["0"]]
    E.reset_counters()
    for step in range(10):
        for node in names:  # warm the whole memo
            if ea["0"].hasNode(node):
                ea["0"].getSpfResult(node, True)
                ea["0"].getSpfResult(node, False)
        db = rng.choice(dbs)
        kind = rng.random()
        if kind < 0.35 or not db.adjacencies:
            db.isOverloaded = not db.isOverloaded
        elif kind < 0.7:
            adj = rng.choice(db.adjacencies)
            adj.metric = rng.randint(1, 20)
        else:
            adj = rng.choice(db.adjacencies)
            adj.isOverloaded = not adj.isOverloaded
        assert ea["0"].updateAdjacencyDatabase(db) == oa["0"].updateAdjacencyDatabase(db)
        for node in names:
            if ea["0"].hasNode(node):
                _spf_equal(ea["0"], oa["0"], node, True)
                _spf_equal(ea["0"], oa["0"], node, False)
        me = names[step % len(names)]
        assert es.buildRouteDb(me, ea, ep) == os_.buildRouteDb(me, oa, op), (step, me)
    c = E.get_counters()
    assert c.get("decision.spf_memo_kept", 0) > 0
    assert c.get("decision.spf_memo_dropped", 0) > 0


@pytest.mark.parametrize("seed", range(2))
def test_kth_paths_beyond_two(mods, seed):
    """getKthPaths accepts any k (LinkState.cpp:760-789: linksToIgnore = the
    links of every lower rank).  k = 5 asked FIRST on a fresh LinkState fills
    ranks 1..4 on the way (a k >= 3 fill used to re-lock its own
    fill lock); then k = 3, 4 hit the memo.  Paths equal the oracle's."""
    E, O = mods
    names, adj_dbs, prefix_dbs = RZ.random_network(800 + seed, n_nodes=20, n_links=70)
    ea, _ = RZ.load(E, adj_dbs, prefix_dbs, seed)
    oa, _ = RZ.load(O, adj_dbs, prefix_dbs, seed)
    src = names[0]
    for d in names[1:8]:
        for k in (5, 3, 4, 1, 2):
            assert _paths(ea["0"], src, d, k) == _paths(oa["0"], src, d, k), (d, k)


def test_spf_runs_fb303_count_per_spf(mods):
    """decision.spf_runs is a COUNT stat bumped once per runSpf (LinkState.cpp:
    813): a what-if batch of n queries exports .count == n, equal to the sum."""
    E, _ = mods
    names, adj_dbs, prefix_dbs = RZ.random_network(9, n_nodes=20, n_links=40)
    ea, _ = RZ.load(E, adj_dbs, prefix_dbs, 1)
    ls = ea["0"]
    links = list(ls.linksFromNode(names[0]))
    E.reset_counters()
    ls.runSpfBatch(names[0], [[l] for l in links], True)
    got = E.get_counters()["decision.spf_runs"]
    assert got == len(links)
    assert E.get_fb303_counters()["decision.spf_runs.count"] == got


def test_invalidate_drops_every_view(mods):
    """LinkState::invalidate releases the device graph and every memoized
    result: the next getSpfResult runs a new SPF (spf_runs + 1) and still
    equals the oracle's."""
    E, O = mods
    names, adj_dbs, prefix_dbs = RZ.random_network(10, n_nodes=20, n_links=40)
    ea, _ = RZ.load(E, adj_dbs, prefix_dbs, 1)
    oa, _ = RZ.load(O, adj_dbs, prefix_dbs, 1)
    ls = ea["0"]
    ls.getSpfResult(names[0], True)
    E.reset_counters()
    ls.getSpfResult(names[0], True)
    assert E.get_counters().get("decision.spf_runs", 0) == 0  # memo hit
    ls.invalidate()
    _spf_equal(ls, oa["0"], names[0], True)
    assert E.get_counters().get("decision.spf_runs", 0) == 1


@pytest.mark.parametrize("seed", range(3))
def test_ksp2_route_db_device_traces(mods, seed, monkeypatch):
    """KSP2 RouteDbs with the k = 2 traces on the device
    (OPENR_KSP2_DEVICE_TRACE=1, spf_query_trace_paths) equal the oracle's,
    spf_runs included (one counted runSpf per (src, dst, 2) key)."""
    monkeypatch.setenv("OPENR_KSP2_DEVICE_TRACE", "1")
    monkeypatch.setenv("OPENR_SPF_TRACE_CAP", "6")  # some traces overflow to the host
    E, O = mods
    names, adj_dbs, prefix_dbs = RZ.random_network(700 + seed, n_nodes=30, n_links=80)
    ea, ep = RZ.load(E, adj_dbs, prefix_dbs, seed)
    oa, op = RZ.load(O, adj_dbs, prefix_dbs, seed)
    E.reset_counters()
    O.reset_counters()
    es = E.SpfSolver(names[0], True, False)
    os_ = O.SpfSolver(names[0], True, False)
    for node in names[:6]:
        assert es.buildRouteDb(node, ea, ep) == os_.buildRouteDb(node, oa, op), node
    assert E.get_counters().get("decision.spf_runs") == O.get_counters().get("decision.spf_runs")


@pytest.mark.parametrize("seed,heavy", [(0, "0"), (1, "0"), (2, "1"), (3, "1")])
def test_ksp2_route_db_trace_step_budget(mods, seed, heavy, monkeypatch):
    """The device trace's per-query step budgets: a k = 2 trace longer than
    the cursor kernel's (OPENR_SPF_TRACE_BUDGET) goes to the heavy launch, and
    one longer than that launch's (OPENR_SPF_TRACE_HEAVY_BUDGET; any, with the
    heavy launch off) is traced on the host from its row.  With budgets of a
    few steps most traces take those paths; the KSP2 RouteDbs still equal the
    oracle's, spf_runs included."""
    monkeypatch.setenv("OPENR_KSP2_DEVICE_TRACE", "1")
    monkeypatch.setenv("OPENR_SPF_TRACE_BUDGET", "3")
    monkeypatch.setenv("OPENR_SPF_TRACE_HEAVY", heavy)
    monkeypatch.setenv("OPENR_SPF_TRACE_HEAVY_BUDGET", "3")
    E, O = mods
    names, adj_dbs, prefix_dbs = RZ.random_network(720 + seed, n_nodes=30, n_links=80)
    ea, ep = RZ.load(E, adj_dbs, prefix_dbs, seed)
    oa, op = RZ.load(O, adj_dbs, prefix_dbs, seed)
    E.reset_counters()
    O.reset_counters()
    es = E.SpfSolver(names[0], True, False)
    os_ = O.SpfSolver(names[0], True, False)
    for node in names[:6]:
        assert es.buildRouteDb(node, ea, ep) == os_.buildRouteDb(node, oa, op), node
    c = E.get_counters()
    assert c.get("decision.spf_runs") == O.get_counters().get("decision.spf_runs")
    assert c.get("decision.kth2_device_overflows", 0) > 0


@pytest.mark.parametrize("net", ["weighted", "uniform", "grid"])
def test_same_node_rebuilds_reuse_query(mods, net):
    """Rebuilding one node's RouteDb under churn: a batch with the same
    sources and flags as the last one reruns the engine's cached query
    (Engine::lastQuery; transit bits are read at run time) and every other
    change of the graph -- a metric patch, a link overload splice -- drops it
    first.  On a uniform metric the LFA batch (the node and its neighbours,
    their neighbours as helper rows) takes the small-area MS-BFS plan.
    Every build equals the oracle's, with and without the cache
    (OPENR_LS_QUERY_CACHE=0).  On the 8x8 grid (the bench's configs[0]
    loop: node drains elsewhere invalidate every row of the batch) the cache
    must be hit."""
    import os
    import random

    from openr_amd import topologies as TP

    E, O = mods
    if net == "grid":
        topo = TP.grid(8)
        names = topo.names
        adj_dbs, prefix_dbs = {"0": topo.adj_dbs()}, topo.prefix_dbs()
        me = "1"
    else:
        names, adj_dbs, prefix_dbs = RZ.random_network(
            700, n_nodes=40, n_links=90, metric_range=(1, 1) if net == "uniform" else (1, 20))
        me = names[0]
    ea, ep = RZ.load(E, adj_dbs, prefix_dbs, 3)
    oa, op = RZ.load(O, adj_dbs, prefix_dbs, 3)
    es = E.SpfSolver(me, True, True)
    os_ = O.SpfSolver(me, True, True)
    rng = random.Random(5)
    dbs = [copy.deepcopy(d) for d in adj_dbs["0"]]
    E.reset_counters()
    try:
        for step in range(30):
            os.environ["OPENR_LS_QUERY_CACHE"] = "0" if step % 8 == 7 else "1"
            db = rng.choice(dbs)
            kind = rng.random()
            if kind < 0.7 or not db.adjacencies:
                db.isOverloaded = not db.isOverloaded
            elif kind < 0.88:
                adj = rng.choice(db.adjacencies)
                adj.metric = 1 if net != "weighted" and step % 3 else rng.randint(1, 20)
            else:
                adj = rng.choice(db.adjacencies)
                adj.isOverloaded = not adj.isOverloaded
            assert ea["0"].updateAdjacencyDatabase(db) == oa["0"].updateAdjacencyDatabase(db)
            for _ in range(2):  # the second build of the same state hits the memo
                assert es.buildRouteDb(me, ea, ep) == os_.buildRouteDb(me, oa, op), step
    finally:
        os.environ.pop("OPENR_LS_QUERY_CACHE", None)
    if net == "grid":
        assert E.get_counters().get("decision.spf_query_reuses", 0) > 0
