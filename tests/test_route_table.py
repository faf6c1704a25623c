"""All-nodes unicast route table on the device.

AllNodesRouteTable (openr_amd/csrc/host/RouteTable.cpp) runs one all-sources
SPF with next hops over an area and spf_route_table_kernel over every IP /
SP_ECMP prefix: the restatement of SpfSolverImpl::selectEcmpOpenr
(openr/decision/Decision.cpp:668-712 with getBestAnnouncingNodes :544-630,
maybeFilterDrainedNodes :651-666, getNextHopsWithMetric :1093-1179,
getNextHopsThrift :1181-1271).  Parity: for EVERY node, the table's routes
equal the unicast entries of SpfSolver::buildRouteDb(node) (itself checked
against the CPU oracle in test_engine_parity_gpu.py) for those prefixes —
seeded random networks with anycast prefixes, drained nodes, overloaded
links, parallel links and v4 / v6 prefixes, and the benchmark fabric.
"""

import pytest

from tests import randomized as RZ

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def E(gpu_ready):
    import openr_amd._openr_spf as E

    return E


def _ecmp_only(unicast):
    # SR_MPLS prefixes (fd00::/64 in the generator) are not in the table
    return {k: v for k, v in unicast.items() if not bytes(k[0][0] if isinstance(k[0], tuple) else k[0]).startswith(b"\xfd\x00")}


@pytest.mark.parametrize("seed", range(6))
@pytest.mark.parametrize("v4", [True, False])
def test_route_table_matches_build_route_db(E, seed, v4):
    names, adj_dbs, prefix_dbs = RZ.random_network(
        700 + seed, n_nodes=40, n_links=90, overload_prob=0.15, link_overload_prob=0.05
    )
    areas, ps = RZ.load(E, adj_dbs, prefix_dbs, seed)
    table = E.AllNodesRouteTable(areas, "0", ps, v4)
    assert table.spf_ms > 0 and table.route_ms > 0
    solver = E.SpfSolver(names[0], v4, False)
    checked = 0
    for node in names:
        db = solver.buildRouteDb(node, areas, ps)
        got = table.routes(node)
        if db is None:
            assert got == {}, node
            continue
        assert got == _ecmp_only(db["unicast"]), node
        checked += len(got)
    assert checked > 0


def test_route_table_fabric(E):
    from openr_amd import topologies as TP

    topo = TP.fabric(600)
    areas = E.AreaLinkStates()
    ls = areas.add("0")
    dbs = topo.adj_dbs(overloaded=[5, 77])
    for db in dbs:
        ls.updateAdjacencyDatabase(db)
    ps = E.PrefixState()
    for pdb in topo.prefix_dbs("0"):
        ps.updatePrefixDatabase(pdb)
    table = E.AllNodesRouteTable(areas, "0", ps, True)
    assert table.num_nodes == topo.num_nodes and table.num_prefixes == topo.num_nodes
    solver = E.SpfSolver("2-0-0", False, False)
    for node in sorted(topo.names)[:: max(1, topo.num_nodes // 25)] + ["2-0-0"]:
        db = solver.buildRouteDb(node, areas, ps)
        assert table.routes(node) == db["unicast"], node
