"""RouteDb goldens of the fabric benchmark node under link flaps (TEST
INFRASTRUCTURE).

Run in the build container:  python tests/golden/make_linkflap_golden.py

Writes tests/golden/fabric_linkflap.json.gz: for each of the first FLAPS
link-down states of bench.py's link-flap loop (the RSW rsw[(it * 7919) % n]
of iteration `it` withdraws its FIRST adjacency, so the link to that FSW goes
down: LinkState.cpp updateAdjacencyDatabase drops a link once one side stops
announcing it), the SP_ECMP RouteDb of "2-0-0" as built by the CPU oracle
(oracle/ref_decision.cpp SpfSolver::buildRouteDb, Decision.cpp:291-542), as
a digest plus the per-route delta against the base state of
tests/golden/fabric_routedb.json.gz (tests/golden/routes.py).
"""

from __future__ import annotations

import multiprocessing as mp
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

NODE = "2-0-0"
OUT = os.path.join(HERE, "fabric_linkflap.json.gz")
FLAPS = 4


def flap_sequence(topo, n=FLAPS):
    """bench.py _rebuild_loop(mode="link")'s RSW choice per iteration."""
    rsw = [i for i, nm in enumerate(topo.names) if nm.startswith("3-")]
    return [rsw[(it * 7919) % len(rsw)] for it in range(n)]


def link_down(dbs, rsw):
    """The flap's down state: the RSW's first adjacency withdrawn (returns
    the full list, to restore)."""
    full = dbs[rsw].adjacencies
    dbs[rsw].adjacencies = full[1:]
    return full


def _job(rsw):
    from oracle import _oracle_ref as O
    from openr_amd import topologies as TP
    from tests.golden import routes as R

    topo = TP.fabric(10000)
    dbs = topo.adj_dbs()
    peer = dbs[rsw].adjacencies[0].otherNodeName
    link_down(dbs, rsw)
    areas = O.AreaLinkStates()
    ls = areas.add("0")
    for db in dbs:
        ls.updateAdjacencyDatabase(db)
    ps = O.PrefixState()
    for pdb in topo.prefix_dbs("0"):
        ps.updatePrefixDatabase(pdb)
    db = O.SpfSolver(NODE, False, False).buildRouteDb(NODE, areas, ps)
    return rsw, peer, R.route_hashes(db)


def main():
    from oracle import build as OB

    OB.build()
    from openr_amd import topologies as TP
    from tests.golden import routes as R

    topo = TP.fabric(10000)
    base = R.load(os.path.join(HERE, "fabric_routedb.json.gz"))["sp_ecmp"]["base"]["hashes"]
    seq = flap_sequence(topo)
    t0 = time.time()
    out = {"topology": "fabric_full(10000)", "node": NODE, "flap_rsws": [topo.names[r] for r in seq],
           "generator": "oracle/ref_decision.cpp SpfSolver::buildRouteDb "
                        "(tests/golden/make_linkflap_golden.py)", "states": {}}
    with mp.get_context("spawn").Pool(min(4, os.cpu_count() or 1)) as pool:
        for rsw, peer, h in pool.imap_unordered(_job, sorted(set(seq))):
            out["states"][f"linkdown:{topo.names[rsw]}"] = {
                "peer": peer, "digest": R.digest(h), "num_unicast": len(h["unicast"]),
                "num_mpls": len(h["mpls"]), "delta_vs_base": R.delta(h, base)}
            print(f"[{time.time() - t0:6.1f}s] {topo.names[rsw]} - {peer}", flush=True)
    R.save(OUT, out)
    print(f"wrote {OUT} ({os.path.getsize(OUT)} bytes) in {time.time() - t0:.0f}s")


if __name__ == "__main__":
    main()
