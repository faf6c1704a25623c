"""Full-size RouteDb goldens of the fabric benchmark node (TEST INFRASTRUCTURE).

Run in the build container:  python tests/golden/make_routedb_golden.py

Writes tests/golden/fabric_routedb.json.gz: the RouteDb of "2-0-0" on
fabric_full(10000) as built by the CPU oracle (oracle/ref_decision.cpp, the
reference-style restatement of SpfSolverImpl::buildRouteDb, Decision.cpp:
291-542, pinned by the reference's known answers), as per-route hashes
(tests/golden/routes.py):

  sp_ecmp/base             every prefix IP / SP_ECMP, LFA off -- the RouteDb
                           DecisionBenchmark rebuilds (DecisionBenchmark.cpp:
                           600-626); full per-route hashes
  sp_ecmp/overload:<rsw>   the same after the bench's RSW overload toggles
                           (bench.py _rebuild_loop picks rsw[(it * 7919) %
                           n] for it = 0..7); digest + delta vs base
  sp_ecmp_lfa/base         LFA on (computeLfaPaths, Decision.cpp:1146-1175);
                           full hashes -- the Decision DecisionBenchmark
                           actually runs (DecisionBenchmark.cpp:74-79)
  sp_ecmp_lfa/overload:<rsw>  LFA on after each of the bench's RSW overload
                           toggles; digest + delta vs base (`--lfa-states`
                           adds these to an existing file without rebuilding
                           the other sections)
  nodes/<name>             SP_ECMP base RouteDb of the other nodes the bench's
                           all-nodes table checks; digest + route counts
  ksp2/base                every prefix SR_MPLS / KSP2_ED_ECMP: the k = 1 and
                           k = 2 edge-disjoint paths to all 9,975 destinations
                           (LinkState.cpp:760-789, selectKsp2 Decision.cpp:
                           909-1066); full hashes
  ksp2/overload:<rsw>      KSP2 after the first overload toggle; delta vs base

The KSP2 builds are split over processes by prefix (each process loads the
whole LSDB and a slice of the prefix databases: a prefix's route reads only
its own announcers and the shared path memo, so the slices' unicast routes
are exactly the full build's; node-label MPLS routes come from slice 0).
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
OUT = os.path.join(HERE, "fabric_routedb.json.gz")
TOGGLES = 8


def rsw_sequence(topo, n=TOGGLES):
    """bench.py _rebuild_loop's RSW choice per iteration."""
    rsw = [i for i, nm in enumerate(topo.names) if nm.startswith("3-")]
    return [rsw[(it * 7919) % len(rsw)] for it in range(n)]


def _job(args):
    kind, overload, node, lfa, chunk, nchunks = args
    from oracle import _oracle_ref as O
    from openr_amd import thrift as T
    from openr_amd import topologies as TP
    from tests.golden import routes as R

    topo = TP.fabric(10000)
    dbs = topo.adj_dbs()
    if overload is not None:
        dbs[overload].isOverloaded = True
    areas = O.AreaLinkStates()
    ls = areas.add("0")
    for db in dbs:
        ls.updateAdjacencyDatabase(db)
    fwd = (T.PrefixForwardingType.SR_MPLS, T.PrefixForwardingAlgorithm.KSP2_ED_ECMP) \
        if kind == "ksp2" else (0, 0)
    pdbs = topo.prefix_dbs("0", *fwd)
    ps = O.PrefixState()
    for pdb in pdbs[chunk::nchunks]:
        ps.updatePrefixDatabase(pdb)
    t0 = time.time()
    db = O.SpfSolver(node, False, lfa).buildRouteDb(node, areas, ps)
    h = R.route_hashes(db)
    if chunk != 0:
        h["mpls"] = {}
    return args, h, time.time() - t0


def lfa_states():
    """Add sp_ecmp_lfa/overload:<rsw> for every toggle of the bench loop to
    the committed file (the other sections are left as they are)."""
    from oracle import build as OB

    OB.build()
    from openr_amd import topologies as TP
    from tests.golden import routes as R

    topo = TP.fabric(10000)
    gold = R.load(OUT)
    base = gold["sp_ecmp_lfa"]["base"]["hashes"]
    toggles = sorted(set(rsw_sequence(topo)))
    jobs = [("sp_ecmp_lfa", t, NODE, True, 0, 1) for t in toggles]
    t0 = time.time()
    with mp.get_context("spawn").Pool(min(8, os.cpu_count() or 1)) as pool:
        for args, h, dt in pool.imap_unordered(_job, jobs):
            ov = args[1]
            gold["sp_ecmp_lfa"][f"overload:{topo.names[ov]}"] = {
                "digest": R.digest(h), "num_unicast": len(h["unicast"]), "num_mpls": len(h["mpls"]),
                "delta_vs_base": R.delta(h, base)}
            print(f"[{time.time() - t0:7.1f}s] sp_ecmp_lfa overload={topo.names[ov]} {dt:.1f}s", flush=True)
    R.save(OUT, gold)
    print(f"wrote {OUT} ({os.path.getsize(OUT)} bytes) in {time.time() - t0:.0f}s")


def main():
    if "--lfa-states" in sys.argv:
        return lfa_states()
    from oracle import build as OB

    OB.build()
    from openr_amd import topologies as TP
    from tests.golden import routes as R

    topo = TP.fabric(10000)
    names = sorted(topo.names)
    toggles = rsw_sequence(topo)
    other_nodes = [names[len(names) // 2], names[-1]]
    nk = 32  # KSP2 slices per state
    jobs = [("sp_ecmp", None, NODE, False, 0, 1), ("sp_ecmp_lfa", None, NODE, True, 0, 1)]
    jobs += [("sp_ecmp", t, NODE, False, 0, 1) for t in sorted(set(toggles))]
    jobs += [("sp_ecmp_lfa", t, NODE, True, 0, 1) for t in sorted(set(toggles))]
    jobs += [("nodes", None, n, False, 0, 1) for n in other_nodes]
    jobs += [("ksp2", ov, NODE, False, c, nk) for ov in (None, toggles[0]) for c in range(nk)]
    t0 = time.time()
    results = {}
    with mp.get_context("spawn").Pool(min(8, os.cpu_count() or 1)) as pool:
        for args, h, dt in pool.imap_unordered(_job, jobs):
            kind, ov, node, lfa, c, n = args
            acc = results.setdefault((kind, ov, node), {"unicast": {}, "mpls": {}})
            for k in ("unicast", "mpls"):
                acc[k].update(h[k])
            print(f"[{time.time() - t0:7.1f}s] {kind} overload={ov} node={node} slice {c}/{n} "
                  f"{dt:.1f}s", flush=True)

    def state_name(ov):
        return "base" if ov is None else f"overload:{topo.names[ov]}"

    out = {"topology": "fabric_full(10000)", "node": NODE, "toggle_rsws": [topo.names[t] for t in toggles],
           "generator": "oracle/ref_decision.cpp SpfSolver::buildRouteDb (tests/golden/make_routedb_golden.py)"}
    for kind in ("sp_ecmp", "sp_ecmp_lfa", "ksp2"):
        base = results[(kind, None, NODE)]
        sec = {"base": {"digest": R.digest(base), "num_unicast": len(base["unicast"]),
                        "num_mpls": len(base["mpls"]), "hashes": base}}
        for (k2, ov, node), h in results.items():
            if k2 == kind and ov is not None:
                sec[state_name(ov)] = {"digest": R.digest(h), "num_unicast": len(h["unicast"]),
                                       "num_mpls": len(h["mpls"]), "delta_vs_base": R.delta(h, base)}
        out[kind] = sec
    out["nodes"] = {node: {"digest": R.digest(h), "num_unicast": len(h["unicast"]), "num_mpls": len(h["mpls"])}
                    for (k2, ov, node), h in results.items() if k2 == "nodes"}
    R.save(OUT, out)
    print(f"wrote {OUT} ({os.path.getsize(OUT)} bytes) in {time.time() - t0:.0f}s")


if __name__ == "__main__":
    main()
