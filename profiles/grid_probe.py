"""BASELINE configs[0] breakdown: the 10x10 grid RouteDb loop of bench.py's
grid_route_db (DecisionBenchmark.cpp:360-431: an overload toggle, then
buildRouteDb("1") with LFA on), engine vs oracle, with the engine's per-phase
counters averaged per build (update / prefetch / SPF batch / device / host).

  python profiles/grid_probe.py [--iters 200]
"""

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--iters", type=int, default=200)
    args = p.parse_args()
    import torch

    torch.cuda.init()
    import openr_amd._openr_spf as E
    from oracle import build as obuild
    from openr_amd import topologies as TP

    obuild.build()
    from oracle import _oracle_ref as O

    E.set_spf_device(0)
    topo = TP.grid(10)
    out = {}
    for tag, M in (("engine", E), ("cpu_oracle", O)):
        areas = M.AreaLinkStates()
        ls = areas.add("0")
        dbs = topo.adj_dbs()
        for db in dbs:
            ls.updateAdjacencyDatabase(db)
        ps = M.PrefixState()
        for pdb in topo.prefix_dbs():
            ps.updatePrefixDatabase(pdb)
        solver = M.SpfSolver("1", False, True)
        for _ in range(5):
            solver.buildRouteDbTimed("1", areas, ps)
        M.reset_counters()
        upd, build, tot = [], [], []
        for it in range(args.iters):
            db = dbs[(it * 37 + 11) % len(dbs)]
            for ov in (True, False):
                db.isOverloaded = ov
                t0 = time.perf_counter()
                ls.updateAdjacencyDatabase(db)
                t1 = time.perf_counter()
                solver.buildRouteDbTimed("1", areas, ps)
                t2 = time.perf_counter()
                upd.append((t1 - t0) * 1e3)
                build.append((t2 - t1) * 1e3)
                tot.append((t2 - t0) * 1e3)
        med = lambda x: round(sorted(x)[len(x) // 2], 4)  # noqa: E731
        n = len(tot)
        c = M.get_counters()
        per = {k: round(v / n, 2) for k, v in sorted(c.items())
               if isinstance(v, (int, float)) and k.endswith("_us")}
        out[tag] = {"ms_median": med(tot), "update_ms_median": med(upd),
                    "build_ms_median": med(build), "samples": n, "per_build_us": per}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
