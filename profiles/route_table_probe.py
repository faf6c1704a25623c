"""Probe: run only bench.py's all-nodes route table section (fabric, one
GPU) so PMC passes over it see spf_route_table_kernel's plain and LFA
launches alone.  With --breakdown: build the table 5 times and print the
per-build split of AllNodesRouteTable's constructor and destructor
(decision.route_table_*_us counters) instead.

  python profiles/route_table_probe.py [--breakdown]
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from openr_amd import topologies as TP  # noqa: E402


def breakdown(topo, n=5):
    import torch

    torch.cuda.init()
    import openr_amd._openr_spf as E

    E.set_spf_device(0)
    areas = E.AreaLinkStates()
    ls = areas.add("0")
    for db in topo.adj_dbs():
        ls.updateAdjacencyDatabase(db)
    ps = E.PrefixState()
    for pdb in topo.prefix_dbs("0"):
        ps.updatePrefixDatabase(pdb)
    t = E.AllNodesRouteTable(areas, "0", ps, True)
    del t
    E.reset_counters()
    walls = []
    table = None
    for _ in range(n):
        t0 = time.perf_counter()
        table = E.AllNodesRouteTable(areas, "0", ps, True)
        walls.append((time.perf_counter() - t0) * 1e3)
        t0 = time.perf_counter()
        del table
        walls[-1] = (walls[-1], (time.perf_counter() - t0) * 1e3)
    c = E.get_counters()
    out = {k.split(".", 1)[1]: round(v / n / 1e3, 3) for k, v in c.items() if "route_table_" in k and k.endswith("_us")}
    print(json.dumps({"builds": n, "build_ms": [round(a, 2) for a, _ in walls],
                      "destroy_ms": [round(b, 2) for _, b in walls], "split_ms": out}), flush=True)


def main():
    topo = TP.fabric(10000)
    if "--breakdown" in sys.argv:
        breakdown(topo)
        return
    r = bench.all_nodes_route_table(topo, 0, reps=1)
    print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
