"""A/B of the fabric RouteDb loops (bench.py route_db_rebuild_ms, LFA off and
on, and ksp2_route_db) under two settings of one environment switch, the
settings interleaved so both see the same box:

    python profiles/rdb_ab.py VAR OFF ON [rounds] [ksp2]

(with "ksp2" the KSP2 loop only)
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: F401,E402

import openr_amd  # noqa: E402
import openr_amd._openr_spf  # noqa: F401,E402
import bench  # noqa: E402
from openr_amd import topologies  # noqa: E402

var, a, b = sys.argv[1:4]
rounds = int(sys.argv[4]) if len(sys.argv) > 4 else 2
topo = topologies.fabric(10000)
res = {a: [], b: []}
for r in range(rounds):
    for val in (a, b):
        os.environ[var] = val
        if "ksp2" in sys.argv[5:]:
            row = {"ksp2": bench.ksp2_route_db(topo, 0, iters=4)}
        else:
            row = {"lfa": bench.route_db_rebuild_ms(topo, 0, lfa=True),
                   "plain": bench.route_db_rebuild_ms(topo, 0)}
        res[val].append({k: {kk: vv for kk, vv in v.items() if kk.endswith("ms_median")}
                         for k, v in row.items()})
        print(var, val, json.dumps(res[val][-1]), flush=True)
print(json.dumps(res))
