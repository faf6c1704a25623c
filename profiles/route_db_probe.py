"""RouteDb rebuild probe: the bench's fabric rebuild loop (LFA off) and the
KSP2 rebuild loop of node "2-0-0", with the warm per-build phase counters.

    python profiles/route_db_probe.py [iters] > gpurun_out/route_db_probe.json
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if os.environ.get("OPENR_PROBE_PKG"):  # A/B: another build of the package first
    sys.path.insert(0, os.environ["OPENR_PROBE_PKG"])

import torch  # noqa: F401,E402  (torch's HIP runtime first, see tests/conftest.py)

import openr_amd  # noqa: E402  (before bench, which puts the repo root first)
import openr_amd._openr_spf  # noqa: F401,E402
import bench  # noqa: E402
from openr_amd import topologies  # noqa: E402

iters = int(sys.argv[1]) if len(sys.argv) > 1 else 6
topo = topologies.fabric(10000)

out = {"package": os.path.dirname(openr_amd.__file__),
       "route_db_rebuild": bench.route_db_rebuild_ms(topo, 0, iters=iters)}
print(json.dumps(out), flush=True)
out["ksp2_route_db"] = bench.ksp2_route_db(topo, 0, iters=max(2, iters // 2))
print(json.dumps(out), flush=True)
