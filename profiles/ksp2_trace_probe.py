"""Probe: the KSP2 rebuild loop (fabric, 2-0-0) with the device-trace
kernel's waves per CU set by OPENR_SPF_TRACE_WPC (the per-wave node-state
arrays are V x 16 B each: fewer waves = a smaller footprint), one JSON line
per setting: build ms and the per-build device trace time."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402,F401

import bench  # noqa: E402
from openr_amd import topologies as TP  # noqa: E402

topo = TP.fabric(10000)
for wpc in sys.argv[1:] or ["16", "8", "4"]:
    os.environ["OPENR_SPF_TRACE_WPC"] = wpc
    r = bench.ksp2_route_db(topo, 0, iters=2)
    pb = r["per_build"]
    print(json.dumps({"wpc": int(wpc), "ms_median": r["ms_median"], "build_ms_median": r["build_ms_median"],
                      "kth2_device_trace_us": pb.get("kth2_device_trace_us"),
                      "spf_device_us": pb.get("spf_device_us"), "parity": r.get("parity_check")}), flush=True)
