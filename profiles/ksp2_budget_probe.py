"""Probe: the KSP2 rebuild loop (fabric, 2-0-0) under env settings given as
arguments ("OPENR_SPF_TRACE_BUDGET=1024,OPENR_SPF_TRACE_HEAVY=1" ...), one
JSON line per setting: build ms and the per-build device trace time."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402,F401

import bench  # noqa: E402
from openr_amd import topologies as TP  # noqa: E402

topo = TP.fabric(10000)
for setting in sys.argv[1:] or [""]:
    env = dict(kv.split("=", 1) for kv in setting.split(",") if kv)
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    r = bench.ksp2_route_db(topo, 0, iters=2)
    pb = r["per_build"]
    print(json.dumps({"env": env, "ms_median": r["ms_median"], "build_ms_median": r["build_ms_median"],
                      "kth2_device_trace_us": pb.get("kth2_device_trace_us"),
                      "kth2_device_overflows": pb.get("kth2_device_overflows"),
                      "spf_device_us": pb.get("spf_device_us"), "parity": r.get("parity_check")}), flush=True)
    for k, v in old.items():
        if v is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = v
