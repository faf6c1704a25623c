"""Probe: device time of the weighted distance plans on the 100k WAN
(sampled sources), one line per env configuration.
usage: tools_wan_probe.py N_SOURCES [ENV=VAL,ENV=VAL ...]   (NH=1: with
next-hop masks)"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from openr_amd import abi  # noqa: E402
from openr_amd import topologies as TP  # noqa: E402

V, L = 100000, 1000000
topo = TP.wan(V, L)
csr = topo.csr()
g = abi.Graph(csr)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 512
for cfg in sys.argv[2:] or ["-"]:
    env = dict(kv.split("=") for kv in cfg.split(",") if "=" in kv)
    flags = abi.SPF_F_NEXTHOPS if env.pop("NH", "0") == "1" else 0
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    srcs = np.arange(0, V, max(1, V // n), dtype=np.uint32)[:n]
    q = g.query(srcs, flags)
    q.run()
    q.run()
    ms = q.elapsed_ms()
    d = q.dist(0)
    print(json.dumps({"cfg": cfg, "n": int(len(srcs)), "kernel": q.kernel, "ms": round(ms, 2),
                      "ms_per_src": round(ms / len(srcs), 5), "sum0": int(d.sum())}), flush=True)
    q.close()
    for k, v in old.items():
        if v is None:
            os.environ.pop(k)
        else:
            os.environ[k] = v
