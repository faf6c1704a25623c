"""Probe: bench.py's link-flap RouteDb loop alone (fabric, one GPU), with
the per-build split (graph_build_us = the LinkState engine flatten +
spf_graph_create)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from openr_amd import topologies as TP  # noqa: E402


def main():
    import torch

    torch.cuda.init()
    print(json.dumps(bench.route_db_link_flap(TP.fabric(10000), 0)), flush=True)


if __name__ == "__main__":
    main()
