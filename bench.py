#!/usr/bin/env python
"""bench.py — BASELINE.json metric: all-sources SPF/sec + GTEPS on the 10k-node
fabric (config 2, DecisionBenchmark.cpp:438-587 with the SSW bug fixed), plus
the full RouteDb rebuild ms of the fabric benchmark node.

One step = one pass of the hot path over one batch: every source of the
fabric (9,976 single-source SPFs with ECMP next-hop sets), inputs (device CSR)
resident in HBM before the timed region, outputs (distance rows + next-hop
masks, ~1.4 GB) written to HBM.  Multi-GPU (one process per GPU, launched by
torch.distributed.run): weak scaling — rank r computes the all-sources table
of drain scenario r (rank 0: no drain; rank r > 0: one RSW drained), no
collective on the data path.  `value` = SPFs of all ranks / max-over-ranks
step time.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--no-cpu-baseline]
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-route-db", action="store_true")
    p.add_argument("--cpu-sample", type=int, default=0, help="oracle sources (0 = auto ~15 s)")
    p.add_argument("--num-sws", type=int, default=10000)
    return p.parse_args()


def algorithmic_bytes(csr, nh_words):
    """SURVEY §8(d) per-SSSP bytes: 8E + 4(V+1) + 4V + 8V*Wm, summed over
    the batch (Wm = next-hop mask words of each source)."""
    V = csr.num_nodes
    E = len(csr.col)
    per = 8 * E + 4 * (V + 1) + 4 * V
    return per * len(nh_words) + 8 * V * int(sum(nh_words))


def cpu_baseline(topo, sample):
    """The oracle's reference-style runSpf (DijkstraQ, string maps, reMake),
    single thread, on a bounded sample of the same all-sources workload."""
    from oracle import build as obuild

    obuild.build()
    from oracle import _oracle_ref as O

    ls = O.LinkState("0")
    for db in topo.adj_dbs():
        ls.updateAdjacencyDatabase(db)
    names = sorted(topo.names)
    step = max(1, len(names) // max(sample, 1))
    srcs = names[::step][:sample] if sample else []
    if not sample:
        # calibrate: time 5 sources, then size the sample to ~15 s
        t5, _ = ls.runSpfTimed(names[:5], True)
        sample = max(5, min(len(names), int(15.0 / max(t5 / 5, 1e-6))))
        step = max(1, len(names) // sample)
        srcs = names[::step][:sample]
    sec, reached = ls.runSpfTimed(srcs, True)
    return {
        "value": round(len(srcs) / sec, 3),
        "unit": "SPF/s",
        "cores": 1,
        "kind": "port",
        "sample": f"{len(srcs)} sources of the 9,976-node fabric, uncached "
        f"runSpf(useLinkMetric=true) each ({sec:.1f} s, {reached} nodes settled); "
        "oracle/ref_decision.cpp restatement of LinkState.cpp:806-880",
    }


def route_db_rebuild_ms(topo, device, iters=5):
    """Full RouteDb rebuild of the benchmark node "2-0-0" after an RSW
    overload toggle (the DecisionBenchmark BM_DecisionFabric loop,
    DecisionBenchmark.cpp:600-626): LinkState update + device graph rebuild
    + SPF (LFA off, as the benchmark's Decision) + RouteDb."""
    import openr_amd._openr_spf as E
    from openr_amd import thrift as T

    E.set_spf_device(device)
    areas = E.AreaLinkStates()
    ls = areas.add("0")
    dbs = topo.adj_dbs()
    for db in dbs:
        ls.updateAdjacencyDatabase(db)
    ps = E.PrefixState()
    for pdb in topo.prefix_dbs():
        ps.updatePrefixDatabase(pdb)
    solver = E.SpfSolver("2-0-0", False, False)
    solver.buildRouteDbTimed("2-0-0", areas, ps)  # cold: builds the device graph
    rsw = [i for i, n in enumerate(topo.names) if n.startswith("3-")]
    times, builds = [], []
    routes = 0
    for it in range(iters):
        db = dbs[rsw[(it * 7919) % len(rsw)]]
        for overloaded in (True, False):
            db.isOverloaded = overloaded
            t0 = time.perf_counter()
            ls.updateAdjacencyDatabase(db)
            nu, nm, us = solver.buildRouteDbTimed("2-0-0", areas, ps)
            times.append((time.perf_counter() - t0) * 1000.0)
            builds.append(us / 1000.0)
            routes = nu + nm
    times.sort()
    builds.sort()
    return {"ms_median": round(times[len(times) // 2], 3),
            "build_ms_median": round(builds[len(builds) // 2], 3),
            "routes": routes, "node": "2-0-0", "samples": len(times),
            "what": "adj-db update (RSW overload toggle) + buildRouteDb, LFA off"}


def main():
    args = parse()
    import numpy as np
    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist

        torch.cuda.set_device(local)
        dist.init_process_group("nccl")
    else:
        torch.cuda.set_device(0)
    from openr_amd import abi, build
    from openr_amd import topologies as TP

    build.build()
    topo = TP.fabric(args.num_sws)
    # drain scenario of this rank (weak scaling: one all-sources table each)
    rsw = [i for i, n in enumerate(topo.names) if n.startswith("3-")]
    drained = [] if rank == 0 else [rsw[(rank * 1009) % len(rsw)]]
    csr = topo.csr(overloaded=drained)
    g = abi.Graph(csr, device=local)
    stream = torch.cuda.Stream()  # a real (non-null) stream shared with the engine
    torch.cuda.set_stream(stream)
    g.set_stream(stream.cuda_stream)
    sources = np.arange(csr.num_nodes, dtype=np.uint32)
    q = g.query(sources, abi.SPF_F_NEXTHOPS)
    nh_words = [q.nh_words(i) for i in range(len(sources))]
    for _ in range(args.warmup):
        q.run(sync=False)
    torch.cuda.synchronize()

    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(args.steps):
        q.run(sync=False)
    ev1.record(stream)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    wall = time.perf_counter() - t0
    kernel_ms = ev0.elapsed_time(ev1) / args.steps
    step_ms = wall * 1000.0 / args.steps
    if dist:
        t = torch.tensor([step_ms, kernel_ms], device="cuda", dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        step_ms, kernel_ms = float(t[0]), float(t[1])

    nsrc = len(sources)
    E = len(csr.col)
    value = world * nsrc / (step_ms / 1000.0)
    abytes = algorithmic_bytes(csr, nh_words)
    achieved = abytes / (kernel_ms / 1000.0) / 1e9
    # spot-check this run against the oracle restatement (3 sources, rank 0)
    check = None
    if rank == 0:
        from oracle import spf_py

        bad = 0
        for i in (0, nsrc // 2, nsrc - 1):
            ref = spf_py.run_spf(csr, int(sources[i]), True)
            d = q.dist(i)
            got = q.nexthop_sets(i, int(sources[i]))
            for v in range(csr.num_nodes):
                if v in ref:
                    bad += int(d[v]) != ref[v][0] or (v != sources[i] and got[v] != ref[v][1])
                else:
                    bad += d[v] != np.uint64(abi.SPF_UNREACHABLE)
        check = "ok" if bad == 0 else f"{bad} mismatches"

    out = {
        "metric": "all-sources SPF/sec + GTEPS on 10k-node fabric; full RouteDb rebuild ms",
        "value": round(value, 1),
        "unit": "SPF/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(step_ms, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic fabric (DecisionBenchmark createFabric, SSW bug fixed), metric 1",
        "config": {
            "workload": "fabric_full all-sources SPF + ECMP next-hop sets",
            "nodes": csr.num_nodes,
            "links": int(csr.num_links),
            "directed_edges": E,
            "sources_per_gpu": nsrc,
            "kernel": q.kernel,
            "parallelism": f"source-batch per GPU, drain scenario per rank (x{world})",
        },
        "gteps": round(world * nsrc * E / (step_ms / 1000.0) / 1e9, 2),
        "kernel_ms": round(kernel_ms, 4),
        "parity_spot_check": check,
        "roofline": {
            "bound": "hbm",
            "achieved": round(achieved, 1),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": None,
            "algorithmic_bytes_per_launch": abytes,
        },
    }
    if rank == 0 and world == 1 and not args.no_route_db:
        try:
            out["route_db_rebuild"] = route_db_rebuild_ms(topo, local)
        except Exception as e:  # reported, never silently replaced
            out["route_db_rebuild"] = {"error": repr(e)}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(topo, args.cpu_sample)
    if rank == 0:
        print(json.dumps(out), flush=True)
    q.close()
    g.close()
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
