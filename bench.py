#!/usr/bin/env python
"""bench.py — BASELINE.json metric: all-sources SPF/sec + GTEPS on the 10k-node
fabric (config 2, DecisionBenchmark.cpp:438-587 with the SSW bug fixed), plus
the full RouteDb rebuild ms of the fabric benchmark node.

One step = one pass of the hot path over one batch: every source of the
fabric (9,976 single-source SPFs with ECMP next-hop sets), inputs (device CSR)
resident in HBM before the timed region, outputs (distance rows + next-hop
masks, ~1.4 GB) written to HBM.  Multi-GPU (one process per GPU, launched by
torch.distributed.run; or --sharded on one GPU): STRONG scaling of the one
9,976-source table through the engine's own multi-GPU path (spf_cluster /
spf_table: contiguous source blocks per GPU, in-place RCCL all-gather of the
rows and next-hop masks over xGMI).  `value` = 9,976 SPFs / max-over-ranks
step time, gather included.

Roofline: the dominant kernel of the step (the one with the larger average
device time over the timed launches, HIP events on the engine's stream) is
priced by its ALGORITHMIC bytes per launch:
  spf_nh_levels_v2_kernel (held / per-node kernels with OPENR_NL_V2=0 /
  OPENR_NL_SWAR=0)      sum_q [ V + V*B_q + 4*V ]
                         (every level row read once, the byte-strided mask
                          row and the u32 distance row written once)
  spf_msbfs_kernel      sum_q V + 4*E + 4*(V+1) (u8 level rows written, CSR
                         read once; the per-level pull scans are L2-served
                         and reported apart as csr_scan_bytes_l2)
`traffic` comes from the rocprofv3 PMC passes committed under profiles/
(profiles/<round>/pmc_traffic.json, written by profiles/collect_pmc.py).

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--no-cpu-baseline]
"""

from __future__ import annotations

import argparse
import glob
import json
import os
import re
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip table)

# the next-hop stage of the MS-BFS plan: the byte-SIMD held-word kernel
# (+ spf_nh_levels_swar_kernel for sources with > 3 mask words, none on the
# fabric) unless OPENR_NL_SWAR=0 selects the per-node spf_nh_levels_kernel
_NL = "spf_nh_levels_kernel" if os.environ.get("OPENR_NL_SWAR") == "0" else "spf_nh_levels_held_kernel"
KERNELS = {
    "msbfs+levels": ("spf_msbfs_kernel", _NL),
    "bfs+rows": ("spf_bfs_kernel", "spf_nh_rows_kernel"),
    "bfs-gmem+rows": ("spf_bfs_kernel", "spf_nh_rows_kernel"),
    "lds+rows": ("spf_sssp_kernel", "spf_nh_rows_kernel"),
    "gmem+rows": ("spf_sssp_kernel", "spf_nh_rows_kernel"),
}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=None,
                   help="number of GPUs (= ranks, one process per GPU); without an outer "
                        "torch.distributed.run this script starts the N rank processes itself")
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-full", action="store_true",
                   help="time BASELINE.md §3 line A fully on all host cores: config 2 (every fabric "
                        "source) and config 4 (getKthPaths k=1,2 to every destination); minutes")
    p.add_argument("--no-route-db", action="store_true")
    p.add_argument("--cpu-sample", type=int, default=0, help="oracle sources (0 = auto ~15 s)")
    p.add_argument("--num-sws", type=int, default=10000)
    p.add_argument("--no-wan", action="store_true", help="skip the 100k WAN all-sources pass")
    p.add_argument("--no-whatif", action="store_true", help="skip the 8,192 what-if SPF batch")
    p.add_argument("--no-repair", action="store_true", help="skip the WAN table-repair events")
    p.add_argument("--wan-nodes", type=int, default=100000)
    p.add_argument("--wan-links", type=int, default=1000000)
    p.add_argument("--sharded", action="store_true",
                   help="use the multi-GPU spf_table path even at N = 1 (tests it on one GPU)")
    return p.parse_args()


def distinct_nbrs(csr):
    """Distinct neighbours per node (= bits of its next-hop masks)."""
    import numpy as np

    V = csr.num_nodes
    row = csr.row_ptr.astype(np.int64)
    src = np.repeat(np.arange(V, dtype=np.int64), np.diff(row))
    key = np.unique(src * V + csr.col.astype(np.int64))
    return np.bincount(key // V, minlength=V)


def lvl_only():
    """The engine's default (OPENR_MS_LVL_ONLY, spf_device.hip lvl_only):
    the next-hop pass, not the BFS, writes the u32 distance rows."""
    return os.environ.get("OPENR_MS_LVL_ONLY", "1") != "0" and \
        os.environ.get("OPENR_NL_SWAR", "1") != "0"


def nh_levels_bytes(csr, nbrs, nh_bytes, level_bytes=1, dist_rows=False):
    """Compulsory bytes of one next-hop pass launch: every source's level row
    read once (the rows of a source's neighbours are other sources' rows:
    re-reads, served by L2 / MALL when the kernel is good), every next-hop
    mask row written once in the device layout (nh_bytes per node per source:
    1 / 2 / 4 bytes up to 8 / 16 / 32 neighbours, else whole u64 words), and
    with `dist_rows` every source's u32 distance row written once (lvl_only)."""
    import numpy as np

    V = csr.num_nodes
    b = np.asarray(nh_bytes, dtype=np.int64)
    return int(V * level_bytes * len(b) + V * int(b.sum()) + (4 * V * len(b) if dist_rows else 0))


def msbfs_bytes(csr, nsrc, levels_per_batch, dist_rows=True):
    """Compulsory HBM bytes of one spf_msbfs_kernel launch: u8 level rows (and
    u32 distance rows unless the next-hop pass writes them) written once and
    the CSR read once.  The per-level pull scans (one per 64-source batch and
    level, bit-shared by the batch's sources) re-read the CSR from L2; they are
    reported apart (msbfs_scan_bytes), never priced against HBM."""
    V = csr.num_nodes
    E = len(csr.col)
    return int((5 if dist_rows else 1) * V * nsrc + 4 * E + 4 * (V + 1))


def msbfs_scan_bytes(csr, levels_per_batch):
    """CSR bytes the bit-parallel pull scans read (L2-served): one scan per
    64-source batch and BFS level."""
    V = csr.num_nodes
    E = len(csr.col)
    return int(sum(levels_per_batch) * (4 * E + 4 * (V + 1)))


def _profile_files(fname):
    """profiles/<round>/<fname>, oldest first in round order: r04z < r04aa
    (a plain sort puts r04al before r04z)."""
    def key(f):
        d = os.path.basename(os.path.dirname(f))
        m = re.match(r"r(\d+)([a-z]*)$", d)
        return (int(m.group(1)), len(m.group(2)), m.group(2)) if m else (-1, 0, d)
    return sorted(glob.glob(os.path.join(ROOT, "profiles", "*", fname)), key=key)


def pmc_traffic(kernel_name):
    """Per-launch HBM bytes of `kernel_name` from the committed PMC passes
    (FETCH_SIZE x2 gfx950 correction + WRITE_SIZE, MI355X_MICROARCH.md)."""
    files = _profile_files("pmc_traffic.json")
    for f in reversed(files):
        try:
            d = json.load(open(f))
        except Exception:
            continue
        k = d.get("kernels", {}).get(kernel_name)
        if k and "hbm_bytes_per_launch" in k:
            return int(k["hbm_bytes_per_launch"]), os.path.relpath(f, ROOT)
    return None, None


def wan_sssp_bytes(plan, V, E):
    """Algorithmic bytes per SSSP of the WAN all-sources plan (SURVEY §8(d)
    per-SSSP figure without the masks this distance-only pass does not
    produce): the out-edges of every settled node read once, in the format
    the kernel reads, the row pointers, and the u32 distance row written
    once.  The LDS-row plan (spf_dlds_kernel) reads packed edges (head |
    metric << bits, 4 bytes); the HBM-row pass spf_dstep_kernel is priced on
    the separate head / metric arrays (8 bytes), as before."""
    if plan == "dstep-ldsrow":
        return 4 * E + 4 * (V + 1) + 4 * V, "spf_dlds_kernel (LDS-resident 12-bit rows, packed edges)"
    return 8 * E + 4 * (V + 1) + 4 * V, "spf_dstep_kernel (push-only, LDS buckets)"


def pmc_traffic_largest(kernel_name):
    """HBM bytes of the largest dispatch of `kernel_name` in the committed
    PMC passes (the measured launch, not a warm-up batch)."""
    files = _profile_files("pmc_traffic.json")
    for f in reversed(files):
        try:
            d = json.load(open(f))
        except Exception:
            continue
        k = d.get("kernels", {}).get(kernel_name)
        if k and "hbm_bytes_largest_launch" in k:
            return int(k["hbm_bytes_largest_launch"]), os.path.relpath(f, ROOT)
    return None, None


GRAPH_PREP_KERNELS = {"spf_graph_derive_kernel", "spf_sell_kernel"}


def pmc_plan_traffic(launched, fname):
    """HBM bytes of one batch of a multi-kernel plan from the newest
    committed profiles/*/<fname> whose kernel set (runtime copies / fills
    aside) is EXACTLY `launched`, the kernels the plan that ran here launched
    (spf_query_kernels): a profile of another plan is refused, not summed.
    Returns (bytes per batch, file, note)."""
    want = set(launched)
    skipped = []
    for f in reversed(_profile_files(fname)):
        try:
            d = json.load(open(f))
        except Exception:
            continue
        ks = d.get("kernels", {})
        runs = d.get("batches")
        # runtime copies / fills and the graph-preparation kernels (run once
        # when the probe builds its graphs, not per batch) are not the plan's
        have = {k for k in ks if not k.startswith("__amd_rocclr") and k not in GRAPH_PREP_KERNELS}
        if not runs or have != want:
            skipped.append(os.path.relpath(f, ROOT))
            continue
        tot = sum(ks[k]["hbm_bytes_per_launch"] * ks[k]["dispatches"] for k in want)
        return int(tot / runs), os.path.relpath(f, ROOT), None
    note = ("no committed PMC profile of this plan's kernel set "
            f"{sorted(want)}" + (f" (refused: {', '.join(skipped)})" if skipped else ""))
    return None, None, note


def pmc_traffic_smallest(kernel_name):
    """HBM bytes of the smallest dispatch of `kernel_name` in the committed
    PMC passes (a kernel launched in two modes: the plain one)."""
    files = _profile_files("pmc_traffic.json")
    for f in reversed(files):
        try:
            d = json.load(open(f))
        except Exception:
            continue
        k = d.get("kernels", {}).get(kernel_name)
        if k and "hbm_bytes_smallest_launch" in k:
            return int(k["hbm_bytes_smallest_launch"]), os.path.relpath(f, ROOT)
    return None, None


def host_cores():
    """Host threads this process may use: the GPU box gives one GPU's share
    (16) of a larger machine whose nproc shows every CPU."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(16, n))


def host_cpu_model():
    """The host CPU's model name (recorded beside `cores`)."""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform

    return platform.processor() or "unknown"


class _Heartbeat:
    """Writes one stderr line a minute while a long host baseline runs, so a
    supervisor watching the output does not take the run for hung."""

    def __init__(self, what, every=60.0):
        import threading

        self.what, self.every, self.stop = what, every, threading.Event()
        self.t0 = time.perf_counter()
        self.thread = threading.Thread(target=self._run, daemon=True)

    def _run(self):
        while not self.stop.wait(self.every):
            print(f"[bench] {self.what}: {time.perf_counter() - self.t0:.0f} s", file=sys.stderr, flush=True)

    def __enter__(self):
        self.thread.start()
        return self

    def __exit__(self, *exc):
        self.stop.set()
        self.thread.join()


def _ksp2_worker(args):
    """One host process of the full config-4 line A: the oracle's LinkState
    for the fabric, then getKthPaths(2-0-0, d, 1) and (…, 2) for its share
    of the destinations (k = 2 runs an un-memoized runSpf per destination,
    LinkState.cpp:776-777)."""
    num_sws, dests = args
    from oracle import _oracle_ref as O
    from openr_amd import topologies as TP

    topo = TP.fabric(num_sws)
    ls = O.LinkState("0")
    for db in topo.adj_dbs():
        ls.updateAdjacencyDatabase(db)
    ls.getSpfResult("2-0-0", True)
    t0 = time.perf_counter()
    paths = 0
    for d in dests:
        paths += len(ls.getKthPaths("2-0-0", d, 1)) + len(ls.getKthPaths("2-0-0", d, 2))
    return time.perf_counter() - t0, paths, len(dests)


def ksp2_cpu_full(topo, num_sws):
    """BASELINE.md §3 line A for config 4, timed fully: every destination of
    2-0-0 on every host core (destinations dealt round-robin to one process
    per core); wall = the slowest process."""
    import multiprocessing as mp

    from oracle import build as obuild

    obuild.build()
    cores = host_cores()
    names = sorted(n for n in topo.names if n != "2-0-0")
    chunks = [names[i::cores] for i in range(cores)]
    with _Heartbeat("config-4 line A (all destinations)"), mp.get_context("spawn").Pool(cores) as pool:
        res = pool.map(_ksp2_worker, [(num_sws, c) for c in chunks])
    wall = max(r[0] for r in res)
    return {"build_s": round(wall, 2), "destinations": len(names), "paths": sum(r[1] for r in res),
            "cores": cores, "kind": "port", "cpu_model": host_cpu_model(),
            "sample": f"ALL {len(names)} destinations of 2-0-0, oracle/ref_decision.cpp getKthPaths "
                      f"k=1,2 over {cores} processes (one per core); slowest process {wall:.1f} s"}


def _oracle_spf_worker(args):
    """One host process of the all-cores reference-style baseline: the
    oracle's LinkState for the fabric, then uncached runSpf of its sources."""
    num_sws, srcs = args
    from oracle import _oracle_ref as O
    from openr_amd import topologies as TP

    topo = TP.fabric(num_sws)
    ls = O.LinkState("0")
    for db in topo.adj_dbs():
        ls.updateAdjacencyDatabase(db)
    sec, reached = ls.runSpfTimed(srcs, True)
    return sec, reached, len(srcs)


def _roofline(kernel, avg_ms, alg_bytes, traffic, traffic_src):
    """Roofline of the dominant kernel: `achieved` / `frac` = ALGORITHMIC
    bytes per launch (the compulsory bytes DESIGN.md §3 restates for this
    kernel) over its launch time measured live here (HIP events on the
    engine's stream).  The rocprofv3 PMC HBM bytes of the same launch
    (profiles/<round>/pmc_traffic.json) are `traffic`; `traffic_frac` is the
    bandwidth they spent and `traffic_over_algorithmic` the waste factor."""
    out = {"bound": "hbm", "kernel": kernel, "peak": HBM_PEAK_GBS, "unit": "GB/s",
           "avg_launch_ms": avg_ms, "algorithmic_bytes": alg_bytes, "traffic": traffic,
           "traffic_source": traffic_src}
    if alg_bytes and avg_ms:
        a = alg_bytes / (avg_ms / 1e3) / 1e9
        out.update(achieved=round(a, 1), frac=round(a / HBM_PEAK_GBS, 4),
                   basis="algorithmic bytes per launch / live HIP-event launch time")
    if traffic and avg_ms:
        t = traffic / (avg_ms / 1e3) / 1e9
        out.update(traffic_achieved=round(t, 1), traffic_frac=round(t / HBM_PEAK_GBS, 4))
        if alg_bytes:
            out["traffic_over_algorithmic"] = round(traffic / alg_bytes, 3)
    return out


def _routedb_golden():
    """Oracle-made RouteDbs of "2-0-0" (tests/golden/make_routedb_golden.py)."""
    from tests.golden import routes as R

    return R, R.load(os.path.join(ROOT, "tests", "golden", "fabric_routedb.json.gz"))


def _golden_state(R, gold, section, state):
    """Per-route hashes of one golden state (base, or base + its delta)."""
    sec = gold[section]
    if state == "base":
        return sec["base"]["hashes"]
    return R.apply_delta(sec["base"]["hashes"], sec[state]["delta_vs_base"])


def _check_routedb(R, got_db, want, what):
    try:
        R.compare(R.route_hashes(got_db), want, what)
        return None
    except AssertionError as e:
        return str(e)


def _routedb_parity(section, ls, solver, areas, ps, dbs, topo, node="2-0-0"):
    """The bench's RouteDb against the oracle's golden: the base state, then
    the first overload toggle of the timed loop (applied and reverted)."""
    R, gold = _routedb_golden()
    if gold["node"] != node:
        return f"golden is for {gold['node']}"
    errs = []
    e = _check_routedb(R, solver.buildRouteDb(node, areas, ps), _golden_state(R, gold, section, "base"),
                       f"{section} base")
    if e:
        errs.append(e)
    rsw = [i for i, n in enumerate(topo.names) if n.startswith("3-")][0]
    state = f"overload:{topo.names[rsw]}"
    if state in gold[section]:
        dbs[rsw].isOverloaded = True
        ls.updateAdjacencyDatabase(dbs[rsw])
        e = _check_routedb(R, solver.buildRouteDb(node, areas, ps), _golden_state(R, gold, section, state),
                           f"{section} {state}")
        if e:
            errs.append(e)
        dbs[rsw].isOverloaded = False
        ls.updateAdjacencyDatabase(dbs[rsw])
    else:
        errs.append(f"golden lacks {section}/{state}")
    return "ok (oracle golden: base + " + state + ")" if not errs else "; ".join(errs)


def cpu_baseline_all_cores(topo, num_sws, per_core_s=12.0, t_per_spf=None, full=False):
    """The reference-style oracle runSpf on every host core (one process per
    core, sources dealt round-robin), plus the optimised flat CPU
    restatement (oracle/csr_spf.h, int CSR + binary heap + next-hop bitsets)
    over ALL fabric sources on the same cores."""
    import multiprocessing as mp

    import numpy as np

    from oracle import build as obuild

    obuild.build()
    from oracle import _oracle_ref as O

    cores = host_cores()
    names = sorted(topo.names)
    per = max(4, int(per_core_s / max(t_per_spf or 0.09, 1e-4)))
    step = max(1, len(names) // (per * cores))
    pick = names if full else names[::step][: per * cores]
    chunks = [pick[i::cores] for i in range(cores)]
    ctx = mp.get_context("spawn")
    with _Heartbeat("reference-style runSpf on all cores"), ctx.Pool(cores) as pool:
        res = pool.map(_oracle_spf_worker, [(num_sws, c) for c in chunks])
    wall = max(r[0] for r in res)
    nspf = sum(r[2] for r in res)
    csr = topo.csr()
    t0 = time.perf_counter()
    S = O.csr_spf_summary(csr.row_ptr, csr.col, csr.metric.astype(np.uint64), csr.link_id,
                          csr.overloaded, np.arange(csr.num_nodes, dtype=np.uint32), None, None,
                          True, True, cores)
    opt_s = time.perf_counter() - t0
    return {
        "reference_style": {
            "value": round(nspf / wall, 2), "unit": "SPF/s", "cores": cores, "kind": "port",
            "sample": f"{'ALL ' if full else ''}{nspf} fabric sources over {cores} processes (one per "
                      f"core), uncached runSpf (oracle/ref_decision.cpp, reference data structures); "
                      f"slowest process {wall:.1f} s", "cpu_model": host_cpu_model()},
        "optimised": {
            "value": round(csr.num_nodes / opt_s, 1), "unit": "SPF/s", "cores": cores, "kind": "port",
            "sample": f"all {csr.num_nodes} fabric sources with ECMP next-hop sets, oracle/csr_spf.h "
                      f"(int CSR, binary heap, next-hop bitsets) on {cores} threads, {opt_s:.2f} s",
            "checksum_pairs": int(S[:, 2].sum()), "cpu_model": host_cpu_model()},
    }


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


def _rebuild_loop(M, topo, iters, timed, fwd=(0, 0), after_cold=None, check=None, mode="overload",
                  lfa=False):
    """DecisionBenchmark BM_DecisionFabric loop (DecisionBenchmark.cpp:
    600-626): toggle an RSW's overload bit, rebuild the RouteDb of "2-0-0".
    fwd = (PrefixForwardingType, PrefixForwardingAlgorithm) of every prefix;
    after_cold() runs once the cold build is done (counter reset).
    mode="link": flap one link instead -- the RSW withdraws its first
    adjacency (the link to that FSW goes down), then announces it again
    (tests/golden/make_linkflap_golden.py holds the down states)."""
    areas = M.AreaLinkStates()
    ls = areas.add("0")
    dbs = topo.adj_dbs()
    for db in dbs:
        ls.updateAdjacencyDatabase(db)
    ps = M.PrefixState()
    for pdb in topo.prefix_dbs("0", fwd[0], fwd[1]):
        ps.updatePrefixDatabase(pdb)
    solver = M.SpfSolver("2-0-0", False, lfa)
    timed(solver, areas, ps)  # cold build (device graph for the engine)
    if after_cold:
        after_cold()
    rsw = [i for i, n in enumerate(topo.names) if n.startswith("3-")]
    tot, upd, bld, rel = [], [], [], []
    routes = 0
    for it in range(iters):
        db = dbs[rsw[(it * 7919) % len(rsw)]]
        full = db.adjacencies
        for down in (True, False):
            if mode == "link":
                db.adjacencies = full[1:] if down else full
            else:
                db.isOverloaded = down
            t0 = time.perf_counter()
            ls.updateAdjacencyDatabase(db)
            t1 = time.perf_counter()
            r = timed(solver, areas, ps)
            routes, us = r[0], r[1]
            t2 = time.perf_counter()
            tot.append((t2 - t0) * 1e3)
            upd.append((t1 - t0) * 1e3)
            bld.append(us / 1e3)
            if len(r) > 2:
                rel.append(r[2] / 1e3)
    med = lambda x: round(sorted(x)[len(x) // 2], 3)  # noqa: E731
    out = {"ms_median": med(tot), "update_ms_median": med(upd),
           "build_ms_median": med(bld), "routes": routes, "samples": len(tot)}
    if check is not None:
        # after the timed loop, on the same LinkState / solver (untimed)
        try:
            out["parity_check"] = check(ls, solver, areas, ps, dbs)
        except Exception as e:  # reported, never silently replaced
            out["parity_check"] = f"error: {e!r}"
    if rel:
        # freeing the old RouteDb (releaseRouteDb, in ms_median)
        out["release_ms_median"] = med(rel)
    return out


def publication_ingest(topo, reps=3):
    """SURVEY §8(f) row 4, the step before the path: Decision::
    processPublication (Decision.cpp:1631-1763) of the whole fabric LSDB —
    one publication holding every "adj:<node>" and "prefix:<node>" key as a
    CompactProtocol blob — decoded and applied to LinkState / PrefixState by
    PublicationIngest (host C++).  Then one churn publication (an RSW's
    adjacency database with its overload bit set).  The CPU line is the
    oracle's reference-style updateAdjacencyDatabase over already-decoded
    objects (no deserialisation), single thread."""
    import openr_amd._openr_spf as E
    from oracle import build as obuild

    dbs = topo.adj_dbs()
    pdbs = topo.prefix_dbs("0")
    kv = {f"adj:{d.thisNodeName}": E.compact_encode_adj_db(d) for d in dbs}
    kv.update({f"prefix:{p.thisNodeName}": E.compact_encode_prefix_db(p) for p in pdbs})
    nbytes = sum(len(v) for v in kv.values())
    full, churn = [], []
    rsw = next(d for d in dbs if d.thisNodeName.startswith("3-"))
    for _ in range(reps):
        areas, ps = E.AreaLinkStates(), E.PrefixState()
        ing = E.PublicationIngest("2-0-0")
        _, us = ing.processPublicationTimed(areas, ps, "0", kv)
        full.append(us / 1e3)
        ing.resetPending()
        rsw.isOverloaded = True
        _, us = ing.processPublicationTimed(areas, ps, "0", {f"adj:{rsw.thisNodeName}": E.compact_encode_adj_db(rsw)})
        rsw.isOverloaded = False
        churn.append(us / 1e3)
        links = areas["0"].numLinks()
    obuild.build()
    from oracle import _oracle_ref as O

    ols = O.LinkState("0")
    t0 = time.perf_counter()
    for d in dbs:
        ols.updateAdjacencyDatabase(d)
    oracle_ms = (time.perf_counter() - t0) * 1e3
    med = lambda x: round(sorted(x)[len(x) // 2], 2)  # noqa: E731
    return {
        "what": "processPublication of the full fabric LSDB (9,976 adj + 9,976 prefix keys, CompactProtocol) "
                "then one RSW overload churn publication",
        "keys": len(kv), "bytes": nbytes, "links": links,
        "full_ms_median": med(full), "churn_ms_median": med(churn),
        "cpu_oracle_adj_only_ms": round(oracle_ms, 1),
        "cpu_oracle_note": "oracle/ref_decision.cpp updateAdjacencyDatabase of the same adjacency "
                           "databases as objects (no decode, no prefixes), 1 thread",
    }


def route_db_link_flap(topo, device, iters=4):
    """Link flap + buildRouteDb: an RSW withdraws its adjacency to one FSW
    (the link goes down; LinkState.cpp updateAdjacencyDatabase), the
    RouteDb of "2-0-0" is rebuilt, then the adjacency comes back and the
    RouteDb is rebuilt again (SP_ECMP, LFA off).  Parity: the down state of
    the first flap against the oracle's RouteDb
    (tests/golden/fabric_linkflap.json.gz)."""
    import openr_amd._openr_spf as E
    from tests.golden import routes as R

    E.set_spf_device(device)

    def timed(solver, areas, ps):
        nu, nm, us, free_us = solver.buildRouteDbTimed("2-0-0", areas, ps)
        return nu + nm, us, free_us

    counters = {}

    def check(ls, solver, areas, ps, dbs):
        counters.update(E.get_counters())
        gold = R.load(os.path.join(ROOT, "tests", "golden", "fabric_linkflap.json.gz"))
        base = _routedb_golden()[1]["sp_ecmp"]["base"]["hashes"]
        rsw = [i for i, n in enumerate(topo.names) if n.startswith("3-")][0]
        st = gold["states"].get(f"linkdown:{topo.names[rsw]}")
        if st is None:
            return f"golden lacks linkdown:{topo.names[rsw]}"
        full = dbs[rsw].adjacencies
        dbs[rsw].adjacencies = full[1:]
        ls.updateAdjacencyDatabase(dbs[rsw])
        e = _check_routedb(R, solver.buildRouteDb("2-0-0", areas, ps), R.apply_delta(base, st["delta_vs_base"]),
                           f"linkdown:{topo.names[rsw]}")
        dbs[rsw].adjacencies = full
        ls.updateAdjacencyDatabase(dbs[rsw])
        return f"ok (oracle golden: linkdown:{topo.names[rsw]} - {st['peer']})" if e is None else e

    out = _rebuild_loop(E, topo, iters, timed, after_cold=E.reset_counters, check=check, mode="link")
    c = counters or E.get_counters()
    n = max(1, c.get("decision.route_build_runs", 1))
    out["per_build_us"] = {k.split(".", 1)[1]: round(c.get(k, 0) / n, 1)
                           for k in ("decision.graph_build_us", "decision.graph_upload_us",
                                     "decision.graph_patch_us", "decision.graph_update_us", "decision.graph_splice_us", "decision.graph_memo_screen_us",
                                     "decision.spf_batch_us", "decision.spf_device_us",
                                     "decision.route_prefetch_us", "decision.route_prefix_pool_us")}
    out["node"] = "2-0-0"
    out["what"] = "link flap (RSW withdraws / restores its adjacency to one FSW) + buildRouteDb, LFA off"
    return out


def route_db_rebuild_ms(topo, device, iters=5, lfa=False):
    """Full RouteDb rebuild of the benchmark node "2-0-0" after an RSW
    overload toggle: LinkState update + SPF on the engine + RouteDb.
    lfa=True is the Decision DecisionBenchmark runs (computeLfaPaths = true,
    DecisionBenchmark.cpp:74-79): the node's SPF plus its 84 neighbours'
    (the RFC 5286 test of Decision.cpp:1146-1175) in one device batch, LFA
    next hops on the SP_ECMP fast path; lfa=False is the lighter LFA-off
    build, reported beside it."""
    import openr_amd._openr_spf as E

    E.set_spf_device(device)

    def timed(solver, areas, ps):
        nu, nm, us, free_us = solver.buildRouteDbTimed("2-0-0", areas, ps)
        return nu + nm, us, free_us

    counters = {}

    def check(ls, solver, areas, ps, dbs):
        counters.update(E.get_counters())  # the timed builds' counters, before the check's
        return _routedb_parity("sp_ecmp_lfa" if lfa else "sp_ecmp", ls, solver, areas, ps, dbs, topo)

    out = _rebuild_loop(E, topo, iters, timed, after_cold=E.reset_counters, check=check, lfa=lfa)
    c = counters or E.get_counters()
    n = max(1, c.get("decision.route_build_runs", 1))
    # warm builds only (counters reset after the cold build)
    out["per_build_us"] = {
        k.split(".", 1)[1]: round(c.get(k, 0) / n, 1)
        for k in ("decision.graph_build_us", "decision.graph_upload_us",
                  "decision.spf_batch_us", "decision.spf_device_us",
                  "decision.route_prefetch_us", "decision.route_prefix_pool_us",
                  "decision.route_merge_us", "decision.route_label_us",
                  "decision.route_label_pool_us", "decision.route_release_us",
                  "decision.ecmp_best_us", "decision.ecmp_nhnodes_us",
                  "decision.ecmp_thrift_us", "decision.ecmp_insert_us")
    }
    out["builds_counted"] = n
    out["releases_counted"] = c.get("decision.route_releases", 0)
    out["node"] = "2-0-0"
    out["what"] = ("adj-db update (RSW overload toggle) + buildRouteDb, "
                   + ("LFA on (DecisionBenchmark's Decision)" if lfa else "LFA off"))
    return out


def all_nodes_route_table(topo, device, reps=3):
    """the unicast RouteDb of EVERY fabric node at once
    (AllNodesRouteTable: one all-sources SPF with next hops + the
    spf_route_table_kernel over all 9,976 prefixes), against one
    buildRouteDb per node on the host path.  Parity: three nodes' table rows
    equal their buildRouteDb unicast entries."""
    import numpy as np

    import openr_amd._openr_spf as E

    E.set_spf_device(device)
    areas = E.AreaLinkStates()
    ls = areas.add("0")
    for db in topo.adj_dbs():
        ls.updateAdjacencyDatabase(db)
    ps = E.PrefixState()
    for pdb in topo.prefix_dbs("0"):
        ps.updatePrefixDatabase(pdb)
    E.AllNodesRouteTable(areas, "0", ps, True)  # warm (kernels, allocations)
    walls, spf, rt = [], [], []
    for _ in range(reps):
        t0 = time.perf_counter()
        table = E.AllNodesRouteTable(areas, "0", ps, True)
        walls.append((time.perf_counter() - t0) * 1e3)
        spf.append(table.spf_ms)
        rt.append(table.route_ms)
    V, P, NL = table.num_nodes, table.num_prefixes, table.num_label_columns
    routes = table.count_routes()
    # parity against the ORACLE's RouteDbs (tests/golden/fabric_routedb.json.gz),
    # not against this engine's own buildRouteDb
    R, gold = _routedb_golden()
    names = sorted(topo.names)
    bad = []
    for node in ("2-0-0", names[len(names) // 2], names[-1]):
        got = R.route_hashes({"unicast": table.routes(node), "mpls": table.mpls_routes(node)})
        if node == gold["node"]:
            e = _check_routedb(R, {"unicast": table.routes(node), "mpls": table.mpls_routes(node)},
                               _golden_state(R, gold, "sp_ecmp", "base"), node)
            if e:
                bad.append(e)
        elif R.digest(got) != gold["nodes"][node]["digest"]:
            bad.append(f"{node}: digest differs ({len(got['unicast'])} unicast, {len(got['mpls'])} mpls "
                       f"vs {gold['nodes'][node]['num_unicast']}, {gold['nodes'][node]['num_mpls']})")
    n_mat, us_mat = table.routes_timed("2-0-0")
    # the same table with loop-free alternates (SPF_RT_LFA): per-link metrics
    # for every (node, column, up link) -- (P + labels) x E cells
    lfa_walls, lfa_rt = [], []
    for _ in range(2):
        t0 = time.perf_counter()
        lt = E.AllNodesRouteTable(areas, "0", ps, True, True)
        lfa_walls.append((time.perf_counter() - t0) * 1e3)
        lfa_rt.append(lt.route_ms)
    lfa_err = _check_routedb(R, {"unicast": lt.routes("2-0-0"), "mpls": lt.mpls_routes("2-0-0")},
                             _golden_state(R, gold, "sp_ecmp_lfa", "base"), "LFA 2-0-0")
    del lt
    # network-wide route delta of one RSW drain (DecisionBenchmark's churn):
    # rebuild the table on the drained topology, diff it on the device
    rsw = next(i for i, n in enumerate(topo.names) if n.startswith("3-"))
    dbs = topo.adj_dbs()
    dbs[rsw].isOverloaded = True
    ls.updateAdjacencyDatabase(dbs[rsw])
    t0 = time.perf_counter()
    drained = E.AllNodesRouteTable(areas, "0", ps, True)
    t1 = time.perf_counter()
    changed = drained.diff(table)
    t2 = time.perf_counter()
    changed = np.asarray(changed, dtype=np.int64)
    upd, dele = drained.delta("2-0-0")
    # the oracle's getRouteDelta of this drain: the golden overload state's
    # delta vs base (unicast part)
    state = f"overload:{topo.names[rsw]}"
    want = gold["sp_ecmp"][state]["delta_vs_base"]["unicast"] if state in gold["sp_ecmp"] else None
    got = {R.key_str(k): R.route_hash(v) for k, v in upd.items()}
    got.update({R.key_str(k): None for k in dele})
    delta_ok = want is not None and got == want
    # algorithmic bytes of spf_route_table_kernel per launch: per (node,
    # prefix) cell the metric + best words written, the link mask written
    # (8 B x link words of the node), the announcer's distance read and its
    # next-hop mask read (SPF_NH_BYTES of the node: the byte-strided rows)
    from openr_amd import abi as _abi

    csr = topo.csr()
    deg = np.diff(csr.row_ptr.astype(np.int64))
    lw = (deg + 63) // 64
    nbr = [len(set(csr.col[csr.row_ptr[u]:csr.row_ptr[u + 1]].tolist())) for u in range(V)]
    nb = np.array([_abi.nh_bytes_for(k) for k in nbr], dtype=np.int64)
    alg = int((P + NL) * (12 * V + 8 * int(lw.sum()) + int(nb.sum())))
    med = lambda x: sorted(x)[len(x) // 2]  # noqa: E731
    k_ms = med(rt)
    # the plain (non-LFA) launches are the smallest of the profiled ones
    rt_traffic, rt_src = pmc_traffic_smallest("spf_route_table_kernel")
    return {
        "what": "unicast + node-label MPLS RouteDb of every node of the fabric at once: "
                "AllNodesRouteTable = all-sources SPF + next hops, then spf_route_table_kernel "
                "(selectEcmpOpenr per node x prefix, getNextHopsWithMetric per node x labelled node)",
        "nodes": V, "prefixes": P, "node_label_columns": NL, "routes": int(routes),
        "build_ms_median": round(med(walls), 2), "spf_ms_median": round(med(spf), 3),
        "route_kernel_ms_median": round(k_ms, 3),
        "route_kernel_roofline": {"bound": "hbm", "algorithmic_bytes": alg,
                                  "achieved": round(alg / (k_ms / 1e3) / 1e9, 1), "peak": HBM_PEAK_GBS,
                                  "unit": "GB/s", "frac": round(alg / (k_ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
                                  "traffic": rt_traffic, "traffic_source": rt_src},
        "materialise_one_node_ms": round(us_mat / 1e3, 3), "materialised_routes": n_mat,
        "parity_check": "ok (oracle goldens: 2-0-0 per route, 2 more nodes by digest)" if not bad
                        else "; ".join(bad),
        "lfa_table": {"what": "same table with loop-free alternates (SPF_RT_LFA, per-link metrics)",
                      "build_ms_min": round(min(lfa_walls), 2),
                      "route_kernel_ms_min": round(min(lfa_rt), 3),
                      "parity_check": "ok (oracle golden)" if not lfa_err else lfa_err},
        "drain_delta": {
            "what": f"RSW {topo.names[rsw]} drained: table rebuilt + spf_route_table_diff_kernel = "
                    "getRouteDelta of every node at once",
            "table_rebuild_ms": round((t1 - t0) * 1e3, 2), "diff_ms": round((t2 - t1) * 1e3, 3),
            "changed_cells": int(changed.sum()), "nodes_with_changes": int((changed > 0).sum()),
            "parity_check": "ok (oracle golden delta)" if delta_ok
                            else f"2-0-0 delta differs from the oracle's ({len(got)} vs "
                                 f"{None if want is None else len(want)} routes)",
        },
    }


def ksp2_route_db(topo, device, iters=2):
    """BASELINE configs[3]: every fabric prefix SR_MPLS / KSP2_ED_ECMP, the
    RouteDb of "2-0-0" after an RSW overload toggle.  Each build traces the
    k=1 edge-disjoint paths to every destination on the host, runs one
    ignore-list SPF per destination (the k=2 second pass, LinkState.cpp:
    760-789) as ONE device batch, traces k=2 and builds the label stacks
    (Decision.cpp:909-1066)."""
    import openr_amd._openr_spf as E
    from openr_amd import thrift as T

    E.set_spf_device(device)

    def timed(solver, areas, ps):
        nu, nm, us, free_us = solver.buildRouteDbTimed("2-0-0", areas, ps)
        return nu + nm, us, free_us

    counters = {}

    def check(ls, solver, areas, ps, dbs):
        counters.update(E.get_counters())  # the timed builds' counters, before the check's
        return _routedb_parity("ksp2", ls, solver, areas, ps, dbs, topo)

    out = _rebuild_loop(E, topo, iters, timed, (T.PrefixForwardingType.SR_MPLS,
                                                T.PrefixForwardingAlgorithm.KSP2_ED_ECMP),
                        after_cold=E.reset_counters, check=check)
    c = counters or E.get_counters()
    n = max(1, c.get("decision.route_build_runs", 1))
    out["per_build"] = {
        "spf_runs": round(c.get("decision.spf_runs", 0) / n, 1),
        **{k.split(".", 1)[1]: round(c.get(k, 0) / n, 1)
           for k in ("decision.route_prefetch_us", "decision.spf_batch_us", "decision.spf_device_us",
                     "decision.route_prefix_pool_us", "decision.route_merge_us",
                     "decision.route_label_us", "decision.route_release_us",
                     "decision.kth_trace_us", "decision.kth_memo_clear_us", "decision.kth2_trace_us",
                     "decision.kth_todo_us", "decision.kth_lists_us", "decision.kth_fill_us",
                     "decision.kth2_base_us", "decision.ksp2_best_us", "decision.ksp2_paths_us",
                     "decision.ksp2_nexthops_us", "decision.ksp2_rest_us",
                     "decision.kth2_device_trace_us", "decision.kth2_device_traces",
                     "decision.kth2_device_overflows",
                     "decision.spf_memo_kept", "decision.spf_memo_dropped")},
    }
    out["what"] = ("adj-db update (RSW overload toggle) + buildRouteDb of 2-0-0, all prefixes "
                   "SR_MPLS/KSP2_ED_ECMP (k=1 + k=2 paths to every node)")
    return out


def ksp2_cpu_sample(topo, sample=12):
    """Reference-style CPU cost per destination of getKthPaths(k=1) +
    (k=2) on the fabric (oracle restatement: k=2 runs an un-memoized runSpf
    per destination, LinkState.cpp:776-777), timed on a sample of
    destinations and extrapolated to all of them."""
    from oracle import build as obuild

    obuild.build()
    from oracle import _oracle_ref as O

    ls = O.LinkState("0")
    for db in topo.adj_dbs():
        ls.updateAdjacencyDatabase(db)
    names = sorted(n for n in topo.names if n != "2-0-0")
    dests = names[:: max(1, len(names) // sample)][:sample]
    ls.getSpfResult("2-0-0", True)  # k=1 reads the memoized SPF of the source
    t0 = time.perf_counter()
    for d in dests:
        ls.getKthPaths("2-0-0", d, 1)
        ls.getKthPaths("2-0-0", d, 2)
    per = (time.perf_counter() - t0) / len(dests)
    return {"ms_per_destination": round(per * 1e3, 2),
            "extrapolated_build_ms": round(per * 1e3 * len(names), 1),
            "cores": 1, "kind": "port",
            "sample": f"{len(dests)} destinations of 2-0-0, oracle/ref_decision.cpp getKthPaths k=1,2; "
                      f"extrapolated x{len(names)} destinations"}


def whatif_batch(world, rank, local, dist, steps=3, cpu_lines=True):
    """BASELINE configs[4]: 8,192 single-link-failure SPFs (runSpf with
    linksToIgnore = {link}, LinkState.cpp:806-880) from the border node
    "2-0-0" of two areas: area A = the 10k fabric, area B = the 10k-node /
    100k-link WAN, 4,096 sampled links each (seed 7), with ECMP next-hop
    masks.  The 8,192 queries are split in contiguous blocks over
    the ranks (strong scaling, no collective)."""
    import numpy as np
    import torch

    from openr_amd import abi
    from openr_amd import allsources as AS
    from openr_amd import topologies as TP

    # the two areas share the border node 2-0-0 (TP.whatif_two_area, the
    # setup of tests/golden/whatif_two_area.*)
    areas = []
    for _, topo, links in TP.whatif_two_area():
        csr = topo.csr()
        r, _ = topo.rank()
        src = int(r[topo.names.index(TP.WHATIF_BORDER)])
        areas.append((csr, src, links.astype(np.uint32)))
    allq = [(a, int(l)) for a, (_, _, links) in enumerate(areas) for l in links]
    first, count = AS.shard(len(allq), world, rank)
    mine = allq[first:first + count]
    streams, graphs, queries = [], [], []
    for a, (csr, src, _) in enumerate(areas):
        ign = [[l] for (aa, l) in mine if aa == a]
        if not ign:
            continue
        g = abi.Graph(csr, device=local)
        st = torch.cuda.Stream(device=local)
        g.set_stream(st.cuda_stream)
        q = g.query(np.full(len(ign), src, dtype=np.uint32), abi.SPF_F_NEXTHOPS, ignore=ign)
        graphs.append((a, g, ign))
        streams.append(st)
        queries.append(q)
    for q in queries:  # warm-up
        q.run(sync=False)
    torch.cuda.synchronize(local)
    times = []
    for _ in range(steps):
        if dist:
            dist.barrier()
        torch.cuda.synchronize(local)
        t0 = time.perf_counter()
        for q in queries:
            q.run(sync=False)  # the two areas overlap on their own streams
        torch.cuda.synchronize(local)
        times.append((time.perf_counter() - t0) * 1e3)
    ms = sorted(times)[len(times) // 2]
    dev_ms = max((q.elapsed_ms() for q in queries), default=0.0)
    t = torch.tensor([ms, dev_ms], dtype=torch.float64, device=f"cuda:{local}")
    if dist:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    ms, dev_ms = float(t[0]), float(t[1])
    # parity spot check (rank 0): 2 queries per area against the literal
    # DijkstraQ replay with the same ignored link
    check = None
    if rank == 0:
        from oracle import spf_py

        bad = 0
        for (a, g, ign), q in zip(graphs, queries):
            csr = areas[a][0]
            for i in (0, len(ign) - 1):
                s = areas[a][1]
                ref = spf_py.run_spf(csr, s, True, frozenset(ign[i]))
                d = q.dist(i)
                got = q.nexthop_sets(i, s)
                for v in range(csr.num_nodes):
                    if v in ref:
                        bad += int(d[v]) != ref[v][0] or (v != s and got[v] != ref[v][1])
                    else:
                        bad += d[v] != np.uint64(abi.SPF_UNREACHABLE)
        check = "ok" if bad == 0 else f"{bad} mismatches"
    kernels = sorted({q.kernel for q in queries})
    launched = sorted(set().union(*(set(q.kernels()) for q in queries)))
    # algorithmic bytes of the batch (both areas): every query's u32
    # distance row and byte-strided mask row written once (SPF_NH_BYTES of
    # the source), plus the baseline SSSP of each area (its CSR read once:
    # row pointers + 8 B per edge, head and metric).  Screened queries copy
    # the baseline rows and repaired ones touch only the edges of their K
    # (DESIGN.md §3), so no per-query CSR term.  Priced against the plan's
    # device time (HIP events around base + screen + repair + narrow)
    alg, screened = 0, 0
    for (a, _, ign), q in zip(graphs, queries):
        csr = areas[a][0]
        V, E = csr.num_nodes, len(csr.col)
        nq = len(ign)
        screened += q.screened() or 0
        B = q.nh_bytes(0)
        alg += nq * (4 * V + V * B) + (4 * (V + 1) + 8 * E)
    gbs = alg / (dev_ms / 1e3) / 1e9 if dev_ms > 0 else 0.0
    wi_traffic = None
    wi_src = None
    wi_note = None
    if world == 1:
        wi_traffic, wi_src, wi_note = pmc_plan_traffic(launched, "pmc_whatif.json")
    for q in queries:
        q.close()
    for _, g, _ in graphs:
        g.close()
    cpu = None
    if rank == 0 and cpu_lines:
        # BASELINE.md §3 line B: oracle/csr_spf.h (int CSR, binary heap,
        # next-hop bitsets) over ALL 8,192 queries on every host core
        from oracle import build as obuild

        obuild.build()
        from oracle import _oracle_ref as O

        cores = host_cores()
        tc = time.perf_counter()
        for a, (csr, src, links) in enumerate(areas):
            n = len(links)
            O.csr_spf_summary(csr.row_ptr, csr.col, csr.metric.astype(np.uint64), csr.link_id,
                              csr.overloaded, np.full(n, src, dtype=np.uint32),
                              np.arange(n + 1, dtype=np.uint32), links.astype(np.uint32), True, True,
                              cores)
        cpu_s = time.perf_counter() - tc
        cpu = {"value": round(len(allq) / cpu_s, 1), "unit": "SPF/s", "cores": cores,
               "kind": "port", "cpu_model": host_cpu_model(),
               "sample": f"ALL {len(allq)} what-if queries (both areas, ECMP next hops), "
                         f"oracle/csr_spf.h on {cores} threads, {cpu_s:.2f} s"}
    return {
        "config": "BASELINE configs[4]: 8,192 single-link-failure SPFs with ECMP next hops from the "
                  "border node 2-0-0 of two areas: A = fabric (9,976 nodes), B = WAN-10k, 4,096 links each",
        "queries": len(allq), "n_gpus": world, "scaling": "strong", "kernels": kernels,
        "ms": round(ms, 3), "device_ms": round(dev_ms, 3),
        "value": round(len(allq) / (ms / 1e3), 1), "unit": "SPF/s",
        "parity_check": check,
        "screened_queries": screened,
        "kernels_launched": launched,
        "roofline": {"bound": "hbm", "kernel": "what-if plan: " + " + ".join(launched),
                     "note": "latency-bound: two dependent chains per area (baseline SSSP, screen, "
                             "then the repair SSSP: one workgroup per query, ~40 us of dependent "
                             "steps each on the fabric; DESIGN.md section 3)",
                     "algorithmic_bytes": int(alg),
                     "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(gbs / HBM_PEAK_GBS, 4), "traffic": wi_traffic,
                     "traffic_source": wi_src,
                     "traffic_over_algorithmic": round(wi_traffic / alg, 3) if wi_traffic and alg else None,
                     **({"traffic_note": wi_note} if wi_note else {})},
        **({"cpu_baseline_optimised_all_cores": cpu} if cpu else {}),
    }


def grid_route_db(device, iters=20):
    """BASELINE configs[0]: DecisionBenchmark's 10x10 grid (DecisionBenchmark.
    cpp:360-431), buildRouteDb("1") with LFA on (the benchmark's Decision,
    :75-83) after an overload toggle of a random node, engine and oracle
    (reference data structures, 1 thread) side by side."""
    import openr_amd._openr_spf as E
    from oracle import build as obuild
    from openr_amd import topologies as TP

    obuild.build()
    from oracle import _oracle_ref as O

    E.set_spf_device(device)
    topo = TP.grid(10)
    out = {"config": "BASELINE configs[0]: 10x10 grid, buildRouteDb(\"1\"), SP_ECMP, LFA on"}
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
        solver.buildRouteDbTimed("1", areas, ps)
        times = []
        routes = 0
        for it in range(iters):
            db = dbs[(it * 37 + 11) % len(dbs)]
            for ov in (True, False):
                db.isOverloaded = ov
                t0 = time.perf_counter()
                ls.updateAdjacencyDatabase(db)
                r = solver.buildRouteDbTimed("1", areas, ps)
                times.append((time.perf_counter() - t0) * 1e3)
                routes = r[0] + r[1]
        out[tag] = {"ms_median": round(sorted(times)[len(times) // 2], 3), "routes": routes,
                    "samples": len(times)}
    return out


def route_db_rebuild_cpu(topo, iters=2):
    """The same loop on the oracle (reference data structures), 1 thread."""
    from oracle import build as obuild

    obuild.build()
    from oracle import _oracle_ref as O

    def timed(solver, areas, ps):
        nu, nm, us = solver.buildRouteDbTimed("2-0-0", areas, ps)[:3]
        return nu + nm, us

    out = _rebuild_loop(O, topo, iters, timed)
    out["cores"] = 1
    out["kind"] = "port"
    return out


def route_db_rebuild_lfa_cpu(topo):
    """The LFA-on rebuild on the oracle (reference data structures), 1
    thread: ONE build after the first RSW overload toggle of the loop (85
    uncached runSpf + the LFA RouteDb, ~15-25 s, so a bounded sample)."""
    from oracle import build as obuild

    obuild.build()
    from oracle import _oracle_ref as O

    areas = O.AreaLinkStates()
    ls = areas.add("0")
    dbs = topo.adj_dbs()
    for db in dbs:
        ls.updateAdjacencyDatabase(db)
    ps = O.PrefixState()
    for pdb in topo.prefix_dbs("0", 0, 0):
        ps.updatePrefixDatabase(pdb)
    solver = O.SpfSolver("2-0-0", False, True)
    rsw = [i for i, n in enumerate(topo.names) if n.startswith("3-")]
    db = dbs[rsw[0]]
    db.isOverloaded = True
    t0 = time.perf_counter()
    ls.updateAdjacencyDatabase(db)
    nu, nm, _ = solver.buildRouteDbTimed("2-0-0", areas, ps)[:3]
    ms = (time.perf_counter() - t0) * 1e3
    db.isOverloaded = False
    return {"ms": round(ms, 1), "routes": nu + nm, "cores": 1, "kind": "port",
            "sample": f"one LFA-on rebuild of 2-0-0 after the {topo.names[rsw[0]]} overload toggle "
                      "(oracle/ref_decision.cpp, reference data structures)"}


def wan_all_sources_table(args, world, rank, local, dist, cluster):
    """BASELINE configs[2] at N > 1 (or --sharded): the 100k-source WAN table
    as ONE engine call -- spf_table over the RCCL cluster: contiguous source
    blocks per GPU (push-only delta-stepping), then the uint32 rows
    all-gathered in place over xGMI inside spf_table_run, so every GPU holds
    the whole 40 GB table.  `ms` = the slowest rank's wall time of the call
    (compute + exchange); parity: the reference's checksum of row n0 and two
    rows (the last one from the last rank's block, read from the gathered
    copy) against scipy."""
    import numpy as np
    import torch

    from openr_amd import abi
    from openr_amd import topologies as TP

    t0 = time.perf_counter()
    topo = TP.wan(args.wan_nodes, args.wan_links)
    csr = topo.csr()
    gen_s = time.perf_counter() - t0
    V, E = csr.num_nodes, len(csr.col)
    g = abi.Graph(csr, device=local)
    g.query(np.arange(min(256, V), dtype=np.uint32), 0).run().close()
    g.close()
    flags = abi.SPF_T_GATHER_ROWS if world > 1 else 0
    tab = abi.Table(cluster, csr, np.arange(V, dtype=np.uint32), flags)
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    tab.run()
    if dist:
        dist.barrier()
    wall_ms = (time.perf_counter() - t1) * 1e3
    comp_ms, gather_ms = tab.elapsed_ms()
    red = torch.tensor([wall_ms, comp_ms, gather_ms], dtype=torch.float64, device=f"cuda:{local}")
    if dist:
        dist.all_reduce(red, op=dist.ReduceOp.MAX)
    wall_ms, comp_ms, gather_ms = (float(x) for x in red)
    check = None
    if rank == 0:
        import scipy.sparse as sp
        import scipy.sparse.csgraph as cg

        anchors = json.load(open(os.path.join(ROOT, "tests", "golden", "wan_anchors.json")))["anchors"]
        want = [a["sum_dist"] for a in anchors if a["V"] == V and a["L"] == args.wan_links and a["S"] == 1]
        bad = 0
        row0 = tab.fetch_rows(0, 1)[0]
        if want and int(row0.astype(np.int64).sum()) != want[0]:
            bad += 1
        A = sp.csr_matrix((csr.metric.astype(np.float64), csr.col, csr.row_ptr), shape=(V, V))
        probe = [0, V - 1]
        D = cg.dijkstra(A, indices=probe)
        for k, i in enumerate(probe):
            ref = np.where(np.isfinite(D[k]), D[k], 0xFFFFFFFF).astype(np.int64)
            bad += int((tab.fetch_rows(i, 1)[0].astype(np.int64) != ref).sum())
        check = "ok" if bad == 0 else f"{bad} mismatches"
    kernel = tab.kernel(0)
    tab.close()
    per_sssp, kdesc = wan_sssp_bytes(kernel, V, E)
    out = {
        "config": "BASELINE configs[2]: 100k-node / 1M-link WAN (SURVEY §8(d) row 3), all sources, "
                  f"one engine call over {world} GPU(s): contiguous source blocks + in-engine RCCL "
                  "all-gather of the uint32 rows",
        "nodes": V, "links": int(csr.num_links), "directed_edges": E, "sources": V,
        "n_gpus": world, "kernel": kernel, "scaling": "strong",
        "ms": round(wall_ms, 2), "device_compute_ms": round(comp_ms, 2),
        "gather_ms": round(gather_ms, 2),
        "value": round(V / (wall_ms / 1e3), 1), "unit": "SPF/s",
        "value_no_gather": round(V / ((wall_ms - gather_ms) / 1e3), 1),
        "gteps": round(V * E / (wall_ms / 1e3) / 1e9, 2),
        "table_bytes": V * V * 4,
        "gather_algbw_gbs": round(V * V * 4 / (gather_ms / 1e3) / 1e9, 1) if world > 1 and gather_ms else None,
        "roofline": {"bound": "hbm", "kernel": kdesc,
                     "algorithmic_bytes_per_sssp": per_sssp,
                     "achieved": round(V * per_sssp / (comp_ms / 1e3) / 1e9 / world, 1),
                     "frac": round(V * per_sssp / (comp_ms / 1e3) / 1e9 / world / HBM_PEAK_GBS, 4),
                     "peak": HBM_PEAK_GBS, "unit": "GB/s", "note": "per GPU"},
        "parity_check": check,
        "generate_s": round(gen_s, 1),
    }
    if not args.no_repair:
        from openr_amd import allsources as AS

        sas = AS.ShardedAllSources(csr, device=local, gather=world > 1)
        sas.run()
        out["table_repair"] = wan_table_repair(topo, csr, sas, world, rank, local, dist)
        sas.close()
    return out


def wan_all_sources(args, world, rank, local, dist):
    """BASELINE configs[2]: all-sources SPF on the 100k-node / 1M-link WAN
    (SURVEY §8(d) row 3 generator), sources sharded in contiguous blocks over
    the ranks, uint32 distance rows all-gathered in place over RCCL (xGMI)
    when N > 1.  One timed pass (a pass is ~4 s of device time on one GPU);
    the kernel is warmed on a 256-source batch first."""
    import numpy as np
    import torch

    from openr_amd import abi
    from openr_amd import allsources as AS
    from openr_amd import topologies as TP

    t0 = time.perf_counter()
    topo = TP.wan(args.wan_nodes, args.wan_links)
    csr = topo.csr()
    gen_s = time.perf_counter() - t0
    V, E = csr.num_nodes, len(csr.col)
    g = abi.Graph(csr, device=local)
    g.query(np.arange(min(256, V), dtype=np.uint32), 0).run().close()
    g.close()
    sas = AS.ShardedAllSources(csr, device=local, gather=world > 1)
    r = sas.run()
    t = torch.tensor([r.wall_ms, r.spf_ms, r.gather_ms, r.fetch_ms, r.extra["compute_wall_ms"]],
                     dtype=torch.float64, device=f"cuda:{local}")
    if dist:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    wall_ms, spf_ms, gather_ms, fetch_ms, compute_ms = (float(x) for x in t)
    n = sas.n
    # parity on rank 0: the row of source "n0" (id 0) reproduces the
    # reference runSpf checksum (tests/golden/wan_anchors.json)
    # and two sampled rows equal an independent CPU Dijkstra (scipy)
    check = None
    cpu = None
    if rank == 0:
        import scipy.sparse as sp
        import scipy.sparse.csgraph as cg

        anchors = json.load(open(os.path.join(ROOT, "tests", "golden", "wan_anchors.json")))["anchors"]
        want = [a["sum_dist"] for a in anchors if a["V"] == V and a["L"] == args.wan_links and a["S"] == 1]
        A = sp.csr_matrix((csr.metric.astype(np.float64), csr.col, csr.row_ptr), shape=(V, V))
        probe = [0, n - 1]
        bad = 0
        row0 = sas.row(0)
        if want and int(row0.astype(np.int64).sum()) != want[0]:
            bad += 1
        D = cg.dijkstra(A, indices=probe)
        for k, i in enumerate(probe):
            ref = np.where(np.isfinite(D[k]), D[k], 0xFFFFFFFF).astype(np.int64)
            bad += int((sas.row(i).astype(np.int64) != ref).sum())
        check = "ok" if bad == 0 else f"{bad} mismatches"
        # optimised CPU line: scipy's C Dijkstra (binary heap over CSR), 1 thread
        S = 16
        ts = time.perf_counter()
        cg.dijkstra(A, indices=list(range(0, V, V // S))[:S])
        cpu_s = (time.perf_counter() - ts) / S
        cpu = {"value": round(1.0 / cpu_s, 2), "unit": "SPF/s", "cores": 1, "kind": "optimised-cpu",
               "sample": f"{S} sources, scipy.sparse.csgraph.dijkstra (C binary-heap Dijkstra over the "
                         "same CSR), single thread; the reference's own runSpf needs ~587 s/SPF here "
                         "(SURVEY §6, reMake per strict improvement)"}
        if not args.no_cpu_baseline:
            # BASELINE.md §3 line B on every host core: oracle/csr_spf.h
            # distances over a fixed source sample, extrapolated to all sources
            from oracle import build as obuild

            obuild.build()
            from oracle import _oracle_ref as O

            cores = host_cores()
            Sa = 48 * cores
            smp = np.arange(0, V, max(1, V // Sa), dtype=np.uint32)[:Sa]
            tc = time.perf_counter()
            Sm = O.csr_spf_summary(csr.row_ptr, csr.col, csr.metric.astype(np.uint64), csr.link_id,
                                   csr.overloaded, smp, None, None, True, False, cores)
            all_s = time.perf_counter() - tc
            cpu["optimised_all_cores"] = {
                "anchor_check": (None if not (want and int(smp[0]) == 0)
                                 else "ok" if int(Sm[0, 1]) == want[0] else "mismatch"),
                "value": round(len(smp) / all_s, 1), "unit": "SPF/s", "cores": cores, "kind": "port",
                "cpu_model": host_cpu_model(),
                "all_sources_s_extrapolated": round(all_s / len(smp) * V, 1),
                "sample": f"{len(smp)} sources (every {V // len(smp)}th), oracle/csr_spf.h distances "
                          f"(int CSR, binary heap) on {cores} threads, {all_s:.2f} s; extrapolated "
                          f"x{V / len(smp):.0f} to all sources"}
    repair = None if args.no_repair else wan_table_repair(topo, csr, sas, world, rank, local, dist)
    sas.close()
    table_bytes = n * V * 4
    # algorithmic bytes per SSSP of the push-only delta-stepping plan: the
    # CSR row of every settled node read once (col + metric u32, row_ptr),
    # the distance row written once (SURVEY §8(d) per-SSSP figure without
    # the next-hop masks this distance-only pass does not produce)
    per_sssp, kdesc = wan_sssp_bytes(r.kernel, V, E)
    kernel_s = spf_ms / 1e3
    achieved = sas.count * per_sssp / kernel_s / 1e9 if kernel_s else None
    traffic, traffic_src = pmc_traffic_largest(kdesc.split()[0])
    out = {
        "config": "BASELINE configs[2]: 100k-node / 1M-link WAN (SURVEY §8(d) row 3), all sources, "
                  "contiguous source blocks per GPU, RCCL all-gather of uint32 rows",
        "nodes": V, "links": int(csr.num_links), "directed_edges": E, "sources": n,
        "n_gpus": world, "kernel": r.kernel,
        "ms": round(wall_ms, 2), "spf_ms": round(spf_ms, 2), "fetch_ms": round(fetch_ms, 2),
        "gather_ms": round(gather_ms, 2), "compute_wall_ms": round(compute_ms, 2),
        "value": round(n / (wall_ms / 1e3), 1), "unit": "SPF/s",
        "value_no_gather": round(n / (compute_ms / 1e3), 1),
        "gteps": round(n * E / (wall_ms / 1e3) / 1e9, 2),
        "table_bytes": table_bytes,
        "gather_algbw_gbs": round(table_bytes / (gather_ms / 1e3) / 1e9, 1) if world > 1 and gather_ms else None,
        "roofline": {"bound": "hbm", "kernel": kdesc,
                     # SURVEY §8(d) per-SSSP figure without masks: CSR of every settled
                     # node read once (in the format the kernel reads) + the distance
                     # row written once
                     # same keys as the headline: achieved / frac = ALGORITHMIC bytes
                     # per live kernel time; traffic_* = PMC bytes (2*FETCH_SIZE +
                     # WRITE_SIZE of the one-GPU 100k-source launch)
                     "algorithmic_bytes_per_sssp": per_sssp,
                     "achieved": round(achieved, 1) if achieved else None,
                     "frac": round(achieved / HBM_PEAK_GBS, 4) if achieved else None,
                     "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "traffic_per_sssp": (traffic // 100000) if traffic else None,
                     "traffic_achieved": round(traffic / 100000 * sas.count / kernel_s / 1e9, 1)
                     if traffic and kernel_s else None,
                     "traffic_frac": round(traffic / 100000 * sas.count / kernel_s / 1e9 / HBM_PEAK_GBS, 4)
                     if traffic and kernel_s else None,
                     "traffic_over_algorithmic": round(traffic / 100000 / per_sssp, 3)
                     if traffic and per_sssp else None,
                     "traffic_source": traffic_src},
        "parity_check": check,
        "generate_s": round(gen_s, 1),
    }
    if cpu:
        out["cpu_baseline"] = cpu
    if repair:
        out["table_repair"] = repair
    return out


def wan_table_repair(topo, csr, sas, world, rank, local, dist):
    """SURVEY §8(f) row 2 on the WAN all-sources table: single churn events
    (link down / up, metric up / down, node drain / undrain) applied with
    ShardedAllSources.update() — edge diff, screen kernel, recompute of the
    affected sources only, row scatter + exchange — instead of the
    reference's drop-everything memo (LinkState.cpp:712-715) and a full
    100k-source recompute.  Parity: the repaired table equals fresh engine
    rows for sampled sources and scipy for one, on the final graph."""
    import random

    import numpy as np
    import torch

    from openr_amd import abi
    from openr_amd import topologies as TP

    rng = random.Random(2024)
    links = list(topo.links)
    ids, _ = topo.rank()
    V = csr.num_nodes
    ov = np.zeros(V, dtype=np.uint8)
    events = []
    gone = None
    cur = csr
    plan = ["link_down", "link_up", "metric_up", "metric_down", "drain", "undrain"]
    drained = None
    for kind in plan:
        if kind == "link_down":
            i = rng.randrange(len(links))
            gone = (i, links.pop(i))
        elif kind == "link_up":
            links.insert(*gone)
        elif kind in ("metric_up", "metric_down"):
            i = rng.randrange(len(links))
            a, b, wab, wba = links[i]
            w = wab * 3 if kind == "metric_up" else max(1, wab // 3)
            links[i] = (a, b, w, w)
        elif kind == "drain":
            drained = int(ids[rng.randrange(V)])
            ov[drained] = 1
        elif kind == "undrain":
            ov[drained] = 0
        if kind in ("link_down", "link_up"):
            nxt = TP.Topology(topo.names, links, None).csr()
            nxt.overloaded = ov.copy()
        else:
            nxt = abi.Csr(cur.num_nodes, cur.row_ptr, cur.col, cur.metric.copy(), cur.link_id,
                          cur.rev, ov.copy(), cur.num_links)
            if kind.startswith("metric"):
                a, b, w, _ = links[i]
                ra, rb = int(ids[a]), int(ids[b])
                for (u, v) in ((ra, rb), (rb, ra)):
                    lo, hi = int(cur.row_ptr[u]), int(cur.row_ptr[u + 1])
                    e = lo + int(np.nonzero(cur.col[lo:hi] == v)[0][0])
                    nxt.metric[e] = w
        rep = sas.update(nxt)
        t = torch.tensor([rep.wall_ms, rep.spf_ms, rep.screen_ms, rep.graph_ms, rep.exchange_ms],
                         dtype=torch.float64, device=f"cuda:{local}")
        if dist:
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
        events.append({"event": kind, "deltas": rep.deltas, "affected_sources": rep.affected_total,
                       "ms": round(float(t[0]), 2), "spf_ms": round(float(t[1]), 2),
                       "screen_ms": round(float(t[2]), 2), "graph_ms": round(float(t[3]), 2),
                       "exchange_ms": round(float(t[4]), 2), "diff_ms": round(rep.diff_ms, 2),
                       "graph_patched_in_place": rep.graph_patched,
                       "result_release_ms": round(rep.extra.get("release_ms", 0.0), 2),
                       "rows": "repaired in place (spf_table_repair)" if rep.relaxed else "recomputed"})
        cur = nxt
    check = None
    if rank == 0 and sas.gather or world == 1:
        import scipy.sparse as sp
        import scipy.sparse.csgraph as cg

        probe = [0, V // 3, V - 1]
        g = abi.Graph(cur, device=local)
        q = g.query(np.asarray(probe, dtype=np.uint32), 0).run()
        bad = 0
        for k, i in enumerate(probe):
            ref = q.dist(k)
            ref = np.where(ref == np.uint64(abi.SPF_UNREACHABLE), np.uint64(0xFFFFFFFF), ref)
            bad += int((sas.row(i).astype(np.uint64) != ref).sum())
        q.close()
        g.close()
        A = sp.csr_matrix((cur.metric.astype(np.float64), cur.col, cur.row_ptr), shape=(V, V))
        D = cg.dijkstra(A, indices=[probe[1]])[0]
        ref = np.where(np.isfinite(D), D, 0xFFFFFFFF).astype(np.int64)
        bad += int((sas.row(probe[1]).astype(np.int64) != ref).sum())
        check = "ok" if bad == 0 else f"{bad} mismatches"
    return {"what": "WAN all-sources uint32 table kept current under single churn events by "
                    "ShardedAllSources.update (diff -> spf_table_screen_kernel -> SSSP of the affected "
                    "sources -> spf_scatter_rows_kernel -> row exchange); compare the full pass 'ms'",
            "events": events, "parity_check": check}


def wide_plan(device=0):
    """The wide plan (spf_wide_kernel) on the two shapes that used to send a
    whole area to the one-thread-per-query literal replay:
    the fabric with ONE metric-0 link (all 9,976 sources + next hops; the
    literal replay timed on 64 sources beside it) and the 100k WAN with
    metrics up to 10^6 (maxw * (V-1) >= 2^32; 2,048 distance rows).  Parity:
    2 fabric rows against the DijkstraQ replay, 2 WAN rows against scipy."""
    import numpy as np
    import scipy.sparse as sp
    import scipy.sparse.csgraph as cg

    from openr_amd import abi
    from openr_amd import topologies as TP
    from oracle import spf_py

    def timed(g, srcs, flags, reps=2):
        q = g.query(srcs, flags)
        best = None
        for _ in range(reps):
            q.run()
            ms = q.elapsed_ms()
            best = ms if best is None else min(best, ms)
        return q, best

    out = {}
    topo = TP.fabric(10000)
    k = len(topo.links) // 2
    a, b, _, _ = topo.links[k]
    topo.links[k] = (a, b, 0, 0)
    csr = topo.csr()
    g = abi.Graph(csr, device=device)
    V = csr.num_nodes
    srcs = np.arange(V, dtype=np.uint32)
    q, ms = timed(g, srcs, abi.SPF_F_NEXTHOPS)
    bad = 0
    for i in (0, V // 2):
        ref = spf_py.run_spf(csr, int(srcs[i]), True)
        d = q.dist(i)
        sets = q.nexthop_sets(i, int(srcs[i]))
        bad += sum(int(d[v]) != m or (v != srcs[i] and sets[v] != nhs)
                   for v, (m, nhs, _, _) in ref.items())
    os.environ["OPENR_SPF_LITERAL"] = "1"
    try:
        ql, ms_l = timed(g, srcs[:64], abi.SPF_F_NEXTHOPS, reps=1)
    finally:
        del os.environ["OPENR_SPF_LITERAL"]
    out["fabric_one_metric0_link"] = {
        "sources": V, "kernel": q.kernel, "ms": round(ms, 2), "value": round(V / (ms / 1e3), 1),
        "unit": "SPF/s", "literal_replay_ms_64_sources": round(ms_l, 2),
        "parity_check": "ok" if bad == 0 else f"{bad} mismatches"}
    q.close()
    ql.close()
    g.close()
    topo = TP.wan(100000, 1000000, wmax=1_000_000)
    csr = topo.csr()
    g = abi.Graph(csr, device=device)
    V = csr.num_nodes
    S = 2048
    srcs = np.arange(0, V, V // S, dtype=np.uint32)[:S]
    q, ms = timed(g, srcs, 0)
    A = sp.csr_matrix((csr.metric.astype(np.float64), csr.col, csr.row_ptr), shape=(V, V))
    D = cg.dijkstra(A, indices=[int(srcs[0]), int(srcs[-1])])
    bad = 0
    for kk, i in enumerate((0, S - 1)):
        ref = np.where(np.isfinite(D[kk]), D[kk], -1).astype(np.int64)
        got = q.dist(i).astype(np.int64)
        got[q.dist(i) == abi.SPF_UNREACHABLE] = -1
        bad += int((ref != got).sum())
    out["wan100k_metrics_to_1e6"] = {
        "sources": S, "kernel": q.kernel, "ms": round(ms, 2), "value": round(S / (ms / 1e3), 1),
        "unit": "SPF/s", "all_sources_s_est": round(ms / S * V / 1e3, 2),
        "parity_check": "ok" if bad == 0 else f"{bad} mismatches"}
    q.close()
    g.close()
    return out


def cluster_for(world, rank, local, dist):
    """The engine's RCCL communicator for this rank (include/openr_spf.h
    spf_cluster_create_rank): rank 0 makes the id, torch.distributed hands
    it to the other ranks (plumbing only; the exchange itself runs inside
    the engine's spf_table_run)."""
    import torch

    from openr_amd import abi

    if world == 1:
        return abi.Cluster(world=1, rank=0, uid=abi.cluster_unique_id(), device=local)
    t = torch.zeros(abi.SPF_CLUSTER_ID_BYTES, dtype=torch.uint8, device=f"cuda:{local}")
    if rank == 0:
        t.copy_(torch.frombuffer(bytearray(abi.cluster_unique_id()), dtype=torch.uint8))
    dist.broadcast(t, 0)
    uid = bytes(t.cpu().numpy().tobytes())
    return abi.Cluster(world=world, rank=rank, uid=uid, device=local)


def _timed_table(t, steps, warmup, dist):
    import torch

    for _ in range(warmup):
        t.run()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        t.run(sync=False)
    t.sync()
    if dist:
        dist.barrier()
    return (time.perf_counter() - t0) * 1000.0 / steps, t.elapsed_ms()


def fabric_sharded(args, topo, world, rank, local, dist, cluster):
    """N > 1 headline: STRONG scaling of the one 9,976-source fabric table.
    The engine splits the sources into contiguous blocks, one per GPU
    (spf_table over a one-process-per-GPU RCCL cluster); each block's rows and
    next-hop masks stay resident on the GPU that computed them (a RouteDb
    reads only its own row).  `value` = 9,976 SPFs / the slowest rank's step.
    The same table with the distance rows all-gathered over xGMI inside the
    engine (ncclAllGather in spf_table_run) is timed beside it."""
    import numpy as np
    import torch

    from openr_amd import abi

    csr = topo.csr()
    V, E = csr.num_nodes, len(csr.col)
    sources = np.arange(V, dtype=np.uint32)
    t = abi.Table(cluster, csr, sources, abi.SPF_F_NEXTHOPS)
    step_ms, (comp_ms, _) = _timed_table(t, args.steps, args.warmup, dist)
    tg = abi.Table(cluster, csr, sources, abi.SPF_F_NEXTHOPS | abi.SPF_T_GATHER_ROWS)
    gstep_ms, (gcomp_ms, gather_ms) = _timed_table(tg, max(3, args.steps // 2), 1, dist)
    red = torch.tensor([step_ms, comp_ms, gstep_ms, gather_ms], dtype=torch.float64,
                       device=f"cuda:{local}")
    if dist:
        dist.all_reduce(red, op=dist.ReduceOp.MAX)
    step_ms, comp_ms, gstep_ms, gather_ms = (float(x) for x in red)
    first, count = t.block(cluster.first_rank)
    # parity (rank 0): rows + next hops of its own block, and rows of the LAST
    # rank's block read from the gathered copy, against the DijkstraQ replay
    check = None
    if rank == 0:
        from oracle import spf_py

        bad = 0
        picks = [first, first + count // 2, first + count - 1]
        rows = {i: t.fetch_rows(i, 1)[0] for i in picks}
        lf, lc = tg.block(world - 1)
        for i in (lf, lf + lc - 1):
            rows[i] = tg.fetch_rows(i, 1)[0]
        g = abi.Graph(csr, device=local)
        for i, d in rows.items():
            ref = spf_py.run_spf(csr, int(sources[i]), True)
            for v in range(V):
                want = ref[v][0] if v in ref else 0xFFFFFFFF
                bad += int(d[v]) != want
            if first <= i < first + count:
                m = t.fetch_nexthops(i, 1).reshape(V, t.nh_words(i))
                nb = g.nbrs(int(sources[i]))
                for v in ref:
                    if v == sources[i]:
                        continue
                    got = {int(nb[w * 64 + b]) for w in range(m.shape[1]) for b in range(64)
                           if (int(m[v, w]) >> b) & 1}
                    bad += got != set(ref[v][1])
        g.close()
        check = "ok" if bad == 0 else f"{bad} mismatches"
    kernel = t.kernel(0)
    t.close()
    tg.close()
    return {
        "metric": "all-sources SPF/sec + GTEPS on 10k-node fabric; full RouteDb rebuild ms",
        "value": round(V / (step_ms / 1000.0), 1),
        "unit": "SPF/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(step_ms, 4),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic fabric (DecisionBenchmark createFabric, SSW bug fixed), metric 1",
        "config": {
            "workload": "fabric_full all-sources SPF + ECMP next-hop sets (BASELINE configs[1]), "
                        "one table sharded over the GPUs",
            "nodes": V, "links": int(csr.num_links), "directed_edges": E,
            "sources_total": V, "kernel": kernel,
            "parallelism": f"contiguous source blocks over {world} GPUs inside the engine "
                           "(spf_table, RCCL cluster); rows stay on their owner GPU",
        },
        "derived": {"gteps_equivalent": {
            "value": round(V * E / (step_ms / 1000.0) / 1e9, 2),
            "note": "per-source-equivalent (sources x directed edges / step), not a measured rate"}},
        "device_compute_ms": round(comp_ms, 4),
        "with_row_gather": {
            "what": "the same table with every GPU's uint32 distance rows all-gathered over xGMI "
                    "(in-place ncclAllGather inside spf_table_run)",
            "ms_per_step": round(gstep_ms, 4), "gather_ms": round(gather_ms, 4),
            "value": round(V / (gstep_ms / 1000.0), 1),
            "gathered_bytes": int(V * V * 4),
        },
        "parity_spot_check": check,
        "communicator": {"world": int(cluster.world), "first_rank": int(cluster.first_rank),
                         "local_devices": int(cluster.local_devices)},
    }


def fabric_single(args, topo, world, rank, local, dist):
    """N = 1 headline: the fabric all-sources step as one query on one GPU,
    with the per-kernel split and roofline."""
    import numpy as np
    import torch

    from openr_amd import abi

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
    nh_bytes = [q.nh_bytes(i) for i in range(len(sources))]
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
    # per-kernel device time of the timed launches (engine-side HIP events on
    # the same stream, recorded around each kernel)
    hist = q.stage_history(args.steps)
    d_ms = sum(h[0] for h in hist) / max(1, len(hist))
    n_ms = sum(h[1] for h in hist) / max(1, len(hist))
    step_ms = wall * 1000.0 / args.steps
    if dist:
        t = torch.tensor([step_ms, kernel_ms], device="cuda", dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        step_ms, kernel_ms = float(t[0]), float(t[1])

    nsrc = len(sources)
    E = len(csr.col)
    value = world * nsrc / (step_ms / 1000.0)
    kname = q.kernel
    dist_k, nh_k = KERNELS.get(kname, (kname, None))
    # the kernels the run actually launched (spf_query_kernels): the MS-BFS
    # plan's next-hop stage is the v2 pass unless OPENR_NL_V2=0 / a plan
    # outside it selects the held kernel
    launched = q.kernels()
    if nh_k == "spf_nh_levels_held_kernel" and "spf_nh_levels_v2_kernel" in launched:
        nh_k = "spf_nh_levels_v2_kernel"
    nbrs = distinct_nbrs(csr)
    # BFS levels per 64-source batch, from the distance rows (unit metric)
    levels = []
    if kname.startswith("msbfs"):
        ecc = np.zeros(nsrc, dtype=np.int64)
        for i in range(0, nsrc, 97):  # sampled eccentricities (fabric: 4-6)
            d = q.dist(i)
            ecc[i] = int(d[d != np.uint64(abi.SPF_UNREACHABLE)].max())
        lv = int(ecc.max()) + 2  # +1 level discovering nothing, +1 source level
        levels = [lv] * ((nsrc + 63) // 64)
    stages = {}
    lo = kname == "msbfs+levels" and lvl_only()
    if nh_k:
        b = nh_levels_bytes(csr, nbrs, nh_bytes, dist_rows=lo) if "levels" in kname else None
        stages[nh_k] = {"avg_ms": round(n_ms, 4), "algorithmic_bytes": b}
    stages[dist_k] = {
        "avg_ms": round(d_ms, 4),
        "algorithmic_bytes": msbfs_bytes(csr, nsrc, levels, dist_rows=not lo) if levels else None,
    }
    if levels:
        # the bit-shared pull scans: one CSR scan per batch and level serves
        # 64 sources, served from L2 (not HBM traffic)
        sb = msbfs_scan_bytes(csr, levels)
        stages[dist_k]["csr_scan_bytes_l2"] = sb
        stages[dist_k]["csr_scan_gbs_l2"] = round(sb / (d_ms / 1e3) / 1e9, 1) if d_ms else None
    dom = max(stages, key=lambda k: stages[k]["avg_ms"])
    dom_bytes = stages[dom]["algorithmic_bytes"]
    dom_ms = stages[dom]["avg_ms"]
    achieved = dom_bytes / (dom_ms / 1e3) / 1e9 if dom_bytes and dom_ms else None
    for k, s in stages.items():
        if s["algorithmic_bytes"] and s["avg_ms"]:
            s["achieved_gbs"] = round(s["algorithmic_bytes"] / (s["avg_ms"] / 1e3) / 1e9, 1)
    traffic, traffic_src = pmc_traffic(dom)
    # compulsory bytes of the step (SURVEY §8(d) restated for
    # the bit-parallel plan): every output written once -- u32 distance row,
    # u8 level row, next-hop mask row per source -- and the CSR read once
    floor_bytes = int(nsrc * 5 * csr.num_nodes + csr.num_nodes * int(np.sum(nh_bytes))
                      + 4 * E + 4 * (csr.num_nodes + 1))

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
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic fabric (DecisionBenchmark createFabric, SSW bug fixed), metric 1",
        "config": {
            "workload": "fabric_full all-sources SPF + ECMP next-hop sets (BASELINE configs[1])",
            "nodes": csr.num_nodes,
            "links": int(csr.num_links),
            "directed_edges": E,
            "sources_per_gpu": nsrc,
            "kernel": kname,
            "parallelism": "one table of every source on one GPU (N > 1 runs fabric_sharded)",
        },
        "derived": {"gteps_equivalent": {
            "value": round(world * nsrc * E / (step_ms / 1000.0) / 1e9, 2),
            "note": "per-source-equivalent, not a measured rate: sources x directed edges per step "
                    "time (a textbook SSSP traverses every edge once); the bit-parallel BFS scans an "
                    "edge once per level for 64 sources, so this counts shared scans, not traffic"}},
        "kernel_ms": round(kernel_ms, 4),
        "kernels": stages,
        "kernels_launched": launched,
        "parity_spot_check": check,
        "roofline": _roofline(dom, dom_ms, dom_bytes, traffic, traffic_src),
        "step_output_floor": {
            "what": "compulsory HBM bytes of one step (u32 + u8 rows and next-hop masks written once, "
                    "CSR read once) over the measured step time",
            "bytes": floor_bytes,
            "achieved": round(floor_bytes / (step_ms / 1e3) / 1e9, 1),
            "frac": round(floor_bytes / (step_ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
        },
    }
    q.close()
    g.close()
    return out


class RankLaunchError(RuntimeError):
    """--gpus N cannot run as N ranks here (too few devices, or an outer
    launcher with a different world size)."""


def visible_devices() -> int:
    """GPUs this process can see.  torch.cuda.device_count() does not
    initialise the GPU on this image (it asks amdsmi), so the launching
    parent stays GPU-free before it starts its rank processes."""
    import torch

    return int(torch.cuda.device_count())


def check_world(gpus, env=None, devices=None) -> int:
    """The world size this run must have, or RankLaunchError.  Under an outer
    torch.distributed.run (WORLD_SIZE set) --gpus must agree with it; either
    way at least N devices must be visible (one process per GPU, one node)."""
    env = os.environ if env is None else env
    outer = env.get("WORLD_SIZE")
    n = gpus if gpus is not None else int(outer or 1)
    if n < 1:
        raise RankLaunchError(f"--gpus {n}: need at least one GPU")
    if outer is not None and int(outer) != n:
        raise RankLaunchError(f"--gpus {n} but the launcher started WORLD_SIZE={outer} ranks")
    have = visible_devices() if devices is None else devices
    if have < n:
        raise RankLaunchError(f"--gpus {n} needs {n} visible GPUs on this node, found {have}")
    return n


def _free_port() -> int:
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n: int, argv, script=None) -> int:
    """--gpus N with no outer launcher: start the N rank processes (one per
    GPU: RANK = LOCAL_RANK = r, WORLD_SIZE = N, rendezvous on 127.0.0.1) as
    children of this GPU-free parent, wait for all of them, and pass rank 0's
    one JSON line through.  A rank that fails ends the others (their exact
    PIDs), so no rank waits forever at a barrier; the exit code is non-zero
    if any rank failed or the line does not report n_gpus == N."""
    import subprocess

    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                   HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
        procs.append(subprocess.Popen([sys.executable, script or os.path.abspath(__file__)] + list(argv),
                                      env=env, stdout=subprocess.PIPE if r == 0 else sys.stderr))
    rcs = [None] * n
    failed = False
    while any(rc is None for rc in rcs):
        for r, p in enumerate(procs):
            if rcs[r] is None:
                rcs[r] = p.poll()
                if rcs[r] not in (None, 0) and not failed:
                    failed = True
                    print(f"bench.py: rank {r} exited with {rcs[r]}; stopping the other ranks",
                          file=sys.stderr)
                    for q in procs:
                        if q.poll() is None:
                            q.terminate()
        time.sleep(0.2)
    line = procs[0].stdout.read().decode().strip()
    if any(rcs):
        print(f"bench.py: rank exit codes {rcs}", file=sys.stderr)
        return max(abs(rc) for rc in rcs if rc) or 1
    try:
        rec = json.loads(line.splitlines()[-1])
    except (ValueError, IndexError):
        print(f"bench.py: rank 0 printed no JSON line ({line[-200:]!r})", file=sys.stderr)
        return 1
    if rec.get("n_gpus") != n:
        print(f"bench.py: rank 0 reported n_gpus={rec.get('n_gpus')} for --gpus {n}", file=sys.stderr)
        return 1
    sys.stdout.write(json.dumps(rec) + "\n")
    sys.stdout.flush()
    return 0


def main():
    args = parse()
    try:
        world_want = check_world(args.gpus)
    except RankLaunchError as e:
        print(f"bench.py: {e}", file=sys.stderr)
        sys.exit(3)
    if world_want > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(world_want, sys.argv[1:]))
    # everything but the final JSON line goes to stderr: RCCL's init banner
    # ("RCCL version : ...") and any library chatter write to fd 1 directly,
    # and the contract is ONE JSON line on rank 0's stdout
    json_fd = os.dup(1)
    sys.stdout.flush()
    os.dup2(2, 1)
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
    from openr_amd import abi
    from openr_amd import topologies as TP

    topo = TP.fabric(args.num_sws)
    if world > 1 or args.sharded:
        cluster = cluster_for(world, rank, local, dist)
        out = fabric_sharded(args, topo, world, rank, local, dist, cluster)
    else:
        cluster = None
        out = fabric_single(args, topo, world, rank, local, dist)
        # the N > 1 code path at N = 1 (spf_table over a one-rank RCCL
        # cluster), so the 1 -> N curve has a same-code N = 1 point beside
        # the headline query
        try:
            c1 = cluster_for(1, 0, local, None)
            tl = fabric_sharded(args, topo, 1, 0, local, None, c1)
            c1.close()
            out["table_path"] = {k: tl[k] for k in ("value", "unit", "ms_per_step", "device_compute_ms",
                                                    "with_row_gather", "parity_spot_check",
                                                    "communicator")}
            out["table_path"]["what"] = ("the headline workload through spf_table over a one-rank "
                                         "RCCL cluster: the code path of every N > 1 line")
        except Exception as e:  # reported, never silently replaced
            out["table_path"] = {"error": repr(e)}
    if not args.no_wan:
        try:
            if cluster is not None:
                out["wan_all_sources"] = wan_all_sources_table(args, world, rank, local, dist, cluster)
            else:
                out["wan_all_sources"] = wan_all_sources(args, world, rank, local, dist)
        except Exception as e:  # reported, never silently replaced
            out["wan_all_sources"] = {"error": repr(e)}
    if not args.no_whatif:
        try:
            out["whatif_batch"] = whatif_batch(world, rank, local, dist,
                                               cpu_lines=not args.no_cpu_baseline)
        except Exception as e:
            out["whatif_batch"] = {"error": repr(e)}
    if rank == 0 and world == 1 and not args.no_route_db:
        try:
            out["grid_route_db"] = grid_route_db(local)
        except Exception as e:
            out["grid_route_db"] = {"error": repr(e)}
        try:
            out["ksp2_route_db"] = ksp2_route_db(topo, local)
        except Exception as e:
            out["ksp2_route_db"] = {"error": repr(e)}
        try:
            out["route_db_rebuild_lfa"] = route_db_rebuild_ms(topo, local, lfa=True)
        except Exception as e:  # reported, never silently replaced
            out["route_db_rebuild_lfa"] = {"error": repr(e)}
        try:
            out["route_db_rebuild"] = route_db_rebuild_ms(topo, local)
        except Exception as e:  # reported, never silently replaced
            out["route_db_rebuild"] = {"error": repr(e)}
        try:
            out["route_db_link_flap"] = route_db_link_flap(topo, local)
        except Exception as e:
            out["route_db_link_flap"] = {"error": repr(e)}
        try:
            out["all_nodes_route_table"] = all_nodes_route_table(topo, local)
        except Exception as e:
            out["all_nodes_route_table"] = {"error": repr(e)}
        try:
            out["publication_ingest"] = publication_ingest(topo)
        except Exception as e:
            out["publication_ingest"] = {"error": repr(e)}
        try:
            out["wide_plan"] = wide_plan(local)
        except Exception as e:
            out["wide_plan"] = {"error": repr(e)}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        one = cpu_baseline(topo, args.cpu_sample)
        t_per = 1.0 / one["value"] if one.get("value") else None
        try:
            allc = cpu_baseline_all_cores(topo, args.num_sws, t_per_spf=t_per, full=args.cpu_full)
            out["cpu_baseline"] = dict(allc["reference_style"])
            out["cpu_baseline"]["single_core"] = one
            out["cpu_baseline"]["optimised_all_cores"] = allc["optimised"]
        except Exception as e:
            out["cpu_baseline"] = one
            out["cpu_baseline"]["all_cores_error"] = repr(e)
        try:
            out["cpu_baseline"]["route_db_rebuild"] = route_db_rebuild_cpu(topo)
        except Exception as e:
            out["cpu_baseline"]["route_db_rebuild"] = {"error": repr(e)}
        try:
            out["cpu_baseline"]["route_db_rebuild_lfa"] = route_db_rebuild_lfa_cpu(topo)
        except Exception as e:
            out["cpu_baseline"]["route_db_rebuild_lfa"] = {"error": repr(e)}
        try:
            out["cpu_baseline"]["ksp2"] = ksp2_cpu_sample(topo)
        except Exception as e:
            out["cpu_baseline"]["ksp2"] = {"error": repr(e)}
        if args.cpu_full:
            try:
                out["cpu_baseline"]["ksp2_full"] = ksp2_cpu_full(topo, args.num_sws)
            except Exception as e:
                out["cpu_baseline"]["ksp2_full"] = {"error": repr(e)}
        out["cpu_baseline"]["cpu_model"] = host_cpu_model()
    if cluster is not None:
        try:
            cluster.close()
        except Exception as e:
            print(f"bench.py: cluster close: {e!r}", file=sys.stderr)
    sys.stdout.flush()
    if rank == 0:
        os.write(json_fd, (json.dumps(out) + "\n").encode())
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
