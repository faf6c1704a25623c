"""ctypes view of the C ABI in include/openr_spf.h.

This is how Python (tests, bench.py) reaches the HIP engine directly; the C++
LinkState/SpfSolver re-implementation (openr_amd/csrc/host) links the same
shared library.  There is deliberately no fallback: if libopenr_spf.so is
missing or the device is unusable, the calls raise.
"""

from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# OPENR_SPF_LIB: load another build of the engine (kernel tuning sweeps)
LIB_PATH = os.environ.get("OPENR_SPF_LIB") or os.path.join(_HERE, "libopenr_spf.so")

SPF_OK = 0
SPF_E_INVALID = -1
SPF_E_NOMEM = -2
SPF_E_DEVICE = -3
SPF_E_UNSUPPORTED = -4
SPF_UNREACHABLE = (1 << 64) - 1
SPF_TRACE_OVERFLOW = 0xFFFFFFFF
SPF_F_UNIT_METRIC = 0x1
SPF_F_NEXTHOPS = 0x2
SPF_F_ORDER = 0x4

# every symbol include/openr_spf.h declares (tests check the .so exports them)
EXPORTED_SYMBOLS = (
    "spf_device_count",
    "spf_error_string",
    "spf_last_error_detail",
    "spf_device_alloc",
    "spf_device_free",
    "spf_device_memcpy",
    "spf_graph_create",
    "spf_graph_destroy",
    "spf_graph_update",
    "spf_graph_set_transit",
    "spf_graph_patch_metrics",
    "spf_graph_set_edges",
    "spf_graph_set_stream",
    "spf_graph_get_stream",
    "spf_graph_needs_exact",
    "spf_graph_num_nbrs",
    "spf_graph_nbrs",
    "spf_query_create",
    "spf_query_destroy",
    "spf_query_run",
    "spf_query_sync",
    "spf_query_elapsed_ms",
    "spf_query_stage_ms",
    "spf_query_stage_history",
    "spf_query_screened",
    "spf_query_kernel_name",
    "spf_query_kernels",
    "spf_query_dist",
    "spf_query_nh_words",
    "spf_query_nh_bytes",
    "spf_query_nh_offset",
    "spf_query_nexthops",
    "spf_query_order",
    "spf_query_order_keys",
    "spf_route_table_create_ex",
    "spf_table_nexthops",
    "spf_route_table_fetch_link_metrics",
    "spf_query_device_rows",
    "spf_query_row_stride",
    "spf_query_fetch_rows",
    "spf_query_fetch_nexthops",
    "spf_query_fetch_host",
    "spf_query_trace_paths",
    "spf_query_trace_fetch",
    "spf_graph_diff",
    "spf_table_screen",
    "spf_query_scatter_rows",
    "spf_table_repair",
    "spf_route_table_create",
    "spf_route_table_destroy",
    "spf_route_table_run",
    "spf_route_table_elapsed_ms",
    "spf_route_table_link_words",
    "spf_route_table_fetch",
    "spf_route_table_diff",
    "spf_route_table_changed",
    "spf_cluster_unique_id",
    "spf_cluster_create_local",
    "spf_cluster_create_rank",
    "spf_cluster_destroy",
    "spf_cluster_info",
    "spf_cluster_last_error",
    "spf_table_layout",
    "spf_table_create",
    "spf_table_destroy",
    "spf_table_run",
    "spf_table_sync",
    "spf_table_elapsed_ms",
    "spf_table_block",
    "spf_table_nh_words",
    "spf_table_nh_bytes",
    "spf_table_fetch_rows",
    "spf_table_fetch_nexthops",
    "spf_table_trace_paths",
    "spf_table_trace_fetch",
    "spf_table_device_buffers",
    "spf_table_kernel_name",
    "spf_cgraph_create",
    "spf_cgraph_destroy",
    "spf_cgraph_set_transit",
    "spf_cgraph_patch_metrics",
    "spf_cgraph_device_graph",
    "spf_table_create_q",
)

SPF_CLUSTER_ID_BYTES = 128
SPF_T_GATHER_ROWS = 0x100
SPF_T_GATHER_NEXTHOPS = 0x200

SPF_DELTA_REMOVED = 1
SPF_DELTA_ADDED = 2
SPF_SCOPE_ALL = 0
SPF_SCOPE_TAIL_ONLY = 1
SPF_SCOPE_NOT_TAIL = 2

# numpy twin of spf_edge_delta (same layout: 24 bytes)
EDGE_DELTA_DTYPE = np.dtype(
    [("tail", np.uint32), ("head", np.uint32), ("metric", np.uint64),
     ("kind", np.uint32), ("scope", np.uint32)]
)


class SpfError(RuntimeError):
    pass


class _GraphDesc(C.Structure):
    _fields_ = [
        ("num_nodes", C.c_uint32),
        ("num_edges", C.c_uint32),
        ("row_ptr", C.POINTER(C.c_uint32)),
        ("col", C.POINTER(C.c_uint32)),
        ("metric", C.POINTER(C.c_uint64)),
        ("link_id", C.POINTER(C.c_uint32)),
        ("rev", C.POINTER(C.c_uint32)),
        ("node_overloaded", C.POINTER(C.c_uint8)),
        ("num_links", C.c_uint32),
        ("device", C.c_int),
    ]


def _graph_desc(csr: "Csr", device: int = 0):
    """(spf_graph_desc, arrays it points into) for a Csr."""
    keep = [
        np.ascontiguousarray(csr.row_ptr, dtype=np.uint32),
        np.ascontiguousarray(csr.col, dtype=np.uint32),
        np.ascontiguousarray(csr.metric, dtype=np.uint64),
        np.ascontiguousarray(csr.link_id, dtype=np.uint32),
        np.ascontiguousarray(csr.rev, dtype=np.uint32),
        np.ascontiguousarray(csr.overloaded, dtype=np.uint8),
    ]
    row, col, met, lid, rev, ov = keep
    d = _GraphDesc(
        csr.num_nodes,
        len(col),
        _p(row, C.c_uint32),
        _p(col, C.c_uint32),
        _p(met, C.c_uint64),
        _p(lid, C.c_uint32),
        _p(rev, C.c_uint32),
        _p(ov, C.c_uint8),
        csr.num_links,
        device,
    )
    return d, keep


class _QueryDesc(C.Structure):
    _fields_ = [
        ("num_queries", C.c_uint32),
        ("sources", C.POINTER(C.c_uint32)),
        ("ignore_offsets", C.POINTER(C.c_uint32)),
        ("ignore_links", C.POINTER(C.c_uint32)),
        ("flags", C.c_uint32),
    ]


def _query_desc(src, flags, ignore=None):
    """spf_query_desc of uint32 sources and optional per-query ignore lists
    (link ids; sorted and de-duplicated here).  Returns (desc, keep-alive)."""
    keep = [src]
    ioff = ilinks = None
    if ignore is not None:
        offs = [0]
        flat = []
        for lst in ignore:
            s = sorted(set(int(x) for x in lst))
            flat.extend(s)
            offs.append(len(flat))
        ioff = np.asarray(offs, dtype=np.uint32)
        ilinks = np.asarray(flat if flat else [0], dtype=np.uint32)
        keep += [ioff, ilinks]
    d = _QueryDesc(
        len(src),
        _p(src, C.c_uint32),
        _p(ioff, C.c_uint32) if ioff is not None else None,
        _p(ilinks, C.c_uint32) if ilinks is not None else None,
        flags,
    )
    return d, keep


_lib = None


def load():
    """Load libopenr_spf.so (raises OSError if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise OSError(
            f"{LIB_PATH} missing: run `python -m openr_amd.build` "
            "(the HIP engine has no CPU fallback)"
        )
    lib = C.CDLL(LIB_PATH)
    vp = C.c_void_p
    u32 = C.c_uint32
    pu32 = C.POINTER(C.c_uint32)
    pu64 = C.POINTER(C.c_uint64)
    sig = {
        "spf_device_count": (C.c_int, []),
        "spf_error_string": (C.c_char_p, [C.c_int]),
        "spf_last_error_detail": (C.c_char_p, []),
        "spf_graph_create": (C.c_int, [C.POINTER(_GraphDesc), C.POINTER(vp)]),
        "spf_device_alloc": (C.c_int, [C.c_int, C.c_size_t, C.POINTER(vp)]),
        "spf_device_free": (C.c_int, [C.c_int, vp]),
        "spf_device_memcpy": (C.c_int, [C.c_int, vp, vp, C.c_size_t, C.c_int]),
        "spf_graph_destroy": (C.c_int, [vp]),
        "spf_graph_update": (C.c_int, [vp, C.POINTER(_GraphDesc)]),
        "spf_graph_set_transit": (C.c_int, [vp, C.POINTER(C.c_uint8)]),
        "spf_graph_patch_metrics": (C.c_int, [vp, u32, pu32, pu64]),
        "spf_graph_set_edges": (C.c_int, [vp, u32, pu32, C.POINTER(C.c_uint8), pu64]),
        "spf_graph_set_stream": (C.c_int, [vp, vp]),
        "spf_graph_get_stream": (vp, [vp]),
        "spf_graph_needs_exact": (C.c_int, [vp]),
        "spf_graph_num_nbrs": (C.c_int, [vp, u32]),
        "spf_graph_nbrs": (C.c_int, [vp, u32, pu32]),
        "spf_query_create": (C.c_int, [vp, C.POINTER(_QueryDesc), C.POINTER(vp)]),
        "spf_query_destroy": (C.c_int, [vp]),
        "spf_query_run": (C.c_int, [vp]),
        "spf_query_sync": (C.c_int, [vp]),
        "spf_query_elapsed_ms": (C.c_int, [vp, C.POINTER(C.c_float)]),
        "spf_query_screened": (C.c_int, [vp, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]),
        "spf_query_stage_ms": (
            C.c_int,
            [vp, C.POINTER(C.c_float), C.POINTER(C.c_float)],
        ),
        "spf_query_stage_history": (
            C.c_int,
            [vp, u32, C.POINTER(C.c_float), C.POINTER(C.c_float), pu32],
        ),
        "spf_query_kernel_name": (C.c_char_p, [vp]),
        "spf_query_kernels": (C.c_int, [vp, C.c_char_p, C.c_size_t]),
        "spf_query_dist": (C.c_int, [vp, u32, pu64]),
        "spf_query_nh_words": (C.c_int, [vp, u32]),
        "spf_query_nh_bytes": (C.c_int, [vp, u32]),
        "spf_query_nh_offset": (C.c_int, [vp, u32, pu64]),
        "spf_query_nexthops": (C.c_int, [vp, u32, pu64]),
        "spf_query_order": (C.c_int, [vp, u32, pu32]),
        "spf_query_order_keys": (C.c_int, [vp, u32, pu64]),
        "spf_query_row_stride": (u32, [vp]),
        "spf_query_fetch_rows": (C.c_int, [vp, u32, u32, vp, C.c_size_t, C.c_int]),
        "spf_query_fetch_nexthops": (C.c_int, [vp, u32, u32, pu64]),
        "spf_query_fetch_host": (C.c_int, [vp, u32, u32, vp, C.c_size_t, vp]),
        "spf_query_trace_paths": (C.c_int, [vp, u32, u32, pu32, pu32, pu32]),
        "spf_query_trace_fetch": (C.c_int, [vp, pu32, pu32]),
        "spf_query_device_rows": (
            C.c_int,
            [vp, C.POINTER(vp), pu32, C.POINTER(vp), pu64],
        ),
        "spf_graph_diff": (
            C.c_int,
            [C.POINTER(_GraphDesc), C.POINTER(_GraphDesc), vp, u32, pu32],
        ),
        "spf_table_screen": (
            C.c_int,
            [vp, vp, C.c_size_t, u32, pu32, vp, u32, C.POINTER(C.c_uint8)],
        ),
        "spf_query_scatter_rows": (C.c_int, [vp, pu32, vp, C.c_size_t]),
        "spf_table_repair": (C.c_int, [vp, vp, C.c_size_t, u32, pu32, pu32, vp, u32]),
        "spf_table_nexthops": (
            C.c_int, [vp, vp, C.c_size_t, C.POINTER(C.c_int32), u32, pu32, vp, pu64]),
        "spf_cluster_unique_id": (C.c_int, [C.POINTER(C.c_uint8)]),
        "spf_cluster_create_local": (C.c_int, [u32, C.POINTER(C.c_int), C.POINTER(vp)]),
        "spf_cluster_create_rank": (C.c_int, [u32, u32, C.POINTER(C.c_uint8), C.c_int, C.POINTER(vp)]),
        "spf_cluster_destroy": (C.c_int, [vp]),
        "spf_cluster_info": (C.c_int, [vp, pu32, pu32, pu32]),
        "spf_cluster_last_error": (C.c_char_p, []),
        "spf_table_layout": (C.c_int, [u32, u32, u32, pu32, pu64, pu64, pu64]),
        "spf_table_create": (C.c_int, [vp, C.POINTER(_GraphDesc), u32, pu32, u32, C.POINTER(vp)]),
        "spf_table_destroy": (C.c_int, [vp]),
        "spf_table_run": (C.c_int, [vp]),
        "spf_table_sync": (C.c_int, [vp]),
        "spf_table_elapsed_ms": (C.c_int, [vp, C.POINTER(C.c_float), C.POINTER(C.c_float)]),
        "spf_table_block": (C.c_int, [vp, u32, pu32, pu32]),
        "spf_table_nh_words": (C.c_int, [vp, u32]),
        "spf_table_nh_bytes": (C.c_int, [vp, u32]),
        "spf_table_fetch_rows": (C.c_int, [vp, u32, u32, pu32]),
        "spf_table_fetch_nexthops": (C.c_int, [vp, u32, u32, pu64]),
        "spf_table_trace_paths": (C.c_int, [vp, pu32, pu32, pu32]),
        "spf_table_trace_fetch": (C.c_int, [vp, pu32, pu32]),
        "spf_table_device_buffers": (C.c_int, [vp, u32, C.POINTER(vp), C.POINTER(vp), pu64]),
        "spf_table_kernel_name": (C.c_int, [vp, u32, C.POINTER(C.c_char_p)]),
        "spf_cgraph_create": (C.c_int, [vp, C.POINTER(_GraphDesc), C.POINTER(vp)]),
        "spf_cgraph_destroy": (C.c_int, [vp]),
        "spf_cgraph_set_transit": (C.c_int, [vp, C.POINTER(C.c_uint8)]),
        "spf_cgraph_patch_metrics": (C.c_int, [vp, u32, pu32, pu64]),
        "spf_cgraph_device_graph": (vp, [vp, u32]),
        "spf_table_create_q": (C.c_int, [vp, C.POINTER(_QueryDesc), u32, C.POINTER(vp)]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def _check(status: int, what: str):
    if status != SPF_OK:
        lib = load()
        raise SpfError(
            f"{what}: {lib.spf_error_string(status).decode()} "
            f"({lib.spf_last_error_detail().decode()})"
        )


def _p(arr, ctype):
    return arr.ctypes.data_as(C.POINTER(ctype))


def device_count() -> int:
    return load().spf_device_count()


@dataclass
class Csr:
    """Directed CSR of the up links of one area (see spf_graph_desc)."""

    num_nodes: int
    row_ptr: np.ndarray  # uint32 [V+1]
    col: np.ndarray  # uint32 [E]
    metric: np.ndarray  # uint64 [E]
    link_id: np.ndarray  # uint32 [E]
    rev: np.ndarray  # uint32 [E]
    overloaded: np.ndarray  # uint8 [V]
    num_links: int

    @staticmethod
    def from_links(num_nodes, links, overloaded=None):
        """links: iterable of (u, v, metric_u_to_v, metric_v_to_u).

        Half-edges of one row keep the input order of `links`.
        """
        links = list(links)
        V = int(num_nodes)
        deg = np.zeros(V + 1, dtype=np.int64)
        for (u, v, _, _) in links:
            deg[u + 1] += 1
            deg[v + 1] += 1
        row = np.cumsum(deg).astype(np.uint32)
        E = int(row[-1])
        fill = row[:-1].astype(np.int64).copy()
        col = np.zeros(E, dtype=np.uint32)
        met = np.zeros(E, dtype=np.uint64)
        lid = np.zeros(E, dtype=np.uint32)
        rev = np.zeros(E, dtype=np.uint32)
        for i, (u, v, muv, mvu) in enumerate(links):
            eu = fill[u]
            fill[u] += 1
            ev = fill[v]
            fill[v] += 1
            col[eu], met[eu], lid[eu], rev[eu] = v, np.uint64(muv % (1 << 64)), i, ev
            col[ev], met[ev], lid[ev], rev[ev] = u, np.uint64(mvu % (1 << 64)), i, eu
        ov = (
            np.zeros(V, dtype=np.uint8)
            if overloaded is None
            else np.asarray(overloaded, dtype=np.uint8)
        )
        return Csr(V, row, col, met, lid, rev, ov, len(links))


class Graph:
    def __init__(self, csr: Csr, device: int = 0):
        lib = load()
        self.csr = csr
        d, self._keep = _graph_desc(csr, device)
        h = C.c_void_p()
        _check(lib.spf_graph_create(C.byref(d), C.byref(h)), "spf_graph_create")
        self.h = h
        self.V = csr.num_nodes
        import weakref

        self._queries = weakref.WeakSet()  # live queries: destroyed before the graph

    def close(self):
        if self.h:
            # a query reads its graph when it is destroyed (device, stream):
            # close the ones still alive first
            for q in list(self._queries):
                q.close()
            # refused (and nothing freed) while a query is alive: the C ABI's
            # lifetime rule, include/openr_spf.h
            _check(load().spf_graph_destroy(self.h), "spf_graph_destroy")
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def needs_exact(self) -> bool:
        return bool(load().spf_graph_needs_exact(self.h))

    def num_nbrs(self, node: int) -> int:
        n = load().spf_graph_num_nbrs(self.h, node)
        if n < 0:
            _check(n, "spf_graph_num_nbrs")
        return int(n)

    def nbrs(self, node: int) -> np.ndarray:
        lib = load()
        n = lib.spf_graph_num_nbrs(self.h, node)
        if n < 0:
            _check(n, "spf_graph_num_nbrs")
        out = np.zeros(max(n, 1), dtype=np.uint32)
        _check(lib.spf_graph_nbrs(self.h, node, _p(out, C.c_uint32)), "nbrs")
        return out[:n]

    def set_transit(self, overloaded):
        ov = np.ascontiguousarray(overloaded, dtype=np.uint8)
        _check(load().spf_graph_set_transit(self.h, _p(ov, C.c_uint8)), "transit")

    def set_edges(self, edges, up, metrics):
        """Half-edges down (up=0) / back up (1) in place (spf_graph_set_edges)."""
        e = np.ascontiguousarray(edges, dtype=np.uint32)
        u = np.ascontiguousarray(up, dtype=np.uint8)
        m = np.ascontiguousarray(metrics, dtype=np.uint64)
        _check(load().spf_graph_set_edges(self.h, len(e), _p(e, C.c_uint32), _p(u, C.c_uint8),
                                          _p(m, C.c_uint64)), "set_edges")

    def patch_metrics(self, edges, metrics):
        """Metrics of existing half-edges, in place (spf_graph_patch_metrics)."""
        e = np.ascontiguousarray(edges, dtype=np.uint32)
        m = np.ascontiguousarray(metrics, dtype=np.uint64)
        if len(e) != len(m):
            raise ValueError("edges / metrics length mismatch")
        _check(load().spf_graph_patch_metrics(self.h, len(e), _p(e, C.c_uint32), _p(m, C.c_uint64)),
               "patch_metrics")

    def update(self, csr: "Csr"):
        """Rebuild in place from a new CSR of the same node set
        (spf_graph_update); no query of this graph may be alive."""
        d, keep = _graph_desc(csr, 0)
        _check(load().spf_graph_update(self.h, C.byref(d)), "spf_graph_update")
        self.csr = csr
        self._keep = keep

    def set_stream(self, stream_ptr: int | None):
        _check(load().spf_graph_set_stream(self.h, stream_ptr), "set_stream")

    def query(self, sources, flags=SPF_F_NEXTHOPS, ignore=None) -> "Query":
        return Query(self, sources, flags, ignore)

    def table_screen(self, rows_ptr: int, pitch: int, sources, deltas) -> np.ndarray:
        """uint8 [len(sources)]: 1 where the uint32 device row of sources[i]
        (rows_ptr + i * pitch elements) can be changed by `deltas`."""
        src = np.ascontiguousarray(sources, dtype=np.uint32)
        dl = np.ascontiguousarray(deltas, dtype=EDGE_DELTA_DTYPE)
        out = np.zeros(max(len(src), 1), dtype=np.uint8)
        _check(
            load().spf_table_screen(
                self.h, rows_ptr, pitch, len(src), _p(src, C.c_uint32),
                dl.ctypes.data if len(dl) else None, len(dl), _p(out, C.c_uint8),
            ),
            "table_screen",
        )
        return out[: len(src)]

    def table_nexthops(self, rows_ptr: int, pitch: int, row_of, sources, masks_ptr: int, mask_off):
        """Next-hop masks of `sources` from a device distance table
        (spf_table_nexthops); row_of[x] = table row of node x (-1 = none)."""
        ro = np.ascontiguousarray(row_of, dtype=np.int32)
        src = np.ascontiguousarray(sources, dtype=np.uint32)
        off = np.ascontiguousarray(mask_off, dtype=np.uint64)
        _check(load().spf_table_nexthops(self.h, rows_ptr, pitch, _p(ro, C.c_int32), len(src),
                                         _p(src, C.c_uint32), masks_ptr, _p(off, C.c_uint64)),
               "table_nexthops")

    def table_repair(self, rows_ptr: int, pitch: int, sources, row_idx, deltas) -> bool:
        """Repair device rows in place after `deltas` (spf_table_repair).
        False when the engine cannot (SPF_E_UNSUPPORTED): recompute instead."""
        src = np.ascontiguousarray(sources, dtype=np.uint32)
        ri = np.ascontiguousarray(row_idx, dtype=np.uint32)
        dl = np.ascontiguousarray(deltas, dtype=EDGE_DELTA_DTYPE)
        if len(src) != len(ri):
            raise ValueError("sources / row_idx length mismatch")
        st = load().spf_table_repair(self.h, rows_ptr, pitch, len(src), _p(src, C.c_uint32),
                                     _p(ri, C.c_uint32), dl.ctypes.data if len(dl) else None, len(dl))
        if st == SPF_E_UNSUPPORTED:
            return False
        _check(st, "table_repair")
        return True


def mask_layout(graph: "Graph", sources) -> tuple:
    """(nh_words per source, word offset per source, total words) of packed
    next-hop mask rows: V * W words per source rounded up to 4 (32 bytes),
    the layout of spf_query masks."""
    V = graph.V
    words = np.array([max(1, (graph.num_nbrs(int(s)) + 63) // 64) for s in sources], dtype=np.uint64)
    sizes = (words * np.uint64(V) + np.uint64(3)) & ~np.uint64(3)
    off = np.zeros(len(sources), dtype=np.uint64)
    if len(sources):
        off[1:] = np.cumsum(sizes)[:-1]
    return words, off, int(sizes.sum())


def graph_diff(before: "Csr", after: "Csr") -> np.ndarray:
    """Directed edge deltas (EDGE_DELTA_DTYPE) turning `before` into `after`
    (host only, spf_graph_diff)."""
    lib = load()
    da, ka = _graph_desc(before)
    db, kb = _graph_desc(after)
    n = C.c_uint32()
    _check(lib.spf_graph_diff(C.byref(da), C.byref(db), None, 0, C.byref(n)), "graph_diff")
    out = np.zeros(max(n.value, 1), dtype=EDGE_DELTA_DTYPE)
    _check(
        lib.spf_graph_diff(C.byref(da), C.byref(db), out.ctypes.data, n.value, C.byref(n)),
        "graph_diff",
    )
    del ka, kb
    return out[: n.value]


def _unpack_traces(n, pc, lc, fetch):
    ok = pc[:n] != SPF_TRACE_OVERFLOW
    links = np.zeros(max(int(lc[:n][ok].sum()), 1), dtype=np.uint32)
    ends = np.zeros(max(int(pc[:n][ok].sum()), 1), dtype=np.uint32)
    fetch(links, ends)
    out, lo, po = [], 0, 0
    for i in range(n):
        if not ok[i]:
            out.append(None)
            continue
        paths, a = [], 0
        for j in range(int(pc[i])):
            b = int(ends[po + j])
            paths.append([int(x) for x in links[lo + a : lo + b]])
            a = b
        out.append(paths)
        lo += int(lc[i])
        po += int(pc[i])
    return out


class Query:
    def __init__(self, graph: Graph, sources, flags, ignore=None):
        lib = load()
        self.graph = graph
        src = np.ascontiguousarray(sources, dtype=np.uint32)
        d, keep = _query_desc(src, flags, ignore)
        h = C.c_void_p()
        _check(lib.spf_query_create(graph.h, C.byref(d), C.byref(h)), "spf_query_create")
        self.h = h
        self._keep = keep
        self.n = len(src)
        self.flags = flags
        graph._queries.add(self)

    def close(self):
        if self.h:
            load().spf_query_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def run(self, sync=True):
        lib = load()
        _check(lib.spf_query_run(self.h), "spf_query_run")
        if sync:
            _check(lib.spf_query_sync(self.h), "spf_query_sync")
        return self

    def sync(self):
        _check(load().spf_query_sync(self.h), "spf_query_sync")

    def elapsed_ms(self) -> float:
        ms = C.c_float()
        _check(load().spf_query_elapsed_ms(self.h, C.byref(ms)), "elapsed")
        return float(ms.value)

    def stage_ms(self):
        """(distance-kernel ms, next-hop-kernel ms) of the last run."""
        a, b = C.c_float(), C.c_float()
        _check(load().spf_query_stage_ms(self.h, C.byref(a), C.byref(b)), "stage_ms")
        return float(a.value), float(b.value)

    def stage_history(self, n: int):
        """[(distance ms, next-hop ms)] of the last min(n, 64) runs."""
        d = (C.c_float * max(n, 1))()
        h = (C.c_float * max(n, 1))()
        got = C.c_uint32()
        _check(load().spf_query_stage_history(self.h, n, d, h, C.byref(got)), "stage_history")
        return [(float(d[i]), float(h[i])) for i in range(got.value)]

    def screened(self):
        """Queries of the last run the what-if screen resolved by copying the
        baseline rows (None: the query has no screen)."""
        n, has = C.c_uint32(), C.c_uint32()
        _check(load().spf_query_screened(self.h, C.byref(n), C.byref(has)), "screened")
        return int(n.value) if has.value else None

    @property
    def kernel(self) -> str:
        return load().spf_query_kernel_name(self.h).decode()

    def kernels(self) -> list:
        """The HIP kernels the last run launched (spf_query_kernels)."""
        lib = load()
        n = lib.spf_query_kernels(self.h, None, 0)
        _check(min(n, 0), "spf_query_kernels")
        buf = C.create_string_buffer(n + 1)
        lib.spf_query_kernels(self.h, buf, n + 1)
        return [k for k in buf.value.decode().split(",") if k]

    def dist(self, i: int) -> np.ndarray:
        out = np.zeros(self.graph.V, dtype=np.uint64)
        _check(load().spf_query_dist(self.h, i, _p(out, C.c_uint64)), "dist")
        return out

    def nh_words(self, i: int) -> int:
        return load().spf_query_nh_words(self.h, i)

    def nh_bytes(self, i: int) -> int:
        """Device bytes per node of query i's masks (SPF_NH_BYTES)."""
        return load().spf_query_nh_bytes(self.h, i)

    def nh_offset(self, i: int) -> int:
        """Byte offset of query i's masks in device_rows()' mask block."""
        o = C.c_uint64()
        _check(load().spf_query_nh_offset(self.h, i, C.byref(o)), "nh_offset")
        return o.value

    def nexthops(self, i: int) -> np.ndarray:
        W = self.nh_words(i)
        out = np.zeros(self.graph.V * W, dtype=np.uint64)
        _check(load().spf_query_nexthops(self.h, i, _p(out, C.c_uint64)), "nexthops")
        return out.reshape(self.graph.V, W)

    def nexthop_sets(self, i: int, src: int):
        """{node: frozenset(first-hop node ids)} for reached nodes."""
        d = self.dist(i)
        masks = self.nexthops(i)
        nb = self.graph.nbrs(src)
        out = {}
        for v in range(self.graph.V):
            if d[v] == np.uint64(SPF_UNREACHABLE):
                continue
            s = set()
            for w in range(masks.shape[1]):
                m = int(masks[v, w])
                while m:
                    b = (m & -m).bit_length() - 1
                    s.add(int(nb[w * 64 + b]))
                    m &= m - 1
            out[v] = frozenset(s)
        return out

    def order(self, i: int) -> np.ndarray:
        out = np.zeros(self.graph.V, dtype=np.uint32)
        _check(load().spf_query_order(self.h, i, _p(out, C.c_uint32)), "order")
        return out

    def order_keys(self, i: int) -> np.ndarray:
        """Wide plan: settle order = lexicographic (dist, key)."""
        out = np.zeros(self.graph.V, dtype=np.uint64)
        _check(load().spf_query_order_keys(self.h, i, _p(out, C.c_uint64)), "order_keys")
        return out

    def fetch_rows(self, first: int, count: int, dst_ptr: int, pitch: int, on_device=True):
        """Copy uint32 distance rows into caller memory (device: async on
        the graph stream)."""
        _check(
            load().spf_query_fetch_rows(self.h, first, count, dst_ptr, pitch, 1 if on_device else 0),
            "fetch_rows",
        )

    def scatter_rows(self, dst_rows, table_ptr: int, pitch: int):
        """Row i of this query -> row dst_rows[i] of a device table (async
        on the graph stream, spf_query_scatter_rows)."""
        dr = np.ascontiguousarray(dst_rows, dtype=np.uint32)
        _check(load().spf_query_scatter_rows(self.h, _p(dr, C.c_uint32), table_ptr, pitch),
               "scatter_rows")

    def fetch_nexthops(self, first: int, count: int) -> np.ndarray:
        """Masks of queries [first, first+count), back to back (V*W_i words
        each), in one device-to-host transfer."""
        n = sum(self.graph.V * self.nh_words(i) for i in range(first, first + count))
        out = np.zeros(max(n, 1), dtype=np.uint64)
        _check(load().spf_query_fetch_nexthops(self.h, first, count, _p(out, C.c_uint64)),
               "fetch_nexthops")
        return out[:n]

    def fetch_host(self, first: int, count: int, rows=True, masks=True):
        """Rows and masks of queries [first, first+count) in one call
        (spf_query_fetch_host): (rows [count, V] uint32 or None, masks as
        fetch_nexthops or None)."""
        V = self.graph.V
        r = np.zeros((count, V), dtype=np.uint32) if rows else None
        m = None
        if masks:
            n = sum(V * self.nh_words(i) for i in range(first, first + count))
            m = np.zeros(max(n, 1), dtype=np.uint64)
        _check(load().spf_query_fetch_host(
            self.h, first, count, r.ctypes.data if rows else None, V * 4,
            m.ctypes.data if masks else None), "fetch_host")
        return r, (m[:n] if masks else None)

    def trace_paths(self, dests, first: int = 0):
        """getKthPaths' trace loop on the device (spf_query_trace_paths +
        spf_query_trace_fetch): per query, a list of paths (each a list of
        link ids, src -> dst), or None when the device trace overflowed."""
        d = np.ascontiguousarray(dests, dtype=np.uint32)
        n = len(d)
        pc = np.zeros(max(n, 1), dtype=np.uint32)
        lc = np.zeros(max(n, 1), dtype=np.uint32)
        lib = load()
        _check(lib.spf_query_trace_paths(self.h, first, n, _p(d, C.c_uint32), _p(pc, C.c_uint32),
                                         _p(lc, C.c_uint32)), "trace_paths")
        return _unpack_traces(n, pc, lc, lambda L, E: _check(
            lib.spf_query_trace_fetch(self.h, _p(L, C.c_uint32), _p(E, C.c_uint32)), "trace_fetch"))

    def device_rows(self):
        dp = C.c_void_p()
        eb = C.c_uint32()
        np_ = C.c_void_p()
        nt = C.c_uint64()
        _check(
            load().spf_query_device_rows(
                self.h, C.byref(dp), C.byref(eb), C.byref(np_), C.byref(nt)
            ),
            "device_rows",
        )
        return dp.value, eb.value, np_.value, nt.value


# ------------------------------------------------- multi-GPU tables (RCCL)


def _check_cl(status: int, what: str):
    if status != SPF_OK:
        lib = load()
        raise SpfError(
            f"{what}: {lib.spf_error_string(status).decode()} "
            f"({lib.spf_cluster_last_error().decode()} / {lib.spf_last_error_detail().decode()})"
        )


def nh_bytes_for(nbrs: int) -> int:
    """Device bytes per node of a source's next-hop masks (SPF_NH_BYTES)."""
    return 1 if nbrs <= 8 else 2 if nbrs <= 16 else 4 if nbrs <= 32 else 8 * ((nbrs + 63) // 64)


def table_layout(n: int, world: int, V: int, nh_bytes=None):
    """spf_table_layout (host only): (block_first uint64[world+1],
    mask_off uint64[n] BYTE offsets, mask_cap bytes per rank slot); nh_bytes
    = device bytes per node of each source's masks (nh_bytes_for)."""
    bf = np.zeros(world + 1, dtype=np.uint64)
    mo = np.zeros(max(n, 1), dtype=np.uint64)
    cap = C.c_uint64()
    w = None if nh_bytes is None else np.ascontiguousarray(nh_bytes, dtype=np.uint32)
    _check_cl(load().spf_table_layout(n, world, V, _p(w, C.c_uint32) if w is not None else None,
                                      _p(bf, C.c_uint64), _p(mo, C.c_uint64), C.byref(cap)),
              "spf_table_layout")
    return bf, mo[:n], int(cap.value)


def cluster_unique_id() -> bytes:
    buf = (C.c_uint8 * SPF_CLUSTER_ID_BYTES)()
    _check_cl(load().spf_cluster_unique_id(buf), "spf_cluster_unique_id")
    return bytes(buf)


class Cluster:
    """RCCL communicator(s) of an all-sources fan-out: every listed local
    device (spf_cluster_create_local) or one rank of a one-process-per-GPU
    job (spf_cluster_create_rank, `uid` from cluster_unique_id on one rank)."""

    def __init__(self, devices=None, *, world=None, rank=None, uid=None, device=0):
        lib = load()
        h = C.c_void_p()
        if world is None:
            devs = (C.c_int * len(devices))(*devices)
            _check_cl(lib.spf_cluster_create_local(len(devices), devs, C.byref(h)),
                      "spf_cluster_create_local")
        else:
            idb = (C.c_uint8 * SPF_CLUSTER_ID_BYTES)(*uid)
            _check_cl(lib.spf_cluster_create_rank(world, rank, idb, device, C.byref(h)),
                      "spf_cluster_create_rank")
        self.h = h
        w, f, n = C.c_uint32(), C.c_uint32(), C.c_uint32()
        _check_cl(lib.spf_cluster_info(h, C.byref(w), C.byref(f), C.byref(n)), "spf_cluster_info")
        self.world, self.first_rank, self.local_devices = w.value, f.value, n.value

    def close(self):
        if self.h:
            # refused (nothing freed, handle kept) while a table or cluster
            # graph over it is alive: include/openr_spf.h "Lifetime"
            _check_cl(load().spf_cluster_destroy(self.h), "spf_cluster_destroy")
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class ClusterGraph:
    """One persistent spf_graph per local device of a Cluster (spf_cgraph_*)."""

    def __init__(self, cluster: Cluster, csr: "Csr"):
        lib = load()
        self.cluster = cluster
        self.V = csr.num_nodes
        d, keep = _graph_desc(csr, 0)
        h = C.c_void_p()
        _check_cl(lib.spf_cgraph_create(cluster.h, C.byref(d), C.byref(h)), "spf_cgraph_create")
        self.h = h
        self._keep = keep

    def close(self):
        if self.h:
            # refused (nothing freed, handle kept) while a table over it lives
            _check_cl(load().spf_cgraph_destroy(self.h), "spf_cgraph_destroy")
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_transit(self, overloaded):
        ov = np.ascontiguousarray(overloaded, dtype=np.uint8)
        _check_cl(load().spf_cgraph_set_transit(self.h, _p(ov, C.c_uint8)), "spf_cgraph_set_transit")

    def patch_metrics(self, edges, metrics):
        e = np.ascontiguousarray(edges, dtype=np.uint32)
        m = np.ascontiguousarray(metrics, dtype=np.uint64)
        _check_cl(load().spf_cgraph_patch_metrics(self.h, len(e), _p(e, C.c_uint32), _p(m, C.c_uint64)),
                  "spf_cgraph_patch_metrics")

    def table(self, sources, flags, ignore=None, gather=0):
        return Table(self.cluster, None, sources, flags | gather, cgraph=self, ignore=ignore)


class Table:
    """All-sources table sharded over a Cluster (spf_table_*); with `cgraph`
    a query table over persistent cluster graphs (spf_table_create_q), whose
    queries may carry ignore lists (one list of link ids per query)."""

    def __init__(self, cluster: Cluster, csr: "Csr", sources, flags, cgraph=None, ignore=None):
        lib = load()
        self.cluster = cluster
        src = np.ascontiguousarray(sources, dtype=np.uint32)
        h = C.c_void_p()
        if cgraph is None:
            self.V = csr.num_nodes
            d, keep = _graph_desc(csr, 0)
            _check_cl(lib.spf_table_create(cluster.h, C.byref(d), len(src), _p(src, C.c_uint32), flags,
                                           C.byref(h)), "spf_table_create")
        else:
            self.V = cgraph.V
            qd, keep = _query_desc(src, flags & 0xFF, ignore)
            _check_cl(lib.spf_table_create_q(cgraph.h, C.byref(qd), flags & ~0xFF, C.byref(h)),
                      "spf_table_create_q")
        self.h = h
        self.n = len(src)
        self.flags = flags
        self._keep = (keep, src, cgraph)

    def close(self):
        if self.h:
            load().spf_table_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def run(self, sync=True):
        _check_cl(load().spf_table_run(self.h), "spf_table_run")
        if sync:
            self.sync()
        return self

    def sync(self):
        _check_cl(load().spf_table_sync(self.h), "spf_table_sync")

    def elapsed_ms(self):
        a, b = C.c_float(), C.c_float()
        _check_cl(load().spf_table_elapsed_ms(self.h, C.byref(a), C.byref(b)), "spf_table_elapsed_ms")
        return float(a.value), float(b.value)

    def block(self, rank: int):
        f, c = C.c_uint32(), C.c_uint32()
        _check_cl(load().spf_table_block(self.h, rank, C.byref(f), C.byref(c)), "spf_table_block")
        return f.value, c.value

    def nh_words(self, i: int) -> int:
        return load().spf_table_nh_words(self.h, i)

    def nh_bytes(self, i: int) -> int:
        return load().spf_table_nh_bytes(self.h, i)

    def kernel(self, local: int = 0) -> str:
        n = C.c_char_p()
        _check_cl(load().spf_table_kernel_name(self.h, local, C.byref(n)), "spf_table_kernel_name")
        return n.value.decode()

    def fetch_rows(self, first: int, count: int) -> np.ndarray:
        out = np.empty((count, self.V), dtype=np.uint32)
        _check_cl(load().spf_table_fetch_rows(self.h, first, count, _p(out, C.c_uint32)),
                  "spf_table_fetch_rows")
        return out

    def fetch_nexthops(self, first: int, count: int) -> np.ndarray:
        n = sum(self.V * self.nh_words(i) for i in range(first, first + count))
        out = np.zeros(max(n, 1), dtype=np.uint64)
        _check_cl(load().spf_table_fetch_nexthops(self.h, first, count, _p(out, C.c_uint64)),
                  "spf_table_fetch_nexthops")
        return out[:n]

    def trace_paths(self, dests):
        """spf_table_trace_paths + spf_table_trace_fetch: per table query,
        its paths (lists of link ids) or None (overflow: trace on the host)."""
        d = np.ascontiguousarray(dests, dtype=np.uint32)
        n = len(d)
        pc = np.zeros(max(n, 1), dtype=np.uint32)
        lc = np.zeros(max(n, 1), dtype=np.uint32)
        lib = load()
        _check_cl(lib.spf_table_trace_paths(self.h, _p(d, C.c_uint32), _p(pc, C.c_uint32),
                                            _p(lc, C.c_uint32)), "spf_table_trace_paths")
        return _unpack_traces(n, pc, lc, lambda L, E: _check_cl(
            lib.spf_table_trace_fetch(self.h, _p(L, C.c_uint32), _p(E, C.c_uint32)),
            "spf_table_trace_fetch"))

    def device_buffers(self, local: int = 0):
        r, m = C.c_void_p(), C.c_void_p()
        cap = C.c_uint64()
        _check_cl(load().spf_table_device_buffers(self.h, local, C.byref(r), C.byref(m), C.byref(cap)),
                  "spf_table_device_buffers")
        return r.value, m.value, int(cap.value)
