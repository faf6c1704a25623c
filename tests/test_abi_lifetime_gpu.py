"""Handle lifetimes at the C ABI (include/openr_spf.h "Lifetime"), straight
through ctypes (not the abi.Graph / abi.Query wrappers, which order their own
closes).

A query reads its graph until it is destroyed (device ordinal, stream, the
device CSR), so spf_graph_destroy with a live query must refuse and free
nothing; the round-4 GPU log showed what happens otherwise: the query's
destroy set a freed graph's device ("invalid device ordinal"), and that sticky
HIP error failed the next test's spf_query_run.  The reference's consumer
contract is the same shape: SpfResult references stay valid until the next
topology change (openr/decision/LinkState.h:269-275).
"""

import ctypes as C

import numpy as np
import pytest

from openr_amd import abi
from oracle import spf_py

pytestmark = pytest.mark.gpu


def _grid_csr(n):
    links = []
    for r in range(n):
        for c in range(n):
            v = r * n + c
            if c + 1 < n:
                links.append((v, v + 1, 1, 1))
            if r + 1 < n:
                links.append((v, v + n, 1, 1))
    return abi.Csr.from_links(n * n, links)


def _graph(lib, csr):
    d, keep = abi._graph_desc(csr, 0)
    h = C.c_void_p()
    assert lib.spf_graph_create(C.byref(d), C.byref(h)) == abi.SPF_OK
    return h, keep


def _query(lib, g, sources, flags=abi.SPF_F_NEXTHOPS):
    src = np.asarray(sources, dtype=np.uint32)
    d, keep = abi._query_desc(src, flags)
    h = C.c_void_p()
    assert lib.spf_query_create(g, C.byref(d), C.byref(h)) == abi.SPF_OK
    return h, keep


def _run_and_check(lib, csr, q, sources):
    assert lib.spf_query_run(q) == abi.SPF_OK
    assert lib.spf_query_sync(q) == abi.SPF_OK
    out = np.zeros(csr.num_nodes, dtype=np.uint64)
    for i, s in enumerate(sources):
        assert lib.spf_query_dist(q, i, out.ctypes.data_as(C.POINTER(C.c_uint64))) == abi.SPF_OK
        ref = spf_py.run_spf(csr, s, True, frozenset())
        for v in range(csr.num_nodes):
            assert int(out[v]) == ref[v][0], (s, v)


def test_graph_destroy_with_live_query_is_refused(gpu_ready):
    lib = abi.load()
    csr = _grid_csr(8)
    g, gk = _graph(lib, csr)
    q, qk = _query(lib, g, [0, 9, 63])
    _run_and_check(lib, csr, q, [0, 9, 63])
    # wrong order: refused, nothing freed
    st = lib.spf_graph_destroy(g)
    assert st == abi.SPF_E_INVALID
    assert b"live queries" in lib.spf_last_error_detail()
    # the graph is still whole: the query runs again and is still exact
    _run_and_check(lib, csr, q, [0, 9, 63])
    # a second query over the same graph, then both gone in the right order
    q2, q2k = _query(lib, g, [5])
    assert lib.spf_graph_destroy(g) == abi.SPF_E_INVALID
    assert lib.spf_query_destroy(q) == abi.SPF_OK
    assert lib.spf_graph_destroy(g) == abi.SPF_E_INVALID  # q2 still alive
    assert lib.spf_query_destroy(q2) == abi.SPF_OK
    assert lib.spf_graph_destroy(g) == abi.SPF_OK
    # no sticky device error: a fresh graph and query run and match the oracle
    g3, g3k = _graph(lib, csr)
    q3, q3k = _query(lib, g3, [7, 56])
    _run_and_check(lib, csr, q3, [7, 56])
    assert lib.spf_query_destroy(q3) == abi.SPF_OK
    assert lib.spf_graph_destroy(g3) == abi.SPF_OK
    # destroying NULL is a no-op
    assert lib.spf_graph_destroy(None) == abi.SPF_OK
    assert lib.spf_query_destroy(None) == abi.SPF_OK


def test_query_destroy_with_live_route_table_is_refused(gpu_ready):
    lib = abi.load()
    lib.spf_route_table_create.restype = C.c_int
    lib.spf_route_table_create.argtypes = [
        C.c_void_p, C.c_uint32, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32),
        C.POINTER(C.c_void_p)]
    lib.spf_route_table_destroy.restype = C.c_int
    lib.spf_route_table_destroy.argtypes = [C.c_void_p]
    csr = _grid_csr(6)
    g, gk = _graph(lib, csr)
    sources = list(range(csr.num_nodes))
    q, qk = _query(lib, g, sources)
    assert lib.spf_query_run(q) == abi.SPF_OK
    assert lib.spf_query_sync(q) == abi.SPF_OK
    off = np.asarray([0, 1, 2], dtype=np.uint32)
    ann = np.asarray([3, 20], dtype=np.uint32)
    t = C.c_void_p()
    assert lib.spf_route_table_create(
        q, 2, off.ctypes.data_as(C.POINTER(C.c_uint32)),
        ann.ctypes.data_as(C.POINTER(C.c_uint32)), C.byref(t)) == abi.SPF_OK
    assert lib.spf_query_destroy(q) == abi.SPF_E_INVALID
    assert b"route tables" in lib.spf_last_error_detail()
    assert lib.spf_graph_destroy(g) == abi.SPF_E_INVALID
    assert lib.spf_route_table_destroy(t) == abi.SPF_OK
    assert lib.spf_query_destroy(q) == abi.SPF_OK
    assert lib.spf_graph_destroy(g) == abi.SPF_OK


def test_cluster_handles_refuse_out_of_order_destroy(gpu_ready):
    lib = abi.load()
    csr = _grid_csr(8)
    devs = (C.c_int * 1)(0)
    c = C.c_void_p()
    assert lib.spf_cluster_create_local(1, devs, C.byref(c)) == abi.SPF_OK
    d, dk = abi._graph_desc(csr, 0)
    cg = C.c_void_p()
    assert lib.spf_cgraph_create(c, C.byref(d), C.byref(cg)) == abi.SPF_OK
    src = np.arange(csr.num_nodes, dtype=np.uint32)
    qd, qk = abi._query_desc(src, abi.SPF_F_NEXTHOPS)
    t = C.c_void_p()
    assert lib.spf_table_create_q(cg, C.byref(qd), abi.SPF_T_GATHER_ROWS, C.byref(t)) == abi.SPF_OK
    assert lib.spf_cgraph_destroy(cg) == abi.SPF_E_INVALID
    assert lib.spf_cluster_destroy(c) == abi.SPF_E_INVALID
    # a query directly over a device graph of the cluster graph
    g0 = lib.spf_cgraph_device_graph(cg, 0)
    q, qk2 = _query(lib, C.c_void_p(g0), [1])
    assert lib.spf_table_destroy(t) == abi.SPF_OK
    assert lib.spf_cgraph_destroy(cg) == abi.SPF_E_INVALID  # q still alive
    assert lib.spf_query_destroy(q) == abi.SPF_OK
    # the table still runs over the cluster graph after the refusals
    t2 = C.c_void_p()
    assert lib.spf_table_create_q(cg, C.byref(qd), abi.SPF_T_GATHER_ROWS, C.byref(t2)) == abi.SPF_OK
    assert lib.spf_table_run(t2) == abi.SPF_OK
    assert lib.spf_table_sync(t2) == abi.SPF_OK
    rows = np.zeros((csr.num_nodes, csr.num_nodes), dtype=np.uint32)
    assert lib.spf_table_fetch_rows(
        t2, 0, csr.num_nodes, rows.ctypes.data_as(C.POINTER(C.c_uint32))) == abi.SPF_OK
    for s in (0, 27, 63):
        ref = spf_py.run_spf(csr, s, True, frozenset())
        assert [int(x) for x in rows[s]] == [ref[v][0] for v in range(csr.num_nodes)]
    assert lib.spf_table_destroy(t2) == abi.SPF_OK
    assert lib.spf_cgraph_destroy(cg) == abi.SPF_OK
    assert lib.spf_cluster_destroy(c) == abi.SPF_OK
