/*
 * openr_spf.h — the C ABI of the MI355X SPF engine (the ONLY entry point to
 * the HIP kernels).  Plain pointers and sizes, no C++ or torch types.
 *
 * What it replaces.  Open/R has no FFI for this path: the boundary is the C++
 * class API of LinkState / SpfSolver.  Every function below replaces the inner
 * arithmetic of one reference member function; the re-implemented LinkState
 * (openr_amd/csrc/host/LinkState.cpp) is the only caller:
 *
 *   spf_graph_create / spf_graph_destroy
 *       replaces the adjacency graph the reference walks in place:
 *       LinkState::linkMap_ / nodeOverloads_   (openr/decision/LinkState.h:457-463)
 *       and Link::isUp / getMetricFromNode     (openr/decision/LinkState.cpp:195-236)
 *   spf_graph_set_transit
 *       replaces LinkState::isNodeOverloaded as read by runSpf
 *                                               (openr/decision/LinkState.cpp:829-836)
 *   spf_query_create / spf_query_run / spf_query_sync
 *       replaces LinkState::runSpf(src, useLinkMetric, linksToIgnore)
 *                                               (openr/decision/LinkState.cpp:806-880)
 *       batched over many sources (getSpfResult memo fill, LFA neighbours,
 *       all-sources views, KSP2 second passes, what-if link failures).
 *   spf_query_dist / spf_query_nexthops / spf_query_order
 *       replace the reads of NodeSpfResult::metric / nextHops / pathLinks
 *       order                                   (openr/decision/LinkState.h:203-257)
 *
 * Conventions
 *   - Status: 0 = OK, negative = error (SPF_E_*).  No exceptions cross the ABI.
 *   - Ownership: every device buffer is owned by the handle that allocated it.
 *     Host buffers passed in are read during the call only; host output
 *     buffers are caller-allocated and filled synchronously.
 *   - Lifetime: a handle must outlive every handle created over it — queries
 *     over a graph, route tables over a query, cluster graphs and tables over
 *     a cluster, tables over a cluster graph.  Destroying a handle while
 *     dependants are alive is refused: spf_graph_destroy, spf_query_destroy,
 *     spf_cgraph_destroy and spf_cluster_destroy then return SPF_E_INVALID
 *     and free nothing (the handle stays valid; destroy the dependants, then
 *     call again).  This mirrors the reference's contract that SpfResult
 *     references stay valid until the next topology change
 *     (openr/decision/LinkState.h:269-275).  Destroying NULL is a no-op.
 *   - Threading: a graph and its queries are used from one host thread.  All
 *     work of a graph is enqueued on one HIP stream (spf_graph_set_stream).
 *   - Node ids are 0..V-1 and MUST equal the lexicographic rank of the node
 *     name (the reference breaks Dijkstra ties by name, LinkState.h:488-498).
 *   - There is no CPU fallback: without a usable gfx950 device every call that
 *     needs one returns SPF_E_DEVICE.
 */
#ifndef OPENR_SPF_H
#define OPENR_SPF_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SPF_OK 0
#define SPF_E_INVALID (-1)     /* bad argument / shape */
#define SPF_E_NOMEM (-2)       /* device or host allocation failed */
#define SPF_E_DEVICE (-3)      /* HIP runtime error / no device */
#define SPF_E_UNSUPPORTED (-4) /* shape outside what the kernels handle */

#define SPF_UNREACHABLE UINT64_MAX

/* query flags */
#define SPF_F_UNIT_METRIC 0x1u /* useLinkMetric == false: every hop costs 1 */
#define SPF_F_NEXTHOPS 0x2u    /* compute ECMP next-hop sets */
#define SPF_F_ORDER 0x4u       /* keep the settle order (pathLinks ordering) */

/* Directed CSR of the UP links of one area (Link::isUp, LinkState.cpp:233).
 * Every undirected link contributes two half-edges e (u->v) and rev[e]
 * (v->u) that share link_id.  metric[e] is the metric advertised by the row
 * node u (Link::getMetricFromNode(u)), as the reference's uint64
 * LinkStateMetric (an i32 adjacency metric sign-extended, LinkState.h:22). */
typedef struct spf_graph_desc {
  uint32_t num_nodes;             /* V */
  uint32_t num_edges;             /* E (directed half-edges) */
  const uint32_t* row_ptr;        /* [V+1] */
  const uint32_t* col;            /* [E] other endpoint */
  const uint64_t* metric;         /* [E] metric advertised by the row node */
  const uint32_t* link_id;        /* [E] undirected link id (< num_links) */
  const uint32_t* rev;            /* [E] index of the reverse half-edge */
  const uint8_t* node_overloaded; /* [V] 1 = no transit (isNodeOverloaded) */
  uint32_t num_links;             /* number of distinct link ids */
  int device;                     /* HIP device ordinal */
} spf_graph_desc;

typedef struct spf_graph spf_graph;
typedef struct spf_query spf_query;

/* One batch of single-source SPF runs.  Query i runs from sources[i]; when
 * ignore_offsets is non-NULL query i skips the links
 * ignore_links[ignore_offsets[i] .. ignore_offsets[i+1]) (sorted ascending,
 * the linksToIgnore set of LinkState::runSpf / getKthPaths k>=2). */
typedef struct spf_query_desc {
  uint32_t num_queries;
  const uint32_t* sources;        /* [num_queries] */
  const uint32_t* ignore_offsets; /* [num_queries+1] or NULL */
  const uint32_t* ignore_links;   /* sorted per query, or NULL */
  uint32_t flags;                 /* SPF_F_* */
} spf_query_desc;

/* ---- device ---- */
int spf_device_count(void);
const char* spf_error_string(int status);
const char* spf_last_error_detail(void); /* thread-local text of last error */

/* ---- device memory (tables a host driver owns, e.g. AllSourcesTable) ---- */
#define SPF_COPY_D2H 0
#define SPF_COPY_H2D 1
#define SPF_COPY_D2D 2
int spf_device_alloc(int device, size_t bytes, void** out);
int spf_device_free(int device, void* p);
/* synchronous copy on `device` (SPF_COPY_*) */
int spf_device_memcpy(int device, void* dst, const void* src, size_t bytes, int kind);

/* ---- graph ---- */
int spf_graph_create(const spf_graph_desc* desc, spf_graph** out);
int spf_graph_destroy(spf_graph* g);
/* Replace the per-node transit bits (overload/drain) in place: node
 * overload toggles are the common churn (DecisionBenchmark.cpp:600-626). */
int spf_graph_set_transit(spf_graph* g, const uint8_t* node_overloaded);
/* Patch metrics of existing half-edges in place (metric churn, a7 deltas).
 * A few edges (n * 64 <= E): only their device words are rewritten. */
int spf_graph_patch_metrics(
    spf_graph* g, uint32_t n, const uint32_t* edge_idx, const uint64_t* metric);
/* Take half-edges down (up[i] = 0) or bring them back up (1) with the given
 * metrics, in place: link removal / re-addition (LinkState.cpp:421-434
 * removeLink / addLink; the reference drops its whole memo, :712-715) without
 * a new device graph.  A down half-edge stays at its CSR position as a
 * self-loop of its tail (never relaxed, never tight); the distinct-neighbour
 * lists (spf_graph_nbrs, the next-hop mask bits) are rebuilt over the up
 * half-edges, so next-hop queries stay exact.  A graph changed this way
 * refuses SPF_F_ORDER (SPF_E_UNSUPPORTED) — rebuild it for settle orders.
 * SPF_E_UNSUPPORTED too for 64-bit graphs, metric 0, or metrics the packed
 * edge words cannot hold. */
int spf_graph_set_edges(
    spf_graph* g, uint32_t n, const uint32_t* edge_idx, const uint8_t* up,
    const uint64_t* metric);
/* Rebuild the graph in place from a new CSR of the same node set (a link
 * added or removed: LinkState::updateAdjacencyDatabase's structural changes,
 * LinkState.cpp:421-434 / :564-717) without a new handle: same device and
 * stream, device buffers reused where they fit.  SPF_E_INVALID while a query
 * of the graph is alive or when num_nodes differs.  On any other failure the
 * graph is left unusable: destroy it. */
int spf_graph_update(spf_graph* g, const spf_graph_desc* desc);
/* Work of this graph is enqueued on `stream` (a hipStream_t, NULL = the
 * graph's own stream). */
int spf_graph_set_stream(spf_graph* g, void* stream);
void* spf_graph_get_stream(spf_graph* g);
/* 1 if metric runs on this graph need 64-bit rows and a settle order: metric
 * 0 or sums that may pass 32 bits (the wide plan), or metrics that wrap
 * (negative i32, the literal DijkstraQ replay). */
int spf_graph_needs_exact(const spf_graph* g);
/* Number of distinct neighbours of `node` = bits in its next-hop masks. */
int spf_graph_num_nbrs(const spf_graph* g, uint32_t node);
/* The distinct neighbours of `node`, ascending by id; bit b of a next-hop
 * mask of a query from `node` stands for out[b]. */
int spf_graph_nbrs(const spf_graph* g, uint32_t node, uint32_t* out);

/* ---- queries ---- */
int spf_query_create(spf_graph* g, const spf_query_desc* desc, spf_query** out);
int spf_query_destroy(spf_query* q);
/* Enqueue the batch on the graph stream (asynchronous). */
int spf_query_run(spf_query* q);
/* Wait for the last run to finish. */
int spf_query_sync(spf_query* q);
/* Device time of the last run's kernels (HIP events), milliseconds. */
int spf_query_elapsed_ms(spf_query* q, float* ms);
/* Device time of the last run split per stage: the distance kernel (plus
 * its small setup memset) and the next-hop kernel of two-stage plans
 * (nh_ms = 0 for single-kernel plans). */
int spf_query_stage_ms(spf_query* q, float* dist_ms, float* nh_ms);
/* The same split for each of the last min(n, runs, 64) runs, oldest first
 * (lets a caller time a loop of asynchronous runs per kernel). */
int spf_query_stage_history(
    spf_query* q, uint32_t n, float* dist_ms, float* nh_ms, uint32_t* got);
/* What-if screen of the last run (batches with ignore lists): *screened =
 * queries whose ignored links were all off the baseline's shortest-path DAG
 * (rows copied from the baseline, no SSSP), *has_screen = 0 when the query
 * has no screen (every query ran its own SSSP).  Synchronises the query. */
int spf_query_screened(spf_query* q, uint32_t* screened, uint32_t* has_screen);
/* Name of the plan the last run used ("lds", "dstep", "msbfs+levels", "wide",
 * "exact", ...). */
const char* spf_query_kernel_name(const spf_query* q);
/* The HIP kernels the last run launched (its sub-queries' included, and the
 * trace calls' since that run: spf_query_trace_paths), sorted
 * and comma-separated, as rocprofv3 names them without template arguments;
 * writes at most cap - 1 bytes and a NUL into buf (may be NULL) and returns
 * the full length, or a negative status.  Lets a measurement check that a
 * profile was taken of the same plan. */
int spf_query_kernels(const spf_query* q, char* buf, size_t cap);

/* Distances of query i, one per node; SPF_UNREACHABLE = not reached. */
int spf_query_dist(spf_query* q, uint32_t i, uint64_t* out /*[V]*/);
/* Words per next-hop mask of query i (ceil(nbrs(src)/64), at least 1). */
int spf_query_nh_words(const spf_query* q, uint32_t i);
/* Next-hop masks of query i: out[v*W + w], W = spf_query_nh_words (host
 * layout: u64 words, whatever the device layout). */
int spf_query_nexthops(spf_query* q, uint32_t i, uint64_t* out /*[V*W]*/);
/* Device layout of the next-hop masks (spf_query_device_rows): query i's row
 * holds spf_query_nh_bytes(q, i) bytes per node, node-major, starting
 * spf_query_nh_offset bytes into the block.  Bytes per node = 1, 2 or 4 for
 * a source with at most 8, 16 or 32 distinct neighbours (bit j of that
 * little-endian integer = the j-th neighbour, spf_graph_nbrs order), else
 * 8 * nh_words (u64 words).  Rows start 32-byte aligned. */
#define SPF_NH_BYTES(nbrs) \
  ((nbrs) <= 8u ? 1u : (nbrs) <= 16u ? 2u : (nbrs) <= 32u ? 4u : 8u * (((nbrs) + 63u) / 64u))
int spf_query_nh_bytes(const spf_query* q, uint32_t i);
int spf_query_nh_offset(const spf_query* q, uint32_t i, uint64_t* byte_off);
/* Settle rank of every node for query i (SPF_F_ORDER): the order in which the
 * reference's DijkstraQ extracts nodes; UINT32_MAX = not reached. */
int spf_query_order(spf_query* q, uint32_t i, uint32_t* out /*[V]*/);
/* Settle keys of query i (SPF_F_ORDER on a graph that needs 64-bit rows and
 * whose metrics do not wrap, i.e. the wide plan): node u settles before node v
 * iff (dist[u], key[u]) < (dist[v], key[v]) lexicographically, so a caller
 * compares instead of sorting; SPF_UNREACHABLE = not reached.
 * SPF_E_UNSUPPORTED for the literal-replay plan (use spf_query_order). */
int spf_query_order_keys(spf_query* q, uint32_t i, uint64_t* out /*[V]*/);
/* Device pointers of the result rows (for RCCL gathers): dist rows are
 * uint32 (fast kernels) or uint64 (exact kernel), spf_query_row_stride
 * elements apart (V entries used per row).  Next-hop rows are packed in the
 * byte layout of spf_query_nh_bytes: query i starts at byte
 * sum_{j<i} roundup32(V * nh_bytes(j)); *nh_total_words = the block's size
 * in 8-byte words. */
int spf_query_device_rows(
    spf_query* q, void** dist_rows, uint32_t* dist_elem_bytes,
    void** nh_rows, uint64_t* nh_total_words);
/* Copy distance rows [first, first+count) as uint32 (V entries each,
 * SPF_UNREACHABLE -> 0xFFFFFFFF) into dst, dst_pitch bytes apart: device
 * memory (asynchronous, on the graph stream — e.g. a slice of a tensor an
 * RCCL all-gather then exchanges) or host memory (synchronous).  The
 * all-sources counterpart of reading NodeSpfResult::metric() per node
 * (LinkState.h:203-257).  SPF_E_UNSUPPORTED for 64-bit (exact) rows. */
int spf_query_fetch_rows(
    spf_query* q, uint32_t first, uint32_t count, void* dst, size_t dst_pitch,
    int dst_on_device);
/* Elements between consecutive distance rows (>= V). */
uint32_t spf_query_row_stride(const spf_query* q);
/* Copy the next-hop masks of queries [first, first+count) to host memory in
 * one transfer, back to back: query i occupies V * nh_words(i) words.  The
 * bulk counterpart of spf_query_nexthops for batches whose every row the
 * caller materialises (NodeSpfResult::nextHops, LinkState.h:203-257). */
int spf_query_fetch_nexthops(
    spf_query* q, uint32_t first, uint32_t count, uint64_t* dst);
/* Both of the above into host memory with ONE synchronisation: the uint32
 * distance rows of queries [first, first+count) into rows (row_pitch bytes
 * apart; NULL skips them) and their next-hop masks into masks (the layout of
 * spf_query_fetch_nexthops; NULL skips them).  Small batches (a RouteDb
 * build's few sources: the node and its LFA neighbours, LinkState.cpp:
 * 1220-1260's per-source getSpfResult) go through a pinned staging buffer,
 * so the two transfers cost one round trip; larger ones take the two calls
 * above.  Same errors as those. */
int spf_query_fetch_host(
    spf_query* q, uint32_t first, uint32_t count, uint32_t* rows, size_t row_pitch,
    uint64_t* masks);
/* getKthPaths' trace loop on the device (LinkState.cpp:776-786 over
 * traceOnePath, :398-419): for queries [first, first+count), repeated
 * traceOnePath from the query's source to dests[i] over the query's own
 * distance row and ignore list, sharing one visited-link set, until a trace
 * fails — the KSP2 second passes of a RouteDb build (SpfSolver
 * selectKsp2 -> getKthPaths(src, dst, 2)) without their rows leaving HBM.
 * Same paths in the same order as the reference (pathLinks order: tail
 * settle rank, then linksFromNode order).  Per query i (host arrays):
 * path_count[i] paths and link_count[i] links in them, or path_count[i] =
 * SPF_TRACE_OVERFLOW when the visited set, the recursion stack or the
 * 1,024-link output of the query was exceeded (trace that query on the
 * host).  The paths stay on the device until spf_query_trace_fetch.
 * SPF_E_UNSUPPORTED for 64-bit (exact) rows. */
#define SPF_TRACE_OVERFLOW 0xFFFFFFFFu
int spf_query_trace_paths(
    spf_query* q, uint32_t first, uint32_t count, const uint32_t* dests, uint32_t* path_count,
    uint32_t* link_count);
/* The last trace's paths, packed in query order (overflowed queries
 * skipped): links[] holds Σ link_count link ids, each path src -> dst;
 * ends[] holds Σ path_count end offsets, each relative to its query's first
 * link. */
int spf_query_trace_fetch(spf_query* q, uint32_t* links, uint32_t* ends);

/* ---- incremental all-sources tables ----
 * The reference drops every memoized SpfResult on any topology change
 * (LinkState.cpp:510-511, 712-715, 728-729, driven by the LinkStateChange
 * of updateAdjacencyDatabase :564-717) and recomputes each source on
 * demand.  Here a resident table of distance rows is repaired instead: the
 * change between two graphs over the same node ids is listed as directed
 * edge deltas, a screen kernel finds the sources whose shortest-path DAG a
 * delta can touch, and only those are recomputed and scattered back. */

#define SPF_DELTA_REMOVED 1u /* usable before the change, not after */
#define SPF_DELTA_ADDED 2u   /* usable after the change, not before */
#define SPF_SCOPE_ALL 0u       /* the tail relaxes it for every source */
#define SPF_SCOPE_TAIL_ONLY 1u /* only for source == tail (tail overloaded) */
#define SPF_SCOPE_NOT_TAIL 2u  /* every source but the tail (transit flip) */

typedef struct spf_edge_delta {
  uint32_t tail, head; /* node ids shared by both graphs */
  uint64_t metric;     /* metric in the graph where the edge is usable */
  uint32_t kind;       /* SPF_DELTA_* */
  uint32_t scope;      /* SPF_SCOPE_* */
} spf_edge_delta;

/* Host-only (no device): the directed edge deltas turning `before` into
 * `after`, which must have the same num_nodes (ids = name ranks).  Per tail
 * node: half-edges (head, metric) only in `before` are REMOVED, only in
 * `after` ADDED (multiset difference, so parallel links count), and when the
 * tail's overload bit flipped its unchanged half-edges are REMOVED / ADDED
 * with SPF_SCOPE_NOT_TAIL (an overloaded node still expands as the source,
 * LinkState.cpp:829-836).  Writes min(n, cap) deltas, *n_out = n. */
int spf_graph_diff(
    const spf_graph_desc* before, const spf_graph_desc* after,
    spf_edge_delta* out, uint32_t cap, uint32_t* n_out);
/* Screen the uint32 distance rows of `num_rows` sources against the deltas
 * (kernel spf_table_screen_kernel on the graph stream): row i is affected
 * iff some delta (u, v, w) in scope of sources[i] with d[u] reached has
 * d[u] + w == d[v] (REMOVED: a tight edge of the DAG disappears) or
 * d[u] + w <= d[v] (ADDED: a new tight or shorter edge).  Unaffected rows
 * keep their distances and next-hop sets exactly (both are defined by the
 * tight usable edges alone).  `rows` is device memory, `pitch` elements
 * apart; `sources` and `affected` (one byte per row) are host memory. */
int spf_table_screen(
    spf_graph* g, const uint32_t* rows, size_t pitch, uint32_t num_rows,
    const uint32_t* sources, const spf_edge_delta* deltas, uint32_t n_deltas,
    uint8_t* affected);
/* Repair rows in place instead of recomputing them: rows[row_idx[i]]
 * (device table, pitch elements apart) hold source sources[i]'s distances
 * on the graph before a change, `g` is the graph after it and `deltas` =
 * spf_graph_diff(before, after).  Per row (spf_dstep_kernel, seeded mode):
 * nodes whose every shortest path may have used a REMOVED edge are found
 * (tight-edge closure from the removed tight edges) and those no longer
 * supported by a surviving tight path are reset to unreached; every value is
 * then an upper bound, and label-correcting delta-stepping from the reset
 * boundary and the tails of the ADDED edges lowers the row to g's distances
 * exactly, touching only the region that changed.  SPF_E_UNSUPPORTED when
 * the bucket image does not fit LDS or g needs the exact kernel (then
 * recompute the rows).  Synchronous. */
int spf_table_repair(
    spf_graph* g, uint32_t* rows, size_t pitch, uint32_t num_rows,
    const uint32_t* sources, const uint32_t* row_idx,
    const spf_edge_delta* deltas, uint32_t n_deltas);
/* Next-hop masks of `num` sources straight from a device table of uint32
 * distance rows (rows[row_of[x]] = node x's row, pitch elements apart): the
 * rule of the all-sources plans (spf_nh_rows_kernel) — bit b of NH(s, v) set
 * iff s's b-th distinct neighbour f has w(s, f) + d(f, v) == d(s, v), f
 * transit or f == v (LinkState.cpp:846-870).  Every source and every
 * neighbour of a source needs a row (row_of[x] >= 0).  Source i's V * W_i
 * words go to masks + mask_off[i] (device), W_i = ceil(nbrs(s_i) / 64) (at
 * least 1).  The repaired rows of spf_table_repair get their next hops back
 * this way.  Synchronous. */
int spf_table_nexthops(
    spf_graph* g, const uint32_t* rows, size_t pitch, const int32_t* row_of, uint32_t num,
    const uint32_t* sources, uint64_t* masks, const uint64_t* mask_off);
/* Copy distance row i of the query (uint32, as spf_query_fetch_rows) to
 * row dst_rows[i] of the device table `table` (pitch bytes apart), for every
 * query, in one kernel on the graph stream (asynchronous). */
int spf_query_scatter_rows(
    spf_query* q, const uint32_t* dst_rows, void* table, size_t pitch);

/* ---- all-nodes unicast route tables ----
 * The RouteDb of EVERY node of an area from one all-sources query, on the
 * device: for query row i (node s) and prefix p, Open/R's ECMP selection
 * (SpfSolverImpl::selectEcmpOpenr, Decision.cpp:668-712 with
 * getBestAnnouncingNodes :544-630, maybeFilterDrainedNodes :651-666,
 * getNextHopsWithMetric :1093-1179, getNextHopsThrift :1181-1271; one area,
 * LFA off, not per destination — the reference runs it per node in
 * buildRouteDb :291-542).  Output per (i, p): metric (UINT32_MAX = no route:
 * s announces p or no announcer is reachable), best (the smallest reachable
 * announcer: bestPrefixEntry's node) and a link mask over s's up links (bit
 * j = the j-th half-edge of s's CSR row, i.e. linksFromNode order): the
 * next hops of the route, each with metric `metric`. */
typedef struct spf_route_table spf_route_table;
/* `q` must be a metric query (no SPF_F_UNIT_METRIC) with SPF_F_NEXTHOPS and
 * no ignore lists; prefix p is announced by announcers[ann_offsets[p] ..
 * ann_offsets[p+1]) (node ids). */
int spf_route_table_create(
    spf_query* q, uint32_t num_prefixes, const uint32_t* ann_offsets,
    const uint32_t* announcers, spf_route_table** out);
/* flags of spf_route_table_create_ex */
#define SPF_RT_LFA 0x1u /* loop-free alternates (computeLfaPaths_, Decision.cpp:1146-1175):
                           every up link to a shortest-path or LFA next-hop node, each with
                           its own metric (spf_route_table_fetch_link_metrics); needs every
                           neighbour's row in the query (all sources) */
int spf_route_table_create_ex(
    spf_query* q, uint32_t num_prefixes, const uint32_t* ann_offsets,
    const uint32_t* announcers, uint32_t flags, spf_route_table** out);
int spf_route_table_destroy(spf_route_table* t);
/* Enqueue spf_route_table_kernel after the query's last run (asynchronous,
 * graph stream). */
int spf_route_table_run(spf_route_table* t);
int spf_route_table_elapsed_ms(spf_route_table* t, float* ms);
/* Link-mask words per prefix of row i (ceil(up links of s / 64)). */
int spf_route_table_link_words(const spf_route_table* t, uint32_t i);
/* Row i to host: metric[P], best[P], links[P * link_words(i)]. */
int spf_route_table_fetch(
    spf_route_table* t, uint32_t i, uint32_t* metric, uint32_t* best, uint64_t* links);

/* SPF_RT_LFA tables: the metric of every link of row i's source per prefix,
 * out[p * deg + j] (deg = up links of the source in CSR order), set where bit
 * j of the cell's link mask is; the diff compares these too. */
int spf_route_table_fetch_link_metrics(spf_route_table* t, uint32_t i, uint32_t* out);

/* Network-wide route delta: compare two tables built
 * over graphs with the same CSR layout (e.g. before and after an overload or
 * metric change) and the same prefixes; cell (i, p) changed iff its metric,
 * best announcer or link mask differs — getRouteDelta's (Decision.cpp:47-85)
 * unicast updates and deletes for every node at once.  changed[i] = changed
 * prefixes of row i (host [num rows]); the per-row bitmap is kept in `newer`
 * (spf_route_table_changed).  SPF_E_UNSUPPORTED if the layouts differ. */
int spf_route_table_diff(spf_route_table* older, spf_route_table* newer, uint32_t* changed);
/* Changed-prefix bitmap of row i from the last diff: bits[ceil(P/64)]. */
int spf_route_table_changed(spf_route_table* t, uint32_t i, uint64_t* bits);

/* ---- multi-GPU all-sources tables ----
 * The reference computes every SpfResult on the one Decision thread
 * (getSpfResult, LinkState.cpp:791-801; all sources = Decision::
 * getDecisionRouteDb per node, Decision.cpp:1437-1462).  Here one call fans
 * an all-sources batch out over devices: sources are split in contiguous
 * blocks (rank r of `world`: n / world sources, the first n % world ranks one
 * more), each block runs as one spf_query on its device, and the rows are
 * exchanged with an in-place RCCL all-gather over xGMI into equal-sized rank
 * slots.  A cluster is either every device of this process
 * (spf_cluster_create_local: ncclCommInitAll) or one rank of a
 * one-process-per-GPU job (spf_cluster_create_rank: ncclCommInitRank over an
 * id from spf_cluster_unique_id that the caller hands to every rank). */
typedef struct spf_cluster spf_cluster;
typedef struct spf_table spf_table;

#define SPF_CLUSTER_ID_BYTES 128
#define SPF_T_GATHER_ROWS 0x100u     /* all-gather the uint32 distance rows */
#define SPF_T_GATHER_NEXTHOPS 0x200u /* all-gather the packed next-hop masks */

int spf_cluster_unique_id(uint8_t* id /*[SPF_CLUSTER_ID_BYTES]*/);
int spf_cluster_create_local(uint32_t num_devices, const int* devices, spf_cluster** out);
int spf_cluster_create_rank(
    uint32_t world, uint32_t rank, const uint8_t* id, int device, spf_cluster** out);
int spf_cluster_destroy(spf_cluster* c);
int spf_cluster_info(
    const spf_cluster* c, uint32_t* world, uint32_t* first_rank, uint32_t* local_devices);
const char* spf_cluster_last_error(void);

/* Host only: the block boundaries (block_first[world + 1]) and, when
 * mask_off is non-NULL, the BYTE offset of every source's next-hop masks in
 * the gathered mask buffer (rank slots of *mask_cap bytes; within a slot the
 * block's sources back to back, V * nh_bytes[i] bytes each rounded up to 32:
 * the device layout of spf_query_nh_bytes / SPF_NH_BYTES).  nh_bytes may be
 * NULL (8 bytes = one word each). */
int spf_table_layout(
    uint32_t num_sources, uint32_t world, uint32_t num_nodes, const uint32_t* nh_bytes,
    uint64_t* block_first, uint64_t* mask_off, uint64_t* mask_cap);
/* One graph per local device from `desc` (desc->device ignored), the local
 * ranks' source blocks as queries.  flags: SPF_F_UNIT_METRIC,
 * SPF_F_NEXTHOPS, SPF_T_GATHER_ROWS, SPF_T_GATHER_NEXTHOPS. */
int spf_table_create(
    spf_cluster* c, const spf_graph_desc* desc, uint32_t num_sources, const uint32_t* sources,
    uint32_t flags, spf_table** out);
int spf_table_destroy(spf_table* t);
/* Enqueue every local block and the all-gathers (asynchronous). */
int spf_table_run(spf_table* t);
int spf_table_sync(spf_table* t);
/* Device time of the last run, max over local devices: the SPF batch (plus
 * the copy into the own slot) and the RCCL exchange. */
int spf_table_elapsed_ms(spf_table* t, float* compute_ms, float* gather_ms);
int spf_table_block(const spf_table* t, uint32_t rank, uint32_t* first, uint32_t* count);
int spf_table_nh_words(const spf_table* t, uint32_t i);
/* Device bytes per node of source i's masks in the gathered buffer. */
int spf_table_nh_bytes(const spf_table* t, uint32_t i);
/* Rows / masks of sources [first, first+count) to host memory (from the
 * local owner, or from the gathered copy; SPF_E_UNSUPPORTED for another
 * rank's rows without the gather flag).  Masks back to back, V * nh_words(i)
 * words each. */
int spf_table_fetch_rows(spf_table* t, uint32_t first, uint32_t count, uint32_t* dst);
int spf_table_fetch_nexthops(spf_table* t, uint32_t first, uint32_t count, uint64_t* dst);
/* spf_query_trace_paths over every local block of the table (each block on
 * its device, concurrently); dests and the counts are indexed by table
 * query.  Other ranks' blocks are not traced (their counts are 0).  Then
 * spf_table_trace_fetch packs the local blocks' paths in table-query order,
 * as spf_query_trace_fetch does. */
int spf_table_trace_paths(
    spf_table* t, const uint32_t* dests, uint32_t* path_count, uint32_t* link_count);
int spf_table_trace_fetch(spf_table* t, uint32_t* links, uint32_t* ends);
/* Gathered buffers on local device `local`: rows [world * cap][V] uint32
 * (cap = ceil(n / world)), masks [world * mask_cap] bytes in the layout of
 * spf_table_layout; NULL when that gather is off. */
int spf_table_device_buffers(
    spf_table* t, uint32_t local, void** rows, void** masks, uint64_t* mask_cap_bytes);
int spf_table_kernel_name(spf_table* t, uint32_t local, const char** name);

/* ---- persistent cluster graphs + query tables ----
 * One spf_graph per local device of a cluster, created once per area and
 * topology and kept across batches (the host LinkState patches it with the
 * same overload / metric churn as its single-device graph), instead of one
 * graph upload per device per table.  Over it, spf_table_create_q shards ANY
 * query batch -- with per-query ignore lists -- over the ranks in contiguous
 * blocks: KSP2 second passes by destination (LinkState::getKthPaths k = 2,
 * runSpf(src, true, linksToIgnore) at LinkState.cpp:776-777), what-if by
 * failed link (runSpf with linksToIgnore, LinkState.cpp:842-847), LFA by
 * neighbour (getSpfResult per neighbour, Decision.cpp:1145-1174). */
typedef struct spf_cgraph spf_cgraph;
int spf_cgraph_create(spf_cluster* c, const spf_graph_desc* desc, spf_cgraph** out);
int spf_cgraph_destroy(spf_cgraph* g);
int spf_cgraph_set_transit(spf_cgraph* g, const uint8_t* node_overloaded);
int spf_cgraph_patch_metrics(
    spf_cgraph* g, uint32_t n, const uint32_t* edge_idx, const uint64_t* metric);
/* The graph of local device `local` (NULL if out of range), e.g. for
 * spf_graph_num_nbrs / spf_graph_nbrs. */
spf_graph* spf_cgraph_device_graph(spf_cgraph* g, uint32_t local);
/* A table over `g` from a full query description: desc->sources /
 * ignore_offsets / ignore_links as in spf_query_create (offsets of the whole
 * batch; each rank's block gets its slice), desc->flags SPF_F_UNIT_METRIC /
 * SPF_F_NEXTHOPS, plus the SPF_T_GATHER_* bits in `flags`.  The table
 * borrows the graphs (destroy the table before the cgraph).  Rows of 64-bit
 * plans (spf_table_fetch_rows -> SPF_E_UNSUPPORTED) are left to the caller's
 * single-device path. */
int spf_table_create_q(
    spf_cgraph* g, const spf_query_desc* desc, uint32_t flags, spf_table** out);

#ifdef __cplusplus
}
#endif

#endif /* OPENR_SPF_H */
