// spf_cluster.hip — multi-GPU all-sources tables inside the C ABI
// (SURVEY.md §8(b) "the multi-GPU fan-out happens inside the call", §8(e)).
//
// Open/R's Decision is one thread in one process (Decision.cpp:1771-1814), so
// the fan-out is first a single-process one: spf_cluster_create_local builds
// one RCCL communicator per local device (ncclCommInitAll) and a table keeps
// one spf_graph + one spf_query per device.  A job launched one process per
// GPU (the benchmark's torchrun mode) joins the same machinery with
// spf_cluster_create_rank (ncclCommInitRank over an id the caller
// distributes).  Sources are sharded in contiguous blocks (block r of n
// sources over `world` ranks: base = n / world, the first n % world ranks one
// more), every block runs as one batch on its device, and the one exchange
// step is an in-place ncclAllGather over xGMI of the uint32 distance rows
// (SPF_T_GATHER_ROWS) and of the packed next-hop masks (SPF_T_GATHER_NEXTHOPS)
// into equal-sized rank slots.  Without the gather flags the rows stay on
// their owner device (a RouteDb needs only its own row; the host fetches
// blocks directly).
//
// This layer composes the single-device ABI (spf_graph_* / spf_query_*) with
// RCCL; it launches no kernels of its own.

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstring>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "openr_spf.h"

#include <rocprofiler-sdk-roctx/roctx.h>

namespace {

struct ClusterRange {
  explicit ClusterRange(const char* name) { roctxRangePushA(name); }
  ~ClusterRange() { roctxRangePop(); }
  ClusterRange(const ClusterRange&) = delete;
  ClusterRange& operator=(const ClusterRange&) = delete;
};
#define SPF_ABI_RANGE_CLUSTER(name) ClusterRange spf_cluster_range_(name)

thread_local std::string g_cluster_err;

int cfail(int status, const std::string& what) {
  g_cluster_err = what;
  return status;
}

#define CL_HIP(expr)                                                        \
  do {                                                                      \
    hipError_t e_ = (expr);                                                 \
    if (e_ != hipSuccess) {                                                 \
      return cfail(SPF_E_DEVICE, std::string(#expr ": ") + hipGetErrorString(e_)); \
    }                                                                       \
  } while (0)

#define CL_NCCL(expr)                                                        \
  do {                                                                       \
    ncclResult_t r_ = (expr);                                                \
    if (r_ != ncclSuccess) {                                                 \
      return cfail(SPF_E_DEVICE, std::string(#expr ": ") + ncclGetErrorString(r_)); \
    }                                                                        \
  } while (0)

#define CL_TRY(expr)        \
  do {                      \
    int s_ = (expr);        \
    if (s_ != SPF_OK) {     \
      return s_;            \
    }                       \
  } while (0)

uint64_t roundup32(uint64_t x) { return (x + 31) & ~31ull; }

} // namespace

// spf_device.hip (same library, not exported)
extern "C" uint32_t spf_graph_live_queries_(const spf_graph* g);

struct spf_cluster {
  uint32_t world = 1;
  uint32_t first_rank = 0; // global rank of local device 0
  std::vector<int> devices;
  std::vector<ncclComm_t> comms;
  // live spf_cgraph / spf_table handles over this cluster: they use its
  // devices and communicators, so spf_cluster_destroy refuses while any lives
  std::atomic<uint32_t> users{0};
};

struct spf_cgraph {
  spf_cluster* c = nullptr;
  uint32_t V = 0;
  std::vector<spf_graph*> g; // one per local device, c->devices order
  // live spf_table handles borrowing these graphs (spf_cgraph_destroy refuses)
  std::atomic<uint32_t> tables{0};
};

struct spf_table {
  spf_cluster* c = nullptr;
  spf_cgraph* cg = nullptr; // the borrowed graphs' owner (spf_table_create_q)
  bool borrowed = false; // graphs belong to an spf_cgraph (not destroyed here)
  uint32_t V = 0, n = 0, flags = 0, cap = 0;
  std::vector<uint32_t> sources;
  std::vector<uint32_t> words;       // next-hop words per source (host layout)
  std::vector<uint32_t> nbytes;      // mask bytes per node per source (device layout)
  std::vector<uint64_t> block_first; // [world + 1] source index boundaries
  std::vector<uint64_t> mask_off;    // byte offset of each source in the gathered masks
  uint64_t mask_cap = 0;             // bytes per rank slot of the gathered masks (x32)
  struct Local {
    int device = 0;
    uint32_t rank = 0;
    spf_graph* g = nullptr;
    spf_query* q = nullptr;
    std::vector<uint32_t> ign_off; // this block's ignore offsets, rebased to 0
    uint32_t* rows = nullptr;  // gathered rows [world * cap][V] (GATHER_ROWS)
    uint8_t* masks = nullptr; // gathered masks [world * mask_cap bytes] (GATHER_NEXTHOPS)
    hipEvent_t e0 = nullptr, e1 = nullptr, e2 = nullptr;
  };
  std::vector<Local> local;
  bool ran = false;
  // spf_table_trace_paths: packed offsets of each local block's paths
  bool traced = false;
  std::vector<uint64_t> trace_link_base, trace_path_base;
};

extern "C" {

const char* spf_cluster_last_error(void) { return g_cluster_err.c_str(); }

int spf_table_layout(
    uint32_t num_sources, uint32_t world, uint32_t num_nodes, const uint32_t* nh_bytes,
    uint64_t* block_first, uint64_t* mask_off, uint64_t* mask_cap) {
  if (world == 0 || !block_first) {
    return cfail(SPF_E_INVALID, "spf_table_layout: world == 0 or no block_first");
  }
  const uint32_t base = num_sources / world, extra = num_sources % world;
  for (uint32_t r = 0; r <= world; ++r) {
    block_first[r] = (uint64_t)r * base + std::min(r, extra);
  }
  uint64_t cap = 0;
  for (uint32_t r = 0; r < world; ++r) {
    uint64_t bytes = 0;
    for (uint64_t i = block_first[r]; i < block_first[r + 1]; ++i) {
      if (mask_off) {
        mask_off[i] = bytes; // within the slot; the slot base is added below
      }
      // a query's row: V * nh_bytes rounded up to 32 bytes (spf_query_nh_offset)
      bytes += roundup32((uint64_t)num_nodes * (nh_bytes ? nh_bytes[i] : 8u));
    }
    cap = std::max(cap, bytes);
  }
  if (mask_off) {
    for (uint32_t r = 0; r < world; ++r) {
      for (uint64_t i = block_first[r]; i < block_first[r + 1]; ++i) {
        mask_off[i] += (uint64_t)r * cap;
      }
    }
  }
  if (mask_cap) {
    *mask_cap = cap;
  }
  return SPF_OK;
}

int spf_cluster_unique_id(uint8_t* id) {
  if (!id) {
    return cfail(SPF_E_INVALID, "spf_cluster_unique_id: null id");
  }
  ncclUniqueId u;
  CL_NCCL(ncclGetUniqueId(&u));
  std::memcpy(id, u.internal, NCCL_UNIQUE_ID_BYTES);
  return SPF_OK;
}

int spf_cluster_create_local(uint32_t num_devices, const int* devices, spf_cluster** out) {
  SPF_ABI_RANGE_CLUSTER("spf_cluster_create_local");
  if (!out || num_devices == 0 || !devices) {
    return cfail(SPF_E_INVALID, "spf_cluster_create_local: no devices");
  }
  int have = 0;
  if (hipGetDeviceCount(&have) != hipSuccess || have <= 0) {
    return cfail(SPF_E_DEVICE, "spf_cluster_create_local: no HIP device");
  }
  for (uint32_t i = 0; i < num_devices; ++i) {
    if (devices[i] < 0 || devices[i] >= have) {
      return cfail(SPF_E_INVALID, "spf_cluster_create_local: device out of range");
    }
  }
  auto c = std::make_unique<spf_cluster>();
  c->world = num_devices;
  c->devices.assign(devices, devices + num_devices);
  c->comms.resize(num_devices);
  CL_NCCL(ncclCommInitAll(c->comms.data(), (int)num_devices, devices));
  *out = c.release();
  return SPF_OK;
}

int spf_cluster_create_rank(
    uint32_t world, uint32_t rank, const uint8_t* id, int device, spf_cluster** out) {
  SPF_ABI_RANGE_CLUSTER("spf_cluster_create_rank");
  if (!out || !id || world == 0 || rank >= world) {
    return cfail(SPF_E_INVALID, "spf_cluster_create_rank: bad rank / world / id");
  }
  CL_HIP(hipSetDevice(device));
  auto c = std::make_unique<spf_cluster>();
  c->world = world;
  c->first_rank = rank;
  c->devices = {device};
  c->comms.resize(1);
  ncclUniqueId u;
  std::memcpy(u.internal, id, NCCL_UNIQUE_ID_BYTES);
  CL_NCCL(ncclCommInitRank(&c->comms[0], (int)world, u, (int)rank));
  *out = c.release();
  return SPF_OK;
}

int spf_cluster_destroy(spf_cluster* c) {
  if (!c) {
    return SPF_OK;
  }
  if (const uint32_t n = c->users.load(std::memory_order_relaxed)) {
    return cfail(SPF_E_INVALID, "spf_cluster_destroy: " + std::to_string(n) +
                                    " live tables / cluster graphs (destroy them first)");
  }
  for (auto comm : c->comms) {
    if (comm) {
      (void)ncclCommDestroy(comm);
    }
  }
  delete c;
  return SPF_OK;
}

int spf_cluster_info(
    const spf_cluster* c, uint32_t* world, uint32_t* first_rank, uint32_t* local_devices) {
  if (!c) {
    return cfail(SPF_E_INVALID, "spf_cluster_info: null cluster");
  }
  if (world) {
    *world = c->world;
  }
  if (first_rank) {
    *first_rank = c->first_rank;
  }
  if (local_devices) {
    *local_devices = (uint32_t)c->devices.size();
  }
  return SPF_OK;
}

static void free_table(spf_table* t) {
  if (t->c) {
    t->c->users.fetch_sub(1, std::memory_order_relaxed);
  }
  if (t->cg) {
    t->cg->tables.fetch_sub(1, std::memory_order_relaxed);
  }
  for (auto& L : t->local) {
    (void)hipSetDevice(L.device);
    if (L.q) {
      spf_query_destroy(L.q);
    }
    if (L.g && !t->borrowed) {
      spf_graph_destroy(L.g);
    }
    if (L.rows) {
      (void)hipFree(L.rows);
    }
    if (L.masks) {
      (void)hipFree(L.masks);
    }
    for (hipEvent_t e : {L.e0, L.e1, L.e2}) {
      if (e) {
        (void)hipEventDestroy(e);
      }
    }
  }
  delete t;
}

int spf_table_destroy(spf_table* t) {
  if (t) {
    free_table(t);
  }
  return SPF_OK;
}

// ---- persistent per-device graphs (spf_cgraph) ----

int spf_cgraph_create(spf_cluster* c, const spf_graph_desc* desc, spf_cgraph** out) {
  SPF_ABI_RANGE_CLUSTER("spf_cgraph_create");
  if (!c || !desc || !out) {
    return cfail(SPF_E_INVALID, "spf_cgraph_create: null argument");
  }
  auto cg = std::make_unique<spf_cgraph>();
  cg->c = c;
  c->users.fetch_add(1, std::memory_order_relaxed); // spf_cgraph_destroy gives it back
  cg->V = desc->num_nodes;
  for (int dev : c->devices) {
    spf_graph_desc gd = *desc;
    gd.device = dev;
    spf_graph* g = nullptr;
    const int s = spf_graph_create(&gd, &g);
    if (s != SPF_OK) {
      spf_cgraph_destroy(cg.release());
      return s;
    }
    cg->g.push_back(g);
  }
  *out = cg.release();
  return SPF_OK;
}

int spf_cgraph_destroy(spf_cgraph* cg) {
  if (!cg) {
    return SPF_OK;
  }
  if (const uint32_t n = cg->tables.load(std::memory_order_relaxed)) {
    return cfail(SPF_E_INVALID, "spf_cgraph_destroy: " + std::to_string(n) +
                                    " live tables over this graph (destroy them first)");
  }
  for (spf_graph* g : cg->g) {
    if (const uint32_t n = spf_graph_live_queries_(g)) {
      return cfail(SPF_E_INVALID, "spf_cgraph_destroy: " + std::to_string(n) +
                                      " live queries on a device graph (destroy them first)");
    }
  }
  for (spf_graph* g : cg->g) {
    spf_graph_destroy(g);
  }
  if (cg->c) {
    cg->c->users.fetch_sub(1, std::memory_order_relaxed);
  }
  delete cg;
  return SPF_OK;
}

int spf_cgraph_set_transit(spf_cgraph* cg, const uint8_t* node_overloaded) {
  if (!cg) {
    return cfail(SPF_E_INVALID, "spf_cgraph_set_transit: null graph");
  }
  for (spf_graph* g : cg->g) {
    CL_TRY(spf_graph_set_transit(g, node_overloaded));
  }
  return SPF_OK;
}

int spf_cgraph_patch_metrics(
    spf_cgraph* cg, uint32_t n, const uint32_t* edge_idx, const uint64_t* metric) {
  if (!cg) {
    return cfail(SPF_E_INVALID, "spf_cgraph_patch_metrics: null graph");
  }
  for (spf_graph* g : cg->g) {
    CL_TRY(spf_graph_patch_metrics(g, n, edge_idx, metric));
  }
  return SPF_OK;
}

spf_graph* spf_cgraph_device_graph(spf_cgraph* cg, uint32_t local) {
  return cg && local < cg->g.size() ? cg->g[local] : nullptr;
}

// The table of queries qd over per-device graphs `graphs` (local device
// order): contiguous query blocks per rank, each block with its own slice of
// the ignore lists (rebased offsets), one spf_query per local block.
static int table_init(
    spf_table* t, spf_cluster* c, const std::vector<spf_graph*>& graphs, uint32_t V,
    const spf_query_desc* qd_all, uint32_t flags) {
  const uint32_t num_sources = qd_all->num_queries;
  const uint32_t* sources = qd_all->sources;
  const uint32_t qflags = flags & (SPF_F_UNIT_METRIC | SPF_F_NEXTHOPS);
  if ((flags & SPF_T_GATHER_NEXTHOPS) && !(flags & SPF_F_NEXTHOPS)) {
    return cfail(SPF_E_INVALID, "spf_table_create: GATHER_NEXTHOPS needs SPF_F_NEXTHOPS");
  }
  if (num_sources && !sources) {
    return cfail(SPF_E_INVALID, "spf_table_create: null sources");
  }
  for (uint32_t i = 0; i < num_sources; ++i) {
    if (sources[i] >= V) {
      return cfail(SPF_E_INVALID, "spf_table_create: source out of range");
    }
  }
  const uint32_t* ioff = qd_all->ignore_offsets;
  if (ioff && (!qd_all->ignore_links && ioff[num_sources] > 0)) {
    return cfail(SPF_E_INVALID, "spf_table_create: ignore offsets without links");
  }
  if (ioff && ioff[0] != 0) {
    return cfail(SPF_E_INVALID, "spf_table_create: ignore_offsets[0] != 0");
  }
  t->c = c;
  c->users.fetch_add(1, std::memory_order_relaxed); // free_table gives it back
  t->V = V;
  t->n = num_sources;
  t->flags = flags;
  t->sources.assign(sources, sources + num_sources);
  t->cap = (num_sources + c->world - 1) / c->world;
  t->block_first.resize(c->world + 1);
  t->local.resize(c->devices.size());
  for (size_t d = 0; d < c->devices.size(); ++d) {
    t->local[d].device = c->devices[d];
    t->local[d].rank = c->first_rank + (uint32_t)d;
    t->local[d].g = graphs[d];
  }
  // next-hop words of every source (the gathered mask layout needs all of
  // them; distinct neighbour counts come from the graph, any device)
  t->words.assign(num_sources, 1);
  t->nbytes.assign(num_sources, 8);
  if (qflags & SPF_F_NEXTHOPS) {
    for (uint32_t i = 0; i < num_sources; ++i) {
      const int nb = spf_graph_num_nbrs(t->local[0].g, sources[i]);
      if (nb < 0) {
        return nb;
      }
      t->words[i] = std::max<uint32_t>(1, ((uint32_t)nb + 63) / 64);
      t->nbytes[i] = SPF_NH_BYTES((uint32_t)nb);
    }
  }
  t->mask_off.resize(num_sources);
  CL_TRY(spf_table_layout(num_sources, c->world, V, t->nbytes.data(), t->block_first.data(),
                          t->mask_off.data(), &t->mask_cap));
  for (auto& L : t->local) {
    CL_HIP(hipSetDevice(L.device));
    const uint64_t first = t->block_first[L.rank], count = t->block_first[L.rank + 1] - first;
    if (count) {
      spf_query_desc qd{};
      qd.num_queries = (uint32_t)count;
      qd.sources = t->sources.data() + first;
      qd.flags = qflags;
      if (ioff) {
        L.ign_off.resize(count + 1);
        for (uint64_t i = 0; i <= count; ++i) {
          L.ign_off[i] = ioff[first + i] - ioff[first];
        }
        qd.ignore_offsets = L.ign_off.data();
        qd.ignore_links = qd_all->ignore_links + ioff[first];
      }
      CL_TRY(spf_query_create(L.g, &qd, &L.q));
      if (qflags & SPF_F_NEXTHOPS) {
        // the block's masks land in its slot as one copy: same layout
        for (uint64_t i = 0; i < count; ++i) {
          uint64_t o = 0;
          CL_TRY(spf_query_nh_offset(L.q, (uint32_t)i, &o));
          if (o + (uint64_t)L.rank * t->mask_cap != t->mask_off[first + i] ||
              (uint32_t)spf_query_nh_bytes(L.q, (uint32_t)i) != t->nbytes[first + i]) {
            return cfail(SPF_E_INVALID, "spf_table_create: query mask layout differs from the slot");
          }
        }
      }
    }
    if (flags & SPF_T_GATHER_ROWS) {
      CL_HIP(hipMalloc((void**)&L.rows, (size_t)c->world * t->cap * t->V * sizeof(uint32_t)));
    }
    if (flags & SPF_T_GATHER_NEXTHOPS) {
      CL_HIP(hipMalloc((void**)&L.masks, (size_t)c->world * t->mask_cap));
    }
    CL_HIP(hipEventCreate(&L.e0));
    CL_HIP(hipEventCreate(&L.e1));
    CL_HIP(hipEventCreate(&L.e2));
  }
  return SPF_OK;
}

int spf_table_create(
    spf_cluster* c, const spf_graph_desc* desc, uint32_t num_sources, const uint32_t* sources,
    uint32_t flags, spf_table** out) {
  SPF_ABI_RANGE_CLUSTER("spf_table_create");
  if (!c || !desc || !out || (num_sources && !sources)) {
    return cfail(SPF_E_INVALID, "spf_table_create: null argument");
  }
  std::unique_ptr<spf_table, void (*)(spf_table*)> t(new spf_table, free_table);
  std::vector<spf_graph*> graphs;
  for (int dev : c->devices) {
    spf_graph_desc gd = *desc;
    gd.device = dev;
    spf_graph* g = nullptr;
    const int s = spf_graph_create(&gd, &g);
    if (s != SPF_OK) {
      for (spf_graph* x : graphs) {
        spf_graph_destroy(x);
      }
      return s;
    }
    graphs.push_back(g);
  }
  // the table owns these graphs from here on (free_table destroys them)
  t->local.resize(graphs.size());
  for (size_t d = 0; d < graphs.size(); ++d) {
    t->local[d].g = graphs[d];
  }
  spf_query_desc qd{};
  qd.num_queries = num_sources;
  qd.sources = sources;
  CL_TRY(table_init(t.get(), c, graphs, desc->num_nodes, &qd, flags));
  *out = t.release();
  return SPF_OK;
}

int spf_table_create_q(spf_cgraph* cg, const spf_query_desc* qd, uint32_t flags, spf_table** out) {
  SPF_ABI_RANGE_CLUSTER("spf_table_create_q");
  if (!cg || !qd || !out) {
    return cfail(SPF_E_INVALID, "spf_table_create_q: null argument");
  }
  if (qd->flags & SPF_F_ORDER) {
    return cfail(SPF_E_UNSUPPORTED, "spf_table_create_q: settle order is single-device");
  }
  std::unique_ptr<spf_table, void (*)(spf_table*)> t(new spf_table, free_table);
  t->borrowed = true;
  t->cg = cg;
  cg->tables.fetch_add(1, std::memory_order_relaxed); // free_table gives it back
  CL_TRY(table_init(t.get(), cg->c, cg->g, cg->V, qd,
                    flags | (qd->flags & (SPF_F_UNIT_METRIC | SPF_F_NEXTHOPS))));
  *out = t.release();
  return SPF_OK;
}

int spf_table_run(spf_table* t) {
  SPF_ABI_RANGE_CLUSTER("spf_table_run");
  if (!t) {
    return cfail(SPF_E_INVALID, "spf_table_run: null table");
  }
  spf_cluster* c = t->c;
  // 1. every local block: one batch on its device, then its rows / masks
  //    into its own slot of the gathered buffers (device to device)
  for (auto& L : t->local) {
    CL_HIP(hipSetDevice(L.device));
    hipStream_t st = (hipStream_t)spf_graph_get_stream(L.g);
    CL_HIP(hipEventRecord(L.e0, st));
    const uint64_t first = t->block_first[L.rank], count = t->block_first[L.rank + 1] - first;
    if (L.q) {
      CL_TRY(spf_query_run(L.q));
      if (L.rows) {
        CL_TRY(spf_query_fetch_rows(L.q, 0, (uint32_t)count,
                                    L.rows + (size_t)L.rank * t->cap * t->V,
                                    (size_t)t->V * sizeof(uint32_t), 1));
      }
      if (L.masks) {
        void* dr = nullptr;
        uint32_t eb = 0;
        void* nh = nullptr;
        uint64_t total = 0;
        CL_TRY(spf_query_device_rows(L.q, &dr, &eb, &nh, &total));
        CL_HIP(hipMemcpyAsync(L.masks + (size_t)L.rank * t->mask_cap, nh,
                              total * sizeof(uint64_t), hipMemcpyDeviceToDevice, st));
        // (total * 8 = the query's byte layout, <= mask_cap)
      }
    }
    CL_HIP(hipEventRecord(L.e1, st));
  }
  // 2. the exchange: in-place all-gathers into equal-sized rank slots
  if (t->flags & (SPF_T_GATHER_ROWS | SPF_T_GATHER_NEXTHOPS)) {
    CL_NCCL(ncclGroupStart());
    for (size_t d = 0; d < t->local.size(); ++d) {
      auto& L = t->local[d];
      CL_HIP(hipSetDevice(L.device));
      hipStream_t st = (hipStream_t)spf_graph_get_stream(L.g);
      if (L.rows) {
        const size_t cnt = (size_t)t->cap * t->V;
        CL_NCCL(ncclAllGather(L.rows + (size_t)L.rank * cnt, L.rows, cnt, ncclUint32,
                              c->comms[d], st));
      }
      if (L.masks) {
        CL_NCCL(ncclAllGather(L.masks + (size_t)L.rank * t->mask_cap, L.masks, t->mask_cap / 8,
                              ncclUint64, c->comms[d], st));
      }
    }
    CL_NCCL(ncclGroupEnd());
  }
  for (auto& L : t->local) {
    CL_HIP(hipSetDevice(L.device));
    CL_HIP(hipEventRecord(L.e2, (hipStream_t)spf_graph_get_stream(L.g)));
  }
  t->ran = true;
  return SPF_OK;
}

int spf_table_sync(spf_table* t) {
  if (!t) {
    return cfail(SPF_E_INVALID, "spf_table_sync: null table");
  }
  for (auto& L : t->local) {
    CL_HIP(hipSetDevice(L.device));
    CL_HIP(hipEventSynchronize(L.e2));
  }
  return SPF_OK;
}

int spf_table_elapsed_ms(spf_table* t, float* compute_ms, float* gather_ms) {
  if (!t || !t->ran) {
    return cfail(SPF_E_INVALID, "spf_table_elapsed_ms: table has not run");
  }
  float cm = 0, gm = 0;
  for (auto& L : t->local) {
    CL_HIP(hipSetDevice(L.device));
    float a = 0, b = 0;
    CL_HIP(hipEventElapsedTime(&a, L.e0, L.e1));
    CL_HIP(hipEventElapsedTime(&b, L.e1, L.e2));
    cm = std::max(cm, a);
    gm = std::max(gm, b);
  }
  if (compute_ms) {
    *compute_ms = cm;
  }
  if (gather_ms) {
    *gather_ms = gm;
  }
  return SPF_OK;
}

int spf_table_block(const spf_table* t, uint32_t rank, uint32_t* first, uint32_t* count) {
  if (!t || rank >= t->c->world) {
    return cfail(SPF_E_INVALID, "spf_table_block: bad rank");
  }
  if (first) {
    *first = (uint32_t)t->block_first[rank];
  }
  if (count) {
    *count = (uint32_t)(t->block_first[rank + 1] - t->block_first[rank]);
  }
  return SPF_OK;
}

int spf_table_nh_words(const spf_table* t, uint32_t i) {
  if (!t || i >= t->n) {
    return cfail(SPF_E_INVALID, "spf_table_nh_words: bad index");
  }
  return (int)t->words[i];
}

int spf_table_nh_bytes(const spf_table* t, uint32_t i) {
  if (!t || i >= t->n) {
    return cfail(SPF_E_INVALID, "spf_table_nh_bytes: bad index");
  }
  return (int)t->nbytes[i];
}

// rank owning source index i
static uint32_t owner_of(const spf_table* t, uint32_t i) {
  const auto it = std::upper_bound(t->block_first.begin(), t->block_first.end(), (uint64_t)i);
  return (uint32_t)(it - t->block_first.begin()) - 1;
}

int spf_table_fetch_rows(spf_table* t, uint32_t first, uint32_t count, uint32_t* dst) {
  SPF_ABI_RANGE_CLUSTER("spf_table_fetch_rows");
  if (!t || !dst || first + (uint64_t)count > t->n) {
    return cfail(SPF_E_INVALID, "spf_table_fetch_rows: bad range");
  }
  uint32_t i = first;
  while (i < first + count) {
    const uint32_t r = owner_of(t, i);
    const uint32_t bend = (uint32_t)std::min<uint64_t>(t->block_first[r + 1], first + count);
    // the owner's device, or any local device holding the gathered rows
    const spf_table::Local* src = nullptr;
    for (const auto& L : t->local) {
      if (L.rank == r) {
        src = &L;
      }
    }
    if (!src || !src->q) {
      if (!(t->flags & SPF_T_GATHER_ROWS)) {
        return cfail(SPF_E_UNSUPPORTED, "spf_table_fetch_rows: rows of another rank (no gather)");
      }
      const auto& L = t->local[0];
      CL_HIP(hipSetDevice(L.device));
      CL_HIP(hipMemcpy(dst + (size_t)(i - first) * t->V,
                       L.rows + ((size_t)r * t->cap + (i - t->block_first[r])) * t->V,
                       (size_t)(bend - i) * t->V * sizeof(uint32_t), hipMemcpyDeviceToHost));
    } else {
      CL_TRY(spf_query_fetch_rows(src->q, (uint32_t)(i - t->block_first[r]), bend - i,
                                  dst + (size_t)(i - first) * t->V,
                                  (size_t)t->V * sizeof(uint32_t), 0));
    }
    i = bend;
  }
  return SPF_OK;
}

int spf_table_trace_paths(
    spf_table* t, const uint32_t* dests, uint32_t* path_count, uint32_t* link_count) {
  SPF_ABI_RANGE_CLUSTER("spf_table_trace_paths");
  if (!t || (t->n && (!dests || !path_count || !link_count))) {
    return cfail(SPF_E_INVALID, "spf_table_trace_paths: null argument");
  }
  if (!t->ran) {
    return cfail(SPF_E_INVALID, "spf_table_trace_paths: table has not run");
  }
  std::fill(path_count, path_count + t->n, 0u);
  std::fill(link_count, link_count + t->n, 0u);
  // every local block on its own device, concurrently (each call waits for
  // its own graph stream only)
  std::vector<int> st(t->local.size(), SPF_OK);
  std::vector<std::string> why(t->local.size());
  std::vector<std::thread> th;
  for (size_t j = 0; j < t->local.size(); ++j) {
    const auto& L = t->local[j];
    if (!L.q) {
      continue;
    }
    const uint64_t first = t->block_first[L.rank];
    const uint32_t count = (uint32_t)(t->block_first[L.rank + 1] - first);
    th.emplace_back([&, j, first, count] {
      if (hipSetDevice(t->local[j].device) != hipSuccess) {
        st[j] = SPF_E_DEVICE;
        return;
      }
      st[j] = spf_query_trace_paths(t->local[j].q, 0, count, dests + first, path_count + first,
                                    link_count + first);
      if (st[j] != SPF_OK) {
        why[j] = spf_last_error_detail();
      }
    });
  }
  for (auto& x : th) {
    x.join();
  }
  for (size_t j = 0; j < st.size(); ++j) {
    if (st[j] != SPF_OK) {
      return cfail(st[j], "spf_table_trace_paths: " + why[j]);
    }
  }
  // packed offsets of every local block (table-query order)
  t->trace_link_base.assign(t->local.size(), 0);
  t->trace_path_base.assign(t->local.size(), 0);
  std::vector<uint64_t> lsum(t->n + 1, 0), psum(t->n + 1, 0);
  for (uint32_t i = 0; i < t->n; ++i) {
    const bool ok = path_count[i] != SPF_TRACE_OVERFLOW;
    lsum[i + 1] = lsum[i] + (ok ? link_count[i] : 0);
    psum[i + 1] = psum[i] + (ok ? path_count[i] : 0);
  }
  for (size_t j = 0; j < t->local.size(); ++j) {
    const uint64_t first = t->block_first[t->local[j].rank];
    t->trace_link_base[j] = lsum[first];
    t->trace_path_base[j] = psum[first];
  }
  t->traced = true;
  return SPF_OK;
}

int spf_table_trace_fetch(spf_table* t, uint32_t* links, uint32_t* ends) {
  SPF_ABI_RANGE_CLUSTER("spf_table_trace_fetch");
  if (!t || !t->traced) {
    return cfail(SPF_E_INVALID, "spf_table_trace_fetch: no trace to fetch");
  }
  std::vector<int> st(t->local.size(), SPF_OK);
  std::vector<std::string> why(t->local.size());
  std::vector<std::thread> th;
  for (size_t j = 0; j < t->local.size(); ++j) {
    if (!t->local[j].q) {
      continue;
    }
    th.emplace_back([&, j] {
      if (hipSetDevice(t->local[j].device) != hipSuccess) {
        st[j] = SPF_E_DEVICE;
        return;
      }
      st[j] = spf_query_trace_fetch(t->local[j].q, links ? links + t->trace_link_base[j] : nullptr,
                                    ends ? ends + t->trace_path_base[j] : nullptr);
      if (st[j] != SPF_OK) {
        why[j] = spf_last_error_detail();
      }
    });
  }
  for (auto& x : th) {
    x.join();
  }
  for (size_t j = 0; j < st.size(); ++j) {
    if (st[j] != SPF_OK) {
      return cfail(st[j], "spf_table_trace_fetch: " + why[j]);
    }
  }
  return SPF_OK;
}

int spf_table_fetch_nexthops(spf_table* t, uint32_t first, uint32_t count, uint64_t* dst) {
  SPF_ABI_RANGE_CLUSTER("spf_table_fetch_nexthops");
  if (!t || !dst || first + (uint64_t)count > t->n || !(t->flags & SPF_F_NEXTHOPS)) {
    return cfail(SPF_E_INVALID, "spf_table_fetch_nexthops: bad range or no next hops");
  }
  uint32_t i = first;
  uint64_t out = 0;
  while (i < first + count) {
    const uint32_t r = owner_of(t, i);
    const uint32_t bend = (uint32_t)std::min<uint64_t>(t->block_first[r + 1], first + count);
    const spf_table::Local* src = nullptr;
    for (const auto& L : t->local) {
      if (L.rank == r) {
        src = &L;
      }
    }
    uint64_t words = 0;
    for (uint32_t k = i; k < bend; ++k) {
      words += (uint64_t)t->V * t->words[k];
    }
    if (src && src->q) {
      CL_TRY(spf_query_fetch_nexthops(src->q, (uint32_t)(i - t->block_first[r]), bend - i, dst + out));
    } else {
      if (!(t->flags & SPF_T_GATHER_NEXTHOPS)) {
        return cfail(SPF_E_UNSUPPORTED, "spf_table_fetch_nexthops: masks of another rank (no gather)");
      }
      const auto& L = t->local[0];
      CL_HIP(hipSetDevice(L.device));
      uint64_t o = out;
      for (uint32_t k = i; k < bend; ++k) {
        const size_t w = (size_t)t->V * t->words[k];
        const uint32_t B = t->nbytes[k];
        if (B >= 8) {
          CL_HIP(hipMemcpy(dst + o, L.masks + t->mask_off[k], w * sizeof(uint64_t),
                           hipMemcpyDeviceToHost));
        } else {
          // narrow row: one B-byte integer per node, widened to u64 words
          std::vector<uint8_t> tmp((size_t)t->V * B);
          CL_HIP(hipMemcpy(tmp.data(), L.masks + t->mask_off[k], tmp.size(),
                           hipMemcpyDeviceToHost));
          for (size_t v = 0; v < t->V; ++v) {
            uint64_t x = 0;
            std::memcpy(&x, tmp.data() + v * B, B);
            dst[o + v] = x;
          }
        }
        o += w;
      }
    }
    out += words;
    i = bend;
  }
  return SPF_OK;
}

int spf_table_device_buffers(
    spf_table* t, uint32_t local, void** rows, void** masks, uint64_t* mask_cap_bytes) {
  if (!t || local >= t->local.size()) {
    return cfail(SPF_E_INVALID, "spf_table_device_buffers: bad local index");
  }
  if (rows) {
    *rows = t->local[local].rows;
  }
  if (masks) {
    *masks = t->local[local].masks;
  }
  if (mask_cap_bytes) {
    *mask_cap_bytes = t->mask_cap;
  }
  return SPF_OK;
}

int spf_table_kernel_name(spf_table* t, uint32_t local, const char** name) {
  if (!t || local >= t->local.size() || !name) {
    return cfail(SPF_E_INVALID, "spf_table_kernel_name: bad local index");
  }
  *name = t->local[local].q ? spf_query_kernel_name(t->local[local].q) : "";
  return SPF_OK;
}

} // extern "C"
