// spf_device.hip — MI355X (gfx950) kernels and the C ABI of include/openr_spf.h
//
// The reference runs one Dijkstra per source on the Decision thread, walking a
// string-keyed graph (openr/decision/LinkState.cpp:806-880).  Here a batch of
// sources is solved at once, one workgroup per source, against a device CSR
// that every workgroup shares through L2:
//
//  * spf_sssp_kernel  (fast path, every usable metric in [1, 2^31)):
//      the per-source state (distance row, frontier bitmaps, node queue) lives
//      in LDS (or, for graphs too large for LDS, in a global scratch slab).
//      Rounds alternate
//        PUSH  — every node whose (dist, next-hops) changed marks the
//                neighbours it could still improve or tie (ds_or on an LDS
//                bitmap), and
//        PULL  — every marked node recomputes its distance and ECMP next-hop
//                mask from ALL its in-edges (min over d[u]+w, OR of the
//                predecessors' masks at the minimum).
//      A node is written only by the group that owns it in PULL, so no
//      distance atomics are needed and the fixpoint is deterministic.  With
//      unit metrics every node is pulled exactly once (level-synchronous
//      BFS); with weights it is a frontier Bellman-Ford.
//      This is the order-free restatement of runSpf validated in SURVEY §8(a):
//        d = Dijkstra where u relaxes only if u==src or !overloaded(u);
//        NH(v) = OR over usable u->v with d[u]+w==d[v] and (u==src ||
//                !overloaded(u)) of (u==src ? {v} : NH(u)).
//  * spf_exact_kernel (metric 0 or 64-bit metric sums): one thread per query
//      replays the reference DijkstraQ literally — (metric, name) ordered
//      extraction of DISCOVERED nodes, >= relaxation into unsettled nodes,
//      union of next hops, "directly connected" rule — with uint64 wrap-around
//      arithmetic, and records the settle order (pathLinks ordering).
//
// Node ids are name ranks, so "ties settle by name" is "ties settle by id".

#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <atomic>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <queue>
#include <string>
#include <map>
#include <mutex>
#include <unordered_map>
#include <vector>

#include "openr_spf.h"
#include "host/Parallel.h"

// roctx ranges around every C-ABI entry point (SURVEY.md §5 tracing): a
// rocprofv3 --marker-trace / --kernel-trace run shows which Decision call
// (graph build, query run, table repair, ...) each kernel belongs to.
#include <rocprofiler-sdk-roctx/roctx.h>
namespace {
struct AbiRange {
  explicit AbiRange(const char* name) { roctxRangePushA(name); }
  ~AbiRange() { roctxRangePop(); }
  AbiRange(const AbiRange&) = delete;
  AbiRange& operator=(const AbiRange&) = delete;
};
} // namespace
#define SPF_ABI_RANGE(name) AbiRange spf_abi_range_(name)

// The kernels the running query launched (spf_query_kernels): every launch
// site goes through SPF_LAUNCH, which notes the kernel expression while a
// spf_query_run is active on this thread (sub-queries of a plan — a what-if
// baseline, the zero-metric fix-up — land in the outermost query's list).
namespace {
thread_local std::vector<const char*>* tl_launched = nullptr;
inline void spf_note_launch(const char* expr) {
  if (tl_launched && std::find(tl_launched->begin(), tl_launched->end(), expr) == tl_launched->end()) {
    tl_launched->push_back(expr);
  }
}
} // namespace
#define SPF_LAUNCH(kern, ...)           \
  do {                                  \
    spf_note_launch(#kern);             \
    hipLaunchKernelGGL(kern, __VA_ARGS__); \
  } while (0)
// a launch through a kernel variable: `name` is the kernel's own name
#define SPF_LAUNCH_AS(name, kern, ...)  \
  do {                                  \
    spf_note_launch(name);              \
    hipLaunchKernelGGL(kern, __VA_ARGS__); \
  } while (0)

namespace {

constexpr uint32_t kBlock = 512;           // threads per workgroup (8 waves)
constexpr uint32_t kWaves = kBlock / 64;
constexpr uint32_t kInf32 = 0xFFFFFFFFu;
// host passes over the CSR go parallel from this many edges per thread
constexpr size_t kHostMinEdges = 1u << 14;

// Node blocks of about equal work (edges + nodes) for the host passes over a
// CSR: name ranks put the fabric's 1,672 FSW / SSW nodes (71 % of its edges)
// into 3-4 of twenty fixed 512-node blocks, so one worker did most of every
// pass (profiles/r05ah).  Boundaries b[0] = 0 < ... < b.back() = V.
std::vector<uint32_t> host_node_blocks(const uint32_t* row, uint32_t V, unsigned nth) {
  std::vector<uint32_t> b{0};
  if (!V) {
    return b;
  }
  const uint64_t work = (uint64_t)row[V] - row[0] + V;
  const uint32_t nb = std::max<uint32_t>(1, std::min<uint32_t>(V, 8 * std::max(1u, nth)));
  const uint64_t target = std::max<uint64_t>(1, work / nb);
  uint32_t u = 0;
  while (u < V) {
    // the first u' > u with (row[u'] - row[u]) + (u' - u) >= target
    uint32_t lo = u + 1, hi = V;
    while (lo < hi) {
      const uint32_t mid = lo + (hi - lo) / 2;
      if ((uint64_t)(row[mid] - row[u]) + (mid - u) >= target) {
        hi = mid;
      } else {
        lo = mid + 1;
      }
    }
    u = lo;
    b.push_back(u);
  }
  return b;
}
constexpr uint32_t kCtlWords = 32;         // qlen + scan scratch (<= 16 waves + 1)
constexpr size_t kLdsLimit = 160 * 1024;   // gfx950 LDS per CU
constexpr uint32_t kIgnLdsMax = 2048;      // ignore-list entries staged in LDS
// internal query flag (never in the ABI): next-hop output rows in the word
// layout (8 * W bytes per node) whatever the neighbour count, for batches
// whose rows another query copies into its working buffer (what-if
// baselines, the zero-metric plan's wide-plan sources)
constexpr uint32_t kQueryWideMasks = 0x80000000u;
// internal query flag: no first-hop nested batch for this query's source-link
// failures (the nested batch itself; spf_whatif_firsthop_kernel)
constexpr uint32_t kQueryNoFirstHop = 0x40000000u;
constexpr uint32_t kNotSeen = 0xFFFFFFFFu; // exact kernel heap states
constexpr uint32_t kSettled = 0xFFFFFFFEu;

thread_local std::string g_last_error;

// 0/1 switch from the environment (A/B knobs of the measured variants)
uint32_t env_flag(const char* name, uint32_t dflt) {
  const char* v = getenv(name);
  return v ? (uint32_t)(atoi(v) != 0) : dflt;
}

// unsigned value from the environment (A/B knobs with a size)
uint32_t env_u32(const char* name, uint32_t dflt) {
  const char* v = getenv(name);
  return v ? (uint32_t)strtoul(v, nullptr, 10) : dflt;
}

int fail(int code, const std::string& what) {
  g_last_error = what;
  return code;
}

#define HIP_TRY(expr)                                                       \
  do {                                                                      \
    hipError_t e_ = (expr);                                                 \
    if (e_ != hipSuccess) {                                                 \
      return fail(                                                          \
          e_ == hipErrorOutOfMemory ? SPF_E_NOMEM : SPF_E_DEVICE,           \
          std::string(#expr) + ": " + hipGetErrorString(e_));               \
    }                                                                       \
  } while (0)

// ---------------------------------------------------------------- device utils

__device__ __forceinline__ uint32_t grp_min(uint32_t x, int G) {
  for (int o = G >> 1; o > 0; o >>= 1) {
    x = min(x, (uint32_t)__shfl_xor((int)x, o, G));
  }
  return x;
}

// Lanes per node for a list of n nodes over a kBlock workgroup: the graph's
// G (median degree), doubled while the whole list still runs in one pass
// (round 6): a short list -- a what-if repair's K, an SSSP's first levels --
// then walks a 84- or 190-edge row in 2-3 steps instead of 21-48 at G = 4
// (the fabric's median degree), each step a dependent global-load trip
__device__ __forceinline__ uint32_t lanes_for(uint32_t n, uint32_t G) {
  while (G < 64 && kBlock / (2 * G) >= n) {
    G <<= 1;
  }
  return G;
}

__device__ __forceinline__ uint64_t grp_or(uint64_t x, int G) {
  for (int o = G >> 1; o > 0; o >>= 1) {
    x |= (uint64_t)__shfl_xor((unsigned long long)x, o, G);
  }
  return x;
}

__device__ __forceinline__ bool in_sorted(
    const uint32_t* a, uint32_t n, uint32_t x) {
  uint32_t lo = 0, hi = n;
  while (lo < hi) {
    uint32_t mid = (lo + hi) >> 1;
    uint32_t m = a[mid];
    if (m == x) {
      return true;
    }
    if (m < x) {
      lo = mid + 1;
    } else {
      hi = mid;
    }
  }
  return false;
}

// A query's ignored links: the sorted list (in_sorted), or, for lists of 8+
// links, an open-addressing hash set in the same LDS words (2^hbits slots,
// load factor <= 1/2, kInf32 = empty): one or two probes per edge instead of
// a binary search (KSP2 second passes ignore every link of the k = 1 paths,
// hundreds per query, and test every relaxed edge)
struct IgnSet {
  const uint32_t* p = nullptr;
  uint32_t n = 0;
  uint32_t hbits = 0;
  __device__ __forceinline__ bool has(uint32_t l) const {
    if (!n) {
      return false;
    }
    if (hbits) {
      const uint32_t mask = (1u << hbits) - 1;
      uint32_t h = (l * 0x9E3779B1u) >> (32 - hbits);
      for (;;) {
        const uint32_t x = p[h];
        if (x == l) {
          return true;
        }
        if (x == kInf32) {
          return false;
        }
        h = (h + 1) & mask;
      }
    }
    return in_sorted(p, n, l);
  }
};

// slots of the hash form for n links (0: keep the sorted list)
__host__ __device__ inline uint32_t ign_hash_slots(uint32_t n) {
  if (n < 8) {
    return 0;
  }
  uint32_t t = 16;
  while (t < 2 * n) {
    t <<= 1;
  }
  return t;
}

// ---- next-hop mask rows (byte-strided layout of spf_query results)
// A query's row holds B bytes per node: B = 1, 2, 4 for sources with at most
// 8, 16, 32 distinct neighbours (bit j of the byte / short / word = the j-th
// neighbour), else 8 * W with W = ceil(neighbours / 64) u64 words, node-major
// (the original layout).  A fabric RSW (8 neighbours) thus writes one byte per
// node instead of a 64-bit word (nh_bytes_for, include/openr_spf.h).
__host__ __device__ __forceinline__ uint32_t nh_bytes_for(uint32_t nbrs) {
  return nbrs <= 8 ? 1u : nbrs <= 16 ? 2u : nbrs <= 32 ? 4u : 8u * ((nbrs + 63) / 64);
}

// word w of node v's mask (w < W; narrow rows have one word)
__device__ __forceinline__ uint64_t nh_load(const uint8_t* row, uint32_t B, uint32_t W,
                                            uint32_t v, uint32_t w) {
  if (B >= 8) {
    return reinterpret_cast<const uint64_t*>(row)[(size_t)v * W + w];
  }
  if (B == 4) {
    return reinterpret_cast<const uint32_t*>(row)[v];
  }
  if (B == 2) {
    return reinterpret_cast<const uint16_t*>(row)[v];
  }
  return row[v];
}

__device__ __forceinline__ void nh_store(uint8_t* row, uint32_t B, uint32_t W, uint32_t v,
                                         uint32_t w, uint64_t x) {
  if (B >= 8) {
    reinterpret_cast<uint64_t*>(row)[(size_t)v * W + w] = x;
  } else if (B == 4) {
    reinterpret_cast<uint32_t*>(row)[v] = (uint32_t)x;
  } else if (B == 2) {
    reinterpret_cast<uint16_t*>(row)[v] = (uint16_t)x;
  } else {
    row[v] = (uint8_t)x;
  }
}

typedef uint32_t nt_u32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t nt_u32x4 __attribute__((ext_vector_type(4)));

// a streaming (write-once, never re-read by this pass) store: NT = true marks
// it non-temporal so the output rows do not evict the level rows the other
// blocks of the pass re-read from L2
template <typename T>
__device__ __forceinline__ void st_stream(T* p, T v, bool nt) {
  if (nt) {
    __builtin_nontemporal_store(v, p);
  } else {
    *p = v;
  }
}

// single-word masks of nodes v0..v0+3 (v0 % 4 == 0) of a narrow row (B < 8):
// one 4 / 8 / 16-byte store when all four nodes exist
__device__ __forceinline__ void nh_store4_narrow(uint8_t* row, uint32_t B, uint32_t v0,
                                                 uint32_t V, const uint64_t (&x)[4],
                                                 bool nt = false) {
  if (v0 + 4 <= V) {
    if (B == 1) {
      st_stream(reinterpret_cast<uint32_t*>(row + v0),
                (uint32_t)(x[0] & 0xFFu) | (uint32_t)(x[1] & 0xFFu) << 8 |
                    (uint32_t)(x[2] & 0xFFu) << 16 | (uint32_t)(x[3] & 0xFFu) << 24,
                nt);
    } else if (B == 2) {
      nt_u32x2 w;
      w.x = (uint32_t)(x[0] & 0xFFFFu) | (uint32_t)(x[1] & 0xFFFFu) << 16;
      w.y = (uint32_t)(x[2] & 0xFFFFu) | (uint32_t)(x[3] & 0xFFFFu) << 16;
      st_stream(reinterpret_cast<nt_u32x2*>(row + 2 * (size_t)v0), w, nt);
    } else {
      nt_u32x4 w;
      w.x = (uint32_t)x[0];
      w.y = (uint32_t)x[1];
      w.z = (uint32_t)x[2];
      w.w = (uint32_t)x[3];
      st_stream(reinterpret_cast<nt_u32x4*>(row + 4 * (size_t)v0), w, nt);
    }
    return;
  }
#pragma unroll
  for (uint32_t i = 0; i < 4; ++i) {
    if (v0 + i < V) {
      nh_store(row, B, 1, v0 + i, 0, x[i]);
    }
  }
}

// Exclusive scan of one value per thread over the workgroup.  `scan` holds
// kWaves+1 LDS words.  Returns the thread's offset; *total = block sum.
template <uint32_t BS = kBlock>
__device__ __forceinline__ uint32_t block_excl_scan(
    uint32_t x, uint32_t* scan, uint32_t* total) {
  constexpr uint32_t kWaves = BS / 64;
  const uint32_t lane = threadIdx.x & 63u, wid = threadIdx.x >> 6;
  uint32_t inc = x;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    uint32_t y = (uint32_t)__shfl_up((int)inc, o, 64);
    if (lane >= (uint32_t)o) {
      inc += y;
    }
  }
  if (lane == 63) {
    scan[wid] = inc;
  }
  __syncthreads();
  if (wid == 0) {
    uint32_t w = lane < kWaves ? scan[lane] : 0;
#pragma unroll
    for (int o = 1; o < (int)kWaves; o <<= 1) {
      uint32_t y = (uint32_t)__shfl_up((int)w, o, 64);
      if (lane >= (uint32_t)o) {
        w += y;
      }
    }
    if (lane < kWaves) {
      scan[lane] = w;
    }
  }
  __syncthreads();
  uint32_t base = wid ? scan[wid - 1] : 0;
  *total = scan[kWaves - 1];
  return base + inc - x;
}

// Turn a node bitmap into a queue of node ids (ascending), clearing the bitmap.
template <typename QT, uint32_t BS = kBlock>
__device__ __forceinline__ uint32_t compact_bits(
    uint32_t* bits, uint32_t nbw, QT* queue, uint32_t* scan) {
  const uint32_t chunk = (nbw + BS - 1) / BS;
  const uint32_t w0 = min(threadIdx.x * chunk, nbw);
  const uint32_t w1 = min(w0 + chunk, nbw);
  uint32_t cnt = 0;
  for (uint32_t w = w0; w < w1; ++w) {
    cnt += __popc(bits[w]);
  }
  uint32_t total;
  uint32_t off = block_excl_scan<BS>(cnt, scan, &total);
  for (uint32_t w = w0; w < w1; ++w) {
    uint32_t b = bits[w];
    if (b) {
      bits[w] = 0;
      do {
        uint32_t k = __ffs(b) - 1;
        b &= b - 1;
        queue[off++] = (QT)(w * 32 + k);
      } while (b);
    }
  }
  return total;
}

struct SsspArgs {
  // graph
  const uint32_t* row;
  const uint32_t* col;
  const uint32_t* wout; // metric of u->v advertised by the row node u
  const uint32_t* win;  // metric of v->u for the entry (u, v): w_out[rev[e]]
  const uint32_t* link;
  const uint32_t* rev;
  const uint32_t* slot; // slot of col[e] among the row node's distinct nbrs
  const uint32_t* trbits;
  // batch
  const uint32_t* src;
  const uint32_t* ign_off;
  const uint32_t* ign;
  const uint64_t* nh_off;
  const uint32_t* nh_w;
  uint32_t* dist_out;
  uint64_t* nh_out;
  uint32_t* gscratch; // GMEM: per-workgroup node queue (V u32)
  uint32_t V;
  uint32_t Vp; // row stride of dist_out
  uint32_t nbw;
  uint32_t nq;
  uint32_t G;       // lanes per node (power of two, <= 64)
  uint32_t ign_cap; // LDS words reserved for the ignore list
  // what-if screen: queries whose rows were copied from the baseline run
  // (skip[q] != 0) are not recomputed; nullptr = none
  const uint32_t* skip;
  // what-if repair (IGN batches behind the screen; base_dist = nullptr: off):
  // a query the screen could not resolve starts from its baseline rows and
  // recomputes only the nodes downstream of its tight ignored links
  // (whatif_repair_init); base rows in the word layout of the query's own
  const uint32_t* base_dist = nullptr; // [nb][Vp]
  const uint64_t* base_nh = nullptr;
  const uint64_t* base_nh_off = nullptr;
  const uint32_t* base_of = nullptr;
  const uint32_t* link_half = nullptr; // [2 * L] half-edges of each link
  uint32_t L = 0;
  // queries beyond the first gridDim.x are claimed from this counter (zeroed
  // per launch); nullptr: static stride
  uint32_t* qctr = nullptr;
  // repair batches: [0] heavy count, [1] total, [2 ..] the queries to run,
  // heavy (skip 2) first (spf_whatif_worklist_kernel); nullptr: every query
  // is claimed and its skip flag tested (two passes)
  const uint32_t* wl = nullptr;
  // OPENR_SPF_WHATIF_STATS: repaired / from-scratch queries, |K| total, PULL
  // rounds, and wall-clock ticks (100 MHz) of copy / init / rounds / output
  unsigned long long* stats = nullptr;
};

__device__ __forceinline__ bool bit_test(const uint32_t* b, uint32_t v) {
  return (b[v >> 5] >> (v & 31)) & 1u;
}
// set bit v; true if this call set it
__device__ __forceinline__ bool bit_claim(uint32_t* b, uint32_t v) {
  const uint32_t m = 1u << (v & 31);
  return !(atomicOr(&b[v >> 5], m) & m);
}

// n elements src -> dst by a workgroup of BS threads, U loads in flight per
// thread (a plain strided loop waits out one load latency per element)
template <typename T, uint32_t BS, int U = 8>
__device__ __forceinline__ void block_copy(T* __restrict__ dst, const T* __restrict__ src, size_t n) {
  size_t i = threadIdx.x;
  for (; i + (size_t)(U - 1) * BS < n; i += (size_t)U * BS) {
    T t[U];
#pragma unroll
    for (int k = 0; k < U; ++k) {
      t[k] = src[i + (size_t)k * BS];
    }
#pragma unroll
    for (int k = 0; k < U; ++k) {
      dst[i + (size_t)k * BS] = t[k];
    }
  }
  for (; i < n; i += BS) {
    dst[i] = src[i];
  }
}

// What-if repair prologue (spf_sssp_kernel, IGN with baseline rows): the
// query's rows start as the baseline run's from the same source, then
//  K  = heads of the ignored links' halves that are tight usable edges of the
//       baseline (d[u] + w == d[v], u the source or transit) and every node
//       reachable from them over tight usable non-ignored edges: no node
//       outside K had a shortest path through an ignored link, so its
//       distance and next-hop set are unchanged (and no path through K can
//       tie it later: a K node's distance only grows, and an edge K -> w
//       that was not tight stays strictly longer);
//  ok = nodes of K reachable over tight usable non-ignored edges from outside
//       K: their distance is still achieved (exact), only their next hops
//       may shrink;
// K \ ok is reset to unreached, and all of K is queued for the PULL step
// (distance + next-hop union from every in-edge), so the rounds that follow
// reach the same fixpoint as a run from scratch.  kb / okb:
// zeroed LDS bitmaps; act / chg: clear on entry and exit.  Returns |K|, with
// K's ids in `queue`, or kInf32 (bitmaps clear) when K passes V / 4 nodes and
// the query should run from scratch instead.
template <typename QT, bool UNIT>
__device__ uint32_t whatif_repair_init(
    const SsspArgs& a, uint32_t src, uint32_t* dist, uint32_t* kb, uint32_t* okb,
    uint32_t* act, const uint32_t* tr, QT* queue, uint32_t* ctl, const uint32_t* ilist,
    uint32_t nign, const IgnSet& ig) {
  (void)act;
  const uint32_t tid = threadIdx.x, V = a.V, nbw = a.nbw;
  // K and ok grow as LDS worklists (round 6): |K| is a handful of nodes, and
  // compacting the V-bit maps after every closure level (a block scan each)
  // was most of this prologue.  K lists into queue[0 ..), ok into
  // queue[V / 2 ..) (|ok| <= |K| <= V / 4 once the size check passed); the
  // tails live in the control words the scans leave alone.
  uint32_t* ktail = ctl + (kCtlWords - 2);
  uint32_t* otail = ctl + (kCtlWords - 3);
  QT* olist = queue + V / 2;
  auto usable = [&](uint32_t u) { return u == src || ((tr[u >> 5] >> (u & 31)) & 1u); };
  auto ignored = [&](uint32_t e) { return ig.has(a.link[e]); };
  auto push = [&](uint32_t* bm, uint32_t* tail, QT* list, uint32_t v) {
    const uint32_t m = 1u << (v & 31);
    if (!(atomicOr(&bm[v >> 5], m) & m)) {
      list[atomicAdd(tail, 1u)] = (QT)v; // each node once: at most V entries
    }
  };
  if (tid == 0) {
    *ktail = 0;
    *otail = 0;
  }
  __syncthreads();
  // seeds: heads of tight ignored halves
  for (uint32_t i = tid; i < 2 * nign; i += kBlock) {
    const uint32_t l = ilist[i >> 1]; // the query's list (the LDS copy may be a hash set)
    const uint32_t e = l < a.L ? a.link_half[2 * (size_t)l + (i & 1)] : kInf32;
    if (e == kInf32) {
      continue;
    }
    const uint32_t u = a.col[a.rev[e]], v = a.col[e];
    const uint32_t du = dist[u];
    if (du != kInf32 && usable(u) && du + (UNIT ? 1u : a.wout[e]) == dist[v]) {
      push(kb, ktail, queue, v);
    }
  }
  __syncthreads();
  // K: closure over tight usable non-ignored edges, level by level
  uint32_t head = 0;
  for (;;) {
    const uint32_t tail = *ktail;
    __syncthreads(); // every lane has its tail before this level pushes
    if (tail * 4 > V) {
      // K spans most of the graph (a failure next to the source): the
      // caller's run from scratch is cheaper than repairing it
      for (uint32_t w = tid; w < nbw; w += kBlock) {
        kb[w] = 0;
      }
      __syncthreads();
      return kInf32;
    }
    if (head == tail) {
      break;
    }
    const uint32_t G = lanes_for(tail - head, a.G);
    const uint32_t lg = tid & (G - 1), grp = tid / G, ngrp = kBlock / G;
    for (uint32_t i = head + grp; i < tail; i += ngrp) {
      const uint32_t u = queue[i];
      if (!usable(u)) {
        continue;
      }
      const uint32_t du = dist[u];
      for (uint32_t e = a.row[u] + lg; e < a.row[u + 1]; e += G) {
        const uint32_t v = a.col[e];
        if (du + (UNIT ? 1u : a.wout[e]) == dist[v] && !bit_test(kb, v) && !ignored(e)) {
          push(kb, ktail, queue, v);
        }
      }
    }
    head = tail;
    __syncthreads();
  }
  const uint32_t nk = head;
  // ok seeds: K nodes with a tight usable non-ignored in-edge from outside K
  {
    const uint32_t G = lanes_for(nk, a.G);
    const uint32_t lg = tid & (G - 1), grp = tid / G, ngrp = kBlock / G;
    for (uint32_t i = grp; i < nk; i += ngrp) {
      const uint32_t v = queue[i];
      const uint32_t dv = dist[v];
      bool found = false;
      for (uint32_t e = a.row[v] + lg; e < a.row[v + 1] && !found; e += G) {
        const uint32_t u = a.col[e];
        if (bit_test(kb, u) || !usable(u)) {
          continue;
        }
        const uint32_t du = dist[u];
        found = du != kInf32 && du + (UNIT ? 1u : a.win[e]) == dv && !ignored(e);
      }
      found = grp_min(found ? 0u : 1u, (int)G) == 0;
      if (found && lg == 0) {
        push(okb, otail, olist, v);
      }
    }
  }
  __syncthreads();
  // ok: closure inside K over tight usable non-ignored edges
  uint32_t oh = 0;
  for (;;) {
    const uint32_t ot = *otail;
    __syncthreads();
    if (oh == ot) {
      break;
    }
    const uint32_t G = lanes_for(ot - oh, a.G);
    const uint32_t lg = tid & (G - 1), grp = tid / G, ngrp = kBlock / G;
    for (uint32_t i = oh + grp; i < ot; i += ngrp) {
      const uint32_t u = olist[i];
      if (!usable(u)) {
        continue;
      }
      const uint32_t du = dist[u];
      for (uint32_t e = a.row[u] + lg; e < a.row[u + 1]; e += G) {
        const uint32_t v = a.col[e];
        if (bit_test(kb, v) && !bit_test(okb, v) && du + (UNIT ? 1u : a.wout[e]) == dist[v] &&
            !ignored(e)) {
          push(okb, otail, olist, v);
        }
      }
    }
    oh = ot;
    __syncthreads();
  }
  // K \ ok reset; all of K (queue[0, nk)) goes to the PULL step
  for (uint32_t i = tid; i < nk; i += kBlock) {
    const uint32_t v = queue[i];
    if (!bit_test(okb, v)) {
      dist[v] = kInf32;
    }
  }
  __syncthreads();
  // the maps leave clear (only K's bits were set)
  for (uint32_t i = tid; i < nk; i += kBlock) {
    const uint32_t v = queue[i];
    kb[v >> 5] = 0;
    okb[v >> 5] = 0;
  }
  __syncthreads();
  return nk;
}

// WMAX: max next-hop words (0 = distances only).  UNIT: every hop costs 1.
// IGN: per-query ignored links.  GMEM: distances / queue in global memory.
template <int WMAX, bool UNIT, bool IGN, bool GMEM>
__global__ __launch_bounds__(kBlock) void spf_sssp_kernel(SsspArgs a) {
  extern __shared__ __align__(16) uint32_t smem[];
  using QT = typename std::conditional<GMEM, uint32_t, uint16_t>::type;

  const uint32_t V = a.V, nbw = a.nbw, G = a.G;
  const uint32_t tid = threadIdx.x;
  const uint32_t lg = tid & (G - 1);
  const uint32_t grp = tid / G, ngrp = kBlock / G;

  uint32_t* act = smem;
  uint32_t* chg = act + nbw;
  uint32_t* tr = chg + nbw;
  uint32_t* ctl = tr + nbw;
  uint32_t* ignl = ctl + kCtlWords;
  // what-if repair bitmaps (K, ok) behind the ignore list
  const bool rep = IGN && a.base_dist != nullptr;
  uint32_t* kb = ignl + a.ign_cap;
  uint32_t* okb = kb + (rep ? nbw : 0);
  QT* queue;
  uint32_t* dist;
  if constexpr (GMEM) {
    queue = a.gscratch + (size_t)blockIdx.x * V;
    dist = nullptr;
  } else {
    queue = reinterpret_cast<QT*>(okb + (rep ? nbw : 0));
    dist = reinterpret_cast<uint32_t*>(queue + ((V + 1) & ~1u));
  }

  for (uint32_t i = tid; i < nbw; i += kBlock) {
    act[i] = 0;
    chg[i] = 0;
    tr[i] = a.trbits[i];
    if (rep) {
      kb[i] = 0;
      okb[i] = 0;
    }
  }
  __syncthreads();

  auto next_query = [&](uint32_t q) -> uint32_t {
    if (!a.qctr) {
      return q + gridDim.x;
    }
    __syncthreads(); // every lane has read ctl[kCtlWords - 1] of this query
    if (tid == 0) {
      ctl[kCtlWords - 1] = gridDim.x + atomicAdd(a.qctr, 1u);
    }
    __syncthreads();
    return ctl[kCtlWords - 1];
  };
  // repair batches claim in two passes: first the queries whose failed link
  // leaves the source (skip == 2, the screen's mark: their K is most of the
  // graph and they run from scratch), then the rest (skip == 0)
  // (with the work list every claim is a query to run: the screened ones
  // no longer cost a claim -- one contended counter add and two barriers each)
  const bool listed = rep && a.wl != nullptr;
  const bool two_pass = rep && a.qctr && !listed;
  const uint32_t nclaim = listed ? a.wl[1] : (two_pass ? 2 * a.nq : a.nq);
  for (uint32_t c = blockIdx.x; c < nclaim; c = next_query(c)) {
    const uint32_t q = listed ? a.wl[2 + c] : (c < a.nq ? c : c - a.nq);
    if (!listed &&
        (two_pass ? a.skip[q] != (c < a.nq ? 2u : 0u) : (a.skip && a.skip[q]))) {
      continue; // uniform per block
    }
    const uint32_t src = a.src[q];
    if constexpr (GMEM) {
      dist = a.dist_out + (size_t)q * a.Vp;
    }
    uint32_t nign = 0;
    const uint32_t* ignp = ignl;
    IgnSet ig;
    if constexpr (IGN) {
      const uint32_t lo = a.ign_off[q];
      nign = a.ign_off[q + 1] - lo;
      const uint32_t slots = ign_hash_slots(nign);
      if (slots && slots <= a.ign_cap) {
        for (uint32_t i = tid; i < slots; i += kBlock) {
          ignl[i] = kInf32;
        }
        __syncthreads();
        const uint32_t hb = __builtin_ctz(slots);
        for (uint32_t i = tid; i < nign; i += kBlock) {
          const uint32_t l = a.ign[lo + i];
          uint32_t h = (l * 0x9E3779B1u) >> (32 - hb);
          for (;;) {
            const uint32_t prev = atomicCAS(&ignl[h], kInf32, l);
            if (prev == kInf32 || prev == l) {
              break;
            }
            h = (h + 1) & (slots - 1);
          }
        }
        ig.hbits = hb;
      } else if (nign <= a.ign_cap) {
        for (uint32_t i = tid; i < nign; i += kBlock) {
          ignl[i] = a.ign[lo + i];
        }
      } else {
        ignp = a.ign + lo;
      }
      ig.p = ignp;
      ig.n = nign;
    }
    uint32_t Wm = 0;
    uint64_t* nhrow = nullptr;
    if constexpr (WMAX > 0) {
      Wm = a.nh_w[q];
      nhrow = a.nh_out + a.nh_off[q];
    }
    uint32_t qlen;
    bool pull_first = false;
    unsigned long long tk0 = 0, tk1 = 0, tk2 = 0;
    uint32_t rounds = 0;
    if (a.stats && tid == 0) {
      tk0 = wall_clock64();
    }
    if (rep) {
      // baseline rows, then only K is recomputed (whatif_repair_init)
      const uint32_t b = a.base_of[q];
      block_copy<uint32_t, kBlock>(dist, a.base_dist + (size_t)b * a.Vp, V);
      if constexpr (WMAX > 0) {
        block_copy<uint64_t, kBlock>(nhrow, a.base_nh + a.base_nh_off[b], (size_t)V * Wm);
      }
      __syncthreads();
      if (a.stats && tid == 0) {
        tk1 = wall_clock64();
      }
      qlen = whatif_repair_init<QT, UNIT>(a, src, dist, kb, okb, act, tr, queue, ctl,
                                          a.ign + a.ign_off[q], nign, ig);
      pull_first = qlen != kInf32;
      if (a.stats && tid == 0) {
        atomicAdd(&a.stats[pull_first ? 0 : 1], 1ull);
        atomicAdd(&a.stats[2], pull_first ? (unsigned long long)qlen : 0ull);
        tk2 = wall_clock64();
        atomicAdd(&a.stats[4], tk1 - tk0);
        atomicAdd(&a.stats[5], tk2 - tk1);
      }
    }
    if (!pull_first) {
      for (uint32_t v = tid; v < V; v += kBlock) {
        dist[v] = kInf32;
      }
      __syncthreads();
      if (tid == 0) {
        dist[src] = 0;
        queue[0] = (QT)src;
        ctl[0] = 1;
      }
      if constexpr (WMAX > 0) {
        if (tid < Wm) {
          nhrow[(size_t)src * Wm + tid] = 0; // the source has no next hop
        }
      }
      __syncthreads();
      qlen = ctl[0];
    }

    if (a.stats && tid == 0 && !tk2) {
      tk2 = wall_clock64();
    }
    while (qlen) {
      ++rounds;
      if (pull_first) {
        pull_first = false; // the queue holds K: straight to the PULL step
      } else {
      // ---- PUSH: changed nodes mark the neighbours they can improve or tie
      const uint32_t G = lanes_for(qlen, a.G);
      const uint32_t lg = tid & (G - 1), grp = tid / G, ngrp = kBlock / G;
      for (uint32_t i = grp; i < qlen; i += ngrp) {
        const uint32_t u = queue[i];
        if (u != src && !((tr[u >> 5] >> (u & 31)) & 1u)) {
          continue; // overloaded: recorded but never transited
        }
        const uint32_t du = dist[u];
        const uint32_t beg = a.row[u], end = a.row[u + 1];
        for (uint32_t e = beg + lg; e < end; e += G) {
          if constexpr (IGN) {
            if (ig.has(a.link[e])) {
              continue;
            }
          }
          const uint32_t v = a.col[e];
          const uint32_t c = du + (UNIT ? 1u : a.wout[e]);
          if (c <= dist[v]) {
            const uint32_t bit = 1u << (v & 31);
            if (!(act[v >> 5] & bit)) {
              atomicOr(&act[v >> 5], bit);
            }
          }
        }
      }
      __syncthreads();
      qlen = compact_bits<QT>(act, nbw, queue, ctl + 1);
      __syncthreads();
      }

      // ---- PULL: marked nodes recompute (dist, next hops) from all in-edges
      const uint32_t G = lanes_for(qlen, a.G);
      const uint32_t lg = tid & (G - 1), grp = tid / G, ngrp = kBlock / G;
      for (uint32_t i = grp; i < qlen; i += ngrp) {
        const uint32_t v = queue[i];
        const uint32_t beg = a.row[v], end = a.row[v + 1];
        uint32_t best = kInf32;
        uint64_t nh[WMAX > 0 ? WMAX : 1];
#pragma unroll
        for (int j = 0; j < (WMAX > 0 ? WMAX : 1); ++j) {
          nh[j] = 0;
        }
        for (uint32_t e = beg + lg; e < end; e += G) {
          if constexpr (IGN) {
            if (ig.has(a.link[e])) {
              continue;
            }
          }
          const uint32_t u = a.col[e];
          const bool isSrc = (u == src);
          if (!isSrc && !((tr[u >> 5] >> (u & 31)) & 1u)) {
            continue;
          }
          const uint32_t du = dist[u];
          if (du == kInf32) {
            continue;
          }
          const uint32_t c = du + (UNIT ? 1u : a.win[e]);
          if (c < best) {
            best = c;
#pragma unroll
            for (int j = 0; j < (WMAX > 0 ? WMAX : 1); ++j) {
              nh[j] = 0;
            }
          }
          if constexpr (WMAX > 0) {
            if (c == best) {
              if (isSrc) {
                // directly connected: the first hop is v itself
                const uint32_t s = a.slot[a.rev[e]];
#pragma unroll
                for (int j = 0; j < WMAX; ++j) {
                  if ((uint32_t)j == (s >> 6)) {
                    nh[j] |= 1ull << (s & 63);
                  }
                }
              } else {
                const uint64_t* p = nhrow + (size_t)u * Wm;
#pragma unroll
                for (int j = 0; j < WMAX; ++j) {
                  if ((uint32_t)j < Wm) {
                    nh[j] |= p[j];
                  }
                }
              }
            }
          }
        }
        const uint32_t gbest = grp_min(best, (int)G);
        if constexpr (WMAX > 0) {
#pragma unroll
          for (int j = 0; j < WMAX; ++j) {
            nh[j] = grp_or(best == gbest ? nh[j] : 0ull, (int)G);
          }
        }
        if (lg == 0 && gbest != kInf32) {
          const uint32_t old = dist[v];
          bool changed = gbest < old;
          uint64_t* row = nullptr;
          if constexpr (WMAX > 0) {
            row = nhrow + (size_t)v * Wm;
            if (!changed && gbest == old) {
#pragma unroll
              for (int j = 0; j < WMAX; ++j) {
                if ((uint32_t)j < Wm && row[j] != nh[j]) {
                  changed = true;
                }
              }
            }
          }
          if (changed) {
            dist[v] = gbest;
            if constexpr (WMAX > 0) {
#pragma unroll
              for (int j = 0; j < WMAX; ++j) {
                if ((uint32_t)j < Wm) {
                  row[j] = nh[j];
                }
              }
            }
            atomicOr(&chg[v >> 5], 1u << (v & 31));
          }
        }
      }
      __syncthreads();
      qlen = compact_bits<QT>(chg, nbw, queue, ctl + 1);
      __syncthreads();
    }

    unsigned long long tk3 = 0;
    if (a.stats && tid == 0) {
      tk3 = wall_clock64();
      atomicAdd(&a.stats[3], (unsigned long long)rounds);
      atomicAdd(&a.stats[6], tk3 - tk2);
    }
    if constexpr (!GMEM) {
      uint32_t* out = a.dist_out + (size_t)q * a.Vp;
      for (uint32_t v = tid; v < V; v += kBlock) {
        out[v] = dist[v];
      }
    }
    if constexpr (WMAX > 0) {
      // rows are written when a node is reached: unreached nodes get the
      // empty set here (the buffer is not cleared between runs)
      for (uint32_t v = tid; v < V; v += kBlock) {
        if (dist[v] == kInf32) {
          for (uint32_t j = 0; j < Wm; ++j) {
            nhrow[(size_t)v * Wm + j] = 0;
          }
        }
      }
    }
    __syncthreads();
    if (a.stats && tid == 0) {
      atomicAdd(&a.stats[7], wall_clock64() - tk3);
    }
  }
}

// ------------------------------------------ delta-stepping (large graphs)
//
// Weighted graphs whose per-source distance row does not fit LDS (the 100k
// WAN): the row stays in HBM (it is the output row), and the work is
// ordered by distance buckets of width 2^shift ("delta-stepping"): only
// PENDING nodes (improved, not yet pushed) whose bucket <= the current one
// push their out-edges; the marked heads PULL (min, next-hop union) from
// all their in-edges exactly as in spf_sssp_kernel.  A frontier
// Bellman-Ford re-relaxes every node each time a longer-hop but shorter
// path reaches it; bucket order pushes most nodes once.  LDS holds the
// per-node bucket byte (V B) and the pending / marked bitmaps, so 100k
// nodes take ~137 KB.  Any processing order reaches the same fixpoint, so
// the result is the order-free restatement of runSpf.
struct DstepArgs {
  SsspArgs s;
  uint32_t shift = 5; // processing bucket width 2^shift
  uint32_t fshift = 0; // LDS bucket bytes quantise d >> fshift (fshift <= shift)
  uint32_t noret = 0;  // bit 0: atomicMin without return, bit 1: coherent gathers,
                       // bit 2: bucket bytes lowered at relaxation time (no
                       // refresh reads), bit 3: no gather into unreached nodes
                       // (packed pass only; skipping every gather would mark
                       // unimproved nodes and ping-pong along tight edges)
  // OPENR_SPF_DSTEP_STATS: per-launch event counts of the push-only pass
  // (expansions, edges, bucket-filtered, gathers, atomics, improvements,
  // relax rounds, refreshed nodes)
  unsigned long long* stats = nullptr;
  // SEED (spf_table_repair): query q repairs table row row_idx[q] in place:
  // nodes whose every shortest path used a removed edge are reset first,
  // then relaxation runs from the seed nodes with the row's values
  uint32_t* table = nullptr;
  size_t pitch = 0;
  const uint32_t* row_idx = nullptr;
  const uint32_t* seed = nullptr; // tails of ADDED deltas
  uint32_t nseed = 0;
  const uint32_t* rm_tail = nullptr; // REMOVED deltas
  const uint32_t* rm_head = nullptr;
  const uint64_t* rm_w = nullptr;
  const uint32_t* rm_scope = nullptr;
  uint32_t nrem = 0;
  uint32_t* gscratch2 = nullptr; // per-workgroup second node queue (V u32)
  // packed out-edges (head | metric << cwbits), 0 bits = unpacked
  const uint32_t* cw = nullptr;
  uint32_t cwbits = 0;
  uint32_t cwvec = 0; // read cw as 16-byte chunks (padded to 4 edges)
  // PK: sources beyond the first gridDim.x are claimed from this counter
  // (zeroed per launch), so the workgroups finish together
  uint32_t* qctr = nullptr;
  // run only queries qlist[0, *qcount) (nullptr: all nq)
  const uint32_t* qlist = nullptr;
  const uint32_t* qcount = nullptr;
};


// Load that bypasses the (non-coherent) vector L1: values other lanes change
// with atomics in L2 during the same phase.
__device__ __forceinline__ uint32_t ld_coh(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Bucket of a node: the LDS byte image (LDS-resident plan) or the node's
// current distance in the HBM row (d >> shift, saturated at 254; the row is
// written by this workgroup only, and every read follows a barrier).
struct BktLds {
  const uint8_t* b;
  __device__ __forceinline__ uint32_t operator()(uint32_t v) const { return b[v]; }
};
struct BktDist {
  const uint32_t* d;
  uint32_t shift;
  __device__ __forceinline__ uint32_t operator()(uint32_t v) const {
    return min(ld_coh(d + v) >> shift, 254u);
  }
};

// pending nodes with bucket <= cur -> queue (ascending), clearing their bits
template <uint32_t BS, class BK>
__device__ __forceinline__ uint32_t compact_bucket(
    uint32_t* pend, BK bkt, uint32_t cur, uint32_t nbw,
    uint32_t* queue, uint32_t* scan) {
  const uint32_t chunk = (nbw + BS - 1) / BS;
  const uint32_t w0 = min(threadIdx.x * chunk, nbw);
  const uint32_t w1 = min(w0 + chunk, nbw);
  uint32_t cnt = 0;
  for (uint32_t w = w0; w < w1; ++w) {
    uint32_t b = pend[w];
    while (b) {
      const uint32_t k = __ffs(b) - 1;
      b &= b - 1;
      cnt += bkt(w * 32 + k) <= cur;
    }
  }
  uint32_t total;
  uint32_t off = block_excl_scan<BS>(cnt, scan, &total);
  for (uint32_t w = w0; w < w1; ++w) {
    uint32_t b = pend[w], sel = 0;
    while (b) {
      const uint32_t k = __ffs(b) - 1;
      b &= b - 1;
      if (bkt(w * 32 + k) <= cur) {
        sel |= 1u << k;
        queue[off++] = w * 32 + k;
      }
    }
    if (sel) {
      pend[w] &= ~sel;
    }
  }
  return total;
}

// smallest bucket among pending nodes (255 = none pending)
template <uint32_t BS, class BK>
__device__ __forceinline__ uint32_t min_pending_bucket(
    const uint32_t* pend, BK bkt, uint32_t nbw, uint32_t* scan) {
  constexpr uint32_t kWaves = BS / 64;
  uint32_t m = 255;
  for (uint32_t w = threadIdx.x; w < nbw; w += BS) {
    uint32_t b = pend[w];
    while (b) {
      const uint32_t k = __ffs(b) - 1;
      b &= b - 1;
      m = min(m, bkt(w * 32 + k));
    }
  }
  m = grp_min(m, 64);
  const uint32_t lane = threadIdx.x & 63u, wid = threadIdx.x >> 6;
  if (lane == 0) {
    scan[wid] = m;
  }
  __syncthreads();
  uint32_t r = 255;
  for (uint32_t i = 0; i < kWaves; ++i) {
    r = min(r, scan[i]);
  }
  __syncthreads();
  return r;
}


// Repair prologue of the seeded delta-stepping run (spf_table_repair) for
// one table row `dist` of source `src`, after edges were REMOVED (link down,
// metric increase, node overload).  Exact rule (tests/test_table_repair.py):
//  K  = heads of removed edges that were tight (d[u] + w == d[v], u in
//       scope) and everything reachable from them over tight usable edges of
//       the new graph — a superset of the nodes whose shortest paths can use
//       a removed edge (every node outside K keeps a surviving tight path);
//  ok = nodes of K reachable from outside K over tight usable edges of the
//       new graph: their distance is still achieved, so it stays exact;
//  K \ ok is reset to unreached, and every reached in-neighbour outside it
//  becomes a seed of the relaxation that follows (added to `pend`).
// `kb` / `ok` are zeroed LDS bitmaps (both zeroed again on exit), q1 / q2
// per-workgroup node queues of V entries, ctl >= 2 LDS words.
template <uint32_t BS>
__device__ void repair_invalidate(
    const DstepArgs& da, uint32_t src, uint32_t* dist, uint32_t* kb,
    uint32_t* ok, uint32_t* pend, uint32_t* q1, uint32_t* q2, uint32_t* ctl) {
  const SsspArgs& a = da.s;
  const uint32_t tid = threadIdx.x, G = a.G;
  const uint32_t lg = tid & (G - 1), grp = tid / G, ngrp = BS / G;
  auto usable = [&](uint32_t u) {
    return u == src || ((a.trbits[u >> 5] >> (u & 31)) & 1u);
  };
  if (tid == 0) {
    ctl[0] = 0;
    ctl[1] = 0;
  }
  __syncthreads();
  // heads of removed tight edges
  for (uint32_t j = tid; j < da.nrem; j += BS) {
    const uint32_t u = da.rm_tail[j], sc = da.rm_scope[j];
    if ((sc == SPF_SCOPE_TAIL_ONLY && src != u) || (sc == SPF_SCOPE_NOT_TAIL && src == u)) {
      continue;
    }
    const uint32_t du = dist[u], v = da.rm_head[j], dv = dist[v];
    if (du != kInf32 && dv != kInf32 && (uint64_t)du + da.rm_w[j] == dv && bit_claim(kb, v)) {
      q1[atomicAdd(&ctl[0], 1u)] = v;
    }
  }
  __syncthreads();
  // K: closure over tight usable edges (q1 accumulates K in BFS order)
  uint32_t lo = 0, hi = ctl[0];
  __syncthreads();
  while (lo < hi) {
    for (uint32_t i = lo + grp; i < hi; i += ngrp) {
      const uint32_t x = q1[i];
      if (!usable(x)) {
        continue;
      }
      const uint32_t dx = dist[x];
      for (uint32_t e = a.row[x] + lg; e < a.row[x + 1]; e += G) {
        const uint32_t z = a.col[e];
        if (dx + a.wout[e] == dist[z] && bit_claim(kb, z)) {
          q1[atomicAdd(&ctl[0], 1u)] = z;
        }
      }
    }
    __syncthreads();
    lo = hi;
    hi = ctl[0];
    __syncthreads();
  }
  const uint32_t nk = hi;
  // ok: K nodes with a tight usable in-edge from outside K ...
  for (uint32_t i = grp; i < nk; i += ngrp) {
    const uint32_t x = q1[i], dx = dist[x];
    for (uint32_t e = a.row[x] + lg; e < a.row[x + 1]; e += G) {
      const uint32_t y = a.col[e];
      if (bit_test(kb, y) || !usable(y)) {
        continue;
      }
      const uint32_t dy = dist[y];
      if (dy != kInf32 && dy + a.win[e] == dx && bit_claim(ok, x)) {
        q2[atomicAdd(&ctl[1], 1u)] = x;
      }
    }
  }
  __syncthreads();
  // ... and everything of K they reach over tight usable edges
  lo = 0;
  hi = ctl[1];
  __syncthreads();
  while (lo < hi) {
    for (uint32_t i = lo + grp; i < hi; i += ngrp) {
      const uint32_t x = q2[i];
      if (!usable(x)) {
        continue;
      }
      const uint32_t dx = dist[x];
      for (uint32_t e = a.row[x] + lg; e < a.row[x + 1]; e += G) {
        const uint32_t z = a.col[e];
        if (bit_test(kb, z) && dx + a.wout[e] == dist[z] && bit_claim(ok, z)) {
          q2[atomicAdd(&ctl[1], 1u)] = z;
        }
      }
    }
    __syncthreads();
    lo = hi;
    hi = ctl[1];
    __syncthreads();
  }
  // reset K \ ok; kb becomes "reset" (K \ ok) for the seed pass
  for (uint32_t i = tid; i < nk; i += BS) {
    const uint32_t x = q1[i];
    if (bit_test(ok, x)) {
      atomicAnd(&kb[x >> 5], ~(1u << (x & 31)));
    } else {
      dist[x] = kInf32;
    }
  }
  __syncthreads();
  // seeds: reached in-neighbours of reset nodes (the reset boundary)
  for (uint32_t i = grp; i < nk; i += ngrp) {
    const uint32_t x = q1[i];
    if (!bit_test(kb, x)) {
      continue;
    }
    for (uint32_t e = a.row[x] + lg; e < a.row[x + 1]; e += G) {
      const uint32_t y = a.col[e];
      if (!bit_test(kb, y) && dist[y] != kInf32) {
        atomicOr(&pend[y >> 5], 1u << (y & 31));
      }
    }
  }
  __syncthreads();
  for (uint32_t i = tid; i < nk; i += BS) {
    const uint32_t x = q1[i];
    kb[x >> 5] = 0;
    ok[x >> 5] = 0;
  }
  __syncthreads();
}

// LBK: bucket bytes in LDS (V B: one workgroup per CU on the 100k WAN);
// otherwise buckets are read from the distance row and the LDS image is the
// two bitmaps only, so several workgroups (sources) share a CU.
// PK: the tuned push-only pass compiled in (packed 16-byte edge chunks,
// coherent gathers, non-returning atomics; dstep_tune), else runtime modes.
template <int WMAX, bool IGN, uint32_t BS, bool LBK, bool SEED = false, bool PK = false>
__global__ __launch_bounds__(BS) void spf_dstep_kernel(DstepArgs da) {
  static_assert(!SEED || (WMAX == 0 && !IGN && LBK), "seeded runs are distance-only");
  static_assert(!PK || (WMAX == 0 && LBK), "the packed pass is push-only with LDS buckets");
  extern __shared__ __align__(16) uint32_t smem[];
  const SsspArgs& a = da.s;
  const uint32_t V = a.V, nbw = a.nbw, G = a.G;
  // LBK: bytes are d >> fshift and a phase takes 2^kg byte values at once;
  // buckets derived from the row use d >> shift directly
  const uint32_t shift = LBK ? da.fshift : da.shift;
  const uint32_t kg = LBK ? da.shift - da.fshift : 0;
  const uint32_t tid = threadIdx.x;
  const uint32_t lg = tid & (G - 1);
  const uint32_t grp = tid / G, ngrp = BS / G;
  uint32_t st[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const bool stats = da.stats != nullptr;

  uint32_t* act = smem;        // marked heads (PULL)
  uint32_t* pend = act + nbw;  // improved, not yet pushed
  uint32_t* ctl = pend + nbw;
  uint32_t* ignl = ctl + kCtlWords;
  uint8_t* bkt = reinterpret_cast<uint8_t*>(ignl + a.ign_cap); // LBK only
  uint32_t* queue = a.gscratch + (size_t)blockIdx.x * V;

  for (uint32_t i = tid; i < nbw; i += BS) {
    act[i] = 0;
    pend[i] = 0;
    if constexpr (SEED) {
      reinterpret_cast<uint32_t*>(bkt + ((V + 15) & ~15u))[i] = 0;
    }
  }
  __syncthreads();

  auto next_query = [&](uint32_t q) -> uint32_t {
    if (!da.qctr) {
      return q + gridDim.x;
    }
    __syncthreads(); // every lane has read ctl[kCtlWords - 2] of this query
    if (tid == 0) {
      ctl[kCtlWords - 2] = gridDim.x + atomicAdd(da.qctr, 1u);
    }
    __syncthreads();
    return ctl[kCtlWords - 2];
  };
  // qlist: only the listed queries (*qcount of them, written by an earlier
  // kernel of the stream: the LDS-row plan's overflows)
  const uint32_t nqd = da.qcount ? *da.qcount : a.nq;
  for (uint32_t qq = blockIdx.x; qq < nqd; qq = next_query(qq)) {
    const uint32_t q = da.qlist ? da.qlist[qq] : qq;
    if (a.skip && a.skip[q]) {
      continue; // uniform per block
    }
    const uint32_t src = a.src[q];
    uint32_t* dist = SEED ? da.table + (size_t)da.row_idx[q] * da.pitch
                          : a.dist_out + (size_t)q * a.Vp;
    uint32_t nign = 0;
    const uint32_t* ignp = ignl;
    if constexpr (IGN) {
      const uint32_t lo = a.ign_off[q];
      nign = a.ign_off[q + 1] - lo;
      if (nign <= a.ign_cap) {
        for (uint32_t i = tid; i < nign; i += BS) {
          ignl[i] = a.ign[lo + i];
        }
      } else {
        ignp = a.ign + lo;
      }
    }
    uint32_t Wm = 0;
    uint64_t* nhrow = nullptr;
    if constexpr (WMAX > 0) {
      Wm = a.nh_w[q];
      nhrow = a.nh_out + a.nh_off[q];
    }
    if constexpr (SEED) {
      if (da.nrem) {
        // third bitmap after the bucket bytes (SEED launches reserve it)
        uint32_t* okb = reinterpret_cast<uint32_t*>(bkt + ((V + 15) & ~15u));
        repair_invalidate<BS>(da, src, dist, act, okb, pend, queue,
                              da.gscratch2 + (size_t)blockIdx.x * V, ctl);
      }
      // every value is now an upper bound on the new distance (unchanged
      // support, or reset): bucket bytes from the row, the seeds pending;
      // relaxation only ever lowers it, to the new fixpoint
      for (uint32_t v = tid; v < V; v += BS) {
        const uint32_t dv = dist[v];
        bkt[v] = dv == kInf32 ? 255 : (uint8_t)min(dv >> shift, 254u);
      }
      __syncthreads();
      for (uint32_t i = tid; i < da.nseed; i += BS) {
        const uint32_t u = da.seed[i];
        if (dist[u] != kInf32) {
          atomicOr(&pend[u >> 5], 1u << (u & 31));
        }
      }
      __syncthreads();
    } else {
      for (uint32_t v = tid; v < V; v += BS) {
        dist[v] = kInf32;
        if constexpr (LBK) {
          bkt[v] = 255;
        }
      }
      if constexpr (WMAX > 0) {
        for (uint32_t i = tid; i < V * Wm; i += BS) {
          nhrow[i] = 0;
        }
      }
      // the row's initial stores land before any wave's atomics
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0) {
        dist[src] = 0;
        if constexpr (LBK) {
          bkt[src] = 0;
        }
        pend[src >> 5] |= 1u << (src & 31);
      }
      __syncthreads();
    }
    uint32_t cur = 0;

    for (;;) {
      uint32_t qlen;
      if (tid == 0) {
        // next queue index a group claims (the first two per group are
        // static); ordered before the relax loop by the compaction barriers
        ctl[kCtlWords - 1] = 2 * ngrp;
      }
      if constexpr (LBK) {
        qlen = compact_bucket<BS>(pend, BktLds{bkt}, cur, nbw, queue, ctl + 1);
      } else {
        qlen = compact_bucket<BS>(pend, BktDist{dist, shift}, cur, nbw, queue, ctl + 1);
      }
      __syncthreads();
      if (qlen == 0) {
        uint32_t m;
        if constexpr (LBK) {
          m = min_pending_bucket<BS>(pend, BktLds{bkt}, nbw, ctl + 1);
        } else {
          m = min_pending_bucket<BS>(pend, BktDist{dist, shift}, nbw, ctl + 1);
        }
        if (m >= 255) {
          break;
        }
        cur = min(((m >> kg) << kg) + (1u << kg) - 1u, 254u);
        continue;
      }
      if constexpr (WMAX == 0) {
        // ---- distances only: push relaxation, atomicMin into the HBM row.
        // One random access per improving edge instead of the PULL pass
        // over every in-edge of every marked head.  An improved node is
        // marked (LBK: in `act`, and its bucket byte is refreshed from one
        // coherent read of its final distance after the phase; otherwise
        // its pending bit is set and the bucket is derived from the row).
        // du is re-read coherently: a drop of dist[u] that landed before u
        // was claimed has already cleared its pending bit.  The header of a
        // group's next node (row range, du) and the id of the one after are
        // loaded while the current node's edges are in flight; a du read
        // early can only miss drops that mark u again (every improvement
        // marks its node), so it stays exact.
        uint32_t nu = grp < qlen ? queue[grp] : kInf32;
        uint32_t nbeg = 0, nend = 0, ndu = kInf32;
        if (nu != kInf32) {
          nbeg = a.row[nu];
          nend = a.row[nu + 1];
          ndu = ld_coh(dist + nu);
        }
        uint32_t nnu = grp + ngrp < qlen ? queue[grp + ngrp] : kInf32;
        // PK: groups claim further nodes from an LDS counter (a group that
        // drew light nodes takes more), so a phase ends with the last NODE,
        // not with the heaviest static share of a group
        for (uint32_t i = grp; PK ? nu != kInf32 : i < qlen; i += ngrp) {
          const uint32_t u = nu, du = ndu, beg = nbeg, end = nend;
          nu = nnu;
          if (nu != kInf32) {
            nbeg = a.row[nu];
            nend = a.row[nu + 1];
            ndu = ld_coh(dist + nu);
          }
          if constexpr (PK) {
            uint32_t nx = 0;
            if (lg == 0) {
              nx = atomicAdd(&ctl[kCtlWords - 1], 1u);
            }
            nx = (uint32_t)__shfl((int)nx, (int)((tid & 63u) & ~(G - 1u)), 64);
            nnu = nx < qlen ? queue[nx] : kInf32;
          } else {
            nnu = i + 2 * ngrp < qlen ? queue[i + 2 * ngrp] : kInf32;
          }
          if (u != src && !((a.trbits[u >> 5] >> (u & 31)) & 1u)) {
            continue; // overloaded: recorded but never transited
          }
          if (SEED && du == kInf32) {
            continue;
          }
          if (stats && lg == 0) {
            st[0] += 1;
            st[1] += end - beg;
          }
          // kPushUnroll edges per lane per step: their (head, metric) loads,
          // then their distance gathers, are independent and issued together
          constexpr uint32_t kPushUnroll = 4;
          auto relax = [&](auto& v, const auto& c) {
            constexpr uint32_t N = sizeof(v) / sizeof(v[0]);
            uint32_t dv[N];
#pragma unroll
            for (uint32_t j = 0; j < N; ++j) {
              if constexpr (LBK) {
                // bucket bytes only ever run ahead of (>=) a node's true
                // bucket, so bkt[v] < bucket(c) proves dist[v] < c: no
                // improvement, and no HBM read of dist[v]
                if (v[j] != kInf32 && bkt[v[j]] < min(c[j] >> shift, 254u)) {
                  v[j] = kInf32;
                  st[2] += stats;
                }
              }
            }
#pragma unroll
            for (uint32_t j = 0; j < N; ++j) {
              // bytes lowered in place (bit 2): 255 = nothing relaxed into v
              // yet, so d[v] is unreached or about to drop to a value a racing
              // lane is writing; atomicMin never raises, so skipping the read
              // costs at most one redundant mark
              const bool nogather = PK && (da.noret & 8u) && v[j] != kInf32 && bkt[v[j]] == 255;
              dv[j] = v[j] == kInf32 ? 0u
                      : nogather ? kInf32
                      : ((PK || (LBK && (da.noret & 2u))) ? ld_coh(dist + v[j]) : dist[v[j]]);
            }
#pragma unroll
            for (uint32_t j = 0; j < N; ++j) {
              st[3] += stats && v[j] != kInf32;
              if (v[j] == kInf32 || c[j] >= dv[j]) {
                continue;
              }
              st[4] += stats;
              if (PK || (LBK && (da.noret & 1u))) {
                // fire-and-forget: the wave does not wait for the old value;
                // a mark lost to a racing lower write only re-expands v once
                // with its current distance (the refresh below reads it)
                atomicMin(&dist[v[j]], c[j]);
                // bytes lowered in place (bit 2): the improved node goes
                // straight to the pending set (compaction only reads it after
                // the phase barrier), no refresh pass over `act`
                atomicOr(PK && (da.noret & 4u) ? &pend[v[j] >> 5] : &act[v[j] >> 5],
                         1u << (v[j] & 31));
                if constexpr (PK) {
                  if (da.noret & 4u) {
                    // d[v] <= c once the atomic lands, so bucket(c) is an
                    // upper bound of v's bucket whatever order racing lanes
                    // store in: the settled filter stays exact and sharpens
                    // within the phase
                    const uint8_t b = (uint8_t)min(c[j] >> shift, 254u);
                    if (b < bkt[v[j]]) {
                      bkt[v[j]] = b;
                    }
                  }
                }
              } else if (atomicMin(&dist[v[j]], c[j]) > c[j]) {
                st[5] += stats;
                atomicOr(LBK ? &act[v[j] >> 5] : &pend[v[j] >> 5], 1u << (v[j] & 31));
              }
            }
          };
          if (PK || da.cwvec) {
            // packed edges four at a time: lane lg takes the aligned 16-byte
            // chunks lg, lg + G, ... of [beg, end) (one load per 4 edges)
            // (PK: two chunks per lane per step, 8 edges in flight)
            const uint32_t mask = (1u << da.cwbits) - 1u;
            constexpr uint32_t kCh = PK ? 2 : 1;
            for (uint32_t k = (beg >> 2) + lg; 4 * k < end; k += kCh * G) {
              uint32_t v[4 * kCh], c[4 * kCh];
#pragma unroll
              for (uint32_t h = 0; h < kCh; ++h) {
                const uint32_t kk = k + h * G;
                const uint4 x = 4 * kk < end ? reinterpret_cast<const uint4*>(da.cw)[kk]
                                             : make_uint4(0, 0, 0, 0);
                const uint32_t xs[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
                for (uint32_t j = 0; j < 4; ++j) {
                  const uint32_t e = 4 * kk + j;
                  bool ok = e >= beg && e < end;
                  if constexpr (IGN) {
                    ok = ok && !(nign && in_sorted(ignp, nign, a.link[e]));
                  }
                  v[4 * h + j] = ok ? (xs[j] & mask) : kInf32;
                  c[4 * h + j] = ok ? du + (xs[j] >> da.cwbits) : kInf32;
                }
              }
              relax(v, c);
            }
          } else {
            for (uint32_t e0 = beg + lg; e0 < end; e0 += kPushUnroll * G) {
              uint32_t v[kPushUnroll], c[kPushUnroll];
#pragma unroll
              for (uint32_t j = 0; j < kPushUnroll; ++j) {
                const uint32_t e = e0 + j * G;
                bool ok = e < end;
                if constexpr (IGN) {
                  ok = ok && !(nign && in_sorted(ignp, nign, a.link[e]));
                }
                if (da.cwbits) {
                  const uint32_t x = ok ? da.cw[e] : 0u;
                  v[j] = ok ? (x & ((1u << da.cwbits) - 1u)) : kInf32;
                  c[j] = ok ? du + (x >> da.cwbits) : kInf32;
                } else {
                  v[j] = ok ? a.col[e] : kInf32;
                  c[j] = ok ? du + a.wout[e] : kInf32;
                }
              }
              relax(v, c);
            }
          }
        }
        // non-returning atomics of every wave reach L2 before the next
        // phase reads distances (a barrier alone drains LDS traffic only)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if constexpr (LBK) {
          // refresh straight from the marked words: each thread owns words
          // tid, tid + BS, ... (sole writer of those pend words in this
          // phase); four coherent distance reads in flight per step
          for (uint32_t w = tid; w < nbw && !(PK && (da.noret & 4u)); w += BS) {
            uint32_t b = act[w];
            if (!b) {
              continue;
            }
            act[w] = 0;
            pend[w] |= b;
            st[7] += stats ? __popc(b) : 0u;
            while (b) {
              uint32_t vs[4], dd[4];
#pragma unroll
              for (uint32_t j = 0; j < 4; ++j) {
                vs[j] = kInf32;
                if (b) {
                  vs[j] = w * 32 + (__ffs(b) - 1);
                  b &= b - 1;
                }
              }
#pragma unroll
              for (uint32_t j = 0; j < 4; ++j) {
                dd[j] = vs[j] != kInf32 ? ld_coh(dist + vs[j]) : 0u;
              }
#pragma unroll
              for (uint32_t j = 0; j < 4; ++j) {
                if (vs[j] != kInf32) {
                  bkt[vs[j]] = (uint8_t)min(dd[j] >> shift, 254u);
                }
              }
            }
          }
          st[6] += stats && tid == 0;
          if (!(PK && (da.noret & 4u))) {
            __syncthreads(); // refresh pass ran (uniform condition)
          }
        }
        continue;
      }
      // ---- PUSH from the selected bucket
      for (uint32_t i = grp; i < qlen; i += ngrp) {
        const uint32_t u = queue[i];
        if (u != src && !((a.trbits[u >> 5] >> (u & 31)) & 1u)) {
          continue; // overloaded: recorded but never transited
        }
        const uint32_t du = dist[u];
        const uint32_t beg = a.row[u], end = a.row[u + 1];
        for (uint32_t e = beg + lg; e < end; e += G) {
          if constexpr (IGN) {
            if (nign && in_sorted(ignp, nign, a.link[e])) {
              continue;
            }
          }
          const uint32_t v = a.col[e];
          const uint32_t c = du + a.wout[e];
          if constexpr (LBK) {
            // bkt[v] >= v's true bucket: bkt[v] < bucket(c) proves
            // dist[v] < c (neither an improvement nor a tie)
            if (bkt[v] < min(c >> shift, 254u)) {
              continue;
            }
          }
          if (c <= dist[v]) {
            const uint32_t bit = 1u << (v & 31);
            if (!(act[v >> 5] & bit)) {
              atomicOr(&act[v >> 5], bit);
            }
          }
        }
      }
      __syncthreads();
      qlen = compact_bits<uint32_t, BS>(act, nbw, queue, ctl + 1);
      __syncthreads();

      // ---- PULL: marked heads recompute (dist, next hops) from all in-edges
      for (uint32_t i = grp; i < qlen; i += ngrp) {
        const uint32_t v = queue[i];
        const uint32_t beg = a.row[v], end = a.row[v + 1];
        uint32_t best = kInf32;
        uint64_t nh[WMAX > 0 ? WMAX : 1];
#pragma unroll
        for (int j = 0; j < (WMAX > 0 ? WMAX : 1); ++j) {
          nh[j] = 0;
        }
        for (uint32_t e = beg + lg; e < end; e += G) {
          if constexpr (IGN) {
            if (nign && in_sorted(ignp, nign, a.link[e])) {
              continue;
            }
          }
          const uint32_t u = a.col[e];
          const bool isSrc = (u == src);
          if (!isSrc && !((a.trbits[u >> 5] >> (u & 31)) & 1u)) {
            continue;
          }
          const uint32_t du = dist[u];
          if (du == kInf32) {
            continue;
          }
          const uint32_t c = du + a.win[e];
          if (c < best) {
            best = c;
#pragma unroll
            for (int j = 0; j < (WMAX > 0 ? WMAX : 1); ++j) {
              nh[j] = 0;
            }
          }
          if constexpr (WMAX > 0) {
            if (c == best) {
              if (isSrc) {
                const uint32_t s = a.slot[a.rev[e]];
#pragma unroll
                for (int j = 0; j < WMAX; ++j) {
                  if ((uint32_t)j == (s >> 6)) {
                    nh[j] |= 1ull << (s & 63);
                  }
                }
              } else {
                const uint64_t* p = nhrow + (size_t)u * Wm;
#pragma unroll
                for (int j = 0; j < WMAX; ++j) {
                  if ((uint32_t)j < Wm) {
                    nh[j] |= p[j];
                  }
                }
              }
            }
          }
        }
        const uint32_t gbest = grp_min(best, (int)G);
        if constexpr (WMAX > 0) {
#pragma unroll
          for (int j = 0; j < WMAX; ++j) {
            nh[j] = grp_or(best == gbest ? nh[j] : 0ull, (int)G);
          }
        }
        if (lg == 0 && gbest != kInf32) {
          const uint32_t old = dist[v];
          bool changed = gbest < old;
          uint64_t* row = nullptr;
          if constexpr (WMAX > 0) {
            row = nhrow + (size_t)v * Wm;
            if (!changed && gbest == old) {
#pragma unroll
              for (int j = 0; j < WMAX; ++j) {
                if ((uint32_t)j < Wm && row[j] != nh[j]) {
                  changed = true;
                }
              }
            }
          }
          if (changed) {
            dist[v] = gbest;
            if constexpr (LBK) {
              bkt[v] = (uint8_t)min(gbest >> shift, 254u);
            }
            if constexpr (WMAX > 0) {
#pragma unroll
              for (int j = 0; j < WMAX; ++j) {
                if ((uint32_t)j < Wm) {
                  row[j] = nh[j];
                }
              }
            }
            atomicOr(&pend[v >> 5], 1u << (v & 31));
          }
        }
      }
      __syncthreads();
    }
    __syncthreads();
  }
  if (stats) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      if (st[k]) {
        atomicAdd(&da.stats[k], (unsigned long long)st[k]);
      }
    }
  }
}

// ----------------- LDS-resident delta-stepping (distance rows, 12-bit fields)
//
// The push-only pass above keeps the distance row in HBM: every relaxation
// that the LDS bucket byte cannot decide gathers d[v] and improves it with
// an HBM atomicMin (360k gathers + 278k atomics per SSSP on the 100k WAN,
// 2.9x the algorithmic bytes).  When every distance a run can hold is small
// (the WAN: metrics <= 1,000, eccentricity ~1,200) the whole row fits LDS as
// 12-bit fields, five per 64-bit word (V <= 104k in 160 KB): relaxation is
// then an LDS read + compare-and-swap, and HBM sees only the CSR stream and
// one coalesced row store per source.
//
// Field value f: the node's tentative distance (0..kDlMaxDist), kDlUnreached
// = not reached.  Buckets [lo, lo + width) are processed in order:
//   SCAN   every field in [lo, hi] -> queue (two passes + block scan); none:
//          jump lo to the smallest field above hi (none: done);
//   EXPAND queued node u (the source, or a transit node: LinkState.cpp:829-836)
//          relaxes its packed out-edges: c = f(u) + w; c < f(v) -> CAS the
//          field down; a node lowered into [lo, hi] is queued again (the
//          light-edge re-expansion of delta-stepping).  Phases repeat until no
//          node of the bucket was lowered.
// Values only decrease and every lowered node of the bucket is expanded
// after its last drop, so the loop ends at the same fixpoint as runSpf
// (Dijkstra where only the source or non-overloaded nodes
// relax).  A relaxation that would store a value above kDlMaxDist into an
// unreached node flags the source: its row is recomputed by the HBM-row
// kernel (DstepArgs::qlist), so the plan is exact for any graph.
constexpr uint32_t kDlUnreached = 0xFFFu;
constexpr uint32_t kDlMaxDist = 0xFFEu;
constexpr uint64_t kDlEmptyWord = 0x0FFFFFFFFFFFFFFFull; // five unreached fields
constexpr uint32_t kDlCtl = 40; // control words after the field image

struct DldsArgs {
  const uint32_t* row;
  const uint32_t* cw; // head | metric << cwbits, padded to 16-byte chunks
  const uint32_t* trbits;
  const uint32_t* src;
  uint32_t* dist_out;  // [nq][Vp]
  uint32_t* gscratch;  // [grid][2 * V] node queues
  uint32_t* ovf_list;  // [nq] queries whose values left the 12-bit range
  uint32_t* ovf_n;     // (count)
  uint32_t* qctr;      // source-claim counter (zeroed per launch)
  unsigned long long* stats; // OPENR_SPF_DSTEP_STATS (8 counters) or nullptr
  uint32_t V, Vp, nq, cwbits, wshift;
};

__device__ __forceinline__ uint32_t dl_field(uint64_t x, uint32_t k) {
  return (uint32_t)(x >> (12 * k)) & 0xFFFu;
}

template <uint32_t BS, uint32_t G, bool PF>
__global__ __launch_bounds__(BS) void spf_dlds_kernel(DldsArgs a) {
  extern __shared__ __align__(16) uint64_t fld[];
  const uint32_t V = a.V, nw = (V + 4) / 5;
  uint32_t* ctl = reinterpret_cast<uint32_t*>(fld + nw);
  // ctl[0..2] appended-node counters (rotating by phase), [3] overflow flag,
  // [4] claimed query, [8, 8 + 2 * waves) scan scratch
  uint32_t* scan = ctl + 8;
  constexpr uint32_t kWv = BS / 64;
  constexpr uint32_t ngrp = BS / G; // G lanes per expanded node
  const uint32_t tid = threadIdx.x, lg = tid & (G - 1), grp = tid / G;
  const uint32_t mask = (1u << a.cwbits) - 1u, width = 1u << a.wshift;
  uint32_t* qa = a.gscratch + (size_t)blockIdx.x * 2 * V;
  uint32_t* qb = qa + V;
  const bool stats = a.stats != nullptr;
  uint32_t st[8] = {0, 0, 0, 0, 0, 0, 0, 0};

  auto ld = [&](uint32_t w) -> uint64_t {
    return __hip_atomic_load(fld + w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  };

  uint32_t q = blockIdx.x;
  while (q < a.nq) {
    const uint32_t src = a.src[q];
    for (uint32_t w = tid; w < nw; w += BS) {
      fld[w] = kDlEmptyWord;
    }
    if (tid < 4) {
      ctl[tid] = 0;
    }
    __syncthreads();
    if (tid == 0) {
      const uint32_t w = src / 5, k = src % 5;
      fld[w] &= ~(0xFFFull << (12 * k));
    }
    __syncthreads();
    uint32_t lo = 0, len = 0, ph = 0;
    bool rescan = true;
    uint32_t* qc = qa;
    uint32_t* qn = qb;
    for (;;) {
      const uint32_t hi = min(lo + width - 1u, kDlMaxDist);
      if (rescan) {
        // SCAN pass 1: fields in [lo, hi], smallest field above hi
        uint32_t cnt = 0, mn = kInf32;
        for (uint32_t w = tid; w < nw; w += BS) {
          const uint64_t x = fld[w];
#pragma unroll
          for (uint32_t k = 0; k < 5; ++k) {
            const uint32_t f = dl_field(x, k);
            cnt += f >= lo && f <= hi;
            if (f > hi && f != kDlUnreached) {
              mn = min(mn, f);
            }
          }
        }
        mn = grp_min(mn, 64);
        if ((tid & 63u) == 0) {
          scan[kWv + (tid >> 6)] = mn;
        }
        uint32_t total;
        uint32_t off = block_excl_scan<BS>(cnt, scan, &total);
        if (total == 0) {
          uint32_t m = kInf32;
#pragma unroll
          for (uint32_t i = 0; i < kWv; ++i) {
            m = min(m, scan[kWv + i]);
          }
          __syncthreads(); // scan scratch reused by the next pass
          if (m == kInf32) {
            break;
          }
          lo = m & ~(width - 1u);
          continue;
        }
        // SCAN pass 2: the bucket's nodes -> qa
        for (uint32_t w = tid; w < nw; w += BS) {
          const uint64_t x = fld[w];
#pragma unroll
          for (uint32_t k = 0; k < 5; ++k) {
            const uint32_t f = dl_field(x, k);
            if (f >= lo && f <= hi) {
              qa[off++] = 5 * w + k;
            }
          }
        }
        st[6] += stats && tid == 0;
        qc = qa;
        qn = qb;
        len = total;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
      }
      // EXPAND qc[0, len).  PF: a group keeps two nodes ahead in flight —
      // the next node's edge chunks and the one after's row range are loaded
      // before the current node's relaxations (LDS work) run, so a group
      // waits for at most one HBM round trip per node instead of two
      // (header, then chunks); without PF only the next header is early.
      uint32_t* cnt = ctl + ph;
      {
        // relax the (up to) 8 edges of a lane's two chunks of node u
        auto relax_chunks = [&](const uint4 (&x)[2], uint32_t kc, uint32_t beg, uint32_t end,
                                uint32_t du) {
          uint32_t v[8], c[8];
#pragma unroll
          for (uint32_t h = 0; h < 2; ++h) {
            const uint32_t kk = kc + h * G;
            const uint32_t xs[4] = {x[h].x, x[h].y, x[h].z, x[h].w};
#pragma unroll
            for (uint32_t j = 0; j < 4; ++j) {
              const uint32_t e = 4 * kk + j;
              const bool ok = e >= beg && e < end;
              v[4 * h + j] = ok ? (xs[j] & mask) : kInf32;
              c[4 * h + j] = du + (xs[j] >> a.cwbits);
            }
          }
          uint64_t old[8];
#pragma unroll
          for (uint32_t j = 0; j < 8; ++j) {
            old[j] = v[j] != kInf32 ? ld(v[j] / 5) : 0ull;
          }
#pragma unroll
          for (uint32_t j = 0; j < 8; ++j) {
            if (v[j] == kInf32) {
              continue;
            }
            const uint32_t w = v[j] / 5, sh = 12 * (v[j] % 5);
            uint64_t o = old[j];
            uint32_t cur = (uint32_t)(o >> sh) & 0xFFFu;
            if (c[j] > kDlMaxDist) {
              // an unreached node whose first value does not fit 12 bits:
              // the source's row goes to the HBM-row pass (a reached node
              // holds a smaller value, so c is no improvement there)
              if (cur == kDlUnreached) {
                ctl[3] = 1;
              }
              continue;
            }
            if (c[j] >= cur) {
              continue;
            }
            bool done = false;
            while (!done && c[j] < cur) {
              const uint64_t nv = (o & ~(0xFFFull << sh)) | ((uint64_t)c[j] << sh);
              const uint64_t p = atomicCAS((unsigned long long*)(fld + w),
                                           (unsigned long long)o, (unsigned long long)nv);
              done = p == o;
              o = p;
              cur = (uint32_t)(o >> sh) & 0xFFFu;
            }
            st[4] += stats;
            if (done) {
              st[5] += stats;
              if (c[j] <= hi) {
                // lowered into the bucket: expanded again next phase (a
                // full queue drops the id; the bucket is rescanned then)
                const uint32_t slot = atomicAdd(cnt, 1u);
                if (slot < V) {
                  qn[slot] = v[j];
                }
              }
            }
          }
        };
        auto load_chunks = [&](uint32_t kc, uint32_t end, uint4 (&x)[2]) {
#pragma unroll
          for (uint32_t h = 0; h < 2; ++h) {
            const uint32_t kk = kc + h * G;
            x[h] = 4 * kk < end ? reinterpret_cast<const uint4*>(a.cw)[kk] : make_uint4(0, 0, 0, 0);
          }
        };
        // the source, or a transit node (overloaded: recorded, never transited)
        auto expands = [&](uint32_t u, uint32_t trb) {
          return u == src || ((trb >> (u & 31)) & 1u);
        };
        uint32_t i = grp;
        uint32_t u = i < len ? qc[i] : kInf32;
        uint32_t nu = i + ngrp < len ? qc[i + ngrp] : kInf32;
        uint32_t beg = 0, end = 0, trb = 0;
        if (u != kInf32) {
          beg = a.row[u];
          end = a.row[u + 1];
          trb = a.trbits[u >> 5];
        }
        uint4 xc[2] = {make_uint4(0, 0, 0, 0), make_uint4(0, 0, 0, 0)};
        uint32_t nbeg = 0, nend = 0, ntrb = 0;
        if constexpr (PF) {
          if (u != kInf32 && expands(u, trb)) {
            load_chunks((beg >> 2) + lg, end, xc);
          }
          if (nu != kInf32) {
            nbeg = a.row[nu];
            nend = a.row[nu + 1];
            ntrb = a.trbits[nu >> 5];
          }
        }
        while (u != kInf32) {
          const uint32_t nnu = i + 2 * ngrp < len ? qc[i + 2 * ngrp] : kInf32;
          uint4 xn[2] = {make_uint4(0, 0, 0, 0), make_uint4(0, 0, 0, 0)};
          uint32_t bb = 0, ee = 0, tt = 0; // the node after next (PF), else the next
          if constexpr (PF) {
            if (nu != kInf32 && expands(nu, ntrb)) {
              load_chunks((nbeg >> 2) + lg, nend, xn);
            }
            if (nnu != kInf32) {
              bb = a.row[nnu];
              ee = a.row[nnu + 1];
              tt = a.trbits[nnu >> 5];
            }
          } else if (nu != kInf32) {
            bb = a.row[nu];
            ee = a.row[nu + 1];
            tt = a.trbits[nu >> 5];
          }
          if (expands(u, trb)) {
            const uint32_t du = dl_field(ld(u / 5), u % 5);
            if (stats && lg == 0) {
              st[0] += 1;
              st[1] += end - beg;
            }
            uint32_t kc = (beg >> 2) + lg;
            if constexpr (PF) {
              relax_chunks(xc, kc, beg, end, du);
              kc += 2 * G;
            }
            for (; 4 * kc < end; kc += 2 * G) {
              uint4 x[2];
              load_chunks(kc, end, x);
              relax_chunks(x, kc, beg, end, du);
            }
          }
          i += ngrp;
          u = nu;
          nu = nnu;
          if constexpr (PF) {
            beg = nbeg;
            end = nend;
            trb = ntrb;
            nbeg = bb;
            nend = ee;
            ntrb = tt;
            xc[0] = xn[0];
            xc[1] = xn[1];
          } else {
            beg = bb;
            end = ee;
            trb = tt;
          }
        }
      }
      // the next phase's counter was last read two phases ago (before the
      // previous phase's barrier): clear it for the next phase
      const uint32_t ph2 = ph == 2 ? 0u : ph + 1u;
      if (tid == 0) {
        ctl[ph2] = 0;
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      const uint32_t n = *cnt;
      ph = ph2;
      st[7] += stats && tid == 0 ? n : 0u;
      if (n == 0) {
        // bucket settled
        if (hi >= kDlMaxDist) {
          break;
        }
        lo = hi + 1;
        rescan = true;
      } else if (n > V) {
        rescan = true; // queue overflowed: the whole bucket again
      } else {
        uint32_t* t = qc;
        qc = qn;
        qn = t;
        len = n;
        rescan = false;
      }
    }
    // the row: 16-byte stores of four nodes per lane
    uint32_t* drow = a.dist_out + (size_t)q * a.Vp;
    for (uint32_t v0 = 4 * tid; v0 < V; v0 += 4 * BS) {
      uint32_t r[4];
#pragma unroll
      for (uint32_t j = 0; j < 4; ++j) {
        const uint32_t v = v0 + j;
        const uint32_t f = v < V ? dl_field(fld[v / 5], v % 5) : kDlUnreached;
        r[j] = f == kDlUnreached ? kInf32 : f;
      }
      *reinterpret_cast<uint4*>(drow + v0) = make_uint4(r[0], r[1], r[2], r[3]);
    }
    __syncthreads(); // every lane read the fields and the overflow flag
    if (tid == 0) {
      if (ctl[3]) {
        a.ovf_list[atomicAdd(a.ovf_n, 1u)] = q;
      }
      ctl[4] = gridDim.x + atomicAdd(a.qctr, 1u);
    }
    __syncthreads();
    q = ctl[4];
    __syncthreads();
  }
  if (stats) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      if (st[k]) {
        atomicAdd(&a.stats[k], (unsigned long long)st[k]);
      }
    }
  }
}

// ------------------------- multi-source delta-stepping (distance rows only)
//
// Many-source distance rows on weighted graphs whose row does not fit LDS
// (the 100k WAN all-sources pass).  One workgroup solves a BATCH of
// kMsdK = 32 sources at once over a node-major slab D[v][32] in HBM — one
// 128-byte line per node — so relaxing an edge u->x fetches ONE line of x
// and serves every source of the batch whose (u, s) is being expanded, where
// a per-source kernel fetches a whole line per (edge, source) and uses 4 B of
// it.  The host groups graph-near sources into a batch (spf_query_create),
// which keeps their bucket fronts aligned so most lanes of a line do work.
//
// State per batch: D (global slab), pend[v] (global, bit s = D[v][s] dropped
// and not yet expanded), bmin[v] (LDS byte: smallest bucket d >> shift among
// v's pending lanes, 255 = none) and a dirty bitmap (LDS).  Loop over
// buckets `cur`:
//   CLAIM  for each candidate node (nodes dirtied by the last RELAX, or — when
//          that leaves nothing in bucket cur — every node whose bmin is the
//          next smallest bucket): pending lanes whose bucket <= cur are
//          claimed (bits cleared) and queued with their lane mask (overloaded
//          nodes keep only the lanes they are the source of), bmin is
//          recomputed over the remaining lanes;
//   RELAX  every queued (v, mask) relaxes v's out-edges for the lanes of the
//          mask: c = D[v][s] + w; atomicMin(D[x][s], c); a drop sets
//          pend[x] bit s and dirty[x].
// The two phases are barrier-separated, so a pend bit is never set and
// cleared concurrently; every drop of D[v][s] is followed by its pend bit and
// every claimed lane is expanded with its CURRENT D[v][s] (<= the claimed
// value).  The loop therefore ends at the unique fixpoint: Dijkstra distances
// in which only the source or non-overloaded nodes relax (LinkState.cpp:
// 806-880).  Reads of D / pend whose value decides a claim or
// an expansion bypass the (non-coherent) vector L1 (agent-scope atomic loads).
constexpr uint32_t kMsdK = 32;     // sources per batch = lanes per node line
constexpr uint32_t kMsdTile = 128; // nodes per LDS transpose tile (row write)

struct MsdArgs {
  const uint32_t* row;
  const uint32_t* col;
  const uint32_t* wout;
  const uint32_t* trbits;
  const uint32_t* src;  // [nq] source node of query i
  const uint32_t* perm; // [nbatch * 32] query of each batch lane (~0 = none)
  uint32_t* dist_out;   // [nq][Vp]
  uint32_t* slab;       // [grid][V][32]
  uint32_t* pend;       // [grid][V]
  uint32_t* qa;         // [grid][V] candidate nodes
  uint32_t* qb;         // [grid][V] claimed nodes
  uint32_t* qm;         // [grid][V] claimed lane masks
  uint32_t V;
  uint32_t Vp;
  uint32_t nbw;
  uint32_t nbatch;
  uint32_t shift; // bucket width 2^shift
};


__device__ __forceinline__ uint32_t min4b(uint32_t x) {
  return min(min(x & 255u, (x >> 8) & 255u), min((x >> 16) & 255u, x >> 24));
}

// smallest bmin byte over the (255-padded) array
template <uint32_t BS>
__device__ __forceinline__ uint32_t msd_min_bucket(
    const uint32_t* bw, uint32_t nw, uint32_t* scan) {
  constexpr uint32_t kW = BS / 64;
  uint32_t m = 255;
  for (uint32_t i = threadIdx.x; i < nw; i += BS) {
    m = min(m, min4b(bw[i]));
  }
  m = grp_min(m, 64);
  if ((threadIdx.x & 63u) == 0) {
    scan[threadIdx.x >> 6] = m;
  }
  __syncthreads();
  uint32_t r = 255;
#pragma unroll
  for (uint32_t i = 0; i < kW; ++i) {
    r = min(r, scan[i]);
  }
  __syncthreads();
  return r;
}

// nodes whose bmin byte is <= cur -> queue (ascending)
template <uint32_t BS>
__device__ __forceinline__ uint32_t msd_compact_le(
    const uint32_t* bw, uint32_t nw, uint32_t cur, uint32_t* queue,
    uint32_t* scan) {
  const uint32_t chunk = (nw + BS - 1) / BS;
  const uint32_t w0 = min(threadIdx.x * chunk, nw);
  const uint32_t w1 = min(w0 + chunk, nw);
  uint32_t cnt = 0;
  for (uint32_t w = w0; w < w1; ++w) {
    const uint32_t x = bw[w];
#pragma unroll
    for (uint32_t k = 0; k < 4; ++k) {
      cnt += ((x >> (8 * k)) & 255u) <= cur;
    }
  }
  uint32_t total;
  uint32_t off = block_excl_scan<BS>(cnt, scan, &total);
  for (uint32_t w = w0; w < w1; ++w) {
    const uint32_t x = bw[w];
#pragma unroll
    for (uint32_t k = 0; k < 4; ++k) {
      if (((x >> (8 * k)) & 255u) <= cur) {
        queue[off++] = w * 4 + k;
      }
    }
  }
  return total;
}

template <uint32_t BS>
__global__ __launch_bounds__(BS) void spf_msdstep_kernel(MsdArgs a) {
  extern __shared__ __align__(16) uint32_t smem[];
  constexpr uint32_t kW = BS / 64;
  const uint32_t V = a.V, nbw = a.nbw, shift = a.shift, tid = threadIdx.x;
  const uint32_t lane = tid & 63u, wid = tid >> 6, s = tid & 31u;
  const uint32_t half = lane >> 5;
  const uint32_t nw = (V + 3) / 4; // bmin words
  uint32_t* ctl = smem;              // [0] claimed count, [1..] scan scratch
  uint32_t* dirty = ctl + kCtlWords; // [nbw]
  uint32_t* tile = dirty + nbw;      // [32][kMsdTile + 1]
  uint32_t* bw = tile + kMsdK * (kMsdTile + 1);
  uint8_t* bmin = reinterpret_cast<uint8_t*>(bw);
  uint32_t* D = a.slab + (size_t)blockIdx.x * V * kMsdK;
  uint32_t* pend = a.pend + (size_t)blockIdx.x * V;
  uint32_t* qa = a.qa + (size_t)blockIdx.x * V;
  uint32_t* qb = a.qb + (size_t)blockIdx.x * V;
  uint32_t* qm = a.qm + (size_t)blockIdx.x * V;

  for (uint32_t i = tid; i < nbw; i += BS) {
    dirty[i] = 0;
  }
  if (tid == 0) {
    ctl[0] = 0;
  }

  for (uint32_t b = blockIdx.x; b < a.nbatch; b += gridDim.x) {
    const uint32_t myq = a.perm[b * kMsdK + s];
    const uint32_t mysrc = myq != kInf32 ? a.src[myq] : kInf32;
    // reset the slab, the pending masks and the buckets
    {
      uint4* D4 = reinterpret_cast<uint4*>(D);
      const uint4 inf4 = make_uint4(kInf32, kInf32, kInf32, kInf32);
      const size_t n4 = (size_t)V * (kMsdK / 4);
      for (size_t i = tid; i < n4; i += BS) {
        D4[i] = inf4;
      }
      for (uint32_t v = tid; v < V; v += BS) {
        pend[v] = 0;
      }
      for (uint32_t i = tid; i < nw; i += BS) {
        bw[i] = 0xFFFFFFFFu;
      }
    }
    __threadfence();
    __syncthreads();
    if (tid < kMsdK && mysrc != kInf32) {
      atomicMin(&D[(size_t)mysrc * kMsdK + s], 0u);
      atomicOr(&pend[mysrc], 1u << s);
      bmin[mysrc] = 0;
    }
    __threadfence();
    __syncthreads();

    uint32_t cur = 0;
    bool from_scan = true;
    for (;;) {
      // ---- candidates
      uint32_t na;
      if (from_scan) {
        const uint32_t m = msd_min_bucket<BS>(bw, nw, ctl + 1);
        if (m >= 255) {
          break;
        }
        cur = m;
        na = msd_compact_le<BS>(bw, nw, cur, qa, ctl + 1);
      } else {
        na = compact_bits<uint32_t, BS>(dirty, nbw, qa, ctl + 1);
      }
      __threadfence();
      __syncthreads();
      // ---- CLAIM: one half-wave per candidate node, lane = source slot
      for (uint32_t i = wid * 2 + half; i < na; i += kW * 2) {
        const uint32_t v = qa[i];
        const uint32_t pm = ld_coh(&pend[v]);
        const bool pl = (pm >> s) & 1u;
        uint32_t bk = 255;
        if (pl) {
          bk = min(ld_coh(&D[(size_t)v * kMsdK + s]) >> shift, 254u);
        }
        const bool el = pl && bk <= cur;
        const uint32_t em = (uint32_t)(__ballot(el) >> (half * 32));
        const uint32_t eqm = (uint32_t)(__ballot(mysrc == v) >> (half * 32));
        const uint32_t rest = grp_min((pl && !el) ? bk : 255u, 32);
        if (s == 0) {
          bmin[v] = (uint8_t)rest;
          if (em) {
            atomicAnd(&pend[v], ~em);
            const bool transit = (a.trbits[v >> 5] >> (v & 31)) & 1u;
            const uint32_t xm = transit ? em : (em & eqm);
            if (xm) {
              const uint32_t k = atomicAdd(&ctl[0], 1u);
              qb[k] = v;
              qm[k] = xm;
            }
          }
        }
      }
      __threadfence();
      __syncthreads();
      const uint32_t nb = ctl[0];
      __syncthreads();
      if (nb == 0) {
        from_scan = true;
        continue;
      }
      if (tid == 0) {
        ctl[0] = 0; // next CLAIM starts after the barrier closing RELAX
      }
      // ---- RELAX: one wave per claimed node, half-waves take alternate
      // edges, 4 edges per half-wave in flight
      for (uint32_t i = wid; i < nb; i += kW) {
        const uint32_t v = qb[i], m = qm[i];
        const bool act = (m >> s) & 1u;
        const uint32_t dv = act ? ld_coh(&D[(size_t)v * kMsdK + s]) : kInf32;
        const uint32_t beg = a.row[v], end = a.row[v + 1];
        for (uint32_t e0 = beg; e0 < end; e0 += 8) {
          uint32_t x[4], w[4], old[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const uint32_t e = e0 + half + 2 * j;
            x[j] = e < end ? a.col[e] : kInf32;
            w[j] = e < end ? a.wout[e] : 0u;
          }
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            old[j] = (act && x[j] != kInf32) ? D[(size_t)x[j] * kMsdK + s] : 0u;
          }
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            bool imp = false;
            if (act && x[j] != kInf32) {
              const uint32_t c = dv + w[j];
              if (c < old[j]) {
                imp = atomicMin(&D[(size_t)x[j] * kMsdK + s], c) > c;
              }
            }
            const uint32_t im = (uint32_t)(__ballot(imp) >> (half * 32));
            if (im && s == 0) {
              atomicOr(&pend[x[j]], im);
              atomicOr(&dirty[x[j] >> 5], 1u << (x[j] & 31));
            }
          }
        }
      }
      __threadfence();
      __syncthreads();
      from_scan = false;
    }

    // ---- rows out: D[v][s] -> dist_out[query of s][v], via LDS tiles
    for (uint32_t v0 = 0; v0 < V; v0 += kMsdTile) {
      for (uint32_t i = tid; i < kMsdTile * kMsdK; i += BS) {
        const uint32_t vv = i / kMsdK, ss = i % kMsdK, v = v0 + vv;
        tile[ss * (kMsdTile + 1) + vv] =
            v < V ? ld_coh(&D[(size_t)v * kMsdK + ss]) : kInf32;
      }
      __syncthreads();
      for (uint32_t i = tid; i < kMsdTile * kMsdK; i += BS) {
        const uint32_t ss = i / kMsdTile, vv = i % kMsdTile, v = v0 + vv;
        const uint32_t q = a.perm[b * kMsdK + ss];
        if (q != kInf32 && v < V) {
          a.dist_out[(size_t)q * a.Vp + v] = tile[ss * (kMsdTile + 1) + vv];
        }
      }
      __syncthreads();
    }
  }
}

// ------------------------------------------- uniform-metric distance kernel
//
// Every usable link has the same metric c (the fabric and grid benchmarks,
// and every useLinkMetric=false run): distances are c * BFS levels.  One
// workgroup per source, direction-optimizing level-synchronous BFS in LDS:
// top-down (frontier rows pushed, first writer wins with an identical value)
// while the frontier is small, bottom-up (each unvisited node scans its own
// row and stops at the first transit frontier neighbour) once the frontier's
// edges outnumber the unvisited edges / 14.  Overloaded nodes are reached
// but never expanded, exactly as the reference (LinkState.cpp:829-836).

struct BfsArgs {
  const uint32_t* row;
  const uint32_t* col;
  const uint32_t* trbits;
  const uint32_t* src;
  uint32_t* dist_out;
  uint32_t* gscratch;
  uint32_t V;
  uint32_t Vp; // row stride of dist_out
  uint32_t nbw;
  uint32_t nq;
  uint32_t E;
  uint32_t G;
  uint32_t scale; // the uniform metric c
};

// next-frontier bitmap -> queue; cur = next; next = 0; returns the queue
// length, *degsum = sum of out-degrees of the queued nodes.
template <typename QT>
__device__ __forceinline__ uint32_t compact_frontier(
    uint32_t* nxt, uint32_t* cur, uint32_t nbw, QT* queue, uint32_t* scan,
    const uint32_t* row, uint32_t* degsum) {
  const uint32_t chunk = (nbw + kBlock - 1) / kBlock;
  const uint32_t w0 = min(threadIdx.x * chunk, nbw);
  const uint32_t w1 = min(w0 + chunk, nbw);
  uint32_t cnt = 0;
  for (uint32_t w = w0; w < w1; ++w) {
    cnt += __popc(nxt[w]);
  }
  uint32_t total;
  uint32_t off = block_excl_scan(cnt, scan, &total);
  uint32_t deg = 0;
  for (uint32_t w = w0; w < w1; ++w) {
    uint32_t b = nxt[w];
    cur[w] = b;
    nxt[w] = 0;
    while (b) {
      const uint32_t k = __ffs(b) - 1;
      b &= b - 1;
      const uint32_t v = w * 32 + k;
      queue[off++] = (QT)v;
      deg += row[v + 1] - row[v];
    }
  }
  __syncthreads();
  uint32_t dtot;
  block_excl_scan(deg, scan, &dtot);
  *degsum = dtot;
  return total;
}

template <bool GMEM>
__global__ __launch_bounds__(kBlock) void spf_bfs_kernel(BfsArgs a) {
  extern __shared__ __align__(16) uint32_t smem[];
  using QT = typename std::conditional<GMEM, uint32_t, uint16_t>::type;
  const uint32_t V = a.V, nbw = a.nbw, G = a.G;
  const uint32_t tid = threadIdx.x;
  const uint32_t lg = tid & (G - 1);
  const uint32_t grp = tid / G, ngrp = kBlock / G;

  uint32_t* cur = smem;
  uint32_t* nxt = cur + nbw;
  uint32_t* tr = nxt + nbw;
  uint32_t* ctl = tr + nbw;
  QT* queue;
  uint32_t* dist;
  if constexpr (GMEM) {
    queue = a.gscratch + (size_t)blockIdx.x * V;
    dist = nullptr;
  } else {
    queue = reinterpret_cast<QT*>(ctl + kCtlWords);
    dist = reinterpret_cast<uint32_t*>(queue + ((V + 1) & ~1u));
  }
  for (uint32_t i = tid; i < nbw; i += kBlock) {
    cur[i] = 0;
    nxt[i] = 0;
    tr[i] = a.trbits[i];
  }

  for (uint32_t q = blockIdx.x; q < a.nq; q += gridDim.x) {
    const uint32_t src = a.src[q];
    if constexpr (GMEM) {
      dist = a.dist_out + (size_t)q * a.Vp;
    }
    for (uint32_t v = tid; v < V; v += kBlock) {
      dist[v] = kInf32;
    }
    __syncthreads();
    if (tid == 0) {
      dist[src] = 0;
      queue[0] = (QT)src;
      cur[src >> 5] |= 1u << (src & 31);
    }
    __syncthreads();
    uint32_t qlen = 1;
    uint64_t frontierEdges = a.row[src + 1] - a.row[src];
    uint64_t unvisitedEdges = a.E - frontierEdges;
    uint32_t level = 0;

    while (qlen) {
      const uint32_t L1 = level + 1;
      const bool bottomUp = frontierEdges * 14 > unvisitedEdges;
      if (!bottomUp) {
        for (uint32_t i = grp; i < qlen; i += ngrp) {
          const uint32_t u = queue[i];
          if (u != src && !((tr[u >> 5] >> (u & 31)) & 1u)) {
            continue;
          }
          const uint32_t end = a.row[u + 1];
          for (uint32_t e = a.row[u] + lg; e < end; e += G) {
            const uint32_t v = a.col[e];
            if (dist[v] == kInf32) {
              dist[v] = L1; // every writer stores the same level
              atomicOr(&nxt[v >> 5], 1u << (v & 31));
            }
          }
        }
      } else {
        for (uint32_t v = tid; v < V; v += kBlock) {
          if (dist[v] != kInf32) {
            continue;
          }
          const uint32_t end = a.row[v + 1];
          for (uint32_t e = a.row[v]; e < end; ++e) {
            const uint32_t u = a.col[e];
            const uint32_t ub = 1u << (u & 31);
            if ((cur[u >> 5] & ub) &&
                (u == src || (tr[u >> 5] & ub))) {
              dist[v] = L1;
              atomicOr(&nxt[v >> 5], 1u << (v & 31));
              break;
            }
          }
        }
      }
      __syncthreads();
      uint32_t degsum;
      qlen = compact_frontier<QT>(nxt, cur, nbw, queue, ctl + 1, a.row, &degsum);
      __syncthreads();
      frontierEdges = degsum;
      unvisitedEdges = unvisitedEdges > degsum ? unvisitedEdges - degsum : 0;
      level = L1;
    }

    if constexpr (!GMEM) {
      uint32_t* out = a.dist_out + (size_t)q * a.Vp;
      for (uint32_t v = tid; v < V; v += kBlock) {
        const uint32_t d = dist[v];
        out[v] = d == kInf32 ? kInf32 : d * a.scale;
      }
    } else if (a.scale != 1) {
      for (uint32_t v = tid; v < V; v += kBlock) {
        const uint32_t d = dist[v];
        dist[v] = d == kInf32 ? kInf32 : d * a.scale;
      }
    }
    __syncthreads();
  }
}

// ------------------------------------------- next hops from distance rows
//
// For positive metrics the reference's next-hop union (LinkState.cpp:855-871)
// equals a first-hop test on distance rows:
//   f in NH_s(v)  <=>  f is a distinct neighbour of s, (f transit or v == f)
//                      and w(s,f) + D_f[v] == D_s[v]
// (w(s,f) = cheapest usable s->f link; D_f is f's own SPF, in which f — the
// source — may transit).  When a batch holds the distance rows of every
// neighbour of its sources (all-sources, LFA neighbourhoods) the masks are
// one streaming pass over those rows: coalesced 16-byte loads, no gathers,
// no atomics.  Grid is chunk-major so that blocks sharing an XCD (b, b+8, ...)
// work on neighbouring sources of the same vertex chunk and share the
// neighbours' row chunks in that XCD's L2.

struct NhRowsArgs {
  const uint32_t* nbr_off;
  const uint32_t* nbrs;
  const uint32_t* nbr_w; // cheapest metric to that neighbour
  const uint32_t* trbits;
  const uint32_t* src;
  const int32_t* row_of; // node -> batch row holding its distances
  const uint32_t* dist;  // [nq][Vp]
  const uint64_t* nh_off;
  const uint32_t* nh_w;
  uint64_t* nh_out;
  uint32_t V;
  uint32_t Vp;
  uint32_t nq;
  uint32_t nchunks;
  uint32_t unit;
  // spf_table_nexthops: the source's own row is row_of[src] (else row q),
  // and rows may be unaligned / unpadded (scalar loads within V)
  uint32_t table = 0;
};

// four consecutive row entries from v0 (16-byte load on padded, aligned
// rows; scalar loads within V otherwise)
__device__ __forceinline__ void nh_ld4(
    const NhRowsArgs& a, const uint32_t* rowp, uint32_t v0, uint32_t (&o)[4]) {
  if (!a.table) {
    const uint4 x = *reinterpret_cast<const uint4*>(rowp + v0);
    o[0] = x.x;
    o[1] = x.y;
    o[2] = x.z;
    o[3] = x.w;
    return;
  }
#pragma unroll
  for (uint32_t k = 0; k < 4; ++k) {
    o[k] = v0 + k < a.V ? rowp[v0 + k] : kInf32;
  }
}

constexpr uint32_t kNhThreads = 256;
constexpr uint32_t kNhPerThread = 4;
constexpr uint32_t kNhChunk = kNhThreads * kNhPerThread;

__global__ __launch_bounds__(kNhThreads) void spf_nh_rows_kernel(NhRowsArgs a) {
  const uint32_t chunk = blockIdx.x / a.nq;
  const uint32_t q = blockIdx.x - chunk * a.nq;
  const uint32_t s = a.src[q];
  const uint32_t v0 = chunk * kNhChunk + threadIdx.x * kNhPerThread;
  if (v0 >= a.V) {
    return;
  }
  const uint32_t Wm = a.nh_w[q];
  uint64_t* nhrow = a.nh_out + a.nh_off[q];
  uint32_t dsv[4];
  nh_ld4(a, a.dist + (size_t)(a.table ? (uint32_t)a.row_of[s] : q) * a.Vp, v0, dsv);
  const uint32_t beg = a.nbr_off[s], n = a.nbr_off[s + 1] - beg;
  for (uint32_t w = 0; w < Wm; ++w) {
    uint64_t acc[4] = {0, 0, 0, 0};
    const uint32_t jend = min(n, (w + 1) * 64);
    for (uint32_t j = w * 64; j < jend; ++j) {
      const uint32_t f = a.nbrs[beg + j];
      const uint64_t wf = a.unit ? 1ull : (uint64_t)a.nbr_w[beg + j];
      const bool tf = (a.trbits[f >> 5] >> (f & 31)) & 1u;
      const int32_t r = a.row_of[f];
      uint32_t dfv[4];
      nh_ld4(a, a.dist + (size_t)r * a.Vp, v0, dfv);
      const uint64_t bit = 1ull << (j & 63);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const uint32_t v = v0 + k;
        if (dsv[k] != kInf32 && dfv[k] != kInf32 && wf + dfv[k] == (uint64_t)dsv[k] &&
            (tf || v == f)) {
          acc[k] |= bit;
        }
      }
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if (v0 + k < a.V) {
        nhrow[(size_t)(v0 + k) * Wm + w] = acc[k];
      }
    }
  }
}

// ------------------------------------- multi-source bit-parallel BFS (MS-BFS)
//
// Uniform metric, many sources: one workgroup advances the BFS of a whole
// batch of B = bits(MT) sources at once.  The frontier is one B-bit mask per
// node in LDS (bit s = "node is on source s's frontier"); each thread owns
// K nodes and keeps their visited masks in registers.  One level is a single
// pull pass over the CSR:
//     new(v) = OR_{u in N(v)} F(u)  &  ~visited(v)
// so every CSR row is read once per level for B sources (the per-source BFS
// reads it once per source).  Transit: a node's frontier bits are published
// only if it may be transited, except at level 0 where each source's own bit
// is always published (LinkState.cpp:829-836 exempts the source).
// The frontier is double-buffered in LDS (read cur, write nxt, one barrier
// per level), so only the visited masks live in registers.  Distances go out
// as 32-bit rows plus an 8-bit level row that the next-hop pass streams
// instead of the 32-bit distances.

#ifndef OPENR_MS_UNROLL8
#define OPENR_MS_UNROLL8 1
#endif
constexpr uint32_t kMsThreads = 1024;
constexpr uint32_t kMsShallowLevel = 127;
constexpr uint32_t kMsMaxK = 20; // nodes per thread -> V <= 20480 (32-bit batches above 10,240 nodes: the
                                 // double buffer is 2 * V * 4 B <= 160 KB of LDS)

struct MsBfsArgs {
  const uint32_t* row;
  const uint32_t* col;
  // sliced-ELL copy of the CSR (one slice = the 64 nodes of one wave's
  // k-th node slot): edge j of lane L of slice c is word j % 4 of uint4
  // sell4[(sell_off[c] + j / 4) * 64 + L]; short rows are padded with the
  // node itself, whose frontier bits are a subset of its visited bits and so
  // drop out of `acc & ~vis`.  nullptr: the plain CSR loop.
  const uint4* sell4;
  const uint32_t* sell_off; // [slices + 1] in 64-uint4 groups
  const uint32_t* trbits;
  const uint32_t* src;
  uint32_t* dist_out; // [nq][Vp]
  uint8_t* lvl_out;   // [nq][Vp8]
  // [0] |= 1 when a level >= 255 occurred (32-bit rows: the byte passes
  // step aside), |= 2 when a level >= kMsShallowLevel did (the v2 pass's
  // one-add byte compare needs every level below it)
  uint32_t* flags;
  // the other launch's flag word, zeroed by block 0 (flags alternate between
  // two words per launch, so no per-run memset: stream order guarantees the
  // last readers of this word, the previous run's next-hop pass, are done)
  uint32_t* flags_clear = nullptr;
  uint32_t V;
  uint32_t Vp;
  uint32_t Vp8;
  uint32_t nq;
  uint32_t scale;
  uint32_t wrec; // 1: wave-cooperative row stores (ms_record_wave)
  // zero-metric plan: (tail, head) pairs of the metric-0 half-edges this
  // pass closes over at every level (ms_zero_close); nz = 0 elsewhere
  const uint32_t* zlist;
  uint32_t nz;
  // 1: distances below level 255 are left to the next-hop pass, which
  // writes them from the level rows as coalesced 16-byte stores
  // (OPENR_MS_LVL_ONLY); levels >= 255 and unreached pairs still go here
  uint32_t lvl_only;
  // per-query ignore lists (KSP2 second passes): ign_mask[b * E + e] = the
  // batch-b queries whose list holds link(e) (bit q - B b), ign_flag[b * nfw
  // + v / 32] bit v: a half-edge of node v's row is ignored by one of them.
  // Flagged nodes pull over the plain CSR with the masks applied, the others
  // over the sliced copy as before; nullptr = no ignore lists
  const uint64_t* ign_mask = nullptr;
  const uint32_t* ign_flag = nullptr;
  uint32_t E = 0;
  uint32_t nfw = 0;
  // measurement only (OPENR_MS_NOREC=1): the BFS without its row stores
  uint32_t norec = 0;
  // per batch: one node that stays non-transit in this batch (kInf32 none;
  // nullptr: no such node) -- the what-if first-hop rows, BFS levels from a
  // source's neighbours through every node but that source
  const uint32_t* blocked = nullptr;
};

// Masks and flags of spf_msbfs_kernel's ignore mode: one block per query,
// both halves of every ignored link (a half-edge h sits in the row of its
// tail, which is where the pull reads it)
__global__ __launch_bounds__(256) void spf_ms_ign_kernel(
    const uint32_t* ign_off, const uint32_t* ign, const uint32_t* link_half,
    const uint32_t* col, const uint32_t* rev, uint32_t L, uint32_t B, uint32_t E,
    uint32_t nfw, uint64_t* mask, uint32_t* flag) {
  const uint32_t q = blockIdx.x, b = q / B, j = q - b * B;
  const uint32_t lo = ign_off[q], hi = ign_off[q + 1];
  for (uint32_t i = lo + threadIdx.x; i < hi; i += blockDim.x) {
    const uint32_t l = ign[i];
    if (l >= L) {
      continue;
    }
    for (uint32_t side = 0; side < 2; ++side) {
      const uint32_t h = link_half[2 * (size_t)l + side];
      if (h == kInf32) {
        continue;
      }
      const uint32_t t = col[rev[h]];
      atomicOr(reinterpret_cast<unsigned long long*>(mask + (size_t)b * E + h), 1ull << j);
      atomicOr(flag + (size_t)b * nfw + (t >> 5), 1u << (t & 31));
    }
  }
}

// Write each (source, node) distance the moment its bit appears (one store
// per bit).  These stores overlap the latency-bound row scans of the later
// levels; writing the rows source-by-source at the end instead (fully
// coalesced, from a per-level history) measured slower on the fabric because
// the write burst then serialises behind the last level.
template <typename MT>
__device__ __forceinline__ void ms_record(
    const MsBfsArgs& a, uint32_t q0, uint32_t v, MT bits, uint32_t level) {
  if (a.norec) {
    return;
  }
  const uint32_t d = level * a.scale;
  const uint8_t l8 = level < 255 ? (uint8_t)level : (uint8_t)255;
  if (level >= kMsShallowLevel && bits) {
    atomicOr(a.flags, level >= 255 ? 3u : 2u);
  }
  const bool wd = !a.lvl_only || level >= 255;
  while (bits) {
    const uint32_t s = (uint32_t)__builtin_ctzll((unsigned long long)bits);
    bits &= bits - 1;
    if (wd) {
      a.dist_out[(size_t)(q0 + s) * a.Vp + v] = d;
    }
    a.lvl_out[(size_t)(q0 + s) * a.Vp8 + v] = l8;
  }
}

// Wave-cooperative form (OPENR_MS_WREC, default): the lanes' bit sets are
// OR-reduced over the wave and the wave walks the union bit by bit, so every
// store instruction writes source s's row at the wave's 64 consecutive nodes
// (256 contiguous bytes of distances, 64 of levels) instead of 64 lanes
// scattering into 64 different rows.  Every lane of the wave must call it.
template <typename MT>
__device__ __forceinline__ void ms_record_wave(
    const MsBfsArgs& a, uint32_t q0, uint32_t v, MT bits, uint32_t level) {
  uint64_t w = (uint64_t)bits;
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    w |= (uint64_t)__shfl_xor((unsigned long long)w, off, 64);
  }
  if (!w) {
    return;
  }
  const uint32_t d = level * a.scale;
  const uint8_t l8 = level < 255 ? (uint8_t)level : (uint8_t)255;
  if (level >= kMsShallowLevel && bits) {
    atomicOr(a.flags, level >= 255 ? 3u : 2u);
  }
  while (w) {
    const uint32_t s = (uint32_t)__builtin_ctzll((unsigned long long)w);
    w &= w - 1;
    if (((uint64_t)bits >> s) & 1u) {
      if (!a.lvl_only || level >= 255) {
        a.dist_out[(size_t)(q0 + s) * a.Vp + v] = d;
      }
      a.lvl_out[(size_t)(q0 + s) * a.Vp8 + v] = l8;
    }
  }
}

// Metric-0 closure of one level (zero-metric plan): the head y
// of a metric-0 half-edge x -> y reaches, at the SAME level, every source
// whose bit x publishes at this level (fr = the level's published frontier:
// transit nodes' new bits, or the sources' own bits at level 0).  The zero
// links are node-disjoint, so one pass closes the level: y's gained bits
// could only flow back to x, which already holds them.  Run by y's owner
// lane (its visited mask lives in that lane's registers).
template <typename MT, uint32_t KMAX>
__device__ __forceinline__ void ms_zero_close(
    const MsBfsArgs& a, uint32_t q0, MT* fr, MT (&vis)[KMAX], uint32_t trm, uint32_t level) {
  for (uint32_t i = 0; i < a.nz; ++i) {
    const uint32_t x = a.zlist[2 * i], y = a.zlist[2 * i + 1];
    if ((y & (kMsThreads - 1)) != threadIdx.x) {
      continue;
    }
    const uint32_t ky = y / kMsThreads;
    const MT fx = fr[x];
#pragma unroll
    for (uint32_t k = 0; k < KMAX; ++k) {
      if (k == ky) { // static register index
        const MT gain = fx & ~vis[k];
        if (gain) {
          vis[k] |= gain;
          if ((trm >> k) & 1u) {
            fr[y] |= gain;
          }
          ms_record<MT>(a, q0, y, gain, level);
        }
      }
    }
  }
}

// GEN = false: the plain batch (no ignore masks, no wave-recorded levels, no
// zero-metric closure) with those paths compiled out of the KMAX unrolled
// node copies.  The general form spilled 79 VGPRs and 164 SGPRs per thread
// (320 B of scratch, ~60 reloads per BFS level on the fabric's KMAX = 12);
// the plain one 24 / 47 (100 B).
template <typename MT, uint32_t KMAX, bool SELL, bool GEN>
__global__ __launch_bounds__(kMsThreads) void spf_msbfs_kernel(MsBfsArgs a) {
  extern __shared__ __align__(16) unsigned char ms_smem[];
  constexpr uint32_t B = sizeof(MT) * 8;
  const uint32_t V = a.V, tid = threadIdx.x;
  const uint32_t K = (V + kMsThreads - 1) / kMsThreads; // <= KMAX
  const uint32_t nbatch = (a.nq + B - 1) / B;
  if (a.flags_clear && blockIdx.x == 0 && tid == 0) {
    *a.flags_clear = 0;
  }

  for (uint32_t b = blockIdx.x; b < nbatch; b += gridDim.x) {
    // frontier double buffer: cur is read during a level, nxt written
    MT* cur = reinterpret_cast<MT*>(ms_smem);
    MT* nxt = cur + V;
    const uint32_t q0 = b * B;
    const uint32_t nb = min(B, a.nq - q0);
    const MT full = nb == B ? ~(MT)0 : (((MT)1 << nb) - 1);
    for (uint32_t v = tid; v < V; v += kMsThreads) {
      cur[v] = 0;
    }
    __syncthreads();
    if (tid < nb) {
      const uint32_t s = a.src[q0 + tid];
      if constexpr (sizeof(MT) == 8) {
        atomicOr(reinterpret_cast<unsigned long long*>(&cur[s]), 1ull << tid);
      } else {
        atomicOr(reinterpret_cast<unsigned int*>(&cur[s]), 1u << tid);
      }
    }
    __syncthreads();
    MT vis[KMAX];
    uint32_t trm = 0; // bit k: this thread's k-th node may be transited
    const uint32_t blk = a.blocked ? a.blocked[b] : kInf32;
#pragma unroll
    for (uint32_t k = 0; k < KMAX; ++k) {
      const uint32_t v = tid + k * kMsThreads;
      if (k < K && v < V && v != blk) {
        trm |= ((a.trbits[v >> 5] >> (v & 31)) & 1u) << k;
      }
      vis[k] = (k < K && v < V) ? cur[v] : (MT)0;
      if (GEN && a.wrec) {
        if (k < K) {
          ms_record_wave<MT>(a, q0, v, vis[k], 0); // level 0 = the sources
        }
      } else if (k < K && v < V && vis[k]) {
        ms_record<MT>(a, q0, v, vis[k], 0);
      }
    }
    if (GEN && a.nz) {
      ms_zero_close<MT, KMAX>(a, q0, cur, vis, trm, 0);
      __syncthreads();
    }
    uint32_t level = 0;
    for (;;) {
      const uint32_t L = level + 1;
      bool any = false;
#pragma unroll
      for (uint32_t k = 0; k < KMAX; ++k) {
        uint32_t v = tid + k * kMsThreads;
        // opaque to the optimizer: keeps per-node addressing from being
        // hoisted out of the level loop (KMAX copies of it spill VGPRs)
        asm volatile("" : "+v"(v));
        if (k >= K) {
          continue; // uniform
        }
        const bool valid = v < V;
        MT nw = 0;
        const bool ignv = GEN && a.ign_flag && valid && vis[k] != full &&
                          ((a.ign_flag[(size_t)b * a.nfw + (v >> 5)] >> (v & 31)) & 1u);
        if (ignv) {
          // a row with ignored half-edges: the plain CSR, each edge's bits
          // masked by the queries that ignore its link
          const uint64_t* m = a.ign_mask + (size_t)b * a.E;
          MT acc = 0;
          for (uint32_t e = a.row[v]; e < a.row[v + 1]; ++e) {
            acc |= cur[a.col[e]] & ~(MT)m[e];
          }
          nw = acc & ~vis[k];
          vis[k] |= nw;
        } else if (SELL && valid && vis[k] != full) {
          // a wave reads 1 KB of its slice per load instead of one line per lane
          const uint32_t c = __builtin_amdgcn_readfirstlane(v >> 6);
          const uint32_t g0 = __builtin_amdgcn_readfirstlane(a.sell_off[c]);
          const uint32_t g1 = __builtin_amdgcn_readfirstlane(a.sell_off[c + 1]);
          const uint4* p = a.sell4 + (size_t)g0 * 64 + (tid & 63u);
          MT acc = 0;
          uint32_t g = g0;
          for (; g + 2 <= g1; g += 2, p += 128) {
            const uint4 c0 = p[0], c1 = p[64];
            acc |= cur[c0.x] | cur[c0.y] | cur[c0.z] | cur[c0.w] | cur[c1.x] | cur[c1.y] |
                   cur[c1.z] | cur[c1.w];
          }
          if (g < g1) {
            const uint4 c0 = p[0];
            acc |= cur[c0.x] | cur[c0.y] | cur[c0.z] | cur[c0.w];
          }
          nw = acc & ~vis[k];
          vis[k] |= nw;
        } else if (!SELL && valid && vis[k] != full) {
          const uint32_t beg = a.row[v], end = a.row[v + 1];
          MT acc = 0;
          uint32_t e = beg;
#if OPENR_MS_UNROLL8
          for (; e + 8 <= end; e += 8) {
            const uint4 c0 = {a.col[e], a.col[e + 1], a.col[e + 2], a.col[e + 3]};
            const uint4 c1 = {a.col[e + 4], a.col[e + 5], a.col[e + 6], a.col[e + 7]};
            acc |= cur[c0.x] | cur[c0.y] | cur[c0.z] | cur[c0.w] | cur[c1.x] | cur[c1.y] |
                   cur[c1.z] | cur[c1.w];
          }
#endif
          for (; e + 4 <= end; e += 4) {
            const uint32_t u0 = a.col[e], u1 = a.col[e + 1], u2 = a.col[e + 2],
                           u3 = a.col[e + 3];
            acc |= cur[u0] | cur[u1] | cur[u2] | cur[u3];
          }
          for (; e < end; ++e) {
            acc |= cur[a.col[e]];
          }
          nw = acc & ~vis[k];
          vis[k] |= nw;
        }
        any |= nw != 0;
        const bool transit = (trm >> k) & 1u;
        if (valid) {
          nxt[v] = transit ? nw : (MT)0;
        }
        if (GEN && a.wrec) {
          ms_record_wave<MT>(a, q0, v, nw, L);
        } else if (nw) {
          ms_record<MT>(a, q0, v, nw, L);
        }
      }
      const bool more = __syncthreads_or(any);
      if (!more) {
        break;
      }
      if (GEN && a.nz) {
        ms_zero_close<MT, KMAX>(a, q0, nxt, vis, trm, L);
        __syncthreads();
      }
      MT* t = cur;
      cur = nxt;
      nxt = t;
      level = L;
    }
    // unreached (source, node) pairs
#pragma unroll
    for (uint32_t k = 0; k < KMAX; ++k) {
      const uint32_t v = tid + k * kMsThreads;
      if (GEN && a.wrec) {
        if (k < K) {
          // unreached pairs as one more "level" whose value is the sentinel
          const MT miss = v < V ? (full & ~vis[k]) : (MT)0;
          uint64_t w = (uint64_t)miss;
#pragma unroll
          for (int off = 32; off >= 1; off >>= 1) {
            w |= (uint64_t)__shfl_xor((unsigned long long)w, off, 64);
          }
          while (w) {
            const uint32_t s = (uint32_t)__builtin_ctzll((unsigned long long)w);
            w &= w - 1;
            if (((uint64_t)miss >> s) & 1u) {
              a.dist_out[(size_t)(q0 + s) * a.Vp + v] = kInf32;
              a.lvl_out[(size_t)(q0 + s) * a.Vp8 + v] = 255;
            }
          }
        }
      } else if (k < K && v < V) {
        MT miss = full & ~vis[k];
        while (miss) {
          const uint32_t s = (uint32_t)__builtin_ctzll((unsigned long long)miss);
          miss &= miss - 1;
          a.dist_out[(size_t)(q0 + s) * a.Vp + v] = kInf32;
          a.lvl_out[(size_t)(q0 + s) * a.Vp8 + v] = 255;
        }
      }
    }
    __syncthreads();
  }
}

// ---- cooperative MS-BFS (a 64-source batch split over P workgroups) ----
//
// spf_msbfs_kernel runs a batch on ONE CU, and a level's pull over all V
// nodes (~14 us on the fabric) is that CU's work: a rank's block of a sharded
// table (20 batches at N = 8) leaves most of the chip idle and its MS-BFS stays
// at the one-batch latency floor.  Here P workgroups share a batch:
// part p owns nodes v = (k P + p) 1024 + tid, keeps its own LDS copy of the
// whole frontier (V words, single-buffered), pulls only its nodes, and
// publishes their next-frontier bits to a global exchange buffer (double-
// buffered by level parity); the P parts meet at a counter barrier per level
// (agent-scope release / acquire, MI355X cross-XCD hand-off recipe) and reload
// the full frontier.  Launched cooperatively (every workgroup co-resident), P
// sized from the occupancy query: the round-4 probe deadlocked because a grid
// of two 1,024-thread workgroups per CU cannot be resident at 128 VGPRs.
// Same rows as spf_msbfs_kernel (the plain instance: no ignore masks,
// wave-recorded levels or zero-metric closure).
struct MsCoopArgs {
  MsBfsArgs a;
  uint64_t* xbuf;  // [nbatch][2][V] published next-frontier bits
  uint32_t* cnt;   // [nbatch] barrier arrivals (zeroed before the launch)
  uint32_t* anyv;  // [nbatch][2][P] "some bit was new" per part and level parity
  uint32_t* err;   // set when a barrier wait gave up (spf_query_sync reports it)
  uint32_t P;
};
constexpr uint32_t kMsCoopSpin = 1u << 26; // polls before a barrier wait gives up

template <uint32_t KMAX>
__global__ __launch_bounds__(kMsThreads) void spf_msbfs_coop_kernel(MsCoopArgs c) {
  extern __shared__ __align__(16) unsigned char ms_smem[];
  const MsBfsArgs& a = c.a;
  uint64_t* cur = reinterpret_cast<uint64_t*>(ms_smem); // this part's frontier copy
  const uint32_t V = a.V, tid = threadIdx.x, P = c.P;
  const uint32_t b = blockIdx.x / P, p = blockIdx.x - b * P;
  const uint32_t nbatch = (a.nq + 63) / 64;
  if (b >= nbatch) {
    return; // whole workgroup (never: the grid is nbatch * P)
  }
  if (a.flags_clear && blockIdx.x == 0 && tid == 0) {
    *a.flags_clear = 0;
  }
  const uint32_t q0 = b * 64, nb = min(64u, a.nq - q0);
  const uint64_t full = nb == 64 ? ~0ull : ((1ull << nb) - 1);
  const uint32_t span = P * kMsThreads;
  const uint32_t Kp = (V + span - 1) / span; // <= KMAX
  for (uint32_t v = tid; v < V; v += kMsThreads) {
    cur[v] = 0;
  }
  __syncthreads();
  if (tid < nb) {
    atomicOr(reinterpret_cast<unsigned long long*>(&cur[a.src[q0 + tid]]), 1ull << tid);
  }
  __syncthreads();
  uint64_t vis[KMAX];
  uint32_t trm = 0;
#pragma unroll
  for (uint32_t k = 0; k < KMAX; ++k) {
    const uint32_t v = (k * P + p) * kMsThreads + tid;
    vis[k] = 0;
    if (k < Kp && v < V) {
      trm |= ((a.trbits[v >> 5] >> (v & 31)) & 1u) << k;
      vis[k] = cur[v];
      if (vis[k]) {
        ms_record<uint64_t>(a, q0, v, vis[k], 0);
      }
    }
  }
  uint64_t* xb = c.xbuf + (size_t)b * 2 * V;
  uint32_t* anyb = c.anyv + (size_t)b * 2 * P;
  bool aborted = false;
  for (uint32_t L = 1;; ++L) {
    uint64_t* xn = xb + (size_t)(L & 1u) * V;
    bool any = false;
#pragma unroll
    for (uint32_t k = 0; k < KMAX; ++k) {
      uint32_t v = (k * P + p) * kMsThreads + tid;
      asm volatile("" : "+v"(v));
      if (k >= Kp) {
        continue; // uniform
      }
      uint64_t nw = 0;
      if (v < V && vis[k] != full) {
        const uint32_t cs = __builtin_amdgcn_readfirstlane(v >> 6);
        const uint32_t g0 = __builtin_amdgcn_readfirstlane(a.sell_off[cs]);
        const uint32_t g1 = __builtin_amdgcn_readfirstlane(a.sell_off[cs + 1]);
        const uint4* pp = a.sell4 + (size_t)g0 * 64 + (tid & 63u);
        uint64_t acc = 0;
        uint32_t g = g0;
        for (; g + 2 <= g1; g += 2, pp += 128) {
          const uint4 c0 = pp[0], c1 = pp[64];
          acc |= cur[c0.x] | cur[c0.y] | cur[c0.z] | cur[c0.w] | cur[c1.x] | cur[c1.y] |
                 cur[c1.z] | cur[c1.w];
        }
        if (g < g1) {
          const uint4 c0 = pp[0];
          acc |= cur[c0.x] | cur[c0.y] | cur[c0.z] | cur[c0.w];
        }
        nw = acc & ~vis[k];
        vis[k] |= nw;
      }
      any |= nw != 0;
      if (v < V) {
        // write-through (sc1) store: visible to the other parts' XCDs with
        // no release fence (an agent-scope release writes back the L2, full
        // of this launch's level rows)
        __hip_atomic_store((__attribute__((address_space(1))) uint64_t*)(xn + v),
                           ((trm >> k) & 1u) ? nw : 0ull, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
      }
      if (nw) {
        ms_record<uint64_t>(a, q0, v, nw, L);
      }
    }
    // publish: this part's bits and its "any" flag, then the barrier
    const bool mine = __syncthreads_or(any);
    if (tid == 0) {
      __hip_atomic_store(anyb + (L & 1u) * P + p, mine ? 1u : 0u, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); // every storing wave drains
    __syncthreads();
    if (tid == 0) {
      __hip_atomic_fetch_add(c.cnt + b, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const uint32_t target = L * P;
      uint32_t spins = 0;
      while (__hip_atomic_load(c.cnt + b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
        __builtin_amdgcn_s_sleep(1);
        if (++spins > kMsCoopSpin) {
          atomicOr(c.err, 1u);
          aborted = true;
          break;
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads(); // every wave reads the other parts' words after the acquire
    uint32_t flag = 0;
    if (tid < P) {
      flag = __hip_atomic_load(anyb + (L & 1u) * P + tid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    const bool more = __syncthreads_or(flag != 0);
    if (__syncthreads_or(aborted) || !more) {
      break;
    }
    for (uint32_t v = tid; v < V; v += kMsThreads) {
      cur[v] = xn[v];
    }
    __syncthreads();
  }
  // unreached (source, node) pairs of this part's nodes
#pragma unroll
  for (uint32_t k = 0; k < KMAX; ++k) {
    const uint32_t v = (k * P + p) * kMsThreads + tid;
    if (k < Kp && v < V) {
      uint64_t miss = full & ~vis[k];
      while (miss) {
        const uint32_t s = (uint32_t)__builtin_ctzll(miss);
        miss &= miss - 1;
        a.dist_out[(size_t)(q0 + s) * a.Vp + v] = kInf32;
        a.lvl_out[(size_t)(q0 + s) * a.Vp8 + v] = 255;
      }
    }
  }
}

// Next hops from 8-bit level rows (uniform metric c: w + D_f == D_s is
// lf + 1 == ls).  16 nodes per thread per 16-byte load.  Falls back to the
// 32-bit rows when the BFS saw a level >= 255 (flags[0]).
struct NhLevelsArgs {
  const uint32_t* nbr_off;
  const uint32_t* nbrs;
  const uint32_t* trbits;
  const uint32_t* src;
  const int32_t* row_of;
  const uint8_t* lvl; // [nq][Vp8]
  const uint32_t* dist; // [nq][Vp]
  const uint32_t* flags;
  const uint64_t* nh_off;
  const uint32_t* nh_w;
  uint64_t* nh_out;
  // the byte-strided output rows (nh_bytes_for) the SWAR kernels write
  // directly; the word-layout kernels above write nh_out (a working buffer
  // narrowed afterwards when the layouts differ)
  uint8_t* nhb;
  const uint64_t* nhb_off;
  const uint32_t* nh_b;
  uint32_t V;
  uint32_t Vp;
  uint32_t Vp8;
  uint32_t nq;
  uint32_t scale;
  uint32_t xcd_swizzle; // 1: XCD-aware block order (OPENR_NL_XCD; default off: 0.69 -> 0.92 ms on the fabric, profiles/r03b)
  uint32_t held_words;  // 1: 2/3-word masks stored node-major from registers (OPENR_NL_HELD)
  // zero-metric plan: source q reads its own and its neighbours' rows from
  // variant table zvar[q] (lvl + zvar[q] * lvl_vstride, dist + zvar[q] *
  // dist_vstride); nullptr: one table
  const uint8_t* zvar;
  uint64_t lvl_vstride;
  uint64_t dist_vstride;
  // MsBfsArgs::lvl_only: the pass writes each source's distances below
  // level 255 (lvl * scale) into dist_w and reads neighbour distances from
  // the level byte when it is below 255
  uint32_t* dist_w;
  // held kernel work order (OPENR_NL_ORDER=1): hardware block b runs item
  // held_order[b] = q * held_nch + chunk (kInf32: none); nullptr = the
  // chunk-major default
  const uint32_t* held_order = nullptr;
  uint32_t held_nch = 0;
  // OPENR_NL_NT=1: the byte-SIMD pass's mask and distance rows as
  // non-temporal stores
  uint32_t nt_store = 0;
};

constexpr uint32_t kNlThreads = 256;
constexpr uint32_t kNlPer = 4;
constexpr uint32_t kNlChunk = kNlThreads * kNlPer;

// 4 nodes per thread: one 4-byte load of a level row (or one 16-byte load of
// a 32-bit row), four compares, and the four next-hop words leave as two
// 16-byte stores, so a wave writes 2 KB of contiguous mask row.  The
// source's neighbour list (row index + transit bit) is staged in LDS first
// and the neighbour rows are loaded kNlUnroll at a time, so a block keeps
// several independent row loads in flight instead of one dependent chain
// (nbrs -> row_of -> trbits -> row) per neighbour.
#ifndef OPENR_NL_UNROLL
#define OPENR_NL_UNROLL 8
#endif
constexpr uint32_t kNlUnroll = OPENR_NL_UNROLL;
constexpr uint32_t kNlStage = 1024; // neighbours staged per pass

template <bool WIDE>
__device__ __forceinline__ void nl_load(
    const NhLevelsArgs& a, uint32_t r, uint32_t v0, uint32_t (&o)[4]) {
  if constexpr (!WIDE) {
    const uint32_t x = *reinterpret_cast<const uint32_t*>(a.lvl + (size_t)r * a.Vp8 + v0);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      o[i] = (x >> (8 * i)) & 0xFFu;
    }
  } else {
    const uint4 x = *reinterpret_cast<const uint4*>(a.dist + (size_t)r * a.Vp + v0);
    o[0] = x.x;
    o[1] = x.y;
    o[2] = x.z;
    o[3] = x.w;
  }
}

template <bool WIDE>
__device__ __forceinline__ void nl_body(
    const NhLevelsArgs& a, uint32_t q, uint32_t s, uint32_t v0, uint32_t* st_row,
    uint32_t* st_node) {
  const uint32_t Wm = a.nh_w[q];
  uint64_t* nhrow = a.nh_out + a.nh_off[q];
  const bool active = v0 < a.V;
  uint32_t ls[4] = {0, 0, 0, 0};
  if (active) {
    nl_load<WIDE>(a, q, v0, ls);
  }
  const uint32_t none = WIDE ? kInf32 : 255u;
  const uint64_t step = WIDE ? (uint64_t)a.scale : 1ull;
  bool live[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    live[i] = active && ls[i] != none && ls[i] != 0;
  }
  const uint32_t beg = a.nbr_off[s], n = a.nbr_off[s + 1] - beg;
  for (uint32_t w = 0; w < Wm; ++w) {
    uint64_t acc[4] = {0, 0, 0, 0};
    const uint32_t jlo = w * 64, jhi = min(n, jlo + 64);
    for (uint32_t base = jlo; base < jhi; base += kNlStage) {
      const uint32_t cnt = min(kNlStage, jhi - base);
      __syncthreads();
      for (uint32_t t = threadIdx.x; t < cnt; t += kNlThreads) {
        const uint32_t f = a.nbrs[beg + base + t];
        const uint32_t tf = (a.trbits[f >> 5] >> (f & 31)) & 1u;
        st_row[t] = (uint32_t)a.row_of[f];
        st_node[t] = f | (tf << 31);
      }
      __syncthreads();
      if (!active) {
        continue;
      }
      uint32_t t = 0;
      for (; t + kNlUnroll <= cnt; t += kNlUnroll) {
        uint32_t lf[kNlUnroll][4];
#pragma unroll
        for (uint32_t u = 0; u < kNlUnroll; ++u) {
          nl_load<WIDE>(a, st_row[t + u], v0, lf[u]);
        }
#pragma unroll
        for (uint32_t u = 0; u < kNlUnroll; ++u) {
          const uint32_t nd = st_node[t + u];
          const uint32_t f = nd & 0x7FFFFFFFu;
          const bool tf = nd >> 31;
          const uint64_t bit = 1ull << ((base + t + u) & 63);
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            if (live[i] && lf[u][i] != none && (uint64_t)lf[u][i] + step == (uint64_t)ls[i] &&
                (tf || v0 + i == f)) {
              acc[i] |= bit;
            }
          }
        }
      }
      for (; t < cnt; ++t) {
        uint32_t lf[4];
        nl_load<WIDE>(a, st_row[t], v0, lf);
        const uint32_t nd = st_node[t];
        const uint32_t f = nd & 0x7FFFFFFFu;
        const bool tf = nd >> 31;
        const uint64_t bit = 1ull << ((base + t) & 63);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          if (live[i] && lf[i] != none && (uint64_t)lf[i] + step == (uint64_t)ls[i] &&
              (tf || v0 + i == f)) {
            acc[i] |= bit;
          }
        }
      }
    }
    if (!active) {
      continue;
    }
    if (Wm == 1 && v0 + 4 <= a.V) {
      ulonglong2* o = reinterpret_cast<ulonglong2*>(nhrow + v0);
      o[0] = make_ulonglong2(acc[0], acc[1]);
      o[1] = make_ulonglong2(acc[2], acc[3]);
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if (v0 + i < a.V) {
          nhrow[(size_t)(v0 + i) * Wm + w] = acc[i];
        }
      }
    }
  }
}

// One block sweeps chunks [c0, c1) of one source: the source's neighbour
// list is staged once per mask word and reused by every chunk, so the
// dependent staging loads (nbrs -> row_of / transit) are paid once per
// block instead of once per 1024-node chunk, and a block keeps up to
// kNlUnroll independent row loads in flight per thread per chunk.
// Sources with more than kNlStage distinct neighbours: the word-outer
// order, staging 64 neighbours per word.
template <bool WIDE>
__device__ __forceinline__ void nl_body_multi_staged(
    const NhLevelsArgs& a, uint32_t q, uint32_t s, uint32_t c0, uint32_t c1,
    uint32_t* st_row, uint32_t* st_node) {
  const uint32_t Wm = a.nh_w[q];
  uint64_t* nhrow = a.nh_out + a.nh_off[q];
  const uint32_t none = WIDE ? kInf32 : 255u;
  const uint64_t step = WIDE ? (uint64_t)a.scale : 1ull;
  const uint32_t beg = a.nbr_off[s], n = a.nbr_off[s + 1] - beg;
  for (uint32_t w = 0; w < Wm; ++w) {
    const uint32_t jlo = w * 64, cnt = min(64u, n - min(n, jlo)); // <= kNlStage
    __syncthreads();
    for (uint32_t t = threadIdx.x; t < cnt; t += kNlThreads) {
      const uint32_t f = a.nbrs[beg + jlo + t];
      const uint32_t tf = (a.trbits[f >> 5] >> (f & 31)) & 1u;
      st_row[t] = (uint32_t)a.row_of[f];
      st_node[t] = f | (tf << 31);
    }
    __syncthreads();
    for (uint32_t c = c0; c < c1; ++c) {
      const uint32_t v0 = c * kNlChunk + threadIdx.x * kNlPer;
      if (v0 >= a.V) {
        break;
      }
      uint32_t ls[4];
      nl_load<WIDE>(a, q, v0, ls);
      bool live[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        live[i] = ls[i] != none && ls[i] != 0;
      }
      uint64_t acc[4] = {0, 0, 0, 0};
      uint32_t t = 0;
      for (; t + kNlUnroll <= cnt; t += kNlUnroll) {
        uint32_t lf[kNlUnroll][4];
#pragma unroll
        for (uint32_t u = 0; u < kNlUnroll; ++u) {
          nl_load<WIDE>(a, st_row[t + u], v0, lf[u]);
        }
#pragma unroll
        for (uint32_t u = 0; u < kNlUnroll; ++u) {
          const uint32_t nd = st_node[t + u];
          const uint32_t f = nd & 0x7FFFFFFFu;
          const bool tf = nd >> 31;
          const uint64_t bit = 1ull << (t + u);
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            if (live[i] && lf[u][i] != none && (uint64_t)lf[u][i] + step == (uint64_t)ls[i] &&
                (tf || v0 + i == f)) {
              acc[i] |= bit;
            }
          }
        }
      }
      for (; t < cnt; ++t) {
        uint32_t lf[4];
        nl_load<WIDE>(a, st_row[t], v0, lf);
        const uint32_t nd = st_node[t];
        const uint32_t f = nd & 0x7FFFFFFFu;
        const bool tf = nd >> 31;
        const uint64_t bit = 1ull << t;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          if (live[i] && lf[i] != none && (uint64_t)lf[i] + step == (uint64_t)ls[i] &&
              (tf || v0 + i == f)) {
            acc[i] |= bit;
          }
        }
      }
      if (Wm == 1 && v0 + 4 <= a.V) {
        ulonglong2* o = reinterpret_cast<ulonglong2*>(nhrow + v0);
        o[0] = make_ulonglong2(acc[0], acc[1]);
        o[1] = make_ulonglong2(acc[2], acc[3]);
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          if (v0 + i < a.V) {
            nhrow[(size_t)(v0 + i) * Wm + w] = acc[i];
          }
        }
      }
    }
  }
}

// WM = the source's mask words when it is 2 or 3 (finished words are held in
// registers and a lane's four nodes x WM words leave as one contiguous
// 32*WM-byte run, so every line of the row is written whole by one wave);
// WM = 1 the single-word path (wave-contiguous 1 KB stores); WM = 0 any width
// (word-strided 8-byte stores).
template <bool WIDE, uint32_t WM>
__device__ __forceinline__ void nl_body_multi(
    const NhLevelsArgs& a, uint32_t q, uint32_t s, uint32_t c0, uint32_t c1,
    uint32_t* st_row, uint32_t* st_node) {
  const uint32_t Wm = WM ? WM : a.nh_w[q];
  uint64_t* nhrow = a.nh_out + a.nh_off[q];
  const uint32_t none = WIDE ? kInf32 : 255u;
  const uint64_t step = WIDE ? (uint64_t)a.scale : 1ull;
  const uint32_t beg = a.nbr_off[s], n = a.nbr_off[s + 1] - beg;
  // every neighbour staged once (n <= kNlStage; bigger sources take
  // nl_body_multi_staged); the words of a chunk are then computed back to back
  // and the source's own level row is loaded once per chunk, not once per word
  __syncthreads();
  for (uint32_t t = threadIdx.x; t < n; t += kNlThreads) {
    const uint32_t f = a.nbrs[beg + t];
    const uint32_t tf = (a.trbits[f >> 5] >> (f & 31)) & 1u;
    st_row[t] = (uint32_t)a.row_of[f];
    st_node[t] = f | (tf << 31);
  }
  __syncthreads();
  for (uint32_t c = c0; c < c1; ++c) {
    const uint32_t v0 = c * kNlChunk + threadIdx.x * kNlPer;
    if (v0 >= a.V) {
      break;
    }
    uint32_t ls[4];
    nl_load<WIDE>(a, q, v0, ls);
    bool live[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      live[i] = ls[i] != none && ls[i] != 0;
    }
    uint64_t held[WM > 1 ? WM : 1][4];
    for (uint32_t w = 0; w < Wm; ++w) {
      const uint32_t jlo = w * 64, jhi = min(n, jlo + 64);
      uint64_t acc[4] = {0, 0, 0, 0};
      uint32_t t = jlo;
      for (; t + kNlUnroll <= jhi; t += kNlUnroll) {
        uint32_t lf[kNlUnroll][4];
#pragma unroll
        for (uint32_t u = 0; u < kNlUnroll; ++u) {
          nl_load<WIDE>(a, st_row[t + u], v0, lf[u]);
        }
#pragma unroll
        for (uint32_t u = 0; u < kNlUnroll; ++u) {
          const uint32_t nd = st_node[t + u];
          const uint32_t f = nd & 0x7FFFFFFFu;
          const bool tf = nd >> 31;
          const uint64_t bit = 1ull << ((t + u) & 63);
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            if (live[i] && lf[u][i] != none && (uint64_t)lf[u][i] + step == (uint64_t)ls[i] &&
                (tf || v0 + i == f)) {
              acc[i] |= bit;
            }
          }
        }
      }
      for (; t < jhi; ++t) {
        uint32_t lf[4];
        nl_load<WIDE>(a, st_row[t], v0, lf);
        const uint32_t nd = st_node[t];
        const uint32_t f = nd & 0x7FFFFFFFu;
        const bool tf = nd >> 31;
        const uint64_t bit = 1ull << (t & 63);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          if (live[i] && lf[i] != none && (uint64_t)lf[i] + step == (uint64_t)ls[i] &&
              (tf || v0 + i == f)) {
            acc[i] |= bit;
          }
        }
      }
      if constexpr (WM > 1) {
#pragma unroll
        for (uint32_t ww = 0; ww < WM; ++ww) {
          if (ww == w) {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              held[ww][i] = acc[i];
            }
          }
        }
        continue;
      }
      const uint32_t wv0 = v0 - 4 * (threadIdx.x & 63u); // first node of the wave
      if (WM == 1 && wv0 + 256 <= a.V) {
        // each store instruction of the wave covers 1 KB contiguously: lane L
        // writes nodes wv0 + 2L, +1 (store 0) and wv0 + 128 + 2L, +1 (store
        // 1), fetched from the lanes that computed them (a lane's own four
        // nodes at a 32-byte stride left every line half-written per store)
        const uint32_t L = threadIdx.x & 63u;
        const int a0 = (int)(L >> 1), a1 = (int)(32u + (L >> 1));
        const bool odd = L & 1u;
        auto sh = [](uint64_t x, int lane) {
          return (uint64_t)__shfl((unsigned long long)x, lane, 64);
        };
        const uint64_t p0 = sh(acc[0], a0), p1 = sh(acc[1], a0), p2 = sh(acc[2], a0),
                       p3 = sh(acc[3], a0);
        const uint64_t r0 = sh(acc[0], a1), r1 = sh(acc[1], a1), r2 = sh(acc[2], a1),
                       r3 = sh(acc[3], a1);
        ulonglong2* o = reinterpret_cast<ulonglong2*>(nhrow + wv0);
        o[L] = odd ? make_ulonglong2(p2, p3) : make_ulonglong2(p0, p1);
        o[64 + L] = odd ? make_ulonglong2(r2, r3) : make_ulonglong2(r0, r1);
      } else if (Wm == 1 && v0 + 4 <= a.V) {
        ulonglong2* o = reinterpret_cast<ulonglong2*>(nhrow + v0);
        o[0] = make_ulonglong2(acc[0], acc[1]);
        o[1] = make_ulonglong2(acc[2], acc[3]);
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          if (v0 + i < a.V) {
            nhrow[(size_t)(v0 + i) * Wm + w] = acc[i];
          }
        }
      }
    }
    if constexpr (WM > 1) {
      // node-major: node v0 + i, word ww at (v0 + i) * WM + ww
      if (v0 + 4 <= a.V) {
        ulonglong2* o = reinterpret_cast<ulonglong2*>(nhrow + (size_t)v0 * WM);
        uint64_t flat[4 * WM];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
#pragma unroll
          for (uint32_t ww = 0; ww < WM; ++ww) {
            flat[i * WM + ww] = held[ww][i];
          }
        }
#pragma unroll
        for (uint32_t k = 0; k < 2 * WM; ++k) {
          o[k] = make_ulonglong2(flat[2 * k], flat[2 * k + 1]);
        }
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          if (v0 + i < a.V) {
#pragma unroll
            for (uint32_t ww = 0; ww < WM; ++ww) {
              nhrow[(size_t)(v0 + i) * WM + ww] = held[ww][i];
            }
          }
        }
      }
    }
  }
}

// Write traffic: a multi-word row (Wm > 1) is stored as 8-byte pieces at a
// stride of 8*Wm bytes; with the word loop outside the chunk loop every line
// was written Wm times, partially (PMC: 1.31 GB written for 0.95 GB of masks
// on the fabric).  Keeping all words in registers (r02 experiment) cost
// occupancy (91 VGPRs, 0.70 -> 0.82 ms); computing the words of a chunk back
// to back (nl_body_multi) keeps one word of accumulators live and lets L2
// merge the pieces of a line.
// chunks of 1024 nodes swept by one block (measured on the fabric: 2 ->
// 0.676 ms, 4 -> 0.682, 16 = whole rows -> 0.710; kNlUnroll 4 / 16 slower)
#ifndef OPENR_NL_CPB
#define OPENR_NL_CPB 2
#endif
constexpr uint32_t kNlChunksPerBlock = OPENR_NL_CPB;

// Logical block of a launch of n blocks such that consecutive logical blocks
// share an XCD (blocks b and b + 8 are dealt to one XCD, MI355X_MICROARCH
// "Workgroup dispatch"): XCD x of the round-robin deal gets the contiguous
// logical range [x*q + min(x, r), ...), q = n / 8, r = n % 8.  Speed only
// (L2 locality), never correctness: every logical block is still run once.
__device__ __forceinline__ uint32_t xcd_logical_block(uint32_t b, uint32_t n) {
  const uint32_t x = b & 7u, i = b >> 3, qn = n >> 3, r = n & 7u;
  return x * qn + min(x, r) + i;
}

// Byte-SIMD (SWAR) next-hop pass.  The compare of spf_nh_levels_kernel,
// lvl(n, v) + 1 == lvl(s, v), costs ~8 VALU ops per (neighbour, node): at
// Σ deg(s) * V = 2.3G pairs on the fabric that alone is ~0.5 ms of the
// chip's VALU issue.  Here a lane owns 16 nodes (one 16-byte load per
// neighbour row) and compares 4 level bytes per 32-bit op: with t = lvl(s, v)
// - 1 bytewise, a neighbour matches node v iff byte v of lvl(n, .) ^ t is 0
// and v is live (lvl(s, v) not 0 = the source, not 255 = unreached).  The
// zero-byte test leaves 0x80 in each matching byte; neighbour j = 8g + k of
// a 64-neighbour mask word ORs it, shifted right by 7 - k, into accumulator
// P[g], so byte i of P[0..7] is node i's mask word, 8 bits per P — a 4x4 byte
// transpose (v_perm) per group of four P hands each node its 64-bit word.
// ~7 VALU ops per (neighbour, 4 nodes).  Non-transit neighbours (drained,
// LinkState.cpp:829-836) match only the node they are (v == n), a uniform
// per-neighbour bit staged with the list.  One 128-thread block per source,
// each wave sweeping 1024-node chunks; mask words are staged 64 neighbours at
// a time, so any degree works.  A BFS deeper than 254 levels (flags[0]) takes
// the generic 32-bit-row compare in the same launch.
constexpr uint32_t kNsThreads = 128;
constexpr uint32_t kNsNodes = 16;
constexpr uint32_t kNsChunk = 64 * kNsNodes;

__device__ __forceinline__ uint32_t swar_zero_bytes(uint32_t x) {
  return ~(((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x | 0x7F7F7F7Fu); // 0x80 per zero byte
}

// byte i of p0..p3 -> out[i] = (p0.i, p1.i, p2.i, p3.i)
__device__ __forceinline__ void swar_transpose4(
    uint32_t p0, uint32_t p1, uint32_t p2, uint32_t p3, uint32_t (&out)[4]) {
  const uint32_t t0 = __builtin_amdgcn_perm(p1, p0, 0x05010400u);
  const uint32_t t1 = __builtin_amdgcn_perm(p1, p0, 0x07030602u);
  const uint32_t t2 = __builtin_amdgcn_perm(p3, p2, 0x05010400u);
  const uint32_t t3 = __builtin_amdgcn_perm(p3, p2, 0x07030602u);
  out[0] = __builtin_amdgcn_perm(t2, t0, 0x05040100u);
  out[1] = __builtin_amdgcn_perm(t2, t0, 0x07060302u);
  out[2] = __builtin_amdgcn_perm(t3, t1, 0x05040100u);
  out[3] = __builtin_amdgcn_perm(t3, t1, 0x07060302u);
}

// MsBfsArgs::lvl_only: source q's distances of nodes v0..v0+3 from their
// level bytes (lvl * scale below 255; 255 = unreached or deep, written by
// the BFS itself), one 16-byte store when all four are below 255
__device__ __forceinline__ void nl_dist_from_levels(
    const NhLevelsArgs& a, uint32_t q, uint32_t v0, uint32_t ls) {
  uint32_t* dw = a.dist_w + (size_t)q * a.Vp + v0;
  const uint32_t b[4] = {ls & 0xFFu, (ls >> 8) & 0xFFu, (ls >> 16) & 0xFFu, ls >> 24};
  if (v0 + 4 <= a.V && !swar_zero_bytes(~ls)) { // no byte is 255
    nt_u32x4 w;
    if (a.scale == 1) { // hop count / metric 1: no multiplies (quarter-rate v_mul_lo)
      w.x = b[0];
      w.y = b[1];
      w.z = b[2];
      w.w = b[3];
    } else {
      w.x = b[0] * a.scale;
      w.y = b[1] * a.scale;
      w.z = b[2] * a.scale;
      w.w = b[3] * a.scale;
    }
    st_stream(reinterpret_cast<nt_u32x4*>(dw), w, a.nt_store != 0);
    return;
  }
#pragma unroll
  for (uint32_t i = 0; i < 4; ++i) {
    if (v0 + i < a.V && b[i] < 255) {
      dw[i] = b[i] * a.scale;
    }
  }
}

// the generic branch (a BFS deeper than 254 levels): 32-bit rows, one node
// at a time; out of line so its registers do not weigh on the byte path
__device__ __noinline__ void nl_swar_deep(
    const NhLevelsArgs& a, const uint32_t* dist, uint32_t q, uint32_t v0, uint32_t w, uint32_t Wm,
    uint32_t cnt, uint64_t ntmask, const uint32_t* st_row, const uint32_t* st_node,
    uint8_t* nhrow, uint32_t B) {
  for (uint32_t i = 0; i < kNsNodes; ++i) {
    const uint32_t v = v0 + i;
    if (v >= a.V) {
      break;
    }
    uint64_t acc = 0;
    auto dget = [&](uint32_t row) {
      if (a.dist_w) { // levels below 255 are not in the 32-bit rows
        const uint32_t l = a.lvl[(size_t)row * a.Vp8 + v];
        if (l < 255) {
          return l * a.scale;
        }
      }
      return dist[(size_t)row * a.Vp + v];
    };
    const uint32_t ds = dget(q);
    if (a.dist_w && w == 0) {
      a.dist_w[(size_t)q * a.Vp + v] = ds;
    }
    if (ds != kInf32 && ds != 0) {
      for (uint32_t j = 0; j < cnt; ++j) {
        // st_row holds level-row byte offsets (row * Vp8)
        const uint32_t df = dget(st_row[j] / a.Vp8);
        const bool tr = !((ntmask >> j) & 1u) || st_node[j] == v;
        if (df != kInf32 && (uint64_t)df + a.scale == (uint64_t)ds && tr) {
          acc |= 1ull << j;
        }
      }
    }
    nh_store(nhrow, B, Wm, v, w, acc);
  }
}

// The SWAR pass for sources with at most kNsHeldMax mask words (every
// fabric source): all neighbours are staged once; a lane owns four nodes in
// each of the chunk's four 256-node segments (4-byte loads, 256 contiguous
// bytes per wave per neighbour row), computes every word of its four nodes
// back to back and stores the 4 x Wm words as one contiguous 32*Wm-byte run,
// so a wave writes 2*Wm KB of mask row contiguously per segment (the per-lane
// 16-node layout stored 16-byte pieces 128 bytes apart: twice the L2 write
// requests, profiles/r03e).
constexpr uint32_t kNsHeldMax = 3;
constexpr uint32_t kNsHeldWide = 8; // the held kernel's wide instance (4-8 words)

template <uint32_t T, uint32_t H>
__device__ __forceinline__ void nl_swar_held(
    const NhLevelsArgs& a, const uint8_t* lvl, uint32_t q, uint32_t c, uint32_t Wm, uint32_t n,
    uint32_t beg, uint8_t* nhrow_b, uint32_t B, const uint8_t* lvl_s, uint32_t* st_row,
    uint32_t* st_node, uint32_t* st_nt) {
  uint64_t* nhrow = reinterpret_cast<uint64_t*>(nhrow_b);
  const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
  for (uint32_t t = threadIdx.x; t < 64 * H; t += T) {
    bool nt = false;
    if (t < n) {
      const uint32_t f = a.nbrs[beg + t];
      nt = !((a.trbits[f >> 5] >> (f & 31)) & 1u);
      st_row[t] = (uint32_t)a.row_of[f] * a.Vp8;
      st_node[t] = f;
    }
    const uint64_t b = __ballot(nt);
    if (lane == 0) {
      st_nt[2 * (t >> 6)] = (uint32_t)b;
      st_nt[2 * (t >> 6) + 1] = (uint32_t)(b >> 32);
    }
  }
  __syncthreads();
  {
    {
      const uint32_t v0 = c * (4 * T) + wv * 256 + 4 * lane;
      if (v0 >= a.V) {
        return;
      }
      const uint32_t ls = *reinterpret_cast<const uint32_t*>(lvl_s + v0);
      const uint32_t tgt = ((ls | 0x80808080u) - 0x01010101u) ^ (~ls & 0x80808080u);
      const uint32_t live =
          0x80808080u & ~(swar_zero_bytes(ls) | swar_zero_bytes(~ls));
      if (a.dist_w) {
        nl_dist_from_levels(a, q, v0, ls);
      }
      uint64_t held[H][4];
#pragma unroll 1
      for (uint32_t w = 0; w < Wm; ++w) {
        {
          const uint32_t jlo = 64 * w, cnt = min(64u, n - min(n, jlo));
          const uint64_t ntmask =
              ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane(st_nt[2 * w + 1]) << 32) |
              (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane(st_nt[2 * w]);
          uint32_t P[8];
#pragma unroll
          for (int g = 0; g < 8; ++g) {
            P[g] = 0;
          }
#pragma unroll
          for (uint32_t g = 0; g < 8; ++g) {
            if (8 * g < cnt) {
              uint32_t lf[8];
#pragma unroll
              for (uint32_t kk = 0; kk < 8; ++kk) {
                lf[kk] = 0xFFFFFFFFu;
                if (8 * g + kk < cnt) {
                  lf[kk] = *reinterpret_cast<const uint32_t*>(lvl + st_row[jlo + 8 * g + kk] + v0);
                }
              }
              const uint32_t ntg = (uint32_t)(ntmask >> (8 * g)) & 0xFFu;
#pragma unroll
              for (uint32_t kk = 0; kk < 8; ++kk) {
                uint32_t m = live & swar_zero_bytes(lf[kk] ^ tgt);
                if ((ntg >> kk) & 1u) {
                  // a drained neighbour is a next hop only to itself
                  const uint32_t r = st_node[jlo + 8 * g + kk] - v0;
                  m &= r < 4u ? (0x80u << (8u * r)) : 0u;
                }
                P[g] |= m >> (7u - kk);
              }
            }
          }
          uint32_t lo[4], hi[4];
          swar_transpose4(P[0], P[1], P[2], P[3], lo);
          swar_transpose4(P[4], P[5], P[6], P[7], hi);
#pragma unroll
          for (uint32_t ww = 0; ww < H; ++ww) {
            if (ww == w) { // static register indices
#pragma unroll
              for (int i = 0; i < 4; ++i) {
                held[ww][i] = ((uint64_t)hi[i] << 32) | lo[i];
              }
            }
          }
        }
      }
      // node-major: node v0 + i, word w at (v0 + i) * Wm + w; narrow rows
      // (B < 8 bytes per node, one word) as one 4 / 8 / 16-byte run
      if (H <= 3 && B < 8) {
        nh_store4_narrow(nhrow_b, B, v0, a.V, held[0], a.nt_store != 0);
      } else if (H <= 3 && v0 + 4 <= a.V) {
        ulonglong2* o = reinterpret_cast<ulonglong2*>(nhrow + (size_t)v0 * Wm);
        if (Wm == 1) {
          o[0] = make_ulonglong2(held[0][0], held[0][1]);
          o[1] = make_ulonglong2(held[0][2], held[0][3]);
        } else if (Wm == 2) {
          o[0] = make_ulonglong2(held[0][0], held[1][0]);
          o[1] = make_ulonglong2(held[0][1], held[1][1]);
          o[2] = make_ulonglong2(held[0][2], held[1][2]);
          o[3] = make_ulonglong2(held[0][3], held[1][3]);
        } else {
          o[0] = make_ulonglong2(held[0][0], held[1][0]);
          o[1] = make_ulonglong2(held[2][0], held[0][1]);
          o[2] = make_ulonglong2(held[1][1], held[2][1]);
          o[3] = make_ulonglong2(held[0][2], held[1][2]);
          o[4] = make_ulonglong2(held[2][2], held[0][3]);
          o[5] = make_ulonglong2(held[1][3], held[2][3]);
        }
      } else {
#pragma unroll
        for (uint32_t i = 0; i < 4; ++i) {
          if (v0 + i < a.V) {
#pragma unroll
            for (uint32_t w = 0; w < H; ++w) {
              if (w < Wm) {
                nhrow[(size_t)(v0 + i) * Wm + w] = held[w][i];
              }
            }
          }
        }
      }
    }
  }
}

__global__ __launch_bounds__(kNsThreads) __attribute__((amdgpu_waves_per_eu(4)))
void spf_nh_levels_swar_kernel(NhLevelsArgs a, const uint32_t* big, uint32_t nbig) {
  __shared__ uint32_t st_row[64];
  __shared__ uint32_t st_node[64];
  __shared__ uint32_t st_nt[2]; // non-transit neighbours of the staged word
  const bool deep = (a.flags[0] & 1u) != 0; // uniform
  // sources with more than kNsHeldMax words (or every source of a deep BFS;
  // the held kernel takes the rest)
  for (uint32_t bi = blockIdx.x;; bi += gridDim.x) {
  if (deep ? bi >= a.nq : bi >= nbig) {
    break;
  }
  const uint32_t q = deep ? bi : big[bi];
  const uint32_t s = a.src[q];
  const uint32_t Wm = a.nh_w[q];
  uint8_t* nhrow_b = a.nhb + a.nhb_off[q];
  const uint32_t B = a.nh_b[q];
  uint64_t* nhrow = reinterpret_cast<uint64_t*>(nhrow_b);
  const uint32_t beg = a.nbr_off[s], n = a.nbr_off[s + 1] - beg;
  const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
  const uint32_t nchunks = (a.V + kNsChunk - 1) / kNsChunk;
  const uint32_t zv = a.zvar ? a.zvar[q] : 0u;
  const uint8_t* lvl = a.lvl + zv * a.lvl_vstride;
  const uint32_t* dist = a.dist + zv * a.dist_vstride;
  const uint8_t* lvl_s = lvl + (size_t)q * a.Vp8;
  for (uint32_t w = 0; w < Wm; ++w) {
    const uint32_t jlo = w * 64, cnt = min(64u, n - min(n, jlo));
    __syncthreads();
    if (threadIdx.x < 64) {
      bool nt = false;
      if (threadIdx.x < cnt) {
        const uint32_t f = a.nbrs[beg + jlo + threadIdx.x];
        nt = !((a.trbits[f >> 5] >> (f & 31)) & 1u);
        st_row[threadIdx.x] = (uint32_t)a.row_of[f] * a.Vp8;
        st_node[threadIdx.x] = f;
      }
      const uint64_t b = __ballot(nt);
      if (threadIdx.x == 0) {
        st_nt[0] = (uint32_t)b;
        st_nt[1] = (uint32_t)(b >> 32);
      }
    }
    __syncthreads();
    // readfirstlane returns int: widen through uint32_t (no sign extension)
    const uint64_t ntmask =
        ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane(st_nt[1]) << 32) |
        (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane(st_nt[0]);
    const uint32_t ngroups = (cnt + 7) / 8;
    for (uint32_t c = wv; c < nchunks; c += kNsThreads / 64) {
      const uint32_t v0 = c * kNsChunk + lane * kNsNodes;
      if (deep) {
        nl_swar_deep(a, dist, q, v0, w, Wm, cnt, ntmask, st_row, st_node, nhrow_b, B);
        continue;
      }
      const bool active = v0 < a.V;
      uint4 ls = make_uint4(0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu);
      if (active) {
        ls = *reinterpret_cast<const uint4*>(lvl_s + v0);
      }
      const uint32_t lsw[4] = {ls.x, ls.y, ls.z, ls.w};
      if (a.dist_w && w == 0 && active) {
#pragma unroll
        for (uint32_t k = 0; k < 4; ++k) {
          nl_dist_from_levels(a, q, v0 + 4 * k, lsw[k]);
        }
      }
      uint32_t tgt[4], live[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        // bytewise ls - 1 (no borrow across bytes), live = not 0, not 255
        tgt[k] = ((lsw[k] | 0x80808080u) - 0x01010101u) ^ (~lsw[k] & 0x80808080u);
        live[k] = 0x80808080u & ~(swar_zero_bytes(lsw[k]) | swar_zero_bytes(~lsw[k]));
      }
      uint32_t P[4][8];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
#pragma unroll
        for (int g = 0; g < 8; ++g) {
          P[k][g] = 0;
        }
      }
      if (active) {
#pragma unroll
        for (uint32_t g = 0; g < 8; ++g) {
          if (g < ngroups) {
            uint4 lf[8];
#pragma unroll
            for (uint32_t kk = 0; kk < 8; ++kk) {
              lf[kk] = make_uint4(0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu);
              if (8 * g + kk < cnt) {
                lf[kk] = *reinterpret_cast<const uint4*>(lvl + st_row[8 * g + kk] + v0);
              }
            }
            const uint32_t ntg = (uint32_t)(ntmask >> (8 * g)) & 0xFFu;
#pragma unroll
            for (uint32_t kk = 0; kk < 8; ++kk) {
              const uint32_t lw[4] = {lf[kk].x, lf[kk].y, lf[kk].z, lf[kk].w};
              uint32_t m[4];
#pragma unroll
              for (int k = 0; k < 4; ++k) {
                m[k] = live[k] & swar_zero_bytes(lw[k] ^ tgt[k]);
              }
              if ((ntg >> kk) & 1u) {
                // a drained neighbour is a next hop only to itself
                const uint32_t f = st_node[8 * g + kk];
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                  const uint32_t r = f - (v0 + 4u * k);
                  m[k] &= r < 4u ? (0x80u << (8u * r)) : 0u;
                }
              }
#pragma unroll
              for (int k = 0; k < 4; ++k) {
                P[k][g] |= m[k] >> (7u - kk);
              }
            }
          }
        }
      }
      if (!active) {
        continue;
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        uint32_t lo[4], hi[4];
        swar_transpose4(P[k][0], P[k][1], P[k][2], P[k][3], lo);
        swar_transpose4(P[k][4], P[k][5], P[k][6], P[k][7], hi);
        const uint32_t vk = v0 + 4u * k;
        if (B < 8) {
          const uint64_t x4[4] = {((uint64_t)hi[0] << 32) | lo[0], ((uint64_t)hi[1] << 32) | lo[1],
                                  ((uint64_t)hi[2] << 32) | lo[2], ((uint64_t)hi[3] << 32) | lo[3]};
          nh_store4_narrow(nhrow_b, B, vk, a.V, x4);
        } else if (Wm == 1 && vk + 4 <= a.V) {
          ulonglong2* o = reinterpret_cast<ulonglong2*>(nhrow + vk);
          o[0] = make_ulonglong2(((uint64_t)hi[0] << 32) | lo[0], ((uint64_t)hi[1] << 32) | lo[1]);
          o[1] = make_ulonglong2(((uint64_t)hi[2] << 32) | lo[2], ((uint64_t)hi[3] << 32) | lo[3]);
        } else {
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            if (vk + i < a.V) {
              nhrow[(size_t)(vk + i) * Wm + w] = ((uint64_t)hi[i] << 32) | lo[i];
            }
          }
        }
      }
    }
  }
  __syncthreads(); // the next source restages the neighbour list
  }
}

// Sources with at most kNsHeldMax mask words (all of the fabric's), unless the
// BFS went deeper than 254 levels (then spf_nh_levels_swar_kernel takes all).
// T threads per block, one block per (source, 4T-node chunk).  H = 3: the
// sources with at most 3 mask words (all of the 10k fabric's); H = 8: the
// sources with 4-8 words, listed in big[0, nmid) (a 20k fabric's SSWs)
template <uint32_t T, uint32_t H>
__global__ __launch_bounds__(T) void spf_nh_levels_held_kernel(
    NhLevelsArgs a, const uint32_t* big, uint32_t nmid) {
  __shared__ uint32_t st_row[H * 64];
  __shared__ uint32_t st_node[H * 64];
  __shared__ uint32_t st_nt[2 * H];
  // consecutive blocks: consecutive sources at the same chunk (neighbouring
  // name ranks share neighbours, so their row reads meet in L2); with
  // OPENR_NL_XCD=1 consecutive logical blocks also share an XCD
  const uint32_t bid = a.xcd_swizzle ? xcd_logical_block(blockIdx.x, gridDim.x) : blockIdx.x;
  const uint32_t nsrc = H <= 3 ? a.nq : nmid;
  uint32_t c = bid / nsrc;
  uint32_t q = H <= 3 ? bid - c * nsrc : big[bid - c * nsrc];
  if (H <= 3 && a.held_order) {
    const uint32_t it = a.held_order[blockIdx.x];
    if (it == kInf32) {
      return;
    }
    q = it / a.held_nch;
    c = it - q * a.held_nch;
  }
  const uint32_t Wm = a.nh_w[q];
  if ((a.flags[0] & 1u) != 0 || Wm > H || (H > 3 && Wm <= 3)) {
    return;
  }
  const uint32_t s = a.src[q];
  const uint32_t beg = a.nbr_off[s], n = a.nbr_off[s + 1] - beg;
  const uint8_t* lvl = a.lvl + (a.zvar ? a.zvar[q] * a.lvl_vstride : 0);
  nl_swar_held<T, H>(a, lvl, q, c, Wm, n, beg, a.nhb + a.nhb_off[q], a.nh_b[q],
                     lvl + (size_t)q * a.Vp8, st_row, st_node, st_nt);
}

// ---- held next-hop pass v2 (round 5): short dependency chains, shared rows
//
// The held kernel above is latency-bound, not bandwidth-bound: a block does
// ~5 KB of output behind a chain of dependent round trips (src[q] ->
// nbr_off[s] -> nbrs[] -> row_of[f] / trbits -> LDS + barrier -> the level
// rows), and 83 % of the fabric's blocks are RSW sources with 8 neighbours.
// Here the chain is cut to three trips and the RSW blocks are shared:
//  * the host lists, per source, its neighbours' level-row indices and node
//    ids once per query (NlEnt); lane j of each wave loads entry j and the
//    rows reach the loads as readlane scalars — no LDS, no barrier;
//  * sources whose distinct-neighbour lists are identical and short (<= GN
//    neighbours, one mask word: the 48 RSWs of a fabric pod share their 8
//    FSWs) form groups; a block serves GS of them on one chunk, holding the
//    neighbours' level words in registers and reading only each source's own
//    level row besides;
//  * block descriptors are indexed straight by blockIdx (one scalar trip).
// Same compare, masks and distance rows as nl_swar_held (byte for byte).
struct NlEnt {
  uint32_t row; // the neighbour's level-row index in the query (row_of)
  uint32_t node;
};
struct NlSolo {
  uint32_t q, n, lo, B; // query, neighbours, first NlEnt, mask bytes per node
  uint64_t nhb_off;     // byte offset of the query's mask row
  uint32_t Wm, pad;
};
struct NlSub { // GS (or fewer) sources with one neighbour list
  uint32_t m0, cnt, n, lo, B, pad;
};
struct NlMem {
  uint32_t q, pad;
  uint64_t nhb_off;
};
struct NlV2Args {
  const NlSolo* solo;
  const NlSub* subs;
  const NlMem* mem;
  const NlEnt* ent;
  uint32_t nsolo, nsub;
  // bytes of the level table (< 2^31: the kernel's buffer descriptor)
  uint32_t lvl_bytes;
  // measurement only (OPENR_NL_V2_DBG): bit 0 skips the solo items, bit 1 the
  // groups, bit 2 computes without storing (the results stay live)
  uint32_t dbg;
  // block order (OPENR_NL_V2_ORDER): 0 = all solo items chunk-major, then
  // all groups; 1 = chunk-major over both kinds (chunk c: its solo items,
  // then its groups); 2 = order 1 with XCD-contiguous logical ranges, so an
  // XCD sweeps ~1/8 of the chunks and the level-row slices its blocks read
  // stay in its L2 (round-robin dealing makes every XCD fetch every row);
  // 3 = chunk-major with the chunk's solo and group items interleaved in
  // proportion, so VALU-heavy solo blocks and store-heavy group blocks are
  // resident together; 4 = item-major; 5 = an explicit block map (xmap):
  // items of one neighbour class (same largest neighbour: a pod's FSWs, a
  // plane's SSWs, a pod's RSW groups) chunk by chunk, cut into 8 cost-
  // balanced ranges, range x on the blocks b = 8 j + x that the dispatcher
  // deals to XCD x, so a class's neighbour rows are fetched into one L2
  uint32_t order;
  const uint32_t* xmap = nullptr; // [nmap] item << 12 | chunk, ~0 = empty
  uint32_t nmap = 0;
  // round 6: 2-bit level rows (spf_lvl_trit_kernel: level mod 3, 3 =
  // unreached; row stride tstride = Vp8 / 4 bytes).  An item whose sources
  // are all transit reads its NEIGHBOURS' rows in this form (a quarter of
  // the bytes); nullptr = every item reads byte rows (the default; opt-in with OPENR_NL_TRIT=1; a
  // graph whose half-edges are not all paired)
  const uint8_t* trit = nullptr;
  uint32_t trit_bytes = 0;
  uint32_t tstride = 0;
  // round 6: 1 = the one-add compare when the BFS stayed below level 127
  // (MsBfsArgs::flags bit 1 clear; OPENR_NL_SHALLOW=0 turns it off)
  uint32_t shallow = 1;
};
constexpr uint32_t kNlGS = 8;  // sources per group block
constexpr uint32_t kNlGN = 16; // neighbours of a group source (one mask word, B <= 2)

__device__ __forceinline__ bool nl_transit(const uint32_t* trbits, uint32_t f) {
  return (trbits[f >> 5] >> (f & 31)) & 1u;
}

// Level words of neighbours base .. base+7 of a source (entries e[base ..]):
// the entries are wave-uniform, so they arrive by scalar loads (the list is
// padded by 64 entries, so reading past its end is safe) and the row offsets
// are scalar products; missing neighbours read as 0xFF bytes, which match no
// live node.
// The pass's per-query tables are read-only for the kernel's lifetime: seen
// through the constant address space, wave-uniform reads of them become
// scalar loads (no vector trip + v_readfirstlane before the row loads)
template <typename T>
using nl_cptr = const __attribute__((address_space(4))) T*;
template <typename T>
__device__ __forceinline__ nl_cptr<T> nl_const(const T* p) {
  return (nl_cptr<T>)p;
}

// A level word through the level table's buffer descriptor: the row offset
// is a scalar (SGPR soffset) and the lane's node offset a 32-bit voffset, so
// a load costs no vector address arithmetic (the 64-bit per-lane address of
// a global load was ~20 % of the pass's VALU instructions, profiles/r05k);
// reads past the table return 0 (hardware bounds check).
__device__ __forceinline__ uint32_t nl_lvl_word(__amdgpu_buffer_rsrc_t rs, uint32_t v0,
                                                uint32_t rowoff) {
  return (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(rs, (int)v0, (int)rowoff, 0);
}

__device__ __forceinline__ void nl_v3_ld8(__amdgpu_buffer_rsrc_t rs, uint32_t v0, uint32_t Vp8,
                                          nl_cptr<NlEnt> e, uint32_t rem, uint32_t (&lf)[8]) {
  uint32_t r[8];
#pragma unroll
  for (uint32_t kk = 0; kk < 8; ++kk) {
    r[kk] = __builtin_amdgcn_readfirstlane(e[kk].row);
  }
#pragma unroll
  for (uint32_t kk = 0; kk < 8; ++kk) {
    lf[kk] = 0xFFFFFFFFu;
    if (kk < rem) {
      lf[kk] = nl_lvl_word(rs, v0, r[kk] * Vp8);
    }
  }
}

// SWAR compares of eight neighbours' level words against the source's
// (tgt = level - 1 bytewise, live = not the source, not unreached): the 0x80
// of a matching byte lands in bit kk of that byte of P.  Drained neighbours
// (bit kk of ntg) match only their own node.
__device__ __forceinline__ uint32_t nl_v3_cmp8(const uint32_t (&lf)[8], uint32_t tgt,
                                               uint32_t live, uint32_t ntg, nl_cptr<NlEnt> e,
                                               uint32_t v0) {
  uint32_t P = 0;
#pragma unroll
  for (uint32_t kk = 0; kk < 8; ++kk) {
    uint32_t m = live & swar_zero_bytes(lf[kk] ^ tgt);
    if ((ntg >> kk) & 1u) {
      const uint32_t r = __builtin_amdgcn_readfirstlane(e[kk].node) - v0;
      m &= r < 4u ? (0x80u << (8u * r)) : 0u;
    }
    P = (P >> 1) | m; // neighbour kk's flag ends at bit kk after the eight steps
  }
  return P;
}

// Shallow compare (round 6): when every level of the batch is below
// kMsShallowLevel, the levels and the targets are below 128 and unreached
// is 255, so a byte of lf ^ tgt is zero iff its low seven bits are -- one
// masked add per neighbour instead of the exact zero-byte test, and no
// live / drained masks per neighbour: the NON-matches accumulate (bit kk of
// byte r set: neighbour kk does not match node r) and the caller applies
// the masks once per group.  A missing neighbour (0xFF bytes) never
// matches: 0xFF ^ tgt keeps low bits for tgt < 127.
__device__ __forceinline__ uint32_t nl_s_cmp8(const uint32_t (&lf)[8], uint32_t tgt) {
  uint32_t Q = 0;
#pragma unroll
  for (uint32_t kk = 0; kk < 8; ++kk) {
    const uint32_t t = ((lf[kk] ^ tgt) & 0x7F7F7F7Fu) + 0x7F7F7F7Fu;
    Q = (Q >> 1) | (t & 0x80808080u);
  }
  return Q;
}

// 0xFF in every byte whose 0x80 is set in `live`
__device__ __forceinline__ uint32_t nl_live8(uint32_t live) {
  const uint32_t x = live >> 7;
  return (x << 8) - x;
}

// the bits drained neighbours may keep: neighbour kk (a bit of ntg) only at
// its own node's byte (P layout: bit kk of byte r)
__device__ __forceinline__ uint32_t nl_s_allow(uint32_t ntg, nl_cptr<NlEnt> e, uint32_t v0) {
  uint32_t allow = 0xFFFFFFFFu;
  for (uint32_t kk = 0; kk < 8; ++kk) {
    if ((ntg >> kk) & 1u) {
      const uint32_t r = __builtin_amdgcn_readfirstlane(e[kk].node) - v0;
      allow &= ~(0x01010101u << kk) | (r < 4u ? 1u << (8u * r + kk) : 0u);
    }
  }
  return allow;
}

// ---- 2-bit neighbour rows (round 6)
//
// On a uniform metric with every half-edge paired, a transit source s and a
// transit neighbour n have BFS levels one apart at most at every node v
// (s -> n -> ... and n -> s -> ... are walks of one more link through a
// transit node), so lvl(n, v) == lvl(s, v) - 1 is decided by the levels mod
// 3.  Rows of 2 bits per node (level mod 3; 3 = unreached, which matches no
// target) carry a neighbour's row in a quarter of the bytes; the source's
// own byte row is still read for its distance row.  Lane layout as the byte
// pass: four consecutive nodes, here one byte (node r in bits 2r, 2r+1).
__device__ __forceinline__ uint32_t nl_trit_byte(__amdgpu_buffer_rsrc_t rt, uint32_t v0,
                                                 uint32_t rowoff) {
  return (uint32_t)__builtin_amdgcn_raw_buffer_load_b8(rt, (int)(v0 >> 2), (int)rowoff, 0);
}

// the source's targets (level - 1) mod 3 per field: 0 -> 2, 1 -> 0, 2 -> 1
__device__ __forceinline__ uint32_t nl_trit_target(uint32_t y) {
  const uint32_t lo = y & 0x55u, hi = (y >> 1) & 0x55u;
  return (hi & ~lo) | ((~(lo | hi) & 0x55u) << 1);
}

// bit 2r: node v0 + r is reached from the source and is not the source
__device__ __forceinline__ uint32_t nl_trit_live(uint32_t y, uint32_t s, uint32_t v0) {
  const uint32_t r = s - v0;
  return ~(y & (y >> 1)) & 0x55u & (r < 4u ? ~(1u << (2u * r)) : 0xFFu);
}

// byte r = 1 where neighbour byte nb's field r equals the target field
// (z's bits 2r moved to bit 8r: z * (1 + 2^6 + 2^12 + 2^18), whose carries
// land only on bits 7, 13 and 19, cleared by the mask)
__device__ __forceinline__ uint32_t nl_trit_match(uint32_t nb, uint32_t t2, uint32_t live2) {
  const uint32_t x = nb ^ t2;
  const uint32_t z = live2 & ~(x | (x >> 1));
  return __umul24(z, 0x41041u) & 0x01010101u;
}

__device__ __forceinline__ void nl_t_ld8(__amdgpu_buffer_rsrc_t rt, uint32_t v0, uint32_t tstride,
                                         nl_cptr<NlEnt> e, uint32_t rem, uint32_t (&lf)[8]) {
  uint32_t r[8];
#pragma unroll
  for (uint32_t kk = 0; kk < 8; ++kk) {
    r[kk] = __builtin_amdgcn_readfirstlane(e[kk].row);
  }
#pragma unroll
  for (uint32_t kk = 0; kk < 8; ++kk) {
    lf[kk] = 0xFFu;
    if (kk < rem) {
      lf[kk] = nl_trit_byte(rt, v0, r[kk] * tstride);
    }
  }
}

// nl_v3_cmp8 over 2-bit rows: same P layout (bit kk of byte r)
__device__ __forceinline__ uint32_t nl_t_cmp8(const uint32_t (&lf)[8], uint32_t t2, uint32_t live2,
                                              uint32_t ntg, nl_cptr<NlEnt> e, uint32_t v0) {
  uint32_t P = 0;
#pragma unroll
  for (uint32_t kk = 0; kk < 8; ++kk) {
    uint32_t m = nl_trit_match(lf[kk], t2, live2);
    if ((ntg >> kk) & 1u) {
      const uint32_t r = __builtin_amdgcn_readfirstlane(e[kk].node) - v0;
      m &= r < 4u ? (1u << (8u * r)) : 0u;
    }
    P |= m << kk;
  }
  return P;
}

// Level rows -> 2-bit rows: one thread per 16 nodes of a row (a 16-byte
// load, a 4-byte store); rows [0, nrows), stride Vp8 bytes in, Vp8 / 4 out.
// Skipped after a BFS deeper than 254 levels (flags[0]: the byte kernels
// then run without the v2 pass)
struct LvlTritArgs {
  const uint8_t* lvl;
  uint8_t* trit;
  const uint32_t* flags;
  uint32_t Vp8, nrows, per_row; // per_row = Vp8 / 16 threads
};

__global__ __launch_bounds__(256) void spf_lvl_trit_kernel(LvlTritArgs a) {
  if (a.flags && (a.flags[0] & 1u) != 0) {
    return;
  }
  const uint64_t t = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  const uint32_t r = (uint32_t)(t / a.per_row), c = (uint32_t)(t - (uint64_t)r * a.per_row);
  if (r >= a.nrows) {
    return;
  }
  const uint4 w = *reinterpret_cast<const uint4*>(a.lvl + (size_t)r * a.Vp8 + 16u * c);
  const uint32_t ws[4] = {w.x, w.y, w.z, w.w};
  uint32_t out = 0;
#pragma unroll
  for (uint32_t k = 0; k < 16; ++k) {
    const uint32_t b = (ws[k >> 2] >> (8u * (k & 3u))) & 0xFFu;
    // b mod 3 = b - 3 floor(b / 3), floor(b / 3) = (171 b) >> 9 for b < 256
    const uint32_t m3 = b - 3u * (__umul24(b, 171u) >> 9);
    out |= (b == 255u ? 3u : m3) << (2u * k);
  }
  *reinterpret_cast<uint32_t*>(a.trit + (size_t)r * (a.Vp8 / 4) + 4u * c) = out;
}

// Mask rows of B = 8 * Wm bytes per node, one wave's 256 nodes: a lane holds
// 4 consecutive nodes (32 * Wm contiguous bytes), so storing from registers
// puts 16-byte pieces 32 * Wm bytes apart in every wave instruction (partial
// cache lines; measured 1.9 TB/s against 4 TB/s for the coalesced distance
// rows, profiles/r05j).  The wave's tile goes through its LDS slice instead
// and leaves as 16 bytes per lane, 1 KB contiguous per instruction.  Every
// lane of the wave calls it.
__device__ __forceinline__ void nl_store_wide(uint8_t* row, uint32_t vbase, uint32_t V,
                                              uint32_t Wm, const uint64_t (&held)[kNsHeldMax][4],
                                              uint64_t* tile, uint32_t lane) {
#pragma unroll
  for (uint32_t i = 0; i < 4; ++i) {
#pragma unroll
    for (uint32_t w = 0; w < kNsHeldMax; ++w) {
      if (w < Wm) {
        tile[(4 * lane + i) * Wm + w] = held[w][i];
      }
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  const uint32_t bytes = min(256u, V - vbase) * 8 * Wm;
  uint8_t* dst = row + (size_t)vbase * 8 * Wm;
  const uint8_t* src = reinterpret_cast<const uint8_t*>(tile);
  for (uint32_t j = 0; j < 2 * Wm; ++j) {
    const uint32_t off = j * 1024 + 16 * lane;
    if (off + 16 <= bytes) {
      *reinterpret_cast<uint4*>(dst + off) = *reinterpret_cast<const uint4*>(src + off);
    } else if (off < bytes) { // bytes is a multiple of 8
      *reinterpret_cast<uint2*>(dst + off) = *reinterpret_cast<const uint2*>(src + off);
    }
  }
}

template <uint32_t T, bool TRIT, bool SH>
__device__ __forceinline__ void nl_v2_solo(const NhLevelsArgs& a, const NlV2Args& v,
                                           uint32_t k, uint32_t c, uint64_t* tile,
                                           __amdgpu_buffer_rsrc_t rs, __amdgpu_buffer_rsrc_t rt) {
  const nl_cptr<NlSolo> dp = nl_const(v.solo) + k;
  const NlSolo d{dp->q, dp->n, dp->lo, dp->B, dp->nhb_off, dp->Wm, 0u};
  const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
  const uint32_t vbase = c * (4 * T) + wv * 256;
  if (vbase >= a.V) {
    return; // wave-uniform
  }
  const uint32_t v0 = vbase + 4 * lane;
  const bool active = v0 < a.V;
  const uint8_t* lvl_v0 = a.lvl + v0;
  const nl_cptr<NlEnt> ent = nl_const(v.ent + d.lo);
  if (v.dbg & 8u) {
    // measurement: the pass's stores alone (same addresses, no loads)
    if (!(v.dbg & 32u) && d.B >= 8 && !(v.dbg & 64u)) {
      // wide masks through the LDS tile, as the pass stores them (every lane)
      uint64_t hx[kNsHeldMax][4];
#pragma unroll
      for (uint32_t w = 0; w < kNsHeldMax; ++w) {
#pragma unroll
        for (uint32_t i = 0; i < 4; ++i) {
          hx[w][i] = v0 + i + w;
        }
      }
      nl_store_wide(a.nhb + d.nhb_off, vbase, a.V, d.Wm, hx, tile, lane);
      if (active && a.dist_w && !(v.dbg & 16u)) {
        nl_dist_from_levels(a, d.q, v0, 0x01010101u * (v0 & 7u));
      }
      return;
    }
    if (!active) {
      return;
    }
    uint64_t x4[4] = {v0, v0 + 1, v0 + 2, v0 + 3};
    if (a.dist_w && !(v.dbg & 16u)) {
      nl_dist_from_levels(a, d.q, v0, 0x01010101u * (v0 & 7u));
    }
    uint8_t* nb = a.nhb + d.nhb_off;
    if (v.dbg & 32u) {
    } else if (d.B < 8) {
      nh_store4_narrow(nb, d.B, v0, a.V, x4);
    } else if (v.dbg & 64u) { // the register-layout stores (before LDS staging)
      uint64_t* nr = reinterpret_cast<uint64_t*>(nb);
      for (uint32_t w = 0; w < d.Wm; ++w) {
#pragma unroll
        for (uint32_t i = 0; i < 4; ++i) {
          if (v0 + i < a.V) {
            nr[(size_t)(v0 + i) * d.Wm + w] = x4[i];
          }
        }
      }
    }
    return;
  }
  // drained neighbours: lane j tests entry 64w + j (every lane takes part)
  uint64_t ntm[kNsHeldMax];
#pragma unroll
  for (uint32_t w = 0; w < kNsHeldMax; ++w) {
    bool nt = false;
    if (w < d.Wm && 64 * w + lane < d.n) {
      nt = !nl_transit(a.trbits, ent[64 * w + lane].node);
    }
    ntm[w] = __ballot(nt);
  }
  const uint32_t ls = active ? nl_lvl_word(rs, v0, d.q * a.Vp8) : 0xFFFFFFFFu;
  const uint32_t tgt = ((ls | 0x80808080u) - 0x01010101u) ^ (~ls & 0x80808080u);
  const uint32_t live = 0x80808080u & ~(swar_zero_bytes(ls) | swar_zero_bytes(~ls));
  uint32_t t2 = 0, live2 = 0;
  if constexpr (TRIT) {
    const uint32_t ys = active ? nl_trit_byte(rt, v0, d.q * v.tstride) : 0xFFu;
    t2 = nl_trit_target(ys);
    live2 = nl_trit_live(ys, nl_const(a.src)[d.q], v0);
  }
  uint64_t held[kNsHeldMax][4];
#pragma unroll 1
  for (uint32_t w = 0; w < d.Wm; ++w) {
    const uint32_t cnt = min(64u, d.n - min(d.n, 64 * w));
    const uint64_t ntmask = w == 0 ? ntm[0] : (w == 1 ? ntm[1] : ntm[2]);
    const nl_cptr<NlEnt> ew = ent + 64 * w;
    uint32_t P[8];
    uint32_t A[8], Bq[8];
    auto ld8 = [&](nl_cptr<NlEnt> e8, uint32_t rem, uint32_t(&lf)[8]) {
      if constexpr (TRIT) {
        nl_t_ld8(rt, v0, v.tstride, e8, rem, lf);
      } else {
        nl_v3_ld8(rs, v0, a.Vp8, e8, rem, lf);
      }
    };
    ld8(ew, cnt, A);
#pragma unroll
    for (uint32_t g = 0; g < 8; ++g) {
      P[g] = 0;
      if (8 * g < cnt) {
        // the next group's loads go out before this group's compares
        if (g + 1 < 8 && 8 * (g + 1) < cnt) {
          if (g & 1u) {
            ld8(ew + 8 * (g + 1), cnt - 8 * (g + 1), A);
          } else {
            ld8(ew + 8 * (g + 1), cnt - 8 * (g + 1), Bq);
          }
        }
        const uint32_t ntg = (uint32_t)(ntmask >> (8 * g)) & 0xFFu;
        if constexpr (TRIT) {
          P[g] = nl_t_cmp8((g & 1u) ? Bq : A, t2, live2, ntg, ew + 8 * g, v0);
        } else if constexpr (SH) {
          const uint32_t Q = nl_s_cmp8((g & 1u) ? Bq : A, tgt);
          P[g] = ~Q & nl_live8(live) & (ntg ? nl_s_allow(ntg, ew + 8 * g, v0) : 0xFFFFFFFFu);
        } else {
          P[g] = nl_v3_cmp8((g & 1u) ? Bq : A, tgt, live, ntg, ew + 8 * g, v0);
        }
      }
    }
    uint32_t lo[4], hi[4];
    swar_transpose4(P[0], P[1], P[2], P[3], lo);
    swar_transpose4(P[4], P[5], P[6], P[7], hi);
#pragma unroll
    for (uint32_t ww = 0; ww < kNsHeldMax; ++ww) {
      if (ww == w) { // static register indices
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          held[ww][i] = ((uint64_t)hi[i] << 32) | lo[i];
        }
      }
    }
  }
  if (v.dbg & 4u) {
    uint64_t x = 0;
#pragma unroll
    for (uint32_t w = 0; w < kNsHeldMax; ++w) {
      x ^= held[w][0] ^ held[w][1] ^ held[w][2] ^ held[w][3];
    }
    if (x != 0x5A5A5A5A12345678ull) {
      return; // measurement: no stores
    }
  }
  uint8_t* nhrow_b = a.nhb + d.nhb_off;
  if (d.B >= 8 && !(v.dbg & 64u)) {
    nl_store_wide(nhrow_b, vbase, a.V, d.Wm, held, tile, lane); // every lane
    if (active && a.dist_w) {
      nl_dist_from_levels(a, d.q, v0, ls);
    }
    return;
  }
  if (!active) {
    return;
  }
  if (a.dist_w) {
    nl_dist_from_levels(a, d.q, v0, ls);
  }
  uint64_t* nhrow = reinterpret_cast<uint64_t*>(nhrow_b);
  const uint32_t Wm = d.Wm;
  if (d.B < 8) {
    nh_store4_narrow(nhrow_b, d.B, v0, a.V, held[0], a.nt_store != 0);
  } else if (v0 + 4 <= a.V) {
    ulonglong2* o = reinterpret_cast<ulonglong2*>(nhrow + (size_t)v0 * Wm);
    if (Wm == 1) {
      o[0] = make_ulonglong2(held[0][0], held[0][1]);
      o[1] = make_ulonglong2(held[0][2], held[0][3]);
    } else if (Wm == 2) {
      o[0] = make_ulonglong2(held[0][0], held[1][0]);
      o[1] = make_ulonglong2(held[0][1], held[1][1]);
      o[2] = make_ulonglong2(held[0][2], held[1][2]);
      o[3] = make_ulonglong2(held[0][3], held[1][3]);
    } else {
      o[0] = make_ulonglong2(held[0][0], held[1][0]);
      o[1] = make_ulonglong2(held[2][0], held[0][1]);
      o[2] = make_ulonglong2(held[1][1], held[2][1]);
      o[3] = make_ulonglong2(held[0][2], held[1][2]);
      o[4] = make_ulonglong2(held[2][2], held[0][3]);
      o[5] = make_ulonglong2(held[1][3], held[2][3]);
    }
  } else {
#pragma unroll
    for (uint32_t i = 0; i < 4; ++i) {
      if (v0 + i < a.V) {
#pragma unroll
        for (uint32_t w = 0; w < kNsHeldMax; ++w) {
          if (w < Wm) {
            nhrow[(size_t)(v0 + i) * Wm + w] = held[w][i];
          }
        }
      }
    }
  }
}

template <uint32_t T, bool TRIT, bool SH>
__device__ __forceinline__ void nl_v2_group(const NhLevelsArgs& a, const NlV2Args& v,
                                            uint32_t k, uint32_t c,
                                            __amdgpu_buffer_rsrc_t rs, __amdgpu_buffer_rsrc_t rt) {
  const nl_cptr<NlSub> dp = nl_const(v.subs) + k;
  const NlSub d{dp->m0, dp->cnt, dp->n, dp->lo, dp->B, 0u};
  const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
  const uint32_t vbase = c * (4 * T) + wv * 256;
  if (vbase >= a.V) {
    return; // wave-uniform
  }
  const uint32_t v0 = vbase + 4 * lane;
  const bool active = v0 < a.V;
  const uint8_t* lvl_v0 = a.lvl + v0;
  const nl_cptr<NlEnt> ent = nl_const(v.ent + d.lo);
  const nl_cptr<NlMem> mem = nl_const(v.mem + d.m0);
  if (v.dbg & 8u) {
    // measurement: the group's stores alone (same addresses, no loads)
    if (!active) {
      return;
    }
    for (uint32_t i = 0; i < d.cnt; ++i) {
      const NlMem m{mem[i].q, 0u, mem[i].nhb_off};
      uint8_t* row = a.nhb + m.nhb_off;
      if (v0 + 4 <= a.V && !(v.dbg & 32u)) {
        if (d.B == 1) {
          *reinterpret_cast<uint32_t*>(row + v0) = v0;
        } else {
          *reinterpret_cast<nt_u32x2*>(row + 2 * (size_t)v0) = nt_u32x2{v0, v0};
        }
      }
      if (a.dist_w && !(v.dbg & 16u)) {
        nl_dist_from_levels(a, m.q, v0, 0x01010101u * (v0 & 7u));
      }
    }
    return;
  }
  bool nt = false;
  if (lane < d.n) {
    nt = !nl_transit(a.trbits, ent[lane].node);
  }
  const uint64_t ntmask = __ballot(nt);
  // the neighbours' level words: loaded once, held for every source
  uint32_t lf[kNlGN];
  {
    uint32_t r[kNlGN];
#pragma unroll
    for (uint32_t j = 0; j < kNlGN; ++j) {
      r[j] = __builtin_amdgcn_readfirstlane(ent[j].row);
    }
#pragma unroll
    for (uint32_t j = 0; j < kNlGN; ++j) {
      lf[j] = TRIT ? 0xFFu : 0xFFFFFFFFu;
      if (j < d.n) {
        if constexpr (TRIT) {
          lf[j] = nl_trit_byte(rt, v0, r[j] * v.tstride);
        } else {
          lf[j] = nl_lvl_word(rs, v0, r[j] * a.Vp8);
        }
      }
    }
  }
  uint32_t qs[kNlGS];
  uint32_t ls[kNlGS];
  uint32_t ys[kNlGS]; // TRIT: the members' own 2-bit words
#pragma unroll
  for (uint32_t i = 0; i < kNlGS; ++i) {
    qs[i] = __builtin_amdgcn_readfirstlane(mem[i].q); // past cnt: padding, unused
  }
#pragma unroll
  for (uint32_t i = 0; i < kNlGS; ++i) {
    ls[i] = 0xFFFFFFFFu;
    ys[i] = 0xFFu;
    if (i < d.cnt) {
      ls[i] = nl_lvl_word(rs, v0, qs[i] * a.Vp8);
      if constexpr (TRIT) {
        ys[i] = nl_trit_byte(rt, v0, qs[i] * v.tstride);
      }
    }
  }
  // per neighbour: the byte lanes a match may set (a drained neighbour only
  // its own node), the same for every source of the group
  uint32_t allow[kNlGN];
#pragma unroll
  for (uint32_t j = 0; j < kNlGN; ++j) {
    allow[j] = 0xFFFFFFFFu;
    if ((ntmask >> j) & 1u) {
      const uint32_t r = __builtin_amdgcn_readfirstlane(ent[j].node) - v0;
      allow[j] = r < 4u ? ((TRIT ? 0x01u : 0x80u) << (8u * r)) : 0u;
    }
  }
  // SH: the drained neighbours' masks in the P layout, once for every member
  uint32_t allow8[2] = {0xFFFFFFFFu, 0xFFFFFFFFu};
  if constexpr (SH) {
    if (ntmask) {
      allow8[0] = nl_s_allow((uint32_t)ntmask & 0xFFu, ent, v0);
      allow8[1] = nl_s_allow((uint32_t)(ntmask >> 8) & 0xFFu, ent + 8, v0);
    }
  }
  if (!active) {
    return;
  }
#pragma unroll
  for (uint32_t i = 0; i < kNlGS; ++i) {
    if (i < d.cnt) {
      const uint32_t x = ls[i];
      uint32_t P0 = 0, P1 = 0;
      if constexpr (TRIT) {
        const uint32_t t2 = nl_trit_target(ys[i]);
        const uint32_t live2 = nl_trit_live(ys[i], nl_const(a.src)[qs[i]], v0);
#pragma unroll
        for (uint32_t j = 0; j < kNlGN; ++j) {
          if (j < d.n) {
            const uint32_t m = allow[j] & nl_trit_match(lf[j], t2, live2);
            if (j < 8) {
              P0 |= m << j;
            } else {
              P1 |= m << (j - 8u);
            }
          }
        }
      } else if constexpr (SH) {
        // one masked add per neighbour, masks once (nl_s_cmp8)
        const uint32_t tgt = ((x | 0x80808080u) - 0x01010101u) ^ (~x & 0x80808080u);
        const uint32_t live = 0x80808080u & ~(swar_zero_bytes(x) | swar_zero_bytes(~x));
        const uint32_t l8 = nl_live8(live);
        uint32_t Q0 = 0;
#pragma unroll
        for (uint32_t j = 0; j < 8; ++j) {
          const uint32_t t = ((lf[j] ^ tgt) & 0x7F7F7F7Fu) + 0x7F7F7F7Fu;
          Q0 = (Q0 >> 1) | (t & 0x80808080u);
        }
        P0 = ~Q0 & l8 & allow8[0];
        if (d.n > 8) {
          uint32_t Q1 = 0;
#pragma unroll
          for (uint32_t j = 8; j < kNlGN; ++j) {
            const uint32_t t = ((lf[j] ^ tgt) & 0x7F7F7F7Fu) + 0x7F7F7F7Fu;
            Q1 = (Q1 >> 1) | (t & 0x80808080u);
          }
          P1 = ~Q1 & l8 & allow8[1];
        }
      } else {
        const uint32_t tgt = ((x | 0x80808080u) - 0x01010101u) ^ (~x & 0x80808080u);
        const uint32_t live = 0x80808080u & ~(swar_zero_bytes(x) | swar_zero_bytes(~x));
#pragma unroll
        for (uint32_t j = 0; j < kNlGN; ++j) {
          if (j < d.n) {
            const uint32_t m = live & allow[j] & swar_zero_bytes(lf[j] ^ tgt);
            if (j < 8) {
              P0 |= m >> (7u - j);
            } else {
              P1 |= m >> (15u - j);
            }
          }
        }
      }
      uint8_t* row = a.nhb + __builtin_amdgcn_readfirstlane((uint32_t)mem[i].nhb_off) +
                     ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(mem[i].nhb_off >> 32)) << 32);
      if ((v.dbg & 4u) && (P0 ^ P1) != 0x5A5A5A5Au) {
        continue; // measurement: no stores
      }
      if (v0 + 4 <= a.V) {
        if (d.B == 1) {
          st_stream(reinterpret_cast<uint32_t*>(row + v0), P0, a.nt_store != 0);
        } else {
          nt_u32x2 w2;
          w2.x = __builtin_amdgcn_perm(P1, P0, 0x05010400u); // nodes 0, 1 (16 bits each)
          w2.y = __builtin_amdgcn_perm(P1, P0, 0x07030602u); // nodes 2, 3
          st_stream(reinterpret_cast<nt_u32x2*>(row + 2 * (size_t)v0), w2, a.nt_store != 0);
        }
      } else {
#pragma unroll
        for (uint32_t b = 0; b < 4; ++b) {
          if (v0 + b < a.V) {
            const uint32_t lo8 = (P0 >> (8 * b)) & 0xFFu, hi8 = (P1 >> (8 * b)) & 0xFFu;
            nh_store(row, d.B, 1, v0 + b, 0, lo8 | (hi8 << 8));
          }
        }
      }
      if (a.dist_w) {
        nl_dist_from_levels(a, qs[i], v0, x);
      }
    }
  }
}

// blocks [0, nsolo * nch): solo (source, chunk) items, chunk-major (the
// heavy SSW / FSW sources of the fabric first); then the groups' (sub-group,
// chunk) items.  A BFS deeper than 254 levels leaves everything to
// spf_nh_levels_swar_kernel.
// TRITS: the instance with the 2-bit neighbour-row path compiled in
// (OPENR_NL_TRIT=1); the default instance carries the byte path alone
template <uint32_t T, bool TRITS>
__global__ __launch_bounds__(T) void spf_nh_levels_v2_kernel(NhLevelsArgs a, NlV2Args v) {
  // per wave: the 256-node mask tile of a wide solo source (nl_store_wide)
  __shared__ uint64_t tiles[T / 64][256 * kNsHeldMax];
  uint64_t* tile = tiles[threadIdx.x >> 6];
  const uint32_t fl = a.flags[0];
  if (fl & 1u) {
    return;
  }
  // every level below kMsShallowLevel: the one-add compare (nl_s_cmp8)
  const bool sh = v.shallow && !(fl & 2u);
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.lvl, (short)0, (int)v.lvl_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rt =
      __builtin_amdgcn_make_buffer_rsrc((void*)v.trit, (short)0, (int)v.trit_bytes, 0x00020000);
  // 2-bit neighbour rows for items whose sources are all transit (read at
  // run time: spf_graph_set_transit patches the bits between runs)
  const nl_cptr<uint32_t> tr = nl_const(a.trbits);
  const nl_cptr<uint32_t> srcs = nl_const(a.src);
  auto transit = [&](uint32_t q) __attribute__((always_inline)) {
    const uint32_t f = srcs[q];
    return ((tr[f >> 5] >> (f & 31u)) & 1u) != 0;
  };
  // (always_inline: as out-of-line calls these took a 440-byte stack frame
  // and 132 VGPRs in the TRITS instance)
  auto nl_v2_solo_t = [&](uint32_t k, uint32_t c) __attribute__((always_inline)) {
    if constexpr (TRITS) {
      if (v.trit && transit(nl_const(v.solo)[k].q)) {
        nl_v2_solo<T, true, false>(a, v, k, c, tile, rs, rt);
        return;
      }
    }
    if (sh) {
      nl_v2_solo<T, false, true>(a, v, k, c, tile, rs, rt);
    } else {
      nl_v2_solo<T, false, false>(a, v, k, c, tile, rs, rt);
    }
  };
  auto nl_v2_group_t = [&](uint32_t k, uint32_t c) __attribute__((always_inline)) {
    bool all = TRITS && v.trit != nullptr;
    if (all) {
      const nl_cptr<NlSub> dp = nl_const(v.subs) + k;
      const uint32_t m0 = dp->m0, cnt = dp->cnt;
      const nl_cptr<NlMem> mem = nl_const(v.mem) + m0;
      for (uint32_t i = 0; i < cnt; ++i) {
        all = all && transit(mem[i].q);
      }
    }
    if constexpr (TRITS) {
      if (all) {
        nl_v2_group<T, true, false>(a, v, k, c, rs, rt);
        return;
      }
    }
    if (sh) {
      nl_v2_group<T, false, true>(a, v, k, c, rs, rt);
    } else {
      nl_v2_group<T, false, false>(a, v, k, c, rs, rt);
    }
  };
  if (v.order == 5) {
    const uint32_t e = v.xmap[blockIdx.x];
    if (e == kInf32) {
      return; // padding of a shorter XCD range
    }
    const uint32_t k = e >> 12, c = e & 0xFFFu;
    if (k < v.nsolo) {
      nl_v2_solo_t(k, c);
    } else {
      nl_v2_group_t(k - v.nsolo, c);
    }
    return;
  }
  if (v.order != 0) {
    const uint32_t bid = v.order == 2 ? xcd_logical_block(blockIdx.x, gridDim.x) : blockIdx.x;
    const uint32_t per = v.nsolo + v.nsub;
    uint32_t c = bid / per, k = bid - c * per;
    if (v.order == 4) { // item-major: an item's chunks back to back
      const uint32_t nch = (a.V + 4 * T - 1) / (4 * T);
      k = bid / nch;
      c = bid - k * nch;
    }
    if (v.order >= 3) {
      // Bresenham spread of the nsub group items over the chunk's items
      const uint32_t gi = (uint32_t)((uint64_t)k * v.nsub / per);
      const bool grp = (uint32_t)((uint64_t)(k + 1) * v.nsub / per) > gi;
      k = grp ? v.nsolo + gi : k - gi;
    }
    if (k < v.nsolo) {
      if (!(v.dbg & 1u)) {
        nl_v2_solo_t(k, c);
      }
    } else if (!(v.dbg & 2u)) {
      nl_v2_group_t(k - v.nsolo, c);
    }
    return;
  }
  const uint32_t bid = blockIdx.x;
  const uint32_t ns = v.nsolo * ((a.V + 4 * T - 1) / (4 * T));
  if (bid < ns) {
    if (v.dbg & 1u) {
      return;
    }
    const uint32_t c = bid / v.nsolo;
    nl_v2_solo_t(bid - c * v.nsolo, c);
  } else {
    if (v.dbg & 2u) {
      return;
    }
    const uint32_t b2 = bid - ns, c = b2 / v.nsub;
    nl_v2_group_t(b2 - c * v.nsub, c);
  }
}

// Working word rows -> byte-strided output rows, after a plan whose kernels
// wrote the word layout (spf_query::narrow): one block per (query, 1,024
// nodes), four nodes per thread; narrow rows (B < 8) keep the low 8 * B bits
// of each node's single word, the others are copied word for word.  Per-query
// offsets / widths from device arrays, or (off == nullptr) the scalars of one
// row.
struct NhNarrowArgs {
  // queries the what-if screen already wrote in the output layout
  // (skip[q] == 1); nullptr: none
  const uint32_t* skip = nullptr;
  const uint64_t* src;
  uint8_t* dst;
  const uint64_t* src_off; // words
  const uint64_t* dst_off; // bytes
  const uint32_t* nb;
  const uint32_t* nw;
  uint64_t src_off1, dst_off1;
  uint32_t nb1, nw1;
  uint32_t V, nq;
};

__global__ __launch_bounds__(256) void spf_nh_narrow_kernel(NhNarrowArgs a) {
  const uint32_t nch = (a.V + 1023) / 1024;
  const uint32_t q = blockIdx.x / nch, c = blockIdx.x - q * nch;
  if (q >= a.nq || (a.skip && a.skip[q] == 1u)) {
    return;
  }
  const bool list = a.src_off != nullptr;
  const uint64_t* s = a.src + (list ? a.src_off[q] : a.src_off1);
  uint8_t* d = a.dst + (list ? a.dst_off[q] : a.dst_off1);
  const uint32_t B = list ? a.nb[q] : a.nb1, W = list ? a.nw[q] : a.nw1;
  const uint32_t v0 = c * 1024 + 4 * threadIdx.x;
  if (v0 >= a.V) {
    return;
  }
  if (B < 8) {
    uint64_t x[4];
#pragma unroll
    for (uint32_t i = 0; i < 4; ++i) {
      x[i] = v0 + i < a.V ? s[v0 + i] : 0ull;
    }
    nh_store4_narrow(d, B, v0, a.V, x);
    return;
  }
  uint64_t* dw = reinterpret_cast<uint64_t*>(d);
  const size_t e1 = (size_t)min(v0 + 4, a.V) * W;
  for (size_t e = (size_t)v0 * W; e < e1; ++e) {
    dw[e] = s[e];
  }
}

// ------------------------------------------------- zero-metric plan helpers
//
// A uniform metric c plus a few node-disjoint metric-0 links (DESIGN.md §2,
// "zero-metric plan").  DijkstraQ settles a plateau {a, b} (equal distance,
// joined by a metric-0 link) in (metric, name) order among DISCOVERED nodes
// (LinkState.h:483-535), and a node takes next hops only from neighbours
// settled before it (LinkState.cpp:842-871), so the metric-0 half-edge from
// the later-settled end into the earlier one never carries next hops.  For a
// source s the reference's next hops are therefore the order-free
// all-sources rule on G minus that half-edge; with k zero links there are
// 2^k such graphs ("variants", bit i set: link i's b end settles first,
// a -> b dropped; clear: b -> a dropped), and each gets its own MS-BFS
// table.  spf_zvar_kernel picks each source's variant from the distances
// (d = min over the variants, which is the distance in G): a plateau end is
// discovered before the plateau starts iff it is the source or the head of
// a usable tight in-edge of positive metric; two such ends settle by name
// rank, else the discovered end first.

struct ZvarArgs {
  const uint32_t* row;
  const uint32_t* col;
  const uint32_t* win; // metric of the half-edge col[e] -> (row owner)
  const uint32_t* trbits;
  const uint32_t* src;
  const uint32_t* dist;  // [nvar][nrows][Vp]
  const uint32_t* links; // [nlinks][2] ends (a < b)
  uint8_t* zvar;         // [nq]
  uint64_t vstride;      // nrows * Vp
  uint32_t Vp, nq, nvar, nlinks;
};

__global__ void spf_zvar_kernel(ZvarArgs a) {
  const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= a.nq) {
    return;
  }
  const uint32_t s = a.src[q];
  const uint32_t* d0 = a.dist + (size_t)q * a.Vp;
  auto dmin = [&](uint32_t x) {
    uint32_t m = kInf32;
    for (uint32_t j = 0; j < a.nvar; ++j) {
      m = min(m, d0[j * a.vstride + x]);
    }
    return m;
  };
  auto seed = [&](uint32_t x, uint32_t dx) {
    if (x == s) {
      return true;
    }
    for (uint32_t e = a.row[x]; e < a.row[x + 1]; ++e) {
      const uint32_t u = a.col[e], w = a.win[e];
      if (w == 0 || !(u == s || ((a.trbits[u >> 5] >> (u & 31)) & 1u))) {
        continue;
      }
      const uint32_t du = dmin(u);
      if (du != kInf32 && (uint64_t)du + w == dx) {
        return true;
      }
    }
    return false;
  };
  uint32_t var = 0;
  for (uint32_t i = 0; i < a.nlinks; ++i) {
    const uint32_t x = a.links[2 * i], y = a.links[2 * i + 1];
    const uint32_t dx = dmin(x), dy = dmin(y);
    if (dx == kInf32 || dx != dy) {
      continue; // no plateau: either variant serves
    }
    const bool sx = seed(x, dx), sy = seed(y, dy);
    if (sy && !sx) { // both discovered: x (the smaller rank) first
      var |= 1u << i;
    }
  }
  a.zvar[q] = (uint8_t)var;
}

// the output rows: source q's distances from its own variant table
__global__ void spf_zrows_kernel(uint32_t* dist, const uint8_t* zvar, uint64_t vstride, uint32_t Vp) {
  const uint32_t q = blockIdx.x;
  const uint32_t zv = zvar[q];
  if (!zv) {
    return;
  }
  const uint4* in = reinterpret_cast<const uint4*>(dist + zv * vstride + (size_t)q * Vp);
  uint4* out = reinterpret_cast<uint4*>(dist + (size_t)q * Vp);
  for (uint32_t i = threadIdx.x; i < Vp / 4; i += blockDim.x) {
    out[i] = in[i];
  }
}

// a 64-bit distance row (wide plan) into a 32-bit one
__global__ void spf_rows64to32_kernel(const uint64_t* in, uint32_t* out, uint32_t V) {
  for (uint32_t v = blockIdx.x * blockDim.x + threadIdx.x; v < V; v += gridDim.x * blockDim.x) {
    const uint64_t d = in[v];
    out[v] = d == SPF_UNREACHABLE ? kInf32 : (uint32_t)d;
  }
}

// six waves per SIMD (<= 80 VGPRs), as before the chunk-inner word loop
__global__ __launch_bounds__(kNlThreads) __attribute__((amdgpu_waves_per_eu(6)))
void spf_nh_levels_kernel(NhLevelsArgs a) {
  __shared__ uint32_t st_row[kNlStage];
  __shared__ uint32_t st_node[kNlStage];
  const uint32_t nchunks = (a.V + kNlChunk - 1) / kNlChunk;
  // sources of one pod / plane are adjacent name ranks and share neighbours:
  // run them on one XCD so its L2 serves their neighbours' level rows (the
  // 8 FSWs of a pod all read its 48 RSW rows; dealt round-robin they fetched
  // each RSW row once per XCD)
  const uint32_t bid = a.xcd_swizzle ? xcd_logical_block(blockIdx.x, gridDim.x) : blockIdx.x;
  const uint32_t cb = bid / a.nq;
  const uint32_t q = bid - cb * a.nq;
  const uint32_t s = a.src[q];
  const uint32_t c0 = cb * kNlChunksPerBlock;
  const uint32_t c1 = min(nchunks, c0 + kNlChunksPerBlock);
  const uint32_t deg = a.nbr_off[s + 1] - a.nbr_off[s];
  const bool big = deg > kNlStage; // uniform per block
  const uint32_t wm = a.nh_w[q];
  if ((a.flags[0] & 1u) != 0) {
    if (big) {
      nl_body_multi_staged<true>(a, q, s, c0, c1, st_row, st_node);
    } else if (wm == 1) {
      nl_body_multi<true, 1>(a, q, s, c0, c1, st_row, st_node);
    } else {
      nl_body_multi<true, 0>(a, q, s, c0, c1, st_row, st_node);
    }
  } else {
    if (big) {
      nl_body_multi_staged<false>(a, q, s, c0, c1, st_row, st_node);
    } else if (wm == 1) {
      nl_body_multi<false, 1>(a, q, s, c0, c1, st_row, st_node);
    } else if (wm == 2 && a.held_words) {
      nl_body_multi<false, 2>(a, q, s, c0, c1, st_row, st_node);
    } else if (wm == 3 && a.held_words) {
      nl_body_multi<false, 3>(a, q, s, c0, c1, st_row, st_node);
    } else {
      nl_body_multi<false, 0>(a, q, s, c0, c1, st_row, st_node);
    }
  }
}

// ------------------------------------------------------------- exact kernel

struct ExactArgs {
  const uint32_t* row;
  const uint32_t* col;
  const uint64_t* w64;
  const uint32_t* link;
  const uint32_t* slot;
  const uint32_t* trbits;
  const uint32_t* src;
  const uint32_t* ign_off;
  const uint32_t* ign;
  const uint64_t* nh_off;
  const uint32_t* nh_w;
  uint64_t* dist_out;
  uint64_t* nh_out;
  uint32_t* order_out;
  uint32_t* scratch; // per query: pos[V] + heap[V]
  uint32_t V;
  uint32_t nq;
  uint32_t unit;
  uint32_t want_nh;
};

__device__ __forceinline__ bool ex_less(
    const uint64_t* d, uint32_t a, uint32_t b) {
  return d[a] < d[b] || (d[a] == d[b] && a < b);
}

__device__ void ex_sift_up(
    uint32_t* heap, uint32_t* pos, const uint64_t* d, uint32_t i) {
  const uint32_t x = heap[i];
  while (i > 0) {
    const uint32_t p = (i - 1) >> 1;
    if (!ex_less(d, x, heap[p])) {
      break;
    }
    heap[i] = heap[p];
    pos[heap[i]] = i;
    i = p;
  }
  heap[i] = x;
  pos[x] = i;
}

__device__ void ex_sift_down(
    uint32_t* heap, uint32_t* pos, const uint64_t* d, uint32_t n, uint32_t i) {
  const uint32_t x = heap[i];
  for (;;) {
    uint32_t c = 2 * i + 1;
    if (c >= n) {
      break;
    }
    if (c + 1 < n && ex_less(d, heap[c + 1], heap[c])) {
      ++c;
    }
    if (!ex_less(d, heap[c], x)) {
      break;
    }
    heap[i] = heap[c];
    pos[heap[i]] = i;
    i = c;
  }
  heap[i] = x;
  pos[x] = i;
}

// One thread per query: the literal DijkstraQ replay (LinkState.cpp:816-873).
__global__ __launch_bounds__(64) void spf_exact_kernel(ExactArgs a) {
  const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= a.nq) {
    return;
  }
  const uint32_t V = a.V;
  const uint32_t src = a.src[q];
  uint64_t* d = a.dist_out + (size_t)q * V;
  uint32_t* order = a.order_out + (size_t)q * V;
  uint32_t* pos = a.scratch + (size_t)q * 2 * V;
  uint32_t* heap = pos + V;
  const uint32_t Wm = a.want_nh ? a.nh_w[q] : 0;
  uint64_t* nhrow = a.want_nh ? a.nh_out + a.nh_off[q] : nullptr;
  const uint32_t ilo = a.ign_off ? a.ign_off[q] : 0;
  const uint32_t nign = a.ign_off ? a.ign_off[q + 1] - ilo : 0;
  const uint32_t* ignp = a.ign ? a.ign + ilo : nullptr;

  for (uint32_t v = 0; v < V; ++v) {
    pos[v] = kNotSeen;
    order[v] = kInf32;
    d[v] = SPF_UNREACHABLE;
  }
  uint32_t n = 0, settled = 0;
  d[src] = 0;
  heap[n++] = src;
  pos[src] = 0;
  while (n) {
    const uint32_t u = heap[0];
    --n;
    if (n) {
      heap[0] = heap[n];
      pos[heap[0]] = 0;
      ex_sift_down(heap, pos, d, n, 0);
    }
    pos[u] = kSettled;
    order[u] = settled++;
    if (u != src && !((a.trbits[u >> 5] >> (u & 31)) & 1u)) {
      continue;
    }
    const uint64_t du = d[u];
    for (uint32_t e = a.row[u]; e < a.row[u + 1]; ++e) {
      const uint32_t v = a.col[e];
      if (pos[v] == kSettled) {
        continue;
      }
      if (nign && in_sorted(ignp, nign, a.link[e])) {
        continue;
      }
      const uint64_t c = du + (a.unit ? 1ull : a.w64[e]);
      if (pos[v] == kNotSeen) {
        d[v] = c;
        heap[n] = v;
        pos[v] = n;
        ex_sift_up(heap, pos, d, n);
        ++n;
      }
      if (d[v] >= c) {
        if (d[v] > c) {
          d[v] = c;
          for (uint32_t j = 0; j < Wm; ++j) {
            nhrow[(size_t)v * Wm + j] = 0;
          }
          ex_sift_up(heap, pos, d, pos[v]);
        }
        if (Wm) {
          uint64_t any = 0;
          for (uint32_t j = 0; j < Wm; ++j) {
            uint64_t m = (u == src) ? 0ull : nhrow[(size_t)u * Wm + j];
            m |= nhrow[(size_t)v * Wm + j];
            nhrow[(size_t)v * Wm + j] = m;
            any |= m;
          }
          if (!any && u == src) {
            const uint32_t s = a.slot[e];
            nhrow[(size_t)v * Wm + (s >> 6)] |= 1ull << (s & 63);
          }
        }
      }
    }
  }
}

// -------------------------------------------------------------- wide kernel
//
// 64-bit distances for the metric graphs the 32-bit plans cannot take
// (metric-0 links, or sums that may pass 2^32), one 1024-thread workgroup per
// query, in parallel where the literal replay above is one thread:
//  1. distances: near-far label-correcting SSSP over the u64 HBM row
//     (pending bitmap in LDS, atomicMin on the row, the band [.., T) advances
//     to the smallest pending distance + delta).  Any processing order
//     reaches the unique fixpoint for non-negative metrics;
//  2. settle keys: DijkstraQ extracts DISCOVERED nodes by (metric, name)
//     (LinkState.h:483-535), so only plateaus of equal distance joined by
//     usable metric-0 edges depart from (distance, id) order.  The plateau
//     nodes that take part -- tails of such edges reached from below ("active
//     seeds") and nodes reached only over metric-0 edges -- are replayed by
//     one lane with a heap keyed (distance, id).  Passive nodes keep key
//     id<<32; a replayed node gets (M<<32)|2^31|j, M the largest id replayed
//     so far on its plateau, j its replay index.  A passive node p is
//     extracted before a replayed node x iff p < M(x) (every passive of the
//     plateau is in the heap from the start and never discovers anything), so
//     (distance, key) order IS the reference's settle order;
//  3. next hops: NH(v) = union over usable tight in-edges u->v with u settled
//     before v of (u == src ? bit(v) : NH(u)) (LinkState.cpp:846-867; the
//     source settles first, so its "directly connected" rule always fires),
//     propagated in Kahn rounds over that DAG: a count of outstanding
//     in-edges per node, 64-bit atomicOr of the masks.
// The literal replay stays only for graphs whose metrics wrap (negative i32
// metrics as uint64, where Dijkstra's order is not a fixpoint).

constexpr uint32_t kWideBlock = 1024;
constexpr uint32_t kWideG = 8; // lanes per node in the edge loops

struct WideArgs {
  const uint32_t* row;
  const uint32_t* col;
  const uint64_t* w64;
  const uint32_t* link;
  const uint32_t* rev;
  const uint32_t* slot;
  const uint32_t* trbits;
  const uint32_t* zero_e; // half-edges with metric 0
  const uint32_t* src;
  const uint32_t* ign_off;
  const uint32_t* ign;
  const uint64_t* nh_off;
  const uint32_t* nh_w;
  uint64_t* dist_out; // [nq][V]
  uint64_t* nh_out;
  uint64_t* key_out;  // [nq][V] settle keys, or null
  uint32_t* scratch;  // per workgroup: wide_stride(V, nbw) words
  uint64_t delta;
  uint32_t V, nq, nbw, n_zero, unit, want_nh;
};

// per-workgroup scratch: two queues, counts, heap [V] u32; keys [V] u64;
// active / discovered / replayed bitmaps [nbw]
__host__ __device__ inline size_t wide_stride(uint32_t V, uint32_t nbw) {
  return (6 * (size_t)V + 3 * (size_t)nbw + 3) & ~(size_t)3;
}

__device__ __forceinline__ uint64_t ld_coh64(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ bool wd_usable(const uint32_t* tr, uint32_t u, uint32_t s) {
  return u == s || ((tr[u >> 5] >> (u & 31)) & 1u);
}

__device__ __forceinline__ bool wd_bit(const uint32_t* b, uint32_t v) {
  return (ld_coh(b + (v >> 5)) >> (v & 31)) & 1u;
}

// x is discovered before its plateau starts: the source, or the head of a
// usable tight in-edge from a smaller distance
__device__ bool wd_seed(
    const WideArgs& a, const uint64_t* d, uint32_t x, uint32_t s,
    const uint32_t* ignp, uint32_t nign) {
  if (x == s) {
    return true;
  }
  const uint64_t dx = ld_coh64(d + x);
  for (uint32_t e = a.row[x]; e < a.row[x + 1]; ++e) {
    const uint32_t u = a.col[e];
    if (!wd_usable(a.trbits, u, s) || (nign && in_sorted(ignp, nign, a.link[e]))) {
      continue;
    }
    const uint64_t du = ld_coh64(d + u);
    if (du < dx && du + a.w64[a.rev[e]] == dx) {
      return true;
    }
  }
  return false;
}

// Workgroup barrier for lanes that talk through GLOBAL memory: a plain
// __syncthreads() only drains LDS traffic (s_waitcnt lgkmcnt), so stores and
// non-returning atomics of other waves may still be on their way to L2.
// Draining vmcnt first puts them in L2 (one XCD's L2 serves the whole
// workgroup, so no agent-scope L2 writeback is needed); readers of data other
// waves wrote use L1-bypassing loads (ld_coh / ld_coh64).
__device__ __forceinline__ void wide_sync() {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
}

__global__ __launch_bounds__(kWideBlock) void spf_wide_kernel(WideArgs a) {
  extern __shared__ uint32_t wlds[];
  uint32_t* pend = wlds; // [nbw]
  __shared__ uint32_t s_qlen;
  __shared__ unsigned long long s_min;
  constexpr uint32_t BS = kWideBlock;
  const uint32_t V = a.V, nbw = a.nbw, tid = threadIdx.x;
  const uint32_t gl = tid % kWideG, gi = tid / kWideG;
  uint32_t* ws = a.scratch + (size_t)blockIdx.x * wide_stride(V, nbw);
  uint32_t* qa = ws;
  uint32_t* qb = ws + V;
  uint32_t* cnt = ws + 2 * (size_t)V;
  uint32_t* heap = ws + 3 * (size_t)V;
  uint64_t* kx = (uint64_t*)(ws + 4 * (size_t)V);
  uint32_t* act = ws + 6 * (size_t)V;
  uint32_t* disc = act + nbw;
  uint32_t* mem = disc + nbw;
  const bool zplat = a.n_zero && !a.unit;

  for (uint32_t q = blockIdx.x; q < a.nq; q += gridDim.x) {
    const uint32_t s = a.src[q];
    uint64_t* d = a.dist_out + (size_t)q * V;
    const uint32_t ilo = a.ign_off ? a.ign_off[q] : 0;
    const uint32_t nign = a.ign_off ? a.ign_off[q + 1] - ilo : 0;
    const uint32_t* ignp = a.ign ? a.ign + ilo : nullptr;
    for (uint32_t v = tid; v < V; v += BS) {
      d[v] = SPF_UNREACHABLE;
    }
    for (uint32_t w = tid; w < nbw; w += BS) {
      pend[w] = 0;
      act[w] = 0;
      disc[w] = 0;
      mem[w] = 0;
    }
    wide_sync();
    if (tid == 0) {
      d[s] = 0;
      pend[s >> 5] = 1u << (s & 31);
    }
    wide_sync();

    // ---- 1. distances (near-far)
    uint64_t T = a.delta;
    for (;;) {
      if (tid == 0) {
        s_qlen = 0;
        s_min = SPF_UNREACHABLE;
      }
      wide_sync();
      uint64_t lmin = SPF_UNREACHABLE;
      for (uint32_t w = tid; w < nbw; w += BS) {
        uint32_t b = pend[w];
        if (!b) {
          continue;
        }
        uint32_t keep = 0;
        while (b) {
          const uint32_t k = __ffs(b) - 1;
          b &= b - 1;
          const uint32_t v = w * 32 + k;
          const uint64_t dv = ld_coh64(d + v);
          if (dv < T) {
            qa[atomicAdd(&s_qlen, 1u)] = v;
          } else {
            keep |= 1u << k;
            lmin = min(lmin, dv);
          }
        }
        pend[w] = keep;
      }
      for (int o = 32; o > 0; o >>= 1) {
        lmin = min(lmin, (uint64_t)__shfl_xor((unsigned long long)lmin, o, 64));
      }
      if ((tid & 63) == 0 && lmin != SPF_UNREACHABLE) {
        atomicMin(&s_min, (unsigned long long)lmin);
      }
      wide_sync();
      const uint32_t n = s_qlen;
      if (n == 0) {
        const uint64_t m = s_min;
        wide_sync();
        if (m == SPF_UNREACHABLE) {
          break;
        }
        T = m + a.delta;
        continue;
      }
      for (uint32_t i = gi; i < n; i += BS / kWideG) {
        const uint32_t u = ld_coh(qa + i);
        if (!wd_usable(a.trbits, u, s)) {
          continue;
        }
        const uint64_t du = ld_coh64(d + u);
        for (uint32_t e = a.row[u] + gl; e < a.row[u + 1]; e += kWideG) {
          if (nign && in_sorted(ignp, nign, a.link[e])) {
            continue;
          }
          const uint32_t v = a.col[e];
          const uint64_t c = du + (a.unit ? 1ull : a.w64[e]);
          if (c < ld_coh64(d + v)) {
            const uint64_t old =
                atomicMin((unsigned long long*)(d + v), (unsigned long long)c);
            if (c < old) {
              atomicOr(&pend[v >> 5], 1u << (v & 31));
            }
          }
        }
      }
      wide_sync();
    }

    // ---- 2. settle keys of metric-0 plateaus
    if (zplat) {
      for (uint32_t i = tid; i < a.n_zero; i += BS) {
        const uint32_t e = a.zero_e[i];
        const uint32_t u = a.col[a.rev[e]], v = a.col[e];
        if (!wd_usable(a.trbits, u, s) || (nign && in_sorted(ignp, nign, a.link[e]))) {
          continue;
        }
        const uint64_t du = ld_coh64(d + u);
        if (du != SPF_UNREACHABLE && du == ld_coh64(d + v)) {
          atomicOr(&act[u >> 5], 1u << (u & 31));
        }
      }
      if (tid == 0) {
        s_qlen = 0;
      }
      wide_sync();
      for (uint32_t w = tid; w < nbw; w += BS) {
        uint32_t b = ld_coh(act + w);
        while (b) {
          const uint32_t x = w * 32 + (__ffs(b) - 1);
          b &= b - 1;
          if (wd_seed(a, d, x, s, ignp, nign)) {
            heap[atomicAdd(&s_qlen, 1u)] = x;
            atomicOr(&disc[x >> 5], 1u << (x & 31));
          }
        }
      }
      wide_sync();
      if (tid == 0) {
        // other lanes wrote the heap: drop stale L1 lines first
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        uint32_t n = s_qlen;
        auto before = [&](uint32_t x, uint32_t y) {
          const uint64_t dx = ld_coh64(d + x), dy = ld_coh64(d + y);
          return dx < dy || (dx == dy && x < y);
        };
        auto sift_down = [&](uint32_t i) {
          const uint32_t x = heap[i];
          for (;;) {
            uint32_t c = 2 * i + 1;
            if (c >= n) {
              break;
            }
            if (c + 1 < n && before(heap[c + 1], heap[c])) {
              ++c;
            }
            if (!before(heap[c], x)) {
              break;
            }
            heap[i] = heap[c];
            i = c;
          }
          heap[i] = x;
        };
        for (uint32_t i = n / 2; i-- > 0;) {
          sift_down(i);
        }
        uint64_t curD = SPF_UNREACHABLE;
        uint32_t M = 0, j = 0;
        while (n) {
          const uint32_t x = heap[0];
          if (--n) {
            heap[0] = heap[n];
            sift_down(0);
          }
          const uint64_t dx = ld_coh64(d + x);
          if (dx != curD) {
            curD = dx;
            M = 0;
          }
          M = max(M, x);
          kx[x] = ((uint64_t)M << 32) | 0x80000000ull | j++;
          atomicOr(&mem[x >> 5], 1u << (x & 31));
          if (!wd_usable(a.trbits, x, s)) {
            continue;
          }
          for (uint32_t e = a.row[x]; e < a.row[x + 1]; ++e) {
            if (a.w64[e] != 0 || (nign && in_sorted(ignp, nign, a.link[e]))) {
              continue;
            }
            const uint32_t y = a.col[e];
            if (ld_coh64(d + y) != dx || wd_bit(disc, y)) {
              continue;
            }
            atomicOr(&disc[y >> 5], 1u << (y & 31));
            if (wd_seed(a, d, y, s, ignp, nign)) {
              continue; // a passive seed: already in the plateau's heap
            }
            uint32_t i = n++;
            while (i > 0) { // sift up
              const uint32_t p = (i - 1) >> 1;
              if (!before(y, heap[p])) {
                break;
              }
              heap[i] = heap[p];
              i = p;
            }
            heap[i] = y;
          }
        }
      }
      wide_sync();
    }
    auto key = [&](uint32_t v) -> uint64_t {
      return (zplat && wd_bit(mem, v)) ? ld_coh64(kx + v) : ((uint64_t)v << 32);
    };

    // ---- 3. next hops (Kahn rounds over the settle-ordered tight DAG)
    if (a.want_nh) {
      const uint32_t W = a.nh_w[q];
      uint64_t* nh = a.nh_out + a.nh_off[q];
      for (uint32_t v = tid; v < V; v += BS) {
        const uint64_t dv = ld_coh64(d + v);
        uint32_t c = 0;
        if (dv != SPF_UNREACHABLE && v != s) {
          for (uint32_t e = a.row[v]; e < a.row[v + 1]; ++e) {
            const uint32_t u = a.col[e];
            if (!wd_usable(a.trbits, u, s) || (nign && in_sorted(ignp, nign, a.link[e]))) {
              continue;
            }
            const uint64_t du = ld_coh64(d + u);
            const uint64_t wu = a.unit ? 1ull : a.w64[a.rev[e]];
            if (du == SPF_UNREACHABLE || du + wu != dv) {
              continue;
            }
            if (wu == 0 && !(key(u) < key(v))) {
              continue;
            }
            ++c;
          }
        }
        cnt[v] = c;
      }
      if (tid == 0) {
        qa[0] = s;
      }
      wide_sync();
      uint32_t n = 1;
      uint32_t *cur = qa, *nxt = qb;
      while (n) {
        if (tid == 0) {
          s_qlen = 0;
        }
        wide_sync();
        for (uint32_t i = gi; i < n; i += BS / kWideG) {
          const uint32_t u = ld_coh(cur + i);
          if (!wd_usable(a.trbits, u, s)) {
            continue;
          }
          const uint64_t du = ld_coh64(d + u);
          const uint64_t ku = key(u);
          for (uint32_t e = a.row[u] + gl; e < a.row[u + 1]; e += kWideG) {
            const uint32_t v = a.col[e];
            if (v == s || (nign && in_sorted(ignp, nign, a.link[e]))) {
              continue;
            }
            const uint64_t w = a.unit ? 1ull : a.w64[e];
            const uint64_t dv = ld_coh64(d + v);
            if (dv == SPF_UNREACHABLE || du + w != dv || (w == 0 && !(ku < key(v)))) {
              continue;
            }
            if (u == s) {
              const uint32_t sl = a.slot[e];
              atomicOr((unsigned long long*)(nh + (size_t)v * W + (sl >> 6)),
                       1ull << (sl & 63));
            } else {
              for (uint32_t k = 0; k < W; ++k) {
                const uint64_t m = ld_coh64(nh + (size_t)u * W + k);
                if (m) {
                  atomicOr((unsigned long long*)(nh + (size_t)v * W + k),
                           (unsigned long long)m);
                }
              }
            }
            if (atomicSub(cnt + v, 1u) == 1u) {
              nxt[atomicAdd(&s_qlen, 1u)] = v;
            }
          }
        }
        wide_sync();
        n = s_qlen;
        uint32_t* t = cur;
        cur = nxt;
        nxt = t;
        wide_sync();
      }
    }

    // ---- 4. settle keys out (SPF_F_ORDER)
    if (a.key_out) {
      uint64_t* ko = a.key_out + (size_t)q * V;
      for (uint32_t v = tid; v < V; v += BS) {
        ko[v] = ld_coh64(d + v) == SPF_UNREACHABLE ? SPF_UNREACHABLE : key(v);
      }
    }
    wide_sync();
  }
}

// ------------------------------------------------ what-if screen (config 5)
//
// Removing a link changes an SPF only if one of its half-edges u->v is a
// USABLE TIGHT edge of the baseline run from the same source: u the source
// or transit, d[u] + w(u->v) == d[v].  Distances and next-hop sets are
// defined by those edges alone, so a query none of whose
// ignored links is tight has exactly the baseline rows.  One block per
// query checks its list against the baseline row and, if nothing is tight,
// copies the baseline distance / next-hop rows and flags the query so the
// SSSP kernel skips it.  Single-link failures off the source's shortest-path
// DAG (most of them) then cost a row copy instead of an SSSP.
struct WhatifArgs {
  const uint32_t* col;
  const uint32_t* rev;
  const uint32_t* wout;
  const uint32_t* trbits;
  const uint32_t* link_half; // [2 * L] half-edges of each link (~0u = none)
  const uint32_t* src;
  const uint32_t* ign_off;
  const uint32_t* ign;
  const uint32_t* base_of;   // query -> baseline row
  const uint32_t* base_dist; // [nb][Vp]
  const uint64_t* base_nh;
  const uint64_t* base_nh_off;
  uint32_t* dist_out;
  uint64_t* nh_out;
  const uint64_t* nh_off;
  const uint32_t* nh_w;
  uint32_t* skip;
  uint32_t V;
  uint32_t Vp;
  uint32_t L; // link ids >= L match no edge (ignored)
  uint32_t want_nh;
  uint32_t unit; // SPF_F_UNIT_METRIC: every hop costs 1
  // repair batches: a tight ignored link of the source itself is flagged
  // skip = 2 (spf_sssp_kernel claims those first), or 3 when the query is
  // one of spf_whatif_heavy_kernel's (wh_mark[q] != 0: it runs them)
  uint32_t mark_heavy;
  const uint8_t* wh_mark = nullptr;
  // narrow rows (spf_query::narrow): a screened query's masks go straight to
  // the output layout (the baseline word row narrowed on the copy), and the
  // narrowing pass skips it; nullptr: word rows, narrowed later
  uint8_t* nhb = nullptr;
  const uint64_t* nhb_off = nullptr;
  const uint32_t* nh_b = nullptr;
};

__global__ __launch_bounds__(256) void spf_whatif_screen_kernel(WhatifArgs a) {
  const uint32_t q = blockIdx.x;
  const uint32_t s = a.src[q], b = a.base_of[q];
  const uint32_t* bd = a.base_dist + (size_t)b * a.Vp;
  const uint32_t lo = a.ign_off[q], n = a.ign_off[q + 1] - lo;
  int tight = 0, heavy = 0;
  for (uint32_t i = threadIdx.x; i < 2 * n; i += blockDim.x) {
    const uint32_t l = a.ign[lo + (i >> 1)];
    const uint32_t e = l < a.L ? a.link_half[2 * (size_t)l + (i & 1)] : kInf32;
    if (e == kInf32) {
      continue;
    }
    const uint32_t u = a.col[a.rev[e]], v = a.col[e];
    const uint32_t du = bd[u];
    if (du == kInf32 || (u != s && !((a.trbits[u >> 5] >> (u & 31)) & 1u))) {
      continue;
    }
    const bool t = du + (a.unit ? 1u : a.wout[e]) == bd[v];
    tight |= t;
    heavy |= t && u == s;
  }
  tight = __syncthreads_or(tight);
  heavy = __syncthreads_or(heavy);
  if (threadIdx.x == 0) {
    a.skip[q] = tight ? (heavy && a.mark_heavy ? (a.wh_mark && a.wh_mark[q] ? 3u : 2u) : 0u)
                      : 1u;
  }
  if (tight) {
    return;
  }
  block_copy<uint32_t, 256>(a.dist_out + (size_t)q * a.Vp, bd, a.V);
  if (a.want_nh) {
    const uint64_t* src = a.base_nh + a.base_nh_off[b];
    const uint32_t W = a.nh_w[q];
    if (!a.nhb) {
      block_copy<uint64_t, 256>(a.nh_out + a.nh_off[q], src, (size_t)a.V * W);
      return;
    }
    uint8_t* d = a.nhb + a.nhb_off[q];
    const uint32_t B = a.nh_b[q];
    if (B >= 8) {
      // B = 8 W: the output layout is the word layout
      block_copy<uint64_t, 256>(reinterpret_cast<uint64_t*>(d), src, (size_t)a.V * W);
      return;
    }
    for (uint32_t v0 = 4 * threadIdx.x; v0 < a.V; v0 += 4 * blockDim.x) {
      uint64_t x[4];
#pragma unroll
      for (uint32_t i = 0; i < 4; ++i) {
        x[i] = v0 + i < a.V ? src[v0 + i] : 0ull; // B < 8: one word per node
      }
      nh_store4_narrow(d, B, v0, a.V, x);
    }
  }
}

// What-if queries whose failed link leaves the source (the screen's skip ==
// 2) on a uniform-metric area: their repair set K is most of the graph, so
// spf_sssp_kernel ran them from scratch on one 512-thread workgroup each, and
// the fabric batch waited ~1.7 ms for the two of them (profiles/r05ah,
// r05al).  Here one 1,024-thread workgroup per such query runs a
// level-synchronous BFS (transit rule, ignored links skipped; the queue is in
// BFS order, so levels are its segments), then the next-hop masks level by
// level over the tight in-edges: nh(v) = OR over u -> v with lvl(u) + 1 =
// lvl(v), u the source or transit, link not ignored, of (u == s ? the bit of
// v's slot in s's neighbour list : nh(u)).  Distances = level x the uniform
// metric.  The screen marks these queries skip = 3, which spf_sssp_kernel
// never claims, and this kernel runs on its own stream beside it.
struct WhatifHeavyArgs {
  const uint32_t* row;
  const uint32_t* col;
  const uint32_t* link;
  const uint32_t* rev;
  const uint32_t* slot;
  const uint32_t* trbits;
  const uint32_t* src;
  const uint32_t* ign_off;
  const uint32_t* ign;
  const uint32_t* cand; // candidate queries (an ignored link at their source)
  uint32_t* skip;
  uint32_t* dist_out;
  uint64_t* nh_out;
  const uint64_t* nh_off;
  const uint32_t* nh_w;
  uint32_t V, Vp, scale;
  uint32_t want_nh; // distance-only batches have no mask rows
  uint32_t* lstart; // [ncand][V + 1] level segments of each candidate's queue
  // OPENR_SPF_WHATIF_STATS=1: per candidate {init, BFS, rows, masks ticks
  // (100 MHz), levels, reached}; nullptr = off
  unsigned long long* stats = nullptr;
  // the pull form (spf_whatif_pull_kernel): the sliced-ELL copy and the
  // links' half-edges
  const uint4* sell4 = nullptr;
  const uint32_t* sell_off = nullptr;
  const uint32_t* link_half = nullptr;
  uint32_t L = 0;
};
constexpr uint32_t kWhThreads = 1024;
constexpr uint32_t kWhIgn = 512; // ignore-list hash slots in LDS
constexpr uint32_t kWhMaxW = 4; // mask words per node handled here

__global__ __launch_bounds__(kWhThreads) void spf_whatif_heavy_kernel(WhatifHeavyArgs a) {
  extern __shared__ __align__(16) uint32_t wh_smem[];
  uint32_t* lvl = wh_smem;         // [V] BFS level, kInf32 = unreached
  uint32_t* queue = lvl + a.V;     // [V] nodes in BFS order
  uint32_t* rowl = queue + a.V;    // [V + 1] the CSR row offsets
  uint32_t* trl = rowl + a.V + 1;  // [V / 32] transit bits
  // level segments of the queue (global: up to V + 1 of them)
  uint32_t* lstart = a.lstart + (size_t)blockIdx.x * (a.V + 1);
  __shared__ uint32_t ign_s[kWhIgn];
  __shared__ uint32_t sh_qb, sh_qe;
  __shared__ uint32_t sh_tail;
  const uint32_t tid = threadIdx.x;
  const uint32_t q = a.cand[blockIdx.x];
  if (a.skip[q] != 3u) {
    return; // screened (rows copied) or repairable: not this kernel's
  }
  unsigned long long tk[5] = {a.stats ? wall_clock64() : 0ull, 0, 0, 0, 0};
  const uint32_t s = a.src[q], V = a.V;
  const uint32_t ilo = a.ign_off[q], nign = a.ign_off[q + 1] - ilo;
  IgnSet ig;
  ig.p = a.ign + ilo;
  ig.n = nign;
  const uint32_t slots = ign_hash_slots(nign);
  if (slots && slots <= kWhIgn) {
    for (uint32_t i = tid; i < slots; i += kWhThreads) {
      ign_s[i] = kInf32;
    }
    __syncthreads();
    const uint32_t hb = __builtin_ctz(slots);
    for (uint32_t i = tid; i < nign; i += kWhThreads) {
      const uint32_t l = a.ign[ilo + i];
      uint32_t h = (l * 0x9E3779B1u) >> (32 - hb);
      for (;;) {
        const uint32_t prev = atomicCAS(&ign_s[h], kInf32, l);
        if (prev == kInf32 || prev == l) {
          break;
        }
        h = (h + 1) & (slots - 1);
      }
    }
    ig.p = ign_s;
    ig.hbits = hb;
  } else if (nign <= kWhIgn) {
    // a short list stays sorted, in LDS (probing it in global memory cost a
    // dependent round trip per edge: ~3 us per frontier node, r05an)
    for (uint32_t i = tid; i < nign; i += kWhThreads) {
      ign_s[i] = a.ign[ilo + i];
    }
    __syncthreads();
    ig.p = ign_s;
  }
  for (uint32_t v = tid; v < V; v += kWhThreads) {
    lvl[v] = v == s ? 0u : kInf32;
    rowl[v] = a.row[v];
  }
  for (uint32_t i = tid; i < (V + 31) / 32; i += kWhThreads) {
    trl[i] = a.trbits[i];
  }
  if (tid == 0) {
    rowl[V] = a.row[V];
    queue[0] = s;
    sh_tail = 1;
    lstart[0] = 0;
    lstart[1] = 1;
    sh_qb = 0;
    sh_qe = 1;
  }
  __syncthreads();
  if (a.stats) {
    tk[1] = wall_clock64();
  }
  auto transit = [&](uint32_t u) { return u == s || ((trl[u >> 5] >> (u & 31)) & 1u); };
  // BFS, level by level: frontier = queue[lstart[L], lstart[L + 1])
  uint32_t L = 0;
  for (;;) {
    const uint32_t qb = sh_qb, qe = sh_qe;
    if (qb == qe) {
      break; // (at most V levels: lstart has V + 1 slots)
    }
    // 8 lanes per frontier node (128 nodes in flight), lanes over its out-edges
    const uint32_t gl = tid & 7u, grp = tid >> 3;
    for (uint32_t i = qb + grp; i < qe; i += kWhThreads / 8) {
      const uint32_t u = queue[i];
      if (!transit(u)) {
        continue; // reached, not expanded (LinkState.cpp:829-836)
      }
      for (uint32_t e = rowl[u] + gl; e < rowl[u + 1]; e += 8) {
        if (nign && ig.has(a.link[e])) {
          continue;
        }
        const uint32_t v = a.col[e];
        if (atomicCAS(&lvl[v], kInf32, L + 1) == kInf32) {
          queue[atomicAdd(&sh_tail, 1u)] = v;
        }
      }
    }
    __syncthreads();
    if (tid == 0) {
      lstart[L + 2] = sh_tail;
      sh_qb = qe;
      sh_qe = sh_tail;
    }
    __syncthreads();
    ++L;
  }
  __syncthreads();
  if (a.stats) {
    tk[2] = wall_clock64();
  }
  const uint32_t nlev = L; // levels 0 .. nlev - 1 hold nodes
  uint32_t* dist = a.dist_out + (size_t)q * a.Vp;
  const uint32_t W = a.want_nh ? a.nh_w[q] : 0u;
  uint64_t* nh = a.want_nh ? a.nh_out + a.nh_off[q] : nullptr;
  for (uint32_t v = tid; v < V; v += kWhThreads) {
    const uint32_t l = lvl[v];
    dist[v] = l == kInf32 ? kInf32 : l * a.scale;
    if (l == kInf32 || v == s) {
      for (uint32_t k = 0; k < W; ++k) {
        nh[(size_t)v * W + k] = 0ull; // unreached (and the source): empty
      }
    }
  }
  __syncthreads();
  if (a.stats) {
    tk[3] = wall_clock64();
  }
  // next hops, level by level (level L reads level L - 1's masks: written
  // by this workgroup before the barrier)
  // 8 lanes per node, lanes over its in-edges, OR-reduced in the group
  const uint32_t gl = tid & 7u, grp = tid >> 3;
  for (uint32_t l = 1; W && l < nlev; ++l) {
    const uint32_t i1 = lstart[l + 1];
    for (uint32_t i0 = lstart[l]; i0 < i1; i0 += kWhThreads / 8) {
      const uint32_t i = i0 + grp; // the loop is uniform: the shuffles below
      const uint32_t v = i < i1 ? queue[i] : 0u;
      uint64_t acc[kWhMaxW] = {0, 0, 0, 0};
      if (i < i1) {
        for (uint32_t e = rowl[v] + gl; e < rowl[v + 1]; e += 8) {
          const uint32_t u = a.col[e]; // e = v -> u; its reverse u -> v is the in-edge
          if (lvl[u] + 1 != l || !transit(u) || (nign && ig.has(a.link[e]))) {
            continue;
          }
          if (u == s) {
            const uint32_t b = a.slot[a.rev[e]]; // v's slot among s's neighbours
            acc[b >> 6] |= 1ull << (b & 63);
          } else {
#pragma unroll
            for (uint32_t k = 0; k < kWhMaxW; ++k) {
              if (k < W) {
                acc[k] |= nh[(size_t)u * W + k];
              }
            }
          }
        }
      }
#pragma unroll
      for (uint32_t k = 0; k < kWhMaxW; ++k) {
#pragma unroll
        for (int off = 4; off >= 1; off >>= 1) {
          acc[k] |= (uint64_t)__shfl_xor((unsigned long long)acc[k], off, 8);
        }
      }
      if (i < i1 && gl < W) {
        uint64_t w = acc[0];
#pragma unroll
        for (uint32_t k = 1; k < kWhMaxW; ++k) {
          w = gl == k ? acc[k] : w;
        }
        nh[(size_t)v * W + gl] = w;
      }
    }
    __syncthreads();
  }
  if (a.stats && tid == 0) {
    unsigned long long* o = a.stats + 6 * (size_t)blockIdx.x;
    o[0] = tk[1] - tk[0];
    o[1] = tk[2] - tk[1];
    o[2] = tk[3] - tk[2];
    o[3] = wall_clock64() - tk[3];
    o[4] = nlev;
    o[5] = sh_tail;
  }
}

// The same queries in pull form (spf_whatif_pull_kernel, the default where
// the graph has its sliced-ELL copy and a query ignores at most kWpIgnE / 2
// links).  The queue form's levels cost ~50 us each: a group walks its
// frontier nodes one after another, each a chain of dependent loads
// (profiles/r05an).  Here thread t owns nodes t, t + 1,024, ... (a wave =
// one 64-node slice of the sliced ELL, read 1 KB per load), and every level
// each unreached node pulls over its row: reached at L + 1 iff some
// neighbour u has lvl(u) = L, is the source or transit, and the half-edge's
// link is not ignored (uniform metric: the row's out-neighbours are its
// in-neighbours, each link has both halves).  The masks come the same way,
// level by level.  The ignored links are their half-edge indices in LDS
// (edge j of v's slice row is CSR edge row[v] + j).
constexpr uint32_t kWpIgnE = 32;

__global__ __launch_bounds__(kWhThreads) void spf_whatif_pull_kernel(WhatifHeavyArgs a) {
  extern __shared__ __align__(16) uint32_t wp_smem[];
  uint32_t* lvl = wp_smem;        // [V] BFS level, kInf32 = unreached
  uint32_t* trl = lvl + a.V;      // [V / 32] transit bits
  __shared__ uint32_t ige[kWpIgnE];
  __shared__ uint32_t sh_nie;
  const uint32_t tid = threadIdx.x, lane = tid & 63u;
  const uint32_t q = a.cand[blockIdx.x];
  if (a.skip[q] != 3u) {
    return; // screened (rows copied) or repairable: not this kernel's
  }
  unsigned long long tk[4] = {a.stats ? wall_clock64() : 0ull, 0, 0, 0};
  const uint32_t s = a.src[q], V = a.V;
  const uint32_t ilo = a.ign_off[q], nign = a.ign_off[q + 1] - ilo;
  if (tid == 0) {
    uint32_t n = 0;
    for (uint32_t i = 0; i < nign; ++i) {
      const uint32_t l = a.ign[ilo + i];
      for (uint32_t side = 0; l < a.L && side < 2; ++side) {
        const uint32_t e = a.link_half[2 * (size_t)l + side];
        if (e != kInf32 && n < kWpIgnE) {
          ige[n++] = e;
        }
      }
    }
    sh_nie = n;
  }
  for (uint32_t v = tid; v < V; v += kWhThreads) {
    lvl[v] = v == s ? 0u : kInf32;
  }
  for (uint32_t i = tid; i < (V + 31) / 32; i += kWhThreads) {
    trl[i] = a.trbits[i];
  }
  __syncthreads();
  const uint32_t nie = sh_nie;
  auto transit = [&](uint32_t u) { return u == s || ((trl[u >> 5] >> (u & 31)) & 1u); };
  auto ignored = [&](uint32_t e) {
    for (uint32_t i = 0; i < nie; ++i) {
      if (ige[i] == e) {
        return true;
      }
    }
    return false;
  };
  const uint32_t K = (V + kWhThreads - 1) / kWhThreads;
  // the BFS: level L + 1 = unreached nodes with a usable neighbour at L
  uint32_t L = 0;
  for (;; ++L) {
    bool any = false;
    for (uint32_t k = 0; k < K; ++k) {
      const uint32_t v = tid + k * kWhThreads;
      // a wave's 64 nodes are one slice: its bounds are wave-uniform
      const uint32_t c = __builtin_amdgcn_readfirstlane(v >> 6);
      if ((c << 6) >= V) {
        continue; // uniform: the whole wave is past the last node
      }
      if (v >= V || lvl[v] != kInf32) {
        continue;
      }
      const uint32_t g0 = a.sell_off[c], g1 = a.sell_off[c + 1];
      const uint32_t r0 = a.row[v], deg = a.row[v + 1] - r0;
      const uint4* p = a.sell4 + (size_t)g0 * 64 + lane;
      bool found = false;
      for (uint32_t gi = 0; gi < g1 - g0 && !found; ++gi) {
        const uint4 w = p[(size_t)gi * 64];
        const uint32_t us[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
        for (uint32_t t = 0; t < 4; ++t) {
          const uint32_t j = gi * 4 + t, u = us[t];
          if (j < deg && lvl[u] == L && transit(u) && !ignored(r0 + j)) {
            found = true;
          }
        }
      }
      if (found) {
        lvl[v] = L + 1;
        any = true;
      }
    }
    if (!__syncthreads_or(any)) {
      break;
    }
  }
  const uint32_t nlev = L + 1; // levels 0 .. L hold nodes
  if (a.stats) {
    tk[1] = wall_clock64();
  }
  uint32_t* dist = a.dist_out + (size_t)q * a.Vp;
  const uint32_t W = a.want_nh ? a.nh_w[q] : 0u;
  uint64_t* nh = a.want_nh ? a.nh_out + a.nh_off[q] : nullptr;
  for (uint32_t v = tid; v < V; v += kWhThreads) {
    const uint32_t l = lvl[v];
    dist[v] = l == kInf32 ? kInf32 : l * a.scale;
    if (l == kInf32 || v == s) {
      for (uint32_t w = 0; w < W; ++w) {
        nh[(size_t)v * W + w] = 0ull; // unreached (and the source): empty
      }
    }
  }
  __syncthreads();
  if (a.stats) {
    tk[2] = wall_clock64();
  }
  // next hops, level by level (level l reads level l - 1's masks, written by
  // this workgroup before the barrier)
  for (uint32_t l = 1; W && l < nlev; ++l) {
    for (uint32_t k = 0; k < K; ++k) {
      const uint32_t v = tid + k * kWhThreads;
      const uint32_t c = __builtin_amdgcn_readfirstlane(v >> 6);
      if ((c << 6) >= V) {
        continue;
      }
      if (v >= V || lvl[v] != l) {
        continue;
      }
      const uint32_t g0 = a.sell_off[c], g1 = a.sell_off[c + 1];
      const uint32_t r0 = a.row[v], deg = a.row[v + 1] - r0;
      const uint4* p = a.sell4 + (size_t)g0 * 64 + lane;
      uint64_t acc[kWhMaxW] = {0, 0, 0, 0};
      for (uint32_t gi = 0; gi < g1 - g0; ++gi) {
        const uint4 w = p[(size_t)gi * 64];
        const uint32_t us[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
        for (uint32_t t = 0; t < 4; ++t) {
          const uint32_t j = gi * 4 + t, u = us[t];
          if (j >= deg || lvl[u] + 1 != l || !transit(u) || ignored(r0 + j)) {
            continue;
          }
          if (u == s) {
            const uint32_t b = a.slot[a.rev[r0 + j]]; // v's slot among s's neighbours
            acc[b >> 6] |= 1ull << (b & 63);
          } else {
#pragma unroll
            for (uint32_t x = 0; x < kWhMaxW; ++x) {
              if (x < W) {
                acc[x] |= nh[(size_t)u * W + x];
              }
            }
          }
        }
      }
#pragma unroll
      for (uint32_t x = 0; x < kWhMaxW; ++x) {
        if (x < W) {
          nh[(size_t)v * W + x] = acc[x];
        }
      }
    }
    __syncthreads();
  }
  if (a.stats && tid == 0) {
    unsigned long long* o = a.stats + 6 * (size_t)blockIdx.x;
    o[0] = 0;
    o[1] = tk[1] - tk[0];
    o[2] = tk[2] - tk[1];
    o[3] = wall_clock64() - tk[2];
    o[4] = nlev;
    o[5] = 0;
  }
}

// The repair SSSP's work list (round 6): the queries the screen left to it,
// heavy ones (skip 2, run from scratch) first, then the repairs (skip 0),
// compacted from the skip flags by one workgroup.  wl[0] = heavy count,
// wl[1] = total, wl[2 ..] = queries.
__global__ __launch_bounds__(1024) void spf_whatif_worklist_kernel(
    const uint32_t* skip, uint32_t nq, uint32_t* wl) {
  __shared__ uint32_t scan[32];
  uint32_t base = 0;
  for (uint32_t pass = 0; pass < 2; ++pass) {
    const uint32_t want = pass == 0 ? 2u : 0u;
    for (uint32_t b0 = 0; b0 < nq; b0 += 1024) {
      const uint32_t q = b0 + threadIdx.x;
      const uint32_t f = q < nq && skip[q] == want ? 1u : 0u;
      uint32_t total = 0;
      const uint32_t off = block_excl_scan<1024>(f, scan, &total);
      if (f) {
        wl[2 + base + off] = q;
      }
      base += total;
      __syncthreads(); // scan[] is rewritten by the next chunk
    }
    if (pass == 0 && threadIdx.x == 0) {
      wl[0] = base;
    }
  }
  if (threadIdx.x == 0) {
    wl[1] = base;
  }
}

// Source-link failures, first-hop form (round 6, spf_whatif_firsthop_kernel,
// OPENR_SPF_WHATIF_FIRSTHOP=0 keeps the pull kernel for them).  On a uniform
// metric a shortest path from s never returns to s, so for a query q that
// ignores links of s alone, every node v != s has
//   lvl_q(v) = 1 + min over usable first hops n of R_s[n][v],
// where R_s[n] is the BFS level from n with every link of s ignored, and v's
// next hops are the slots of the first hops reaching that minimum (a drained
// first hop n reaches only itself: R = 0 at v = n, unreached elsewhere).  The
// rows R_s of every such source's neighbours are ONE nested distance batch
// (q->hop: the bit-parallel BFS with ignore masks, all neighbours of s at
// once), computed per run; this kernel then combines them per (query, 256-node
// chunk) instead of one 1,024-thread workgroup running a whole BFS and a
// level-by-level mask pass per query (0.9 ms on the fabric, the what-if
// batch's longest chain).  Usable first hops are read at run time: a half-edge
// set down is a self-loop (spf_graph_set_edges), the transit bits are the
// graph's current ones, slots are d_slot's.
struct WhatifHopArgs {
  const uint32_t* row;
  const uint32_t* col;
  const uint32_t* link;
  const uint32_t* slot;
  const uint32_t* trbits;
  const uint32_t* src;
  const uint32_t* ign_off;
  const uint32_t* ign;
  const uint32_t* skip;
  const uint32_t* fh_q;      // [nfh] the queries
  const uint32_t* fh_h;      // [nfh] their hop source
  const uint32_t* hop_row0;  // [nhop] first row of the source's neighbours in the batch
  const uint32_t* hop_cnt;   // [nhop] neighbours (sorted ids at hop_nodes + hop_off)
  const uint32_t* hop_off;
  const uint32_t* hop_nodes;
  const uint32_t* rows;      // the nested batch's distance rows (levels)
  uint32_t rows_pitch;
  uint32_t* dist_out;
  uint64_t* nh_out;
  const uint64_t* nh_off;
  const uint32_t* nh_w;
  uint32_t V, Vp, scale, want_nh;
};
constexpr uint32_t kFhSlots = 64 * kWhMaxW; // the candidates' neighbour bound
constexpr uint32_t kFhChunk = 256;          // nodes per workgroup
constexpr uint32_t kFhGroup = 16;           // row loads in flight per thread

__global__ __launch_bounds__(256) void spf_whatif_firsthop_kernel(WhatifHopArgs a) {
  __shared__ int32_t sl_row[kFhSlots];  // -1 unusable, -2 drained (itself only)
  __shared__ uint32_t sl_node[kFhSlots];
  __shared__ uint32_t sh_nslot;
  const uint32_t i = blockIdx.x, q = a.fh_q[i];
  if (a.skip[q] != 3u) {
    return; // screened (rows copied): not this kernel's
  }
  const uint32_t h = a.fh_h[i], s = a.src[q], tid = threadIdx.x;
  for (uint32_t j = tid; j < kFhSlots; j += 256) {
    sl_row[j] = -1;
  }
  if (tid == 0) {
    sh_nslot = 0;
  }
  __syncthreads();
  const uint32_t e0 = a.row[s], e1 = a.row[s + 1];
  const uint32_t ilo = a.ign_off[q], nign = a.ign_off[q + 1] - ilo;
  for (uint32_t e = e0 + tid; e < e1; e += 256) {
    const uint32_t n = a.col[e];
    if (n == s) {
      continue; // a half-edge set down
    }
    const uint32_t l = a.link[e];
    bool ig = false;
    for (uint32_t k = 0; k < nign && !ig; ++k) {
      ig = a.ign[ilo + k] == l;
    }
    const uint32_t j = a.slot[e];
    if (!ig && j < kFhSlots) {
      sl_row[j] = 0; // usable (parallel links: the same value)
      sl_node[j] = n;
      atomicMax(&sh_nslot, j + 1);
    }
  }
  __syncthreads();
  const uint32_t nslot = sh_nslot;
  for (uint32_t j = tid; j < nslot; j += 256) {
    if (sl_row[j] < 0) {
      continue;
    }
    const uint32_t n = sl_node[j];
    const uint32_t* nodes = a.hop_nodes + a.hop_off[h];
    uint32_t lo = 0, hi = a.hop_cnt[h];
    while (lo < hi) {
      const uint32_t mid = (lo + hi) >> 1;
      if (nodes[mid] < n) {
        lo = mid + 1;
      } else {
        hi = mid;
      }
    }
    const bool transit = (a.trbits[n >> 5] >> (n & 31)) & 1u;
    // (every head of s's half-edges is in the batch: found by construction)
    sl_row[j] = transit ? (int32_t)(a.hop_row0[h] + lo) : -2;
  }
  __syncthreads();
  const uint32_t v = blockIdx.y * kFhChunk + tid;
  if (v >= a.V) {
    return;
  }
  uint32_t m = kInf32;
  uint64_t acc[kWhMaxW] = {0, 0, 0, 0};
  if (v != s) {
    for (uint32_t j0 = 0; j0 < nslot; j0 += kFhGroup) {
      uint32_t d[kFhGroup];
#pragma unroll
      for (uint32_t k = 0; k < kFhGroup; ++k) {
        const uint32_t j = j0 + k;
        const int32_t r = j < nslot ? sl_row[j] : -1;
        d[k] = r >= 0 ? a.rows[(size_t)r * a.rows_pitch + v]
                      : (r == -2 && sl_node[j] == v ? 0u : kInf32);
      }
#pragma unroll
      for (uint32_t k = 0; k < kFhGroup; ++k) {
        const uint32_t j = j0 + k;
        if (d[k] == kInf32) {
          continue;
        }
        const uint64_t bit = 1ull << (j & 63u);
        if (d[k] < m) {
          m = d[k];
#pragma unroll
          for (uint32_t x = 0; x < kWhMaxW; ++x) {
            acc[x] = x == (j >> 6) ? bit : 0ull;
          }
        } else if (d[k] == m) {
#pragma unroll
          for (uint32_t x = 0; x < kWhMaxW; ++x) {
            acc[x] |= x == (j >> 6) ? bit : 0ull;
          }
        }
      }
    }
  }
  a.dist_out[(size_t)q * a.Vp + v] = v == s ? 0u : (m == kInf32 ? kInf32 : (m + 1) * a.scale);
  if (a.want_nh) {
    const uint32_t W = a.nh_w[q];
    uint64_t* nh = a.nh_out + a.nh_off[q] + (size_t)v * W;
#pragma unroll
    for (uint32_t x = 0; x < kWhMaxW; ++x) {
      if (x < W) {
        nh[x] = acc[x];
      }
    }
  }
}

// Table repair screen (spf_table_screen): one lane per source row, every
// lane walks the same delta list (wave-uniform loads of the delta arrays).
// Reads two uint32 of the lane's row per in-scope delta and stops at the
// first hit; the rows are untouched.
struct ScreenArgs {
  const uint32_t* rows;
  size_t pitch;
  const uint32_t* src;
  const uint32_t* tail;
  const uint32_t* head;
  const uint64_t* metric;
  const uint32_t* kind; // SPF_DELTA_* | scope << 4
  uint32_t nrows;
  uint32_t ndelta;
  uint8_t* affected;
};

__global__ __launch_bounds__(256) void spf_table_screen_kernel(ScreenArgs a) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= a.nrows) {
    return;
  }
  const uint32_t s = a.src[i];
  const uint32_t* d = a.rows + (size_t)i * a.pitch;
  uint8_t hit = 0;
  for (uint32_t j = 0; j < a.ndelta && !hit; ++j) {
    const uint32_t u = a.tail[j], k = a.kind[j];
    const uint32_t scope = k >> 4;
    if ((scope == SPF_SCOPE_TAIL_ONLY && s != u) ||
        (scope == SPF_SCOPE_NOT_TAIL && s == u)) {
      continue;
    }
    const uint32_t du = d[u];
    if (du == kInf32) {
      continue;
    }
    const uint64_t c = (uint64_t)du + a.metric[j];
    const uint32_t dv = d[a.head[j]];
    const uint64_t dv64 = dv == kInf32 ? ~0ull : (uint64_t)dv;
    hit = (k & SPF_DELTA_REMOVED) ? (c == dv64) : (c <= dv64);
  }
  a.affected[i] = hit;
}

// Row scatter (spf_query_scatter_rows): workgroup (query, chunk) copies one
// 16-byte-vectorised slice of query row q into table row dst[q].
__global__ __launch_bounds__(256) void spf_scatter_rows_kernel(
    const uint32_t* __restrict__ from, uint32_t from_pitch,
    const uint32_t* __restrict__ dst_rows, char* __restrict__ table,
    size_t pitch, uint32_t V) {
  const uint32_t q = blockIdx.x;
  const uint32_t* src = from + (size_t)q * from_pitch;
  uint32_t* out = (uint32_t*)(table + (size_t)dst_rows[q] * pitch);
  const uint32_t chunk = blockDim.x * 4 * 4; // 4 x uint4 per lane
  const uint32_t lo = blockIdx.y * chunk;
  const uint32_t hi = min(V, lo + chunk);
  const bool vec = (reinterpret_cast<uintptr_t>(out) & 15) == 0 && (from_pitch & 3) == 0;
  if (vec) {
    const uint32_t n4 = (hi - lo) / 4;
    for (uint32_t t = threadIdx.x; t < n4; t += blockDim.x) {
      reinterpret_cast<uint4*>(out + lo)[t] = reinterpret_cast<const uint4*>(src + lo)[t];
    }
    for (uint32_t v = lo + n4 * 4 + threadIdx.x; v < hi; v += blockDim.x) {
      out[v] = src[v];
    }
  } else {
    for (uint32_t v = lo + threadIdx.x; v < hi; v += blockDim.x) {
      out[v] = src[v];
    }
  }
}

// All-nodes unicast route table (spf_route_table_run): for source row q
// (node s) and prefix p, the reference's Open/R ECMP route selection
// (SpfSolverImpl::selectEcmpOpenr, Decision.cpp:668-712, with
// getBestAnnouncingNodes :544-630, maybeFilterDrainedNodes :651-666,
// getNextHopsWithMetric :1093-1179 and getNextHopsThrift :1181-1271, one
// area, LFA off, not per destination):
//   no route if s announces p, or no announcer is reachable;
//   best  = smallest reachable announcer (bestPrefixEntry's node);
//   drop drained (overloaded) announcers unless all reachable ones are;
//   min   = min d(s, a) over the rest; NH = OR of the next-hop masks of s at
//           every announcer at distance min;
//   links = up links l of s to a neighbour in NH whose metric(l) + min -
//           d(s, nbr) == min, i.e. metric(l) == d(s, nbr) — bit j = the j-th
//           half-edge of s's CSR row (linksFromNode order).
// One workgroup per source row, one lane per prefix; the source's out-edges
// (neighbour, metric, slot) are staged in LDS.
constexpr uint32_t kRtStage = 1024;
constexpr uint32_t kRtMaskWords = 4; // register fast path: sources with <= 256 neighbours
struct RouteTableArgs {
  const uint32_t* row;
  const uint32_t* col;
  const uint32_t* wout;
  const uint32_t* slot;
  const uint32_t* trbits;
  const uint32_t* src;
  const uint32_t* dist; // query rows, stride Vp
  const uint8_t* nh;      // byte-strided mask rows (nh_bytes_for)
  const uint64_t* nh_off; // byte offset of each query's rows
  const uint32_t* nh_b;   // bytes per node
  const uint32_t* nh_w;
  const uint32_t* ann_off; // [P+1]
  const uint32_t* ann;
  const uint64_t* lk_off; // per query: first link-mask word
  uint32_t* metric_out; // [nq][P]
  uint32_t* best_out;   // [nq][P]
  uint64_t* link_out;
  // SPF_RT_LFA: query row of every node, per-link metrics [P][deg] per row
  const int32_t* row_of;
  const uint64_t* lm_off;
  uint32_t* lmet_out;
  uint32_t Vp, P, nq, lfa;
};

__global__ __launch_bounds__(256) void spf_route_table_kernel(RouteTableArgs a) {
  __shared__ uint32_t st_nbr[kRtStage];
  __shared__ uint32_t st_w[kRtStage];
  __shared__ uint32_t st_slot[kRtStage];
  __shared__ uint32_t st_slotall[kRtStage]; // LFA: slot of every link
  __shared__ uint32_t st_dns[kRtStage];     // LFA: d(nbr, s)
  for (uint32_t q = blockIdx.x; q < a.nq; q += gridDim.x) {
    const uint32_t s = a.src[q];
    const uint32_t* d = a.dist + (size_t)q * a.Vp;
    const uint8_t* nhq = a.nh + a.nh_off[q];
    const uint32_t W = a.nh_w[q], NB = a.nh_b[q];
    const uint32_t e0 = a.row[s], deg = a.row[s + 1] - e0;
    const uint32_t WL = (deg + 63) / 64;
    uint64_t* lk = a.link_out + a.lk_off[q];
    const bool staged = deg <= kRtStage;
    __syncthreads();
    if (staged) {
      for (uint32_t j = threadIdx.x; j < deg; j += blockDim.x) {
        const uint32_t nb = a.col[e0 + j];
        // a link is a shortest-path link iff metric(l) == d(s, nbr): keep
        // the slot only for those (others can never be selected)
        st_nbr[j] = nb;
        st_w[j] = a.wout[e0 + j];
        st_slot[j] = a.wout[e0 + j] == d[nb] ? a.slot[e0 + j] : kInf32;
        if (a.lfa) {
          st_slotall[j] = a.slot[e0 + j];
          st_dns[j] = a.dist[(size_t)a.row_of[nb] * a.Vp + s];
        }
      }
    }
    __syncthreads();
    for (uint32_t p = threadIdx.x; p < a.P; p += blockDim.x) {
      const uint32_t lo = a.ann_off[p], hi = a.ann_off[p + 1];
      bool self = false;
      uint32_t best = kInf32, reach = 0, undrained = 0;
      for (uint32_t i = lo; i < hi; ++i) {
        const uint32_t x = a.ann[i];
        self |= x == s;
        if (d[x] == kInf32) {
          continue;
        }
        best = min(best, x);
        ++reach;
        undrained += (a.trbits[x >> 5] >> (x & 31)) & 1u;
      }
      const size_t o = (size_t)q * a.P + p;
      uint64_t* lkp = lk + (size_t)p * WL;
      uint32_t* lm = a.lfa ? a.lmet_out + a.lm_off[q] + (size_t)p * deg : nullptr;
      if (self || reach == 0) {
        a.metric_out[o] = kInf32;
        a.best_out[o] = kInf32;
        for (uint32_t k = 0; k < WL; ++k) {
          lkp[k] = 0;
        }
        for (uint32_t j = 0; lm && j < deg; ++j) {
          lm[j] = kInf32;
        }
        continue;
      }
      const bool filt = undrained > 0;
      uint32_t mn = kInf32;
      for (uint32_t i = lo; i < hi; ++i) {
        const uint32_t x = a.ann[i];
        if (d[x] != kInf32 && (!filt || ((a.trbits[x >> 5] >> (x & 31)) & 1u))) {
          mn = min(mn, d[x]);
        }
      }
      a.metric_out[o] = mn;
      a.best_out[o] = best;
      if (staged && W <= kRtMaskWords) {
        // OR of the next-hop masks of the min-cost announcers (registers),
        // then slot -> link bits through the staged row (LDS broadcast)
        uint64_t m[kRtMaskWords];
#pragma unroll
        for (uint32_t k = 0; k < kRtMaskWords; ++k) {
          m[k] = 0;
        }
        for (uint32_t i = lo; i < hi; ++i) {
          const uint32_t x = a.ann[i];
          if (d[x] == mn && (!filt || ((a.trbits[x >> 5] >> (x & 31)) & 1u))) {
#pragma unroll
            for (uint32_t k = 0; k < kRtMaskWords; ++k) {
              if (k < W) {
                m[k] |= nh_load(nhq, NB, W, x, k);
              }
            }
          }
        }
        if (a.lfa) {
          // getNextHopsWithMetric with LFA (Decision.cpp:1126-1175) and
          // getNextHopsThrift without the shortest-metric filter: every up
          // link to a next-hop node n, metric w(link) + value(n), value =
          // mn - d(s, n) for shortest-path next hops, lowered to d(n, x) for
          // any destination x with d(n, x) < mn + d(n, s) (RFC 5286)
          for (uint32_t k = 0; k < WL; ++k) {
            uint64_t out = 0;
            const uint32_t j1 = min(deg, 64 * k + 64);
            for (uint32_t j = 64 * k; j < j1; ++j) {
              const uint32_t n = st_nbr[j], sl = st_slotall[j];
              uint64_t w = 0;
#pragma unroll
              for (uint32_t kk = 0; kk < kRtMaskWords; ++kk) {
                w = (sl >> 6) == kk ? m[kk] : w;
              }
              uint32_t v = ((w >> (sl & 63)) & 1ull) ? mn - d[n] : kInf32;
              const uint32_t* rn = a.dist + (size_t)a.row_of[n] * a.Vp;
              const uint64_t lim = (uint64_t)mn + st_dns[j];
              for (uint32_t i = lo; i < hi; ++i) {
                const uint32_t x = a.ann[i];
                if (d[x] == kInf32 || (filt && !((a.trbits[x >> 5] >> (x & 31)) & 1u))) {
                  continue;
                }
                const uint32_t dx = rn[x];
                if (dx != kInf32 && (uint64_t)dx < lim) {
                  v = min(v, dx);
                }
              }
              lm[j] = v == kInf32 ? kInf32 : st_w[j] + v;
              out |= (uint64_t)(v != kInf32) << (j & 63);
            }
            lkp[k] = out;
          }
          continue;
        }
        for (uint32_t k = 0; k < WL; ++k) {
          uint64_t out = 0;
          const uint32_t j1 = min(deg, 64 * k + 64);
          for (uint32_t j = 64 * k; j < j1; ++j) {
            const uint32_t sl = st_slot[j];
            uint64_t w = 0;
#pragma unroll
            for (uint32_t kk = 0; kk < kRtMaskWords; ++kk) {
              w = (sl >> 6) == kk ? m[kk] : w;
            }
            out |= (sl == kInf32 ? 0ull : (w >> (sl & 63)) & 1ull) << (j & 63);
          }
          lkp[k] = out;
        }
        continue;
      }
      // general path (high-degree source): word by word from HBM
      for (uint32_t k = 0; k < WL; ++k) {
        uint64_t out = 0;
        const uint32_t j1 = min(deg, 64 * k + 64);
        for (uint32_t j = 64 * k; j < j1; ++j) {
          uint32_t sl;
          if (staged) {
            sl = st_slot[j];
          } else {
            const uint32_t nb = a.col[e0 + j];
            sl = a.wout[e0 + j] == d[nb] ? a.slot[e0 + j] : kInf32;
          }
          if (sl == kInf32) {
            continue;
          }
          uint64_t mm = 0;
          for (uint32_t i = lo; i < hi && !mm; ++i) {
            const uint32_t x = a.ann[i];
            if (d[x] == mn && (!filt || ((a.trbits[x >> 5] >> (x & 31)) & 1u))) {
              mm = (nh_load(nhq, NB, W, x, sl >> 6) >> (sl & 63)) & 1ull;
            }
          }
          out |= mm << (j & 63);
        }
        lkp[k] = out;
      }
    }
  }
}

// Route-table diff (spf_route_table_diff): cell (q, p) changed iff its
// metric, best announcer or link mask differs between the two tables — the
// route-selection part of RibUnicastEntry equality, so the changed cells are
// getRouteDelta's (Decision.cpp:47-85) unicast updates + deletes for every
// node at once.  One wave per 64 prefixes of a row: the ballot of changed
// lanes is the row's bitmap word; popcounts add up per row.
__global__ __launch_bounds__(256) void spf_route_table_diff_kernel(
    const uint32_t* __restrict__ ma, const uint32_t* __restrict__ ba,
    const uint64_t* __restrict__ la, const uint32_t* __restrict__ mb,
    const uint32_t* __restrict__ bb, const uint64_t* __restrict__ lb,
    const uint64_t* __restrict__ lk_off, uint32_t P, uint32_t nq, uint32_t pw,
    uint64_t* __restrict__ bits, uint32_t* __restrict__ count,
    const uint32_t* __restrict__ lma, const uint32_t* __restrict__ lmb,
    const uint64_t* __restrict__ lm_off) {
  const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
  for (uint32_t q = blockIdx.x; q < nq; q += gridDim.x) {
    const uint32_t WL = P ? (uint32_t)((lk_off[q + 1] - lk_off[q]) / P) : 0;
    const uint64_t* la_q = la + lk_off[q];
    const uint64_t* lb_q = lb + lk_off[q];
    uint32_t n = 0;
    for (uint32_t w = wv; w < pw; w += blockDim.x / 64) {
      const uint32_t p = w * 64 + lane;
      bool ch = false;
      if (p < P) {
        const size_t o = (size_t)q * P + p;
        ch = ma[o] != mb[o] || ba[o] != bb[o];
        for (uint32_t k = 0; k < WL && !ch; ++k) {
          ch = la_q[(size_t)p * WL + k] != lb_q[(size_t)p * WL + k];
        }
        if (lma && !ch) { // LFA tables: per-link metrics too
          const uint64_t deg = (lm_off[q + 1] - lm_off[q]) / P;
          const size_t b0 = lm_off[q] + (size_t)p * deg;
          for (uint64_t j = 0; j < deg && !ch; ++j) {
            ch = lma[b0 + j] != lmb[b0 + j];
          }
        }
      }
      const uint64_t word = __ballot(ch);
      if (lane == 0) {
        bits[(size_t)q * pw + w] = word;
        n += __popcll(word);
      }
    }
    if (lane == 0 && n) {
      atomicAdd(&count[q], n);
    }
  }
}

// ------------------------------------------------ k-th path traces (KSP2)
//
// getKthPaths' trace loop (LinkState.cpp:776-786) over one query row: repeated
// traceOnePath (LinkState.cpp:398-419) from the query's source to its
// destination with one visited-link set, until a trace fails.  One wave per
// query; the recursion is an explicit stack in LDS whose frames hold a
// cursor into the node's pathLinks order.  pathLinks(v) = the usable tight
// in-links u -> v (u reached, u the source or transit, link not ignored,
// d[u] + w(u->v) == d[v]) ordered by the tail's settle rank (d[u], u) and then
// by the half-edge's position in u's row (linksFromNode(u) order); on the
// 32-bit plans every metric is >= 1, so each such tail settles before v.  A
// frame's next pathLink is the smallest key (d[u] << 32 | u, half-edge + 1)
// above its cursor: the wave scans v's in-edges 64 at a time and reduces.
// Visited links live in a per-wave open-addressing set in LDS (64 slots
// probed per step); nodes whose search failed in a second one (the host
// trace's `dead` memo: every pathLink of such a node is already visited, so a
// repeat search fails with no side effect).  A query whose set, stack or
// output would overflow reports kTraceOverflow and is traced on the host.
constexpr uint32_t kTraceWaves = 4;      // queries per 256-thread block
constexpr uint32_t kTraceHash = 1024;    // visited-link slots per wave (<= 1/2 full)
constexpr uint32_t kTraceDead = 512;     // failed-node slots per wave
constexpr uint32_t kTraceDepth = 128;    // recursion frames per wave
constexpr uint32_t kTraceOverflow = 0xFFFFFFFFu;
constexpr uint32_t kTraceCap = 4096;     // links (and paths) per query
constexpr uint32_t kTraceEmpty = 0xFFFFFFFFu;

struct TraceArgs {
  const uint32_t* row;
  const uint32_t* col;
  const uint32_t* rev;
  const uint32_t* link;
  const uint32_t* wout;
  const uint32_t* trbits;
  const uint32_t* src;     // [nq]
  const uint32_t* dst;     // [nq]
  const uint32_t* ign_off; // [nq + 1] or nullptr
  const uint32_t* ign;
  const uint32_t* dist;    // [nq][Vp]
  uint32_t* out_n;         // [nq] paths, or kTraceOverflow
  uint32_t* out_len;       // [nq] links of all its paths
  uint32_t* out_links;     // [nq][cap] link ids, paths back to back (src -> dst)
  uint32_t* out_ends;      // [nq][cap] end offset of each path in out_links
  uint32_t Vp;
  uint32_t nq;
  uint32_t cap;
  uint32_t unit;
};

__device__ __forceinline__ uint32_t trace_hash(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352dU;
  x ^= x >> 15;
  x *= 0x846ca68bU;
  x ^= x >> 16;
  return x;
}

// wave-uniform insert of key into a linear-probing set of `cap` slots:
// 1 = inserted, 0 = present, -1 = full (more than half the slots used)
template <uint32_t CAP>
__device__ __forceinline__ int trace_set_insert(uint32_t* set, uint32_t& used, uint32_t key,
                                                uint32_t lane) {
  uint32_t h = trace_hash(key);
  for (uint32_t probe = 0; probe < CAP; probe += 64, h += 64) {
    const uint32_t slot = (h + lane) & (CAP - 1);
    const uint32_t x = set[slot];
    if (__ballot(x == key)) {
      return 0;
    }
    const uint64_t empty = __ballot(x == kTraceEmpty);
    if (empty) {
      if (2 * (used + 1) > CAP) {
        return -1;
      }
      const uint32_t first = (uint32_t)__builtin_ctzll(empty);
      if (lane == first) {
        set[slot] = key;
      }
      ++used;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      return 1;
    }
  }
  return -1;
}

template <uint32_t CAP>
__device__ __forceinline__ bool trace_set_has(const uint32_t* set, uint32_t key, uint32_t lane) {
  uint32_t h = trace_hash(key);
  for (uint32_t probe = 0; probe < CAP; probe += 64, h += 64) {
    const uint32_t x = set[(h + lane) & (CAP - 1)];
    if (__ballot(x == key)) {
      return true;
    }
    if (__ballot(x == kTraceEmpty)) {
      return false;
    }
  }
  return false;
}

__global__ __launch_bounds__(64 * kTraceWaves) void spf_trace_paths_kernel(TraceArgs a) {
  __shared__ uint32_t vis_s[kTraceWaves][kTraceHash];
  __shared__ uint32_t dead_s[kTraceWaves][kTraceDead];
  __shared__ uint64_t cp_s[kTraceWaves][kTraceDepth];
  __shared__ uint32_t ce_s[kTraceWaves][kTraceDepth];
  __shared__ uint32_t node_s[kTraceWaves][kTraceDepth];
  __shared__ uint32_t lnk_s[kTraceWaves][kTraceDepth];
  const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
  const uint32_t q = blockIdx.x * kTraceWaves + wv;
  if (q >= a.nq) {
    return; // whole wave: no block-level barrier below
  }
  uint32_t* vis = vis_s[wv];
  uint32_t* dead = dead_s[wv];
  uint64_t* cp = cp_s[wv];
  uint32_t* ce = ce_s[wv];
  uint32_t* node = node_s[wv];
  uint32_t* lnk = lnk_s[wv];
  for (uint32_t i = lane; i < kTraceHash; i += 64) {
    vis[i] = kTraceEmpty;
  }
  for (uint32_t i = lane; i < kTraceDead; i += 64) {
    dead[i] = kTraceEmpty;
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  const uint32_t s = a.src[q], d = a.dst[q];
  const uint32_t* dist = a.dist + (size_t)q * a.Vp;
  const uint32_t ilo = a.ign_off ? a.ign_off[q] : 0u;
  const uint32_t ihi = a.ign_off ? a.ign_off[q + 1] : 0u;
  uint32_t* out_links = a.out_links + (size_t)q * a.cap;
  uint32_t* out_ends = a.out_ends + (size_t)q * a.cap;
  uint32_t npaths = 0, nl = 0, vused = 0, dused = 0;
  bool overflow = false;
  if (s != d && dist[d] != kInf32) {
    for (;;) { // one traceOnePath per iteration
      uint32_t depth = 0;
      node[0] = d;
      cp[0] = 0;
      ce[0] = 0;
      bool found = false;
      for (;;) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        const uint32_t v = node[depth];
        const uint64_t ccp = cp[depth];
        const uint32_t cce = ce[depth];
        const uint64_t dv = dist[v];
        // next pathLink of v after the cursor (ccp, cce)
        uint64_t bp = ~0ull;
        uint32_t bk = kInf32, be = kInf32;
        const uint32_t e0 = a.row[v], e1 = a.row[v + 1];
        for (uint32_t base = e0; base < e1; base += 64) {
          const uint32_t e = base + lane;
          uint64_t p = ~0ull;
          uint32_t k2 = kInf32;
          if (e < e1) {
            const uint32_t u = a.col[e];
            const uint32_t du = dist[u];
            bool ok = du != kInf32 && (u == s || ((a.trbits[u >> 5] >> (u & 31)) & 1u));
            uint32_t eu = 0;
            if (ok) {
              eu = a.rev[e];
              const uint64_t w = a.unit ? 1ull : (uint64_t)a.wout[eu];
              ok = (uint64_t)du + w == dv;
            }
            if (ok && ihi > ilo) {
              const uint32_t l = a.link[e];
              for (uint32_t i = ilo; i < ihi; ++i) {
                if (a.ign[i] == l) {
                  ok = false;
                  break;
                }
              }
            }
            if (ok) {
              const uint64_t pk = ((uint64_t)du << 32) | u;
              if (pk > ccp || (pk == ccp && eu + 1 > cce)) {
                p = pk;
                k2 = eu + 1;
              }
            }
          }
          if (p < bp || (p == bp && k2 < bk)) {
            bp = p;
            bk = k2;
            be = e;
          }
        }
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) {
          const uint64_t op = (uint64_t)__shfl_xor((unsigned long long)bp, off, 64);
          const uint32_t ok2 = (uint32_t)__shfl_xor((int)bk, off, 64);
          const uint32_t oe = (uint32_t)__shfl_xor((int)be, off, 64);
          if (op < bp || (op == bp && ok2 < bk)) {
            bp = op;
            bk = ok2;
            be = oe;
          }
        }
        if (bp == ~0ull) {
          // v exhausted: the search from v fails (dead memo, best effort)
          if (trace_set_insert<kTraceDead>(dead, dused, v, lane) < 0) {
            dused = kTraceDead; // full: stop recording (an optimisation only)
          }
          if (depth == 0) {
            break;
          }
          --depth;
          continue;
        }
        cp[depth] = bp;
        ce[depth] = bk;
        const uint32_t l = a.link[be];
        const int ins = trace_set_insert<kTraceHash>(vis, vused, l, lane);
        if (ins < 0) {
          overflow = true;
          break;
        }
        if (ins == 0) {
          continue; // link already taken by some trace
        }
        lnk[depth] = l;
        const uint32_t u = a.col[be];
        if (u == s) {
          found = true;
          break;
        }
        if (trace_set_has<kTraceDead>(dead, u, lane)) {
          continue; // the recursive search fails at once
        }
        if (depth + 1 >= kTraceDepth) {
          overflow = true;
          break;
        }
        ++depth;
        node[depth] = u;
        cp[depth] = 0;
        ce[depth] = 0;
      }
      if (overflow || !found) {
        break;
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      const uint32_t len = depth + 1;
      if (nl + len > a.cap || npaths + 1 > a.cap) {
        overflow = true;
        break;
      }
      // frames deepest first: the path runs src -> dst
      for (uint32_t i = lane; i < len; i += 64) {
        out_links[nl + i] = lnk[depth - i];
      }
      nl += len;
      if (lane == 0) {
        out_ends[npaths] = nl;
      }
      ++npaths;
    }
  }
  if (lane == 0) {
    a.out_n[q] = overflow ? kTraceOverflow : npaths;
    a.out_len[q] = overflow ? 0u : nl;
  }
}

// Cursor DFS (spf_trace_cursor_kernel, the default).  traceOnePath's visited
// set only ever grows, and a link u -> v is examined only by the loop over
// pathLinks(v) (on the 32-bit plans every metric is >= 1, so a link is a
// pathLink of at most one of its ends), in pathLinks order, from the start,
// inserting every link it examines (LinkState.cpp:407-416).  The examined
// links of v are therefore always a PREFIX of pathLinks(v), and the whole
// visited set is one cursor per node: a step is "take pathLinks(v)[cursor(v)++]",
// a node whose cursor reached the end fails at once (the host trace's dead
// memo), and a later traceOnePath of the same loop resumes every node where
// the last one left it.  pathLinks(v) is built once per (query, node) when
// the search first enters v: v's in-edges are filtered (usable, tight, tail
// the source or transit, link not ignored), ranked by (d[u], u, u's row
// position) and written to a per-wave arena in global scratch; node states
// {query tag, arena offset, length, cursor} live in a per-wave node array.
// The whole search is one wave's chain of dependent L2 round trips (the
// fabric's slowest query, 24,859 steps over 5,301 lists, was the entire
// 23.7 ms launch: profiles/r04ab), so a step is a BATCH: the 64 next
// pathLinks of v and their tails' states {state, d, row bounds} in two round
// trips, every entry whose tail already failed taken at once, the first live
// one entered with its build inputs already in registers, and a just-built
// list scanned from its LDS ranking instead of the arena.
// Only the recursion stack is in LDS, so nothing but a path longer than
// kTcDepth links, a node with more than kTcSort pathLinks or a full arena
// overflows to the host.
constexpr uint32_t kTcWaves = 4;    // waves (queries in flight) per block (16 per CU)
constexpr uint32_t kTcDepth = 256;  // recursion frames per wave
constexpr uint32_t kTcSort = 256;   // pathLinks of one node ranked in LDS
constexpr uint32_t kTcIgn = 512;    // ignore-list LDS words per query (hash slots or the sorted list)

struct TraceCursorArgs {
  TraceArgs t;
  uint4* nstate;   // [waves][V] {tag, arena offset, length, cursor}
  uint2* arena;    // [waves][arena_cap] {tail, link} of pathLinks(v), in order
  uint32_t arena_cap;
  // DFS steps one query may take on the device (OPENR_SPF_TRACE_BUDGET,
  // default unlimited): a query past it is reported as an overflow and traced
  // on the host from its row.
  uint32_t budget = 0xFFFFFFFFu;
  uint32_t V;
  // OPENR_SPF_TRACE_STATS=1: per query {wall ticks (100 MHz), DFS steps,
  // pathLinks lists built, their filter ticks, rank ticks, entries}; nullptr = off
  unsigned long long* qstat = nullptr;
  // queries past the first nwaves are claimed from this counter (zeroed per
  // launch) by the wave that frees up first; nullptr: static stride
  uint32_t* qctr = nullptr;
};
constexpr uint32_t kTcStat = 6;

__device__ __forceinline__ void tc_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

__device__ __forceinline__ uint2 ld_coh2(const uint2* p) {
  const uint64_t x = __hip_atomic_load(reinterpret_cast<const uint64_t*>(p), __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
  return make_uint2((uint32_t)x, (uint32_t)(x >> 32));
}

__device__ __forceinline__ uint4 tc_load4(const uint4* p) {
  // the state may have been written by another lane of this wave (or by
  // this wave for an earlier query): read it from L2, not the vector L1
  const uint32_t* w = reinterpret_cast<const uint32_t*>(p);
  return make_uint4(ld_coh(w), ld_coh(w + 1), ld_coh(w + 2), ld_coh(w + 3));
}

// STATS: the OPENR_SPF_TRACE_STATS build of the kernel (per-query clocks and
// counts); the default build carries no instrumentation
template <bool STATS>
__global__ __launch_bounds__(64 * kTcWaves) void spf_trace_cursor_kernel(TraceCursorArgs A) {
  const TraceArgs& a = A.t;
  __shared__ uint32_t stk_s[kTcWaves][kTcDepth];  // node of each frame
  __shared__ uint32_t lnk_s[kTcWaves][kTcDepth];  // link taken at each frame
  __shared__ uint4 fst_s[kTcWaves][kTcDepth];     // the frame node's state (cursor in LDS)
  __shared__ uint64_t key_s[kTcWaves][kTcSort];   // (d[u] << 32 | u), then the ranked list
  __shared__ uint32_t sub_s[kTcWaves][kTcSort];   // u's row position (tie-break)
  __shared__ uint32_t edg_s[kTcWaves][kTcSort];   // link of the in-edge
  __shared__ uint32_t ign_s[kTcWaves][kTcIgn];
  const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
  const uint32_t gw = blockIdx.x * kTcWaves + wv, nwaves = gridDim.x * kTcWaves;
  uint4* ns = A.nstate + (size_t)gw * A.V;
  uint2* arena = A.arena + (size_t)gw * A.arena_cap;
  uint32_t* stk = stk_s[wv];
  uint32_t* lnk = lnk_s[wv];
  uint4* fst = fst_s[wv];
  uint64_t* keys = key_s[wv];
  uint2* srt = reinterpret_cast<uint2*>(key_s[wv]); // the last built list, ranked
  uint32_t* subs = sub_s[wv];
  uint32_t* lnks = edg_s[wv];
  uint32_t* ignl = ign_s[wv];
  const uint64_t lt_mask = lane ? (~0ull >> (64 - lane)) : 0ull;
  // a wave's own node-state / arena stores are waited for before its next
  // coherent read of that array (one s_waitcnt, not one per store; the
  // arena's after a build, so a fresh list's scan does not wait on them).
  // A macro on plain locals: flags captured by a lambda around the asm's
  // memory clobber were kept in scratch, a vector memory round trip per test.
  bool pend_a = false, pend_n = false;
#define TC_DRAIN(p)                                     \
  do {                                                  \
    if (p) {                                            \
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); \
      pend_a = pend_n = false;                          \
    }                                                   \
  } while (0)
  // the next query of this wave: claimed dynamically (a wave that drew
  // short traces takes more of them; with the static stride the slowest
  // wave's share set the launch), or the static stride
  auto next_query = [&](uint32_t q) -> uint32_t {
    if (!A.qctr) {
      return q + nwaves;
    }
    uint32_t c = 0;
    if (lane == 0) {
      c = atomicAdd(A.qctr, 1u);
    }
    return nwaves + (uint32_t)__builtin_amdgcn_readfirstlane((int)c);
  };
  for (uint32_t q = gw; q < a.nq; q = next_query(q)) { // wave-uniform loop
    const uint32_t tag = q + 1;
    const uint32_t s = a.src[q], d = a.dst[q];
    const uint32_t* dist = a.dist + (size_t)q * a.Vp;
    const uint32_t ilo = a.ign_off ? a.ign_off[q] : 0u;
    const uint32_t nign = a.ign_off ? a.ign_off[q + 1] - ilo : 0u;
    // the ignore list (the k = 1 paths' links, hundreds on the fabric) as an
    // LDS hash set: one or two probes per filtered in-edge, not a binary search
    IgnSet ig;
    ig.p = a.ign + ilo;
    ig.n = nign;
    const uint32_t slots = ign_hash_slots(nign);
    if (slots && slots <= kTcIgn) {
      for (uint32_t i = lane; i < slots; i += 64) {
        ignl[i] = kInf32;
      }
      tc_sync();
      const uint32_t hb = __builtin_ctz(slots);
      for (uint32_t i = lane; i < nign; i += 64) {
        const uint32_t l = a.ign[ilo + i];
        uint32_t h = (l * 0x9E3779B1u) >> (32 - hb);
        for (;;) {
          const uint32_t prev = atomicCAS(&ignl[h], kInf32, l);
          if (prev == kInf32 || prev == l) {
            break;
          }
          h = (h + 1) & (slots - 1);
        }
      }
      ig.p = ignl;
      ig.hbits = hb;
    } else if (nign <= kTcIgn) {
      for (uint32_t i = lane; i < nign; i += 64) {
        ignl[i] = a.ign[ilo + i];
      }
      ig.p = ignl;
    }
    tc_sync();
    uint32_t* out_links = a.out_links + (size_t)q * a.cap;
    uint32_t* out_ends = a.out_ends + (size_t)q * a.cap;
    uint32_t npaths = 0, nl = 0, atop = 0;
    bool overflow = false;
    unsigned long long tq0 = STATS ? wall_clock64() : 0ull, nsteps = 0, nbuilt = 0;
    unsigned long long tbuild = 0, trank = 0, nlen = 0; // stats: filter / rank ticks, list entries
    // pathLinks(v) into the arena (and ranked into srt): v's in-edges e0..e1
    // filtered (usable, tight against dv, tail the source or transit, link
    // not ignored) and ranked by (d[u], u, u's row position).  Returns v's
    // new state {tag, offset, length, 0}, or cursor kInf32 on overflow.
    auto build = [&](uint32_t v, uint32_t dv, uint32_t e0, uint32_t e1) -> uint4 {
      ++nbuilt;
      const unsigned long long tb0 = STATS ? wall_clock64() : 0ull;
      uint32_t n = 0;
      for (uint32_t base = e0; base < e1; base += 64) {
        const uint32_t e = base + lane;
        bool ok = false;
        uint32_t u = 0, du = 0, eu = 0, l = 0;
        if (e < e1) {
          // two dependent round trips: the edge's words, then its tail's
          u = a.col[e];
          eu = a.rev[e];
          l = a.link[e];
          du = dist[u];
          const uint32_t tb = a.trbits[u >> 5];
          const uint64_t w = a.unit ? 1ull : (uint64_t)a.wout[eu];
          ok = du != kInf32 && (u == s || ((tb >> (u & 31)) & 1u)) && (uint64_t)du + w == dv;
          if (ok && nign) {
            ok = !ig.has(l);
          }
        }
        const uint64_t m = __ballot(ok);
        const uint32_t pos = n + (uint32_t)__popcll(m & lt_mask);
        if (ok && pos < kTcSort) {
          keys[pos] = ((uint64_t)du << 32) | u;
          subs[pos] = eu;
          lnks[pos] = l;
        }
        n += (uint32_t)__popcll(m);
      }
      tc_sync();
      if (n > kTcSort || atop + n > A.arena_cap) {
        return make_uint4(0, 0, 0, kInf32); // overflow marker
      }
      const unsigned long long tb1 = STATS ? wall_clock64() : 0ull;
      uint32_t rr[kTcSort / 64], tl[kTcSort / 64], lk[kTcSort / 64];
      if (n <= 64) {
        // one entry per lane: rank against the others' keys read across
        // lanes (no LDS round trip per comparison)
        const bool in = lane < n;
        const uint64_t key = in ? keys[lane] : ~0ull;
        const uint32_t su = in ? subs[lane] : ~0u;
        const uint32_t klo = (uint32_t)key, khi = (uint32_t)(key >> 32);
        uint32_t r = 0;
        for (uint32_t j = 0; j < n; ++j) {
          const uint32_t jlo = (uint32_t)__builtin_amdgcn_readlane((int)klo, (int)j);
          const uint32_t jhi = (uint32_t)__builtin_amdgcn_readlane((int)khi, (int)j);
          const uint32_t js = (uint32_t)__builtin_amdgcn_readlane((int)su, (int)j);
          const uint64_t kj = ((uint64_t)jhi << 32) | jlo;
          r += (uint32_t)(kj < key) | ((uint32_t)(kj == key) & (uint32_t)(js < su));
        }
        rr[0] = r;
        tl[0] = klo;
        lk[0] = in ? lnks[lane] : 0u;
      } else {
#pragma unroll
        for (uint32_t k = 0; k < kTcSort / 64; ++k) {
          const uint32_t i = lane + 64 * k;
          if (i < n) {
            const uint64_t key = keys[i];
            const uint32_t su = subs[i];
            uint32_t r = 0;
            for (uint32_t j = 0; j < n; ++j) {
              const uint64_t kj = keys[j];
              r += (uint32_t)(kj < key) | ((uint32_t)(kj == key) & (uint32_t)(subs[j] < su));
            }
            rr[k] = r;
            tl[k] = (uint32_t)key;
            lk[k] = lnks[i];
          }
        }
      }
      tc_sync(); // every rank read the keys: srt reuses their words
#pragma unroll
      for (uint32_t k = 0; k < kTcSort / 64; ++k) {
        if (lane + 64 * k < n) {
          // the tail and the link: a scan reads one 8-byte entry per lane
          const uint2 ent = make_uint2(tl[k], lk[k]);
          srt[rr[k]] = ent;
          arena[atop + rr[k]] = ent;
        }
      }
      const uint4 st = make_uint4(tag, atop, n, 0);
      atop += n;
      if (n == 0 && lane == 0) {
        ns[v] = st; // no pathLink: every later visit fails at once
      }
      tc_sync();
      if (STATS) {
        const unsigned long long tb2 = wall_clock64();
        tbuild += tb1 - tb0;
        trank += tb2 - tb1;
        nlen += n;
      }
      return st;
    };
    if (s != d && dist[d] != kInf32) {
      for (;;) { // one traceOnePath per iteration
        uint32_t depth = 0, fresh = kTcDepth; // fresh: the frame whose list is in srt
        TC_DRAIN(pend_n);
        uint4 st = tc_load4(ns + d);
        if (st.x != tag) {
          st = build(d, dist[d], a.row[d], a.row[d + 1]);
          (st.z ? pend_a : pend_n) = true;
          fresh = 0;
          if (st.w == kInf32) {
            overflow = true;
            break;
          }
        }
        if (lane == 0) {
          stk[0] = d;
          fst[0] = st;
        }
        tc_sync();
        bool found = false;
        for (;;) {
          if (++nsteps > A.budget) {
            overflow = true;
            break;
          }
          st = fst[depth];
          if (st.w >= st.z) {
            // v exhausted: the search through it fails; its state goes back
            if (lane == 0) {
              ns[stk[depth]] = st;
            }
            pend_n = true;
            if (depth == 0) {
              break;
            }
            --depth;
            continue;
          }
          // a batch of v's next pathLinks and the states of their tails in
          // two round trips: entries whose tail already failed are taken
          // (their link becomes visited) and skipped without a step each
          const uint32_t cnt = min(64u, st.z - st.w);
          const bool have = lane < cnt;
          uint2 ent = make_uint2(kInf32, 0);
          if (have) {
            if (depth == fresh) {
              ent = srt[st.w + lane];
            } else {
              TC_DRAIN(pend_a);
              ent = ld_coh2(arena + st.y + st.w + lane);
            }
          }
          const uint32_t u = ent.x;
          uint4 su = make_uint4(0, 0, 0, 0);
          uint32_t du = 0, r0 = 0, r1 = 0;
          TC_DRAIN(pend_n);
          if (have && u != s) {
            su = tc_load4(ns + u);
            du = dist[u];
            r0 = a.row[u];
            r1 = a.row[u + 1];
          }
          const bool live = have && (u == s || su.x != tag || su.w < su.z);
          const uint64_t lm = __ballot(live);
          if (lm == 0) {
            st.w += cnt;
            if (lane == 0) {
              fst[depth] = st;
            }
            tc_sync();
            continue;
          }
          const int f = (int)__builtin_ctzll(lm);
          const uint32_t fu = (uint32_t)__builtin_amdgcn_readlane((int)u, f);
          st.w += (uint32_t)f + 1;
          if (lane == 0) {
            fst[depth] = st;
            lnk[depth] = (uint32_t)__builtin_amdgcn_readlane((int)ent.y, f);
          }
          if (fu == s) {
            found = true;
            break;
          }
          if (depth + 1 >= kTcDepth) {
            overflow = true;
            break;
          }
          uint4 sf = make_uint4((uint32_t)__builtin_amdgcn_readlane((int)su.x, f),
                                (uint32_t)__builtin_amdgcn_readlane((int)su.y, f),
                                (uint32_t)__builtin_amdgcn_readlane((int)su.z, f),
                                (uint32_t)__builtin_amdgcn_readlane((int)su.w, f));
          bool built = false;
          if (sf.x != tag) {
            sf = build(fu, (uint32_t)__builtin_amdgcn_readlane((int)du, f),
                       (uint32_t)__builtin_amdgcn_readlane((int)r0, f),
                       (uint32_t)__builtin_amdgcn_readlane((int)r1, f));
            if (sf.w == kInf32) {
              overflow = true;
              break;
            }
            (sf.z ? pend_a : pend_n) = true;
            built = true;
            if (sf.z == 0) {
              fresh = kTcDepth;
              tc_sync();
              continue; // u's search fails at once: next pathLink of v
            }
          }
          ++depth;
          fresh = built ? depth : kTcDepth;
          if (lane == 0) {
            stk[depth] = fu;
            fst[depth] = sf;
          }
          tc_sync();
        }
        if (overflow || !found) {
          break;
        }
        tc_sync();
        // every frame's cursor moved on: the states go back
        for (uint32_t f = lane; f <= depth; f += 64) {
          ns[stk[f]] = fst[f];
        }
        pend_n = true;
        const uint32_t len = depth + 1;
        if (nl + len > a.cap || npaths + 1 > a.cap) {
          overflow = true;
          break;
        }
        // frames deepest first: the path runs src -> dst
        for (uint32_t i = lane; i < len; i += 64) {
          out_links[nl + i] = lnk[depth - i];
        }
        nl += len;
        if (lane == 0) {
          out_ends[npaths] = nl;
        }
        ++npaths;
        tc_sync();
      }
    }
    if (lane == 0) {
      a.out_n[q] = overflow ? kTraceOverflow : npaths;
      a.out_len[q] = overflow ? 0u : nl;
      if (STATS) {
        unsigned long long* o = A.qstat + kTcStat * (size_t)q;
        o[0] = wall_clock64() - tq0;
        o[1] = nsteps;
        o[2] = nbuilt;
        o[3] = tbuild;
        o[4] = trank;
        o[5] = nlen;
      }
    }
    TC_DRAIN(pend_a || pend_n); // the next query's tag check reads node states
    tc_sync(); // the next query restages the ignore list
  }
#undef TC_DRAIN
}

// Heavy queries (the ones past the cursor kernel's step budget: on the fabric
// ONE destination's trace was that whole 17 ms launch, 15,304 serial steps,
// profiles/r04ab) get a launch of their own, in two kernels:
//  * spf_trace_heavy_build_kernel, one wave per (query, node) over the whole
//    grid: pathLinks(v) of every node of the query's row, filtered and ranked
//    exactly as the cursor kernel's build, into an arena slotted by CSR row
//    (pathLinks(v) <= in-degree(v) = row[v + 1] - row[v] entries at row[v]);
//  * spf_trace_heavy_kernel, one wave per query: every node's {cursor,
//    length} and arena base in LDS, so a DFS step is ONE global round trip
//    (the 64 next entries of v's list) and the tails' states are LDS reads.
// Same DFS, same output as spf_trace_cursor_kernel (the cursor argument
// above); a list over kTcSort entries or a path over kTcDepth links is still
// an overflow, traced on the host.
constexpr uint32_t kHvMaxV = 16384; // LDS: 2 words per node
// the cursor kernel's default step budget when the heavy launch is on
constexpr uint32_t kTcHeavyBudget = 1024;
constexpr uint32_t kHvWaves = 4;    // build waves per block

struct TraceHeavyArgs {
  TraceArgs t;
  const uint32_t* hq; // [nh] query indices (into t's queries)
  uint32_t nh;
  uint32_t V, E;
  uint2* arena;       // [nh][E] {tail, link}, pathLinks(v) at row[v]
  uint32_t* len;      // [nh][V] pathLinks(v) length, or kInf32 (over kTcSort)
  uint32_t budget;    // DFS steps per query (0xFFFFFFFF: none)
  // OPENR_SPF_TRACE_STATS=1: per heavy query {wall ticks (100 MHz), steps,
  // pushes, global batch loads}; nullptr = off
  unsigned long long* hstat;
  // blocks of query hi built on XCD hi % 8, the XCD its DFS block runs on
  // (blocks go round-robin over the 8 XCDs): its arena is read from that
  // XCD's L2 instead of across the fabric.  0: plain item order.
  uint32_t xcd;
  uint32_t L;         // link ids (the removed-link bitset of the reach kernel)
  uint32_t* fq;       // [nh][2][V] the reach kernel's BFS frontiers
  const uint32_t* nodes; // [V] build order: in-degree <= 16 first (nsmall), then the rest
  uint32_t nsmall;
};

// Blocks of the build per heavy query: nodes of in-degree <= 16 four to a
// wave (16 lanes each: the fabric's RSWs, 83% of its nodes, have 8), the
// others one per wave.
// work units of one query (a unit = one block's pass); a block takes
// kHvRounds of them (4 measured slower than 1: 1.24 vs 1.08 ms, profiles/r05af)
constexpr uint32_t kHvRounds = 1;
__host__ __device__ inline uint32_t hv_units(uint32_t nsmall, uint32_t nbig) {
  return (nsmall + 4 * kHvWaves - 1) / (4 * kHvWaves) + (nbig + kHvWaves - 1) / kHvWaves;
}
__host__ __device__ inline uint32_t hv_blocks(uint32_t nsmall, uint32_t nbig) {
  return (hv_units(nsmall, nbig) + kHvRounds - 1) / kHvRounds;
}

__global__ __launch_bounds__(64 * kHvWaves) void spf_trace_heavy_build_kernel(TraceHeavyArgs H) {
  const TraceArgs& a = H.t;
  __shared__ uint64_t key_s[kHvWaves][kTcSort];
  __shared__ uint32_t sub_s[kHvWaves][kTcSort];
  __shared__ uint32_t lnk_s[kHvWaves][kTcSort];
  __shared__ uint32_t ign_s[kTcIgn];
  const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
  const uint32_t nbig = H.V - H.nsmall;
  const uint32_t bs = (H.nsmall + 4 * kHvWaves - 1) / (4 * kHvWaves);
  const uint32_t bq = hv_blocks(H.nsmall, nbig);
  uint32_t hi, k;
  if (H.xcd) {
    const uint32_t ka = blockIdx.x >> 3;
    hi = (ka / bq) * 8u + (blockIdx.x & 7u);
    k = ka % bq;
  } else {
    hi = blockIdx.x / bq;
    k = blockIdx.x % bq;
  }
  if (hi >= H.nh) {
    return; // whole block
  }
  const uint32_t q = H.hq[hi];
  const uint32_t s = a.src[q];
  const uint32_t* dist = a.dist + (size_t)q * a.Vp;
  const uint32_t ilo = a.ign_off ? a.ign_off[q] : 0u;
  const uint32_t nign = a.ign_off ? a.ign_off[q + 1] - ilo : 0u;
  // the query's ignore list as an LDS hash set (one block = one query)
  IgnSet ig;
  ig.p = a.ign + ilo;
  ig.n = nign;
  const uint32_t slots = ign_hash_slots(nign);
  if (slots && slots <= kTcIgn) {
    for (uint32_t i = threadIdx.x; i < slots; i += 64 * kHvWaves) {
      ign_s[i] = kInf32;
    }
    __syncthreads();
    const uint32_t hb = __builtin_ctz(slots);
    for (uint32_t i = threadIdx.x; i < nign; i += 64 * kHvWaves) {
      const uint32_t l = a.ign[ilo + i];
      uint32_t h = (l * 0x9E3779B1u) >> (32 - hb);
      for (;;) {
        const uint32_t prev = atomicCAS(&ign_s[h], kInf32, l);
        if (prev == kInf32 || prev == l) {
          break;
        }
        h = (h + 1) & (slots - 1);
      }
    }
    __syncthreads();
    ig.p = ign_s;
    ig.hbits = hb;
  }
  uint32_t* lenq = H.len + (size_t)hi * H.V;
  uint2* arq = H.arena + (size_t)hi * H.E;
  // in-edge e of v (tail u = col[e]) as a pathLink: usable, tight, tail the
  // source or transit, link not ignored (the cursor kernel's filter)
  auto tight = [&](uint32_t e, uint32_t dv, uint32_t& u, uint32_t& du, uint32_t& eu,
                   uint32_t& l) -> bool {
    u = a.col[e];
    eu = a.rev[e];
    l = a.link[e];
    du = dist[u];
    const uint32_t tb = a.trbits[u >> 5];
    const uint64_t w = a.unit ? 1ull : (uint64_t)a.wout[eu];
    bool ok = du != kInf32 && (u == s || ((tb >> (u & 31)) & 1u)) && (uint64_t)du + w == dv;
    if (ok && nign) {
      ok = !ig.has(l);
    }
    return ok;
  };
  const uint32_t nunits = hv_units(H.nsmall, nbig);
  for (uint32_t rd = 0; rd < kHvRounds; ++rd) {
  const uint32_t un = k * kHvRounds + rd; // block-uniform
  if (un >= nunits) {
    break;
  }
  if (un < bs) {
    // four small nodes per wave, 16 lanes each: filter in one pass, rank
    // the group's keys across its lanes
    const uint32_t g = lane >> 4, gl = lane & 15u;
    const uint32_t slot = (un * kHvWaves + wv) * 4 + g;
    const bool act = slot < H.nsmall;
    const uint32_t v = act ? H.nodes[slot] : 0u;
    const uint32_t dv = act ? dist[v] : kInf32;
    uint32_t e0 = 0, e1 = 0;
    if (dv != kInf32) {
      e0 = a.row[v];
      e1 = a.row[v + 1];
    }
    bool ok = false;
    uint32_t u = 0, du = 0, eu = 0, l = 0;
    if (e0 + gl < e1) {
      ok = tight(e0 + gl, dv, u, du, eu, l);
    }
    const uint32_t gm = (uint32_t)(__ballot(ok) >> (16 * g)) & 0xFFFFu;
    const uint64_t key = ((uint64_t)du << 32) | u;
    uint32_t r = 0;
#pragma unroll
    for (uint32_t j = 0; j < 16; ++j) {
      const uint32_t src = 16 * g + j;
      const uint32_t jlo = (uint32_t)__shfl((int)u, (int)src, 64);
      const uint32_t jhi = (uint32_t)__shfl((int)du, (int)src, 64);
      const uint32_t js = (uint32_t)__shfl((int)eu, (int)src, 64);
      const uint64_t kj = ((uint64_t)jhi << 32) | jlo;
      r += ((gm >> j) & 1u) & ((uint32_t)(kj < key) | ((uint32_t)(kj == key) & (uint32_t)(js < eu)));
    }
    if (ok) {
      arq[e0 + r] = make_uint2(u, l);
    }
    if (act && gl == 0) {
      lenq[v] = (uint32_t)__popc(gm);
    }
    continue;
  }
  const uint32_t bi = (un - bs) * kHvWaves + wv;
  if (bi >= nbig) {
    continue; // whole wave; no block barrier below
  }
  const uint32_t v = H.nodes[H.nsmall + bi];
  const uint32_t dv = dist[v];
  if (dv == kInf32) {
    if (lane == 0) {
      lenq[v] = 0;
    }
    continue;
  }
  uint64_t* keys = key_s[wv];
  uint32_t* subs = sub_s[wv];
  uint32_t* lnks = lnk_s[wv];
  const uint64_t lt_mask = lane ? (~0ull >> (64 - lane)) : 0ull;
  const uint32_t e0 = a.row[v], e1 = a.row[v + 1];
  uint32_t n = 0;
  for (uint32_t base = e0; base < e1; base += 64) {
    const uint32_t e = base + lane;
    bool ok = false;
    uint32_t u = 0, du = 0, eu = 0, l = 0;
    if (e < e1) {
      ok = tight(e, dv, u, du, eu, l);
    }
    const uint64_t m = __ballot(ok);
    const uint32_t pos = n + (uint32_t)__popcll(m & lt_mask);
    if (ok && pos < kTcSort) {
      keys[pos] = ((uint64_t)du << 32) | u;
      subs[pos] = eu;
      lnks[pos] = l;
    }
    n += (uint32_t)__popcll(m);
  }
  tc_sync();
  if (n > kTcSort) {
    if (lane == 0) {
      lenq[v] = kInf32;
    }
    continue;
  }
  uint2* ar = arq + e0;
  for (uint32_t i = lane; i < n; i += 64) {
    const uint64_t key = keys[i];
    const uint32_t su = subs[i];
    uint32_t r = 0;
    for (uint32_t j = 0; j < n; ++j) {
      const uint64_t kj = keys[j];
      r += (uint32_t)(kj < key) | ((uint32_t)(kj == key) & (uint32_t)(subs[j] < su));
    }
    ar[r] = make_uint2((uint32_t)key, lnks[i]);
  }
  if (lane == 0) {
    lenq[v] = n;
  }
  tc_sync(); // the wave's next pass reuses its LDS key buffer
  }
}

// The DFS of one heavy query.  The current frame (node, cursor, length,
// arena base, the batch of its next 64 entries: one per lane) lives in
// registers; a push saves the frame's batch to LDS (frames < kHvCache), so a
// pop resumes without a global round trip.  A step is then one LDS gather of
// the tails' states when it resumes a frame, plus one global load when it
// enters a new node (or runs past a 64-entry batch).
constexpr uint32_t kHvCache = 16;

__global__ __launch_bounds__(64) void spf_trace_heavy_kernel(TraceHeavyArgs H) {
  const TraceArgs& a = H.t;
  __shared__ uint32_t st[kHvMaxV];   // cursor << 16 | length
  __shared__ uint32_t rp[kHvMaxV];   // row[v]: v's arena base
  __shared__ uint32_t stk[kTcDepth]; // node of each frame
  __shared__ uint32_t lnk[kTcDepth]; // link taken at each frame
  __shared__ uint32_t fbs[kHvCache]; // first entry of each cached batch
  __shared__ uint2 cache[kHvCache][64];
  const uint32_t lane = threadIdx.x;
  const uint32_t hi = blockIdx.x;
  const uint32_t q = H.hq[hi];
  const uint32_t s = a.src[q], d = a.dst[q];
  const uint32_t* lenq = H.len + (size_t)hi * H.V;
  const uint2* ar = H.arena + (size_t)hi * H.E;
  bool bad = false;
  for (uint32_t v = lane; v < H.V; v += 64) {
    const uint32_t n = lenq[v];
    bad = bad || n == kInf32;
    st[v] = n == kInf32 ? 0u : n;
    rp[v] = a.row[v];
  }
  bool overflow = __ballot(bad) != 0;
  tc_sync();
  uint32_t* out_links = a.out_links + (size_t)q * a.cap;
  uint32_t* out_ends = a.out_ends + (size_t)q * a.cap;
  uint32_t npaths = 0, nl = 0, nsteps = 0, npush = 0, nload = 0;
  const unsigned long long t0 = H.hstat ? wall_clock64() : 0ull;
  // entries [bs, bs + 64) of the frame's list, one per lane
  auto load = [&](uint32_t base, uint32_t bs, uint32_t n) -> uint2 {
    ++nload;
    return bs + lane < n ? ar[base + bs + lane] : make_uint2(kInf32, 0u);
  };
  if (!overflow && s != d && a.dist[(size_t)q * a.Vp + d] != kInf32) {
    for (;;) { // one traceOnePath per iteration
      uint32_t depth = 0, v = d;
      uint32_t x = st[v];
      uint32_t c = x >> 16, n = x & 0xFFFFu, base = rp[v], bs = c;
      uint2 ent = load(base, bs, n);
      if (lane == 0) {
        stk[0] = d;
      }
      bool found = false;
      for (;;) {
        if (++nsteps > H.budget) {
          overflow = true;
          break;
        }
        if (c >= n) {
          // v exhausted: the search through it fails; back to its parent
          if (lane == 0) {
            st[v] = (n << 16) | n;
          }
          if (depth == 0) {
            break;
          }
          --depth;
          tc_sync();
          v = stk[depth];
          x = st[v];
          c = x >> 16;
          n = x & 0xFFFFu;
          base = rp[v];
          if (depth < kHvCache && c - fbs[depth] < 64u) {
            bs = fbs[depth];
            ent = cache[depth][lane];
          } else {
            bs = c;
            ent = load(base, bs, n);
          }
          continue;
        }
        if (c - bs >= 64u) {
          bs = c;
          ent = load(base, bs, n);
        }
        const uint32_t idx = bs + lane;
        const uint32_t u = ent.x;
        bool live = false;
        if (idx >= c && idx < n) {
          if (u == s) {
            live = true;
          } else {
            const uint32_t su = st[u];
            live = (su >> 16) < (su & 0xFFFFu);
          }
        }
        const uint64_t lm = __ballot(live);
        if (lm == 0) {
          // every remaining entry of the batch has a failed tail: taken
          c = min(n, bs + 64u);
          continue;
        }
        const uint32_t f = (uint32_t)__builtin_ctzll(lm);
        const uint32_t fu = (uint32_t)__builtin_amdgcn_readlane((int)u, (int)f);
        const uint32_t fl = (uint32_t)__builtin_amdgcn_readlane((int)ent.y, (int)f);
        c = bs + f + 1;
        if (lane == 0) {
          lnk[depth] = fl;
        }
        if (fu == s) {
          found = true;
          break;
        }
        if (depth + 1 >= kTcDepth) {
          overflow = true;
          break;
        }
        // push: v's cursor and batch saved, fu entered
        ++npush;
        if (lane == 0) {
          st[v] = (c << 16) | n;
        }
        if (depth < kHvCache) {
          cache[depth][lane] = ent;
          if (lane == 0) {
            fbs[depth] = bs;
          }
        }
        ++depth;
        if (lane == 0) {
          stk[depth] = fu;
        }
        tc_sync();
        v = fu;
        x = st[v];
        c = x >> 16;
        n = x & 0xFFFFu;
        base = rp[v];
        bs = c;
        ent = load(base, bs, n);
      }
      if (overflow) {
        break;
      }
      // the frame the search ended in keeps its cursor
      if (lane == 0) {
        st[v] = (c << 16) | n;
      }
      tc_sync();
      if (!found) {
        break;
      }
      const uint32_t len = depth + 1;
      if (nl + len > a.cap || npaths + 1 > a.cap) {
        overflow = true;
        break;
      }
      // frames deepest first: the path runs src -> dst
      for (uint32_t i = lane; i < len; i += 64) {
        out_links[nl + i] = lnk[depth - i];
      }
      nl += len;
      if (lane == 0) {
        out_ends[npaths] = nl;
      }
      ++npaths;
      tc_sync();
    }
  }
  if (lane == 0) {
    a.out_n[q] = overflow ? kTraceOverflow : npaths;
    a.out_len[q] = overflow ? 0u : nl;
    if (H.hstat) {
      unsigned long long* o = H.hstat + 4 * (size_t)hi;
      o[0] = wall_clock64() - t0;
      o[1] = nsteps;
      o[2] = npush;
      o[3] = nload;
    }
  }
}

// The same traces without the DFS (spf_trace_reach_kernel, the default heavy
// kernel).  traceOnePath from v succeeds iff the source reaches v over links
// not yet visited (DFS completeness on the pathLinks DAG: a failed branch only
// visits links whose tail the source cannot reach, so it never cuts a path
// another branch needs).  The DFS therefore returns the GREEDY walk from the
// destination: at each node the first pathLink whose link is unvisited and
// whose tail is the source or reachable; and the links a failed branch
// visits never matter again (reachability only shrinks).  So the kernel keeps
//   cnt[v] = # pathLinks of v with a live link and a reachable tail
// (reachable = cnt > 0; initially every node of the row: cnt = length),
// walks one path per iteration (one wave, a global load per node), removes
// the path's links and propagates the nodes whose count drops to 0 along
// their out-edges (all waves, level by level).  Output identical to the DFS
// (tests/test_trace_paths_gpu.py: the literal recursion); a 16-deep DAG
// walk replaces ~15k dependent DFS steps on the fabric's slowest query.
// LDS words of the reach kernel's per-node and per-link arrays (dynamic
// LDS, sized per launch): st, dist, row [V + 1], transit and ancestor
// bitsets, removed-link bitset
__host__ __device__ inline size_t reach_lds_words(uint32_t V, uint32_t L) {
  return 3 * (size_t)V + 1 + 2 * (((size_t)V + 31) / 32) + ((size_t)L + 31) / 32;
}
constexpr size_t kRqMaxLds = 150u << 10;
constexpr uint32_t kRqThreads = 1024;

// st[v] fields: live-pathLink count (cnt), list length, next candidate index
__device__ __forceinline__ uint32_t rq_cnt(uint32_t x) { return x & 0xFFFu; }
__device__ __forceinline__ uint32_t rq_len(uint32_t x) { return (x >> 12) & 0x3FFu; }
__device__ __forceinline__ uint32_t rq_pos(uint32_t x) { return x >> 22; }

__global__ __launch_bounds__(kRqThreads) void spf_trace_reach_kernel(TraceHeavyArgs H) {
  const TraceArgs& a = H.t;
  extern __shared__ __align__(16) uint32_t rq_smem[];
  const uint32_t V = H.V;
  uint32_t* st = rq_smem;            // [V] pos << 22 | len << 12 | cnt
  uint32_t* dl = st + V;             // [V] the row's distances
  uint32_t* rp = dl + V;             // [V + 1] CSR row offsets = arena bases
  uint32_t* tr = rp + V + 1;         // [V / 32] transit bits
  uint32_t* inc = tr + (V + 31) / 32; // [V / 32] the destination's ancestors
  uint32_t* rm = inc + (V + 31) / 32; // [L / 32] removed (ignored or found) links
  __shared__ uint32_t lnk[kTcDepth];   // the walk's links, destination first
  __shared__ uint32_t wnode[kTcDepth]; // the walk's nodes (heads of lnk)
  __shared__ uint32_t sh_len, sh_flag, sh_fn[2];
  const uint32_t tid = threadIdx.x, lane = tid & 63u, wv = tid >> 6;
  constexpr uint32_t nw = kRqThreads / 64;
  const uint32_t hi = blockIdx.x;
  const uint32_t q = H.hq[hi];
  const uint32_t s = a.src[q], d = a.dst[q];
  const uint32_t* dist = a.dist + (size_t)q * a.Vp;
  const uint32_t* lenq = H.len + (size_t)hi * V;
  const uint2* ar = H.arena + (size_t)hi * H.E;
  const uint32_t ilo = a.ign_off ? a.ign_off[q] : 0u;
  const uint32_t nign = a.ign_off ? a.ign_off[q + 1] - ilo : 0u;
  // frontiers in global scratch: a node enters each BFS at most once, so V
  // slots per level never overflow (a fabric level of RSWs can be thousands)
  uint32_t* fq[2] = {H.fq + (size_t)hi * 2 * V, H.fq + (size_t)hi * 2 * V + V};
  const uint64_t t0 = H.hstat ? wall_clock64() : 0ull;
  uint32_t nwalk = 0, ncas = 0;
  if (tid == 0) {
    sh_flag = 0;
  }
  bool bad = false;
  for (uint32_t v = tid; v < V; v += kRqThreads) {
    const uint32_t n = lenq[v];
    bad = bad || n == kInf32;
    st[v] = n == kInf32 ? 0u : (n << 12) | n;
    dl[v] = dist[v];
    rp[v] = a.row[v];
  }
  if (tid == 0) {
    rp[V] = a.row[V];
  }
  for (uint32_t i = tid; i < (V + 31) / 32; i += kRqThreads) {
    tr[i] = a.trbits[i];
    inc[i] = 0u;
  }
  for (uint32_t i = tid; i < (H.L + 31) / 32; i += kRqThreads) {
    rm[i] = 0u;
  }
  __syncthreads();
  if (bad) {
    sh_flag = 1; // a list over kTcSort entries: traced on the host
  }
  // ignored links never tighten a pathLink: removed from the start (the
  // cascade's edge test then needs no ignore-list lookup)
  for (uint32_t i = tid; i < nign; i += kRqThreads) {
    const uint32_t l = a.ign[ilo + i];
    if (l < H.L) {
      atomicOr(&rm[l >> 5], 1u << (l & 31));
    }
  }
  // the walk only visits ancestors of d in the pathLinks DAG, and a node
  // outside that set never feeds one inside (its out-neighbours are outside
  // too): counts are kept, and cascades followed, on the ancestors only
  if (tid == 0) {
    inc[d >> 5] |= 1u << (d & 31);
    fq[0][0] = d;
    sh_fn[0] = 1;
  }
  __syncthreads();
  const uint32_t sub = lane >> 4, sl = lane & 15u; // 4 nodes per wave, 16 lanes each
  if (sh_flag == 0 && s != d && dl[d] != kInf32) {
    uint32_t cur = 0;
    for (;;) {
      const uint32_t fn = sh_fn[cur];
      if (fn == 0) {
        break;
      }
      __syncthreads();
      if (tid == 0) {
        sh_fn[cur ^ 1] = 0;
      }
      __syncthreads();
      for (uint32_t i = wv * 4 + sub; i < fn; i += nw * 4) {
        const uint32_t v = fq[cur][i];
        const uint32_t n = rq_len(st[v]), base = rp[v];
        for (uint32_t j = sl; j < n; j += 16) {
          const uint32_t u = ar[base + j].x;
          if (u != s && !(atomicOr(&inc[u >> 5], 1u << (u & 31)) & (1u << (u & 31)))) {
            fq[cur ^ 1][atomicAdd(&sh_fn[cur ^ 1], 1u)] = u;
          }
        }
      }
      __syncthreads();
      cur ^= 1;
    }
  }
  __syncthreads();
  bool overflow = sh_flag != 0;
  uint32_t* out_links = a.out_links + (size_t)q * a.cap;
  uint32_t* out_ends = a.out_ends + (size_t)q * a.cap;
  uint32_t npaths = 0, nl = 0;
  auto removed = [&](uint32_t l) { return (rm[l >> 5] >> (l & 31)) & 1u; };
  if (!overflow && s != d && dl[d] != kInf32) {
    for (;;) { // one traceOnePath per iteration
      if (rq_cnt(st[d]) == 0) {
        break; // the destination is no longer reachable: the trace fails
      }
      // the walk (wave 0): the first live pathLink with a reachable tail
      if (wv == 0) {
        uint32_t v = d, h = 0;
        bool ovf = false;
        for (;;) {
          if (++nwalk > H.budget) {
            ovf = true;
            break;
          }
          const uint32_t x = st[v];
          const uint32_t n = rq_len(x), base = rp[v];
          uint32_t p = rq_pos(x);
          uint32_t f = kInf32;
          uint2 ent = make_uint2(kInf32, 0u);
          for (; p < n; p += 64) {
            const uint32_t idx = p + lane;
            ent = idx < n ? ar[base + idx] : make_uint2(kInf32, 0u);
            bool ok = false;
            if (idx < n && !removed(ent.y)) {
              ok = ent.x == s || rq_cnt(st[ent.x]) != 0;
            }
            const uint64_t m = __ballot(ok);
            if (m) {
              f = (uint32_t)__builtin_ctzll(m);
              break;
            }
          }
          if (f == kInf32 || h >= kTcDepth) {
            ovf = true; // no live entry cannot happen while cnt[v] > 0
            break;
          }
          const uint32_t u = (uint32_t)__builtin_amdgcn_readlane((int)ent.x, (int)f);
          const uint32_t l = (uint32_t)__builtin_amdgcn_readlane((int)ent.y, (int)f);
          if (lane == 0) {
            // earlier entries are dead for good
            st[v] = ((p + f) << 22) | (x & 0x3FFFFFu);
            lnk[h] = l;
            wnode[h] = v;
          }
          ++h;
          if (u == s) {
            break;
          }
          v = u;
        }
        if (lane == 0) {
          sh_len = h;
          if (ovf) {
            sh_flag = 1;
          }
        }
      }
      __syncthreads();
      if (sh_flag) {
        overflow = true;
        break;
      }
      const uint32_t len = sh_len;
      if (nl + len > a.cap || npaths + 1 > a.cap) {
        overflow = true;
        break;
      }
      // the path out (source first), then its links removed: each head
      // loses one reachable pathLink; heads left with none start the cascade
      for (uint32_t i = tid; i < len; i += kRqThreads) {
        out_links[nl + i] = lnk[len - 1 - i];
      }
      nl += len;
      if (tid == 0) {
        out_ends[npaths] = nl;
        sh_fn[0] = 0;
      }
      ++npaths;
      __syncthreads();
      for (uint32_t i = tid; i < len; i += kRqThreads) {
        const uint32_t l = lnk[i], v = wnode[i];
        atomicOr(&rm[l >> 5], 1u << (l & 31));
        if (rq_cnt(atomicSub(&st[v], 1u)) == 1u) {
          fq[0][atomicAdd(&sh_fn[0], 1u)] = v;
        }
      }
      __syncthreads();
      // cascade, level by level: a node that lost its last reachable
      // pathLink takes the support it gave its out-neighbours' lists
      uint32_t cur = 0;
      for (;;) {
        const uint32_t fn = sh_fn[cur];
        if (fn == 0) {
          break;
        }
        __syncthreads();
        if (tid == 0) {
          sh_fn[cur ^ 1] = 0;
        }
        __syncthreads();
        for (uint32_t i = wv * 4 + sub; i < fn; i += nw * 4) {
          ++ncas;
          const uint32_t v = fq[cur][i];
          if (v != s && !((tr[v >> 5] >> (v & 31)) & 1u)) {
            continue; // not transit: the tail of no pathLink
          }
          const uint32_t dv = dl[v];
          const uint32_t e1 = rp[v + 1];
          for (uint32_t e = rp[v] + sl; e < e1; e += 16) {
            const uint32_t w = a.col[e], l = a.link[e];
            const uint64_t wt = a.unit ? 1ull : (uint64_t)a.wout[e];
            if (((inc[w >> 5] >> (w & 31)) & 1u) && (uint64_t)dv + wt == dl[w] && !removed(l)) {
              if (rq_cnt(atomicSub(&st[w], 1u)) == 1u) {
                fq[cur ^ 1][atomicAdd(&sh_fn[cur ^ 1], 1u)] = w;
              }
            }
          }
        }
        __syncthreads();
        cur ^= 1;
      }
      __syncthreads();
    }
  }
  if (tid == 0) {
    a.out_n[q] = overflow ? kTraceOverflow : npaths;
    a.out_len[q] = overflow ? 0u : nl;
    if (H.hstat) {
      unsigned long long* o = H.hstat + 4 * (size_t)hi;
      o[0] = wall_clock64() - t0;
      o[1] = nwalk;
      o[2] = npaths;
      o[3] = ncas;
    }
  }
}

struct TracePackArgs {
  const uint32_t* out_n;
  const uint32_t* out_len;
  const uint32_t* links;
  const uint32_t* ends;
  const uint32_t* off_links;
  const uint32_t* off_ends;
  uint32_t* dst_links;
  uint32_t* dst_ends;
  uint32_t cap;
  uint32_t nq;
};

// trace scratch [nq][cap] -> packed arrays (offsets from the host scan)
__global__ __launch_bounds__(64) void spf_trace_pack_kernel(TracePackArgs a) {
  const uint32_t q = blockIdx.x;
  const uint32_t n = a.out_n[q];
  if (n == kTraceOverflow) {
    return;
  }
  const uint32_t len = a.out_len[q];
  for (uint32_t i = threadIdx.x; i < len; i += 64) {
    a.dst_links[a.off_links[q] + i] = a.links[(size_t)q * a.cap + i];
  }
  for (uint32_t i = threadIdx.x; i < n; i += 64) {
    a.dst_ends[a.off_ends[q] + i] = a.ends[(size_t)q * a.cap + i];
  }
}

constexpr int kPatch32 = 6; // wout, win, nbr_w, cw, col, sell (u32 words)
struct PatchArgs {
  const uint32_t* pk;   // (index, value) pairs per u32 array, then (index, lo, hi)
  uint32_t* dst32[kPatch32];
  uint32_t n32[kPatch32];
  uint32_t off32[kPatch32];
  uint64_t* dst64;
  uint32_t n64;
  uint32_t off64;
};

// scatter of a metric patch's words (spf_graph_patch_metrics, sparse path)
__global__ void spf_patch_words_kernel(PatchArgs a) {
  for (int k = 0; k < kPatch32; ++k) {
    for (uint32_t i = threadIdx.x; i < a.n32[k]; i += blockDim.x) {
      const uint32_t* p = a.pk + a.off32[k] + 2 * i;
      a.dst32[k][p[0]] = p[1];
    }
  }
  for (uint32_t i = threadIdx.x; i < a.n64; i += blockDim.x) {
    const uint32_t* p = a.pk + a.off64 + 3 * i;
    a.dst64[p[0]] = ((uint64_t)p[2] << 32) | p[1];
  }
}

__global__ void fill_u32_kernel(uint32_t* p, size_t n, uint32_t v) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  size_t stride = (size_t)gridDim.x * blockDim.x;
  for (; i < n; i += stride) {
    p[i] = v;
  }
}

} // namespace

// ==================================================================== host side

struct spf_graph {
  int device = 0;
  hipStream_t own_stream = nullptr;
  hipStream_t stream = nullptr;
  uint32_t V = 0, E = 0, L = 0, nbw = 0;
  bool exact = false;     // metric runs need 64-bit rows (wide or literal plan)
  bool wrap = false;      // a metric above 2^31-1 (negative i32): literal replay
  uint32_t n_zero = 0;    // half-edges with metric 0 (wide plan plateaus)
  uint32_t uniform = 0;   // every metric equals this value (0 = mixed)
  uint32_t G = 8;
  int num_cus = 256;
  // host copies
  std::vector<uint32_t> row, col, link, rev, slot, nbr_off, nbrs, nbr_w, trbits;
  std::vector<uint64_t> w64;
  // device copies
  uint32_t *d_row = nullptr, *d_col = nullptr, *d_wout = nullptr,
           *d_win = nullptr, *d_link = nullptr, *d_rev = nullptr,
           *d_slot = nullptr, *d_tr = nullptr, *d_nbr_off = nullptr,
           *d_nbrs = nullptr, *d_nbr_w = nullptr;
  uint64_t* d_w64 = nullptr;
  uint32_t* d_link_half = nullptr; // [2L] half-edges of each link (what-if screen)
  uint32_t* d_zero_e = nullptr;    // [n_zero] half-edges with metric 0
  uint64_t wide_delta = 1;         // wide plan band width (mean metric)
  // out-edges packed as head | metric << cw_bits (one u32 per edge) when
  // both fit; cw_bits = 0: not packed
  uint32_t* d_cw = nullptr;
  uint32_t cw_bits = 0;
  uint64_t ecc_est = 0; // graph_ecc cache (0 = not computed)
  uint64_t maxw = 0;       // largest metric (refresh_exact)
  bool hop_bounded = false; // 32-bit rows justified by transit_hop_bound
  // sliced-ELL CSR for the MS-BFS pull (MsBfsArgs::sell4), V <= 16 Ki only
  uint4* d_sell = nullptr;
  uint32_t* d_sell_off = nullptr;
  std::vector<uint32_t> sell_off; // host copy (spf_graph_set_edges patches entries)
  // spf_graph_set_edges: half-edges taken down in place are self-loops of
  // their tail (col_orig keeps the head); next-hop queries are refused on
  // such a graph (the distinct-neighbour lists still hold the old heads)
  std::vector<uint32_t> col_orig;
  std::vector<uint8_t> edge_up;
  bool links_patched = false;
  // every up half-edge's reverse is up (false only after spf_graph_set_edges
  // took one half of a link down): kernels that read a node's out-edges as
  // its in-edges (the what-if source-link kernels, the v2 pass's 2-bit rows)
  // need it
  bool paired = true;
  size_t nbr_cap = 0; // entries of d_nbrs / d_nbr_w (set_edges re-sizes them)
  // allocated entries of the edge-sized device arrays (d_col, d_link, d_rev,
  // d_slot; d_wout, d_win, d_w64; d_cw) and of d_link_half: spf_graph_update
  // rebuilds in place and reallocates only what outgrew its buffer
  size_t cap_e = 0, cap_w = 0, cap_cw = 0, cap_half = 0;
  // host scratch of the preparation passes, kept for in-place rebuilds
  std::vector<uint32_t> scratch_e, scratch_v, scratch_slot;
  // spf_graph_update: the CSR and neighbour lists it replaced (reused rows)
  std::vector<uint32_t> old_row, old_col, old_nbr_off, old_nbrs, old_slot;
  size_t cap_sell = 0, cap_sell_off = 0;
  // pinned staging of the preparation uploads (g_stage): one DMA per array
  // on the graph stream instead of a pageable synchronous hipMemcpy each
  char* pin = nullptr;
  size_t pin_cap = 0, pin_off = 0;
  // spf_table_repair's delta block + per-workgroup queues, kept between
  // calls (a 100k-node graph needs 200 MB: allocating it per churn event
  // cost more than the screen)
  char* d_repair = nullptr;
  size_t repair_bytes = 0;
  // live spf_query handles over this graph (their own base / zfix sub-queries
  // included): spf_graph_destroy refuses while any is alive, since a query
  // reads g->device / g->stream / the device CSR until it is destroyed
  std::atomic<uint32_t> live_queries{0};
  // bumped whenever the distinct-neighbour lists are rebuilt (creation,
  // spf_graph_set_edges): per-query tables built from them (the v2 next-hop
  // pass) are stale after a change
  uint64_t nbr_gen = 0;
};

// How a batch is computed.
enum class DistPlan { SsspLds, SsspGmem, BfsLds, BfsGmem, MsBfs, Dstep, MsDstep, Wide, Exact };
enum class NhPlan { None, Inline, Rows, Levels };

struct spf_query {
  spf_graph* g = nullptr;
  uint32_t nq = 0, flags = 0;
  uint32_t nrows = 0; // distance / level rows computed: nq + MS-BFS helper sources
  DistPlan dist = DistPlan::SsspLds;
  NhPlan nh = NhPlan::None;
  int wmax = 0;
  int ms_bits = 64; // MS-BFS batch width (32 or 64 sources per workgroup)
  // MS-BFS over queries with ignore lists (KSP2 second passes): per-batch
  // masks of ignored half-edges and flags of the rows holding one
  bool ms_ign = false;
  uint64_t* d_ms_mask = nullptr;
  uint32_t* d_ms_flag = nullptr;
  uint32_t ms_nfw = 0, ms_nbatch = 0;
  uint32_t dstep_shift = 5; // delta-stepping bucket width 2^shift
  bool dstep_lbk = false;    // bucket bytes in LDS (else from the dist row)
  uint32_t dstep_bs = 1024;  // delta-stepping workgroup size
  uint32_t dstep_fshift = 5; // bucket-byte resolution (dstep_tune)
  uint32_t dstep_noret = 0;  // relaxation mode bits (dstep_tune)
  uint32_t dstep_pack = 0;   // packed out-edges: 0 off, 1 scalar, 2 vector
  // LDS-resident rows (spf_dlds_kernel) first, the HBM-row pass only for the
  // sources whose values left the 12-bit range
  bool dlds = false;
  // what-if batch behind the screen whose tight queries start from the
  // baseline rows (spf_sssp_kernel repair mode, OPENR_SPF_WHATIF_REPAIR)
  bool repair = false;
  // what-if queries with an ignored link at their source, run by
  // spf_whatif_heavy_kernel (uniform-metric areas; d_wh_cand: pool block)
  std::vector<uint32_t> wh_cand;
  uint32_t* d_wh_cand = nullptr;
  uint8_t* d_wh_mark = nullptr;       // [nq] 1 = a candidate (the screen's skip = 3)
  uint32_t* d_wh_lstart = nullptr;    // [ncand][V + 1] level segments
  hipStream_t wh_stream = nullptr;    // the heavy kernel's stream (beside the SSSP)
  hipEvent_t wh_ev0 = nullptr, wh_ev1 = nullptr;
  hipEvent_t wh_ev2 = nullptr;        // the side stream's fork before the baseline (hop rows)
  // internal batches: launch_msbfs's stream instead of the graph's (the hop
  // rows on the what-if side stream) and the per-batch blocked node
  hipStream_t stream_override = nullptr;
  uint32_t* d_ms_blocked = nullptr;
  bool wh_pending = false;            // the graph stream still has to join wh_ev1
  bool wh_pull = false;               // spf_whatif_pull_kernel (sliced ELL, short lists)
  // the candidates the pull / heavy kernel runs (d_wh_cand); the others
  // (every ignored link at the source) go to spf_whatif_firsthop_kernel over
  // the nested batch `hop` (rows of the sources' neighbours, links of the
  // source ignored); d_fh packs fh_q, fh_h and the hop tables
  std::vector<uint32_t> wh_pull_cand;
  spf_query* hop = nullptr;
  uint32_t* d_fh = nullptr;
  uint32_t nfh = 0, nhop = 0, nhop_nodes = 0;
  uint32_t dlds_shift = 4, dlds_grid = 0;
  size_t dlds_lds = 0;
  uint32_t* d_ovf = nullptr; // [0] overflow count, [1] claim counter, [2..] list
  uint32_t ign_cap = 0, grid = 0, Vp = 0, Vp8 = 0;
  uint32_t dstep_ign_cap = 0; // the delta-stepping kernels' ignore-list words
  uint8_t* d_lvl = nullptr;
  uint32_t* d_flags = nullptr;
  uint32_t ms_par = 0; // the flag word (0 / 1) of the last MS-BFS launch
  // cooperative MS-BFS (spf_msbfs_coop_kernel): exchange buffer, barrier
  // counters, per-part flags and the error word, in one pooled block
  void* d_coop = nullptr;
  size_t coop_bytes = 0;
  uint32_t coop_p = 0; // parts per batch of the last launch (0: plain kernel)
  size_t lds_bytes = 0;
  bool has_ign = false;
  // next-hop masks.  Working layout (u64 words, nh_w[i] per node, query i at
  // word nh_off[i], nh_total words in d_nh): what the SSSP / rows / wide /
  // exact kernels read and write.  Output layout (byte-strided, nh_b[i] =
  // nh_bytes_for(neighbours) bytes per node, query i at byte nhb_off[i],
  // nhb_total bytes in d_nhb): what the ABI hands out.  The two coincide
  // (d_nhb aliases d_nh) unless some source has at most 32 neighbours
  // (`narrow`); then the SWAR next-hop kernels write d_nhb directly
  // (`nh_direct`, no working buffer) and every other plan is narrowed by
  // spf_nh_narrow_kernel after it ran.
  std::vector<uint64_t> nh_off;
  std::vector<uint32_t> nh_w;
  uint64_t nh_total = 0;
  std::vector<uint64_t> nhb_off;
  std::vector<uint32_t> nh_b;
  uint64_t nhb_total = 0;
  bool narrow = false, nh_direct = false;
  bool screen_direct = false; // the last screen wrote its copies narrowed (run_screen)
  bool nl_swar = true; // the byte-SIMD next-hop kernels (OPENR_NL_SWAR, read at creation)
  uint8_t* d_nhb = nullptr;
  uint64_t* d_nhb_off = nullptr;
  uint32_t* d_nh_b = nullptr;
  uint32_t *d_src = nullptr, *d_ign_off = nullptr, *d_ign = nullptr,
           *d_nh_w = nullptr, *d_order = nullptr, *d_scratch = nullptr;
  int32_t* d_row_of = nullptr;
  // multi-source delta-stepping: lane -> query map, node-major slab and
  // per-workgroup pend / candidate / claimed / mask arrays
  uint32_t msd_nbatch = 0;
  uint32_t *d_perm = nullptr, *d_slab = nullptr, *d_msd = nullptr;
  // what-if screen: baseline runs (one per distinct source, no ignore list)
  spf_query* base = nullptr;
  uint32_t *d_base_of = nullptr, *d_skip = nullptr;
  // spf_query_scatter_rows: destination row of every query
  uint32_t* d_scatter = nullptr;
  uint64_t* d_nh_off = nullptr;
  void* d_dist = nullptr;
  uint64_t* d_nh = nullptr;
  uint64_t* d_key = nullptr; // wide plan settle keys (SPF_F_ORDER)
  uint32_t* d_qctr = nullptr; // dstep source-claim counter
  uint32_t* d_wl = nullptr;   // repair work list (spf_whatif_worklist_kernel)
  uint32_t* d_big = nullptr;  // nh_levels: queries with more than kNsHeldMax mask words
  uint32_t* d_held_order = nullptr; // OPENR_NL_ORDER=1: XCD-contiguous held-kernel work order
  // the v2 next-hop pass (spf_nh_levels_v2_kernel, OPENR_NL_V2): solo / group
  // descriptors, members and neighbour entries in one pooled block, valid
  // while the graph's neighbour lists are those of nbr_gen
  void* d_v2 = nullptr;
  // 2-bit level rows of the v2 pass (spf_lvl_trit_kernel), nullptr = off
  uint8_t* d_trit = nullptr;
  NlV2Args v2{};
  bool has_v2 = false;
  uint64_t v2_gen = 0;
  uint32_t held_blocks = 0, held_nch = 0, held_t = 0;
  uint32_t nbig = 0;
  uint32_t nmid = 0;          // the first nmid of them have at most kNsHeldWide words
  // zero-metric plan (spf_zvar_kernel): variant tables, their closure pairs
  // (variant j: pairs [zoff[j], zoff[j+1]) of d_zl, then the links' ends at
  // pair zoff[zvars]), each source's variant, and the wide-plan run of the
  // sources with a metric-0 out-link (their first hop costs 0, outside the
  // byte rule) whose rows replace this query's rows zfix_rows
  uint32_t zvars = 0, zscale = 0, znlinks = 0;
  std::vector<uint32_t> zoff;
  uint32_t* d_zl = nullptr;
  uint8_t* d_zvar = nullptr;
  spf_query* zfix = nullptr;
  std::vector<uint32_t> zfix_rows;
  // k-th path traces (spf_query_trace_paths): device scratch and the last
  // trace's per-query path / link counts
  uint32_t* d_trace = nullptr;
  size_t trace_words = 0;
  char* d_tcs = nullptr; // spf_trace_cursor_kernel node states + arenas
  uint32_t trace_heavy = 0; // queries of the last trace call re-run by spf_trace_heavy_kernel
  size_t tcs_bytes = 0;
  uint32_t trace_n = 0, trace_cap = 0;
  uint64_t trace_links = 0, trace_paths = 0;
  std::vector<uint32_t> trace_pc, trace_lc;
  void* d_pack = nullptr;     // the batch's index arrays (one pooled block)
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  hipEvent_t evm = nullptr; // after the distance stage, before next hops
  bool ran = false;
  bool two_stage = false; // evm recorded between two kernels
  // live spf_route_table handles reading this query's rows (spf_query_destroy
  // refuses while any is alive)
  std::atomic<uint32_t> live_tables{0};
  // SPF_LAUNCH expressions of the last run (spf_query_kernels)
  std::vector<const char*> launched;
  // per-run event triples (start, after distance stage, end) of the last
  // kHist runs, for per-kernel averages over a timed loop without syncs
  static constexpr uint32_t kHist = 64;
  hipEvent_t hist[kHist][3] = {};
  bool hist_two[kHist] = {};
  uint64_t runs = 0;
};

namespace {

// Process-wide caching allocator for the per-query buffers: a RouteDb build
// creates and destroys a few small queries (the node, its LFA neighbours,
// KSP2 second passes), and hipMalloc / hipFree per buffer cost more than
// the SPFs of a small area.  Blocks are power-of-two size classes per
// device; blocks above kPoolMaxBlock (all-sources tables) and anything past
// kPoolMaxCached cached bytes go straight back to the driver.
constexpr size_t kPoolMaxBlock = 64ull << 20;
constexpr size_t kPoolMaxCached = 1ull << 30;
struct DevPool {
  std::mutex mu;
  std::unordered_map<size_t, std::vector<void*>> free;
  std::unordered_map<void*, size_t> cls; // live pool blocks -> size class
  size_t cached = 0;
};
DevPool& dev_pool() {
  static std::mutex m;
  static std::unordered_map<int, std::unique_ptr<DevPool>> pools;
  int dev = 0;
  (void)hipGetDevice(&dev);
  std::lock_guard<std::mutex> g(m);
  auto& p = pools[dev];
  if (!p) {
    p = std::make_unique<DevPool>();
  }
  return *p;
}
hipError_t pool_malloc(void** p, size_t n) {
  if (n > kPoolMaxBlock) {
    return hipMalloc(p, n);
  }
  size_t c = 256;
  while (c < n) {
    c <<= 1;
  }
  DevPool& P = dev_pool();
  {
    std::lock_guard<std::mutex> g(P.mu);
    auto& v = P.free[c];
    if (!v.empty()) {
      *p = v.back();
      v.pop_back();
      P.cached -= c;
      P.cls[*p] = c;
      return hipSuccess;
    }
  }
  const hipError_t e = hipMalloc(p, c);
  if (e == hipSuccess) {
    std::lock_guard<std::mutex> g(P.mu);
    P.cls[*p] = c;
  }
  return e;
}
// callers make sure no queued work still reads `p`
void pool_free(void* p) {
  if (!p) {
    return;
  }
  DevPool& P = dev_pool();
  {
    std::lock_guard<std::mutex> g(P.mu);
    auto it = P.cls.find(p);
    if (it != P.cls.end()) {
      const size_t c = it->second;
      P.cls.erase(it);
      if (P.cached + c <= kPoolMaxCached) {
        P.free[c].push_back(p);
        P.cached += c;
        return;
      }
    }
  }
  (void)hipFree(p);
}
// Recycled HIP events of finished queries (per device; a query records up
// to 3 + 3 * kHist of them).
std::mutex g_ev_mu;
std::unordered_map<int, std::vector<hipEvent_t>> g_ev_free;
hipError_t ev_get(hipEvent_t* e) {
  int dev = 0;
  (void)hipGetDevice(&dev);
  {
    std::lock_guard<std::mutex> g(g_ev_mu);
    auto& v = g_ev_free[dev];
    if (!v.empty()) {
      *e = v.back();
      v.pop_back();
      return hipSuccess;
    }
  }
  return hipEventCreate(e);
}
// callers make sure the event has completed (the stream was synchronised)
void ev_put(hipEvent_t e) {
  if (!e) {
    return;
  }
  int dev = 0;
  (void)hipGetDevice(&dev);
  std::lock_guard<std::mutex> g(g_ev_mu);
  auto& v = g_ev_free[dev];
  if (v.size() < 4096) {
    v.push_back(e);
    return;
  }
  (void)hipEventDestroy(e);
}

// host copy of a narrow mask row (B = 1, 2, 4 bytes per node) as one u64
// word per node (the ABI's host layout)
void widen_masks(const uint8_t* src, size_t B, size_t V, uint64_t* out) {
  for (size_t v = 0; v < V; ++v) {
    uint64_t x = 0;
    std::memcpy(&x, src + v * B, B); // little-endian: the low bytes of the word
    out[v] = x;
  }
}

template <typename T>
int dev_upload_q(T** dst, const T* src, size_t n) {
  *dst = nullptr;
  if (n == 0) {
    return SPF_OK;
  }
  HIP_TRY(pool_malloc((void**)dst, n * sizeof(T)));
  HIP_TRY(hipMemcpy(*dst, src, n * sizeof(T), hipMemcpyHostToDevice));
  return SPF_OK;
}

template <typename T>
int dev_upload(T** dst, const T* src, size_t n) {
  *dst = nullptr;
  if (n == 0) {
    return SPF_OK;
  }
  HIP_TRY(hipMalloc((void**)dst, n * sizeof(T)));
  HIP_TRY(hipMemcpy(*dst, src, n * sizeof(T), hipMemcpyHostToDevice));
  return SPF_OK;
}

// The v2 next-hop pass's tables (spf_nh_levels_v2_kernel): every source with
// at most kNsHeldMax mask words is a solo item or a member of a group of
// sources with the same short distinct-neighbour list (<= kNlGN neighbours,
// one word); entries list each solo source's / group's neighbours as
// (level-row index, node).
int build_nl_v2(spf_query* q, const uint32_t* sources, const std::vector<int32_t>& row_of) {
  const spf_graph* g = q->g;
  std::vector<NlSolo> solo;
  std::vector<NlSub> subs;
  std::vector<NlMem> mem;
  std::vector<NlEnt> ent;
  std::map<std::vector<uint32_t>, std::vector<uint32_t>> groups;
  std::vector<const std::vector<uint32_t>*> order; // groups in first-member order
  auto addEnt = [&](uint32_t s) -> uint32_t {
    const uint32_t lo = (uint32_t)ent.size();
    for (uint32_t k = g->nbr_off[s]; k < g->nbr_off[s + 1]; ++k) {
      const uint32_t f = g->nbrs[k];
      ent.push_back(NlEnt{(uint32_t)row_of[f], f});
    }
    return lo;
  };
  std::vector<uint32_t> soloQ;
  for (uint32_t i = 0; i < q->nq; ++i) {
    if (q->nh_w[i] > kNsHeldMax) {
      continue;
    }
    const uint32_t s = sources[i], n = g->nbr_off[s + 1] - g->nbr_off[s];
    for (uint32_t k = g->nbr_off[s]; k < g->nbr_off[s + 1]; ++k) {
      if (row_of.empty() || row_of[g->nbrs[k]] < 0) {
        return SPF_OK; // a neighbour without a row: keep the held kernel
      }
    }
    if (n >= 1 && n <= kNlGN && q->nh_w[i] == 1) {
      std::vector<uint32_t> key(g->nbrs.begin() + g->nbr_off[s], g->nbrs.begin() + g->nbr_off[s + 1]);
      auto [it, fresh] = groups.try_emplace(std::move(key));
      if (fresh) {
        order.push_back(&it->first);
      }
      it->second.push_back(i);
    } else {
      soloQ.push_back(i);
    }
  }
  for (const auto* key : order) {
    const auto& members = groups[*key];
    if (members.size() == 1) {
      soloQ.push_back(members[0]);
      continue;
    }
    const uint32_t s = sources[members[0]];
    const uint32_t lo = addEnt(s), n = (uint32_t)key->size();
    for (size_t m = 0; m < members.size(); m += kNlGS) {
      NlSub sb{};
      sb.m0 = (uint32_t)mem.size();
      sb.cnt = (uint32_t)std::min<size_t>(kNlGS, members.size() - m);
      sb.n = n;
      sb.lo = lo;
      sb.B = q->nh_b[members[0]];
      for (uint32_t x = 0; x < sb.cnt; ++x) {
        const uint32_t i = members[m + x];
        mem.push_back(NlMem{i, 0u, q->nhb_off[i]});
      }
      subs.push_back(sb);
    }
  }
  // heavy solo sources first: their blocks are the longest
  std::stable_sort(soloQ.begin(), soloQ.end(), [&](uint32_t x, uint32_t y) {
    const uint32_t sx = sources[x], sy = sources[y];
    return g->nbr_off[sx + 1] - g->nbr_off[sx] > g->nbr_off[sy + 1] - g->nbr_off[sy];
  });
  for (const uint32_t i : soloQ) {
    const uint32_t s = sources[i];
    NlSolo so{};
    so.q = i;
    so.n = g->nbr_off[s + 1] - g->nbr_off[s];
    so.lo = addEnt(s);
    so.B = q->nh_b[i];
    so.nhb_off = q->nhb_off[i];
    so.Wm = q->nh_w[i];
    solo.push_back(so);
  }
  const uint32_t nch = (g->V + 1023) / 1024;
  if ((uint64_t)(solo.size() + subs.size()) * nch > 0x7FFFFFFFull) {
    return SPF_OK; // the held kernel's own limit check reports it
  }
  const uint32_t vorder = std::min<uint32_t>(5, env_u32("OPENR_NL_V2_ORDER", 4));
  std::vector<uint32_t> xmap;
  if (vorder == 5 && solo.size() + subs.size() < (1u << 20) && nch <= 4096) {
    // items by neighbour class (largest neighbour id), chunk by chunk within
    // a class; cost ~ the neighbour rows a block reads plus its outputs
    struct It {
      uint32_t key, k, cost;
    };
    std::vector<It> items;
    for (uint32_t k = 0; k < solo.size(); ++k) {
      const uint32_t s = sources[solo[k].q];
      items.push_back({g->nbrs[g->nbr_off[s + 1] - 1], k, 4 + solo[k].n + 2 * solo[k].B});
    }
    for (uint32_t j = 0; j < subs.size(); ++j) {
      const NlSub& sb = subs[j];
      items.push_back({ent[sb.lo + sb.n - 1].node, (uint32_t)solo.size() + j, 4 + sb.n + 2 * sb.cnt});
    }
    std::stable_sort(items.begin(), items.end(), [](const It& x, const It& y) { return x.key < y.key; });
    std::vector<uint32_t> blocks;
    std::vector<uint64_t> cost;
    for (size_t i = 0; i < items.size();) {
      size_t j = i;
      while (j < items.size() && items[j].key == items[i].key) {
        ++j;
      }
      for (uint32_t c = 0; c < nch; ++c) {
        for (size_t x = i; x < j; ++x) {
          blocks.push_back(items[x].k << 12 | c);
          cost.push_back(items[x].cost);
        }
      }
      i = j;
    }
    uint64_t total = 0;
    for (uint64_t c : cost) {
      total += c;
    }
    std::vector<std::vector<uint32_t>> rng(8);
    uint64_t acc = 0;
    for (size_t i = 0; i < blocks.size(); ++i) {
      const uint32_t x = (uint32_t)std::min<uint64_t>(7, acc * 8 / std::max<uint64_t>(total, 1));
      rng[x].push_back(blocks[i]);
      acc += cost[i];
    }
    size_t mx = 0;
    for (const auto& r : rng) {
      mx = std::max(mx, r.size());
    }
    xmap.assign(8 * mx, kInf32);
    for (uint32_t x = 0; x < 8; ++x) {
      for (size_t j = 0; j < rng[x].size(); ++j) {
        xmap[8 * j + x] = rng[x][j];
      }
    }
  }
  const uint64_t lvl_bytes = (uint64_t)q->nrows * q->Vp8;
  if (lvl_bytes >= 0x80000000ull) {
    return SPF_OK; // beyond one buffer descriptor: the held kernel
  }
  // the kernel reads entries and members by whole groups of 8 / 16 / GS with
  // scalar loads: zero padding past the ends
  ent.resize(ent.size() + 64, NlEnt{0u, 0u});
  mem.resize(mem.size() + kNlGS, NlMem{0u, 0u, 0ull});
  auto al = [](size_t x) { return (x + 15) & ~(size_t)15; };
  const size_t o_solo = 0, o_sub = al(o_solo + solo.size() * sizeof(NlSolo)),
               o_mem = al(o_sub + subs.size() * sizeof(NlSub)),
               o_ent = al(o_mem + mem.size() * sizeof(NlMem)),
               o_map = al(o_ent + ent.size() * sizeof(NlEnt)),
               total = al(o_map + xmap.size() * 4);
  std::vector<uint8_t> host(total, 0);
  std::memcpy(host.data() + o_map, xmap.data(), xmap.size() * 4);
  std::memcpy(host.data() + o_solo, solo.data(), solo.size() * sizeof(NlSolo));
  std::memcpy(host.data() + o_sub, subs.data(), subs.size() * sizeof(NlSub));
  std::memcpy(host.data() + o_mem, mem.data(), mem.size() * sizeof(NlMem));
  std::memcpy(host.data() + o_ent, ent.data(), ent.size() * sizeof(NlEnt));
  if (pool_malloc(&q->d_v2, total) != hipSuccess ||
      hipMemcpy(q->d_v2, host.data(), total, hipMemcpyHostToDevice) != hipSuccess) {
    return fail(SPF_E_NOMEM, "v2 next-hop tables");
  }
  uint8_t* b = static_cast<uint8_t*>(q->d_v2);
  q->v2.solo = reinterpret_cast<const NlSolo*>(b + o_solo);
  q->v2.subs = reinterpret_cast<const NlSub*>(b + o_sub);
  q->v2.mem = reinterpret_cast<const NlMem*>(b + o_mem);
  q->v2.ent = reinterpret_cast<const NlEnt*>(b + o_ent);
  q->v2.nsolo = (uint32_t)solo.size();
  q->v2.nsub = (uint32_t)subs.size();
  q->v2.lvl_bytes = (uint32_t)lvl_bytes;
  q->v2.dbg = env_u32("OPENR_NL_V2_DBG", 0);
  q->v2.shallow = env_flag("OPENR_NL_SHALLOW", 1) ? 1u : 0u;
  // item-major (4): measured fastest with the LDS-staged wide tiles
  // (profiles/r05k: 0.364 ms against 0.385-0.389 for the chunk-major orders)
  q->v2.order = vorder == 5 && xmap.empty() ? 4u : vorder;
  q->v2.xmap = reinterpret_cast<const uint32_t*>(b + o_map);
  q->v2.nmap = (uint32_t)xmap.size();
  // 2-bit neighbour rows (OPENR_NL_TRIT=1, opt-in): exact when every
  // half-edge is paired with an up reverse (uniform metric is the plan's
  // own condition), checked here since spf_graph_set_edges bumps nbr_gen and
  // retires these tables; the per-item transit test runs in the kernel
  const bool paired = g->paired;
  const uint64_t trit_bytes = (uint64_t)q->nrows * (q->Vp8 / 4);
  // opt-in: same-process A/B on the fabric (profiles/r06c): v2 0.338 vs
  // 0.322 ms per launch plus 0.028 ms for the pack kernel -- the pass is
  // bound by its dependent load chains, not by the bytes the rows move
  if (paired && env_flag("OPENR_NL_TRIT", 0) && trit_bytes < 0x80000000ull) {
    if (pool_malloc((void**)&q->d_trit, trit_bytes) != hipSuccess) {
      return fail(SPF_E_NOMEM, "2-bit level rows");
    }
    q->v2.trit = q->d_trit;
    q->v2.trit_bytes = (uint32_t)trit_bytes;
    q->v2.tstride = q->Vp8 / 4;
  }
  q->has_v2 = true;
  q->v2_gen = g->nbr_gen;
  return SPF_OK;
}

// the 2-bit rows of every level row, before the v2 pass reads them
int launch_lvl_trits(spf_query* q) {
  spf_graph* g = q->g;
  if (!q->d_trit || !q->has_v2 || q->v2_gen != g->nbr_gen) {
    return SPF_OK;
  }
  LvlTritArgs t{};
  t.lvl = q->d_lvl;
  t.trit = q->d_trit;
  t.flags = q->d_flags ? q->d_flags + q->ms_par : nullptr;
  t.Vp8 = q->Vp8;
  t.nrows = q->nrows;
  t.per_row = q->Vp8 / 16;
  const uint64_t threads = (uint64_t)t.nrows * t.per_row;
  const uint64_t blocks = (threads + 255) / 256;
  if (blocks > 0x7FFFFFFFull) {
    return fail(SPF_E_UNSUPPORTED, "batch too large for the 2-bit level rows");
  }
  SPF_LAUNCH(spf_lvl_trit_kernel, dim3((uint32_t)blocks), dim3(256), 0, g->stream, t);
  HIP_TRY(hipGetLastError());
  return SPF_OK;
}

// ---- graph preparation on the device (spf_graph_create / _update) ----
// The raw CSR goes up once; the arrays derived from it per edge are built
// here instead of on the host and uploaded (a link flap's rebuild spent
// ~0.8 ms of host passes and 4 MB of staging on them, profiles/r05aj).
struct DeriveArgs {
  const uint32_t* col;
  const uint32_t* rev;
  const uint32_t* link;
  const uint64_t* w64;
  uint32_t* wout;      // min(w64[e], 2^32 - 1)
  uint32_t* win;       // wout of the reverse half-edge
  uint32_t* cw;        // col | wout << cw_bits (nullptr: not packed); [E4], zero tail
  uint32_t* link_half; // [2L] half-edges of each link (pre-filled with ~0)
  uint32_t E, E4, cw_bits;
};

__global__ __launch_bounds__(256) void spf_graph_derive_kernel(DeriveArgs a) {
  const uint32_t e = blockIdx.x * 256 + threadIdx.x;
  if (e >= a.E4) {
    return;
  }
  if (e >= a.E) {
    if (a.cw) {
      a.cw[e] = 0u; // padding of the last 16-byte chunk
    }
    return;
  }
  const uint32_t r = a.rev[e];
  const uint32_t wo = (uint32_t)min(a.w64[e], (uint64_t)0xFFFFFFFFull);
  a.wout[e] = wo;
  a.win[e] = (uint32_t)min(a.w64[r], (uint64_t)0xFFFFFFFFull);
  if (a.cw) {
    a.cw[e] = a.col[e] | (wo << a.cw_bits);
  }
  a.link_half[2 * (size_t)a.link[e] + (e < r ? 0 : 1)] = e;
}

// The sliced-ELL copy (layout at upload_sell): one thread per word.
struct SellArgs {
  const uint32_t* row;
  const uint32_t* col;
  const uint32_t* sell_off; // [ns + 1] in 64-uint4 groups
  uint32_t* sell;           // [sell_off[ns] * 256]
  uint32_t V, ns, words;
};

__global__ __launch_bounds__(256) void spf_sell_kernel(SellArgs a) {
  const uint32_t w = blockIdx.x * 256 + threadIdx.x;
  if (w >= a.words) {
    return;
  }
  const uint32_t grp = w >> 8, L = (w >> 2) & 63u;
  // the slice holding this group (sell_off is ascending)
  uint32_t lo = 0, hi = a.ns;
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (a.sell_off[mid] <= grp) {
      lo = mid;
    } else {
      hi = mid;
    }
  }
  const uint32_t c = lo, j = (grp - a.sell_off[c]) * 4 + (w & 3u);
  const uint32_t v = 64 * c + L;
  uint32_t x = v < a.V ? v : 0u; // short rows padded with the node itself
  if (v < a.V) {
    const uint32_t r0 = a.row[v];
    if (j < a.row[v + 1] - r0) {
      x = a.col[r0 + j];
    }
  }
  a.sell[w] = x;
}

// memcpy in 256 KB chunks on the host pool (a graph rebuild moves tens of MB
// through host copies: single-threaded they cost ~25 GB/s)
void par_copy(void* dst, const void* src, size_t bytes) {
  constexpr size_t kChunk = (size_t)256 << 10;
  const size_t n = (bytes + kChunk - 1) / kChunk;
  const unsigned nth = openr::hostThreads(n, 2);
  if (nth <= 1) {
    std::memcpy(dst, src, bytes);
    return;
  }
  openr::parallelFor(n, nth, [&](size_t i, unsigned) {
    const size_t o = i * kChunk;
    std::memcpy(static_cast<char*>(dst) + o, static_cast<const char*>(src) + o,
                std::min(kChunk, bytes - o));
  }, 1);
}

template <typename T>
void par_assign(std::vector<T>& v, const T* src, size_t n) {
  v.resize(n);
  par_copy(v.data(), src, n * sizeof(T));
}

// several copies in ONE parallel section (256 KB chunks of all of them): a
// section costs ~40-100 us of worker wake-ups, and a graph rebuild made ~30
// of them one array at a time (profiles/r05w linkflap.err)
struct CopyItem {
  void* dst;
  const void* src;
  size_t bytes;
};

void par_copy_many(const CopyItem* it, size_t n) {
  constexpr size_t kChunk = (size_t)256 << 10;
  std::vector<std::pair<uint32_t, size_t>> chunks; // (item, offset)
  for (size_t i = 0; i < n; ++i) {
    for (size_t o = 0; o < it[i].bytes; o += kChunk) {
      chunks.emplace_back((uint32_t)i, o);
    }
  }
  openr::parallelFor(chunks.size(), openr::hostThreads(chunks.size(), 2),
                     [&](size_t c, unsigned) {
    const CopyItem& x = it[chunks[c].first];
    const size_t o = chunks[c].second;
    std::memcpy(static_cast<char*>(x.dst) + o, static_cast<const char*>(x.src) + o,
                std::min(kChunk, x.bytes - o));
  }, 1);
}

// Host -> device upload through the graph's pinned staging buffer: the bytes
// are copied into it and one async DMA is queued on the graph stream
// (pageable hipMemcpy measured ~1-2 GB/s in a link flap's rebuild,
// profiles/r05p).  g_stage_flush waits for them.
int g_stage(spf_graph* g, void* dst, const void* src, size_t bytes) {
  if (!bytes) {
    return SPF_OK;
  }
  const size_t need = (bytes + 255) & ~(size_t)255;
  if (g->pin_off + need > g->pin_cap) {
    HIP_TRY(hipStreamSynchronize(g->stream)); // queued copies read the buffer
    g->pin_off = 0;
    if (need > g->pin_cap) {
      if (g->pin) {
        (void)hipHostFree(g->pin);
      }
      g->pin = nullptr;
      g->pin_cap = 0;
      const size_t c = std::max<size_t>(need, (size_t)16 << 20);
      if (hipHostMalloc((void**)&g->pin, c, hipHostMallocDefault) != hipSuccess) {
        g->pin = nullptr;
        (void)hipGetLastError();
        HIP_TRY(hipMemcpy(dst, src, bytes, hipMemcpyHostToDevice)); // unpinned fallback
        return SPF_OK;
      }
      g->pin_cap = c;
    }
  }
  par_copy(g->pin + g->pin_off, src, bytes);
  HIP_TRY(hipMemcpyAsync(dst, g->pin + g->pin_off, bytes, hipMemcpyHostToDevice, g->stream));
  g->pin_off += need;
  return SPF_OK;
}

// g_stage of several arrays with one parallel staging copy (they must fit
// the pinned buffer together, else one by one)
int g_stage_many(spf_graph* g, std::initializer_list<CopyItem> items) {
  size_t need = 0;
  for (const CopyItem& x : items) {
    need += (x.bytes + 255) & ~(size_t)255;
  }
  if (g->pin_off + need > g->pin_cap) {
    HIP_TRY(hipStreamSynchronize(g->stream)); // queued copies read the buffer
    g->pin_off = 0;
  }
  if (need > g->pin_cap) {
    for (const CopyItem& x : items) {
      if (const int s = g_stage(g, x.dst, x.src, x.bytes)) {
        return s;
      }
    }
    return SPF_OK;
  }
  std::vector<CopyItem> host;
  std::vector<size_t> off;
  for (const CopyItem& x : items) {
    if (x.bytes) {
      off.push_back(g->pin_off);
      host.push_back({g->pin + g->pin_off, x.src, x.bytes});
      g->pin_off += (x.bytes + 255) & ~(size_t)255;
    }
  }
  par_copy_many(host.data(), host.size());
  size_t i = 0;
  for (const CopyItem& x : items) {
    if (x.bytes) {
      HIP_TRY(hipMemcpyAsync(x.dst, g->pin + off[i++], x.bytes, hipMemcpyHostToDevice,
                             g->stream));
    }
  }
  return SPF_OK;
}

int g_stage_flush(spf_graph* g) {
  HIP_TRY(hipStreamSynchronize(g->stream));
  g->pin_off = 0;
  return SPF_OK;
}

template <typename T>
int dev_upload_g(spf_graph* g, T** dst, const T* src, size_t n) {
  *dst = nullptr;
  if (n == 0) {
    return SPF_OK;
  }
  HIP_TRY(hipMalloc((void**)dst, n * sizeof(T)));
  return g_stage(g, *dst, src, n * sizeof(T));
}

// OPENR_SPF_CREATE_TIMING=1: phase times of spf_graph_create / _update on
// stderr (measurement); mark("phase") closes the phase that ends there
struct PhaseTimer {
  const char* who;
  bool on;
  std::vector<std::pair<const char*, std::chrono::steady_clock::time_point>> m;
  explicit PhaseTimer(const char* w) : who(w), on(env_flag("OPENR_SPF_CREATE_TIMING", 0)) {
    (*this)("start");
  }
  void operator()(const char* what) {
    if (on) {
      m.emplace_back(what, std::chrono::steady_clock::now());
    }
  }
  ~PhaseTimer() {
    for (size_t i = 1; i < m.size(); ++i) {
      std::fprintf(stderr, "[%s] %-12s %8.3f ms\n", who, m[i].first,
                   std::chrono::duration<double, std::milli>(m[i].second - m[i - 1].second).count());
    }
  }
};

// the running create / update's timer (upload_weights marks its sub-phases)
thread_local PhaseTimer* tl_phase = nullptr;

// spf_graph_create / spf_graph_update: the CSR arrays are present and every
// half-edge has a consistent reverse (node blocks on the host pool; the lowest
// bad edge is reported)
int validate_graph_desc(const spf_graph_desc* desc) {
  const uint32_t V = desc->num_nodes, E = desc->num_edges;
  if (!desc->row_ptr || (E && (!desc->col || !desc->metric ||
                               !desc->link_id || !desc->rev)) ||
      (V && !desc->node_overloaded)) {
    return fail(SPF_E_INVALID, "missing graph array");
  }
  if (desc->row_ptr[0] != 0 || desc->row_ptr[V] != E) {
    return fail(SPF_E_INVALID, "row_ptr does not span [0, E]");
  }
  for (uint32_t u = 0; u < V; ++u) {
    if (desc->row_ptr[u + 1] < desc->row_ptr[u]) {
      return fail(SPF_E_INVALID, "row_ptr not monotone");
    }
  }
  {
    // half-edge consistency, node blocks on the host pool; the lowest bad
    // edge is reported (same message as a sequential scan)
    std::atomic<uint32_t> bad{kInf32};
    const unsigned nth = openr::hostThreads(E, kHostMinEdges);
    const std::vector<uint32_t> blk = host_node_blocks(desc->row_ptr, V, nth);
    openr::parallelFor(blk.size() - 1, nth, [&](size_t b, unsigned) {
      for (uint32_t u = blk[b]; u < blk[b + 1]; ++u) {
        for (uint32_t e = desc->row_ptr[u]; e < desc->row_ptr[u + 1]; ++e) {
          const uint32_t v = desc->col[e], r = desc->rev[e];
          if (v >= V || v == u || r >= E || desc->rev[r] != e ||
              desc->col[r] != u || desc->link_id[e] >= desc->num_links ||
              desc->link_id[r] != desc->link_id[e]) {
            uint32_t cur = bad.load();
            while (e < cur && !bad.compare_exchange_weak(cur, e)) {
            }
            return;
          }
        }
      }
    }, 1);
    if (bad.load() != kInf32) {
      return fail(SPF_E_INVALID, "inconsistent half-edge at " +
                                     std::to_string(bad.load()));
    }
  }
  return SPF_OK;
}

void free_graph(spf_graph* g) {
  if (!g) {
    return;
  }
  (void)hipSetDevice(g->device);
  if (g->stream) {
    (void)hipStreamSynchronize(g->stream); // staged uploads may still be in flight
  }
  for (void* p :
       {(void*)g->d_row, (void*)g->d_col, (void*)g->d_wout, (void*)g->d_win,
        (void*)g->d_link, (void*)g->d_rev, (void*)g->d_slot, (void*)g->d_tr,
        (void*)g->d_w64, (void*)g->d_nbr_off, (void*)g->d_nbrs,
        (void*)g->d_nbr_w, (void*)g->d_link_half, (void*)g->d_cw,
        (void*)g->d_zero_e, (void*)g->d_sell, (void*)g->d_sell_off, (void*)g->d_repair}) {
    if (p) {
      (void)hipFree(p);
    }
  }
  if (g->own_stream) {
    (void)hipStreamDestroy(g->own_stream);
  }
  if (g->pin) {
    (void)hipHostFree(g->pin);
  }
  delete g;
}

void free_query(spf_query* q) {
  if (!q) {
    return;
  }
  (void)hipSetDevice(q->g->device);
  // the buffers go back to the pool: nothing queued may still use them --
  // including the what-if source-link kernel on the query's own stream,
  // which the graph stream joins only once the rest of the plan launched
  // (an error return after that kernel leaves wh_pending set)
  if (q->wh_stream) {
    (void)hipStreamSynchronize(q->wh_stream);
    q->wh_pending = false;
  }
  (void)hipStreamSynchronize(q->g->stream);
  // d_src, d_ign_off, d_ign, d_nh_off, d_nh_w, d_row_of live in d_pack
  for (void* p :
       {q->d_pack, (void*)q->d_order, (void*)q->d_scratch,
        q->d_dist, (void*)q->d_nh,
        (void*)q->d_lvl, (void*)q->d_flags, (void*)q->d_perm,
        (void*)q->d_slab, (void*)q->d_msd, (void*)q->d_base_of,
        (void*)q->d_skip, (void*)q->d_key, (void*)q->d_qctr, (void*)q->d_wl, (void*)q->d_scatter,
        (void*)q->d_trace, (void*)q->d_big, (void*)q->d_held_order, (void*)q->d_zl,
        (void*)q->d_zvar, (void*)q->d_ms_mask, (void*)q->d_ms_flag,
        (void*)q->d_ovf, q->narrow ? (void*)q->d_nhb : nullptr, (void*)q->d_tcs, q->d_v2,
        (void*)q->d_trit,
        q->d_coop, (void*)q->d_wh_cand, (void*)q->d_wh_mark, (void*)q->d_wh_lstart,
        (void*)q->d_fh, (void*)q->d_ms_blocked}) {
    pool_free(p);
  }
  if (q->base) {
    free_query(q->base);
  }
  if (q->hop) {
    free_query(q->hop);
  }
  if (q->zfix) {
    free_query(q->zfix);
  }
  if (q->ev0) {
    ev_put(q->ev0);
  }
  if (q->ev1) {
    ev_put(q->ev1);
  }
  if (q->evm) {
    ev_put(q->evm);
  }
  if (q->wh_ev0) {
    ev_put(q->wh_ev0);
  }
  if (q->wh_ev1) {
    ev_put(q->wh_ev1);
  }
  if (q->wh_ev2) {
    ev_put(q->wh_ev2);
  }
  if (q->wh_stream) {
    (void)hipStreamDestroy(q->wh_stream);
  }
  for (auto& h : q->hist) {
    for (hipEvent_t e : h) {
      if (e) {
        ev_put(e);
      }
    }
  }
  q->g->live_queries.fetch_sub(1, std::memory_order_relaxed);
  delete q;
}

// Distinct neighbours per node over its UP half-edges (ascending id = name
// order) and each half-edge's slot among them (sorted unique neighbours of u
// staged in scratch[row[u] ..], counted, then packed; node blocks on the host
// pool).  A half-edge taken down in place (spf_graph_set_edges) is no
// neighbour; its slot is 0 (it is never tight, so never read).
// (reuse: the previous CSR's row / col / nbr_off / nbrs / slot, when the
// graph is rebuilt in place: a row whose heads are unchanged keeps its
// distinct-neighbour list and slots, shifted to the new offsets)
struct NbrReuse {
  const std::vector<uint32_t>* row = nullptr;
  const std::vector<uint32_t>* col = nullptr;
  const std::vector<uint32_t>* nbr_off = nullptr;
  const std::vector<uint32_t>* nbrs = nullptr;
  const std::vector<uint32_t>* slot = nullptr;
};

void build_nbr_lists(spf_graph* g, const NbrReuse* old = nullptr) {
  ++g->nbr_gen;
  const uint32_t V = g->V, E = g->E;
  const bool patched = !g->edge_up.empty();
  g->nbr_off.resize(V + 1);
  g->nbr_off[0] = 0;
  g->slot.resize(E); // every up half-edge's slot is written below
  if (patched) {
    std::fill(g->slot.begin(), g->slot.end(), 0u);
  }
  // kept between calls (a link flap rebuilds the lists; fresh vectors cost
  // their page faults every time)
  std::vector<uint32_t>& scratch = g->scratch_e;
  std::vector<uint32_t>& cnt = g->scratch_v;
  scratch.resize(E);
  cnt.resize(V);
  const unsigned nth = openr::hostThreads(E, kHostMinEdges);
  const std::vector<uint32_t> blk = host_node_blocks(g->row.data(), V, nth);
  // per worker: neighbour -> slot of the row being processed (written before
  // it is read, never cleared)
  if (g->scratch_slot.size() < (size_t)nth * V) {
    g->scratch_slot.resize((size_t)nth * V);
  }
  openr::parallelFor(blk.size() - 1, nth, [&](size_t b, unsigned w) {
    uint32_t* idx = g->scratch_slot.data() + (size_t)w * V;
    for (uint32_t u = blk[b]; u < blk[b + 1]; ++u) {
      const uint32_t e0 = g->row[u], e1 = g->row[u + 1];
      uint32_t* lo = scratch.data() + e0;
      if (old && !patched) {
        const uint32_t o0 = (*old->row)[u], o1 = (*old->row)[u + 1];
        if (o1 - o0 == e1 - e0 &&
            std::equal(g->col.begin() + e0, g->col.begin() + e1, old->col->begin() + o0)) {
          const uint32_t n0 = (*old->nbr_off)[u], n1 = (*old->nbr_off)[u + 1];
          std::copy(old->nbrs->begin() + n0, old->nbrs->begin() + n1, lo);
          std::copy(old->slot->begin() + o0, old->slot->begin() + o1, g->slot.begin() + e0);
          cnt[u] = n1 - n0;
          continue;
        }
      }
      uint32_t* hi = lo;
      bool sorted = true;
      uint32_t prev = 0;
      for (uint32_t e = e0; e < e1; ++e) {
        if (!patched || g->edge_up[e]) {
          const uint32_t c = g->col[e];
          sorted = sorted && (hi == lo || c > prev);
          prev = c;
          *hi++ = c;
        }
      }
      if (sorted && !patched) {
        // the common row: distinct neighbours already ascending
        cnt[u] = (uint32_t)(hi - lo);
        for (uint32_t e = e0; e < e1; ++e) {
          g->slot[e] = e - e0;
        }
        continue;
      }
      if (!sorted) {
        std::sort(lo, hi);
        hi = std::unique(lo, hi);
      }
      cnt[u] = (uint32_t)(hi - lo);
      for (uint32_t* p = lo; p < hi; ++p) {
        idx[*p] = (uint32_t)(p - lo);
      }
      for (uint32_t e = e0; e < e1; ++e) {
        if (!patched || g->edge_up[e]) {
          g->slot[e] = idx[g->col[e]];
        }
      }
    }
  }, 1);
  for (uint32_t u = 0; u < V; ++u) {
    g->nbr_off[u + 1] = g->nbr_off[u] + cnt[u];
  }
  g->nbrs.resize(g->nbr_off[V]);
  openr::parallelFor(blk.size() - 1, nth, [&](size_t b, unsigned) {
    for (uint32_t u = blk[b]; u < blk[b + 1]; ++u) {
      std::copy_n(scratch.data() + g->row[u], cnt[u], g->nbrs.data() + g->nbr_off[u]);
    }
  }, 1);
}

// Upper bound on the hop count of some valid path from any node to any node
// it reaches: 2 * ecc(r) for a transit hub r whose transit-only BFS (a node
// is expanded iff it is r or may be transited, LinkState.cpp:829-836)
// reaches every node.  For a source s and a node v it reaches, the BFS tree
// paths s <- r and r -> v have transit interiors and r is transit, so their
// concatenation is a walk the SPF from s may take (the source is exempt) of
// at most 2 * ecc(r) links.  0 = no such hub (no transit node, or the hub
// does not reach every node: partitioned by drained nodes).
uint64_t transit_hop_bound(const std::vector<uint32_t>& row, const std::vector<uint32_t>& col,
                           const std::vector<uint32_t>& trbits, uint32_t V) {
  auto transit = [&](uint32_t v) { return (trbits[v >> 5] >> (v & 31)) & 1u; };
  uint32_t r = kInf32, best = 0;
  for (uint32_t v = 0; v < V; ++v) {
    const uint32_t d = row[v + 1] - row[v];
    if (transit(v) && (r == kInf32 || d > best)) {
      r = v;
      best = d;
    }
  }
  if (r == kInf32) {
    return 0;
  }
  std::vector<uint32_t> lvl(V, kInf32), cur{r}, nxt;
  lvl[r] = 0;
  uint32_t reached = 1, depth = 0;
  while (!cur.empty()) {
    nxt.clear();
    for (uint32_t u : cur) {
      if (u != r && !transit(u)) {
        continue;
      }
      for (uint32_t e = row[u]; e < row[u + 1]; ++e) {
        const uint32_t v = col[e];
        if (lvl[v] == kInf32) {
          lvl[v] = depth + 1;
          nxt.push_back(v);
          ++reached;
        }
      }
    }
    if (!nxt.empty()) {
      ++depth;
    }
    cur.swap(nxt);
  }
  return reached == V ? 2ull * depth : 0;
}

// g->exact: the batch needs 64-bit rows (wide / literal plans).  A metric 0
// or a wrapping metric always does; otherwise 32-bit rows are exact when no
// distance (nor distance + one link) can reach 2^32 - 1 (kInf32): first the
// coarse maxw * (V - 1) bound, then maxw * (transit_hop_bound + 1), so a
// WAN with metrics to 10^6 keeps the 32-bit plans.  Re-run when transit bits
// change (a drain can lengthen paths).
void refresh_exact(spf_graph* g) {
  const uint32_t V = g->V;
  const uint64_t maxw = g->maxw;
  bool exact = g->wrap || g->n_zero > 0;
  g->hop_bounded = false;
  if (!exact && V > 1 && maxw > 0 &&
      (unsigned __int128)maxw * (V - 1) >= 0xFFFFFFFFull) {
    const uint64_t h = env_flag("OPENR_SPF_HOP_BOUND", 1)
                           ? transit_hop_bound(g->row, g->col, g->trbits, V)
                           : 0;
    if (h && (unsigned __int128)maxw * (h + 1) < 0xFFFFFFFFull) {
      g->hop_bounded = true;
    } else {
      exact = true;
    }
  }
  g->exact = exact;
}

// fast-path weights, exactness, uniformity and per-neighbour cheapest metric
// lanes per node of the frontier kernels (a.G): the median degree, rounded
// to a power of two in [4, 64]; spf_graph_create and spf_graph_update
void set_lanes_per_node(spf_graph* g) {
  const uint32_t V = g->V;
  std::vector<uint32_t> deg(V);
  for (uint32_t u = 0; u < V; ++u) {
    deg[u] = g->row[u + 1] - g->row[u];
  }
  uint32_t med = 4;
  if (V) {
    std::nth_element(deg.begin(), deg.begin() + V / 2, deg.end());
    med = deg[V / 2];
  }
  uint32_t G = 4;
  while (G < med && G < 64) {
    G <<= 1;
  }
  g->G = G;
}

int upload_weights(spf_graph* g) {
  const uint32_t E = g->E, V = g->V;
  const unsigned nth = openr::hostThreads(E, kHostMinEdges);
  const std::vector<uint32_t> blk = host_node_blocks(g->row.data(), V, nth);
  std::vector<uint64_t> wmax(nth, 0), wsum(nth, 0);
  std::vector<uint8_t> wwrap(nth, 0), wsame(nth, 1);
  std::vector<std::vector<uint32_t>> zeros(nth);
  const uint64_t w0 = E ? g->w64[0] : 0;
  // the packed out-edge words use ceil(log2 V) bits for the head
  uint32_t bits = 1;
  while (bits < 32 && (1ull << bits) < V) {
    ++bits;
  }
  g->nbr_w.resize(g->nbrs.size());
  const bool patched = !g->edge_up.empty();
  // ONE pass over node blocks (a parallel section costs ~40-100 us of worker
  // wake-ups): the metric scan (max, sum, wrap, uniformity, metric-0 edges)
  // and the cheapest usable link to each distinct neighbour (parallel links;
  // its host mirror serves the sparse metric patches).  The per-edge arrays
  // (wout, win, packed edges, link halves) are derived on the device
  // (spf_graph_derive_kernel).  Per-block locals, folded into the per-worker
  // slots once per block (slots of all workers share cache lines: per-edge
  // updates were ~6 ms of false sharing, profiles/r05s).
  openr::parallelFor(blk.size() - 1, nth, [&](size_t b, unsigned w) {
    uint64_t mx = 0, sm = 0;
    bool wrap = false, same = true;
    for (uint32_t u = blk[b]; u < blk[b + 1]; ++u) {
      uint32_t* nw = g->nbr_w.data() + g->nbr_off[u];
      std::fill(nw, g->nbr_w.data() + g->nbr_off[u + 1], 0xFFFFFFFFu);
      for (uint32_t e = g->row[u]; e < g->row[u + 1]; ++e) {
        const uint64_t m = g->w64[e];
        if (m > 0x7FFFFFFFull) {
          wrap = true;
        } else {
          sm += m;
        }
        if (m == 0) {
          zeros[w].push_back(e);
        }
        mx = std::max(mx, m);
        same = same && m == w0;
        if (!patched || g->edge_up[e]) { // a down half-edge is no usable link
          uint32_t& x = nw[g->slot[e]];
          x = std::min(x, (uint32_t)std::min<uint64_t>(m, 0xFFFFFFFFull));
        }
      }
    }
    wmax[w] = std::max(wmax[w], mx);
    wsum[w] += sm;
    wwrap[w] |= (uint8_t)wrap;
    wsame[w] &= (uint8_t)same;
  }, 1);
  uint64_t maxw = 0, sumw = 0;
  bool wrap = false;
  std::vector<uint32_t> zero_e;
  for (unsigned w = 0; w < nth; ++w) {
    maxw = std::max(maxw, wmax[w]);
    sumw += wsum[w];
    wrap = wrap || wwrap[w];
    zero_e.insert(zero_e.end(), zeros[w].begin(), zeros[w].end());
  }
  if (tl_phase) (*tl_phase)("w:pass");
  std::sort(zero_e.begin(), zero_e.end());
  g->wrap = wrap;
  g->n_zero = (uint32_t)zero_e.size();
  g->maxw = maxw;
  refresh_exact(g);
  const bool exact = g->exact;
  // wide plan band: the mean metric (near-far's delta ~ a typical edge)
  g->wide_delta = E ? std::max<uint64_t>(1, sumw / E) : 1;
  if (g->d_zero_e) {
    (void)hipFree(g->d_zero_e);
    g->d_zero_e = nullptr;
  }
  if (!zero_e.empty()) {
    HIP_TRY(hipMalloc((void**)&g->d_zero_e, zero_e.size() * 4));
    if (const int st = g_stage(g, g->d_zero_e, zero_e.data(), zero_e.size() * 4)) {
      return st;
    }
  }
  g->uniform = 0;
  if (!exact && E) {
    bool same = true;
    for (unsigned w = 0; w < nth; ++w) {
      same = same && wsame[w];
    }
    g->uniform = same ? (uint32_t)w0 : 0;
  }
  g->ecc_est = 0;
  // packed out-edges for the push-only delta-stepping pass
  const bool pack = E && bits < 32 && maxw < (1ull << (32 - bits));
  if (g->d_cw && !pack) {
    (void)hipFree(g->d_cw);
    g->d_cw = nullptr;
  }
  g->cw_bits = 0;
  // packed words padded to whole 16-byte chunks (the vector reads of the last one)
  const size_t e4 = ((size_t)E + 3) & ~(size_t)3;
  if (pack) {
    if (!g->d_cw || e4 > g->cap_cw) {
      if (g->d_cw) {
        (void)hipFree(g->d_cw);
        g->d_cw = nullptr;
        g->cap_cw = 0;
      }
      const size_t c = (e4 + e4 / 8 + 3) & ~(size_t)3;
      HIP_TRY(hipMalloc((void**)&g->d_cw, c * 4));
      g->cap_cw = c;
    }
    g->cw_bits = bits;
  }
  if (E) {
    if (!g->d_wout || E > g->cap_w) {
      // freed pointers are cleared at once and the capacity is 0 until all
      // three allocations succeed, so a failed allocation on a live graph
      // (spf_graph_update) leaves nothing that free_graph would free twice
      for (uint32_t** p : {&g->d_wout, &g->d_win}) {
        if (*p) {
          (void)hipFree(*p);
          *p = nullptr;
        }
      }
      if (g->d_w64) {
        (void)hipFree(g->d_w64);
        g->d_w64 = nullptr;
      }
      g->cap_w = 0;
      const size_t c = (size_t)E + E / 8; // headroom for in-place rebuilds
      HIP_TRY(hipMalloc((void**)&g->d_wout, c * 4));
      HIP_TRY(hipMalloc((void**)&g->d_win, c * 4));
      HIP_TRY(hipMalloc((void**)&g->d_w64, c * 8));
      g->cap_w = c;
    }
    if (!g->d_nbr_w || g->nbr_w.size() > g->nbr_cap) {
      // d_nbrs / d_nbr_w share nbr_cap (the caller sizes d_nbrs first)
      return fail(SPF_E_INVALID, "neighbour-weight buffer smaller than the neighbour lists");
    }
    if (const int st = g_stage_many(g, {{g->d_w64, g->w64.data(), (size_t)E * 8},
                                        {g->d_nbr_w, g->nbr_w.data(), g->nbr_w.size() * 4}})) {
      return st;
    }
  }
  // link halves: [2L], the derive kernel scatters them over a ~0 fill
  if (!g->d_link_half || 2 * (size_t)g->L > g->cap_half) {
    if (g->d_link_half) {
      (void)hipFree(g->d_link_half);
      g->d_link_half = nullptr;
    }
    const size_t c = std::max<size_t>(1, 2 * (size_t)g->L + g->L / 4);
    HIP_TRY(hipMalloc((void**)&g->d_link_half, c * 4));
    g->cap_half = c;
  }
  HIP_TRY(hipMemsetAsync(g->d_link_half, 0xFF, 2 * (size_t)g->L * 4, g->stream));
  if (E) {
    DeriveArgs da{g->d_col, g->d_rev, g->d_link, g->d_w64, g->d_wout, g->d_win,
                  pack ? g->d_cw : nullptr, g->d_link_half, E, (uint32_t)e4, g->cw_bits};
    SPF_LAUNCH(spf_graph_derive_kernel, dim3((uint32_t)((e4 + 255) / 256)), dim3(256), 0,
               g->stream, da);
    HIP_TRY(hipGetLastError());
  }
  if (tl_phase) (*tl_phase)("w:stage");
  return SPF_OK;
}

// Sliced-ELL copy of the CSR for spf_msbfs_kernel: slice c = nodes
// [64c, 64c + 64) (one wave's node slot), width = the slice's largest degree
// rounded up to 4; lane L's edge j sits in word j % 4 of the uint4 at group
// sell_off[c] + j / 4, so one wave load covers 1 KB.  Rows are padded with
// the node's own id (harmless in the pull, see MsBfsArgs).  Name ranks keep
// nodes of one role (SSW / FSW / RSW) adjacent, so the padding is small
// (fabric: 232,512 edges -> 233,472 slots).
// The sliced-ELL copy for spf_msbfs_kernel (V <= 16 Ki): slice c = nodes
// [64c, 64c + 64) (one wave's node slot), width = the slice's largest degree
// rounded up to 4; lane L's edge j sits in word j % 4 of the uint4 at group
// sell_off[c] + j / 4, so one wave load covers 1 KB.  Rows are padded with
// the node's own id (harmless in the pull, see MsBfsArgs).  Name ranks keep
// nodes of one role (SSW / FSW / RSW) adjacent, so the padding is small
// (fabric: 232,512 edges -> 233,472 slots).  The widths are a host scan;
// the words are written on the device (spf_sell_kernel) from the uploaded
// CSR.
int upload_sell(spf_graph* g) {
  const uint32_t V = g->V;
  if (!V || V > kMsThreads * kMsMaxK) {
    return SPF_OK;
  }
  const uint32_t ns = (V + 63) / 64;
  std::vector<uint32_t>& off = g->sell_off;
  off.assign(ns + 1, 0);
  for (uint32_t c = 0; c < ns; ++c) {
    uint32_t w = 0;
    for (uint32_t v = 64 * c; v < std::min(V, 64 * c + 64); ++v) {
      w = std::max(w, g->row[v + 1] - g->row[v]);
    }
    off[c + 1] = off[c] + (w + 3) / 4;
  }
  const size_t words = (size_t)off[ns] * 256;
  // device buffers kept across in-place rebuilds while they fit
  auto fit = [&](uint32_t** d, size_t n, size_t& cap) -> int {
    if (*d && n <= cap) {
      return SPF_OK;
    }
    if (*d) {
      (void)hipFree(*d);
      *d = nullptr;
    }
    cap = 0;
    const size_t c = std::max<size_t>(1, n + n / 8);
    HIP_TRY(hipMalloc((void**)d, c * 4));
    cap = c;
    return SPF_OK;
  };
  int s = fit(&g->d_sell_off, off.size(), g->cap_sell_off);
  if (s == SPF_OK) {
    s = fit((uint32_t**)&g->d_sell, words, g->cap_sell);
  }
  if (s == SPF_OK) {
    s = g_stage(g, g->d_sell_off, off.data(), off.size() * 4);
  }
  if (s == SPF_OK && words) {
    SellArgs sa{g->d_row, g->d_col, g->d_sell_off, reinterpret_cast<uint32_t*>(g->d_sell), V, ns,
                (uint32_t)words};
    SPF_LAUNCH(spf_sell_kernel, dim3((uint32_t)((words + 255) / 256)), dim3(256), 0, g->stream,
               sa);
    HIP_TRY(hipGetLastError());
  }
  return s;
}

// A few metrics changed (adjacency churn, LinkState.cpp:621-660): patch the
// host mirrors and scatter only the device words those edges feed — w64[e],
// wout[e], win[rev[e]], the cheapest-link metric of e's neighbour slot and
// the packed edge word — instead of upload_weights' full recompute and
// upload (26 ms per event on the WAN-100k, bench table_repair).  The graph
// scalars (maxw, mean metric, uniformity, exactness) come from one parallel
// scan of w64.  SPF_E_UNSUPPORTED (nothing changed) when the patch would
// change the set of metric-0 edges, the wrap flag or the packed-edge layout:
// the caller then runs upload_weights.
// graph scalars after an in-place metric / link patch: maxw, the wide-plan
// band (mean metric), uniformity and the 32-bit row bound, in one parallel
// scan of the host metrics
void rescan_scalars(spf_graph* g) {
  const uint32_t E = g->E;
  const unsigned nth = openr::hostThreads(E, kHostMinEdges);
  const size_t chunk = (E + nth - 1) / std::max(1u, nth);
  std::vector<uint64_t> wmax(nth, 0), wsum(nth, 0);
  std::vector<uint8_t> same(nth, 1);
  const uint64_t c0 = E ? g->w64[0] : 0;
  openr::parallelFor(nth, nth, [&](size_t t, unsigned) {
    const size_t lo = t * chunk, hi = std::min<size_t>(E, lo + chunk);
    uint64_t mx = 0, sm = 0;
    bool eq = true;
    for (size_t e = lo; e < hi; ++e) {
      const uint64_t w = g->w64[e];
      mx = std::max(mx, w);
      sm += w <= 0x7FFFFFFFull ? w : 0;
      eq = eq && w == c0;
    }
    wmax[t] = mx;
    wsum[t] = sm;
    same[t] = eq;
  }, 1);
  uint64_t maxw = 0, sumw = 0;
  bool uni = true;
  for (unsigned t = 0; t < nth; ++t) {
    maxw = std::max(maxw, wmax[t]);
    sumw += wsum[t];
    uni = uni && same[t];
  }
  g->maxw = maxw;
  refresh_exact(g);
  g->wide_delta = E ? std::max<uint64_t>(1, sumw / E) : 1;
  g->uniform = (!g->exact && E && uni) ? (uint32_t)c0 : 0;
}

int patch_weights_sparse(spf_graph* g, uint32_t n, const uint32_t* edge_idx, const uint64_t* m) {
  const uint32_t E = g->E;
  for (uint32_t i = 0; i < n; ++i) {
    const uint64_t o = g->w64[edge_idx[i]], w = m[i];
    if ((o == 0) != (w == 0) || (o > 0x7FFFFFFFull) != (w > 0x7FFFFFFFull)) {
      return SPF_E_UNSUPPORTED; // zero-edge list / wrap flag change
    }
    if (g->cw_bits && w >= (1ull << (32 - g->cw_bits))) {
      return SPF_E_UNSUPPORTED; // no longer packable
    }
  }
  HIP_TRY(hipStreamSynchronize(g->stream)); // queued kernels read the old words
  for (uint32_t i = 0; i < n; ++i) {
    g->w64[edge_idx[i]] = m[i];
  }
  rescan_scalars(g);
  // the device words (u32 index, u32 lo, u32 hi) per array, one upload
  std::vector<uint32_t> pk;
  uint32_t counts[5] = {0, 0, 0, 0, 0};
  std::vector<uint32_t> lists[5];
  std::vector<uint64_t> vals64;
  std::vector<uint32_t> idx64;
  for (uint32_t i = 0; i < n; ++i) {
    const uint32_t e = edge_idx[i];
    const uint64_t w = g->w64[e];
    const uint32_t w32 = (uint32_t)std::min<uint64_t>(w, 0xFFFFFFFFull);
    idx64.push_back(e);
    vals64.push_back(w);
    lists[0].push_back(e);
    lists[0].push_back(w32); // wout[e]
    lists[1].push_back(g->rev[e]);
    lists[1].push_back(w32); // win[rev[e]]
    // cheapest usable link to the neighbour of slot[e] (parallel links)
    uint32_t u = (uint32_t)(std::upper_bound(g->row.begin(), g->row.end(), e) - g->row.begin()) - 1;
    uint32_t best = 0xFFFFFFFFu;
    for (uint32_t f = g->row[u]; f < g->row[u + 1]; ++f) {
      if (g->slot[f] == g->slot[e]) {
        best = std::min<uint32_t>(best, (uint32_t)std::min<uint64_t>(g->w64[f], 0xFFFFFFFFull));
      }
    }
    const uint32_t ns = g->nbr_off[u] + g->slot[e];
    g->nbr_w[ns] = best;
    lists[2].push_back(ns);
    lists[2].push_back(best);
    if (g->cw_bits) {
      lists[3].push_back(e);
      lists[3].push_back(g->col[e] | (w32 << g->cw_bits));
    }
  }
  PatchArgs a{};
  uint32_t* arrays[4] = {g->d_wout, g->d_win, g->d_nbr_w, g->d_cw};
  size_t off = 0;
  for (int k = 4; k < kPatch32; ++k) {
    a.dst32[k] = nullptr;
    a.n32[k] = 0;
  }
  for (int k = 0; k < 4; ++k) {
    counts[k] = (uint32_t)(lists[k].size() / 2);
    a.dst32[k] = arrays[k];
    a.n32[k] = arrays[k] ? counts[k] : 0;
    a.off32[k] = (uint32_t)off;
    pk.insert(pk.end(), lists[k].begin(), lists[k].end());
    off = pk.size();
  }
  const size_t o64 = pk.size();
  for (uint32_t i = 0; i < n; ++i) {
    pk.push_back(idx64[i]);
    pk.push_back((uint32_t)vals64[i]);
    pk.push_back((uint32_t)(vals64[i] >> 32));
  }
  a.dst64 = g->d_w64;
  a.n64 = n;
  a.off64 = (uint32_t)o64;
  uint32_t* d = nullptr;
  HIP_TRY(pool_malloc((void**)&d, pk.size() * 4));
  HIP_TRY(hipMemcpyAsync(d, pk.data(), pk.size() * 4, hipMemcpyHostToDevice, g->stream));
  a.pk = d;
  SPF_LAUNCH(spf_patch_words_kernel, dim3(1), dim3(256), 0, g->stream, a);
  const hipError_t le = hipGetLastError();
  const hipError_t se = hipStreamSynchronize(g->stream); // pk is host memory too
  pool_free(d);
  HIP_TRY(le);
  HIP_TRY(se);
  g->ecc_est = 0; // dstep tuning re-estimates the eccentricity
  return SPF_OK;
}

inline size_t lds_ctl_bytes(const spf_graph* g, uint32_t ign_cap) {
  return (3 * (size_t)g->nbw + kCtlWords + ign_cap) * sizeof(uint32_t);
}

inline size_t lds_state_bytes(uint32_t V) {
  return (size_t)((V + 1) & ~1u) * 2 + (size_t)V * 4; // u16 queue + u32 dist
}

inline size_t msd_lds_bytes(const spf_graph* g) {
  return ((size_t)kCtlWords + g->nbw + kMsdK * (kMsdTile + 1) + (g->V + 3) / 4) * 4;
}

// Batches of kMsdK queries for spf_msdstep_kernel, graph-near sources
// together: from each unassigned seed, a Dijkstra truncated at `cap` settled
// nodes collects the nearest sources of unassigned queries.  Seeds whose
// search cannot fill a batch leave their queries to a tail that is packed in
// query order.  Any grouping gives the same rows; this one keeps the bucket
// fronts of a batch aligned (more useful lanes per fetched line).
std::vector<uint32_t> msd_batches(
    const spf_graph* g, const uint32_t* srcs, uint32_t nq, bool cluster) {
  std::vector<uint32_t> perm;
  perm.reserve(((size_t)nq + kMsdK - 1) / kMsdK * kMsdK);
  if (!cluster) {
    for (uint32_t i = 0; i < nq; ++i) {
      perm.push_back(i);
    }
  } else {
    const uint32_t V = g->V;
    std::vector<uint32_t> head(V + 1, 0), at(nq);
    for (uint32_t i = 0; i < nq; ++i) {
      ++head[srcs[i] + 1];
    }
    for (uint32_t v = 0; v < V; ++v) {
      head[v + 1] += head[v];
    }
    {
      std::vector<uint32_t> fill(head.begin(), head.end() - 1);
      for (uint32_t i = 0; i < nq; ++i) {
        at[fill[srcs[i]]++] = i;
      }
    }
    std::vector<uint32_t> taken(V, 0); // queries of node v already assigned
    std::vector<uint32_t> stamp(V, 0), dist(V, 0);
    std::vector<uint32_t> tail, batch;
    uint32_t epoch = 0;
    const uint32_t cap = (uint32_t)std::min<uint64_t>(
        8192, std::max<uint64_t>(256, 8ull * kMsdK * V / std::max(nq, 1u)));
    using HE = std::pair<uint64_t, uint32_t>;
    std::vector<HE> heap;
    for (uint32_t i = 0; i < nq; ++i) {
      const uint32_t s0 = srcs[i];
      if (taken[s0] == head[s0 + 1] - head[s0]) {
        continue; // every query of this source is placed
      }
      ++epoch;
      batch.clear();
      heap.clear();
      heap.push_back({0, s0});
      stamp[s0] = epoch;
      dist[s0] = 0;
      uint32_t settled = 0;
      while (!heap.empty() && batch.size() < kMsdK && settled < cap) {
        std::pop_heap(heap.begin(), heap.end(), std::greater<HE>());
        const HE top = heap.back();
        heap.pop_back();
        const uint32_t u = top.second;
        if (top.first != dist[u]) {
          continue;
        }
        ++settled;
        while (taken[u] < head[u + 1] - head[u] && batch.size() < kMsdK) {
          batch.push_back(at[head[u] + taken[u]++]);
        }
        for (uint32_t e = g->row[u]; e < g->row[u + 1]; ++e) {
          const uint32_t x = g->col[e];
          const uint32_t c = (uint32_t)std::min<uint64_t>(
              (uint64_t)dist[u] + std::max<uint64_t>(g->w64[e], 1), 0xFFFFFFFEull);
          if (stamp[x] != epoch || c < dist[x]) {
            stamp[x] = epoch;
            dist[x] = c;
            heap.push_back({c, x});
            std::push_heap(heap.begin(), heap.end(), std::greater<HE>());
          }
        }
      }
      auto& dst = batch.size() == kMsdK ? perm : tail;
      dst.insert(dst.end(), batch.begin(), batch.end());
    }
    perm.insert(perm.end(), tail.begin(), tail.end());
  }
  while (perm.size() % kMsdK) {
    perm.push_back(kInf32);
  }
  return perm;
}

// delta-stepping bucket width 2^shift: ~ mean metric / mean degree
// (delta-stepping's Delta = Theta(w/d)); push-only (distance) runs 4x wider,
// measured fastest; OPENR_SPF_DSTEP_SHIFT overrides
uint32_t dstep_bucket_shift(const spf_graph* g, bool want_nh) {
  uint64_t wsum = 0;
  for (uint32_t e = 0; e < g->E; ++e) {
    wsum += std::min<uint64_t>(g->w64[e], 0xFFFFFFFFull);
  }
  const double meanw = g->E ? (double)wsum / g->E : 1.0;
  const double meandeg = g->V ? (double)g->E / g->V : 1.0;
  uint32_t shift = 0;
  while (shift < 20 && (double)(2u << shift) <= meanw / std::max(meandeg, 1.0)) {
    ++shift;
  }
  if (!want_nh) {
    shift += 2;
  }
  if (const char* env = getenv("OPENR_SPF_DSTEP_SHIFT")) {
    shift = (uint32_t)std::min(24, std::max(0, atoi(env)));
  }
  return shift;
}

// Largest distance from one node (host Dijkstra over the 64-bit metrics),
// cached per graph: sizes the bucket-byte resolution of the push-only
// delta-stepping pass (upload_weights resets it).
uint64_t graph_ecc(spf_graph* g) {
  if (g->ecc_est || !g->V) {
    return g->ecc_est;
  }
  std::vector<uint64_t> dist(g->V, UINT64_MAX);
  using HE = std::pair<uint64_t, uint32_t>;
  std::priority_queue<HE, std::vector<HE>, std::greater<HE>> pq;
  dist[0] = 0;
  pq.push({0, 0});
  uint64_t ecc = 1;
  while (!pq.empty()) {
    const HE t = pq.top();
    pq.pop();
    if (t.first != dist[t.second]) {
      continue;
    }
    ecc = std::max(ecc, t.first);
    const uint32_t u = t.second;
    for (uint32_t e = g->row[u]; e < g->row[u + 1]; ++e) {
      const uint64_t c = t.first + g->w64[e];
      if (c < dist[g->col[e]]) {
        dist[g->col[e]] = c;
        pq.push({c, g->col[e]});
      }
    }
  }
  g->ecc_est = ecc;
  return ecc;
}

// Push-only delta-stepping (distance rows, LDS bucket bytes), measured on the
// 100k / 1M WAN (profiles/quick_wan.py; 8,361 sources, 24.0 -> 15.7 us/SPF):
// the bucket bytes quantise d at 1/16 of the processing bucket width (a
// sharper settled filter; twice as wide processing buckets, so fewer rounds),
// down to the resolution that still spreads 1.25x one node's eccentricity
// over the 254 byte values (saturation is exact, only slower); relaxations gather d[v] coherently and issue
// non-returning atomicMin; out-edges are read as packed 16-byte chunks.
// OPENR_SPF_DSTEP_FINE (byte bits below the bucket width), _NORET (bit 0
// non-returning atomics, bit 1 coherent gathers) and _PACK (0 off, 1 scalar,
// 2 vector) override.
void dstep_tune(spf_graph* g, spf_query* q, bool push_only) {
  q->dstep_fshift = q->dstep_shift;
  q->dstep_noret = 0;
  q->dstep_pack = 0;
  if (!push_only || !q->dstep_lbk) {
    return;
  }
  uint32_t fine = 4;
  if (getenv("OPENR_SPF_DSTEP_SHIFT") == nullptr) {
    q->dstep_shift += 1;
  }
  const uint64_t span = graph_ecc(g) + graph_ecc(g) / 4;
  uint32_t fs = q->dstep_shift - std::min(fine, q->dstep_shift);
  while (fs < q->dstep_shift && (span >> fs) > 250) {
    ++fs;
  }
  if (const char* env = getenv("OPENR_SPF_DSTEP_FINE")) {
    fine = (uint32_t)std::max(0, atoi(env));
    fs = q->dstep_shift - std::min(fine, q->dstep_shift);
  }
  q->dstep_fshift = fs;
  // bits 2-3 (bytes lowered at relaxation time, no gather into unreached
  // nodes): 14.9 -> 14.0 us/SPF on the 100k WAN (profiles/quick_wan.py)
  q->dstep_noret = 15;
  if (const char* env = getenv("OPENR_SPF_DSTEP_NORET")) {
    q->dstep_noret = (uint32_t)std::max(0, std::min(15, atoi(env)));
  }
  q->dstep_pack = g->cw_bits ? 2 : 0;
  if (const char* env = getenv("OPENR_SPF_DSTEP_PACK")) {
    q->dstep_pack = g->cw_bits ? (uint32_t)std::max(0, std::min(2, atoi(env))) : 0;
  }
}

// bucket width for spf_msdstep_kernel: the eccentricity of one source (host
// Dijkstra) spread over ~200 of the 255 bucket bytes; at least the
// delta-stepping Delta ~ mean metric / mean degree.
uint32_t msd_shift(const spf_graph* g, uint32_t s0) {
  const uint32_t V = g->V;
  std::vector<uint64_t> dist(V, UINT64_MAX);
  using HE = std::pair<uint64_t, uint32_t>;
  std::priority_queue<HE, std::vector<HE>, std::greater<HE>> pq;
  dist[s0] = 0;
  pq.push({0, s0});
  uint64_t ecc = 0, wsum = 0;
  while (!pq.empty()) {
    const HE t = pq.top();
    pq.pop();
    if (t.first != dist[t.second]) {
      continue;
    }
    ecc = std::max(ecc, t.first);
    const uint32_t u = t.second;
    for (uint32_t e = g->row[u]; e < g->row[u + 1]; ++e) {
      const uint64_t c = t.first + g->w64[e];
      if (c < dist[g->col[e]]) {
        dist[g->col[e]] = c;
        pq.push({c, g->col[e]});
      }
    }
  }
  for (uint32_t e = 0; e < g->E; ++e) {
    wsum += g->w64[e];
  }
  const double delta = g->E && V ? ((double)wsum / g->E) / ((double)g->E / V) : 1.0;
  uint32_t shift = 0;
  while (shift < 24 && ((ecc >> shift) > 200 || (double)(2u << shift) <= delta)) {
    ++shift;
  }
  if (const char* env = getenv("OPENR_SPF_MSD_SHIFT")) {
    shift = (uint32_t)std::min(24, std::max(0, atoi(env)));
  }
  return shift;
}

} // namespace

extern "C" {

int spf_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) {
    return 0;
  }
  return n;
}

const char* spf_error_string(int status) {
  switch (status) {
  case SPF_OK:
    return "ok";
  case SPF_E_INVALID:
    return "invalid argument";
  case SPF_E_NOMEM:
    return "out of memory";
  case SPF_E_DEVICE:
    return "device error";
  case SPF_E_UNSUPPORTED:
    return "unsupported shape";
  default:
    return "unknown status";
  }
}

const char* spf_last_error_detail(void) {
  return g_last_error.c_str();
}

int spf_graph_create(const spf_graph_desc* desc, spf_graph** out) {
  SPF_ABI_RANGE("spf_graph_create");
  if (!desc || !out) {
    return fail(SPF_E_INVALID, "null argument");
  }
  PhaseTimer mark("spf_graph_create");
  *out = nullptr;
  const uint32_t V = desc->num_nodes, E = desc->num_edges;
  if (const int vs = validate_graph_desc(desc)) {
    return vs;
  }
  mark("validate");
  const int ndev = spf_device_count();
  if (ndev <= 0) {
    return fail(SPF_E_DEVICE, "no HIP device visible");
  }
  if (desc->device < 0 || desc->device >= ndev) {
    return fail(SPF_E_INVALID, "bad device ordinal");
  }

  spf_graph* g = new spf_graph();
  g->device = desc->device;
  g->V = V;
  g->E = E;
  g->L = desc->num_links;
  g->nbw = (V + 31) / 32;
  g->row.assign(desc->row_ptr, desc->row_ptr + V + 1);
  g->col.assign(desc->col, desc->col + E);
  g->link.assign(desc->link_id, desc->link_id + E);
  g->rev.assign(desc->rev, desc->rev + E);
  g->w64.assign(desc->metric, desc->metric + E);
  g->trbits.assign(std::max<uint32_t>(g->nbw, 1), 0);
  for (uint32_t v = 0; v < V; ++v) {
    if (!desc->node_overloaded[v]) {
      g->trbits[v >> 5] |= 1u << (v & 31);
    }
  }
  mark("host copy");
  // distinct neighbours per node (ascending id = name order) and edge slots
  build_nbr_lists(g);
  mark("nbr lists");
  set_lanes_per_node(g);

  auto bail = [&](int s) {
    free_graph(g);
    return s;
  };
  if (hipSetDevice(g->device) != hipSuccess) {
    return bail(fail(SPF_E_DEVICE, "hipSetDevice failed"));
  }
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, g->device) == hipSuccess &&
      prop.multiProcessorCount > 0) {
    g->num_cus = prop.multiProcessorCount;
  }
  if (hipStreamCreateWithFlags(&g->own_stream, hipStreamNonBlocking) !=
      hipSuccess) {
    return bail(fail(SPF_E_DEVICE, "hipStreamCreate failed"));
  }
  g->stream = g->own_stream;
  mark("dev/stream");
  int s = SPF_OK;
  if ((s = dev_upload_g(g, &g->d_row, g->row.data(), V + 1)) ||
      (s = dev_upload_g(g, &g->d_col, g->col.data(), E)) ||
      (s = dev_upload_g(g, &g->d_link, g->link.data(), E)) ||
      (s = dev_upload_g(g, &g->d_rev, g->rev.data(), E)) ||
      (s = dev_upload_g(g, &g->d_slot, g->slot.data(), E)) ||
      (s = dev_upload_g(g, &g->d_tr, g->trbits.data(), g->trbits.size())) ||
      (s = dev_upload_g(g, &g->d_nbr_off, g->nbr_off.data(), V + 1)) ||
      (s = dev_upload_g(g, &g->d_nbrs, g->nbrs.data(), g->nbrs.size()))) {
    return bail(s);
  }
  g->nbr_cap = g->nbrs.size();
  g->cap_e = E;
  if (hipMalloc((void**)&g->d_nbr_w, std::max<size_t>(g->nbr_cap, 1) * 4) != hipSuccess) {
    return bail(fail(SPF_E_NOMEM, "neighbour weights"));
  }
  mark("csr upload");
  if ((s = upload_weights(g))) {
    return bail(s);
  }
  mark("weights");
  if ((s = upload_sell(g))) {
    return bail(s);
  }
  if ((s = g_stage_flush(g))) {
    return bail(s);
  }
  mark("sliced ELL");
  *out = g;
  return SPF_OK;
}

// In-place rebuild (LinkState::patchStructure's link flaps): same device,
// stream and node set; every host array and derived structure is recomputed
// from `desc`, and the device buffers are rewritten where they are large
// enough (reallocated with headroom otherwise), so a flap costs the host
// passes and the uploads, not an allocation / free of every array, a stream
// and the device-property query.
int spf_graph_update(spf_graph* g, const spf_graph_desc* desc) {
  SPF_ABI_RANGE("spf_graph_update");
  if (!g || !desc) {
    return fail(SPF_E_INVALID, "null argument");
  }
  if (const uint32_t n = g->live_queries.load(std::memory_order_relaxed)) {
    return fail(SPF_E_INVALID, "spf_graph_update: " + std::to_string(n) +
                                   " live queries read this graph (destroy them first)");
  }
  if (desc->num_nodes != g->V) {
    return fail(SPF_E_INVALID, "spf_graph_update: the node set changed (create a new graph)");
  }
  PhaseTimer mark("spf_graph_update");
  struct PhaseScope {
    explicit PhaseScope(PhaseTimer* t) { tl_phase = t->on ? t : nullptr; }
    ~PhaseScope() { tl_phase = nullptr; }
  } phase_scope(&mark);
  if (const int vs = validate_graph_desc(desc)) {
    return vs;
  }
  mark("validate");
  const uint32_t V = desc->num_nodes, E = desc->num_edges;
  HIP_TRY(hipSetDevice(g->device));
  HIP_TRY(hipStreamSynchronize(g->stream)); // queued work reads the old arrays
  mark("sync");
  // the previous CSR and its neighbour lists: unchanged rows keep theirs
  // (a flap changes the rows of its two endpoints only)
  const bool reuse = !g->links_patched && g->edge_up.empty();
  std::swap(g->row, g->old_row);
  std::swap(g->col, g->old_col);
  std::swap(g->nbr_off, g->old_nbr_off);
  std::swap(g->nbrs, g->old_nbrs);
  std::swap(g->slot, g->old_slot);
  g->E = E;
  g->L = desc->num_links;
  g->row.resize((size_t)V + 1);
  g->col.resize(E);
  g->link.resize(E);
  g->rev.resize(E);
  g->w64.resize(E);
  {
    const CopyItem cp[] = {{g->row.data(), desc->row_ptr, ((size_t)V + 1) * 4},
                           {g->col.data(), desc->col, (size_t)E * 4},
                           {g->link.data(), desc->link_id, (size_t)E * 4},
                           {g->rev.data(), desc->rev, (size_t)E * 4},
                           {g->w64.data(), desc->metric, (size_t)E * 8}};
    par_copy_many(cp, 5);
  }
  std::fill(g->trbits.begin(), g->trbits.end(), 0u);
  for (uint32_t v = 0; v < V; ++v) {
    if (!desc->node_overloaded[v]) {
      g->trbits[v >> 5] |= 1u << (v & 31);
    }
  }
  // a fresh CSR: no half-edge is down in place any more
  g->col_orig.clear();
  g->edge_up.clear();
  g->links_patched = false;
  g->paired = true;
  mark("host copy");
  NbrReuse nr{&g->old_row, &g->old_col, &g->old_nbr_off, &g->old_nbrs, &g->old_slot};
  build_nbr_lists(g, reuse && g->old_row.size() == (size_t)V + 1 ? &nr : nullptr);
  set_lanes_per_node(g); // as spf_graph_create (it drifted after flaps)
  mark("nbr lists");
  // edge-sized arrays: rewritten in place, or reallocated with headroom
  auto fit32 = [&](uint32_t** d, size_t n, size_t& cap) -> int {
    if (!*d || n > cap) {
      if (*d) {
        (void)hipFree(*d);
        *d = nullptr;
      }
      const size_t c = std::max<size_t>(1, n + n / 8);
      HIP_TRY(hipMalloc((void**)d, c * 4));
      cap = c;
    }
    return SPF_OK;
  };
  int s = SPF_OK;
  size_t cap_e = g->cap_e, cap_nbr = g->nbr_cap, cap_v = (size_t)V + 1;
  // col / link / rev / slot share cap_e: grow them together
  if (E > g->cap_e) {
    for (uint32_t** d : {&g->d_col, &g->d_link, &g->d_rev, &g->d_slot}) {
      if (*d) {
        (void)hipFree(*d);
        *d = nullptr;
      }
    }
  }
  size_t c1 = cap_e, c2 = cap_e, c3 = cap_e, c4 = cap_e;
  if ((s = fit32(&g->d_col, E, c1)) || (s = fit32(&g->d_link, E, c2)) ||
      (s = fit32(&g->d_rev, E, c3)) || (s = fit32(&g->d_slot, E, c4)) ||
      (s = fit32(&g->d_row, (size_t)V + 1, cap_v)) ||
      (s = fit32(&g->d_nbr_off, (size_t)V + 1, cap_v))) {
    return s;
  }
  g->cap_e = std::max(c1, (size_t)E);
  if (g->nbrs.size() > cap_nbr || !g->d_nbrs) {
    for (uint32_t** d : {&g->d_nbrs, &g->d_nbr_w}) {
      if (*d) {
        (void)hipFree(*d);
        *d = nullptr;
      }
    }
    const size_t c = std::max<size_t>(1, g->nbrs.size() + g->nbrs.size() / 8);
    HIP_TRY(hipMalloc((void**)&g->d_nbrs, c * 4));
    HIP_TRY(hipMalloc((void**)&g->d_nbr_w, c * 4));
    g->nbr_cap = c;
  }
  if ((s = g_stage_many(g, {{g->d_col, g->col.data(), (size_t)E * 4},
                            {g->d_link, g->link.data(), (size_t)E * 4},
                            {g->d_rev, g->rev.data(), (size_t)E * 4},
                            {g->d_slot, g->slot.data(), (size_t)E * 4},
                            {g->d_row, g->row.data(), ((size_t)V + 1) * 4},
                            {g->d_nbr_off, g->nbr_off.data(), ((size_t)V + 1) * 4},
                            {g->d_tr, g->trbits.data(), g->trbits.size() * 4},
                            {g->d_nbrs, g->nbrs.data(), g->nbrs.size() * 4}}))) {
    return s;
  }
  mark("csr upload");
  if ((s = upload_weights(g))) {
    return s;
  }
  mark("weights");
  if ((s = upload_sell(g))) {
    return s;
  }
  if ((s = g_stage_flush(g))) {
    return s;
  }
  mark("sliced ELL");
  return SPF_OK;
}

int spf_device_alloc(int device, size_t bytes, void** out) {
  SPF_ABI_RANGE("spf_device_alloc");
  if (!out) {
    return fail(SPF_E_INVALID, "null argument");
  }
  *out = nullptr;
  if (device < 0 || device >= spf_device_count()) {
    return fail(SPF_E_INVALID, "bad device ordinal");
  }
  HIP_TRY(hipSetDevice(device));
  if (bytes && hipMalloc(out, bytes) != hipSuccess) {
    *out = nullptr;
    return fail(SPF_E_NOMEM, "device table");
  }
  return SPF_OK;
}

int spf_device_free(int device, void* p) {
  SPF_ABI_RANGE("spf_device_free");
  if (p) {
    HIP_TRY(hipSetDevice(device));
    HIP_TRY(hipFree(p));
  }
  return SPF_OK;
}

int spf_device_memcpy(int device, void* dst, const void* src, size_t bytes, int kind) {
  SPF_ABI_RANGE("spf_device_memcpy");
  if (bytes && (!dst || !src)) {
    return fail(SPF_E_INVALID, "null argument");
  }
  if (!bytes) {
    return SPF_OK;
  }
  HIP_TRY(hipSetDevice(device));
  const hipMemcpyKind k = kind == SPF_COPY_D2H   ? hipMemcpyDeviceToHost
                          : kind == SPF_COPY_H2D ? hipMemcpyHostToDevice
                                                 : hipMemcpyDeviceToDevice;
  HIP_TRY(hipMemcpy(dst, src, bytes, k));
  return SPF_OK;
}

// live queries of a graph (not exported: spf_cgraph_destroy checks every
// device graph before it frees any)
__attribute__((visibility("hidden"))) uint32_t spf_graph_live_queries_(const spf_graph* g) {
  return g ? g->live_queries.load(std::memory_order_relaxed) : 0u;
}

int spf_graph_destroy(spf_graph* g) {
  SPF_ABI_RANGE("spf_graph_destroy");
  if (g) {
    if (const uint32_t n = g->live_queries.load(std::memory_order_relaxed)) {
      // destroying it would leave those queries reading freed memory (their
      // destroy sets g->device and syncs g->stream): refuse, free nothing
      return fail(SPF_E_INVALID, "spf_graph_destroy: " + std::to_string(n) +
                                     " live queries on this graph (destroy them first)");
    }
  }
  free_graph(g);
  return SPF_OK;
}

int spf_graph_set_transit(spf_graph* g, const uint8_t* node_overloaded) {
  SPF_ABI_RANGE("spf_graph_set_transit");
  if (!g || (g->V && !node_overloaded)) {
    return fail(SPF_E_INVALID, "null argument");
  }
  std::fill(g->trbits.begin(), g->trbits.end(), 0u);
  for (uint32_t v = 0; v < g->V; ++v) {
    if (!node_overloaded[v]) {
      g->trbits[v >> 5] |= 1u << (v & 31);
    }
  }
  HIP_TRY(hipSetDevice(g->device));
  // ordered on the graph stream: kernels queued before read the old bits,
  // kernels queued after the new ones (a pageable source is staged before
  // the call returns, so trbits may change again right away)
  HIP_TRY(hipMemcpyAsync(g->d_tr, g->trbits.data(), g->trbits.size() * 4,
                         hipMemcpyHostToDevice, g->stream));
  if (g->hop_bounded || (g->maxw && !g->wrap && !g->n_zero &&
                         (unsigned __int128)g->maxw * (g->V - 1) >= 0xFFFFFFFFull)) {
    refresh_exact(g); // the hop bound depends on which nodes may be transited
  }
  return SPF_OK;
}

int spf_graph_patch_metrics(
    spf_graph* g, uint32_t n, const uint32_t* edge_idx, const uint64_t* m) {
  SPF_ABI_RANGE("spf_graph_patch_metrics");
  if (!g || (n && (!edge_idx || !m))) {
    return fail(SPF_E_INVALID, "null argument");
  }
  for (uint32_t i = 0; i < n; ++i) {
    if (edge_idx[i] >= g->E) {
      return fail(SPF_E_INVALID, "edge index out of range");
    }
  }
  HIP_TRY(hipSetDevice(g->device));
  if (n && (uint64_t)n * 64 <= g->E && env_flag("OPENR_SPF_PATCH_INPLACE", 1)) {
    const int st = patch_weights_sparse(g, n, edge_idx, m);
    if (st != SPF_E_UNSUPPORTED) {
      return st;
    }
  }
  for (uint32_t i = 0; i < n; ++i) {
    g->w64[edge_idx[i]] = m[i];
  }
  HIP_TRY(hipStreamSynchronize(g->stream));
  if (const int st = upload_weights(g)) {
    return st;
  }
  return g_stage_flush(g);
}

int spf_graph_set_edges(
    spf_graph* g, uint32_t n, const uint32_t* edge_idx, const uint8_t* up,
    const uint64_t* metric) {
  SPF_ABI_RANGE("spf_graph_set_edges");
  if (!g || (n && (!edge_idx || !up || !metric))) {
    return fail(SPF_E_INVALID, "null argument");
  }
  if (g->exact || g->wrap || g->n_zero) {
    return fail(SPF_E_UNSUPPORTED, "in-place link changes need 32-bit rows and no metric 0");
  }
  for (uint32_t i = 0; i < n; ++i) {
    if (edge_idx[i] >= g->E) {
      return fail(SPF_E_INVALID, "edge index out of range");
    }
    if (metric[i] == 0 || metric[i] > 0x7FFFFFFFull ||
        (g->cw_bits && metric[i] >= (1ull << (32 - g->cw_bits)))) {
      return fail(SPF_E_UNSUPPORTED, "metric outside the in-place range (0, wrap or unpackable)");
    }
  }
  if (g->col_orig.empty()) {
    g->col_orig = g->col;
    g->edge_up.assign(g->E, 1);
  }
  HIP_TRY(hipSetDevice(g->device));
  HIP_TRY(hipStreamSynchronize(g->stream)); // queued kernels read the old words
  std::vector<uint32_t> lists[kPatch32];
  std::vector<uint32_t> w64l;
  for (uint32_t i = 0; i < n; ++i) {
    const uint32_t e = edge_idx[i];
    const uint32_t u =
        (uint32_t)(std::upper_bound(g->row.begin(), g->row.end(), e) - g->row.begin()) - 1;
    g->edge_up[e] = up[i] ? 1 : 0;
    // a down half-edge is a self-loop of its tail with a positive metric:
    // d[u] + w > d[u], so it never relaxes, is never tight, and the pull
    // reads u's own frontier bits (a subset of its visited bits)
    g->col[e] = up[i] ? g->col_orig[e] : u;
    g->w64[e] = metric[i];
    const uint32_t w32 = (uint32_t)metric[i];
    lists[0].insert(lists[0].end(), {e, w32});           // wout[e]
    lists[1].insert(lists[1].end(), {g->rev[e], w32});   // win[rev[e]]
    if (g->cw_bits) {
      lists[3].insert(lists[3].end(), {e, g->col[e] | (w32 << g->cw_bits)});
    }
    lists[4].insert(lists[4].end(), {e, g->col[e]});
    if (g->d_sell) {
      const uint32_t j = e - g->row[u], c = u >> 6, L = u & 63u;
      const uint32_t idx = ((g->sell_off[c] + j / 4) * 64 + L) * 4 + (j & 3);
      lists[5].insert(lists[5].end(), {idx, g->col[e]});
    }
    w64l.insert(w64l.end(), {e, (uint32_t)metric[i], (uint32_t)(metric[i] >> 32)});
  }
  // graph scalars and the 32-bit row bound (the transit hop bound reads the
  // patched heads)
  rescan_scalars(g);
  g->ecc_est = 0;
  g->links_patched = true;
  g->paired = true;
  for (uint32_t e = 0; e < g->E && g->paired; ++e) {
    g->paired = g->edge_up[e] == g->edge_up[g->rev[e]];
  }
  // distinct-neighbour lists over the up half-edges (a neighbour whose every
  // link went down leaves its source's list; one coming back re-enters it),
  // edge slots and cheapest metric per neighbour, so next-hop queries stay
  // exact on the patched graph; re-uploaded whole (O(E), no graph rebuild)
  build_nbr_lists(g);
  g->nbr_w.assign(g->nbrs.size(), 0xFFFFFFFFu);
  for (uint32_t u = 0; u < g->V; ++u) {
    for (uint32_t e = g->row[u]; e < g->row[u + 1]; ++e) {
      if (g->edge_up[e]) {
        uint32_t& w = g->nbr_w[g->nbr_off[u] + g->slot[e]];
        w = std::min<uint32_t>(w, (uint32_t)std::min<uint64_t>(g->w64[e], 0xFFFFFFFFull));
      }
    }
  }
  {
    const size_t nn = g->nbrs.size();
    if (nn != g->nbr_cap) {
      (void)hipFree(g->d_nbrs);
      (void)hipFree(g->d_nbr_w);
      g->d_nbrs = nullptr;
      g->d_nbr_w = nullptr;
      HIP_TRY(hipMalloc((void**)&g->d_nbrs, std::max<size_t>(nn, 1) * 4));
      HIP_TRY(hipMalloc((void**)&g->d_nbr_w, std::max<size_t>(nn, 1) * 4));
      g->nbr_cap = nn;
    }
    HIP_TRY(hipMemcpy(g->d_slot, g->slot.data(), (size_t)g->E * 4, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(g->d_nbr_off, g->nbr_off.data(), ((size_t)g->V + 1) * 4,
                      hipMemcpyHostToDevice));
    if (nn) {
      HIP_TRY(hipMemcpy(g->d_nbrs, g->nbrs.data(), nn * 4, hipMemcpyHostToDevice));
      HIP_TRY(hipMemcpy(g->d_nbr_w, g->nbr_w.data(), nn * 4, hipMemcpyHostToDevice));
    }
  }
  PatchArgs a{};
  uint32_t* arrays[kPatch32] = {g->d_wout, g->d_win, nullptr, g->d_cw, g->d_col,
                                reinterpret_cast<uint32_t*>(g->d_sell)};
  std::vector<uint32_t> pk;
  for (int k = 0; k < kPatch32; ++k) {
    a.dst32[k] = arrays[k];
    a.n32[k] = arrays[k] ? (uint32_t)(lists[k].size() / 2) : 0;
    a.off32[k] = (uint32_t)pk.size();
    pk.insert(pk.end(), lists[k].begin(), lists[k].end());
  }
  a.dst64 = g->d_w64;
  a.n64 = n;
  a.off64 = (uint32_t)pk.size();
  pk.insert(pk.end(), w64l.begin(), w64l.end());
  if (pk.empty()) {
    return SPF_OK;
  }
  uint32_t* d = nullptr;
  HIP_TRY(pool_malloc((void**)&d, pk.size() * 4));
  HIP_TRY(hipMemcpyAsync(d, pk.data(), pk.size() * 4, hipMemcpyHostToDevice, g->stream));
  a.pk = d;
  SPF_LAUNCH(spf_patch_words_kernel, dim3(1), dim3(256), 0, g->stream, a);
  const hipError_t le = hipGetLastError();
  const hipError_t se = hipStreamSynchronize(g->stream);
  pool_free(d);
  HIP_TRY(le);
  HIP_TRY(se);
  return SPF_OK;
}

int spf_graph_set_stream(spf_graph* g, void* stream) {
  if (!g) {
    return fail(SPF_E_INVALID, "null graph");
  }
  g->stream = stream ? (hipStream_t)stream : g->own_stream;
  return SPF_OK;
}

void* spf_graph_get_stream(spf_graph* g) {
  return g ? (void*)g->stream : nullptr;
}

int spf_graph_needs_exact(const spf_graph* g) {
  return g && g->exact ? 1 : 0;
}

int spf_graph_num_nbrs(const spf_graph* g, uint32_t node) {
  if (!g || node >= g->V) {
    return fail(SPF_E_INVALID, "bad node");
  }
  return (int)(g->nbr_off[node + 1] - g->nbr_off[node]);
}

int spf_graph_nbrs(const spf_graph* g, uint32_t node, uint32_t* out) {
  if (!g || node >= g->V || !out) {
    return fail(SPF_E_INVALID, "bad node");
  }
  std::copy(g->nbrs.begin() + g->nbr_off[node],
            g->nbrs.begin() + g->nbr_off[node + 1], out);
  return SPF_OK;
}

namespace {

// Zero-metric plan eligibility (spf_zvar_kernel): every metric is 0 or one
// value c (c * V below 2^32 - 1), and the metric-0 half-edges join at most
// kZeroLinks node pairs that share no node.  Parallel metric-0 links of one
// pair count once (the plan reasons about the pair's settle order).
constexpr uint32_t kZeroLinks = 3;
struct ZeroLink {
  uint32_t a, b; // a < b
  bool ab, ba;   // a -> b / b -> a has metric 0
};

bool zero_plan_links(const spf_graph* g, std::vector<ZeroLink>& out, uint32_t& c) {
  out.clear();
  c = 0;
  if (g->wrap || !g->n_zero || g->V < 2) {
    return false;
  }
  for (uint32_t u = 0; u < g->V; ++u) {
    for (uint32_t e = g->row[u]; e < g->row[u + 1]; ++e) {
      const uint64_t m = g->w64[e];
      if (m != 0) {
        if (c == 0) {
          c = (uint32_t)m;
        } else if (m != c) {
          return false;
        }
        continue;
      }
      const uint32_t v = g->col[e];
      if (v == u) {
        return false;
      }
      const uint32_t a = std::min(u, v), b = std::max(u, v);
      auto it = std::find_if(out.begin(), out.end(),
                             [&](const ZeroLink& z) { return z.a == a && z.b == b; });
      if (it == out.end()) {
        if (out.size() == kZeroLinks) {
          return false;
        }
        out.push_back({a, b, false, false});
        it = out.end() - 1;
      }
      (u == a ? it->ab : it->ba) = true;
    }
  }
  std::vector<uint32_t> ends;
  for (const auto& z : out) {
    ends.push_back(z.a);
    ends.push_back(z.b);
  }
  std::sort(ends.begin(), ends.end());
  if (std::adjacent_find(ends.begin(), ends.end()) != ends.end()) {
    return false; // links share a node: a plateau of three or more nodes
  }
  return c != 0 && (uint64_t)c * g->V < 0xFFFFFFFFull && !out.empty();
}

} // namespace

int spf_query_create(spf_graph* g, const spf_query_desc* desc, spf_query** out) {
  SPF_ABI_RANGE("spf_query_create");
  if (!g || !desc || !out) {
    return fail(SPF_E_INVALID, "null argument");
  }
  *out = nullptr;
  const uint32_t nq = desc->num_queries, V = g->V;
  if (nq && !desc->sources) {
    return fail(SPF_E_INVALID, "null sources");
  }
  for (uint32_t i = 0; i < nq; ++i) {
    if (desc->sources[i] >= V) {
      return fail(SPF_E_INVALID, "source out of range");
    }
  }
  bool has_ign = false;
  uint32_t max_ign = 0;
  if (desc->ignore_offsets) {
    if (desc->ignore_offsets[0] != 0) {
      return fail(SPF_E_INVALID, "ignore_offsets[0] != 0");
    }
    for (uint32_t i = 0; i < nq; ++i) {
      const uint32_t lo = desc->ignore_offsets[i],
                     hi = desc->ignore_offsets[i + 1];
      if (hi < lo || (hi > lo && !desc->ignore_links)) {
        return fail(SPF_E_INVALID, "bad ignore_offsets");
      }
      for (uint32_t k = lo + 1; k < hi; ++k) {
        if (desc->ignore_links[k - 1] >= desc->ignore_links[k]) {
          return fail(SPF_E_INVALID, "ignore list not strictly sorted");
        }
      }
      max_ign = std::max(max_ign, hi - lo);
    }
    has_ign = max_ign > 0;
  }

  spf_query* q = new spf_query();
  q->g = g;
  g->live_queries.fetch_add(1, std::memory_order_relaxed); // free_query gives it back
  q->nq = nq;
  q->flags = desc->flags;
  q->has_ign = has_ign;
  q->Vp = (V + 15) & ~15u;
  q->Vp8 = (V + 15) & ~15u;
  auto bail = [&](int s) {
    free_query(q);
    return s;
  };
  const bool unit = desc->flags & SPF_F_UNIT_METRIC;
  const bool want_nh = desc->flags & SPF_F_NEXTHOPS;
  const bool want_order = desc->flags & SPF_F_ORDER;
  if (want_order && g->links_patched) {
    return bail(fail(SPF_E_UNSUPPORTED,
                     "settle order on a graph whose links were set in place "
                     "(spf_graph_set_edges): rebuild the graph"));
  }

  // next-hop mask geometry: the working word layout and the byte-strided
  // output layout (kQueryWideMasks: output = working, for internal batches
  // whose rows are copied into another query's working buffer)
  uint32_t maxw = 0;
  q->nh_off.assign(nq, 0);
  q->nh_w.assign(nq, 0);
  q->nhb_off.assign(nq, 0);
  q->nh_b.assign(nq, 0);
  if (want_nh) {
    uint64_t off = 0, boff = 0;
    for (uint32_t i = 0; i < nq; ++i) {
      const uint32_t s = desc->sources[i];
      const uint32_t nn = g->nbr_off[s + 1] - g->nbr_off[s];
      const uint32_t w = std::max<uint32_t>(1, (nn + 63) / 64);
      const uint32_t b = (desc->flags & kQueryWideMasks) ? 8 * w : nh_bytes_for(nn);
      q->nh_off[i] = off;
      q->nh_w[i] = w;
      off += ((uint64_t)w * V + 3) & ~3ull; // 32-byte aligned rows
      q->nhb_off[i] = boff;
      q->nh_b[i] = b;
      boff += ((uint64_t)b * V + 31) & ~31ull;
      q->narrow = q->narrow || b < 8;
      maxw = std::max(maxw, w);
    }
    q->nh_total = off;
    q->nhb_total = boff;
  }

  // ---- plan: which kernels compute this batch
  std::vector<int32_t> row_of;
  std::vector<uint32_t> helpers; // MS-BFS helper sources (rows nq, nq+1, ...)
  std::vector<uint32_t> msd_perm;
  // metrics that wrap (negative i32 as uint64): the literal DijkstraQ
  // replay; metric 0 / sums past 32 bits / a settle order: the wide plan
  // (OPENR_SPF_LITERAL=1 forces the replay on any 64-bit graph: measurement)
  const char* lit_env = getenv("OPENR_SPF_LITERAL");
  const bool literal =
      (g->wrap && !unit) || (g->exact && !unit && lit_env && atoi(lit_env) == 1);
  // metric-0 links on an otherwise uniform metric: MS-BFS variant tables
  // (spf_zvar_kernel) instead of the wide plan (OPENR_SPF_ZERO_MSBFS=0: wide)
  std::vector<ZeroLink> zlinks;
  uint32_t zc = 0;
  const bool zcand = !unit && !literal && !want_order && !has_ign && g->exact && g->n_zero &&
                     nq >= 32 && V <= kMsThreads * kMsMaxK && 2 * (size_t)V * 4 <= kLdsLimit &&
                     env_flag("OPENR_SPF_ZERO_MSBFS", 1) &&
                     !(getenv("OPENR_SPF_MSBFS") && atoi(getenv("OPENR_SPF_MSBFS")) == 0) &&
                     zero_plan_links(g, zlinks, zc);
  const bool exact = ((g->exact && !unit) || want_order) && !zcand;
  const bool uniform = unit || g->uniform != 0 || zcand;
  bool rows_ok = false;
  bool few_rows = false; // weighted few-source batch with helper rows (below)
  if (want_nh && !exact && !has_ign) {
    // next hops from distance rows need every neighbour's row in the batch
    row_of.assign(V, -1);
    for (uint32_t i = nq; i-- > 0;) {
      row_of[desc->sources[i]] = (int32_t)i;
    }
    rows_ok = true;
    for (uint32_t i = 0; i < nq && rows_ok; ++i) {
      const uint32_t s = desc->sources[i];
      for (uint32_t k = g->nbr_off[s]; k < g->nbr_off[s + 1]; ++k) {
        if (row_of[g->nbrs[k]] < 0) {
          rows_ok = false;
          break;
        }
      }
    }
    // an MS-BFS batch whose sources' neighbours lie outside it (one rank's
    // block of a sharded all-sources table): the missing neighbours ride
    // along as helper sources — their level rows are computed after the
    // batch's own rows and serve only the next-hop pass — instead of the
    // batch dropping to per-source SSSP (fabric block of 1,247 sources:
    // 1.93 ms on the lds plan, profiles/r03j)
    // (a batch below 32 sources qualifies when its helpers bring it there:
    // one source and its neighbours' rows in one MS-BFS pass beat the
    // single-workgroup SSSP of that source, e.g. a what-if baseline)
    const bool msbfs_candidate = !rows_ok && uniform && !literal &&
                                 V <= kMsThreads * kMsMaxK &&
                                 2 * (size_t)V * 4 <= kLdsLimit &&
                                 !(getenv("OPENR_SPF_MSBFS") && atoi(getenv("OPENR_SPF_MSBFS")) == 0) &&
                                 env_flag("OPENR_SPF_MSBFS_HELPERS", 1);
    if (msbfs_candidate) {
      // no bound on the helper count: it is < V, and one MS-BFS pass over
      // the batch and all its helpers still beats per-source SSSP on the
      // batch alone (a 64-source workgroup costs about one source's SSSP)
      std::vector<uint32_t> extra;
      for (uint32_t i = 0; i < nq; ++i) {
        const uint32_t s = desc->sources[i];
        for (uint32_t k = g->nbr_off[s]; k < g->nbr_off[s + 1]; ++k) {
          const uint32_t f = g->nbrs[k];
          if (row_of[f] < 0) {
            row_of[f] = (int32_t)(nq + extra.size());
            extra.push_back(f);
          }
        }
      }
      // (and a small area, one node per MS-BFS thread, at any batch size: a
      // RouteDb build's few sources on the 100-node grid take one MS-BFS
      // workgroup and the level pass instead of one SSSP workgroup per
      // source with next hops inline, 78.7 us, profiles/r06an;
      // OPENR_SPF_MSBFS_SMALL=0 disables)
      if (nq >= 32 || (nq + extra.size() >= 32 && env_flag("OPENR_SPF_MSBFS_FEW", 1)) ||
          (V <= kMsThreads && env_flag("OPENR_SPF_MSBFS_SMALL", 1))) {
        rows_ok = true;
        helpers = std::move(extra);
      }
    }
    // a few sources of a weighted graph (a what-if baseline, a RouteDb
    // build's prefetch): their neighbours ride along as helper sources of a
    // distances-only delta-stepping pass (one workgroup per row, all in
    // parallel), and the next hops come from the rows (spf_nh_rows_kernel)
    // instead of the PULL rounds of one workgroup per source
    // (OPENR_SPF_FEW_ROWS=0 disables)
    // (exactly the batches the planner below sends to the few-source
    // delta-stepping plan: weighted, V in [4096, 65535], the LDS-plan image
    // fits, at most one source per 16 CUs, <= 16 mask words; and LDS-row
    // eligible: 12-bit metrics, packed edges)
    if (!rows_ok && !uniform && !literal && V >= 4096 && V <= 65535 &&
        lds_ctl_bytes(g, 0) + lds_state_bytes(V) <= kLdsLimit && maxw <= 16 &&
        (size_t)nq * 16 <= (size_t)g->num_cus && g->cw_bits && g->maxw <= kDlMaxDist &&
        env_flag("OPENR_SPF_FEW_DSTEP", 1) && getenv("OPENR_SPF_DSTEP") == nullptr &&
        env_flag("OPENR_SPF_DSTEP_LDSROW", 1) && env_flag("OPENR_SPF_FEW_ROWS", 1)) {
      std::vector<uint32_t> extra;
      for (uint32_t i = 0; i < nq; ++i) {
        const uint32_t s = desc->sources[i];
        for (uint32_t k = g->nbr_off[s]; k < g->nbr_off[s + 1]; ++k) {
          const uint32_t f = g->nbrs[k];
          if (row_of[f] < 0) {
            row_of[f] = (int32_t)(nq + extra.size());
            extra.push_back(f);
          }
        }
      }
      if (nq + extra.size() <= (size_t)g->num_cus) {
        rows_ok = true;
        helpers = std::move(extra);
        few_rows = true;
      }
    }
    if (!rows_ok) {
      row_of.clear();
    }
  }
  if (literal) {
    q->dist = DistPlan::Exact;
    q->nh = want_nh ? NhPlan::Inline : NhPlan::None;
  } else if (exact || (want_nh && !rows_ok && maxw > 16)) {
    q->dist = DistPlan::Wide;
    q->nh = want_nh ? NhPlan::Inline : NhPlan::None;
    q->lds_bytes = (size_t)g->nbw * 4;
    if (q->lds_bytes + 64 > kLdsLimit) {
      return bail(fail(SPF_E_UNSUPPORTED, "wide plan: pending bitmap exceeds LDS"));
    }
    q->grid = std::min<uint32_t>(std::max<uint32_t>(nq, 1), (uint32_t)g->num_cus * 2);
  } else {
    q->nh = !want_nh ? NhPlan::None : (rows_ok ? NhPlan::Rows : NhPlan::Inline);
    // weighted graph whose distance row does not fit LDS: delta-stepping
    // with next hops inline (the rows plan would read every neighbour's
    // 4V-byte row per source: 8E*V bytes per all-sources pass)
    const bool big = lds_ctl_bytes(g, 0) + lds_state_bytes(V) > kLdsLimit || V > 65535;
    // delta-stepping LDS image: pending + marked bitmaps + the bucket bytes
    // (OPENR_SPF_DSTEP_LDSBKT=0: buckets derived from the distance row, a
    // 25 KB image, 2 workgroups per CU — measured slower on the 100k WAN:
    // the second 400 KB row per CU and the per-phase row reads of pending
    // nodes cost more than the extra waves hide)
    const char* lbk_env = getenv("OPENR_SPF_DSTEP_LDSBKT");
    q->dstep_lbk = !(lbk_env && atoi(lbk_env) == 0);
    q->dstep_ign_cap = has_ign ? std::min(max_ign, kIgnLdsMax) : 0; // sorted list only
    const size_t dstep_lds =
        (2 * (size_t)g->nbw + kCtlWords + q->dstep_ign_cap) * 4 +
        (q->dstep_lbk ? (((size_t)V + 15) & ~(size_t)15) : 0);
    // a few sources of a weighted graph that fits LDS (a what-if baseline, a
    // RouteDb build's SPFs): one workgroup per source either way, and bucket
    // order relaxes most nodes once where the frontier rounds of
    // spf_sssp_kernel re-relax them (OPENR_SPF_FEW_DSTEP=0 disables)
    const bool few = !big && !has_ign && V >= 4096 && (size_t)nq * 16 <= (size_t)g->num_cus &&
                     env_flag("OPENR_SPF_FEW_DSTEP", 1);
    const bool dstep = (big || few) && !uniform && dstep_lds <= kLdsLimit && maxw <= 16 &&
                       getenv("OPENR_SPF_DSTEP") == nullptr;
    // many distance-only rows of such a graph: 32 sources per workgroup over
    // a node-major slab.  Measured slower than per-source delta-stepping on
    // the 100k WAN (0.145 vs 0.100 ms/SPF at 8192 sources: the 12.8 MB slab
    // per workgroup does not stay on chip), so opt-in: OPENR_SPF_MSD=1.
    const char* msd_env = getenv("OPENR_SPF_MSD");
    const bool msd = big && !uniform && !want_nh && !has_ign && nq >= 2 * kMsdK &&
                     msd_lds_bytes(g) <= kLdsLimit && msd_env && atoi(msd_env) == 1;
    if (dstep && q->nh == NhPlan::Rows && !few_rows) {
      q->nh = NhPlan::Inline;
    }
    const bool bfs = uniform && !has_ign && q->nh != NhPlan::Inline;
    q->wmax = q->nh != NhPlan::Inline ? 0 : (maxw <= 1 ? 1 : (maxw <= 4 ? 4 : 16));
    // LDS words for a query's ignore list: the sorted list, or its hash form
    // (ign_hash_slots) when that fits
    q->ign_cap = has_ign ? std::min(std::max(max_ign, ign_hash_slots(max_ign)), kIgnLdsMax) : 0;
    const size_t ctl = lds_ctl_bytes(g, q->ign_cap);
    const size_t lds = ctl + lds_state_bytes(V);
    if (msd) {
      q->dist = DistPlan::MsDstep;
      q->nh = NhPlan::None;
      q->wmax = 0;
      q->lds_bytes = msd_lds_bytes(g);
      q->dstep_shift = msd_shift(g, desc->sources[0]);
      const char* cl = getenv("OPENR_SPF_MSD_CLUSTER");
      msd_perm = msd_batches(g, desc->sources, nq, !(cl && atoi(cl) == 0));
      q->msd_nbatch = (uint32_t)(msd_perm.size() / kMsdK);
      q->grid = std::min<uint32_t>(q->msd_nbatch, (uint32_t)g->num_cus);
    } else if (V <= 65535 && lds <= kLdsLimit && !(few && dstep) && !few_rows) {
      q->dist = bfs ? DistPlan::BfsLds : DistPlan::SsspLds;
      q->lds_bytes = lds;
      const uint32_t per_cu =
          std::max<uint32_t>(1, std::min<uint32_t>(4, kLdsLimit / lds));
      q->grid = std::min<uint32_t>(std::max<uint32_t>(nq, 1),
                                   (uint32_t)g->num_cus * per_cu);
    } else if (dstep) {
      q->dist = DistPlan::Dstep;
      q->lds_bytes = dstep_lds;
      // bucket width ~ mean metric / mean degree (delta-stepping's
      // Delta = Theta(w/d)), a power of two; OPENR_SPF_DSTEP_SHIFT overrides
      q->dstep_shift = dstep_bucket_shift(g, want_nh);
      dstep_tune(g, q, !want_nh);
      const char* bs_env = getenv("OPENR_SPF_DSTEP_BS");
      q->dstep_bs = (bs_env && atoi(bs_env) == 512) ? 512 : 1024;
      // workgroups per CU: 2048 threads per CU, LDS permitting
      uint32_t per_cu = (uint32_t)std::max<size_t>(
          1, std::min<size_t>(2048 / q->dstep_bs, kLdsLimit / std::max<size_t>(dstep_lds, 1)));
      if (const char* pc = getenv("OPENR_SPF_DSTEP_PERCU")) {
        per_cu = std::max<uint32_t>(1, std::min<uint32_t>(per_cu, (uint32_t)atoi(pc)));
      }
      const uint32_t nr = nq + (uint32_t)helpers.size();
      q->grid = std::min<uint32_t>(std::max<uint32_t>(nr, 1), (uint32_t)g->num_cus * per_cu);
      // distance rows whose every value fits 12 bits (metrics <= 4,094; the
      // kernel flags a source whose values do not, and the pass above redoes
      // only those): the row lives in LDS (OPENR_SPF_DSTEP_LDSROW=0 disables)
      const size_t dl_lds = (size_t)((V + 4) / 5) * 8 + kDlCtl * 4;
      q->dlds = q->nh != NhPlan::Inline && !has_ign && g->cw_bits && g->maxw <= kDlMaxDist &&
                dl_lds <= kLdsLimit && env_flag("OPENR_SPF_DSTEP_LDSROW", 1);
      if (q->dlds) {
        q->dlds_lds = dl_lds;
        q->dlds_grid = std::min<uint32_t>(std::max<uint32_t>(nr, 1), (uint32_t)g->num_cus);
        // bucket width: 8x the delta-stepping Delta (mean metric / mean
        // degree): with the row in LDS a bucket scan is cheap, and wider
        // buckets mean fewer phases (100k WAN, profiles/r04c: 2^4 9.5,
        // 2^5 7.7, 2^7 6.7 us/SPF)
        q->dlds_shift = std::min<uint32_t>(dstep_bucket_shift(g, false) + 1, 11);
        if (const char* env = getenv("OPENR_SPF_DSTEP_LSHIFT")) {
          q->dlds_shift = (uint32_t)std::min(11, std::max(0, atoi(env)));
        }
      }
    } else if (ctl <= kLdsLimit) {
      q->dist = bfs ? DistPlan::BfsGmem : DistPlan::SsspGmem;
      q->lds_bytes = ctl;
      q->grid = std::min<uint32_t>(std::max<uint32_t>(nq, 1),
                                   (uint32_t)g->num_cus * 2);
    } else {
      return bail(fail(SPF_E_UNSUPPORTED, "graph too large for one device"));
    }
  }

  DistPlan ms_ign_prev = q->dist;
  // distance-only batches with ignore lists on a uniform metric (KSP2 second
  // passes: 9,975 per fabric build, each ignoring the links of its k = 1
  // paths): the bit-parallel BFS with per-batch masks of the ignored
  // half-edges instead of one SSSP workgroup per query (OPENR_SPF_MSBFS_IGN=0
  // disables).  Mask memory: 8 B per (batch, half-edge), at most 1 GiB.
  if (has_ign && uniform && !want_nh && !want_order && !literal && !exact && nq >= 32 &&
      V <= kMsThreads * kMsMaxK && helpers.empty() &&
      (q->dist == DistPlan::SsspLds || q->dist == DistPlan::SsspGmem) &&
      env_flag("OPENR_SPF_MSBFS_IGN", 1) &&
      !(getenv("OPENR_SPF_MSBFS") && atoi(getenv("OPENR_SPF_MSBFS")) == 0) &&
      (uint64_t)((nq + 63) / 64) * g->E * 8 <= (1ull << 30)) {
    ms_ign_prev = q->dist;
    q->dist = DistPlan::BfsLds; // becomes MS-BFS just below
    q->ms_ign = true;
  }
  // many sources on a uniform metric: bit-parallel multi-source BFS
  // (OPENR_SPF_MSBFS=0 disables, =32 / =64 picks the batch width)
  if ((q->dist == DistPlan::BfsLds || q->dist == DistPlan::BfsGmem) &&
      V <= kMsThreads * kMsMaxK && (nq + helpers.size() >= 32 || !helpers.empty())) {
    const char* env = getenv("OPENR_SPF_MSBFS");
    int width = env ? atoi(env) : 64;
    if (width == 64 && 2 * (size_t)V * 8 > kLdsLimit) {
      width = 32; // the 64-bit frontier double buffer does not fit LDS
    }
    if ((width == 32 || width == 64) && 2 * (size_t)V * (width / 8) <= kLdsLimit) {
      q->dist = DistPlan::MsBfs;
      q->ms_bits = width;
      q->lds_bytes = 2 * (size_t)V * (width / 8); // frontier double buffer
      const uint32_t nrows = nq + (uint32_t)helpers.size();
      const uint32_t nbatch = (nrows + width - 1) / width;
      const uint32_t per_cu = (uint32_t)std::max<size_t>(
          1, std::min<size_t>(2048 / kMsThreads, kLdsLimit / std::max<size_t>(q->lds_bytes, 1)));
      q->grid = std::min<uint32_t>(nbatch, (uint32_t)g->num_cus * per_cu);
      if (q->nh == NhPlan::Rows) {
        q->nh = NhPlan::Levels;
      }
    }
  }
  if (q->ms_ign && q->dist != DistPlan::MsBfs) {
    q->dist = ms_ign_prev; // the MS-BFS plan did not apply: back to per-query SSSP
    q->ms_ign = false;
  }
  if (!helpers.empty() && !(q->dist == DistPlan::MsBfs && q->nh == NhPlan::Levels) &&
      !(few_rows && q->dist == DistPlan::Dstep && q->nh == NhPlan::Rows && q->dlds)) {
    return bail(fail(SPF_E_INVALID, "internal: helper sources outside the MS-BFS plan"));
  }
  if (zcand && !(q->dist == DistPlan::MsBfs && (!want_nh || q->nh == NhPlan::Levels))) {
    return bail(fail(SPF_E_INVALID, "internal: zero-metric plan outside MS-BFS"));
  }
  q->nrows = nq + (uint32_t)helpers.size();
  if (zcand) {
    // next hops: one table per variant; distances alone: one table closed
    // over every metric-0 half-edge
    q->zvars = want_nh ? (1u << zlinks.size()) : 1u;
    q->zscale = zc;
    q->znlinks = (uint32_t)zlinks.size();
    std::vector<uint32_t> zl;
    for (uint32_t j = 0; j < q->zvars; ++j) {
      q->zoff.push_back((uint32_t)(zl.size() / 2));
      for (uint32_t i = 0; i < zlinks.size(); ++i) {
        const ZeroLink& z = zlinks[i];
        const bool bfirst = want_nh && ((j >> i) & 1u);
        const bool afirst = want_nh && !((j >> i) & 1u);
        if (z.ab && !bfirst) {
          zl.push_back(z.a);
          zl.push_back(z.b);
        }
        if (z.ba && !afirst) {
          zl.push_back(z.b);
          zl.push_back(z.a);
        }
      }
    }
    q->zoff.push_back((uint32_t)(zl.size() / 2));
    for (const ZeroLink& z : zlinks) {
      zl.push_back(z.a);
      zl.push_back(z.b);
    }
    if (dev_upload_q(&q->d_zl, zl.data(), zl.size()) != SPF_OK) {
      return bail(fail(SPF_E_NOMEM, "zero-metric closure lists"));
    }
    if (want_nh) {
      if (pool_malloc((void**)&q->d_zvar, std::max<size_t>(nq, 16)) != hipSuccess) {
        return bail(fail(SPF_E_NOMEM, "zero-metric variants"));
      }
      // sources whose first hop may cost 0: the wide plan, rows copied in
      std::vector<uint32_t> fix;
      for (uint32_t i = 0; i < nq; ++i) {
        const uint32_t x = desc->sources[i];
        for (const ZeroLink& z : zlinks) {
          if ((x == z.a && z.ab) || (x == z.b && z.ba)) {
            fix.push_back(x);
            q->zfix_rows.push_back(i);
            break;
          }
        }
      }
      if (!fix.empty()) {
        spf_query_desc fd{};
        fd.num_queries = (uint32_t)fix.size();
        fd.sources = fix.data();
        fd.flags = SPF_F_NEXTHOPS | kQueryWideMasks;
        int fs = spf_query_create(g, &fd, &q->zfix);
        if (fs != SPF_OK) {
          return bail(fs);
        }
        if (q->zfix->dist != DistPlan::Wide) {
          return bail(fail(SPF_E_INVALID, "internal: zero-metric fix-up outside the wide plan"));
        }
      }
    }
  }

  if (hipSetDevice(g->device) != hipSuccess) {
    return bail(fail(SPF_E_DEVICE, "hipSetDevice failed"));
  }
  int s = SPF_OK;
  // every index array of the batch in ONE pooled block and ONE copy (a
  // RouteDb build creates small batches whose separate blocking uploads
  // cost more than their SPFs): sources, ignore lists, mask offsets / words,
  // the rows plan's node -> row map, each at a 256-byte aligned offset
  {
    size_t off = 0;
    auto seg = [&](size_t bytes) {
      const size_t o = off;
      off += (bytes + 255) & ~(size_t)255;
      return o;
    };
    const uint32_t total_ign = has_ign ? desc->ignore_offsets[nq] : 0;
    const size_t o_src = seg((size_t)q->nrows * 4);
    const size_t o_ioff = has_ign ? seg((size_t)(nq + 1) * 4) : 0;
    const size_t o_ign = has_ign ? seg((size_t)total_ign * 4) : 0;
    const size_t o_nhoff = want_nh ? seg((size_t)nq * 8) : 0;
    const size_t o_nhw = want_nh ? seg((size_t)nq * 4) : 0;
    const size_t o_nhboff = want_nh ? seg((size_t)nq * 8) : 0;
    const size_t o_nhb = want_nh ? seg((size_t)nq * 4) : 0;
    const size_t o_rowof = !row_of.empty() ? seg((size_t)V * 4) : 0;
    if (off) {
      std::vector<uint8_t> host(off, 0);
      std::memcpy(host.data() + o_src, desc->sources, (size_t)nq * 4);
      if (!helpers.empty()) {
        std::memcpy(host.data() + o_src + (size_t)nq * 4, helpers.data(), helpers.size() * 4);
      }
      if (has_ign) {
        std::memcpy(host.data() + o_ioff, desc->ignore_offsets, (size_t)(nq + 1) * 4);
        std::memcpy(host.data() + o_ign, desc->ignore_links, (size_t)total_ign * 4);
      }
      if (want_nh) {
        std::memcpy(host.data() + o_nhoff, q->nh_off.data(), (size_t)nq * 8);
        std::memcpy(host.data() + o_nhw, q->nh_w.data(), (size_t)nq * 4);
        std::memcpy(host.data() + o_nhboff, q->nhb_off.data(), (size_t)nq * 8);
        std::memcpy(host.data() + o_nhb, q->nh_b.data(), (size_t)nq * 4);
      }
      if (!row_of.empty()) {
        std::memcpy(host.data() + o_rowof, row_of.data(), (size_t)V * 4);
      }
      if (pool_malloc(&q->d_pack, off) != hipSuccess ||
          hipMemcpy(q->d_pack, host.data(), off, hipMemcpyHostToDevice) != hipSuccess) {
        return bail(fail(SPF_E_NOMEM, "batch index arrays"));
      }
      uint8_t* base = static_cast<uint8_t*>(q->d_pack);
      q->d_src = nq ? reinterpret_cast<uint32_t*>(base + o_src) : nullptr;
      if (has_ign) {
        q->d_ign_off = reinterpret_cast<uint32_t*>(base + o_ioff);
        q->d_ign = total_ign ? reinterpret_cast<uint32_t*>(base + o_ign) : nullptr;
      }
      if (want_nh && nq) {
        q->d_nh_off = reinterpret_cast<uint64_t*>(base + o_nhoff);
        q->d_nh_w = reinterpret_cast<uint32_t*>(base + o_nhw);
        q->d_nhb_off = reinterpret_cast<uint64_t*>(base + o_nhboff);
        q->d_nh_b = reinterpret_cast<uint32_t*>(base + o_nhb);
      }
      if (!row_of.empty()) {
        q->d_row_of = reinterpret_cast<int32_t*>(base + o_rowof);
      }
    }
  }
  if (q->dist == DistPlan::MsBfs && q->nh == NhPlan::Levels) {
    // 4-8 mask words first (the wide held kernel), then the rest (generic)
    std::vector<uint32_t> big;
    for (uint32_t i = 0; i < nq; ++i) {
      if (q->nh_w[i] > kNsHeldMax && q->nh_w[i] <= kNsHeldWide) {
        big.push_back(i);
      }
    }
    q->nmid = (uint32_t)big.size();
    for (uint32_t i = 0; i < nq; ++i) {
      if (q->nh_w[i] > kNsHeldWide) {
        big.push_back(i);
      }
    }
    q->nbig = (uint32_t)big.size();
    if (!big.empty() && dev_upload_q(&q->d_big, big.data(), big.size()) != SPF_OK) {
      return bail(fail(SPF_E_NOMEM, "next-hop source list"));
    }
    if (q->zvars == 0 && env_flag("OPENR_NL_V2", 1) && env_u32("OPENR_NL_ORDER", 0) != 1) {
      if (const int s = build_nl_v2(q, desc->sources, row_of); s != SPF_OK) {
        return bail(s);
      }
    }
    // OPENR_NL_ORDER=1: the held kernel's (source, chunk) items cut into 8
    // contiguous source ranges of equal cost (8 + neighbours per item), one
    // per XCD (hardware block b runs on XCD b % 8), source-major inside a
    // range: the rows an XCD's resident blocks read (a pod's RSW / FSW rows)
    // stay in its L2 instead of every XCD fetching nearly every row
    if (env_u32("OPENR_NL_ORDER", 0) == 1) {
      const uint32_t ht = env_u32("OPENR_NL_HT", 256);
      const uint32_t T = ht == 1024 ? 1024u : (ht == 512 ? 512u : 256u);
      const uint32_t nch = (V + 4 * T - 1) / (4 * T);
      double total = 0;
      for (uint32_t i = 0; i < nq; ++i) {
        if (q->nh_w[i] <= kNsHeldMax) {
          const uint32_t s = desc->sources[i];
          total += (double)nch * (8.0 + (g->nbr_off[s + 1] - g->nbr_off[s]));
        }
      }
      std::vector<std::vector<uint32_t>> lists(8);
      double acc = 0;
      for (uint32_t i = 0; i < nq; ++i) {
        if (q->nh_w[i] > kNsHeldMax) {
          continue;
        }
        const uint32_t s = desc->sources[i];
        const double cst = (double)nch * (8.0 + (g->nbr_off[s + 1] - g->nbr_off[s]));
        const uint32_t x = std::min<uint32_t>(7, (uint32_t)(8.0 * (acc + 0.5 * cst) / total));
        acc += cst;
        for (uint32_t c = 0; c < nch; ++c) {
          lists[x].push_back(i * nch + c);
        }
      }
      size_t maxlen = 0;
      for (const auto& l : lists) {
        maxlen = std::max(maxlen, l.size());
      }
      std::vector<uint32_t> order(8 * maxlen, kInf32);
      for (uint32_t x = 0; x < 8; ++x) {
        for (size_t i = 0; i < lists[x].size(); ++i) {
          order[i * 8 + x] = lists[x][i];
        }
      }
      if (!order.empty() && nq * (uint64_t)nch < 0xFFFFFFFFull) {
        if (dev_upload_q(&q->d_held_order, order.data(), order.size()) != SPF_OK) {
          return bail(fail(SPF_E_NOMEM, "next-hop work order"));
        }
        q->held_blocks = (uint32_t)order.size();
        q->held_nch = nch;
        q->held_t = T;
      }
    }
  }
  const size_t ntab = std::max<uint32_t>(1, q->zvars); // MS-BFS tables (zero-metric variants)
  if (q->dist == DistPlan::MsBfs) {
    if (pool_malloc((void**)&q->d_lvl, ntab * q->nrows * q->Vp8) != hipSuccess ||
        pool_malloc((void**)&q->d_flags, 16) != hipSuccess) {
      return bail(fail(SPF_E_NOMEM, "level rows"));
    }
    if (hipMemsetAsync(q->d_flags, 0, 16, g->stream) != hipSuccess) { // once: launches alternate words
      return bail(fail(SPF_E_DEVICE, "level flags"));
    }
    if (q->ms_ign) {
      q->ms_nbatch = (q->nrows + q->ms_bits - 1) / q->ms_bits;
      q->ms_nfw = (V + 31) / 32;
      if (pool_malloc((void**)&q->d_ms_mask, (size_t)q->ms_nbatch * g->E * 8) != hipSuccess ||
          pool_malloc((void**)&q->d_ms_flag, (size_t)q->ms_nbatch * q->ms_nfw * 4) !=
              hipSuccess) {
        return bail(fail(SPF_E_NOMEM, "ignored half-edge masks"));
      }
    }
  }
  if (want_nh) {
    // the SWAR next-hop kernels write the output layout themselves
    q->nl_swar = env_flag("OPENR_NL_SWAR", 1) || q->zvars;
    q->nh_direct = q->dist == DistPlan::MsBfs && q->nh == NhPlan::Levels && q->nl_swar;
    if (!q->narrow) {
      if (q->nh_total && pool_malloc((void**)&q->d_nh, q->nh_total * 8) != hipSuccess) {
        return bail(fail(SPF_E_NOMEM, "next-hop rows"));
      }
      q->d_nhb = reinterpret_cast<uint8_t*>(q->d_nh);
    } else {
      if (pool_malloc((void**)&q->d_nhb, q->nhb_total) != hipSuccess ||
          (!q->nh_direct && pool_malloc((void**)&q->d_nh, q->nh_total * 8) != hipSuccess)) {
        return bail(fail(SPF_E_NOMEM, "next-hop rows"));
      }
    }
  }
  const bool ex = q->dist == DistPlan::Exact;
  const bool wide = q->dist == DistPlan::Wide;
  const size_t dist_bytes = (ex || wide) ? (size_t)nq * V * 8 : ntab * q->nrows * q->Vp * 4;
  if (dist_bytes && pool_malloc(&q->d_dist, dist_bytes) != hipSuccess) {
    return bail(fail(SPF_E_NOMEM, "distance rows"));
  }
  if ((q->dist == DistPlan::SsspGmem || q->dist == DistPlan::BfsGmem ||
       q->dist == DistPlan::Dstep) &&
      pool_malloc((void**)&q->d_scratch,
                  std::max<size_t>((size_t)q->grid, q->dlds ? 2 * (size_t)q->dlds_grid : 0) * V *
                      4) != hipSuccess) {
    return bail(fail(SPF_E_NOMEM, "queue scratch"));
  }
  if (q->dlds && pool_malloc((void**)&q->d_ovf, ((size_t)q->nrows + 2) * 4) != hipSuccess) {
    return bail(fail(SPF_E_NOMEM, "overflow list"));
  }
  if (q->dist == DistPlan::MsDstep) {
    const size_t gv = (size_t)q->grid * V;
    if ((s = dev_upload_q(&q->d_perm, msd_perm.data(), msd_perm.size()))) {
      return bail(s);
    }
    if (pool_malloc((void**)&q->d_slab, gv * kMsdK * 4) != hipSuccess ||
        pool_malloc((void**)&q->d_msd, gv * 4 * 4) != hipSuccess) {
      return bail(fail(SPF_E_NOMEM, "multi-source slab"));
    }
  }
  if (ex && (size_t)nq * V) {
    if (pool_malloc((void**)&q->d_scratch, (size_t)nq * V * 8) != hipSuccess ||
        pool_malloc((void**)&q->d_order, (size_t)nq * V * 4) != hipSuccess) {
      return bail(fail(SPF_E_NOMEM, "exact-kernel scratch"));
    }
  }
  if (wide && (size_t)nq * V) {
    if (pool_malloc((void**)&q->d_scratch, (size_t)q->grid * wide_stride(V, g->nbw) * 4) !=
            hipSuccess ||
        (want_order && pool_malloc((void**)&q->d_key, (size_t)nq * V * 8) != hipSuccess)) {
      return bail(fail(SPF_E_NOMEM, "wide-plan scratch"));
    }
  }
  // what-if screen (OPENR_SPF_WHATIF_SCREEN=0 disables): batches with
  // ignore lists on the fast plans run one baseline SPF per distinct source
  // first; queries whose ignored links are all off the baseline's shortest
  // path DAG copy its rows instead of running
  const char* scr = getenv("OPENR_SPF_WHATIF_SCREEN");
  if (has_ign && !(scr && atoi(scr) == 0) &&
      (q->dist == DistPlan::SsspLds || q->dist == DistPlan::SsspGmem ||
       q->dist == DistPlan::Dstep)) {
    std::vector<uint32_t> base_srcs, base_of(nq);
    std::unordered_map<uint32_t, uint32_t> idx;
    for (uint32_t i = 0; i < nq; ++i) {
      auto it = idx.emplace(desc->sources[i], (uint32_t)base_srcs.size()).first;
      if (it->second == base_srcs.size()) {
        base_srcs.push_back(desc->sources[i]);
      }
      base_of[i] = it->second;
    }
    if (base_srcs.size() < nq) { // screening pays only if sources repeat
      spf_query_desc bd{};
      bd.num_queries = (uint32_t)base_srcs.size();
      bd.sources = base_srcs.data();
      bd.flags = desc->flags | kQueryWideMasks;
      if ((s = spf_query_create(g, &bd, &q->base)) ||
          (s = dev_upload_q(&q->d_base_of, base_of.data(), nq))) {
        return bail(s);
      }
      if (pool_malloc((void**)&q->d_skip, (size_t)nq * 4) != hipSuccess) {
        return bail(fail(SPF_E_NOMEM, "what-if screen flags"));
      }
      // repair mode: the K / ok bitmaps join the workgroup's LDS image
      // (positive metrics only: the K rule needs a DAG of tight edges)
      const size_t extra = 2 * (size_t)g->nbw * 4;
      if ((q->dist == DistPlan::SsspLds || q->dist == DistPlan::SsspGmem) && !g->n_zero &&
          q->lds_bytes + extra <= kLdsLimit && env_flag("OPENR_SPF_WHATIF_REPAIR", 1)) {
        q->repair = true;
        q->lds_bytes += extra;
        if (q->dist == DistPlan::SsspLds) {
          const uint32_t per_cu =
              std::max<uint32_t>(1, std::min<uint32_t>(4, kLdsLimit / q->lds_bytes));
          q->grid = std::min<uint32_t>(std::max<uint32_t>(nq, 1), (uint32_t)g->num_cus * per_cu);
        }
        if (!q->d_qctr && pool_malloc((void**)&q->d_qctr, 4) != hipSuccess) {
          return bail(fail(SPF_E_NOMEM, "what-if claim counter"));
        }
        if (env_flag("OPENR_SPF_WHATIF_WORKLIST", 1) &&
            pool_malloc((void**)&q->d_wl, ((size_t)nq + 2) * 4) != hipSuccess) {
          return bail(fail(SPF_E_NOMEM, "what-if work list"));
        }
        // queries whose failed link leaves the source: their own BFS launch
        // on a uniform-metric area (spf_whatif_heavy_kernel)
        // (both kernels read v's out-edges as its in-edges: every half-edge
        // paired with an up reverse)
        const bool uni = (desc->flags & SPF_F_UNIT_METRIC) || g->uniform;
        const size_t wh_lds = (3 * (size_t)g->V + 1 + (g->V + 31) / 32) * 4;
        if (uni && g->paired && wh_lds <= kLdsLimit && desc->ignore_offsets &&
            env_flag("OPENR_SPF_WHATIF_HEAVY", 1)) {
          for (uint32_t i = 0; i < nq; ++i) {
            const uint32_t s0 = desc->sources[i];
            if (g->nbr_off[s0 + 1] - g->nbr_off[s0] > 64 * kWhMaxW) {
              continue; // wider masks than the kernel keeps in registers
            }
            bool hit = false;
            for (uint32_t j = desc->ignore_offsets[i]; j < desc->ignore_offsets[i + 1] && !hit; ++j) {
              for (uint32_t e = g->row[s0]; e < g->row[s0 + 1]; ++e) {
                if (g->link[e] == desc->ignore_links[j]) {
                  hit = true;
                  break;
                }
              }
            }
            if (hit) {
              q->wh_cand.push_back(i);
            }
          }
          // candidates whose every ignored link leaves the source (or names
          // no link): the first-hop form over one nested batch of the
          // sources' neighbour rows (spf_whatif_firsthop_kernel); the rest
          // keep the pull / heavy kernel
          q->wh_pull_cand.clear();
          if (!(desc->flags & kQueryNoFirstHop) && env_flag("OPENR_SPF_WHATIF_FIRSTHOP", 1)) {
            const std::vector<uint32_t>& heads = g->col_orig.empty() ? g->col : g->col_orig;
            std::unordered_map<uint32_t, uint32_t> hop_of;
            std::vector<uint32_t> fh_q, fh_h, hop_s, hop_cnt, hop_off, hop_nodes;
            std::vector<std::vector<uint32_t>> hop_links;
            for (uint32_t i : q->wh_cand) {
              const uint32_t s0 = desc->sources[i];
              bool pure = true;
              for (uint32_t j = desc->ignore_offsets[i]; j < desc->ignore_offsets[i + 1] && pure;
                   ++j) {
                const uint32_t l = desc->ignore_links[j];
                bool at = l >= g->L;
                for (uint32_t e = g->row[s0]; e < g->row[s0 + 1] && !at; ++e) {
                  at = g->link[e] == l;
                }
                pure = at;
              }
              if (!pure) {
                q->wh_pull_cand.push_back(i);
                continue;
              }
              auto it = hop_of.find(s0);
              if (it == hop_of.end()) {
                std::vector<uint32_t> nb, links;
                for (uint32_t e = g->row[s0]; e < g->row[s0 + 1]; ++e) {
                  if (heads[e] != s0) {
                    nb.push_back(heads[e]);
                  }
                  links.push_back(g->link[e]);
                }
                std::sort(nb.begin(), nb.end());
                nb.erase(std::unique(nb.begin(), nb.end()), nb.end());
                std::sort(links.begin(), links.end());
                links.erase(std::unique(links.begin(), links.end()), links.end());
                if (nb.empty()) {
                  q->wh_pull_cand.push_back(i);
                  continue;
                }
                it = hop_of.emplace(s0, (uint32_t)hop_s.size()).first;
                hop_s.push_back(s0);
                hop_cnt.push_back((uint32_t)nb.size());
                hop_off.push_back((uint32_t)hop_nodes.size());
                hop_nodes.insert(hop_nodes.end(), nb.begin(), nb.end());
                hop_links.push_back(std::move(links));
              }
              fh_q.push_back(i);
              fh_h.push_back(it->second);
            }
            std::vector<uint32_t> hop_row0;
            if (!fh_q.empty()) {
              // (a) the plain bit-parallel BFS with the source non-transit in
              // its neighbours' batches (MsBfsArgs::blocked): each source's
              // neighbours padded to whole 64-row batches
              std::vector<uint32_t> hsrc, unit32; // unit32: blocked node per 32 rows
              for (size_t h = 0; h < hop_s.size(); ++h) {
                hop_row0.push_back((uint32_t)hsrc.size());
                const uint32_t* nb = hop_nodes.data() + hop_off[h];
                const uint32_t padded = (hop_cnt[h] + 63) / 64 * 64;
                for (uint32_t k = 0; k < padded; ++k) {
                  hsrc.push_back(nb[k < hop_cnt[h] ? k : 0]);
                }
                unit32.insert(unit32.end(), padded / 32, hop_s[h]);
              }
              spf_query_desc hd{};
              hd.num_queries = (uint32_t)hsrc.size();
              hd.sources = hsrc.data();
              hd.flags = SPF_F_UNIT_METRIC | kQueryNoFirstHop;
              if ((s = spf_query_create(g, &hd, &q->hop))) {
                return bail(s);
              }
              spf_query* hq = q->hop;
              if (hq->dist == DistPlan::MsBfs && hq->nh == NhPlan::None && !hq->zvars &&
                  hq->nrows == hq->nq && (hq->ms_bits == 64 || hq->ms_bits == 32) &&
                  env_flag("OPENR_SPF_WHATIF_FIRSTHOP_BLOCKED", 1)) {
                std::vector<uint32_t> blk;
                const uint32_t per = hq->ms_bits / 32;
                for (size_t u = 0; u < unit32.size(); u += per) {
                  blk.push_back(unit32[u]);
                }
                if ((s = dev_upload_q(&hq->d_ms_blocked, blk.data(), blk.size()))) {
                  return bail(s);
                }
              } else {
                // (b) any other plan: every link of the source ignored, rows
                // unpadded
                free_query(q->hop);
                q->hop = nullptr;
                hsrc.clear();
                hop_row0.clear();
                std::vector<uint32_t> hoff{0}, hign;
                for (size_t h = 0; h < hop_s.size(); ++h) {
                  hop_row0.push_back((uint32_t)hsrc.size());
                  for (uint32_t k = 0; k < hop_cnt[h]; ++k) {
                    hsrc.push_back(hop_nodes[hop_off[h] + k]);
                    hign.insert(hign.end(), hop_links[h].begin(), hop_links[h].end());
                    hoff.push_back((uint32_t)hign.size());
                  }
                }
                hd.num_queries = (uint32_t)hsrc.size();
                hd.sources = hsrc.data();
                hd.ignore_offsets = hoff.data();
                hd.ignore_links = hign.data();
                if ((s = spf_query_create(g, &hd, &q->hop))) {
                  return bail(s);
                }
              }
              std::vector<uint32_t> pack;
              for (const auto* v : {&fh_q, &fh_h, &hop_row0, &hop_cnt, &hop_off, &hop_nodes}) {
                pack.insert(pack.end(), v->begin(), v->end());
              }
              if ((s = dev_upload_q(&q->d_fh, pack.data(), pack.size()))) {
                return bail(s);
              }
              q->nfh = (uint32_t)fh_q.size();
              q->nhop = (uint32_t)hop_row0.size();
              q->nhop_nodes = (uint32_t)hop_nodes.size();
            }
          } else {
            q->wh_pull_cand = q->wh_cand;
          }
          q->wh_pull = g->d_sell != nullptr && env_flag("OPENR_SPF_WHATIF_PULL", 1);
          for (uint32_t i : q->wh_pull_cand) {
            if (desc->ignore_offsets[i + 1] - desc->ignore_offsets[i] > kWpIgnE / 2) {
              q->wh_pull = false;
            }
          }
          if (!q->wh_cand.empty()) {
            std::vector<uint8_t> mark(nq, 0);
            for (uint32_t i : q->wh_cand) {
              mark[i] = 1;
            }
            if ((s = dev_upload_q(&q->d_wh_mark, mark.data(), mark.size()))) {
              return bail(s);
            }
          }
          if (!q->wh_pull_cand.empty()) {
            if ((s = dev_upload_q(&q->d_wh_cand, q->wh_pull_cand.data(), q->wh_pull_cand.size()))) {
              return bail(s);
            }
            if (pool_malloc((void**)&q->d_wh_lstart,
                            q->wh_pull_cand.size() * ((size_t)g->V + 1) * 4) != hipSuccess) {
              return bail(fail(SPF_E_NOMEM, "what-if heavy level segments"));
            }
          }
          if (!q->wh_pull_cand.empty() || q->nfh) {
            // high priority: its two big-LDS workgroups must be placed before
            // the SSSP's hundreds fill every CU (they waited ~0.6 ms, r05an)
            int plo = 0, phi = 0;
            (void)hipDeviceGetStreamPriorityRange(&plo, &phi);
            if (hipStreamCreateWithPriority(&q->wh_stream, hipStreamNonBlocking, phi) != hipSuccess ||
                ev_get(&q->wh_ev0) != hipSuccess || ev_get(&q->wh_ev1) != hipSuccess ||
                ev_get(&q->wh_ev2) != hipSuccess) {
              return bail(fail(SPF_E_DEVICE, "what-if heavy stream"));
            }
          }
        }
      }
    }
  }
  if (ev_get(&q->ev0) != hipSuccess || ev_get(&q->ev1) != hipSuccess ||
      ev_get(&q->evm) != hipSuccess) {
    return bail(fail(SPF_E_DEVICE, "hipEventCreate failed"));
  }
  *out = q;
  return SPF_OK;
}

int spf_query_destroy(spf_query* q) {
  SPF_ABI_RANGE("spf_query_destroy");
  if (q) {
    if (const uint32_t n = q->live_tables.load(std::memory_order_relaxed)) {
      return fail(SPF_E_INVALID, "spf_query_destroy: " + std::to_string(n) +
                                     " live route tables over this query (destroy them first)");
    }
  }
  free_query(q);
  return SPF_OK;
}

} // extern "C"

namespace {

template <int WMAX, bool UNIT, bool IGN, bool GMEM>
int launch_sssp(spf_query* q) {
  spf_graph* g = q->g;
  SsspArgs a;
  a.row = g->d_row;
  a.col = g->d_col;
  a.wout = g->d_wout;
  a.win = g->d_win;
  a.link = g->d_link;
  a.rev = g->d_rev;
  a.slot = g->d_slot;
  a.trbits = g->d_tr;
  a.src = q->d_src;
  a.ign_off = q->d_ign_off;
  a.ign = q->d_ign;
  a.nh_off = q->d_nh_off;
  a.nh_w = q->d_nh_w;
  a.dist_out = (uint32_t*)q->d_dist;
  a.nh_out = q->d_nh;
  a.gscratch = q->d_scratch;
  a.V = g->V;
  a.Vp = q->Vp;
  a.nbw = g->nbw;
  a.nq = q->nq;
  a.G = g->G;
  a.ign_cap = q->ign_cap;
  a.skip = q->d_skip;
  if (q->repair) {
    const spf_query* b = q->base;
    if (b->Vp != q->Vp || b->nq == 0) {
      return fail(SPF_E_INVALID, "baseline row layout differs");
    }
    a.base_dist = (const uint32_t*)b->d_dist;
    a.base_nh = b->d_nh;
    a.base_nh_off = b->d_nh_off;
    a.base_of = q->d_base_of;
    a.link_half = g->d_link_half;
    a.L = g->L;
    a.qctr = q->d_qctr;
    HIP_TRY(hipMemsetAsync(q->d_qctr, 0, 4, g->stream));
    if (q->d_wl) {
      SPF_LAUNCH(spf_whatif_worklist_kernel, dim3(1), dim3(1024), 0, g->stream, q->d_skip,
                 q->nq, q->d_wl);
      HIP_TRY(hipGetLastError());
      a.wl = q->d_wl;
    }
    if (env_flag("OPENR_SPF_WHATIF_STATS", 0)) {
      HIP_TRY(hipMalloc((void**)&a.stats, 8 * sizeof(unsigned long long)));
      HIP_TRY(hipMemsetAsync(a.stats, 0, 8 * sizeof(unsigned long long), g->stream));
    }
  }
  auto kern = spf_sssp_kernel<WMAX, UNIT, IGN, GMEM>;
  HIP_TRY(hipFuncSetAttribute(
      (const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
      (int)q->lds_bytes));
  SPF_LAUNCH_AS("spf_sssp_kernel", 
      kern, dim3(q->grid), dim3(kBlock), q->lds_bytes, g->stream, a);
  HIP_TRY(hipGetLastError());
  if (q->wh_pending) {
    // the heavy what-if queries ran beside it: later work waits for them
    HIP_TRY(hipStreamWaitEvent(g->stream, q->wh_ev1, 0));
    q->wh_pending = false;
  }
  if (a.stats) {
    unsigned long long h[8];
    HIP_TRY(hipStreamSynchronize(g->stream));
    HIP_TRY(hipMemcpy(h, a.stats, sizeof(h), hipMemcpyDeviceToHost));
    HIP_TRY(hipFree(a.stats));
    fprintf(stderr,
            "[whatif stats] nq=%u grid=%u repaired=%llu scratch=%llu K=%llu rounds=%llu "
            "ticks(100MHz, summed over queries) copy=%llu init=%llu rounds=%llu output=%llu\n",
            q->nq, q->grid, h[0], h[1], h[2], h[3], h[4], h[5], h[6], h[7]);
  }
  return SPF_OK;
}

template <int WMAX>
int dispatch_flags(spf_query* q, bool unit, bool ign, bool gmem) {
  if (unit) {
    if (ign) {
      return gmem ? launch_sssp<WMAX, true, true, true>(q)
                  : launch_sssp<WMAX, true, true, false>(q);
    }
    return gmem ? launch_sssp<WMAX, true, false, true>(q)
                : launch_sssp<WMAX, true, false, false>(q);
  }
  if (ign) {
    return gmem ? launch_sssp<WMAX, false, true, true>(q)
                : launch_sssp<WMAX, false, true, false>(q);
  }
  return gmem ? launch_sssp<WMAX, false, false, true>(q)
              : launch_sssp<WMAX, false, false, false>(q);
}

template <int WMAX, bool IGN, uint32_t BS>
int launch_dstep_t(spf_query* q) {
  spf_graph* g = q->g;
  DstepArgs d;
  SsspArgs& a = d.s;
  a.row = g->d_row;
  a.col = g->d_col;
  a.wout = g->d_wout;
  a.win = g->d_win;
  a.link = g->d_link;
  a.rev = g->d_rev;
  a.slot = g->d_slot;
  a.trbits = g->d_tr;
  a.src = q->d_src;
  a.ign_off = q->d_ign_off;
  a.ign = q->d_ign;
  a.nh_off = q->d_nh_off;
  a.nh_w = q->d_nh_w;
  a.dist_out = (uint32_t*)q->d_dist;
  a.nh_out = q->d_nh;
  a.gscratch = q->d_scratch;
  a.V = g->V;
  a.Vp = q->Vp;
  a.nbw = g->nbw;
  a.nq = q->nrows; // the batch + its helper sources (few-source rows plan)
  a.G = g->G;
  a.ign_cap = q->dstep_ign_cap;
  a.skip = q->d_skip;
  // lanes per node: fewer than the median degree, so more nodes (and more
  // independent HBM gathers) are in flight per CU (4: measured on the 100k
  // WAN for the PULL pass of next-hop runs and for the push-only runs with
  // 16-byte edge chunks); OPENR_SPF_DSTEP_G overrides
  uint32_t G = 4;
  if (const char* env = getenv("OPENR_SPF_DSTEP_G")) {
    const int x = atoi(env);
    if (x == 1 || x == 2 || x == 4 || x == 8 || x == 16 || x == 32 || x == 64) {
      G = (uint32_t)x;
    }
  }
  a.G = G;
  d.shift = q->dstep_shift;
  d.fshift = q->dstep_fshift;
  d.noret = q->dstep_noret;
  if (WMAX == 0 && q->dstep_pack && g->cw_bits) {
    d.cw = g->d_cw;
    d.cwbits = g->cw_bits;
    d.cwvec = q->dstep_pack == 2;
  }
  auto kern = q->dstep_lbk ? spf_dstep_kernel<WMAX, IGN, BS, true>
                           : spf_dstep_kernel<WMAX, IGN, BS, false>;
  if constexpr (WMAX == 0) {
    if (q->dstep_lbk && d.cwvec && (d.noret & 3u) == 3u) {
      kern = spf_dstep_kernel<WMAX, IGN, BS, true, false, true>;
      if (q->nrows > q->grid) {
        if (!q->d_qctr) {
          HIP_TRY(pool_malloc((void**)&q->d_qctr, 4));
        }
        HIP_TRY(hipMemsetAsync(q->d_qctr, 0, 4, g->stream));
        d.qctr = q->d_qctr;
      }
    }
  }
  if (q->dlds) {
    // after spf_dlds_kernel: only the sources it flagged
    d.qcount = q->d_ovf;
    d.qlist = q->d_ovf + 2;
  }
  const size_t lds = q->lds_bytes;
  HIP_TRY(hipFuncSetAttribute(
      (const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
      (int)lds));
  const char* st_env = getenv("OPENR_SPF_DSTEP_STATS");
  if (st_env && atoi(st_env) == 1) {
    HIP_TRY(hipMalloc((void**)&d.stats, 8 * sizeof(unsigned long long)));
    HIP_TRY(hipMemsetAsync(d.stats, 0, 8 * sizeof(unsigned long long), g->stream));
  }
  SPF_LAUNCH_AS("spf_dstep_kernel", kern, dim3(q->grid), dim3(BS), lds, g->stream, d);
  HIP_TRY(hipGetLastError());
  if (d.stats) {
    unsigned long long h[8];
    HIP_TRY(hipStreamSynchronize(g->stream));
    HIP_TRY(hipMemcpy(h, d.stats, sizeof(h), hipMemcpyDeviceToHost));
    HIP_TRY(hipFree(d.stats));
    fprintf(stderr,
            "[dstep stats] nq=%u expand=%llu edges=%llu filtered=%llu gathers=%llu "
            "atomics=%llu improved=%llu rounds=%llu refreshed=%llu\n",
            q->nq, h[0], h[1], h[2], h[3], h[4], h[5], h[6], h[7]);
  }
  return SPF_OK;
}

template <uint32_t BS>
int launch_dstep_bs(spf_query* q) {
  const bool ign = q->has_ign;
  switch (q->wmax) {
  case 0:
    return ign ? launch_dstep_t<0, true, BS>(q) : launch_dstep_t<0, false, BS>(q);
  case 1:
    return ign ? launch_dstep_t<1, true, BS>(q) : launch_dstep_t<1, false, BS>(q);
  case 4:
    return ign ? launch_dstep_t<4, true, BS>(q) : launch_dstep_t<4, false, BS>(q);
  default:
    return ign ? launch_dstep_t<16, true, BS>(q) : launch_dstep_t<16, false, BS>(q);
  }
}

int launch_dlds(spf_query* q) {
  spf_graph* g = q->g;
  DldsArgs a{};
  a.row = g->d_row;
  a.cw = g->d_cw;
  a.trbits = g->d_tr;
  a.src = q->d_src;
  a.dist_out = (uint32_t*)q->d_dist;
  a.gscratch = q->d_scratch;
  a.ovf_n = q->d_ovf;
  a.qctr = q->d_ovf + 1;
  a.ovf_list = q->d_ovf + 2;
  a.V = g->V;
  a.Vp = q->Vp;
  a.nq = q->nrows; // the batch + its helper sources (few-source rows plan)
  a.cwbits = g->cw_bits;
  a.wshift = q->dlds_shift;
  if (!g->d_cw || !g->cw_bits) {
    return fail(SPF_E_INVALID, "internal: LDS-row plan without packed edges");
  }
  HIP_TRY(hipMemsetAsync(q->d_ovf, 0, 8, g->stream));
  const char* st_env = getenv("OPENR_SPF_DSTEP_STATS");
  if (st_env && atoi(st_env) == 1) {
    HIP_TRY(hipMalloc((void**)&a.stats, 8 * sizeof(unsigned long long)));
    HIP_TRY(hipMemsetAsync(a.stats, 0, 8 * sizeof(unsigned long long), g->stream));
  }
  // lanes per node (OPENR_SPF_DSTEP_LG 1/2/4/8) and the two-node prefetch
  // (OPENR_SPF_DSTEP_LPF=0 disables)
  const bool pf = env_flag("OPENR_SPF_DSTEP_LPF", 1);
  auto kern = pf ? spf_dlds_kernel<1024, 4, true> : spf_dlds_kernel<1024, 4, false>;
  switch (env_u32("OPENR_SPF_DSTEP_LG", 4)) {
  case 1:
    kern = pf ? spf_dlds_kernel<1024, 1, true> : spf_dlds_kernel<1024, 1, false>;
    break;
  case 2:
    kern = pf ? spf_dlds_kernel<1024, 2, true> : spf_dlds_kernel<1024, 2, false>;
    break;
  case 8:
    kern = pf ? spf_dlds_kernel<1024, 8, true> : spf_dlds_kernel<1024, 8, false>;
    break;
  default:
    break;
  }
  HIP_TRY(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)q->dlds_lds));
  SPF_LAUNCH_AS("spf_dlds_kernel", kern, dim3(q->dlds_grid), dim3(1024), q->dlds_lds, g->stream, a);
  HIP_TRY(hipGetLastError());
  if (a.stats) {
    unsigned long long h[8];
    uint32_t novf = 0;
    HIP_TRY(hipStreamSynchronize(g->stream));
    HIP_TRY(hipMemcpy(h, a.stats, sizeof(h), hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(&novf, q->d_ovf, 4, hipMemcpyDeviceToHost));
    HIP_TRY(hipFree(a.stats));
    fprintf(stderr,
            "[dlds stats] nq=%u expand=%llu edges=%llu improving=%llu lowered=%llu "
            "buckets=%llu requeued=%llu overflowed=%u\n",
            q->nq, h[0], h[1], h[4], h[5], h[6], h[7], novf);
  }
  return SPF_OK;
}

// 1024-thread workgroups: one per CU with the LDS bucket image (2 when the
// buckets come from the distance row)
int launch_dstep(spf_query* q) {
  return q->dstep_bs == 512 ? launch_dstep_bs<512>(q) : launch_dstep_bs<1024>(q);
}

int launch_msdstep(spf_query* q) {
  spf_graph* g = q->g;
  MsdArgs a;
  a.row = g->d_row;
  a.col = g->d_col;
  a.wout = g->d_wout;
  a.trbits = g->d_tr;
  a.src = q->d_src;
  a.perm = q->d_perm;
  a.dist_out = (uint32_t*)q->d_dist;
  a.slab = q->d_slab;
  const size_t gv = (size_t)q->grid * g->V;
  a.pend = q->d_msd;
  a.qa = q->d_msd + gv;
  a.qb = q->d_msd + 2 * gv;
  a.qm = q->d_msd + 3 * gv;
  a.V = g->V;
  a.Vp = q->Vp;
  a.nbw = g->nbw;
  a.nbatch = q->msd_nbatch;
  a.shift = q->dstep_shift;
  auto kern = spf_msdstep_kernel<1024>;
  HIP_TRY(hipFuncSetAttribute(
      (const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
      (int)q->lds_bytes));
  SPF_LAUNCH_AS("spf_msdstep_kernel", kern, dim3(q->grid), dim3(1024), q->lds_bytes, g->stream, a);
  HIP_TRY(hipGetLastError());
  return SPF_OK;
}

int launch_bfs(spf_query* q, bool unit) {
  spf_graph* g = q->g;
  BfsArgs a;
  a.row = g->d_row;
  a.col = g->d_col;
  a.trbits = g->d_tr;
  a.src = q->d_src;
  a.dist_out = (uint32_t*)q->d_dist;
  a.gscratch = q->d_scratch;
  a.V = g->V;
  a.Vp = q->Vp;
  a.nbw = g->nbw;
  a.nq = q->nq;
  a.E = g->E;
  a.G = g->G;
  a.scale = unit ? 1u : g->uniform;
  const bool gmem = q->dist == DistPlan::BfsGmem;
  auto kern = gmem ? spf_bfs_kernel<true> : spf_bfs_kernel<false>;
  HIP_TRY(hipFuncSetAttribute(
      (const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
      (int)q->lds_bytes));
  SPF_LAUNCH_AS("spf_bfs_kernel", 
      kern, dim3(q->grid), dim3(kBlock), q->lds_bytes, g->stream, a);
  HIP_TRY(hipGetLastError());
  return SPF_OK;
}

int launch_nh_rows(spf_query* q, bool unit) {
  spf_graph* g = q->g;
  NhRowsArgs a;
  a.nbr_off = g->d_nbr_off;
  a.nbrs = g->d_nbrs;
  a.nbr_w = g->d_nbr_w;
  a.trbits = g->d_tr;
  a.src = q->d_src;
  a.row_of = q->d_row_of;
  a.dist = (const uint32_t*)q->d_dist;
  a.nh_off = q->d_nh_off;
  a.nh_w = q->d_nh_w;
  a.nh_out = q->d_nh;
  a.V = g->V;
  a.Vp = q->Vp;
  a.nq = q->nq;
  a.nchunks = (g->V + kNhChunk - 1) / kNhChunk;
  a.unit = unit ? 1 : 0;
  const uint64_t blocks = (uint64_t)a.nchunks * q->nq;
  if (blocks > 0x7FFFFFFFull) {
    return fail(SPF_E_UNSUPPORTED, "batch too large for the next-hop pass");
  }
  SPF_LAUNCH(
      spf_nh_rows_kernel, dim3((uint32_t)blocks), dim3(kNhThreads), 0,
      g->stream, a);
  HIP_TRY(hipGetLastError());
  return SPF_OK;
}

// distances below level 255 written by the next-hop pass from the level
// rows (OPENR_MS_LVL_ONLY=0: by the BFS).  The BFS stores one 4-byte
// distance per (source, node) bit as it appears, scattered over 64 rows;
// the next-hop pass already reads each source's level row in order and
// writes them as 16-byte runs: fabric msbfs 0.228 -> 0.155 ms, next hops
// 0.451 -> 0.499 ms, step 0.691 -> 0.666 ms (profiles/r03w)
inline bool lvl_only(const spf_query* q) {
  // (the byte pass chosen when the query was created, q->nl_swar -- not the
  // environment at run time, which could pair the BFS's skipped distance
  // stores with a next-hop kernel that does not write them)
  return q->nh == NhPlan::Levels && !q->zvars && q->nl_swar &&
         env_flag("OPENR_MS_LVL_ONLY", 1);
}

int launch_msbfs(spf_query* q, bool unit) {
  spf_graph* g = q->g;
  hipStream_t st = q->stream_override ? q->stream_override : g->stream;
  MsBfsArgs a;
  a.row = g->d_row;
  a.col = g->d_col;
  const bool sell = g->d_sell && env_flag("OPENR_MS_SELL", 1);
  a.sell4 = g->d_sell;
  a.sell_off = g->d_sell_off;
  a.trbits = g->d_tr;
  a.src = q->d_src;
  a.dist_out = (uint32_t*)q->d_dist;
  a.lvl_out = q->d_lvl;
  a.flags = q->d_flags;
  a.V = g->V;
  a.Vp = q->Vp;
  a.Vp8 = q->Vp8;
  a.nq = q->nrows; // the batch + its helper sources
  a.scale = unit ? 1u : (q->zvars ? q->zscale : g->uniform);
  a.wrec = env_flag("OPENR_MS_WREC", 0); // measured slower (0.212 -> 0.232 ms, profiles/r03g)
  a.zlist = nullptr;
  a.nz = 0;
  a.lvl_only = lvl_only(q) ? 1u : 0u;
  a.norec = env_u32("OPENR_MS_NOREC", 0);
  a.blocked = q->d_ms_blocked;
  q->ms_par ^= 1u;
  a.flags = q->d_flags + q->ms_par;
  a.flags_clear = q->d_flags + (q->ms_par ^ 1u);
  if (q->ms_ign) {
    HIP_TRY(hipMemsetAsync(q->d_ms_mask, 0, (size_t)q->ms_nbatch * g->E * 8, st));
    HIP_TRY(hipMemsetAsync(q->d_ms_flag, 0, (size_t)q->ms_nbatch * q->ms_nfw * 4, st));
    if (q->nq) {
      SPF_LAUNCH(spf_ms_ign_kernel, dim3(q->nq), dim3(256), 0, st, q->d_ign_off,
                         q->d_ign, g->d_link_half, g->d_col, g->d_rev, g->L,
                         (uint32_t)q->ms_bits, g->E, q->ms_nfw, q->d_ms_mask, q->d_ms_flag);
      HIP_TRY(hipGetLastError());
    }
    a.ign_mask = q->d_ms_mask;
    a.ign_flag = q->d_ms_flag;
    a.E = g->E;
    a.nfw = q->ms_nfw;
  }
  const uint32_t K = (g->V + kMsThreads - 1) / kMsThreads;
  const void* kern = nullptr;
  // OPENR_MS_GEN=1: the general instance for every batch (A/B of the plain one)
  const bool gen = q->ms_ign || a.wrec || q->zvars || env_flag("OPENR_MS_GEN", 0);
#define MS_PICK(MT, KM)                                                                      \
  kern = gen ? (sell ? (const void*)spf_msbfs_kernel<MT, KM, true, true>                     \
                     : (const void*)spf_msbfs_kernel<MT, KM, false, true>)                   \
             : (sell ? (const void*)spf_msbfs_kernel<MT, KM, true, false>                    \
                     : (const void*)spf_msbfs_kernel<MT, KM, false, false>)
  if (q->ms_bits == 64) {
    if (K <= 4) {
      MS_PICK(uint64_t, 4);
    } else if (K <= 8) {
      MS_PICK(uint64_t, 8);
    } else if (K <= 10 && env_flag("OPENR_MS_K10", 1)) {
      // the 10k fabric (K = 10): the plain instance spills 2 VGPRs, not 24
      MS_PICK(uint64_t, 10);
    } else if (K <= 12) {
      MS_PICK(uint64_t, 12);
    } else {
      MS_PICK(uint64_t, 16);
    }
  } else {
    if (K <= 4) {
      MS_PICK(uint32_t, 4);
    } else if (K <= 8) {
      MS_PICK(uint32_t, 8);
    } else if (K <= 12) {
      MS_PICK(uint32_t, 12);
    } else if (K <= 16) {
      MS_PICK(uint32_t, 16);
    } else {
      MS_PICK(uint32_t, 20);
    }
  }
#undef MS_PICK
  // a block of a sharded table (few batches): split each batch over P
  // workgroups when P >= 2 of them fit beside one another (OPENR_MS_COOP)
  q->coop_p = 0;
  // opt-in (OPENR_MS_COOP=1): measured slower than one workgroup per batch at
  // every rank size (N = 8 block: 0.122 vs 0.117 ms; with the row stores off
  // 0.122 vs 0.064 ms, profiles/r05u): a level's barrier, acquire and frontier
  // reload cost ~7 us against ~8 us of pull work split P ways
  if (!gen && !a.blocked && q->ms_bits == 64 && sell && q->zvars == 0 &&
      g->V <= 8u * kMsThreads * 2u &&
      env_flag("OPENR_MS_COOP", 0)) {
    const uint32_t nbatch = (q->nrows + 63) / 64;
    const void* ck = (const void*)spf_msbfs_coop_kernel<8>;
    const size_t clds = (size_t)g->V * 8;
    int per_cu = 0;
    if (nbatch && hipFuncSetAttribute(ck, hipFuncAttributeMaxDynamicSharedMemorySize, (int)clds) ==
            hipSuccess &&
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, ck, kMsThreads, clds) == hipSuccess &&
        per_cu > 0) {
      const uint32_t cap = (uint32_t)per_cu * (uint32_t)g->num_cus;
      const uint32_t pmax = std::max<uint32_t>(1, std::min<uint32_t>(16, env_u32("OPENR_MS_COOP_P", 8)));
      uint32_t P = std::min<uint32_t>(pmax, cap / nbatch);
      // each part owns whole 1,024-node slots: no more parts than slots
      P = std::min<uint32_t>(P, (g->V + kMsThreads - 1) / kMsThreads);
      if (P >= 2) {
        const size_t xb = (size_t)nbatch * 2 * g->V * 8;
        const size_t need = xb + (size_t)nbatch * 4 + (size_t)nbatch * 2 * P * 4 + 16;
        if (q->d_coop && q->coop_bytes < need) {
          HIP_TRY(hipStreamSynchronize(st));
          pool_free(q->d_coop);
          q->d_coop = nullptr;
        }
        if (!q->d_coop) {
          HIP_TRY(pool_malloc(&q->d_coop, need));
          q->coop_bytes = need;
          HIP_TRY(hipMemsetAsync(q->d_coop, 0, need, st));
        }
        MsCoopArgs c;
        c.a = a;
        c.xbuf = reinterpret_cast<uint64_t*>(q->d_coop);
        c.cnt = reinterpret_cast<uint32_t*>(static_cast<char*>(q->d_coop) + xb);
        c.anyv = c.cnt + nbatch;
        c.err = c.anyv + (size_t)nbatch * 2 * P;
        c.P = P;
        HIP_TRY(hipMemsetAsync(c.cnt, 0, (size_t)nbatch * 4, st));
        void* cargs[] = {&c};
        spf_note_launch("spf_msbfs_coop_kernel");
        const hipError_t le = hipLaunchCooperativeKernel(ck, dim3(nbatch * P), dim3(kMsThreads),
                                                         cargs, (unsigned)clds, st);
        if (le == hipSuccess) {
          q->coop_p = P;
          return SPF_OK;
        }
        (void)hipGetLastError(); // not co-resident: the plain kernel below
      }
    }
  }
  HIP_TRY(hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)q->lds_bytes));
  const uint32_t ntab = std::max<uint32_t>(1, q->zvars);
  for (uint32_t j = 0; j < ntab; ++j) {
    if (q->zvars) { // zero-metric variant j: its own table and closure pairs
      a.dist_out = (uint32_t*)q->d_dist + (size_t)j * q->nrows * q->Vp;
      a.lvl_out = q->d_lvl + (size_t)j * q->nrows * q->Vp8;
      a.zlist = q->d_zl + 2 * (size_t)q->zoff[j];
      a.nz = q->zoff[j + 1] - q->zoff[j];
    }
    void* args[] = {&a};
    spf_note_launch("spf_msbfs_kernel");
    HIP_TRY(hipLaunchKernel(kern, dim3(q->grid), dim3(kMsThreads), args,
                            q->lds_bytes, st));
    HIP_TRY(hipGetLastError());
  }
  if (q->zvars && q->d_zvar) {
    ZvarArgs z;
    z.row = g->d_row;
    z.col = g->d_col;
    z.win = g->d_win;
    z.trbits = g->d_tr;
    z.src = q->d_src;
    z.dist = (const uint32_t*)q->d_dist;
    z.links = q->d_zl + 2 * (size_t)q->zoff[q->zvars];
    z.zvar = q->d_zvar;
    z.vstride = (uint64_t)q->nrows * q->Vp;
    z.Vp = q->Vp;
    z.nq = q->nq;
    z.nvar = q->zvars;
    z.nlinks = q->znlinks;
    SPF_LAUNCH(spf_zvar_kernel, dim3((q->nq + 255) / 256), dim3(256), 0, g->stream, z);
    HIP_TRY(hipGetLastError());
  }
  return SPF_OK;
}

// zero-metric plan, after the next-hop pass: every source's distance row from
// its own variant table, then the wide-plan rows of the sources with a
// metric-0 out-link
int finish_zero_plan(spf_query* q);

int launch_nh_levels(spf_query* q, bool unit) {
  spf_graph* g = q->g;
  NhLevelsArgs a{};
  a.nbr_off = g->d_nbr_off;
  a.nbrs = g->d_nbrs;
  a.trbits = g->d_tr;
  a.src = q->d_src;
  a.row_of = q->d_row_of;
  a.lvl = q->d_lvl;
  a.dist = (const uint32_t*)q->d_dist;
  a.flags = q->d_flags ? q->d_flags + q->ms_par : nullptr;
  a.nt_store = env_flag("OPENR_NL_NT", 0) ? 1u : 0u;
  a.nh_off = q->d_nh_off;
  a.nh_w = q->d_nh_w;
  a.nh_out = q->d_nh;
  a.nhb = q->d_nhb;
  a.nhb_off = q->d_nhb_off;
  a.nh_b = q->d_nh_b;
  a.V = g->V;
  a.Vp = q->Vp;
  a.Vp8 = q->Vp8;
  a.nq = q->nq;
  a.scale = unit ? 1u : (q->zvars ? q->zscale : g->uniform);
  a.xcd_swizzle = env_flag("OPENR_NL_XCD", 0);
  a.held_words = env_flag("OPENR_NL_HELD", 1);
  a.zvar = q->d_zvar;
  a.lvl_vstride = (uint64_t)q->nrows * q->Vp8;
  a.dist_vstride = (uint64_t)q->nrows * q->Vp;
  a.dist_w = lvl_only(q) ? (uint32_t*)q->d_dist : nullptr;
  const uint32_t nchunks = (g->V + kNlChunk - 1) / kNlChunk;
  const uint64_t blocks =
      (uint64_t)((nchunks + kNlChunksPerBlock - 1) / kNlChunksPerBlock) * q->nq;
  if (blocks > 0x7FFFFFFFull) {
    return fail(SPF_E_UNSUPPORTED, "batch too large for the next-hop pass");
  }
  if (q->nl_swar) {
    // held kernel: every source with <= kNsHeldMax mask words; the generic
    // byte kernel: the rest (q->d_big), or every source after a deep BFS
    // threads per block (OPENR_NL_HT = 256 / 512 / 1024; chunk = 4 nodes per thread)
    const uint32_t ht = env_u32("OPENR_NL_HT", 256);
    const uint32_t T = ht == 1024 ? 1024u : (ht == 512 ? 512u : 256u);
    uint64_t hblocks = (uint64_t)q->nq * ((g->V + 4 * T - 1) / (4 * T));
    if (q->d_held_order && q->held_t == T) {
      a.held_order = q->d_held_order;
      a.held_nch = q->held_nch;
      hblocks = q->held_blocks;
    }
    if (hblocks > 0x7FFFFFFFull) {
      return fail(SPF_E_UNSUPPORTED, "batch too large for the next-hop pass");
    }
    const uint32_t* nolist = nullptr;
    if (q->has_v2 && q->v2_gen == g->nbr_gen && T == 256 && !a.held_order) {
      // v2: solo items and shared-neighbour groups (spf_nh_levels_v2_kernel)
      const uint64_t vblocks = q->v2.order == 5 ? (uint64_t)q->v2.nmap
                                                : (uint64_t)(q->v2.nsolo + q->v2.nsub) *
                                                      ((g->V + 1023) / 1024);
      if (vblocks && q->v2.trit) {
        SPF_LAUNCH((spf_nh_levels_v2_kernel<256, true>), dim3((uint32_t)vblocks), dim3(256), 0,
                           g->stream, a, q->v2);
      } else if (vblocks) {
        SPF_LAUNCH((spf_nh_levels_v2_kernel<256, false>), dim3((uint32_t)vblocks), dim3(256), 0,
                           g->stream, a, q->v2);
      }
    } else if (T == 1024) {
      SPF_LAUNCH((spf_nh_levels_held_kernel<1024, kNsHeldMax>), dim3((uint32_t)hblocks),
                         dim3(1024), 0, g->stream, a, nolist, 0u);
    } else if (T == 512) {
      SPF_LAUNCH((spf_nh_levels_held_kernel<512, kNsHeldMax>), dim3((uint32_t)hblocks),
                         dim3(512), 0, g->stream, a, nolist, 0u);
    } else {
      SPF_LAUNCH((spf_nh_levels_held_kernel<256, kNsHeldMax>), dim3((uint32_t)hblocks),
                         dim3(256), 0, g->stream, a, nolist, 0u);
    }
    HIP_TRY(hipGetLastError());
    if (q->nmid && env_flag("OPENR_NL_WIDE", 1)) {
      // sources with 4-8 words: the same per-(source, chunk) pass
      const uint64_t mblocks = (uint64_t)q->nmid * ((g->V + 1023) / 1024);
      SPF_LAUNCH((spf_nh_levels_held_kernel<256, kNsHeldWide>), dim3((uint32_t)mblocks),
                         dim3(256), 0, g->stream, a, (const uint32_t*)q->d_big, q->nmid);
      HIP_TRY(hipGetLastError());
    }
    const uint32_t skip = env_flag("OPENR_NL_WIDE", 1) ? q->nmid : 0;
    // with no wide source left the kernel only serves a BFS deeper than 254
    // levels, which a graph of at most 254 nodes cannot have: no launch (a
    // small area's RouteDb batch, e.g. the 10x10 grid)
    if (q->nbig == skip && g->V <= 254 && env_flag("OPENR_NL_SWAR_SKIP", 1)) {
      return SPF_OK;
    }
    const uint32_t grid = std::max<uint32_t>(q->nbig - skip, std::min<uint32_t>(q->nq, 1024));
    SPF_LAUNCH(spf_nh_levels_swar_kernel, dim3(grid), dim3(kNsThreads), 0, g->stream,
                       a, (const uint32_t*)q->d_big + skip, q->nbig - skip);
    HIP_TRY(hipGetLastError());
    return SPF_OK;
  }
  SPF_LAUNCH(spf_nh_levels_kernel, dim3((uint32_t)blocks),
                     dim3(kNlThreads), 0, g->stream, a);
  HIP_TRY(hipGetLastError());
  return SPF_OK;
}

int launch_exact(spf_query* q) {
  spf_graph* g = q->g;
  ExactArgs a;
  a.row = g->d_row;
  a.col = g->d_col;
  a.w64 = g->d_w64;
  a.link = g->d_link;
  a.slot = g->d_slot;
  a.trbits = g->d_tr;
  a.src = q->d_src;
  a.ign_off = q->d_ign_off;
  a.ign = q->d_ign;
  a.nh_off = q->d_nh_off;
  a.nh_w = q->d_nh_w;
  a.dist_out = (uint64_t*)q->d_dist;
  a.nh_out = q->d_nh;
  a.order_out = q->d_order;
  a.scratch = q->d_scratch;
  a.V = g->V;
  a.nq = q->nq;
  a.unit = (q->flags & SPF_F_UNIT_METRIC) ? 1 : 0;
  a.want_nh = (q->flags & SPF_F_NEXTHOPS) ? 1 : 0;
  if (q->d_nh && q->nh_total) {
    HIP_TRY(hipMemsetAsync(q->d_nh, 0, q->nh_total * 8, g->stream));
  }
  const uint32_t threads = 64;
  SPF_LAUNCH(
      spf_exact_kernel, dim3((q->nq + threads - 1) / threads), dim3(threads),
      0, g->stream, a);
  HIP_TRY(hipGetLastError());
  return SPF_OK;
}

// 64-bit distance rows (literal replay or wide plan)
inline bool rows64(const spf_query* q) {
  return q->dist == DistPlan::Exact || q->dist == DistPlan::Wide;
}

int launch_wide(spf_query* q) {
  spf_graph* g = q->g;
  WideArgs a;
  a.row = g->d_row;
  a.col = g->d_col;
  a.w64 = g->d_w64;
  a.link = g->d_link;
  a.rev = g->d_rev;
  a.slot = g->d_slot;
  a.trbits = g->d_tr;
  a.zero_e = g->d_zero_e;
  a.src = q->d_src;
  a.ign_off = q->d_ign_off;
  a.ign = q->d_ign;
  a.nh_off = q->d_nh_off;
  a.nh_w = q->d_nh_w;
  a.dist_out = (uint64_t*)q->d_dist;
  a.nh_out = q->d_nh;
  a.key_out = q->d_key;
  a.scratch = q->d_scratch;
  a.V = g->V;
  a.nq = q->nq;
  a.nbw = g->nbw;
  a.unit = (q->flags & SPF_F_UNIT_METRIC) ? 1 : 0;
  a.n_zero = a.unit ? 0 : g->n_zero;
  a.delta = a.unit ? 1 : g->wide_delta;
  if (const char* dv = getenv("OPENR_SPF_WIDE_DELTA")) {
    a.delta = std::max<uint64_t>(1, strtoull(dv, nullptr, 10));
  }
  a.want_nh = (q->flags & SPF_F_NEXTHOPS) ? 1 : 0;
  if (g->nbw * 32 < g->V) {
    return fail(SPF_E_INVALID, "bitmap words do not cover the nodes");
  }
  if (q->d_nh && q->nh_total) {
    HIP_TRY(hipMemsetAsync(q->d_nh, 0, q->nh_total * 8, g->stream));
  }
  SPF_LAUNCH(spf_wide_kernel, dim3(q->grid), dim3(kWideBlock), q->lds_bytes,
                     g->stream, a);
  HIP_TRY(hipGetLastError());
  return SPF_OK;
}

// Event between the distance kernel and the next-hop kernel of a two-stage
// plan, so spf_query_stage_ms can split the device time per kernel.
// A what-if baseline (q->base) runs through run_plan alone, without
// spf_query_run's per-run events: nothing to mark then.
int mark_stage(spf_query* q) {
  hipEvent_t h = q->hist[q->runs % spf_query::kHist][1];
  if (!h) {
    return SPF_OK;
  }
  HIP_TRY(hipEventRecord(q->evm, q->g->stream));
  HIP_TRY(hipEventRecord(h, q->g->stream));
  q->two_stage = true;
  return SPF_OK;
}

int run_plan(spf_query* q);

int finish_zero_plan(spf_query* q) {
  spf_graph* g = q->g;
  if (!q->d_zvar) {
    return SPF_OK; // distances alone: one table, already in place
  }
  SPF_LAUNCH(spf_zrows_kernel, dim3(q->nq), dim3(256), 0, g->stream, (uint32_t*)q->d_dist,
                     (const uint8_t*)q->d_zvar, (uint64_t)q->nrows * q->Vp, q->Vp);
  HIP_TRY(hipGetLastError());
  if (!q->zfix) {
    return SPF_OK;
  }
  spf_query* f = q->zfix;
  int s = run_plan(f);
  if (s != SPF_OK) {
    return s;
  }
  const uint32_t V = g->V;
  for (uint32_t j = 0; j < f->nq; ++j) {
    const uint32_t i = q->zfix_rows[j];
    if (f->nh_w[j] != q->nh_w[i]) {
      return fail(SPF_E_INVALID, "internal: zero-metric fix-up mask width differs");
    }
    if (!q->narrow) {
      HIP_TRY(hipMemcpyAsync(q->d_nh + q->nh_off[i], f->d_nh + f->nh_off[j],
                             (size_t)q->nh_w[i] * V * 8, hipMemcpyDeviceToDevice, g->stream));
    } else {
      // f's rows are in the word layout (kQueryWideMasks): narrow row i
      NhNarrowArgs na{};
      na.src = f->d_nh;
      na.dst = q->d_nhb;
      na.src_off1 = f->nh_off[j];
      na.dst_off1 = q->nhb_off[i];
      na.nb1 = q->nh_b[i];
      na.nw1 = q->nh_w[i];
      na.V = V;
      na.nq = 1;
      SPF_LAUNCH(spf_nh_narrow_kernel, dim3((V + 1023) / 1024), dim3(256), 0, g->stream,
                         na);
      HIP_TRY(hipGetLastError());
    }
    SPF_LAUNCH(spf_rows64to32_kernel, dim3((V + 255) / 256), dim3(256), 0, g->stream,
                       (const uint64_t*)f->d_dist + (size_t)j * V,
                       (uint32_t*)q->d_dist + (size_t)i * q->Vp, V);
    HIP_TRY(hipGetLastError());
  }
  return SPF_OK;
}

int run_screen(spf_query* q) {
  spf_query* b = q->base;
  spf_graph* g = q->g;
  if (!q->wh_cand.empty() && !g->paired) {
    // the source-link kernels were chosen for a graph whose half-edges were
    // paired; spf_graph_set_edges has since taken one half of a link down
    return fail(SPF_E_UNSUPPORTED,
                "what-if query: a half-edge went down alone since creation (recreate the query)");
  }
  if (!q->wh_cand.empty() && !((q->flags & SPF_F_UNIT_METRIC) || g->uniform)) {
    // the source-link kernels compute levels x the uniform metric
    return fail(SPF_E_UNSUPPORTED,
                "what-if query: the metrics stopped being uniform since creation (recreate the query)");
  }
  int s = SPF_OK;
  if (q->hop) {
    // the first-hop rows: BFS levels from the sources' neighbours through
    // every node but the source (independent of the baseline).  The blocked
    // form runs on the side stream beside the baseline and the screen; the
    // ignore-list form (its own mask kernel and memsets) on the graph stream
    if (q->hop->d_ms_blocked && q->wh_stream) {
      HIP_TRY(hipEventRecord(q->wh_ev2, g->stream));
      HIP_TRY(hipStreamWaitEvent(q->wh_stream, q->wh_ev2, 0));
      q->hop->stream_override = q->wh_stream;
      q->wh_pending = true; // (the graph stream joins wh_ev1 after the SSSP launch)
    }
    s = run_plan(q->hop);
    if (s != SPF_OK) {
      return s;
    }
  }
  s = run_plan(b);
  if (s != SPF_OK) {
    return s;
  }
  WhatifArgs a;
  a.col = g->d_col;
  a.rev = g->d_rev;
  a.wout = g->d_wout;
  a.trbits = g->d_tr;
  a.link_half = g->d_link_half;
  a.src = q->d_src;
  a.ign_off = q->d_ign_off;
  a.ign = q->d_ign;
  a.base_of = q->d_base_of;
  a.base_dist = (const uint32_t*)b->d_dist;
  a.base_nh = b->d_nh;
  a.base_nh_off = b->d_nh_off;
  a.dist_out = (uint32_t*)q->d_dist;
  a.nh_out = q->d_nh;
  a.nh_off = q->d_nh_off;
  a.nh_w = q->d_nh_w;
  a.skip = q->d_skip;
  a.V = g->V;
  a.Vp = q->Vp;
  a.L = g->L;
  a.want_nh = (q->flags & SPF_F_NEXTHOPS) ? 1u : 0u;
  a.unit = (q->flags & SPF_F_UNIT_METRIC) ? 1u : 0u;
  a.mark_heavy = q->repair ? 1u : 0u;
  a.wh_mark = q->repair ? q->d_wh_mark : nullptr;
  // screened rows straight into the output layout (the narrowing pass skips
  // them: OPENR_SPF_SCREEN_DIRECT=0 keeps the word copy)
  q->screen_direct = q->narrow && !q->nh_direct && a.want_nh && q->d_nhb && q->d_nhb_off &&
                     env_flag("OPENR_SPF_SCREEN_DIRECT", 1);
  if (q->screen_direct) {
    a.nhb = q->d_nhb;
    a.nhb_off = q->d_nhb_off;
    a.nh_b = q->d_nh_b;
  }
  if (b->Vp != q->Vp) {
    return fail(SPF_E_INVALID, "baseline row stride differs");
  }
  SPF_LAUNCH(spf_whatif_screen_kernel, dim3(q->nq), dim3(256), 0, g->stream, a);
  HIP_TRY(hipGetLastError());
  if (q->repair && q->nfh) {
    const spf_query* hq = q->hop;
    WhatifHopArgs f{};
    f.row = g->d_row;
    f.col = g->d_col;
    f.link = g->d_link;
    f.slot = g->d_slot;
    f.trbits = g->d_tr;
    f.src = q->d_src;
    f.ign_off = q->d_ign_off;
    f.ign = q->d_ign;
    f.skip = q->d_skip;
    f.fh_q = q->d_fh;
    f.fh_h = q->d_fh + q->nfh;
    f.hop_row0 = q->d_fh + 2 * (size_t)q->nfh;
    f.hop_cnt = f.hop_row0 + q->nhop;
    f.hop_off = f.hop_cnt + q->nhop;
    f.hop_nodes = f.hop_off + q->nhop;
    f.rows = (const uint32_t*)hq->d_dist;
    f.rows_pitch = hq->Vp;
    f.dist_out = (uint32_t*)q->d_dist;
    f.nh_out = q->d_nh;
    f.nh_off = q->d_nh_off;
    f.nh_w = q->d_nh_w;
    f.V = g->V;
    f.Vp = q->Vp;
    f.scale = (q->flags & SPF_F_UNIT_METRIC) ? 1u : g->uniform;
    f.want_nh = (q->flags & SPF_F_NEXTHOPS) ? 1u : 0u;
    if (rows64(hq) || !hq->d_dist) {
      return fail(SPF_E_INVALID, "internal: first-hop rows are not 32-bit distance rows");
    }
    // after the screen (skip) on the side stream, behind the hop rows
    hipStream_t fs = g->stream;
    if (q->wh_stream) {
      HIP_TRY(hipEventRecord(q->wh_ev0, g->stream));
      HIP_TRY(hipStreamWaitEvent(q->wh_stream, q->wh_ev0, 0));
      fs = q->wh_stream;
    }
    SPF_LAUNCH(spf_whatif_firsthop_kernel, dim3(q->nfh, (g->V + kFhChunk - 1) / kFhChunk),
               dim3(256), 0, fs, f);
    HIP_TRY(hipGetLastError());
    if (q->wh_stream && q->wh_pull_cand.empty()) {
      HIP_TRY(hipEventRecord(q->wh_ev1, q->wh_stream));
      q->wh_pending = true;
    }
  }
  if (q->repair && !q->wh_pull_cand.empty()) {
    WhatifHeavyArgs h{};
    h.row = g->d_row;
    h.col = g->d_col;
    h.link = g->d_link;
    h.rev = g->d_rev;
    h.slot = g->d_slot;
    h.trbits = g->d_tr;
    h.src = q->d_src;
    h.ign_off = q->d_ign_off;
    h.ign = q->d_ign;
    h.cand = q->d_wh_cand;
    h.skip = q->d_skip;
    h.dist_out = (uint32_t*)q->d_dist;
    h.nh_out = q->d_nh;
    h.nh_off = q->d_nh_off;
    h.nh_w = q->d_nh_w;
    h.V = g->V;
    h.Vp = q->Vp;
    h.scale = (q->flags & SPF_F_UNIT_METRIC) ? 1u : g->uniform;
    h.want_nh = (q->flags & SPF_F_NEXTHOPS) ? 1u : 0u;
    h.lstart = q->d_wh_lstart;
    h.sell4 = g->d_sell;
    h.sell_off = g->d_sell_off;
    h.link_half = g->d_link_half;
    h.L = g->L;
    if (env_flag("OPENR_SPF_WHATIF_STATS", 0)) {
      HIP_TRY(hipMalloc((void**)&h.stats, 6 * q->wh_pull_cand.size() * 8));
      HIP_TRY(hipMemset(h.stats, 0, 6 * q->wh_pull_cand.size() * 8));
    }
    const size_t lds = q->wh_pull ? ((size_t)g->V + (g->V + 31) / 32) * 4
                                  : (3 * (size_t)g->V + 1 + (g->V + 31) / 32) * 4;
    const void* hk = q->wh_pull ? (const void*)spf_whatif_pull_kernel
                                : (const void*)spf_whatif_heavy_kernel;
    HIP_TRY(hipFuncSetAttribute(hk, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    // on its own (high-priority) stream beside the SSSP of the rest, the
    // graph stream joining it after that launch (launch_sssp): fabric batch
    // 1.38 ms, against 1.54 ms in order on the graph stream
    // (OPENR_SPF_WHATIF_HEAVY_STREAM=0; the kernel alone is 0.75 ms there,
    // beside the SSSP its two 122 KB workgroups wait for free CUs)
    const bool side = env_flag("OPENR_SPF_WHATIF_HEAVY_STREAM", 1);
    hipStream_t hstream = side ? q->wh_stream : g->stream;
    if (side) {
      HIP_TRY(hipEventRecord(q->wh_ev0, g->stream));
      HIP_TRY(hipStreamWaitEvent(q->wh_stream, q->wh_ev0, 0));
    }
    if (q->wh_pull) {
      SPF_LAUNCH(spf_whatif_pull_kernel, dim3((uint32_t)q->wh_pull_cand.size()),
                 dim3(kWhThreads), lds, hstream, h);
    } else {
      SPF_LAUNCH(spf_whatif_heavy_kernel, dim3((uint32_t)q->wh_pull_cand.size()),
                 dim3(kWhThreads), lds, hstream, h);
    }
    HIP_TRY(hipGetLastError());
    if (side) {
      HIP_TRY(hipEventRecord(q->wh_ev1, q->wh_stream));
      q->wh_pending = true;
    }
    if (h.stats) {
      std::vector<unsigned long long> hs(6 * q->wh_pull_cand.size());
      HIP_TRY(hipStreamSynchronize(side ? q->wh_stream : g->stream));
      HIP_TRY(hipMemcpy(hs.data(), h.stats, hs.size() * 8, hipMemcpyDeviceToHost));
      HIP_TRY(hipFree(h.stats));
      for (size_t i = 0; i < q->wh_pull_cand.size(); ++i) {
        const unsigned long long* o = hs.data() + 6 * i;
        if (o[4]) {
          fprintf(stderr, "[whatif heavy] query %u: init %llu bfs %llu rows %llu masks %llu ticks "
                  "(100 MHz), %llu levels, %llu reached\n", q->wh_pull_cand[i], o[0], o[1], o[2], o[3],
                  o[4], o[5]);
        }
      }
    }
  }
  return SPF_OK;
}

int run_plan_kernels(spf_query* q);

// the plan's kernels, then (word-layout plans of a query with narrow rows)
// the working rows narrowed into the output layout
int run_plan(spf_query* q) {
  const int s = run_plan_kernels(q);
  if (s != SPF_OK || !q->narrow || q->nh_direct || !q->d_nh) {
    return s;
  }
  NhNarrowArgs na{};
  na.src = q->d_nh;
  na.dst = q->d_nhb;
  na.src_off = q->d_nh_off;
  na.dst_off = q->d_nhb_off;
  na.nb = q->d_nh_b;
  na.nw = q->d_nh_w;
  na.V = q->g->V;
  na.nq = q->nq;
  na.skip = q->base && q->screen_direct ? q->d_skip : nullptr;
  const uint64_t blocks = (uint64_t)q->nq * ((q->g->V + 1023) / 1024);
  if (blocks > 0x7FFFFFFFull) {
    return fail(SPF_E_UNSUPPORTED, "batch too large for the mask narrowing pass");
  }
  SPF_LAUNCH(spf_nh_narrow_kernel, dim3((uint32_t)blocks), dim3(256), 0, q->g->stream,
                     na);
  HIP_TRY(hipGetLastError());
  return SPF_OK;
}

int run_plan_kernels(spf_query* q) {
  const bool unit = q->flags & SPF_F_UNIT_METRIC;
  if (q->base) {
    const int s = run_screen(q);
    if (s != SPF_OK) {
      return s;
    }
  }
  switch (q->dist) {
  case DistPlan::Exact:
    return launch_exact(q);
  case DistPlan::Wide:
    return launch_wide(q);
  case DistPlan::Dstep: {
    int s = q->dlds ? launch_dlds(q) : SPF_OK;
    s = s == SPF_OK ? launch_dstep(q) : s;
    if (s == SPF_OK && q->nh == NhPlan::Rows) {
      // few-source rows plan: next hops from the batch's + helpers' rows
      s = mark_stage(q);
      if (s == SPF_OK) {
        s = launch_nh_rows(q, unit);
      }
    }
    return s;
  }
  case DistPlan::MsDstep:
    return launch_msdstep(q);
  case DistPlan::MsBfs: {
    int s = launch_msbfs(q, unit);
    if (s == SPF_OK && q->nh == NhPlan::Levels && q->d_trit) {
      // part of the distance stage: the level rows' 2-bit copies
      s = launch_lvl_trits(q);
    }
    if (s == SPF_OK && q->nh == NhPlan::Levels) {
      s = mark_stage(q);
      if (s == SPF_OK) {
        s = launch_nh_levels(q, unit);
      }
    }
    if (s == SPF_OK && q->zvars) {
      s = finish_zero_plan(q);
    }
    return s;
  }
  case DistPlan::BfsLds:
  case DistPlan::BfsGmem: {
    int s = launch_bfs(q, unit);
    if (s == SPF_OK && q->nh == NhPlan::Rows) {
      s = mark_stage(q);
      if (s == SPF_OK) {
        s = launch_nh_rows(q, unit);
      }
    }
    return s;
  }
  default: {
    const bool gmem = q->dist == DistPlan::SsspGmem;
    int s = SPF_OK;
    switch (q->wmax) {
    case 0:
      s = dispatch_flags<0>(q, unit, q->has_ign, gmem);
      break;
    case 1:
      s = dispatch_flags<1>(q, unit, q->has_ign, gmem);
      break;
    case 4:
      s = dispatch_flags<4>(q, unit, q->has_ign, gmem);
      break;
    default:
      s = dispatch_flags<16>(q, unit, q->has_ign, gmem);
      break;
    }
    if (s == SPF_OK && q->nh == NhPlan::Rows) {
      s = mark_stage(q);
      if (s == SPF_OK) {
        s = launch_nh_rows(q, unit);
      }
    }
    return s;
  }
  }
}

} // namespace

extern "C" {

int spf_query_run(spf_query* q) {
  SPF_ABI_RANGE("spf_query_run");
  if (!q) {
    return fail(SPF_E_INVALID, "null query");
  }
  spf_graph* g = q->g;
  HIP_TRY(hipSetDevice(g->device));
  const uint32_t h = q->runs % spf_query::kHist;
  if (!q->hist[h][0]) {
    for (auto& e : q->hist[h]) {
      HIP_TRY(ev_get(&e));
    }
  }
  HIP_TRY(hipEventRecord(q->ev0, g->stream));
  HIP_TRY(hipEventRecord(q->hist[h][0], g->stream));
  q->two_stage = false;
  struct LaunchLog {
    bool own = false;
    explicit LaunchLog(spf_query* x) {
      if (!tl_launched) {
        x->launched.clear();
        tl_launched = &x->launched;
        own = true;
      }
    }
    ~LaunchLog() {
      if (own) {
        tl_launched = nullptr;
      }
    }
  } launch_log(q);
  int s = SPF_OK;
  if (q->nq && g->V) {
    s = run_plan(q);
  }
  HIP_TRY(hipEventRecord(q->ev1, g->stream));
  HIP_TRY(hipEventRecord(q->hist[h][2], g->stream));
  q->hist_two[h] = q->two_stage;
  ++q->runs;
  q->ran = true;
  return s;
}

int spf_query_kernels(const spf_query* q, char* buf, size_t cap) {
  if (!q) {
    return fail(SPF_E_INVALID, "null query");
  }
  std::vector<std::string> names;
  for (const char* e : q->launched) {
    std::string n(e);
    const size_t b = n.find_first_not_of("( ");
    if (b == std::string::npos) {
      continue;
    }
    const size_t x = n.find_first_of("<), ", b);
    n = n.substr(b, x == std::string::npos ? std::string::npos : x - b);
    if (std::find(names.begin(), names.end(), n) == names.end()) {
      names.push_back(n);
    }
  }
  std::sort(names.begin(), names.end());
  std::string out;
  for (const auto& n : names) {
    out += (out.empty() ? "" : ",") + n;
  }
  if (buf && cap) {
    const size_t k = std::min(cap - 1, out.size());
    std::memcpy(buf, out.data(), k);
    buf[k] = '\0';
  }
  return (int)out.size();
}

int spf_query_sync(spf_query* q) {
  SPF_ABI_RANGE("spf_query_sync");
  if (!q) {
    return fail(SPF_E_INVALID, "null query");
  }
  HIP_TRY(hipSetDevice(q->g->device));
  HIP_TRY(hipStreamSynchronize(q->g->stream));
  if (q->coop_p) {
    // a cooperative MS-BFS barrier that gave up leaves its rows incomplete
    const uint32_t nbatch = (q->nrows + 63) / 64;
    const size_t off = (size_t)nbatch * 2 * q->g->V * 8 + (size_t)nbatch * 4 +
                       (size_t)nbatch * 2 * q->coop_p * 4;
    uint32_t err = 0;
    HIP_TRY(hipMemcpy(&err, static_cast<char*>(q->d_coop) + off, 4, hipMemcpyDeviceToHost));
    if (err) {
      HIP_TRY(hipMemset(static_cast<char*>(q->d_coop) + off, 0, 4));
      return fail(SPF_E_DEVICE, "cooperative MS-BFS: a level barrier timed out");
    }
  }
  return SPF_OK;
}

int spf_query_elapsed_ms(spf_query* q, float* ms) {
  if (!q || !ms || !q->ran) {
    return fail(SPF_E_INVALID, "query has not run");
  }
  HIP_TRY(hipEventSynchronize(q->ev1));
  HIP_TRY(hipEventElapsedTime(ms, q->ev0, q->ev1));
  return SPF_OK;
}

int spf_query_screened(spf_query* q, uint32_t* screened, uint32_t* has_screen) {
  if (!q || !screened || !has_screen || !q->ran) {
    return fail(SPF_E_INVALID, "query has not run");
  }
  *screened = 0;
  *has_screen = q->d_skip ? 1u : 0u;
  if (!q->d_skip) {
    return SPF_OK;
  }
  HIP_TRY(hipEventSynchronize(q->ev1));
  std::vector<uint32_t> skip(q->nq);
  HIP_TRY(hipMemcpy(skip.data(), q->d_skip, (size_t)q->nq * 4, hipMemcpyDeviceToHost));
  for (uint32_t v : skip) {
    *screened += v == 1; // 2 = a heavy repair (not screened)
  }
  return SPF_OK;
}

int spf_query_stage_ms(spf_query* q, float* dist_ms, float* nh_ms) {
  if (!q || !dist_ms || !nh_ms || !q->ran) {
    return fail(SPF_E_INVALID, "query has not run");
  }
  HIP_TRY(hipEventSynchronize(q->ev1));
  if (q->two_stage) {
    HIP_TRY(hipEventElapsedTime(dist_ms, q->ev0, q->evm));
    HIP_TRY(hipEventElapsedTime(nh_ms, q->evm, q->ev1));
  } else {
    HIP_TRY(hipEventElapsedTime(dist_ms, q->ev0, q->ev1));
    *nh_ms = 0.0f;
  }
  return SPF_OK;
}

int spf_query_stage_history(
    spf_query* q, uint32_t n, float* dist_ms, float* nh_ms, uint32_t* got) {
  if (!q || !got || (n && (!dist_ms || !nh_ms))) {
    return fail(SPF_E_INVALID, "bad arguments");
  }
  const uint64_t avail = std::min<uint64_t>(q->runs, spf_query::kHist);
  const uint32_t m = (uint32_t)std::min<uint64_t>(n, avail);
  for (uint32_t i = 0; i < m; ++i) {
    // oldest of the last m runs first
    const uint32_t h = (uint32_t)((q->runs - m + i) % spf_query::kHist);
    HIP_TRY(hipEventSynchronize(q->hist[h][2]));
    if (q->hist_two[h]) {
      HIP_TRY(hipEventElapsedTime(&dist_ms[i], q->hist[h][0], q->hist[h][1]));
      HIP_TRY(hipEventElapsedTime(&nh_ms[i], q->hist[h][1], q->hist[h][2]));
    } else {
      HIP_TRY(hipEventElapsedTime(&dist_ms[i], q->hist[h][0], q->hist[h][2]));
      nh_ms[i] = 0.0f;
    }
  }
  *got = m;
  return SPF_OK;
}

const char* spf_query_kernel_name(const spf_query* q) {
  if (!q) {
    return "none";
  }
  switch (q->dist) {
  case DistPlan::SsspLds:
    return q->nh == NhPlan::Rows ? "lds+rows" : "lds";
  case DistPlan::SsspGmem:
    return q->nh == NhPlan::Rows ? "gmem+rows" : "gmem";
  case DistPlan::BfsLds:
    return q->nh == NhPlan::Rows ? "bfs+rows" : "bfs";
  case DistPlan::BfsGmem:
    return q->nh == NhPlan::Rows ? "bfs-gmem+rows" : "bfs-gmem";
  case DistPlan::MsBfs:
    if (q->zvars) {
      return q->nh == NhPlan::Levels ? "msbfs0+levels" : "msbfs0";
    }
    return q->nh == NhPlan::Levels ? "msbfs+levels" : "msbfs";
  case DistPlan::Dstep:
    return q->dlds ? "dstep-ldsrow" : "dstep";
  case DistPlan::MsDstep:
    return "msdstep";
  case DistPlan::Wide:
    return "wide";
  default:
    return "exact";
  }
}

int spf_query_dist(spf_query* q, uint32_t i, uint64_t* out) {
  SPF_ABI_RANGE("spf_query_dist");
  if (!q || !out || i >= q->nq) {
    return fail(SPF_E_INVALID, "bad query row");
  }
  const uint32_t V = q->g->V;
  HIP_TRY(hipSetDevice(q->g->device));
  HIP_TRY(hipStreamSynchronize(q->g->stream));
  if (q->dist == DistPlan::Exact) {
    HIP_TRY(hipMemcpy(out, (uint64_t*)q->d_dist + (size_t)i * V, V * 8ull,
                      hipMemcpyDeviceToHost));
    std::vector<uint32_t> order(V);
    HIP_TRY(hipMemcpy(order.data(), q->d_order + (size_t)i * V, V * 4ull,
                      hipMemcpyDeviceToHost));
    for (uint32_t v = 0; v < V; ++v) {
      if (order[v] == kInf32) {
        out[v] = SPF_UNREACHABLE;
      }
    }
    return SPF_OK;
  }
  if (q->dist == DistPlan::Wide) {
    HIP_TRY(hipMemcpy(out, (uint64_t*)q->d_dist + (size_t)i * V, V * 8ull,
                      hipMemcpyDeviceToHost));
    return SPF_OK;
  }
  std::vector<uint32_t> d(V);
  HIP_TRY(hipMemcpy(d.data(), (uint32_t*)q->d_dist + (size_t)i * q->Vp,
                    V * 4ull, hipMemcpyDeviceToHost));
  for (uint32_t v = 0; v < V; ++v) {
    out[v] = d[v] == kInf32 ? SPF_UNREACHABLE : (uint64_t)d[v];
  }
  return SPF_OK;
}

int spf_query_nh_words(const spf_query* q, uint32_t i) {
  if (!q || i >= q->nq) {
    return fail(SPF_E_INVALID, "bad query row");
  }
  return (int)q->nh_w[i];
}

int spf_query_nexthops(spf_query* q, uint32_t i, uint64_t* out) {
  SPF_ABI_RANGE("spf_query_nexthops");
  if (!q || !out || i >= q->nq || !(q->flags & SPF_F_NEXTHOPS)) {
    return fail(SPF_E_INVALID, "no next hops for this row");
  }
  HIP_TRY(hipSetDevice(q->g->device));
  HIP_TRY(hipStreamSynchronize(q->g->stream));
  const size_t V = q->g->V, W = q->nh_w[i], B = q->nh_b[i];
  if (V && B >= 8) {
    HIP_TRY(hipMemcpy(out, q->d_nhb + q->nhb_off[i], V * W * 8, hipMemcpyDeviceToHost));
  } else if (V) {
    std::vector<uint8_t> tmp(V * B);
    HIP_TRY(hipMemcpy(tmp.data(), q->d_nhb + q->nhb_off[i], V * B, hipMemcpyDeviceToHost));
    widen_masks(tmp.data(), B, V, out);
  }
  return SPF_OK;
}

int spf_query_nh_bytes(const spf_query* q, uint32_t i) {
  if (!q || i >= q->nq) {
    return fail(SPF_E_INVALID, "bad query row");
  }
  return (int)q->nh_b[i];
}

int spf_query_nh_offset(const spf_query* q, uint32_t i, uint64_t* byte_off) {
  if (!q || !byte_off || i >= q->nq) {
    return fail(SPF_E_INVALID, "bad query row");
  }
  *byte_off = q->nhb_off[i];
  return SPF_OK;
}

int spf_query_order_keys(spf_query* q, uint32_t i, uint64_t* out) {
  SPF_ABI_RANGE("spf_query_order_keys");
  if (!q || !out || i >= q->nq || !(q->flags & SPF_F_ORDER)) {
    return fail(SPF_E_INVALID, "no settle order for this row");
  }
  if (q->dist != DistPlan::Wide) {
    return fail(SPF_E_UNSUPPORTED, "settle keys come from the wide plan; use spf_query_order");
  }
  HIP_TRY(hipSetDevice(q->g->device));
  HIP_TRY(hipStreamSynchronize(q->g->stream));
  HIP_TRY(hipMemcpy(out, q->d_key + (size_t)i * q->g->V, q->g->V * 8ull,
                    hipMemcpyDeviceToHost));
  return SPF_OK;
}

int spf_query_order(spf_query* q, uint32_t i, uint32_t* out) {
  SPF_ABI_RANGE("spf_query_order");
  if (!q || !out || i >= q->nq ||
      !(q->dist == DistPlan::Exact || (q->dist == DistPlan::Wide && q->d_key))) {
    return fail(SPF_E_INVALID, "no settle order for this row");
  }
  HIP_TRY(hipSetDevice(q->g->device));
  HIP_TRY(hipStreamSynchronize(q->g->stream));
  if (q->dist == DistPlan::Wide) {
    // settle rank = position in (distance, key) order of the reached nodes
    const uint32_t V = q->g->V;
    std::vector<uint64_t> d(V), k(V);
    HIP_TRY(hipMemcpy(d.data(), (uint64_t*)q->d_dist + (size_t)i * V, V * 8ull,
                      hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(k.data(), q->d_key + (size_t)i * V, V * 8ull, hipMemcpyDeviceToHost));
    std::vector<uint32_t> idx;
    idx.reserve(V);
    for (uint32_t v = 0; v < V; ++v) {
      out[v] = kInf32;
      if (d[v] != SPF_UNREACHABLE) {
        idx.push_back(v);
      }
    }
    std::sort(idx.begin(), idx.end(), [&](uint32_t a, uint32_t b) {
      return d[a] != d[b] ? d[a] < d[b] : k[a] < k[b];
    });
    for (uint32_t r = 0; r < idx.size(); ++r) {
      out[idx[r]] = r;
    }
    return SPF_OK;
  }
  HIP_TRY(hipMemcpy(out, q->d_order + (size_t)i * q->g->V, q->g->V * 4ull,
                    hipMemcpyDeviceToHost));
  return SPF_OK;
}

int spf_query_device_rows(
    spf_query* q, void** dist_rows, uint32_t* dist_elem_bytes,
    void** nh_rows, uint64_t* nh_total_words) {
  if (!q) {
    return fail(SPF_E_INVALID, "null query");
  }
  if (dist_rows) {
    *dist_rows = q->d_dist;
  }
  if (dist_elem_bytes) {
    *dist_elem_bytes = rows64(q) ? 8 : 4;
  }
  if (nh_rows) {
    *nh_rows = q->d_nhb;
  }
  if (nh_total_words) {
    *nh_total_words = q->nhb_total / 8; // rows are 32-byte aligned
  }
  return SPF_OK;
}

int spf_query_fetch_rows(
    spf_query* q, uint32_t first, uint32_t count, void* dst, size_t dst_pitch,
    int dst_on_device) {
  SPF_ABI_RANGE("spf_query_fetch_rows");
  if (!q || (count && !dst)) {
    return fail(SPF_E_INVALID, "null argument");
  }
  if (!q->ran) {
    return fail(SPF_E_INVALID, "query has not run");
  }
  if ((uint64_t)first + count > q->nq) {
    return fail(SPF_E_INVALID, "row range out of bounds");
  }
  if (rows64(q)) {
    return fail(SPF_E_UNSUPPORTED, "64-bit distance rows: use spf_query_dist");
  }
  const size_t V = q->g->V;
  if (dst_pitch < V * 4) {
    return fail(SPF_E_INVALID, "destination pitch < 4*V");
  }
  if (count == 0 || V == 0) {
    return SPF_OK;
  }
  HIP_TRY(hipSetDevice(q->g->device));
  const char* srcp = (const char*)q->d_dist + (size_t)first * q->Vp * 4;
  HIP_TRY(hipMemcpy2DAsync(
      dst, dst_pitch, srcp, (size_t)q->Vp * 4, V * 4, count,
      dst_on_device ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost, q->g->stream));
  if (!dst_on_device) {
    HIP_TRY(hipStreamSynchronize(q->g->stream));
  }
  return SPF_OK;
}

int spf_query_trace_paths(
    spf_query* q, uint32_t first, uint32_t count, const uint32_t* dests, uint32_t* path_count,
    uint32_t* link_count) {
  SPF_ABI_RANGE("spf_query_trace_paths");
  if (!q || (count && (!dests || !path_count || !link_count))) {
    return fail(SPF_E_INVALID, "null argument");
  }
  if (!q->ran) {
    return fail(SPF_E_INVALID, "query has not run");
  }
  if ((uint64_t)first + count > q->nq) {
    return fail(SPF_E_INVALID, "query range out of bounds");
  }
  if (rows64(q)) {
    return fail(SPF_E_UNSUPPORTED, "64-bit distance rows (settle keys): trace on the host");
  }
  const spf_graph* g = q->g;
  for (uint32_t i = 0; i < count; ++i) {
    if (dests[i] >= g->V) {
      return fail(SPF_E_INVALID, "destination out of range");
    }
  }
  q->trace_n = 0;
  q->trace_links = 0;
  q->trace_paths = 0;
  if (count == 0) {
    return SPF_OK;
  }
  HIP_TRY(hipSetDevice(g->device));
  // the trace kernels join the run's launch list (spf_query_kernels)
  struct TraceLog {
    bool own = false;
    explicit TraceLog(spf_query* x) {
      if (!tl_launched) {
        tl_launched = &x->launched;
        own = true;
      }
    }
    ~TraceLog() {
      if (own) {
        tl_launched = nullptr;
      }
    }
  } trace_log(q);
  // scratch: dests | out_n | out_len | links [count][cap] | ends [count][cap]
  // (OPENR_SPF_TRACE_CAP lowers the per-query capacity: overflow tests)
  const uint32_t cap = std::max<uint32_t>(1, std::min(kTraceCap, env_u32("OPENR_SPF_TRACE_CAP", kTraceCap)));
  q->trace_cap = cap;
  const size_t cells = (size_t)count * cap;
  const size_t words = 3 * (size_t)count + 2 * cells;
  if (q->d_trace && q->trace_words < words) {
    HIP_TRY(hipStreamSynchronize(g->stream));
    pool_free(q->d_trace);
    q->d_trace = nullptr;
  }
  if (!q->d_trace) {
    HIP_TRY(pool_malloc((void**)&q->d_trace, words * 4));
    q->trace_words = words;
  }
  uint32_t* buf = q->d_trace;
  HIP_TRY(hipMemcpyAsync(buf, dests, (size_t)count * 4, hipMemcpyHostToDevice, g->stream));
  TraceArgs a;
  a.row = g->d_row;
  a.col = g->d_col;
  a.rev = g->d_rev;
  a.link = g->d_link;
  a.wout = g->d_wout;
  a.trbits = g->d_tr;
  a.src = q->d_src + first;
  a.dst = buf;
  a.ign_off = q->d_ign_off ? q->d_ign_off + first : nullptr;
  a.ign = q->d_ign;
  a.dist = (const uint32_t*)q->d_dist + (size_t)first * q->Vp;
  a.out_n = buf + count;
  a.out_len = buf + 2 * (size_t)count;
  a.out_links = buf + 3 * (size_t)count;
  a.out_ends = buf + 3 * (size_t)count + cells;
  a.Vp = q->Vp;
  a.nq = count;
  a.cap = cap;
  a.unit = (q->flags & SPF_F_UNIT_METRIC) ? 1u : 0u;
  const bool cursor = env_flag("OPENR_SPF_TRACE_CURSOR", 1);
  // queries past the cursor kernel's step budget go to the heavy launch
  // (spf_trace_heavy_kernel; its node states live in LDS: V <= kHvMaxV)
  const bool heavy = cursor && g->V <= kHvMaxV && env_flag("OPENR_SPF_TRACE_HEAVY", 1);
  // the heavy queries' kernel: the reachability walk (its arrays fit LDS), or
  // the DFS with LDS cursors (OPENR_SPF_TRACE_REACH=0)
  const bool reach =
      reach_lds_words(g->V, g->L) * 4 <= kRqMaxLds && env_flag("OPENR_SPF_TRACE_REACH", 1);
  if (cursor) {
    // cursor DFS: per-wave node states + pathLinks arena (zeroed per launch:
    // a state's tag is its query index + 1)
    // 16 waves per CU (a wave's DFS is a chain of L2 round trips: the more
    // queries in flight, the better); scratch bounded for large graphs
    const uint32_t wpc = std::max<uint32_t>(1, std::min<uint32_t>(16, env_u32("OPENR_SPF_TRACE_WPC", 16)));
    const uint32_t maxw = g->V > 50000 ? 1024u : (uint32_t)g->num_cus * wpc;
    const uint32_t nw = std::min<uint32_t>((count + kTcWaves - 1) / kTcWaves * kTcWaves, maxw);
    const uint32_t acap = std::max<uint32_t>(1024, std::min<uint32_t>(g->E, 1u << 15));
    // node states | arenas | the query-claim counter
    const size_t o_ctr = (size_t)nw * g->V * sizeof(uint4) + (size_t)nw * acap * sizeof(uint2);
    const size_t need = o_ctr + 256;
    if (q->d_tcs && q->tcs_bytes < need) {
      HIP_TRY(hipStreamSynchronize(g->stream));
      pool_free(q->d_tcs);
      q->d_tcs = nullptr;
    }
    if (!q->d_tcs) {
      HIP_TRY(pool_malloc((void**)&q->d_tcs, need));
      q->tcs_bytes = need;
    }
    TraceCursorArgs ta{};
    ta.t = a;
    ta.nstate = reinterpret_cast<uint4*>(q->d_tcs);
    ta.arena = reinterpret_cast<uint2*>(q->d_tcs + (size_t)nw * g->V * sizeof(uint4));
    ta.arena_cap = acap;
    ta.V = g->V;
    // without the heavy launch no budget by default: at 4,096 steps 252
    // fabric queries went to the host, whose traces cost more than the
    // device's (KSP2 build 58 -> 74 ms, profiles/r05s)
    ta.budget = env_u32("OPENR_SPF_TRACE_BUDGET", heavy ? kTcHeavyBudget : 0xFFFFFFFFu);
    HIP_TRY(hipMemsetAsync(q->d_tcs, 0, (size_t)nw * g->V * sizeof(uint4), g->stream));
    if (env_flag("OPENR_SPF_TRACE_DYN", 1) && count > nw) {
      ta.qctr = reinterpret_cast<uint32_t*>(q->d_tcs + o_ctr);
      HIP_TRY(hipMemsetAsync(ta.qctr, 0, 4, g->stream));
    }
    if (env_flag("OPENR_SPF_TRACE_STATS", 0)) {
      HIP_TRY(hipMalloc((void**)&ta.qstat, (size_t)count * kTcStat * 8));
      HIP_TRY(hipMemsetAsync(ta.qstat, 0, (size_t)count * kTcStat * 8, g->stream));
    }
    if (ta.qstat) {
      SPF_LAUNCH(spf_trace_cursor_kernel<true>, dim3(nw / kTcWaves), dim3(64 * kTcWaves),
                         0, g->stream, ta);
    } else {
      SPF_LAUNCH(spf_trace_cursor_kernel<false>, dim3(nw / kTcWaves), dim3(64 * kTcWaves),
                         0, g->stream, ta);
    }
    if (ta.qstat) {
      // per-query cost and the per-wave sums (wave w ran queries w, w + nw, ...)
      std::vector<unsigned long long> h((size_t)count * kTcStat);
      HIP_TRY(hipStreamSynchronize(g->stream));
      HIP_TRY(hipMemcpy(h.data(), ta.qstat, h.size() * 8, hipMemcpyDeviceToHost));
      HIP_TRY(hipFree(ta.qstat));
      unsigned long long sum = 0, mx = 0, msteps = 0, ssteps = 0, sbuilt = 0;
      uint32_t imax = 0;
      std::vector<unsigned long long> wave(nw, 0);
      for (uint32_t i = 0; i < count; ++i) {
        const unsigned long long* r = h.data() + (size_t)kTcStat * i;
        sum += r[0];
        ssteps += r[1];
        sbuilt += r[2];
        msteps = std::max(msteps, r[1]);
        if (r[0] > mx) {
          mx = r[0];
          imax = i;
        }
        wave[i % nw] += r[0];
      }
      const unsigned long long wmax = *std::max_element(wave.begin(), wave.end());
      const unsigned long long* r = h.data() + (size_t)kTcStat * imax;
      fprintf(stderr,
              "[trace stats] queries=%u waves=%u ticks(100MHz): sum=%llu mean=%.1f max=%llu "
              "(query %u: %llu steps, %llu lists of %llu entries, filter %llu rank %llu ticks) "
              "wave-max=%llu; steps mean=%.1f max=%llu; lists mean=%.1f\n",
              count, nw, sum, (double)sum / count, mx, imax, r[1], r[2], r[5], r[3], r[4], wmax,
              (double)ssteps / count, msteps, (double)sbuilt / count);
    }
  } else {
    SPF_LAUNCH(spf_trace_paths_kernel, dim3((count + kTraceWaves - 1) / kTraceWaves),
                       dim3(64 * kTraceWaves), 0, g->stream, a);
  }
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpyAsync(path_count, a.out_n, (size_t)count * 4, hipMemcpyDeviceToHost,
                         g->stream));
  HIP_TRY(hipMemcpyAsync(link_count, a.out_len, (size_t)count * 4, hipMemcpyDeviceToHost,
                         g->stream));
  HIP_TRY(hipStreamSynchronize(g->stream));
  if (heavy) {
    std::vector<uint32_t> hq;
    for (uint32_t i = 0; i < count; ++i) {
      if (path_count[i] == SPF_TRACE_OVERFLOW) {
        hq.push_back(i);
      }
    }
    // build order: nodes of in-degree <= 16 first (four per wave)
    std::vector<uint32_t> hv_nodes;
    uint32_t hv_nsmall = 0;
    if (!hq.empty()) {
      hv_nodes.reserve(g->V);
      for (uint32_t v = 0; v < g->V; ++v) {
        if (g->row[v + 1] - g->row[v] <= 16) {
          hv_nodes.push_back(v);
        }
      }
      hv_nsmall = (uint32_t)hv_nodes.size();
      for (uint32_t v = 0; v < g->V; ++v) {
        if (g->row[v + 1] - g->row[v] > 16) {
          hv_nodes.push_back(v);
        }
      }
    }
    // chunks: arena + lengths bounded to ~1 GiB per launch
    const size_t per = (size_t)g->E * sizeof(uint2) + (size_t)g->V * 12;
    const size_t chunk = std::max<size_t>(1, std::min<size_t>(1024, ((size_t)1 << 30) / per));
    for (size_t c0 = 0; c0 < hq.size(); c0 += chunk) {
      const uint32_t nh = (uint32_t)std::min(chunk, hq.size() - c0);
      char* hb = nullptr; // nodes [V] | hq [nh] | len [nh][V] | frontiers [nh][2][V] | arena [nh][E]
      const size_t o_hq = ((size_t)g->V * 4 + 255) & ~(size_t)255;
      const size_t o_len = (o_hq + (size_t)nh * 4 + 255) & ~(size_t)255;
      const size_t o_fq = (o_len + (size_t)nh * g->V * 4 + 255) & ~(size_t)255;
      const size_t o_ar = (o_fq + (size_t)nh * g->V * 8 + 255) & ~(size_t)255;
      HIP_TRY(pool_malloc((void**)&hb, o_ar + (size_t)nh * g->E * sizeof(uint2)));
      struct Free {
        char* p;
        hipStream_t st;
        ~Free() {
          (void)hipStreamSynchronize(st);
          pool_free(p);
        }
      } guard{hb, g->stream};
      HIP_TRY(hipMemcpyAsync(hb, hv_nodes.data(), (size_t)g->V * 4, hipMemcpyHostToDevice,
                             g->stream));
      HIP_TRY(hipMemcpyAsync(hb + o_hq, hq.data() + c0, (size_t)nh * 4, hipMemcpyHostToDevice,
                             g->stream));
      TraceHeavyArgs h{};
      h.t = a;
      h.hq = reinterpret_cast<const uint32_t*>(hb + o_hq);
      h.nodes = reinterpret_cast<const uint32_t*>(hb);
      h.nsmall = hv_nsmall;
      h.nh = nh;
      h.V = g->V;
      h.E = g->E;
      h.len = reinterpret_cast<uint32_t*>(hb + o_len);
      h.fq = reinterpret_cast<uint32_t*>(hb + o_fq);
      h.arena = reinterpret_cast<uint2*>(hb + o_ar);
      h.budget = env_u32("OPENR_SPF_TRACE_HEAVY_BUDGET", 0xFFFFFFFFu);
      const bool stats = env_flag("OPENR_SPF_TRACE_STATS", 0);
      if (stats) {
        HIP_TRY(hipMalloc((void**)&h.hstat, (size_t)nh * 32));
      }
      h.xcd = env_flag("OPENR_SPF_TRACE_HEAVY_XCD", 1) ? 1u : 0u;
      const uint64_t bq = hv_blocks(hv_nsmall, g->V - hv_nsmall);
      const uint64_t nblk = h.xcd ? 8 * ((nh + 7) / 8) * bq : (uint64_t)nh * bq;
      SPF_LAUNCH(spf_trace_heavy_build_kernel, dim3((uint32_t)nblk), dim3(64 * kHvWaves), 0,
                 g->stream, h);
      h.L = g->L;
      if (reach) {
        const size_t lds = reach_lds_words(g->V, g->L) * 4;
        HIP_TRY(hipFuncSetAttribute((const void*)spf_trace_reach_kernel,
                                    hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        SPF_LAUNCH(spf_trace_reach_kernel, dim3(nh), dim3(kRqThreads), lds, g->stream, h);
      } else {
        SPF_LAUNCH(spf_trace_heavy_kernel, dim3(nh), dim3(64), 0, g->stream, h);
      }
      HIP_TRY(hipGetLastError());
      if (stats) {
        std::vector<unsigned long long> hs((size_t)nh * 4);
        HIP_TRY(hipStreamSynchronize(g->stream));
        HIP_TRY(hipMemcpy(hs.data(), h.hstat, hs.size() * 8, hipMemcpyDeviceToHost));
        HIP_TRY(hipFree(h.hstat));
        size_t im = 0;
        for (size_t i = 1; i < nh; ++i) {
          if (hs[4 * i] > hs[4 * im]) {
            im = i;
          }
        }
        fprintf(stderr, "[trace heavy stats] nh=%u slowest: ticks=%llu steps=%llu pushes=%llu loads=%llu\n",
                nh, hs[4 * im], hs[4 * im + 1], hs[4 * im + 2], hs[4 * im + 3]);
      }
    }
    if (!hq.empty()) {
      HIP_TRY(hipMemcpyAsync(path_count, a.out_n, (size_t)count * 4, hipMemcpyDeviceToHost,
                             g->stream));
      HIP_TRY(hipMemcpyAsync(link_count, a.out_len, (size_t)count * 4, hipMemcpyDeviceToHost,
                             g->stream));
      HIP_TRY(hipStreamSynchronize(g->stream));
    }
    q->trace_heavy = (uint32_t)hq.size();
    if (!hq.empty() && env_flag("OPENR_SPF_TRACE_STATS", 0)) {
      uint32_t still = 0;
      for (uint32_t i : hq) {
        still += path_count[i] == SPF_TRACE_OVERFLOW;
      }
      fprintf(stderr, "[trace heavy] queries=%u re-traced=%zu still-overflow=%u\n", count,
              hq.size(), still);
    }
  }
  q->trace_n = count;
  q->trace_pc.assign(path_count, path_count + count);
  q->trace_lc.assign(link_count, link_count + count);
  for (uint32_t i = 0; i < count; ++i) {
    if (path_count[i] != SPF_TRACE_OVERFLOW) {
      q->trace_links += link_count[i];
      q->trace_paths += path_count[i];
    }
  }
  return SPF_OK;
}

int spf_query_trace_fetch(spf_query* q, uint32_t* links, uint32_t* ends) {
  SPF_ABI_RANGE("spf_query_trace_fetch");
  if (!q || (q->trace_links && !links) || (q->trace_paths && !ends)) {
    return fail(SPF_E_INVALID, "null argument");
  }
  const uint32_t count = q->trace_n;
  if (count == 0 || (q->trace_links == 0 && q->trace_paths == 0)) {
    return SPF_OK;
  }
  spf_graph* g = q->g;
  HIP_TRY(hipSetDevice(g->device));
  // destination offsets of every query's links and ends (host scan), then
  // one pack kernel and two copies
  std::vector<uint32_t> off(2 * (size_t)count);
  uint64_t lo = 0, po = 0;
  for (uint32_t i = 0; i < count; ++i) {
    const bool ok = q->trace_pc[i] != SPF_TRACE_OVERFLOW;
    off[i] = (uint32_t)lo;
    off[count + i] = (uint32_t)po;
    lo += ok ? q->trace_lc[i] : 0;
    po += ok ? q->trace_pc[i] : 0;
  }
  uint32_t* pk = nullptr; // offsets [2 * count] | links [lo] | ends [po]
  HIP_TRY(pool_malloc((void**)&pk, (2 * (size_t)count + lo + po) * 4));
  struct Free {
    uint32_t* p;
    hipStream_t st;
    ~Free() {
      (void)hipStreamSynchronize(st);
      pool_free(p);
    }
  } guard{pk, g->stream};
  HIP_TRY(hipMemcpyAsync(pk, off.data(), off.size() * 4, hipMemcpyHostToDevice, g->stream));
  const size_t cells = (size_t)count * q->trace_cap;
  uint32_t* buf = q->d_trace;
  TracePackArgs a;
  a.out_n = buf + count;
  a.out_len = buf + 2 * (size_t)count;
  a.links = buf + 3 * (size_t)count;
  a.ends = buf + 3 * (size_t)count + cells;
  a.off_links = pk;
  a.off_ends = pk + count;
  a.dst_links = pk + 2 * (size_t)count;
  a.dst_ends = pk + 2 * (size_t)count + lo;
  a.cap = q->trace_cap;
  a.nq = count;
  SPF_LAUNCH(spf_trace_pack_kernel, dim3(count), dim3(64), 0, g->stream, a);
  HIP_TRY(hipGetLastError());
  if (lo) {
    HIP_TRY(hipMemcpyAsync(links, a.dst_links, lo * 4, hipMemcpyDeviceToHost, g->stream));
  }
  if (po) {
    HIP_TRY(hipMemcpyAsync(ends, a.dst_ends, po * 4, hipMemcpyDeviceToHost, g->stream));
  }
  HIP_TRY(hipStreamSynchronize(g->stream));
  return SPF_OK;
}

int spf_query_fetch_nexthops(
    spf_query* q, uint32_t first, uint32_t count, uint64_t* dst) {
  SPF_ABI_RANGE("spf_query_fetch_nexthops");
  if (!q || (count && !dst)) {
    return fail(SPF_E_INVALID, "null argument");
  }
  if (!(q->flags & SPF_F_NEXTHOPS) || !q->ran) {
    return fail(SPF_E_INVALID, "no next hops for this query");
  }
  if ((uint64_t)first + count > q->nq) {
    return fail(SPF_E_INVALID, "row range out of bounds");
  }
  if (count == 0 || q->g->V == 0) {
    return SPF_OK;
  }
  const size_t V = q->g->V;
  const uint64_t lo = q->nhb_off[first];
  const uint64_t hi = first + count < q->nq ? q->nhb_off[first + count] : q->nhb_total;
  std::vector<uint8_t> tmp(hi - lo);
  HIP_TRY(hipSetDevice(q->g->device));
  HIP_TRY(hipStreamSynchronize(q->g->stream));
  HIP_TRY(hipMemcpy(tmp.data(), q->d_nhb + lo, hi - lo, hipMemcpyDeviceToHost));
  uint64_t out = 0;
  for (uint32_t i = first; i < first + count; ++i) {
    const size_t n = V * q->nh_w[i];
    const uint8_t* src = tmp.data() + (q->nhb_off[i] - lo);
    if (q->nh_b[i] >= 8) {
      std::memcpy(dst + out, src, n * 8);
    } else {
      widen_masks(src, q->nh_b[i], V, dst + out);
    }
    out += n;
  }
  return SPF_OK;
}

} // extern "C"

namespace {
// pinned host staging for spf_query_fetch_host: one buffer per process
// (portable across devices), grown to the largest small request, never freed
struct HostStage {
  std::mutex mu;
  uint8_t* p = nullptr;
  size_t cap = 0;
};
HostStage& host_stage() {
  static HostStage s;
  return s;
}
constexpr size_t kHostStageMax = (size_t)4 << 20;
} // namespace

extern "C" {

int spf_query_fetch_host(
    spf_query* q, uint32_t first, uint32_t count, uint32_t* rows, size_t row_pitch,
    uint64_t* masks) {
  SPF_ABI_RANGE("spf_query_fetch_host");
  if (!q) {
    return fail(SPF_E_INVALID, "null argument");
  }
  if (!q->ran) {
    return fail(SPF_E_INVALID, "query has not run");
  }
  if ((uint64_t)first + count > q->nq) {
    return fail(SPF_E_INVALID, "row range out of bounds");
  }
  if (masks && !(q->flags & SPF_F_NEXTHOPS)) {
    return fail(SPF_E_INVALID, "no next hops for this query");
  }
  if (rows && rows64(q)) {
    return fail(SPF_E_UNSUPPORTED, "64-bit distance rows: use spf_query_dist");
  }
  const size_t V = q->g->V;
  if (rows && row_pitch < V * 4) {
    return fail(SPF_E_INVALID, "destination pitch < 4*V");
  }
  if (count == 0 || V == 0 || (!rows && !masks)) {
    return SPF_OK;
  }
  const size_t rb = rows ? (((size_t)count * V * 4 + 255) & ~(size_t)255) : 0;
  const uint64_t lo = masks ? q->nhb_off[first] : 0;
  const uint64_t hi =
      !masks ? 0 : (first + count < q->nq ? q->nhb_off[first + count] : q->nhb_total);
  const size_t mb = (size_t)(hi - lo);
  if (rb + mb > kHostStageMax || !env_flag("OPENR_SPF_FETCH_STAGE", 1)) {
    if (rows) {
      if (const int st = spf_query_fetch_rows(q, first, count, rows, row_pitch, 0)) {
        return st;
      }
    }
    return masks ? spf_query_fetch_nexthops(q, first, count, masks) : SPF_OK;
  }
  HostStage& hs = host_stage();
  std::lock_guard<std::mutex> lk(hs.mu);
  HIP_TRY(hipSetDevice(q->g->device));
  if (hs.cap < rb + mb) {
    if (hs.p) {
      HIP_TRY(hipHostFree(hs.p));
      hs.p = nullptr;
      hs.cap = 0;
    }
    const size_t want = std::max<size_t>(rb + mb, (size_t)64 << 10);
    HIP_TRY(hipHostMalloc((void**)&hs.p, want, hipHostMallocPortable));
    hs.cap = want;
  }
  hipStream_t st = q->g->stream;
  if (rows) {
    HIP_TRY(hipMemcpy2DAsync(hs.p, V * 4, (const char*)q->d_dist + (size_t)first * q->Vp * 4,
                             (size_t)q->Vp * 4, V * 4, count, hipMemcpyDeviceToHost, st));
  }
  if (mb) {
    HIP_TRY(hipMemcpyAsync(hs.p + rb, q->d_nhb + lo, mb, hipMemcpyDeviceToHost, st));
  }
  HIP_TRY(hipStreamSynchronize(st));
  if (rows) {
    for (uint32_t i = 0; i < count; ++i) {
      std::memcpy(reinterpret_cast<uint8_t*>(rows) + (size_t)i * row_pitch,
                  hs.p + (size_t)i * V * 4, V * 4);
    }
  }
  if (masks) {
    uint64_t out = 0;
    for (uint32_t i = first; i < first + count; ++i) {
      const size_t n = V * q->nh_w[i];
      const uint8_t* src = hs.p + rb + (q->nhb_off[i] - lo);
      if (q->nh_b[i] >= 8) {
        std::memcpy(masks + out, src, n * 8);
      } else {
        widen_masks(src, q->nh_b[i], V, masks + out);
      }
      out += n;
    }
  }
  return SPF_OK;
}

uint32_t spf_query_row_stride(const spf_query* q) {
  if (!q) {
    return 0;
  }
  return rows64(q) ? q->g->V : q->Vp;
}

} // extern "C"

// ============================================ incremental all-sources tables

extern "C" {

int spf_graph_diff(
    const spf_graph_desc* before, const spf_graph_desc* after,
    spf_edge_delta* out, uint32_t cap, uint32_t* n_out) {
  SPF_ABI_RANGE("spf_graph_diff");
  if (!before || !after || !n_out || (cap && !out)) {
    return fail(SPF_E_INVALID, "null argument");
  }
  if (before->num_nodes != after->num_nodes) {
    return fail(SPF_E_INVALID, "graphs differ in node count (ids are not shared)");
  }
  const uint32_t V = before->num_nodes;
  for (const spf_graph_desc* d : {before, after}) {
    if (!d->row_ptr || (d->num_edges && (!d->col || !d->metric)) ||
        (V && !d->node_overloaded) || d->row_ptr[V] != d->num_edges) {
      return fail(SPF_E_INVALID, "malformed graph description");
    }
  }
  // node blocks in parallel, each into its own list; the lists are then
  // concatenated in node order (the serial scan's output order)
  const unsigned nth =
      openr::hostThreads((size_t)before->num_edges + after->num_edges, kHostMinEdges);
  const std::vector<uint32_t> bnd = host_node_blocks(after->row_ptr, V, nth);
  const uint32_t nblk = (uint32_t)bnd.size() - 1;
  std::vector<std::vector<spf_edge_delta>> found(nblk);
  openr::parallelFor(nblk, nth, [&](size_t blk, unsigned) {
  std::vector<spf_edge_delta>& lst = found[blk];
  auto emit = [&](uint32_t u, uint32_t v, uint64_t w, uint32_t kind, uint32_t scope) {
    lst.push_back(spf_edge_delta{u, v, w, kind, scope});
  };
  using HE = std::pair<uint32_t, uint64_t>; // (head, metric)
  std::vector<HE> a, b;
  for (uint32_t u = bnd[blk]; u < bnd[blk + 1]; ++u) {
    const bool trA = !before->node_overloaded[u], trB = !after->node_overloaded[u];
    const uint32_t ra = before->row_ptr[u], na = before->row_ptr[u + 1] - ra;
    const uint32_t rb = after->row_ptr[u], nb = after->row_ptr[u + 1] - rb;
    if (na == nb && std::equal(before->col + ra, before->col + ra + na, after->col + rb) &&
        std::equal(before->metric + ra, before->metric + ra + na, after->metric + rb)) {
      // the common case: this row is unchanged (only its transit bit may flip)
      if (trA != trB) {
        for (uint32_t k = 0; k < na; ++k) {
          emit(u, before->col[ra + k], before->metric[ra + k],
               trA ? SPF_DELTA_REMOVED : SPF_DELTA_ADDED, SPF_SCOPE_NOT_TAIL);
        }
      }
      continue;
    }
    a.clear();
    b.clear();
    for (uint32_t e = before->row_ptr[u]; e < before->row_ptr[u + 1]; ++e) {
      a.emplace_back(before->col[e], before->metric[e]);
    }
    for (uint32_t e = after->row_ptr[u]; e < after->row_ptr[u + 1]; ++e) {
      b.emplace_back(after->col[e], after->metric[e]);
    }
    std::sort(a.begin(), a.end());
    std::sort(b.begin(), b.end());
    size_t i = 0, j = 0;
    while (i < a.size() || j < b.size()) {
      if (j == b.size() || (i < a.size() && a[i] < b[j])) {
        emit(u, a[i].first, a[i].second, SPF_DELTA_REMOVED, trA ? SPF_SCOPE_ALL : SPF_SCOPE_TAIL_ONLY);
        ++i;
      } else if (i == a.size() || b[j] < a[i]) {
        emit(u, b[j].first, b[j].second, SPF_DELTA_ADDED, trB ? SPF_SCOPE_ALL : SPF_SCOPE_TAIL_ONLY);
        ++j;
      } else {
        if (trA && !trB) {
          emit(u, a[i].first, a[i].second, SPF_DELTA_REMOVED, SPF_SCOPE_NOT_TAIL);
        } else if (!trA && trB) {
          emit(u, a[i].first, a[i].second, SPF_DELTA_ADDED, SPF_SCOPE_NOT_TAIL);
        }
        ++i;
        ++j;
      }
    }
  }
  }, 1);
  uint64_t n = 0;
  for (const auto& lst : found) {
    for (const spf_edge_delta& d : lst) {
      if (n < cap) {
        out[n] = d;
      }
      ++n;
    }
  }
  if (n > 0xFFFFFFFFull) {
    return fail(SPF_E_UNSUPPORTED, "more than 2^32 deltas");
  }
  *n_out = (uint32_t)n;
  return SPF_OK;
}

int spf_table_screen(
    spf_graph* g, const uint32_t* rows, size_t pitch, uint32_t num_rows,
    const uint32_t* sources, const spf_edge_delta* deltas, uint32_t n_deltas,
    uint8_t* affected) {
  SPF_ABI_RANGE("spf_table_screen");
  if (!g || (num_rows && (!rows || !sources || !affected)) || (n_deltas && !deltas)) {
    return fail(SPF_E_INVALID, "null argument");
  }
  if (num_rows && pitch < g->V) {
    return fail(SPF_E_INVALID, "row pitch < V");
  }
  for (uint32_t i = 0; i < num_rows; ++i) {
    if (sources[i] >= g->V) {
      return fail(SPF_E_INVALID, "source out of range");
    }
  }
  for (uint32_t j = 0; j < n_deltas; ++j) {
    if (deltas[j].tail >= g->V || deltas[j].head >= g->V ||
        (deltas[j].kind != SPF_DELTA_REMOVED && deltas[j].kind != SPF_DELTA_ADDED) ||
        deltas[j].scope > SPF_SCOPE_NOT_TAIL) {
      return fail(SPF_E_INVALID, "bad delta " + std::to_string(j));
    }
  }
  if (num_rows == 0) {
    return SPF_OK;
  }
  if (n_deltas == 0) {
    std::memset(affected, 0, num_rows);
    return SPF_OK;
  }
  HIP_TRY(hipSetDevice(g->device));
  // one device block: sources | tail | head | kind | metric (8-aligned) | flags
  const size_t nd = n_deltas;
  const size_t words = (size_t)num_rows + 3 * nd;
  const size_t moff = (words * 4 + 7) & ~(size_t)7;
  const size_t bytes = moff + nd * 8 + num_rows;
  std::vector<char> h(bytes);
  std::memcpy(h.data(), sources, (size_t)num_rows * 4);
  uint32_t* ht = (uint32_t*)(h.data() + (size_t)num_rows * 4);
  uint64_t* hm = (uint64_t*)(h.data() + moff);
  for (size_t j = 0; j < nd; ++j) {
    ht[j] = deltas[j].tail;
    ht[nd + j] = deltas[j].head;
    ht[2 * nd + j] = deltas[j].kind | (deltas[j].scope << 4);
    hm[j] = deltas[j].metric;
  }
  char* d = nullptr;
  HIP_TRY(hipMalloc((void**)&d, bytes));
  int st = SPF_OK;
  if (hipMemcpyAsync(d, h.data(), moff + nd * 8, hipMemcpyHostToDevice, g->stream) != hipSuccess) {
    st = fail(SPF_E_DEVICE, "delta upload failed");
  }
  if (st == SPF_OK) {
    ScreenArgs a;
    a.rows = rows;
    a.pitch = pitch;
    a.src = (const uint32_t*)d;
    a.tail = (const uint32_t*)(d + (size_t)num_rows * 4);
    a.head = a.tail + nd;
    a.kind = a.tail + 2 * nd;
    a.metric = (const uint64_t*)(d + moff);
    a.nrows = num_rows;
    a.ndelta = n_deltas;
    a.affected = (uint8_t*)(d + moff + nd * 8);
    SPF_LAUNCH(spf_table_screen_kernel, dim3((num_rows + 255) / 256), dim3(256), 0,
                       g->stream, a);
    if (hipGetLastError() != hipSuccess ||
        hipMemcpyAsync(affected, a.affected, num_rows, hipMemcpyDeviceToHost, g->stream) != hipSuccess ||
        hipStreamSynchronize(g->stream) != hipSuccess) {
      st = fail(SPF_E_DEVICE, "screen kernel failed");
    }
  }
  (void)hipStreamSynchronize(g->stream);
  (void)hipFree(d);
  return st;
}

int spf_query_scatter_rows(
    spf_query* q, const uint32_t* dst_rows, void* table, size_t pitch) {
  SPF_ABI_RANGE("spf_query_scatter_rows");
  if (!q || (q->nq && (!dst_rows || !table))) {
    return fail(SPF_E_INVALID, "null argument");
  }
  if (!q->ran) {
    return fail(SPF_E_INVALID, "query has not run");
  }
  if (rows64(q)) {
    return fail(SPF_E_UNSUPPORTED, "64-bit distance rows: use spf_query_dist");
  }
  const uint32_t V = q->g->V;
  if (pitch < (size_t)V * 4) {
    return fail(SPF_E_INVALID, "destination pitch < 4*V");
  }
  if (q->nq == 0 || V == 0) {
    return SPF_OK;
  }
  HIP_TRY(hipSetDevice(q->g->device));
  if (!q->d_scatter) {
    HIP_TRY(pool_malloc((void**)&q->d_scatter, (size_t)q->nq * 4));
  }
  // the previous scatter of this query may still read d_scatter
  HIP_TRY(hipStreamSynchronize(q->g->stream));
  HIP_TRY(hipMemcpy(q->d_scatter, dst_rows, (size_t)q->nq * 4, hipMemcpyHostToDevice));
  const uint32_t chunk = 256 * 16;
  SPF_LAUNCH(spf_scatter_rows_kernel, dim3(q->nq, (V + chunk - 1) / chunk), dim3(256), 0,
                     q->g->stream, (const uint32_t*)q->d_dist, q->Vp, q->d_scatter,
                     (char*)table, pitch, V);
  HIP_TRY(hipGetLastError());
  return SPF_OK;
}

} // extern "C"

extern "C" {

int spf_table_nexthops(
    spf_graph* g, const uint32_t* rows, size_t pitch, const int32_t* row_of, uint32_t num,
    const uint32_t* sources, uint64_t* masks, const uint64_t* mask_off) {
  SPF_ABI_RANGE("spf_table_nexthops");
  if (!g || (num && (!rows || !row_of || !sources || !masks || !mask_off))) {
    return fail(SPF_E_INVALID, "null argument");
  }
  if (num == 0 || g->V == 0) {
    return SPF_OK;
  }
  if (g->exact) {
    return fail(SPF_E_UNSUPPORTED, "64-bit rows");
  }
  if (pitch < g->V || pitch > 0xFFFFFFFFull) {
    return fail(SPF_E_INVALID, "pitch");
  }
  const uint32_t V = g->V;
  // every source's row and every neighbour's row must be in the table
  for (uint32_t i = 0; i < num; ++i) {
    const uint32_t s0 = sources[i];
    if (s0 >= V || row_of[s0] < 0) {
      return fail(SPF_E_INVALID, "source without a table row");
    }
    for (uint32_t k = g->nbr_off[s0]; k < g->nbr_off[s0 + 1]; ++k) {
      if (row_of[g->nbrs[k]] < 0) {
        return fail(SPF_E_INVALID, "neighbour without a table row");
      }
    }
  }
  std::vector<uint32_t> nw(num);
  for (uint32_t i = 0; i < num; ++i) {
    const uint32_t nn = g->nbr_off[sources[i] + 1] - g->nbr_off[sources[i]];
    nw[i] = std::max<uint32_t>(1, (nn + 63) / 64);
  }
  HIP_TRY(hipSetDevice(g->device));
  uint32_t *d_src = nullptr, *d_w = nullptr;
  int32_t* d_row_of = nullptr;
  uint64_t* d_off = nullptr;
  int st = SPF_OK;
  auto release = [&]() {
    (void)hipStreamSynchronize(g->stream);
    pool_free(d_src);
    pool_free(d_w);
    pool_free(d_row_of);
    pool_free(d_off);
  };
  if ((st = dev_upload_q(&d_src, sources, num)) || (st = dev_upload_q(&d_w, nw.data(), num)) ||
      (st = dev_upload_q(&d_row_of, row_of, V)) || (st = dev_upload_q(&d_off, mask_off, num))) {
    release();
    return st;
  }
  NhRowsArgs a;
  a.nbr_off = g->d_nbr_off;
  a.nbrs = g->d_nbrs;
  a.nbr_w = g->d_nbr_w;
  a.trbits = g->d_tr;
  a.src = d_src;
  a.row_of = d_row_of;
  a.dist = rows;
  a.nh_off = d_off;
  a.nh_w = d_w;
  a.nh_out = masks;
  a.V = V;
  a.Vp = (uint32_t)pitch;
  a.nq = num;
  a.nchunks = (V + kNhChunk - 1) / kNhChunk;
  a.unit = 0;
  a.table = 1;
  const uint64_t blocks = (uint64_t)a.nchunks * num;
  if (blocks > 0x7FFFFFFFull) {
    release();
    return fail(SPF_E_UNSUPPORTED, "too many rows for one next-hop pass");
  }
  SPF_LAUNCH(spf_nh_rows_kernel, dim3((uint32_t)blocks), dim3(kNhThreads), 0, g->stream, a);
  const hipError_t le = hipGetLastError();
  release(); // waits for the pass: the index buffers go back to the pool
  if (le != hipSuccess) {
    return fail(SPF_E_DEVICE, std::string("spf_nh_rows_kernel: ") + hipGetErrorString(le));
  }
  return SPF_OK;
}

int spf_table_repair(
    spf_graph* g, uint32_t* rows, size_t pitch, uint32_t num_rows,
    const uint32_t* sources, const uint32_t* row_idx,
    const spf_edge_delta* deltas, uint32_t n_deltas) {
  SPF_ABI_RANGE("spf_table_repair");
  if (!g || (num_rows && (!rows || !sources || !row_idx)) || (n_deltas && !deltas)) {
    return fail(SPF_E_INVALID, "null argument");
  }
  if (num_rows && pitch < g->V) {
    return fail(SPF_E_INVALID, "row pitch < V");
  }
  if (g->exact) {
    return fail(SPF_E_UNSUPPORTED, "metric 0 / 64-bit sums: rows need the exact kernel");
  }
  for (uint32_t i = 0; i < num_rows; ++i) {
    if (sources[i] >= g->V) {
      return fail(SPF_E_INVALID, "source out of range");
    }
  }
  std::vector<uint32_t> seeds, rt, rh, rs;
  std::vector<uint64_t> rw;
  for (uint32_t j = 0; j < n_deltas; ++j) {
    const spf_edge_delta& d = deltas[j];
    if (d.tail >= g->V || d.head >= g->V || d.scope > SPF_SCOPE_NOT_TAIL ||
        (d.kind != SPF_DELTA_REMOVED && d.kind != SPF_DELTA_ADDED)) {
      return fail(SPF_E_INVALID, "bad delta " + std::to_string(j));
    }
    if (d.kind == SPF_DELTA_ADDED) {
      seeds.push_back(d.tail);
    } else {
      rt.push_back(d.tail);
      rh.push_back(d.head);
      rs.push_back(d.scope);
      rw.push_back(d.metric);
    }
  }
  std::sort(seeds.begin(), seeds.end());
  seeds.erase(std::unique(seeds.begin(), seeds.end()), seeds.end());
  const size_t bk = ((size_t)g->V + 15) & ~(size_t)15;
  const size_t lds = (2 * (size_t)g->nbw + kCtlWords) * 4 + bk + (size_t)g->nbw * 4;
  if (lds > kLdsLimit) {
    return fail(SPF_E_UNSUPPORTED, "bucket image beyond LDS");
  }
  if (num_rows == 0 || n_deltas == 0 || g->V == 0) {
    return SPF_OK;
  }
  HIP_TRY(hipSetDevice(g->device));
  const uint32_t nrem = (uint32_t)rt.size(), nseed = (uint32_t)seeds.size();
  const uint32_t grid = std::min<uint32_t>(num_rows, (uint32_t)g->num_cus);
  // u32 block: sources | row_idx | seeds | rm_tail | rm_head | rm_scope, then
  // the u64 removed metrics, then two V-entry queues per workgroup
  const size_t n32 = (size_t)2 * num_rows + nseed + 3 * (size_t)nrem;
  const size_t off64 = (n32 * 4 + 7) & ~(size_t)7;
  const size_t meta = off64 + (size_t)nrem * 8;
  const size_t offq = (meta + 255) & ~(size_t)255;
  const size_t bytes = offq + (size_t)grid * g->V * 8;
  std::vector<char> h(meta);
  uint32_t* h32 = (uint32_t*)h.data();
  std::memcpy(h32, sources, (size_t)num_rows * 4);
  std::memcpy(h32 + num_rows, row_idx, (size_t)num_rows * 4);
  size_t o = 2 * (size_t)num_rows;
  for (auto* v : {&seeds, &rt, &rh, &rs}) {
    if (!v->empty()) {
      std::memcpy(h32 + o, v->data(), v->size() * 4);
    }
    o += v->size();
  }
  if (nrem) {
    std::memcpy(h.data() + off64, rw.data(), (size_t)nrem * 8);
  }
  if (g->repair_bytes < bytes) {
    HIP_TRY(hipStreamSynchronize(g->stream));
    if (g->d_repair) {
      HIP_TRY(hipFree(g->d_repair));
      g->d_repair = nullptr;
      g->repair_bytes = 0;
    }
    HIP_TRY(hipMalloc((void**)&g->d_repair, bytes));
    g->repair_bytes = bytes;
  }
  char* d = g->d_repair;
  int st = SPF_OK;
  if (hipMemcpyAsync(d, h.data(), meta, hipMemcpyHostToDevice, g->stream) != hipSuccess) {
    st = fail(SPF_E_DEVICE, "delta upload failed");
  }
  if (st == SPF_OK) {
    const uint32_t* d32 = (const uint32_t*)d;
    DstepArgs da;
    SsspArgs& a = da.s;
    std::memset(&a, 0, sizeof(a));
    a.row = g->d_row;
    a.col = g->d_col;
    a.wout = g->d_wout;
    a.win = g->d_win;
    a.link = g->d_link;
    a.rev = g->d_rev;
    a.slot = g->d_slot;
    a.trbits = g->d_tr;
    a.src = d32;
    a.gscratch = (uint32_t*)(d + offq);
    a.V = g->V;
    a.Vp = (uint32_t)std::min<size_t>(pitch, 0xFFFFFFFFu);
    a.nbw = g->nbw;
    a.nq = num_rows;
    a.G = 8;
    da.shift = dstep_bucket_shift(g, false);
    da.fshift = da.shift;
    // coherent gathers + non-returning atomics and 16-byte packed edges, as
    // the full pass (dstep_tune); bucket bytes at the bucket width
    da.noret = 3;
    if (g->cw_bits) {
      da.cw = g->d_cw;
      da.cwbits = g->cw_bits;
      da.cwvec = 1;
    }
    da.table = rows;
    da.pitch = pitch;
    da.row_idx = d32 + num_rows;
    da.seed = d32 + 2 * (size_t)num_rows;
    da.nseed = nseed;
    da.rm_tail = da.seed + nseed;
    da.rm_head = da.rm_tail + nrem;
    da.rm_scope = da.rm_head + nrem;
    da.rm_w = (const uint64_t*)(d + off64);
    da.nrem = nrem;
    da.gscratch2 = a.gscratch + (size_t)grid * g->V;
    auto kern = g->cw_bits ? spf_dstep_kernel<0, false, 1024, true, true, true>
                           : spf_dstep_kernel<0, false, 1024, true, true, false>;
    if (hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)lds) != hipSuccess) {
      st = fail(SPF_E_DEVICE, "LDS attribute");
    } else {
      SPF_LAUNCH_AS("spf_dstep_kernel", kern, dim3(grid), dim3(1024), lds, g->stream, da);
      if (hipGetLastError() != hipSuccess || hipStreamSynchronize(g->stream) != hipSuccess) {
        st = fail(SPF_E_DEVICE, "repair kernel failed");
      }
    }
  }
  (void)hipStreamSynchronize(g->stream);
  return st;
}

} // extern "C"

// ============================================ all-nodes unicast route table

struct spf_route_table {
  spf_query* q = nullptr;
  uint32_t P = 0;
  std::vector<uint64_t> lk_off; // [nq + 1]
  uint32_t *d_ann_off = nullptr, *d_ann = nullptr, *d_metric = nullptr, *d_best = nullptr;
  uint64_t *d_lk_off = nullptr, *d_links = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  bool ran = false;
  // spf_route_table_diff against an older table: changed-cell bitmap
  uint64_t* d_diff = nullptr;
  uint32_t* d_count = nullptr;
  // SPF_RT_LFA
  bool lfa = false;
  std::vector<uint64_t> lm_off; // [nq + 1] per-link metric offsets (P * deg)
  uint64_t* d_lm_off = nullptr;
  uint32_t* d_lmet = nullptr;
  int32_t* d_row_of = nullptr;
};

namespace {
void free_route_table(spf_route_table* t) {
  if (!t) {
    return;
  }
  (void)hipSetDevice(t->q->g->device);
  t->q->live_tables.fetch_sub(1, std::memory_order_relaxed);
  for (void* p : {(void*)t->d_ann_off, (void*)t->d_ann, (void*)t->d_metric, (void*)t->d_best,
                  (void*)t->d_lk_off, (void*)t->d_links, (void*)t->d_diff, (void*)t->d_count,
                  (void*)t->d_lm_off, (void*)t->d_lmet, (void*)t->d_row_of}) {
    if (p) {
      (void)hipFree(p);
    }
  }
  if (t->ev0) {
    (void)hipEventDestroy(t->ev0);
  }
  if (t->ev1) {
    (void)hipEventDestroy(t->ev1);
  }
  delete t;
}
} // namespace

extern "C" {

int spf_route_table_create(
    spf_query* q, uint32_t num_prefixes, const uint32_t* ann_offsets,
    const uint32_t* announcers, spf_route_table** out) {
  return spf_route_table_create_ex(q, num_prefixes, ann_offsets, announcers, 0, out);
}

int spf_route_table_create_ex(
    spf_query* q, uint32_t num_prefixes, const uint32_t* ann_offsets,
    const uint32_t* announcers, uint32_t flags, spf_route_table** out) {
  SPF_ABI_RANGE("spf_route_table_create");
  if (!q || !out || (num_prefixes && !ann_offsets)) {
    return fail(SPF_E_INVALID, "null argument");
  }
  *out = nullptr;
  if (!(q->flags & SPF_F_NEXTHOPS) || (q->flags & SPF_F_UNIT_METRIC) || q->has_ign) {
    return fail(SPF_E_INVALID, "route tables need a metric query with next hops and no ignore lists");
  }
  if (rows64(q)) {
    return fail(SPF_E_UNSUPPORTED, "64-bit distance rows");
  }
  const spf_graph* g = q->g;
  if (ann_offsets && ann_offsets[0] != 0) {
    return fail(SPF_E_INVALID, "ann_offsets[0] != 0");
  }
  const uint32_t na = num_prefixes ? ann_offsets[num_prefixes] : 0;
  if (na && !announcers) {
    return fail(SPF_E_INVALID, "null announcers");
  }
  for (uint32_t p = 0; p < num_prefixes; ++p) {
    if (ann_offsets[p + 1] < ann_offsets[p]) {
      return fail(SPF_E_INVALID, "ann_offsets not monotone");
    }
  }
  for (uint32_t i = 0; i < na; ++i) {
    if (announcers[i] >= g->V) {
      return fail(SPF_E_INVALID, "announcer out of range");
    }
  }
  std::vector<uint32_t> src(q->nq);
  HIP_TRY(hipSetDevice(g->device));
  HIP_TRY(hipMemcpy(src.data(), q->d_src, (size_t)q->nq * 4, hipMemcpyDeviceToHost));
  const bool lfa = flags & SPF_RT_LFA;
  std::vector<int32_t> row_of;
  if (lfa) {
    // every neighbour's row must be in the batch, every source on the
    // staged register path (degree <= kRtStage, <= 256 distinct neighbours)
    row_of.assign(g->V, -1);
    for (uint32_t i = q->nq; i-- > 0;) {
      row_of[src[i]] = (int32_t)i;
    }
    for (uint32_t i = 0; i < q->nq; ++i) {
      const uint32_t s0 = src[i];
      if (g->row[s0 + 1] - g->row[s0] > kRtStage || q->nh_w[i] > kRtMaskWords) {
        return fail(SPF_E_UNSUPPORTED, "LFA route table: a source with more than 1024 links "
                                       "or 256 neighbours");
      }
      for (uint32_t e = g->row[s0]; e < g->row[s0 + 1]; ++e) {
        if (row_of[g->col[e]] < 0) {
          return fail(SPF_E_UNSUPPORTED, "LFA route table: a neighbour's row is not in the batch");
        }
      }
    }
  }
  auto* t = new spf_route_table();
  t->q = q;
  q->live_tables.fetch_add(1, std::memory_order_relaxed); // free_route_table gives it back
  t->P = num_prefixes;
  t->lfa = lfa;
  t->lk_off.assign(q->nq + 1, 0);
  t->lm_off.assign(q->nq + 1, 0);
  for (uint32_t i = 0; i < q->nq; ++i) {
    const uint32_t deg = g->row[src[i] + 1] - g->row[src[i]];
    t->lk_off[i + 1] = t->lk_off[i] + (uint64_t)num_prefixes * ((deg + 63) / 64);
    t->lm_off[i + 1] = t->lm_off[i] + (lfa ? (uint64_t)num_prefixes * deg : 0);
  }
  auto bail = [&](int st) {
    free_route_table(t);
    return st;
  };
  if (lfa) {
    int s1 = SPF_OK;
    if ((s1 = dev_upload(&t->d_row_of, row_of.data(), row_of.size())) ||
        (s1 = dev_upload(&t->d_lm_off, t->lm_off.data(), t->lm_off.size()))) {
      return bail(s1);
    }
    if (t->lm_off.back() &&
        hipMalloc((void**)&t->d_lmet, t->lm_off.back() * 4) != hipSuccess) {
      return bail(fail(SPF_E_NOMEM, "LFA link metrics"));
    }
  }
  const size_t cells = (size_t)q->nq * num_prefixes;
  std::vector<uint32_t> off(ann_offsets, ann_offsets + num_prefixes + 1);
  if (num_prefixes == 0) {
    off.assign(1, 0);
  }
  int st = SPF_OK;
  if ((st = dev_upload(&t->d_ann_off, off.data(), off.size())) ||
      (na && (st = dev_upload(&t->d_ann, announcers, na))) ||
      (st = dev_upload(&t->d_lk_off, t->lk_off.data(), t->lk_off.size()))) {
    return bail(st);
  }
  if (cells) {
    if (hipMalloc((void**)&t->d_metric, cells * 4) != hipSuccess ||
        hipMalloc((void**)&t->d_best, cells * 4) != hipSuccess ||
        (t->lk_off.back() &&
         hipMalloc((void**)&t->d_links, t->lk_off.back() * 8) != hipSuccess)) {
      return bail(fail(SPF_E_NOMEM, "route table allocation"));
    }
  }
  if (hipEventCreate(&t->ev0) != hipSuccess || hipEventCreate(&t->ev1) != hipSuccess) {
    return bail(fail(SPF_E_DEVICE, "hipEventCreate"));
  }
  *out = t;
  return SPF_OK;
}

int spf_route_table_destroy(spf_route_table* t) {
  SPF_ABI_RANGE("spf_route_table_destroy");
  free_route_table(t);
  return SPF_OK;
}

int spf_route_table_run(spf_route_table* t) {
  SPF_ABI_RANGE("spf_route_table_run");
  if (!t) {
    return fail(SPF_E_INVALID, "null table");
  }
  spf_query* q = t->q;
  if (!q->ran) {
    return fail(SPF_E_INVALID, "the query has not run");
  }
  spf_graph* g = q->g;
  HIP_TRY(hipSetDevice(g->device));
  HIP_TRY(hipEventRecord(t->ev0, g->stream));
  if (q->nq && t->P) {
    RouteTableArgs a;
    a.row = g->d_row;
    a.col = g->d_col;
    a.wout = g->d_wout;
    a.slot = g->d_slot;
    a.trbits = g->d_tr;
    a.src = q->d_src;
    a.dist = (const uint32_t*)q->d_dist;
    a.nh = q->d_nhb;
    a.nh_off = q->d_nhb_off;
    a.nh_b = q->d_nh_b;
    a.nh_w = q->d_nh_w;
    a.ann_off = t->d_ann_off;
    a.ann = t->d_ann;
    a.lk_off = t->d_lk_off;
    a.metric_out = t->d_metric;
    a.best_out = t->d_best;
    a.link_out = t->d_links;
    a.row_of = t->d_row_of;
    a.lm_off = t->d_lm_off;
    a.lmet_out = t->d_lmet;
    a.lfa = t->lfa ? 1u : 0u;
    a.Vp = q->Vp;
    a.P = t->P;
    a.nq = q->nq;
    const uint32_t grid = std::min<uint32_t>(q->nq, (uint32_t)g->num_cus * 8);
    SPF_LAUNCH(spf_route_table_kernel, dim3(grid), dim3(256), 0, g->stream, a);
    HIP_TRY(hipGetLastError());
  }
  HIP_TRY(hipEventRecord(t->ev1, g->stream));
  t->ran = true;
  return SPF_OK;
}

int spf_route_table_elapsed_ms(spf_route_table* t, float* ms) {
  if (!t || !ms || !t->ran) {
    return fail(SPF_E_INVALID, "no run to time");
  }
  HIP_TRY(hipEventSynchronize(t->ev1));
  HIP_TRY(hipEventElapsedTime(ms, t->ev0, t->ev1));
  return SPF_OK;
}

int spf_route_table_link_words(const spf_route_table* t, uint32_t i) {
  if (!t || i >= t->q->nq) {
    return fail(SPF_E_INVALID, "row out of range");
  }
  return t->P ? (int)((t->lk_off[i + 1] - t->lk_off[i]) / t->P) : 0;
}

int spf_route_table_fetch(
    spf_route_table* t, uint32_t i, uint32_t* metric, uint32_t* best, uint64_t* links) {
  SPF_ABI_RANGE("spf_route_table_fetch");
  if (!t || i >= t->q->nq || (t->P && (!metric || !best))) {
    return fail(SPF_E_INVALID, "bad argument");
  }
  if (!t->ran) {
    return fail(SPF_E_INVALID, "table has not run");
  }
  if (t->P == 0) {
    return SPF_OK;
  }
  spf_graph* g = t->q->g;
  HIP_TRY(hipSetDevice(g->device));
  HIP_TRY(hipStreamSynchronize(g->stream));
  const size_t o = (size_t)i * t->P;
  HIP_TRY(hipMemcpy(metric, t->d_metric + o, (size_t)t->P * 4, hipMemcpyDeviceToHost));
  HIP_TRY(hipMemcpy(best, t->d_best + o, (size_t)t->P * 4, hipMemcpyDeviceToHost));
  const uint64_t nw = t->lk_off[i + 1] - t->lk_off[i];
  if (nw) {
    if (!links) {
      return fail(SPF_E_INVALID, "null links");
    }
    HIP_TRY(hipMemcpy(links, t->d_links + t->lk_off[i], nw * 8, hipMemcpyDeviceToHost));
  }
  return SPF_OK;
}

int spf_route_table_fetch_link_metrics(spf_route_table* t, uint32_t i, uint32_t* out) {
  SPF_ABI_RANGE("spf_route_table_fetch_link_metrics");
  if (!t || i >= t->q->nq) {
    return fail(SPF_E_INVALID, "bad argument");
  }
  if (!t->lfa) {
    return fail(SPF_E_INVALID, "not an LFA table (every next hop has the cell metric)");
  }
  if (!t->ran) {
    return fail(SPF_E_INVALID, "table has not run");
  }
  const uint64_t n = t->lm_off[i + 1] - t->lm_off[i];
  if (!n) {
    return SPF_OK;
  }
  if (!out) {
    return fail(SPF_E_INVALID, "null out");
  }
  spf_graph* g = t->q->g;
  HIP_TRY(hipSetDevice(g->device));
  HIP_TRY(hipStreamSynchronize(g->stream));
  HIP_TRY(hipMemcpy(out, t->d_lmet + t->lm_off[i], n * 4, hipMemcpyDeviceToHost));
  return SPF_OK;
}

} // extern "C"

extern "C" {

int spf_route_table_diff(spf_route_table* older, spf_route_table* newer, uint32_t* changed) {
  SPF_ABI_RANGE("spf_route_table_diff");
  if (!older || !newer || (newer->q->nq && !changed)) {
    return fail(SPF_E_INVALID, "null argument");
  }
  if (!older->ran || !newer->ran) {
    return fail(SPF_E_INVALID, "both tables must have run");
  }
  const spf_graph* ga = older->q->g;
  const spf_graph* gb = newer->q->g;
  if (ga->device != gb->device || older->q->nq != newer->q->nq || older->P != newer->P ||
      older->lk_off != newer->lk_off || ga->row != gb->row || ga->col != gb->col ||
      older->lfa != newer->lfa) {
    return fail(SPF_E_UNSUPPORTED,
                "tables differ in rows, prefixes or link layout (rematerialise instead)");
  }
  const uint32_t nq = newer->q->nq, P = newer->P, pw = (P + 63) / 64;
  if (nq == 0) {
    return SPF_OK;
  }
  HIP_TRY(hipSetDevice(gb->device));
  if (!newer->d_count) {
    HIP_TRY(hipMalloc((void**)&newer->d_count, (size_t)nq * 4));
    if (pw) {
      HIP_TRY(hipMalloc((void**)&newer->d_diff, (size_t)nq * pw * 8));
    }
  }
  // the older table's rows are read on the newer table's stream
  HIP_TRY(hipStreamSynchronize(ga->stream));
  HIP_TRY(hipMemsetAsync(newer->d_count, 0, (size_t)nq * 4, gb->stream));
  if (P) {
    const uint32_t grid = std::min<uint32_t>(nq, (uint32_t)gb->num_cus * 8);
    SPF_LAUNCH(spf_route_table_diff_kernel, dim3(grid), dim3(256), 0, gb->stream,
                       older->d_metric, older->d_best, older->d_links, newer->d_metric,
                       newer->d_best, newer->d_links, newer->d_lk_off, P, nq, pw,
                       newer->d_diff, newer->d_count, older->d_lmet, newer->d_lmet,
                       newer->d_lm_off);
    HIP_TRY(hipGetLastError());
  }
  HIP_TRY(hipMemcpyAsync(changed, newer->d_count, (size_t)nq * 4, hipMemcpyDeviceToHost,
                         gb->stream));
  HIP_TRY(hipStreamSynchronize(gb->stream));
  return SPF_OK;
}

int spf_route_table_changed(spf_route_table* t, uint32_t i, uint64_t* bits) {
  if (!t || i >= t->q->nq || !bits) {
    return fail(SPF_E_INVALID, "bad argument");
  }
  if (!t->d_count) {
    return fail(SPF_E_INVALID, "no diff has run on this table");
  }
  const uint32_t pw = (t->P + 63) / 64;
  if (!pw) {
    return SPF_OK;
  }
  HIP_TRY(hipSetDevice(t->q->g->device));
  HIP_TRY(hipStreamSynchronize(t->q->g->stream));
  HIP_TRY(hipMemcpy(bits, t->d_diff + (size_t)i * pw, (size_t)pw * 8, hipMemcpyDeviceToHost));
  return SPF_OK;
}

} // extern "C"
