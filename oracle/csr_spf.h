// csr_spf.h — CPU ORACLE, fast flat restatement (TEST INFRASTRUCTURE ONLY).
//
// The order-free restatement of LinkState::runSpf (LinkState.cpp:806-880)
// that SURVEY.md §8(a) validated against the reference (0 mismatches over
// 120,000 (src, dst) pairs, positive metrics):
//   d[]   = Dijkstra over the up half-edges, relax weight = metric advertised
//           by the tail (or 1 for useLinkMetric = false); a node u relaxes its
//           edges only if u == src or !overloaded(u) (LinkState.cpp:829-836);
//           half-edges whose undirected link id is in the query's ignore list
//           are skipped (linksToIgnore, LinkState.cpp:842-845);
//   NH(v) = union over tight usable in-edges u->v of (u == src ? {v} : NH(u))
//           (LinkState.cpp:855-871).
// Integer CSR, binary heap with lazy deletion, next-hop sets as bitsets over
// the source's distinct neighbours, sources spread over host threads.  Not
// valid for metric-0 edges (the discovery-ordered plateaus of SURVEY §8(a));
// the callers (goldens, the all-cores CPU baseline) use positive metrics.
//
// Used by tests/golden/make_golden.py (config-sized checksums the GPU tests
// compare against) and bench.py's cpu_baseline leg (the optimised-CPU line on
// every host core).  The product never links it.
#pragma once

#include <algorithm>
#include <atomic>
#include <cstdint>
#include <queue>
#include <thread>
#include <utility>
#include <vector>

namespace oracle {
namespace csr {

struct Graph {
  uint32_t V = 0;
  const uint32_t* row = nullptr;   // [V+1]
  const uint32_t* col = nullptr;   // [E]
  const uint64_t* w = nullptr;     // [E] metric advertised by the row node
  const uint32_t* link = nullptr;  // [E] undirected link id
  const uint8_t* overloaded = nullptr; // [V]
};

struct Query {
  uint32_t src;
  const uint32_t* ign = nullptr; // sorted link ids to skip
  uint32_t nign = 0;
};

constexpr uint64_t kInf = ~0ull;

inline uint64_t splitmix64(uint64_t x) {
  x += 0x9e3779b97f4a7c15ULL;
  x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ULL;
  x = (x ^ (x >> 27)) * 0x94d049bb133111ebULL;
  return x ^ (x >> 31);
}

// Per-query summary: reached nodes, sum of distances, number of (node,
// next-hop) pairs and an order-free mix of every (node, distance) and
// (node, next-hop node) pair:
//   mix = sum_v splitmix64((d[v] << 24) ^ v) + sum_{(v, n in NH(v))} splitmix64(((v + 1) << 32) | n)
struct Summary {
  uint64_t reached = 0, sumDist = 0, sumNh = 0, mix = 0;
};

// Scratch for one thread; `dist` and, when wanted, the next-hop bitsets.
struct Work {
  std::vector<uint64_t> dist;
  std::vector<uint8_t> done;
  std::vector<uint64_t> nh;    // V * W words
  std::vector<uint32_t> slotOf; // node -> slot among src's distinct nbrs (or ~0)
  std::vector<uint32_t> nbrs;   // slot -> node
};

// One SSSP.  Fills w.dist (kInf = unreached) and, if wantNh, w.nh with W
// words per node; returns W.
inline uint32_t run(const Graph& g, const Query& q, bool useMetric, bool wantNh, Work& w) {
  const uint32_t V = g.V;
  w.dist.assign(V, kInf);
  w.done.assign(V, 0);
  uint32_t W = 0;
  if (wantNh) {
    w.slotOf.assign(V, ~0u);
    w.nbrs.clear();
    for (uint32_t e = g.row[q.src]; e < g.row[q.src + 1]; ++e) {
      const uint32_t v = g.col[e];
      if (w.slotOf[v] == ~0u) {
        w.slotOf[v] = 0;
        w.nbrs.push_back(v);
      }
    }
    std::sort(w.nbrs.begin(), w.nbrs.end());
    for (uint32_t i = 0; i < w.nbrs.size(); ++i) w.slotOf[w.nbrs[i]] = i;
    W = std::max<uint32_t>(1, (uint32_t)((w.nbrs.size() + 63) / 64));
    w.nh.assign((size_t)V * W, 0);
  }
  using Item = std::pair<uint64_t, uint32_t>;
  std::priority_queue<Item, std::vector<Item>, std::greater<Item>> pq;
  w.dist[q.src] = 0;
  pq.push({0, q.src});
  while (!pq.empty()) {
    const auto [du, u] = pq.top();
    pq.pop();
    if (w.done[u] || du != w.dist[u]) continue;
    w.done[u] = 1;
    if (u != q.src && g.overloaded[u]) continue; // settled, never transited
    for (uint32_t e = g.row[u]; e < g.row[u + 1]; ++e) {
      const uint32_t v = g.col[e];
      if (w.done[v]) continue;
      if (q.nign && std::binary_search(q.ign, q.ign + q.nign, g.link[e])) continue;
      const uint64_t c = du + (useMetric ? g.w[e] : 1ull);
      if (c > w.dist[v]) continue;
      if (wantNh) {
        uint64_t* dst = &w.nh[(size_t)v * W];
        if (c < w.dist[v]) std::fill(dst, dst + W, 0ull);
        if (u == q.src) {
          const uint32_t s = w.slotOf[v];
          dst[s >> 6] |= 1ull << (s & 63);
        } else {
          const uint64_t* src = &w.nh[(size_t)u * W];
          for (uint32_t k = 0; k < W; ++k) dst[k] |= src[k];
        }
      }
      if (c < w.dist[v]) {
        w.dist[v] = c;
        pq.push({c, v});
      }
    }
  }
  return W;
}

inline Summary summarize(const Graph& g, bool wantNh, uint32_t W, const Work& w) {
  Summary s;
  for (uint32_t v = 0; v < g.V; ++v) {
    const uint64_t d = w.dist[v];
    if (d == kInf) continue;
    ++s.reached;
    s.sumDist += d;
    s.mix += splitmix64((d << 24) ^ v);
    if (!wantNh) continue;
    for (uint32_t k = 0; k < W; ++k) {
      uint64_t m = w.nh[(size_t)v * W + k];
      while (m) {
        const uint32_t b = (uint32_t)__builtin_ctzll(m);
        m &= m - 1;
        const uint32_t n = w.nbrs[k * 64 + b];
        ++s.sumNh;
        s.mix += splitmix64((((uint64_t)v + 1) << 32) | n);
      }
    }
  }
  return s;
}

// Every query on `threads` host threads (dynamic source claiming).
inline std::vector<Summary> summaries(const Graph& g, const std::vector<Query>& qs, bool useMetric,
                                      bool wantNh, unsigned threads) {
  std::vector<Summary> out(qs.size());
  std::atomic<size_t> next{0};
  auto worker = [&]() {
    Work w;
    for (size_t i; (i = next.fetch_add(1)) < qs.size();) {
      const uint32_t W = run(g, qs[i], useMetric, wantNh, w);
      out[i] = summarize(g, wantNh, W, w);
    }
  };
  threads = std::max(1u, threads);
  std::vector<std::thread> pool;
  for (unsigned t = 1; t < threads; ++t) pool.emplace_back(worker);
  worker();
  for (auto& t : pool) t.join();
  return out;
}

} // namespace csr
} // namespace oracle
