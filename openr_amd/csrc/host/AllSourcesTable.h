// AllSourcesTable.h — the distance rows of EVERY source of an area, resident
// on the device(s) and kept current under adjacency churn (SURVEY.md §8(f)
// row 2).
//
// The reference memoizes one SpfResult per (node, useLinkMetric) and drops
// the whole memo on every topology change (LinkState.cpp:510-511, 712-715,
// 728-729); a view of all nodes' distances (breeze / ctrl views, what-if
// tooling) recomputes every source after each change.  This table keeps
// one uint32 row per source (0xFFFFFFFF = unreached) in HBM and, after a
// change, repairs only what the change can reach:
//
//   spf_graph_diff (old, new CSR)            edge deltas (REMOVED / ADDED)
//   graph patch                              transit bits / metrics in place;
//                                            links down / back up in place
//                                            (spf_graph_set_edges, the
//                                            half-edges keep their slots);
//                                            a new link rebuilds the graph
//   spf_table_screen                         rows whose shortest-path DAG a
//                                            delta touches
//   spf_table_repair (or recompute+scatter)  those rows only
//
// The result equals a fresh all-sources pass bit for bit
// (tests/test_all_sources_table_gpu.py).  With devices configured
// (setSpfDevices) the sources are split into contiguous blocks, one per
// device; each device keeps the rows of its own block (the "no-gather" mode
// of SURVEY §8(e): every step runs on each device independently, no
// collective), and row() reads from the owner.  The C++ counterpart of
// openr_amd/allsources.py's ShardedAllSources, for a host that links the
// library directly (Open/R's Decision process).
#pragma once

#include <cstdint>
#include <optional>
#include <string>
#include <unordered_map>
#include <vector>

#include "LinkState.h"
#include "openr_spf.h"

namespace openr {

class AllSourcesTable {
 public:
  struct UpdateStats {
    uint32_t deltas{0};
    uint32_t affected{0};    // rows recomputed or repaired, over all blocks
    bool graphPatched{false}; // device graphs patched in place (no rebuild)
    bool relaxed{false};      // rows repaired in place (spf_table_repair)
    double diffMs{0}, graphMs{0}, screenMs{0}, spfMs{0}, nextHopsMs{0}, wallMs{0};
  };

  // Every node of `ls`'s area as a source, link metrics (getSpfResult(node,
  // true)).  `devices` empty: LinkState::getSpfDevices(), else device 0.
  // Throws std::invalid_argument for graphs that need 64-bit rows (metric 0,
  // sums that may pass 32 bits) and std::runtime_error on engine failures.
  explicit AllSourcesTable(const LinkState& ls, std::vector<int> devices = {});
  // withNextHops: also every source's ECMP next-hop masks (getSpfResult's
  // nextHops per node), kept current under churn from the table rows
  // (spf_table_nexthops, the all-sources rule).  A source's masks read its
  // neighbours' rows: with several devices each block also keeps "halo"
  // rows -- the neighbours of its sources that other blocks own, computed
  // and repaired on the block's own device with its rows -- so every step
  // still runs per device with no collective (round 6).
  AllSourcesTable(const LinkState& ls, std::vector<int> devices, bool withNextHops);
  ~AllSourcesTable();
  AllSourcesTable(const AllSourcesTable&) = delete;
  AllSourcesTable& operator=(const AllSourcesTable&) = delete;

  // Bring the rows to `ls`'s current topology (same node set; otherwise
  // std::invalid_argument: rebuild the table).  A topology that needs 64-bit
  // rows throws std::invalid_argument and leaves the table stale: row()
  // throws std::logic_error until an update() to a 32-bit topology succeeds.
  UpdateStats update(const LinkState& ls);
  // Recompute every row on the current graphs (device time in lastSpfMs()).
  void recompute();

  size_t numNodes() const { return names_.size(); }
  const std::vector<std::string>& nodeNames() const { return names_; }
  size_t numDevices() const { return blocks_.size(); }
  // distances from `src` to every node (node-name-rank order, see
  // nodeNames(); 0xFFFFFFFF = unreachable); std::out_of_range if unknown
  std::vector<uint32_t> row(const std::string& src) const;
  // getMetricFromAToB of the memoized SpfResult (nullopt if unreachable)
  std::optional<uint64_t> distance(const std::string& src, const std::string& dst) const;
  // next-hop node names from `src` towards `dst` (sorted by name; empty if
  // unreachable or src == dst); std::logic_error without withNextHops
  std::vector<std::string> nextHops(const std::string& src, const std::string& dst) const;
  bool hasNextHops() const { return withNh_; }
  double lastSpfMs() const { return lastSpfMs_; }

 private:
  struct Csr {
    std::vector<uint32_t> row, col, linkId, rev;
    std::vector<uint64_t> metric;
    std::vector<uint8_t> overloaded;
    uint32_t numLinks{0};
    spf_graph_desc desc(int device) const;
  };
  struct Block {
    int device{0};
    uint32_t first{0}, count{0};
    spf_graph* graph{nullptr};
    // device [sources.size()][V]: the block's own sources first (rows
    // 0..count-1), then its halo (withNextHops: neighbours owned elsewhere)
    uint32_t* rows{nullptr};
    size_t rowCap{0}; // rows allocated
    std::vector<uint32_t> sources;
    // next-hop masks of the own sources (withNextHops): device words,
    // per-source word offsets and widths, node -> row index (-1: none)
    uint64_t* masks{nullptr};
    size_t maskBytes{0};
    std::vector<uint64_t> maskOff;
    std::vector<uint32_t> maskWords;
    std::vector<int32_t> rowOf;
  };
  Csr snapshot(const LinkState& ls) const;
  void buildGraphs(const Csr& c);
  void computeBlock(Block& b, const std::vector<uint32_t>& idx, bool scatter);
  // withNextHops: the block's halo from the resident layout's heads (a
  // superset of every later neighbour list until the graphs are rebuilt);
  // true when it changed (rows reallocated: recompute the block)
  bool setHalo(Block& b);
  bool linksInPlace(const std::vector<spf_edge_delta>& deltas, std::vector<uint32_t>& edges,
                    std::vector<uint8_t>& up, std::vector<uint64_t>& w);
  // (re)compute the masks of block b's own rows idx (empty: every own row;
  // the layout is re-derived from the graph's current neighbour lists)
  void refreshMasks(Block& b, const std::vector<uint32_t>& idx);

  std::vector<std::string> names_;
  std::unordered_map<std::string, uint32_t> ids_;
  Csr cur_;
  // half-edge layout of the resident graphs (heads as created, up flags,
  // current metrics): links taken down / up in place keep their slots
  std::vector<uint32_t> layRow_, layCol_, layRev_;
  std::vector<uint8_t> layUp_;
  std::vector<uint64_t> layW_;
  std::vector<Block> blocks_;
  double lastSpfMs_{0};
  // an update() that threw after the graphs were patched (the new topology
  // needs 64-bit rows) left rows of the old topology: the next update()
  // rebuilds and recomputes, row() refuses until then
  bool stale_{false};
  bool withNh_{false};
};

} // namespace openr
