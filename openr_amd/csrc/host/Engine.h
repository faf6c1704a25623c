// Engine.h — LinkState's device-side state (internal to the host library).
//
// One per area: the flat CSR of the up links (ids = name ranks, rows in
// linksFromNode order), the spf_graph handle and the flat SPF memo.  Shared
// by LinkState.cpp and RouteTable.cpp; not part of the public API.
#pragma once

#include <array>
#include <map>
#include <memory>
#include <mutex>
#include <shared_mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "LinkState.h"
#include "openr_spf.h"

namespace openr {

struct LinkState::Engine {
  bool built{false};
  std::vector<std::string> names; // id -> name, ascending
  std::unordered_map<std::string, uint32_t> ids;
  std::vector<uint32_t> row, col, linkId, rev;
  std::vector<uint64_t> metric;
  std::vector<uint8_t> overloaded;
  std::vector<std::shared_ptr<Link>> links; // link id -> Link
  // Link -> link id of this build: the tag buildGraph left on the Link
  // (Link::engineEpoch / engineId), ~0u for links that are not up links of it
  uint64_t epoch{0};
  // (a copy of a Link carries the tag too, and freed ids are reused by
  // patchStructure: the id only counts if it still names this very Link)
  uint32_t linkIdOf(const Link* l) const {
    if (l->engineEpoch != epoch) {
      return ~0u;
    }
    const uint32_t id = l->engineId;
    return id < links.size() && links[id].get() == l ? id : ~0u;
  }
  std::vector<std::array<uint32_t, 2>> halves; // link id -> half-edge from first/second node
  // the arrays the last in-place link splice retired (patchStructure reuses
  // their capacity: no fresh pages per flap)
  std::vector<uint32_t> spareRow, spareCol, spareLinkId, spareRev;
  std::vector<uint64_t> spareMetric;
  std::vector<std::array<uint32_t, 2>> spareHalves; // the halves a splice replaced
  std::vector<uint8_t> spareAlive;
  // link ids freed by in-place link removals (LinkState::patchStructure):
  // links[id] == nullptr, reused by the next link that comes up
  std::vector<uint32_t> freeIds;
  spf_graph* graph{nullptr};
  // the same graph on every device of the multi-GPU fan-out (setSpfDevices),
  // created on the first fanned-out batch and patched with the same churn as
  // `graph`; cgraphGen = the cluster generation it was built for
  spf_cgraph* cgraph{nullptr};
  uint64_t cgraphGen{0};
  // host block the 32-bit rows of a batch land in (runBatch): reused while no
  // view of an earlier batch holds it, so big batches (the KSP2 second
  // passes: 9,975 x 9,976 rows on the fabric) skip the zero fill and the
  // page faults of a fresh 400 MB allocation
  std::shared_ptr<std::vector<uint32_t>> rowBlock;
  bool exact{false};
  float lastMs{0};
  std::unordered_map<uint32_t, std::unique_ptr<SpfView>> memo[2];
  std::unordered_map<uint32_t, std::unique_ptr<SpfView>> prefetched[2];
  std::map<std::pair<uint32_t, uint32_t>, std::unique_ptr<SpfView>> kthPrefetch;
  std::unordered_map<std::string, std::unique_ptr<SpfView>> isolated;
  // spfView may be called from the RouteDb worker threads of one build:
  // memo hits take viewMu shared, fills (and kthPrefetch inserts) exclusive;
  // a k = 2 fill moves its own prefetched view out under the shared lock
  // (the emptied entry stays until the next topology change); every
  // device call of this graph is serialised by devMu (the C ABI is
  // single-threaded per graph)
  std::shared_mutex viewMu;
  std::mutex devMu;
  // graphs the engine let go of while the C ABI refused to free them (a
  // query over them was still alive: include/openr_spf.h "Lifetime"); they
  // are freed by the next retireGraph / reapRetired that the ABI accepts,
  // never overwritten or leaked
  std::vector<spf_graph*> retired;

  // the last batch's query (runBatch), rerun when the next batch asks for the
  // same sources and flags with no ignore lists: transit bits are read at run
  // time (spf_graph_set_transit keeps it), every other change of the graph
  // (metric patches, link splices, a rebuild) drops it first.  A RouteDb
  // build on a small area (<= 4,096 nodes) pays the plan, the allocations
  // and the uploads of spf_query_create once instead of per build.
  // (OPENR_LS_QUERY_CACHE=0 disables)
  spf_query* lastQuery{nullptr};
  std::vector<uint32_t> lastSources;
  uint32_t lastFlags{0};
  void dropQuery() {
    if (lastQuery) {
      spf_query_destroy(lastQuery);
      lastQuery = nullptr;
    }
    lastSources.clear();
  }

  // drop `graph`: freed now, or kept in `retired` if the ABI refuses
  void retireGraph() {
    dropQuery();
    if (graph && spf_graph_destroy(graph) != SPF_OK) {
      retired.push_back(graph);
    }
    graph = nullptr;
    reapRetired();
  }
  void reapRetired() {
    std::vector<spf_graph*> keep;
    for (spf_graph* g : retired) {
      if (spf_graph_destroy(g) != SPF_OK) {
        keep.push_back(g);
      }
    }
    retired.swap(keep);
  }

  ~Engine() {
    if (cgraph) {
      spf_cgraph_destroy(cgraph);
    }
    retireGraph();
  }
};

} // namespace openr
