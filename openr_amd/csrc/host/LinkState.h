// LinkState.h — drop-in replacement of openr/decision/LinkState.h whose SPF
// runs on MI355X through the C ABI in include/openr_spf.h.
//
// Public surface kept identical to the reference (LinkState.h:36-469):
// HoldableValue, Link, LinkState (getSpfResult, getKthPaths,
// updateAdjacencyDatabase, deleteAdjacencyDatabase, decrementHolds, hop/metric
// queries, linksFromNode, ...), nested NodeSpfResult / PathLink / LinkSet /
// Path / LinkStateChange, std::hash<Link>.  The graph bookkeeping uses the same
// container types as the reference because their iteration orders are
// observable (parallel-link choice in KSP2 traces, duplicate adj labels).
//
// What changes is where the shortest paths come from: instead of a
// string-keyed DijkstraQ on the Decision thread (LinkState.cpp:806-880) the
// up-link graph is flattened into a device CSR (node id = name rank) and each
// SPF is a row of a batched GPU query.  `SpfView` is the flat per-source
// result (distances + next-hop masks); getSpfResult() materialises the
// reference's map form from it on demand.  Extensions beyond the reference API
// (prefetchSpf, spfView, prefetchKthPaths) let SpfSolver batch many sources
// into one launch.
#pragma once

#include <algorithm>
#include <limits>
#include <memory>
#include <optional>
#include <mutex>
#include <shared_mutex>
#include <string>
#include <thread>
#include <array>
#include <atomic>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "Types.h"

namespace openr {

using LinkStateMetric = uint64_t;

// RFC 6976 ordered-FIB hold (reference: LinkState.h:36-58, .cpp:54-125).
template <class T>
class HoldableValue {
 public:
  explicit HoldableValue(T val);
  void operator=(T val);
  const T& value() const;
  bool hasHold() const;
  // return true if the call changes value()
  bool decrementTtl();
  bool updateValue(T val, LinkStateMetric holdUpTtl, LinkStateMetric holdDownTtl);

 private:
  bool isChangeBringingUp(T val);
  T val_;
  std::optional<T> heldVal_;
  LinkStateMetric holdTtl_{0};
};

class Link {
 public:
  Link(
      const std::string& area,
      const std::string& nodeName1,
      const std::string& if1,
      const std::string& nodeName2,
      const std::string& if2);
  Link(
      const std::string& area,
      const std::string& nodeName1,
      const thrift::Adjacency& adj1,
      const std::string& nodeName2,
      const thrift::Adjacency& adj2);

 private:
  const std::string area_;
  const std::string n1_, n2_, if1_, if2_;
  HoldableValue<LinkStateMetric> metric1_{1}, metric2_{1};
  HoldableValue<bool> overload1_{false}, overload2_{false};
  int32_t adjLabel1_{0}, adjLabel2_{0};
  thrift::BinaryAddress nhV41_, nhV42_, nhV61_, nhV62_;
  LinkStateMetric holdUpTtl_{0};
  const std::pair<
      std::pair<std::string, std::string>,
      std::pair<std::string, std::string>>
      orderedNames_;

 public:
  const size_t hash{0};
  // the engine build that last numbered this link (LinkState.cpp buildGraph)
  // and the id it gave; bookkeeping of the device CSR, not link state
  mutable uint64_t engineEpoch{0};
  mutable uint32_t engineId{0};

  void setHoldUpTtl(LinkStateMetric ttl);
  bool isUp() const;
  bool decrementHolds();
  bool hasHolds() const;
  const std::string& getArea() const { return area_; }
  const std::string& getOtherNodeName(const std::string& nodeName) const;
  const std::string& firstNodeName() const;
  const std::string& secondNodeName() const;
  const std::string& getIfaceFromNode(const std::string& nodeName) const;
  LinkStateMetric getMetricFromNode(const std::string& nodeName) const;
  int32_t getAdjLabelFromNode(const std::string& nodeName) const;
  bool getOverloadFromNode(const std::string& nodeName) const;
  const thrift::BinaryAddress& getNhV4FromNode(const std::string& nodeName) const;
  const thrift::BinaryAddress& getNhV6FromNode(const std::string& nodeName) const;
  void setNhV4FromNode(const std::string& nodeName, const thrift::BinaryAddress& nhV4);
  void setNhV6FromNode(const std::string& nodeName, const thrift::BinaryAddress& nhV6);
  bool setMetricFromNode(
      const std::string& nodeName,
      LinkStateMetric d,
      LinkStateMetric holdUpTtl,
      LinkStateMetric holdDownTtl);
  void setAdjLabelFromNode(const std::string& nodeName, int32_t adjLabel);
  bool setOverloadFromNode(
      const std::string& nodeName,
      bool overload,
      LinkStateMetric holdUpTtl,
      LinkStateMetric holdDownTtl);
  const std::pair<
      std::pair<std::string, std::string>,
      std::pair<std::string, std::string>>&
  orderedNames() const {
    return orderedNames_;
  }
  bool operator<(const Link& other) const;
  bool operator==(const Link& other) const;
  std::string toString() const;
  std::string directionalToString(const std::string& fromNode) const;
};

// Flat single-source SPF result as produced by the device (one batch row).
// Distances of one SPF row, by node id: either an owned uint64 row (exact
// plan) or a window into a uint32 block shared by every row of one device
// batch (fast plans: one transfer, no per-row copy; 0xFFFFFFFF = not reached).
class DistRow {
 public:
  static constexpr uint64_t kUnreachable = ~0ull;
  // the 32-bit row this view shares, or nullptr (64-bit row)
  const uint32_t* raw32() const { return d32_; }
  uint64_t operator[](size_t v) const {
    if (d32_) {
      const uint32_t x = d32_[v];
      return x == 0xFFFFFFFFu ? kUnreachable : (uint64_t)x;
    }
    return d64_[v];
  }
  size_t size() const { return n_; }
  uint64_t* resize64(size_t n) {
    d64_.assign(n, kUnreachable);
    block_.reset();
    d32_ = nullptr;
    n_ = n;
    return d64_.data();
  }
  void share32(std::shared_ptr<const std::vector<uint32_t>> block, size_t offset, size_t n) {
    d64_.clear();
    d32_ = block->data() + offset;
    block_ = std::move(block);
    n_ = n;
  }

 private:
  std::vector<uint64_t> d64_;
  std::shared_ptr<const std::vector<uint32_t>> block_;
  const uint32_t* d32_{nullptr};
  size_t n_{0};
};

inline uint64_t nextSpfViewSerial() {
  static std::atomic<uint64_t> serial{0};
  return ++serial;
}

struct SpfView {
  uint64_t serial{nextSpfViewSerial()}; // identity for per-view caches
  uint32_t src{0};            // node id (name rank) of the source
  bool useLinkMetric{true};
  bool exact{false};          // settle order came from the exact kernel
  DistRow dist;               // per node id; kUnreachable = not reached
  uint32_t words{1};          // words per next-hop mask
  std::vector<uint64_t> nh;   // [V * words]
  std::vector<uint32_t> nbrs; // mask bit -> node id
  std::vector<uint32_t> order; // literal replay: settle rank per node id
  std::vector<uint64_t> okey;  // wide plan: settle order = (dist, okey)
  std::vector<uint32_t> ignored; // sorted link ids this run skipped
  static constexpr uint64_t kUnreachable = ~0ull;

  bool reached(uint32_t v) const { return v < dist.size() && dist[v] != kUnreachable; }
  // DijkstraQ's settle order between two reached nodes (LinkState.h:483-535)
  bool settlesBefore(uint32_t u, uint32_t v) const {
    if (exact && okey.empty()) {
      return order[u] < order[v];
    }
    const uint64_t du = dist[u], dv = dist[v];
    if (du != dv) {
      return du < dv;
    }
    return okey.empty() ? u < v : okey[u] < okey[v];
  }
  template <class Fn>
  void forEachNextHop(uint32_t v, Fn&& fn) const {
    const uint64_t* m = nh.data() + (size_t)v * words;
    for (uint32_t w = 0; w < words; ++w) {
      uint64_t b = m[w];
      while (b) {
        const int k = __builtin_ctzll(b);
        b &= b - 1;
        fn(nbrs[w * 64 + k]);
      }
    }
  }
};

class LinkState {
 public:
  explicit LinkState(const std::string& area);
  ~LinkState();
  LinkState(LinkState&&) noexcept;
  LinkState& operator=(LinkState&&) = delete;
  LinkState(const LinkState&) = delete;
  LinkState& operator=(const LinkState&) = delete;

  struct LinkPtrHash {
    size_t operator()(const std::shared_ptr<Link>& l) const;
  };
  struct LinkPtrLess {
    bool operator()(const std::shared_ptr<Link>& lhs, const std::shared_ptr<Link>& rhs) const;
  };
  struct LinkPtrEqual {
    bool operator()(const std::shared_ptr<Link>& lhs, const std::shared_ptr<Link>& rhs) const;
  };

  using LinkSet = std::unordered_set<std::shared_ptr<Link>, LinkPtrHash, LinkPtrEqual>;

  class NodeSpfResult {
   public:
    class PathLink {
     public:
      PathLink(std::shared_ptr<Link> const& l, std::string const& n)
          : link(l), prevNode(n) {}
      std::shared_ptr<Link> const link;
      std::string const prevNode;
    };
    explicit NodeSpfResult(LinkStateMetric m) : metric_(m) {}
    void reset(LinkStateMetric newMetric) {
      metric_ = newMetric;
      pathLinks_.clear();
      nextHops_.clear();
    }
    std::vector<PathLink> const& pathLinks() const { return pathLinks_; }
    std::unordered_set<std::string> const& nextHops() const { return nextHops_; }
    LinkStateMetric metric() const { return metric_; }
    void addPath(std::shared_ptr<Link> const& link, std::string const& prevNode) {
      pathLinks_.emplace_back(link, prevNode);
    }
    void addNextHops(std::unordered_set<std::string> const& toInsert) {
      nextHops_.insert(toInsert.begin(), toInsert.end());
    }
    void addNextHop(std::string const& toInsert) { nextHops_.insert(toInsert); }

   private:
    LinkStateMetric metric_{std::numeric_limits<LinkStateMetric>::max()};
    std::vector<PathLink> pathLinks_;
    std::unordered_set<std::string> nextHops_;
  };

  using SpfResult = std::unordered_map<std::string, NodeSpfResult>;
  using Path = std::vector<std::shared_ptr<Link>>;

  // memoized until the next topology change (reference: LinkState.cpp:791)
  SpfResult const& getSpfResult(const std::string& nodeName, bool useLinkMetric = true) const;

  // edge-disjoint path tracing (reference: LinkState.cpp:760-789)
  std::vector<Path> const& getKthPaths(
      const std::string& src, const std::string& dest, size_t k) const;

  class LinkStateChange {
   public:
    LinkStateChange() = default;
    LinkStateChange(bool topo, bool link, bool node)
        : topologyChanged(topo), linkAttributesChanged(link), nodeLabelChanged(node) {}
    bool operator==(LinkStateChange const& other) const {
      return topologyChanged == other.topologyChanged &&
          linkAttributesChanged == other.linkAttributesChanged &&
          nodeLabelChanged == other.nodeLabelChanged;
    }
    bool topologyChanged{false};
    bool linkAttributesChanged{false};
    bool nodeLabelChanged{false};
  };

  LinkStateChange decrementHolds();
  LinkStateChange updateAdjacencyDatabase(
      thrift::AdjacencyDatabase const& adjacencyDb,
      LinkStateMetric holdUpTtl = 0,
      LinkStateMetric holdDownTtl = 0);
  LinkStateChange updateAdjacencyDatabase(
      thrift::AdjacencyDatabase&& adjacencyDb,
      LinkStateMetric holdUpTtl = 0,
      LinkStateMetric holdDownTtl = 0);
  LinkStateChange deleteAdjacencyDatabase(const std::string& nodeName);

  std::optional<LinkStateMetric> getMetricFromAToB(
      std::string const& a, std::string const& b, bool useLinkMetric = true) const;
  std::optional<LinkStateMetric> getHopsFromAToB(std::string const& a, std::string const& b) const {
    return getMetricFromAToB(a, b, false);
  }
  LinkStateMetric getMaxHopsToNode(const std::string& nodeName) const;

  const std::string& getArea() const { return area_; }
  bool hasNode(const std::string& nodeName) const {
    return 0 != adjacencyDatabases_.count(nodeName);
  }
  const LinkSet& linksFromNode(const std::string& nodeName) const;
  bool isNodeOverloaded(const std::string& nodeName) const;
  bool hasHolds() const;
  size_t numLinks() const { return allLinks_.size(); }
  size_t numNodes() const { return linkMap_.size(); }
  std::unordered_map<std::string, thrift::AdjacencyDatabase> const&
  getAdjacencyDatabases() const {
    return adjacencyDatabases_;
  }

  // path A is a contiguous sub-path of B (reference: LinkState.h:395-410)
  static bool pathAInPathB(Path const& a, Path const& b);

  // Flat form of getKthPaths' result, the form it is computed and memoized
  // in: path i is links [begin(i), end(i)), device-graph link ids (linkOfId)
  // in path order.  Same paths in the same order, no Link refcounts touched;
  // valid until the next topology change.
  struct KthPathIds {
    std::vector<uint32_t> off{0};
    std::vector<uint32_t> links;
    size_t size() const { return off.size() - 1; }
    const uint32_t* begin(size_t i) const { return links.data() + off[i]; }
    const uint32_t* end(size_t i) const { return links.data() + off[i + 1]; }
  };
  const KthPathIds& kthPathIds(const std::string& src, const std::string& dest, size_t k) const;
  const Link& linkOfId(uint32_t id) const;

  // ---- MI355X engine extensions (not part of the reference API) ----

  // Flat SPF of `node`, memoized like getSpfResult (shares its spf_runs
  // accounting: the first access of a (node, useLinkMetric) counts one run).
  const SpfView& spfView(const std::string& node, bool useLinkMetric = true) const;
  // Compute the SPFs of many sources in one device batch (no counting until
  // they are first accessed through spfView/getSpfResult).
  void prefetchSpf(const std::vector<std::string>& nodes, bool useLinkMetric = true) const;
  // Run every second-pass (k = 2) SPF that getKthPaths(src, d, 2) would need
  // for d in dests, as one device batch.
  void prefetchKthPaths(const std::string& src, const std::vector<std::string>& dests) const;
  // node id (name rank) in the current device graph
  std::optional<uint32_t> nodeId(const std::string& name) const;
  const std::string& nodeNameOf(uint32_t id) const;
  // id -> name of the device graph (valid until the next topology change)
  const std::vector<std::string>& nodeNames() const;
  uint32_t numGraphNodes() const;
  // one hop of a path of device link ids (kthPathIds): from node id `from`
  // over link `linkId` to `to`, at the link's metric from `from`'s side;
  // false when the link is not an up link of the graph or `from` is not one
  // of its ends (the engine must be built: a RouteDb build's prefetch did)
  bool linkHop(uint32_t linkId, uint32_t from, uint32_t& to, LinkStateMetric& metric) const;
  // What-if link-failure SPFs (BASELINE config 5, LFA / failure
  // precomputation): runSpf(src, useLinkMetric, linksToIgnore[i])
  // (LinkState.cpp:806-880 -- the reference's own ignore-set semantics, which
  // it reaches only through getKthPaths, :776-777) for every i, as ONE device
  // batch.  Each query counts one decision.spf_runs, as each runSpf does.
  // Results stay flat; result(i) materialises the reference's SpfResult
  // (pathLinks in reference order) and, like getSpfResult's reference, is
  // valid only until the next topology change of this LinkState
  // (std::logic_error afterwards).
  class SpfBatch {
   public:
    size_t size() const { return views_.size(); }
    const SpfView& view(size_t i) const { return *views_.at(i); }
    SpfResult result(size_t i) const;

   private:
    friend class LinkState;
    const LinkState* ls_{nullptr};
    uint64_t gen_{0};
    std::string src_;
    std::vector<std::unique_ptr<SpfView>> views_;
  };
  std::unique_ptr<SpfBatch> runSpfBatch(
      const std::string& src,
      const std::vector<LinkSet>& linksToIgnore,
      bool useLinkMetric = true) const;
  // device time of the last batch, ms (HIP events)
  float lastDeviceMs() const;
  // release the device graph and every memoized result
  void invalidate() const;

  struct Engine; // device graph + flat memo (Engine.h)
  friend class AllNodesRouteTable; // reads the device graph (RouteTable.h)
  friend class AllSourcesTable;    // reads the flat CSR (AllSourcesTable.h)
  friend class AllAreasRouteTable; // checks the graph's row width (RouteTable.h)

 private:
  void clearMemo() const;
  // reference-form SpfResult of one flat view of the current device graph
  SpfResult materialize(const SpfView& view, const std::string& srcName) const;
  // bumped on every topology change (clearMemo / patchMemo): flat views of an
  // older generation are stale
  mutable uint64_t topoGen_{0};
  void patchMemo(
      const std::vector<std::string>& transitNodes,
      const std::vector<std::pair<std::shared_ptr<Link>, std::string>>& metricPatches) const;
  // links going down / coming up with the node set unchanged (link flaps):
  // the affected rows of the flat CSR are spliced in place and the memo is
  // screened with the edge deltas; false = not applicable (full rebuild)
  bool patchStructure(
      const std::vector<std::shared_ptr<Link>>& down,
      const std::vector<std::shared_ptr<Link>>& up,
      const std::vector<std::string>& transitNodes,
      const std::vector<std::pair<std::shared_ptr<Link>, std::string>>& metricPatches) const;
  Engine& engine() const;
  struct TraceMemo; // per getKthPaths call (LinkState.cpp)
  bool traceOnePath(
      uint32_t src, uint32_t dest, const SpfView& result, TraceMemo& memo,
      std::vector<uint32_t>& links) const;
  void addLink(std::shared_ptr<Link> link);
  void removeLink(std::shared_ptr<Link> link);
  void removeNode(const std::string& nodeName);
  bool updateNodeOverloaded(
      const std::string& nodeName,
      bool isOverloaded,
      LinkStateMetric holdUpTtl,
      LinkStateMetric holdDownTtl);
  std::shared_ptr<Link> maybeMakeLink(
      const std::string& nodeName, const thrift::Adjacency& adj) const;
  std::vector<std::shared_ptr<Link>> getOrderedLinkSet(
      const thrift::AdjacencyDatabase& adjDb) const;
  std::vector<std::shared_ptr<Link>> orderedLinksFromNode(const std::string& nodeName) const;

  const std::string area_;
  std::unordered_map<std::string, LinkSet> linkMap_;
  LinkSet allLinks_;
  std::unordered_map<std::string, HoldableValue<bool>> nodeOverloads_;
  std::unordered_map<std::string, thrift::AdjacencyDatabase> adjacencyDatabases_;

  // reference-form memo (materialised lazily from the flat results)
  mutable std::unordered_map<std::string, SpfResult> spfResultsMetric_;
  mutable std::unordered_map<std::string, SpfResult> spfResultsHops_;
  struct KthKey {
    std::string src, dst;
    size_t k;
    bool operator==(const KthKey& o) const {
      return k == o.k && src == o.src && dst == o.dst;
    }
  };
  struct KthKeyHash {
    size_t operator()(const KthKey& key) const;
  };
  // The paths of (src, dst, k) as link ids, and their reference form
  // (materialised on the first getKthPaths of the key).  getKthPaths / spfView
  // may be called from the worker threads of one RouteDb build (Parallel.h):
  // the memo is split into stripes by key hash, each with its own lock (memo
  // hits share it, fills take it), so the threads of a build seldom meet.
  struct KthStripe {
    std::shared_mutex mu;
    std::unordered_map<KthKey, KthPathIds, KthKeyHash> ids;
    std::unordered_map<KthKey, std::vector<Path>, KthKeyHash> paths;
  };
  static constexpr size_t kKthStripes = 64;
  mutable std::unique_ptr<std::array<KthStripe, kKthStripes>> kth_ =
      std::make_unique<std::array<KthStripe, kKthStripes>>();
  KthStripe& kthStripe(const KthKey& key) const {
    return (*kth_)[KthKeyHash{}(key) % kKthStripes];
  }
  void clearKthMemo() const;
  // frees a cleared k-th path memo off the update path (clearKthMemo)
  mutable std::thread kthReaper_;
  // once-only fills of kthIds_ (the reference memo runs each
  // (src, dst, k) once, and decision.spf_runs counts it once): a fill holds
  // the stripe of its key; stripes are per k (k = 1, 2; one lock for k >= 3).
  // The lower-rank paths a k-fill needs are filled before it takes its lock,
  // so no thread ever holds two fill locks (no cycle, no re-entry)
  struct KthFillLocks {
    static constexpr size_t kStripes = 1024; // a fill holds its stripe for a whole trace
    std::mutex k1[kStripes], k2[kStripes], kN;
  };
  mutable std::unique_ptr<KthFillLocks> kthFill_ = std::make_unique<KthFillLocks>();
  mutable std::unique_ptr<Engine> engine_;
  // the engine a structural change retired: the next graph build keeps its
  // memo views whose shortest-path DAG no edge delta touches (screenMemo)
  mutable std::unique_ptr<Engine> retired_;
};

// Process-wide counters mirroring the fb303 keys the reference bumps
// (decision.spf_runs, decision.spf_ms, ...).  Tests assert exact spf_runs.
// add() is fb303::fbData->addStatValue(key, v, <export type>): the sum and
// the number of samples are kept; fb303Snapshot() renders them under the
// names fb303 exports for the key's type (Decision.cpp:105-127,
// LinkState.cpp:813/878): COUNT -> "<key>.count[.60|.600|.3600]", SUM ->
// "<key>.sum[...]", AVG -> "<key>.avg[...]".  There are no time windows here:
// the windowed names carry the all-time value.
struct Counters {
  static void add(const std::string& key, int64_t v);
  // `samples` add() calls of total value `sum` in one step (a batch of SPFs)
  static void addSamples(const std::string& key, int64_t sum, int64_t samples);
  static int64_t samples(const std::string& key);
  static int64_t get(const std::string& key);
  static std::unordered_map<std::string, int64_t> snapshot();
  static std::unordered_map<std::string, int64_t> fb303Snapshot();
  static void reset();
};

// Which HIP device new LinkStates bind to (one process per GPU).
void setSpfDevice(int device);
int getSpfDevice();
// Devices of the multi-GPU fan-out: when non-empty,
// every device batch of at least clusterMinSources() queries on a 32-bit plan
// -- prefetchSpf (all-sources views, a RouteDb's node + LFA neighbours),
// prefetchKthPaths (the KSP2 second passes, by destination), runSpfBatch
// (what-if link failures) -- is split over these devices in one call
// (spf_cluster_create_local + a persistent spf_cgraph per area + one
// spf_table_create_q per batch, ignore lists sliced per block) and every
// block's rows come back to the host from its own device.  Empty (the
// default) = everything on getSpfDevice().
void setSpfDevices(const std::vector<int>& devices);
std::vector<int> getSpfDevices();
constexpr size_t kClusterMinSources = 64;
// the fan-out threshold (default kClusterMinSources; tests lower it)
void setClusterMinSources(size_t n);
size_t clusterMinSources();

} // namespace openr

namespace std {
template <>
struct hash<openr::Link> {
  size_t operator()(openr::Link const& link) const { return link.hash; }
};
template <>
struct hash<openr::LinkState::LinkSet> {
  size_t operator()(openr::LinkState::LinkSet const& set) const;
};
template <>
struct equal_to<openr::LinkState::LinkSet> {
  bool operator()(
      openr::LinkState::LinkSet const& a, openr::LinkState::LinkSet const& b) const;
};
} // namespace std
