// SpfSolver.cpp — RouteDb generation (reference: openr/decision/Decision.cpp
// :47-1321) over the MI355X LinkState.
//
// The selection rules (announcer choice, drain filtering, ECMP across areas,
// RFC 5286 LFA, next-hop expansion to links, MPLS actions, KSP2 label
// stacks, BGP metric vectors) are restated rule for rule.  What differs is
// how shortest paths are fetched: instead of one lazily computed string-keyed
// SpfResult per source, buildRouteDb first asks each area's LinkState for all
// the SPFs it is going to read (myNode, and with LFA every up neighbour; the
// KSP2 second passes of every SR_MPLS prefix) as one device batch, then reads
// distances / next-hop masks by node id (SpfView).

#include "SpfSolver.h"

#include <atomic>
#include <cstdlib>
#include <chrono>
#include <memory>
#include <string_view>
#include <thread>
#include <list>

#include "Parallel.h"
#include "Util.h"

namespace openr {

using Metric = LinkStateMetric;
namespace mvu = MetricVectorUtils;

// ---------------------------------------------------------------- RouteDb

thrift::UnicastRoute RibUnicastEntry::toThrift() const {
  thrift::UnicastRoute r;
  r.dest = prefix;
  r.nextHops.assign(nexthops.begin(), nexthops.end());
  r.doNotInstall = doNotInstall;
  if (bestPrefixEntry.type == thrift::PrefixType::BGP) {
    r.prefixType = thrift::PrefixType::BGP;
    r.data = bestPrefixEntry.data;
    r.bestNexthop = bestNexthop.value();
  }
  return r;
}

thrift::MplsRoute RibMplsEntry::toThrift() const {
  thrift::MplsRoute r;
  r.topLabel = label;
  r.nextHops.assign(nexthops.begin(), nexthops.end());
  return r;
}

thrift::RouteDatabase DecisionRouteDb::toThrift() const {
  thrift::RouteDatabase db;
  for (const auto& [_, e] : unicastEntries) {
    db.unicastRoutes.push_back(e.toThrift());
  }
  for (const auto& [_, e] : mplsEntries) {
    db.mplsRoutes.push_back(e.toThrift());
  }
  return db;
}

static size_t routeShardOf(const thrift::IpPrefix& prefix, unsigned shards) {
  return std::hash<thrift::IpPrefix>()(prefix) % shards;
}

static size_t routeShardOf(int32_t label, unsigned shards) {
  return (uint32_t)label % shards;
}

void releaseRouteDb(DecisionRouteDb&& db) {
  // Each worker frees the routes of one shard, with the shard split the
  // build used (recorded in the RouteDb): a shard's routes were allocated by
  // one build worker, so they come from one malloc arena and the frees of
  // different workers mostly take different arena locks.  Shards are handed
  // out dynamically in both passes, so the freeing thread is not guaranteed
  // to be the allocating one; the measured gain (fabric release 67 -> 13-22
  // ms) is for this split on the bench's route mix and 16 host threads.  The
  // map nodes are unlinked here first (one pass, no frees) and destroyed,
  // payload and node together, by the shard workers.  (A background reaper
  // thread was measured worse: its frees contend with the next build's
  // allocations, 113 -> 121 ms per fabric rebuild.)
  const auto t0 = std::chrono::steady_clock::now();
  auto& u = db.unicastEntries;
  const unsigned us = db.unicastShards ? db.unicastShards : routeShards(u.size());
  std::vector<std::vector<decltype(u.extract(u.begin()))>> uNodes(us);
  while (!u.empty()) {
    auto node = u.extract(u.begin());
    uNodes[routeShardOf(node.key(), us)].push_back(std::move(node));
  }
  auto& m = db.mplsEntries;
  const unsigned ms = db.mplsShards ? db.mplsShards : routeShards(m.size());
  std::vector<std::vector<decltype(m.extract(m.begin()))>> mNodes(ms);
  while (!m.empty()) {
    auto node = m.extract(m.begin());
    mNodes[routeShardOf(node.key(), ms)].push_back(std::move(node));
  }
  parallelShards(std::max(us, ms), [&](unsigned s) {
    if (s < us) {
      uNodes[s].clear();
    }
    if (s < ms) {
      mNodes[s].clear();
    }
  });
  DecisionRouteDb gone(std::move(db));
  Counters::add("decision.route_releases", 1);
  Counters::add(
      "decision.route_release_us",
      std::chrono::duration_cast<std::chrono::microseconds>(
          std::chrono::steady_clock::now() - t0)
          .count());
}

DecisionRouteUpdate getRouteDelta(const DecisionRouteDb& newDb, const DecisionRouteDb& oldDb) {
  DecisionRouteUpdate delta;
  for (const auto& [prefix, entry] : newDb.unicastEntries) {
    auto it = oldDb.unicastEntries.find(prefix);
    if (it == oldDb.unicastEntries.end() || !(it->second == entry)) {
      delta.unicastRoutesToUpdate.push_back(entry);
    }
  }
  for (const auto& [prefix, _] : oldDb.unicastEntries) {
    if (!newDb.unicastEntries.count(prefix)) {
      delta.unicastRoutesToDelete.push_back(prefix);
    }
  }
  for (const auto& [label, entry] : newDb.mplsEntries) {
    auto it = oldDb.mplsEntries.find(label);
    if (it == oldDb.mplsEntries.end() || !(it->second == entry)) {
      delta.mplsRoutesToUpdate.push_back(entry);
    }
  }
  for (const auto& [label, _] : oldDb.mplsEntries) {
    if (!newDb.mplsEntries.count(label)) {
      delta.mplsRoutesToDelete.push_back(label);
    }
  }
  return delta;
}

// ------------------------------------------------------------ SPF reads

namespace {

using AreaLinkStates = std::unordered_map<std::string, LinkState>;

struct PairHash {
  size_t operator()(const std::pair<std::string_view, std::string_view>& p) const {
    return detail::mix(
        std::hash<std::string_view>()(p.first), std::hash<std::string_view>()(p.second));
  }
};
// (next-hop node, destination or "") -> metric beyond the next hop.  The
// views point at names owned by the LinkState engine / the Link objects /
// the caller's destination set, all alive for the whole RouteDb build.
using NextHopNodes =
    std::unordered_map<std::pair<std::string_view, std::string_view>, Metric, PairHash>;
const std::string kNoDestName;

// Name-keyed reads of one SPF row (what the reference does with
// SpfResult::find / at(...).metric() / nextHops()).
class SpfRead {
 public:
  SpfRead(const LinkState& ls, const std::string& src, bool useLinkMetric = true)
      : ls_(ls), src_(src), view_(ls.spfView(src, useLinkMetric)), names_(ls.nodeNames()) {}
  // over an already resolved (link-metric) view of src
  SpfRead(const LinkState& ls, const std::string& src, const SpfView& view)
      : ls_(ls), src_(src), view_(view), names_(ls.nodeNames()) {}

  std::optional<Metric> metric(const std::string& node) const {
    return metricById(ls_.nodeId(node), node);
  }
  // metric() with the node's id already looked up (ls.nodeId(node))
  std::optional<Metric> metricById(std::optional<uint32_t> id, const std::string& node) const {
    if (view_.src == ~0u) {
      return node == src_ ? std::optional<Metric>(0) : std::nullopt;
    }
    if (!id || !view_.reached(*id)) {
      return std::nullopt;
    }
    return view_.dist[*id];
  }

  template <class Fn>
  void forEachNextHop(const std::string& node, Fn&& fn) const {
    if (view_.src == ~0u) {
      return;
    }
    auto id = ls_.nodeId(node);
    if (!id || !view_.reached(*id)) {
      return;
    }
    view_.forEachNextHop(*id, [&](uint32_t h) { fn(names_[h]); });
  }

  // fn(name, metric to that next hop) — metric = getMetricFromAToB(src, nh)
  const SpfView& view() const { return view_; }

  template <class Fn>
  void forEachNextHopWithMetric(const std::string& node, Fn&& fn) const {
    if (view_.src == ~0u) {
      return;
    }
    auto id = ls_.nodeId(node);
    if (!id || !view_.reached(*id)) {
      return;
    }
    view_.forEachNextHop(*id, [&](uint32_t h) { fn(names_[h], view_.dist[h]); });
  }

 private:
  const LinkState& ls_;
  const std::string& src_;
  const SpfView& view_;
  const std::vector<std::string>& names_;
};

// Per-thread phase clocks of selectEcmpOpenr (summed over workers, flushed
// into counters once per route shard).
struct EcmpClock {
  // ECMP: best nodes, next-hop nodes, thrift, insert; KSP2: best nodes,
  // paths (k = 1, 2), next hops + label stacks, rest
  int64_t ns[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  void flush() {
    static const char* kKeys[8] = {
        "decision.ecmp_best_us", "decision.ecmp_nhnodes_us", "decision.ecmp_thrift_us",
        "decision.ecmp_insert_us", "decision.ksp2_best_us", "decision.ksp2_paths_us",
        "decision.ksp2_nexthops_us", "decision.ksp2_rest_us"};
    for (int i = 0; i < 8; ++i) {
      if (ns[i]) {
        Counters::add(kKeys[i], ns[i] / 1000);
        ns[i] = 0;
      }
    }
  }
};
thread_local EcmpClock tEcmpClock;
// A/B switch: `name`=0 in the environment turns a fast path off
bool getenv_flag_off(const char* name) {
  const char* v = std::getenv(name);
  return v && std::atoi(v) == 0;
}
inline int64_t nowNs() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

} // namespace

// ------------------------------------------------------------------- impl

class SpfSolver::SpfSolverImpl {
 public:
  // buildRouteDbPartial: unicast prefixes to leave out, and whether to skip MPLS
  const std::unordered_set<thrift::IpPrefix>* skipPrefixes_{nullptr};
  bool skipMpls_{false};
  SpfSolverImpl(
      const std::string& myNodeName,
      bool enableV4,
      bool computeLfaPaths,
      bool enableOrderedFib,
      bool bgpDryRun,
      bool bgpUseIgpMetric)
      : myNodeName_(myNodeName),
        enableV4_(enableV4),
        computeLfaPaths_(computeLfaPaths),
        enableOrderedFib_(enableOrderedFib),
        bgpDryRun_(bgpDryRun),
        bgpUseIgpMetric_(bgpUseIgpMetric) {}

  bool staticRoutesUpdated() const { return !staticRoutesUpdates_.empty(); }
  void pushRoutesDeltaUpdates(thrift::RouteDatabaseDelta& d) {
    staticRoutesUpdates_.push_back(std::move(d));
  }
  std::optional<DecisionRouteUpdate> processStaticRouteUpdates();
  thrift::StaticRoutes const& getStaticRoutes() const { return staticRoutes_; }

  std::optional<DecisionRouteDb> buildRouteDb(
      const std::string& myNodeName,
      AreaLinkStates const& areaLinkStates,
      PrefixState const& prefixState);

 private:
  void prefetch(
      const std::string& myNodeName,
      AreaLinkStates const& areaLinkStates,
      PrefixState const& prefixState) const;

  BestPathCalResult getBestAnnouncingNodes(
      const std::string& myNodeName,
      const thrift::IpPrefix& prefix,
      const thrift::PrefixEntries& prefixEntries,
      bool hasBgp,
      bool useKsp2EdAlgo,
      AreaLinkStates const& areaLinkStates);

  BestPathCalResult runBestPathSelectionBgp(
      const std::string& myNodeName,
      const thrift::IpPrefix& prefix,
      const thrift::PrefixEntries& prefixEntries,
      AreaLinkStates const& areaLinkStates);

  BestPathCalResult maybeFilterDrainedNodes(
      BestPathCalResult&& result, AreaLinkStates const& areaLinkStates) const;

  std::optional<int64_t> getMinNextHopThreshold(
      const BestPathCalResult& nodes, const thrift::PrefixEntries& prefixEntries) const;

  void selectEcmpOpenr(
      std::unordered_map<thrift::IpPrefix, RibUnicastEntry>& unicastEntries,
      const std::string& myNodeName,
      const thrift::IpPrefix& prefix,
      const thrift::PrefixEntries& prefixEntries,
      bool isV4,
      AreaLinkStates const& areaLinkStates);

  void selectEcmpBgp(
      std::unordered_map<thrift::IpPrefix, RibUnicastEntry>& unicastEntries,
      const std::string& myNodeName,
      const thrift::IpPrefix& prefix,
      const thrift::PrefixEntries& prefixEntries,
      bool isV4,
      AreaLinkStates const& areaLinkStates,
      PrefixState const& prefixState);

  void selectKsp2(
      std::unordered_map<thrift::IpPrefix, RibUnicastEntry>& unicastEntries,
      const thrift::IpPrefix& prefix,
      const std::string& myNodeName,
      const BestPathCalResult& best,
      const thrift::PrefixEntries& prefixEntries,
      bool hasBgp,
      AreaLinkStates const& areaLinkStates,
      PrefixState const& prefixState,
      thrift::PrefixForwardingAlgorithm algo);

  std::pair<Metric, NextHopNodes> getNextHopsWithMetric(
      const std::string& myNodeName,
      const std::set<std::string>& dstNodeNames,
      bool perDestination,
      AreaLinkStates const& areaLinkStates);

  std::unordered_set<thrift::NextHopThrift> getNextHopsThrift(
      const std::string& myNodeName,
      const std::set<std::string>& dstNodeNames,
      bool isV4,
      bool perDestination,
      Metric minMetric,
      const NextHopNodes& nextHopNodes,
      std::optional<int32_t> swapLabel,
      AreaLinkStates const& areaLinkStates,
      const std::set<std::string>& prefixAreas) const;

  // myNode's links of one area in linksFromNode() order with the per-link
  // values every prefix reads (computed once per RouteDb build)
  struct MyLink {
    const Link* link;
    const std::string* nbr;
    std::string_view nbrView;
    bool up;
    Metric metric;
    const thrift::BinaryAddress* nhV4;
    const thrift::BinaryAddress* nhV6;
    const std::string* iface;
  };
  // a loop-free-alternate candidate: an up link's neighbour, its SPF view
  // and its distance back to myNode (getNextHopsWithMetric's LFA loop)
  struct LfaNbr {
    const std::string* nbr;
    SpfRead read;
    std::optional<Metric> toHere;
  };
  struct MyLinks {
    std::string node;
    std::vector<MyLink> links;
    std::unordered_map<std::string_view, std::vector<uint32_t>> byNbr;
    // computeLfaPaths_: every up link of myNode in linksFromNode() order
    std::vector<LfaNbr> lfa;
    // node's own link-metric SPF view, resolved on first read (spfView's
    // memo lock is then off the per-prefix path of the worker pool)
    mutable std::atomic<const SpfView*> view{nullptr};
  };
  const MyLinks& myLinks(
      const std::string& myNodeName, const std::string& area, const LinkState& ls) const {
    auto it = myLinks_.find(area);
    if (it != myLinks_.end()) {
      return it->second;
    }
    MyLinks& v = myLinks_[area];
    v.node = myNodeName;
    for (const auto& link : ls.linksFromNode(myNodeName)) {
      const std::string& nbr = link->getOtherNodeName(myNodeName);
      v.byNbr[std::string_view(nbr)].push_back((uint32_t)v.links.size());
      v.links.push_back(MyLink{
          link.get(), &nbr, std::string_view(nbr), link->isUp(),
          link->getMetricFromNode(myNodeName), &link->getNhV4FromNode(myNodeName),
          &link->getNhV6FromNode(myNodeName), &link->getIfaceFromNode(myNodeName)});
      if (computeLfaPaths_ && link->isUp()) {
        // the neighbour's view resolved once per build (prefetched), not per
        // prefix and per neighbour under spfView's memo lock
        SpfRead r(ls, nbr);
        const auto toHere = r.metric(myNodeName);
        v.lfa.push_back(LfaNbr{&nbr, std::move(r), toHere});
      }
    }
    return v;
  }
  // the per-build cache of `area` if it was filled for myNodeName
  const MyLinks* cachedLinks(const std::string& myNodeName, const std::string& area) const {
    auto it = myLinks_.find(area);
    return it != myLinks_.end() && it->second.node == myNodeName ? &it->second : nullptr;
  }
  mutable std::unordered_map<std::string, MyLinks> myLinks_;
  // SpfRead of myNodeName's own SPF in `area` (the per-build cached view)
  SpfRead myRead(const std::string& myNodeName, const std::string& area, const LinkState& ls) const {
    auto it = myLinks_.find(area);
    if (it == myLinks_.end() || it->second.node != myNodeName) {
      return SpfRead(ls, myNodeName);
    }
    const SpfView* v = it->second.view.load(std::memory_order_acquire);
    if (!v) {
      v = &ls.spfView(myNodeName, true);
      it->second.view.store(v, std::memory_order_release);
    }
    return SpfRead(ls, myNodeName, *v);
  }

  // SP_ECMP fast path (one area): myNode's links per next-hop mask bit of
  // its own SPF row, with next-hop templates (metric set per prefix), built
  // once per RouteDb build before the worker pool.  LFA off: only the
  // shortest-path links of each bit (metric(link) == d(nbr)).  LFA on: every
  // up link of each bit, plus the neighbours' own SPF views for the RFC 5286
  // test (getNextHopsWithMetric Decision.cpp:1146-1175)
  struct FastEcmp {
    bool ok{false};
    bool lfa{false};
    const LinkState* ls{nullptr};
    const std::string* area{nullptr};
    const SpfView* view{nullptr};
    std::vector<std::vector<uint32_t>> bitLinks; // mask bit -> template index
    std::vector<thrift::NextHopThrift> tmpl4, tmpl6;
    std::vector<uint32_t> tmplNbr; // node id of each template's neighbour
    std::vector<Metric> tmplMetric; // the template link's metric from myNode
    // LFA: one entry per distinct up neighbour (linksFromNode order of its
    // first link): its mask bit, its SPF view, its distance back to myNode
    struct LfaBit {
      uint32_t bit;
      const SpfView* view;
      Metric toHere;
    };
    std::vector<LfaBit> lfaBits;
  };
  // LFA fast path: the metric beyond each next-hop neighbour (bit) for the
  // announcers `ids` at distance `shortest`, kNoValue where the neighbour is
  // neither a shortest-path next hop (its bit in `mask`) nor a loop-free
  // alternate; false if no neighbour has a value
  static constexpr Metric kNoValue = std::numeric_limits<Metric>::max();
  bool fastLfaValues(const uint32_t* ids, size_t nIds, Metric shortest, const uint64_t* mask,
                     std::vector<Metric>& val) const;
  FastEcmp fast_;
  // per build, one area: node labels by device node id (selectKsp2)
  struct Ksp2Fast {
    bool ok{false};
    const LinkState* ls{nullptr};
    const std::string* area{nullptr};
    uint32_t me{0};
    std::vector<int32_t> labels;
  };
  Ksp2Fast ksp2Fast_;
  void buildFastEcmp(const std::string& myNodeName, AreaLinkStates const& areaLinkStates);
  // node label `label` held by `owner` (a single holder, not myNode):
  // getNextHopsWithMetric + getNextHopsThrift with the swap label, from the
  // fast path's bit templates (false: take the general path)
  bool fastLabelRoute(int32_t label, const std::string& owner, const std::string& area,
                      std::unordered_map<int32_t, RibMplsEntry>& out);
  bool fastEcmpOpenr(
      std::unordered_map<thrift::IpPrefix, RibUnicastEntry>& unicastEntries,
      const std::string& myNodeName,
      const thrift::IpPrefix& prefix,
      const thrift::PrefixEntries& prefixEntries,
      bool isV4);

  thrift::StaticRoutes staticRoutes_;
  std::vector<thrift::RouteDatabaseDelta> staticRoutesUpdates_;
  const std::string myNodeName_;
  const bool enableV4_;
  const bool computeLfaPaths_;
  const bool enableOrderedFib_;
  const bool bgpDryRun_;
  const bool bgpUseIgpMetric_;
};

std::optional<DecisionRouteUpdate> SpfSolver::SpfSolverImpl::processStaticRouteUpdates() {
  std::unordered_map<int32_t, thrift::MplsRoute> toUpdate;
  std::unordered_set<int32_t> toDelete;
  for (const auto& delta : staticRoutesUpdates_) {
    for (const auto& r : delta.mplsRoutesToUpdate) {
      toUpdate[r.topLabel] = r;
      toDelete.erase(r.topLabel);
    }
    for (const auto label : delta.mplsRoutesToDelete) {
      toDelete.insert(label);
      toUpdate.erase(label);
    }
  }
  staticRoutesUpdates_.clear();
  if (toUpdate.empty() && toDelete.empty()) {
    return std::nullopt;
  }
  DecisionRouteUpdate ret;
  for (const auto& [label, route] : toUpdate) {
    staticRoutes_.mplsRoutes[label] = route.nextHops;
    ret.mplsRoutesToUpdate.push_back(RibMplsEntry::fromThrift(route));
  }
  for (const auto label : toDelete) {
    staticRoutes_.mplsRoutes.erase(label);
    ret.mplsRoutesToDelete.push_back(label);
  }
  return ret;
}

// Ask every area for the SPF rows this build will read, one batch per area.
void SpfSolver::SpfSolverImpl::prefetch(
    const std::string& myNodeName,
    AreaLinkStates const& areaLinkStates,
    PrefixState const& prefixState) const {
  std::vector<std::string> ksp2Dests;
  bool anyPrefix = false;
  for (const auto& [prefix, entries] : prefixState.prefixes()) {
    anyPrefix = true;
    if (getPrefixForwardingType(entries) == thrift::PrefixForwardingType::SR_MPLS &&
        getPrefixForwardingAlgorithm(entries) ==
            thrift::PrefixForwardingAlgorithm::KSP2_ED_ECMP) {
      for (const auto& [node, _] : entries) {
        if (node != myNodeName) {
          ksp2Dests.push_back(node);
        }
      }
    }
  }
  std::sort(ksp2Dests.begin(), ksp2Dests.end());
  ksp2Dests.erase(std::unique(ksp2Dests.begin(), ksp2Dests.end()), ksp2Dests.end());
  for (const auto& [area, ls] : areaLinkStates) {
    std::vector<std::string> sources{myNodeName};
    if (computeLfaPaths_ && anyPrefix) {
      for (const auto& link : ls.linksFromNode(myNodeName)) {
        if (link->isUp()) {
          sources.push_back(link->getOtherNodeName(myNodeName));
        }
      }
    }
    ls.prefetchSpf(sources, true);
    if (!ksp2Dests.empty()) {
      ls.prefetchKthPaths(myNodeName, ksp2Dests);
    }
  }
}

std::optional<DecisionRouteDb> SpfSolver::SpfSolverImpl::buildRouteDb(
    const std::string& myNodeName,
    AreaLinkStates const& areaLinkStates,
    PrefixState const& prefixState) {
  bool known = false;
  for (const auto& [_, ls] : areaLinkStates) {
    known |= ls.hasNode(myNodeName);
  }
  if (!known) {
    return std::nullopt;
  }
  const auto t0 = std::chrono::steady_clock::now();
  Counters::add("decision.route_build_runs", 1);
  myLinks_.clear();
  prefetch(myNodeName, areaLinkStates, prefixState);
  Counters::add(
      "decision.route_prefetch_us",
      std::chrono::duration_cast<std::chrono::microseconds>(
          std::chrono::steady_clock::now() - t0)
          .count());

  DecisionRouteDb routeDb;

  // unicast routes: IP and IP->MPLS
  struct PrefixWork {
    const thrift::IpPrefix* prefix;
    const thrift::PrefixEntries* entries;
    bool srMpls;
    bool hasBGP;
    bool isV4;
    thrift::PrefixForwardingAlgorithm algo;
  };
  std::vector<PrefixWork> work;
  for (const auto& [prefix, prefixEntries] : prefixState.prefixes()) {
    if (skipPrefixes_ && skipPrefixes_->count(prefix)) {
      continue; // served by the caller (AllAreasRouteTable's device table)
    }
    bool hasBGP = false, hasNonBGP = false, missingMv = false;
    for (const auto& [node, byArea] : prefixEntries) {
      for (const auto& [area, entry] : byArea) {
        const bool isBGP = entry.type == thrift::PrefixType::BGP;
        hasBGP |= isBGP;
        hasNonBGP |= !isBGP;
        missingMv |= isBGP && !entry.mv.has_value();
      }
    }
    if (hasBGP && (hasNonBGP || missingMv)) {
      Counters::add("decision.skipped_unicast_route", 1);
      continue;
    }
    if (prefixEntries.count(myNodeName) && !hasBGP) {
      continue; // we advertise it ourselves
    }
    const bool isV4Prefix = prefix.prefixAddress.addr.size() == 4;
    if (isV4Prefix && !enableV4_) {
      Counters::add("decision.skipped_unicast_route", 1);
      continue;
    }
    const auto algo = getPrefixForwardingAlgorithm(prefixEntries);
    const auto type = getPrefixForwardingType(prefixEntries);
    if (type == thrift::PrefixForwardingType::SR_MPLS) {
      work.push_back({&prefix, &prefixEntries, true, hasBGP, isV4Prefix, algo});
    } else if (algo == thrift::PrefixForwardingAlgorithm::SP_ECMP) {
      if (hasBGP) {
        selectEcmpBgp(
            routeDb.unicastEntries, myNodeName, prefix, prefixEntries, isV4Prefix,
            areaLinkStates, prefixState);
      } else {
        work.push_back({&prefix, &prefixEntries, false, hasBGP, isV4Prefix, algo});
      }
    } else {
      // KSP2 is not supported for plain IP routing
      Counters::add("decision.incompatible_forwarding_type", 1);
    }
  }
  // Open/R ECMP and SR-MPLS KSP2 prefixes only read the prefetched SPF rows
  // and the (thread-safe) path memo: one worker pool, per-worker route maps
  // merged afterwards (prefixes are distinct keys)
  // Prefixes go to route shards (one per worker, Parallel.h) so that
  // releaseRouteDb frees each shard on one thread too
  const unsigned shards = routeShards(work.size());
  routeDb.unicastShards = shards;
  std::vector<std::vector<uint32_t>> shardWork(shards);
  for (size_t i = 0; i < work.size(); ++i) {
    shardWork[routeShardOf(*work[i].prefix, shards)].push_back((uint32_t)i);
  }
  for (const auto& [area, ls] : areaLinkStates) {
    myLinks(myNodeName, area, ls); // fill the per-build cache before the workers read it
  }
  buildFastEcmp(myNodeName, areaLinkStates);
  std::vector<std::unordered_map<thrift::IpPrefix, RibUnicastEntry>> parts(shards);
  const auto tpar = std::chrono::steady_clock::now();
  parallelShards(shards, [&](unsigned s) {
    for (const uint32_t i : shardWork[s]) {
      const PrefixWork& x = work[i];
      if (x.srMpls) {
        const int64_t tb = nowNs();
        const auto nodes = getBestAnnouncingNodes(
            myNodeName, *x.prefix, *x.entries, x.hasBGP, true, areaLinkStates);
        tEcmpClock.ns[4] += nowNs() - tb;
        if (!nodes.success || nodes.nodes.empty()) {
          continue;
        }
        selectKsp2(
            parts[s], *x.prefix, myNodeName, nodes, *x.entries, x.hasBGP, areaLinkStates,
            prefixState, x.algo);
      } else if (!fastEcmpOpenr(parts[s], myNodeName, *x.prefix, *x.entries, x.isV4)) {
        selectEcmpOpenr(parts[s], myNodeName, *x.prefix, *x.entries, x.isV4, areaLinkStates);
      }
    }
    tEcmpClock.flush();
  });
  const auto tmerge = std::chrono::steady_clock::now();
  Counters::add("decision.route_prefix_pool_us",
                std::chrono::duration_cast<std::chrono::microseconds>(tmerge - tpar).count());
  // move the workers' map nodes themselves (no re-allocation): one thread
  // merges them into the RouteDb's map while the label phase below runs on
  // the pool (the two touch disjoint maps and only read the SPF views)
  size_t built = routeDb.unicastEntries.size();
  for (const auto& part : parts) {
    built += part.size();
  }
  routeDb.unicastEntries.reserve(built);
  auto mergeUnicast = [&routeDb, &parts, tmerge] {
    for (auto& part : parts) {
      while (!part.empty()) {
        routeDb.unicastEntries.insert(part.extract(part.begin()));
      }
    }
    Counters::add("decision.route_merge_us",
                  std::chrono::duration_cast<std::chrono::microseconds>(
                      std::chrono::steady_clock::now() - tmerge)
                      .count());
  };
  struct Merger {
    std::thread t;
    ~Merger() {
      if (t.joinable()) {
        t.join(); // every exit path (a throwing label route included)
      }
    }
  } merger;
  // a thread per build costs more than merging a small RouteDb (the 10x10
  // grid: ~100 routes, DecisionBenchmark.cpp:360-431): overlap only big ones.
  // OPENR_ROUTE_MERGE_INLINE=1 always merges inline (read once).
  static const bool mergeInlineEnv = std::getenv("OPENR_ROUTE_MERGE_INLINE") != nullptr;
  constexpr size_t kMergeThreadMinRoutes = 2048;
  if (skipMpls_ || mergeInlineEnv || built - routeDb.unicastEntries.size() < kMergeThreadMinRoutes) {
    mergeUnicast();
  } else {
    merger.t = std::thread(mergeUnicast);
  }

  // node-label MPLS routes: on a label collision the smaller node name wins.
  // Labels held by a single (other) node cannot collide: they are expanded
  // on the worker pool straight into per-shard route maps (spliced into the
  // RouteDb like the unicast routes).  The sequential pass applies the
  // collision rule to the rest, computing in place as the reference does.
  const auto tlabel = std::chrono::steady_clock::now();
  if (skipMpls_) {
    return routeDb; // unicast only (AllAreasRouteTable brings the MPLS routes)
  }
  struct LabelItem {
    int32_t label;
    const std::string* area;
    const thrift::AdjacencyDatabase* db;
  };
  std::vector<LabelItem> labelItems; // valid labels, adjacency-database order
  for (const auto& [area, ls] : areaLinkStates) {
    for (const auto& [_, adjDb] : ls.getAdjacencyDatabases()) {
      if (adjDb.nodeLabel == 0) {
        continue; // not SR
      }
      if (!isMplsLabelValid(adjDb.nodeLabel)) {
        Counters::add("decision.skipped_mpls_route", 1);
        continue;
      }
      labelItems.push_back({adjDb.nodeLabel, &area, &adjDb});
    }
  }
  std::unordered_map<int32_t, uint32_t> labelUse;
  labelUse.reserve(labelItems.size());
  for (const auto& it : labelItems) {
    ++labelUse[it.label];
  }
  std::vector<uint8_t> single(labelItems.size(), 0);
  std::vector<uint32_t> labelJobs;
  for (size_t i = 0; i < labelItems.size(); ++i) {
    if (labelUse[labelItems[i].label] == 1 && labelItems[i].db->thisNodeName != myNodeName) {
      single[i] = 1;
      labelJobs.push_back((uint32_t)i);
    }
  }
  const unsigned labelShards = routeShards(labelJobs.size());
  routeDb.mplsShards = labelShards;
  std::vector<std::vector<uint32_t>> labelShardJobs(labelShards);
  for (const uint32_t i : labelJobs) {
    labelShardJobs[routeShardOf(labelItems[i].label, labelShards)].push_back(i);
  }
  std::vector<std::unordered_map<int32_t, RibMplsEntry>> labelParts(labelShards);
  const auto tLabelPool = std::chrono::steady_clock::now();
  parallelShards(labelShards, [&](unsigned s) {
    for (const uint32_t i : labelShardJobs[s]) {
      const auto& db = *labelItems[i].db;
      if (fastLabelRoute(db.nodeLabel, db.thisNodeName, *labelItems[i].area, labelParts[s])) {
        continue;
      }
      const auto metricNhs =
          getNextHopsWithMetric(myNodeName, {db.thisNodeName}, false, areaLinkStates);
      if (metricNhs.second.empty()) {
        Counters::add("decision.no_route_to_label", 1);
        continue;
      }
      labelParts[s].emplace(
          db.nodeLabel,
          RibMplsEntry(
              db.nodeLabel,
              getNextHopsThrift(
                  myNodeName, {db.thisNodeName}, false, false, metricNhs.first,
                  metricNhs.second, db.nodeLabel, areaLinkStates, {*labelItems[i].area})));
    }
  });
  Counters::add("decision.route_label_pool_us",
                std::chrono::duration_cast<std::chrono::microseconds>(
                    std::chrono::steady_clock::now() - tLabelPool)
                    .count());
  auto& mplsEntries = routeDb.mplsEntries;
  mplsEntries.reserve(labelItems.size() + 64);
  for (auto& part : labelParts) {
    while (!part.empty()) {
      mplsEntries.insert(part.extract(part.begin()));
    }
  }
  // label -> node holding it so far (colliding labels and our own)
  std::unordered_map<int32_t, const std::string*> labelOwner;
  auto claimLabel = [&](int32_t label, const std::string& node, RibMplsEntry&& entry) {
    labelOwner[label] = &node;
    mplsEntries.insert_or_assign(label, std::move(entry));
  };
  for (size_t i = 0; i < labelItems.size(); ++i) {
    if (single[i]) {
      continue;
    }
    const int32_t topLabel = labelItems[i].label;
    const auto& adjDb = *labelItems[i].db;
    const std::string& area = *labelItems[i].area;
    auto it = labelOwner.find(topLabel);
    if (it != labelOwner.end()) {
      Counters::add("decision.duplicate_node_label", 1);
      if (*it->second < adjDb.thisNodeName) {
        continue;
      }
    }
    if (adjDb.thisNodeName == myNodeName) {
      thrift::NextHopThrift nh;
      nh.address.addr = std::string(16, '\0'); // "::"
      nh.area = area;
      nh.mplsAction = createMplsAction(thrift::MplsActionCode::POP_AND_LOOKUP);
      claimLabel(topLabel, adjDb.thisNodeName, RibMplsEntry(topLabel, {nh}));
      continue;
    }
    const auto metricNhs =
        getNextHopsWithMetric(myNodeName, {adjDb.thisNodeName}, false, areaLinkStates);
    if (metricNhs.second.empty()) {
      Counters::add("decision.no_route_to_label", 1);
      continue;
    }
    claimLabel(
        topLabel, adjDb.thisNodeName,
        RibMplsEntry(
            topLabel,
            getNextHopsThrift(
                myNodeName, {adjDb.thisNodeName}, false, false, metricNhs.first,
                metricNhs.second, topLabel, areaLinkStates, {area})));
  }

  // adjacency-label PHP routes of our own links
  for (const auto& [_, ls] : areaLinkStates) {
    for (const auto& link : ls.linksFromNode(myNodeName)) {
      const int32_t topLabel = link->getAdjLabelFromNode(myNodeName);
      if (topLabel == 0) {
        continue;
      }
      if (!isMplsLabelValid(topLabel)) {
        Counters::add("decision.skipped_mpls_route", 1);
        continue;
      }
      routeDb.mplsEntries.emplace(
          topLabel,
          RibMplsEntry(
              topLabel,
              {createNextHop(
                  link->getNhV6FromNode(myNodeName), link->getIfaceFromNode(myNodeName),
                  (int32_t)link->getMetricFromNode(myNodeName),
                  createMplsAction(thrift::MplsActionCode::PHP), false, link->getArea())}));
    }
  }

  Counters::add("decision.route_label_us",
                std::chrono::duration_cast<std::chrono::microseconds>(
                    std::chrono::steady_clock::now() - tlabel)
                    .count());
  if (merger.t.joinable()) {
    merger.t.join();
  }
  const auto elapsed = std::chrono::steady_clock::now() - t0;
  Counters::add(
      "decision.route_build_us",
      std::chrono::duration_cast<std::chrono::microseconds>(elapsed).count());
  // Decision.cpp:536-540 (AVG of whole milliseconds)
  Counters::add(
      "decision.route_build_ms",
      std::chrono::duration_cast<std::chrono::milliseconds>(elapsed).count());
  return routeDb;
}

BestPathCalResult SpfSolver::SpfSolverImpl::getBestAnnouncingNodes(
    const std::string& myNodeName,
    const thrift::IpPrefix& prefix,
    const thrift::PrefixEntries& prefixEntries,
    bool hasBgp,
    bool useKsp2EdAlgo,
    AreaLinkStates const& areaLinkStates) {
  BestPathCalResult ret;
  if (!hasBgp) {
    // every reachable announcer is a best node; the smallest name is "best"
    if (prefixEntries.count(myNodeName)) {
      return BestPathCalResult{};
    }
    for (const auto& [node, byArea] : prefixEntries) {
      for (const auto& [area, entry] : byArea) {
        const SpfRead mine = myRead(myNodeName, area, areaLinkStates.at(area));
        if (!mine.metric(node)) {
          continue; // unreachable announcer
        }
        if (ret.bestNode.empty() || node < ret.bestNode) {
          ret.bestNode = node;
          ret.bestArea = area;
        }
        ret.nodes.insert(node);
        ret.areas.insert(area);
      }
    }
    ret.success = true;
    return maybeFilterDrainedNodes(std::move(ret), areaLinkStates);
  }

  ret = runBestPathSelectionBgp(myNodeName, prefix, prefixEntries, areaLinkStates);
  if (!ret.success) {
    Counters::add("decision.no_route_to_prefix", 1);
    return BestPathCalResult{};
  }
  if (!useKsp2EdAlgo) {
    if (ret.nodes.count(myNodeName)) {
      return BestPathCalResult{}; // best path originated by ourselves
    }
    return maybeFilterDrainedNodes(std::move(ret), areaLinkStates);
  }
  // KSP2: program our own prefix only when others announce it too and we
  // carry a prepend label
  bool myLabel = false;
  auto mine = prefixEntries.find(myNodeName);
  if (mine != prefixEntries.end()) {
    for (const auto& [_, entry] : mine->second) {
      myLabel |= entry.prependLabel.has_value();
    }
  }
  if (!ret.nodes.count(myNodeName) || (ret.nodes.size() > 1 && myLabel)) {
    return maybeFilterDrainedNodes(std::move(ret), areaLinkStates);
  }
  return BestPathCalResult{};
}

BestPathCalResult SpfSolver::SpfSolverImpl::runBestPathSelectionBgp(
    const std::string& myNodeName,
    const thrift::IpPrefix& /* prefix */,
    const thrift::PrefixEntries& prefixEntries,
    AreaLinkStates const& areaLinkStates) {
  BestPathCalResult ret;
  for (const auto& [nodeName, byArea] : prefixEntries) {
    for (const auto& [area, entry] : byArea) {
      SpfRead mine(areaLinkStates.at(area), myNodeName);
      const auto igp = mine.metric(nodeName);
      if (!igp) {
        continue;
      }
      const thrift::MetricVector& mvIn = entry.mv.value();
      if (mvu::getMetricEntityByType(mvIn, mvu::kOpenrIgpCostType)) {
        continue; // OPENR_IGP_COST must not be advertised
      }
      thrift::MetricVector metricVector = mvIn;
      if (bgpUseIgpMetric_) {
        const int64_t igpMetric = (int64_t)*igp;
        if (!ret.bestIgpMetric || *ret.bestIgpMetric > igpMetric) {
          ret.bestIgpMetric = igpMetric;
        }
        metricVector.metrics.push_back(mvu::createMetricEntity(
            mvu::kOpenrIgpCostType, mvu::kOpenrIgpCostPriority,
            thrift::CompareType::WIN_IF_NOT_PRESENT, false, {-1 * igpMetric}));
      }
      mvu::CompareResult cmp = mvu::CompareResult::WINNER;
      if (ret.bestVector) {
        cmp = mvu::compareMetricVectors(metricVector, *ret.bestVector);
      }
      switch (cmp) {
      case mvu::CompareResult::WINNER:
        ret.nodes.clear();
        [[fallthrough]];
      case mvu::CompareResult::TIE_WINNER:
        ret.bestVector = std::move(metricVector);
        ret.bestNode = nodeName;
        ret.bestArea = area;
        [[fallthrough]];
      case mvu::CompareResult::TIE_LOOSER:
        ret.nodes.insert(nodeName);
        ret.areas.insert(area);
        break;
      case mvu::CompareResult::TIE:
      case mvu::CompareResult::ERROR:
        return ret; // cannot order: no route (success stays false)
      default:
        break;
      }
    }
  }
  ret.success = true;
  return maybeFilterDrainedNodes(std::move(ret), areaLinkStates);
}

BestPathCalResult SpfSolver::SpfSolverImpl::maybeFilterDrainedNodes(
    BestPathCalResult&& result, AreaLinkStates const& areaLinkStates) const {
  BestPathCalResult filtered = result;
  for (const auto& [_, ls] : areaLinkStates) {
    for (auto it = filtered.nodes.begin(); it != filtered.nodes.end();) {
      it = ls.isNodeOverloaded(*it) ? filtered.nodes.erase(it) : std::next(it);
    }
  }
  // drained announcers are used only when every announcer is drained
  return filtered.nodes.empty() ? result : filtered;
}

std::optional<int64_t> SpfSolver::SpfSolverImpl::getMinNextHopThreshold(
    const BestPathCalResult& nodes, const thrift::PrefixEntries& prefixEntries) const {
  std::optional<int64_t> threshold;
  for (const auto& node : nodes.nodes) {
    auto it = prefixEntries.find(node);
    if (it == prefixEntries.end()) {
      continue;
    }
    for (const auto& [_, entry] : it->second) {
      if (entry.minNexthop && (!threshold || *entry.minNexthop > *threshold)) {
        threshold = entry.minNexthop;
      }
    }
  }
  return threshold;
}

// The SP_ECMP route of a prefix in the common case -- one area, LFA off, IP
// forwarding -- read straight from myNode's flat SPF row with the reference's
// exact rules (getBestAnnouncingNodes :544-630 with maybeFilterDrainedNodes
// :651-666, getNextHopsWithMetric :1093-1179, getNextHopsThrift :1181-1271):
// announcers resolved by node id, the next-hop neighbours read as mask bits,
// and a neighbour's links taken iff metric(link) + (min - d(nbr)) == min,
// i.e. metric(link) == d(nbr) -- a per-build property of the bit, so each
// bit's next hops are templates whose metric is set to the prefix's min.
// No std::set<std::string> of announcers, no name-keyed next-hop map.
void SpfSolver::SpfSolverImpl::buildFastEcmp(
    const std::string& myNodeName, AreaLinkStates const& areaLinkStates) {
  fast_ = FastEcmp{};
  ksp2Fast_ = Ksp2Fast{};
  if (areaLinkStates.size() == 1 && !getenv_flag_off("OPENR_KSP2_FAST")) {
    // node labels by device node id for selectKsp2's label stacks
    const auto& [area, ls] = *areaLinkStates.begin();
    if (const auto me = ls.nodeId(myNodeName)) {
      const auto& names = ls.nodeNames();
      const auto& adj = ls.getAdjacencyDatabases();
      ksp2Fast_.labels.assign(names.size(), 0);
      bool ok = true;
      for (uint32_t i = 0; i < names.size() && ok; ++i) {
        auto it = adj.find(names[i]);
        ok = it != adj.end();
        ksp2Fast_.labels[i] = ok ? it->second.nodeLabel : 0;
      }
      ksp2Fast_.ok = ok;
      ksp2Fast_.ls = &ls;
      ksp2Fast_.area = &area;
      ksp2Fast_.me = *me;
    }
  }
  if (areaLinkStates.size() != 1 || getenv_flag_off("OPENR_ECMP_FAST")) {
    return;
  }
  const auto& [area, ls] = *areaLinkStates.begin();
  const MyLinks* mls = cachedLinks(myNodeName, area);
  if (!mls) {
    return;
  }
  const SpfView& view = ls.spfView(myNodeName, true);
  if (view.src == ~0u || view.exact || !view.useLinkMetric) {
    return;
  }
  fast_.ls = &ls;
  fast_.area = &area;
  fast_.view = &view;
  fast_.lfa = computeLfaPaths_;
  fast_.bitLinks.assign(view.nbrs.size(), {});
  std::unordered_map<uint32_t, uint32_t> bitOf;
  for (uint32_t j = 0; j < view.nbrs.size(); ++j) {
    bitOf[view.nbrs[j]] = j;
  }
  for (uint32_t li = 0; li < mls->links.size(); ++li) {
    const MyLink& ml = mls->links[li];
    if (!ml.up) {
      continue;
    }
    const auto id = ls.nodeId(*ml.nbr);
    if (!id) {
      if (fast_.lfa) {
        return; // an up link the device row has no bit for: general path
      }
      continue;
    }
    auto b = bitOf.find(*id);
    if (fast_.lfa) {
      if (b == bitOf.end()) {
        return;
      }
    } else if (b == bitOf.end() || !view.reached(*id) || ml.metric != view.dist[*id]) {
      continue; // never a shortest-path link (distOverLink != minMetric)
    }
    fast_.bitLinks[b->second].push_back((uint32_t)fast_.tmpl4.size());
    fast_.tmplNbr.push_back(*id);
    fast_.tmplMetric.push_back(ml.metric);
    fast_.tmpl4.push_back(createNextHop(*ml.nhV4, *ml.iface, 0, std::nullopt, false,
                                        ml.link->getArea()));
    fast_.tmpl6.push_back(createNextHop(*ml.nhV6, *ml.iface, 0, std::nullopt, false,
                                        ml.link->getArea()));
  }
  if (fast_.lfa) {
    // the LFA candidates: every up neighbour, once (the reference's loop over
    // links revisits a neighbour of parallel links with the same values)
    std::vector<uint8_t> seen(view.nbrs.size(), 0);
    for (const LfaNbr& ln : mls->lfa) {
      const SpfView& nv = ln.read.view();
      const auto id = ls.nodeId(*ln.nbr);
      if (!ln.toHere || nv.src == ~0u || nv.exact || !nv.useLinkMetric || !id) {
        return; // the general path (which throws where the reference does)
      }
      auto b = bitOf.find(*id);
      if (b == bitOf.end()) {
        return;
      }
      if (!seen[b->second]) {
        seen[b->second] = 1;
        fast_.lfaBits.push_back({b->second, &nv, *ln.toHere});
      }
    }
  }
  fast_.ok = true;
}

bool SpfSolver::SpfSolverImpl::fastLfaValues(
    const uint32_t* ids, size_t nIds, Metric shortest, const uint64_t* mask,
    std::vector<Metric>& val) const {
  const SpfView& view = *fast_.view;
  const uint32_t W = view.words;
  val.assign(view.nbrs.size(), kNoValue);
  bool any = false;
  // shortest-path next hops: metric beyond = shortest - d(nbr)
  for (uint32_t w = 0; w < W; ++w) {
    for (uint64_t b = mask[w]; b; b &= b - 1) {
      const uint32_t bit = w * 64 + (uint32_t)__builtin_ctzll(b);
      val[bit] = shortest - view.dist[view.nbrs[bit]];
      any = true;
    }
  }
  // loop-free alternates: d(n, dst) < shortest + d(n, me), over every
  // announcer; the smallest such d(n, dst) if below the value so far
  for (const auto& lb : fast_.lfaBits) {
    const SpfView& nv = *lb.view;
    const Metric bound = shortest + lb.toHere;
    Metric& v = val[lb.bit];
    for (size_t i = 0; i < nIds; ++i) {
      if (!nv.reached(ids[i])) {
        continue;
      }
      const Metric d = nv.dist[ids[i]];
      if (d < bound && d < v) {
        v = d;
        any = true;
      }
    }
  }
  return any;
}

bool SpfSolver::SpfSolverImpl::fastLabelRoute(
    int32_t label, const std::string& owner, const std::string& area,
    std::unordered_map<int32_t, RibMplsEntry>& out) {
  if (!fast_.ok || area != *fast_.area) {
    return false;
  }
  const SpfView& view = *fast_.view;
  const auto id = fast_.ls->nodeId(owner);
  if (!id || !view.reached(*id)) {
    // getNextHopsWithMetric finds no next hop (Decision.cpp:449-452)
    Counters::add("decision.no_route_to_label", 1);
    return true;
  }
  const uint32_t W = view.words;
  const uint64_t* row = view.nh.data() + (size_t)*id * W;
  const Metric shortest = view.dist[*id];
  if (fast_.lfa) {
    // getNextHopsWithMetric(me, {owner}) with LFAs, then every up link of a
    // next-hop neighbour at link metric + value (no shortest filter)
    thread_local std::vector<Metric> val;
    const uint32_t owner = *id;
    if (!fastLfaValues(&owner, 1, shortest, row, val)) {
      Counters::add("decision.no_route_to_label", 1);
      return true;
    }
    std::unordered_set<thrift::NextHopThrift> nextHops;
    for (uint32_t bit = 0; bit < val.size(); ++bit) {
      if (val[bit] == kNoValue) {
        continue;
      }
      for (const uint32_t k : fast_.bitLinks[bit]) {
        thrift::NextHopThrift nh = fast_.tmpl6[k];
        nh.metric = (int32_t)(fast_.tmplMetric[k] + val[bit]);
        nh.mplsAction = fast_.tmplNbr[k] == owner
            ? createMplsAction(thrift::MplsActionCode::PHP)
            : createMplsAction(thrift::MplsActionCode::SWAP, label);
        nextHops.insert(std::move(nh));
      }
    }
    out.emplace(label, RibMplsEntry(label, std::move(nextHops)));
    return true;
  }
  size_t cnt = 0;
  for (uint32_t w = 0; w < W; ++w) {
    for (uint64_t b = row[w]; b; b &= b - 1) {
      cnt += fast_.bitLinks[w * 64 + (uint32_t)__builtin_ctzll(b)].size();
    }
  }
  if (cnt == 0) {
    bool any = false;
    for (uint32_t w = 0; w < W; ++w) {
      any |= row[w] != 0;
    }
    if (!any) {
      Counters::add("decision.no_route_to_label", 1);
      return true;
    }
  }
  std::unordered_set<thrift::NextHopThrift> nextHops;
  nextHops.reserve(cnt);
  for (uint32_t w = 0; w < W; ++w) {
    for (uint64_t b = row[w]; b; b &= b - 1) {
      for (const uint32_t k : fast_.bitLinks[w * 64 + (uint32_t)__builtin_ctzll(b)]) {
        thrift::NextHopThrift nh = fast_.tmpl6[k];
        nh.metric = (int32_t)shortest;
        // PHP into the label's owner, else SWAP (getNextHopsThrift :1211-1217)
        nh.mplsAction = fast_.tmplNbr[k] == *id
            ? createMplsAction(thrift::MplsActionCode::PHP)
            : createMplsAction(thrift::MplsActionCode::SWAP, label);
        nextHops.insert(std::move(nh));
      }
    }
  }
  out.emplace(label, RibMplsEntry(label, std::move(nextHops)));
  return true;
}

bool SpfSolver::SpfSolverImpl::fastEcmpOpenr(
    std::unordered_map<thrift::IpPrefix, RibUnicastEntry>& unicastEntries,
    const std::string& myNodeName,
    const thrift::IpPrefix& prefix,
    const thrift::PrefixEntries& prefixEntries,
    bool isV4) {
  if (!fast_.ok) {
    return false;
  }
  auto& clk = tEcmpClock;
  int64_t t = nowNs();
  auto lap = [&](int i) {
    const int64_t n = nowNs();
    clk.ns[i] += n - t;
    t = n;
  };
  const LinkState& ls = *fast_.ls;
  const SpfView& view = *fast_.view;
  // reachable announcers in name order (the first is the best node)
  struct Ann {
    const std::string* node;
    const std::string* area;
    uint32_t id;
    bool drained;
  };
  Ann anns[16];
  std::vector<Ann> more;
  size_t n = 0;
  for (const auto& [node, byArea] : prefixEntries) {
    if (node == myNodeName) {
      return false; // (the caller filters these) general path
    }
    for (const auto& [area, entry] : byArea) {
      if (area != *fast_.area) {
        return false; // an area this build does not hold: general path
      }
      const auto id = ls.nodeId(node);
      if (!id || !view.reached(*id)) {
        continue;
      }
      const Ann a{&node, &area, *id, ls.isNodeOverloaded(node)};
      if (n < 16) {
        anns[n] = a;
      } else {
        more.push_back(a);
      }
      ++n;
    }
  }
  auto ann = [&](size_t i) -> const Ann& { return i < 16 ? anns[i] : more[i - 16]; };
  lap(0);
  if (n == 0) {
    Counters::add("decision.no_route_to_prefix", 1);
    return true;
  }
  // drained announcers count only when every reachable one is drained
  bool anyUndrained = false;
  for (size_t i = 0; i < n; ++i) {
    anyUndrained |= !ann(i).drained;
  }
  Metric shortest = std::numeric_limits<Metric>::max();
  for (size_t i = 0; i < n; ++i) {
    if (!anyUndrained || !ann(i).drained) {
      shortest = std::min<Metric>(shortest, view.dist[ann(i).id]);
    }
  }
  const uint32_t W = view.words;
  uint64_t m[4] = {0, 0, 0, 0};
  std::vector<uint64_t> mw(W > 4 ? W : 0, 0);
  uint64_t* mask = W > 4 ? mw.data() : m;
  for (size_t i = 0; i < n; ++i) {
    const Ann& a = ann(i);
    if ((!anyUndrained || !a.drained) && view.dist[a.id] == shortest) {
      const uint64_t* row = view.nh.data() + (size_t)a.id * W;
      for (uint32_t w = 0; w < W; ++w) {
        mask[w] |= row[w];
      }
    }
  }
  if (fast_.lfa) {
    // the announcers getNextHopsWithMetric sees (drain-filtered), their
    // loop-free alternates, then every up link of a next-hop neighbour
    thread_local std::vector<Metric> val;
    thread_local std::vector<uint32_t> ids;
    ids.clear();
    for (size_t i = 0; i < n; ++i) {
      if (!anyUndrained || !ann(i).drained) {
        ids.push_back(ann(i).id);
      }
    }
    const bool anyNh = fastLfaValues(ids.data(), ids.size(), shortest, mask, val);
    lap(1);
    if (!anyNh) {
      Counters::add("decision.no_route_to_prefix", 1);
      return true;
    }
    const auto& tmpl = isV4 ? fast_.tmpl4 : fast_.tmpl6;
    std::unordered_set<thrift::NextHopThrift> nextHops;
    size_t cnt = 0;
    for (uint32_t bit = 0; bit < val.size(); ++bit) {
      cnt += val[bit] == kNoValue ? 0 : fast_.bitLinks[bit].size();
    }
    nextHops.reserve(cnt);
    for (uint32_t bit = 0; bit < val.size(); ++bit) {
      if (val[bit] == kNoValue) {
        continue;
      }
      for (const uint32_t k : fast_.bitLinks[bit]) {
        thrift::NextHopThrift nh = tmpl[k];
        nh.metric = (int32_t)(fast_.tmplMetric[k] + val[bit]);
        nextHops.insert(std::move(nh));
      }
    }
    const Ann& best = ann(0);
    RibUnicastEntry entry(prefix, std::move(nextHops), prefixEntries.at(*best.node).at(*best.area),
                          *best.area);
    lap(2);
    unicastEntries.emplace(prefix, std::move(entry));
    lap(3);
    return true;
  }
  bool any = false;
  for (uint32_t w = 0; w < W; ++w) {
    any |= mask[w] != 0;
  }
  lap(1);
  if (!any) {
    Counters::add("decision.no_route_to_prefix", 1);
    return true;
  }
  std::unordered_set<thrift::NextHopThrift> nextHops;
  {
    size_t cnt = 0;
    for (uint32_t w = 0; w < W; ++w) {
      for (uint64_t b = mask[w]; b; b &= b - 1) {
        cnt += fast_.bitLinks[w * 64 + (uint32_t)__builtin_ctzll(b)].size();
      }
    }
    nextHops.reserve(cnt);
  }
  const auto& tmpl = isV4 ? fast_.tmpl4 : fast_.tmpl6;
  for (uint32_t w = 0; w < W; ++w) {
    for (uint64_t b = mask[w]; b; b &= b - 1) {
      const uint32_t bit = w * 64 + (uint32_t)__builtin_ctzll(b);
      for (const uint32_t k : fast_.bitLinks[bit]) {
        thrift::NextHopThrift nh = tmpl[k];
        nh.metric = (int32_t)shortest;
        nextHops.insert(std::move(nh));
      }
    }
  }
  const Ann& best = ann(0);
  RibUnicastEntry entry(prefix, std::move(nextHops), prefixEntries.at(*best.node).at(*best.area),
                        *best.area);
  lap(2);
  unicastEntries.emplace(prefix, std::move(entry));
  lap(3);
  return true;
}

void SpfSolver::SpfSolverImpl::selectEcmpOpenr(
    std::unordered_map<thrift::IpPrefix, RibUnicastEntry>& unicastEntries,
    const std::string& myNodeName,
    const thrift::IpPrefix& prefix,
    const thrift::PrefixEntries& prefixEntries,
    bool isV4,
    AreaLinkStates const& areaLinkStates) {
  auto& clk = tEcmpClock;
  int64_t t = nowNs();
  auto lap = [&](int i) {
    const int64_t n = nowNs();
    clk.ns[i] += n - t;
    t = n;
  };
  const auto ret =
      getBestAnnouncingNodes(myNodeName, prefix, prefixEntries, false, false, areaLinkStates);
  lap(0);
  if (!ret.success) {
    return;
  }
  const bool perDestination =
      getPrefixForwardingType(prefixEntries) == thrift::PrefixForwardingType::SR_MPLS;
  const auto metricNhs =
      getNextHopsWithMetric(myNodeName, ret.nodes, perDestination, areaLinkStates);
  lap(1);
  if (metricNhs.second.empty()) {
    Counters::add("decision.no_route_to_prefix", 1);
    return;
  }
  RibUnicastEntry entry(
      prefix,
      getNextHopsThrift(
          myNodeName, ret.nodes, isV4, perDestination, metricNhs.first, metricNhs.second,
          std::nullopt, areaLinkStates, ret.areas),
      prefixEntries.at(ret.bestNode).at(ret.bestArea),
      ret.bestArea);
  lap(2);
  unicastEntries.emplace(prefix, std::move(entry));
  lap(3);
}

void SpfSolver::SpfSolverImpl::selectEcmpBgp(
    std::unordered_map<thrift::IpPrefix, RibUnicastEntry>& unicastEntries,
    const std::string& myNodeName,
    const thrift::IpPrefix& prefix,
    const thrift::PrefixEntries& prefixEntries,
    bool isV4,
    AreaLinkStates const& areaLinkStates,
    PrefixState const& prefixState) {
  const auto dst =
      getBestAnnouncingNodes(myNodeName, prefix, prefixEntries, true, false, areaLinkStates);
  if (!dst.success) {
    return;
  }
  if (dst.nodes.empty() || dst.nodes.count(myNodeName)) {
    if (!dst.nodes.count(myNodeName)) {
      Counters::add("decision.no_route_to_prefix", 1);
    }
    return;
  }
  auto bestNextHop = prefixState.getLoopbackVias({dst.bestNode}, isV4, dst.bestIgpMetric);
  if (bestNextHop.size() != 1) {
    Counters::add("decision.missing_loopback_addr", 1);
    return;
  }
  const auto nhs = getNextHopsWithMetric(myNodeName, dst.nodes, false, areaLinkStates);
  RibUnicastEntry entry(
      prefix,
      getNextHopsThrift(
          myNodeName, dst.nodes, isV4, false, nhs.first, nhs.second, std::nullopt,
          areaLinkStates, dst.areas),
      prefixEntries.at(dst.bestNode).at(dst.bestArea),
      dst.bestArea,
      bgpDryRun_,
      bestNextHop.at(0));
  unicastEntries.emplace(prefix, std::move(entry));
}

void SpfSolver::SpfSolverImpl::selectKsp2(
    std::unordered_map<thrift::IpPrefix, RibUnicastEntry>& unicastEntries,
    const thrift::IpPrefix& prefix,
    const std::string& myNodeName,
    const BestPathCalResult& best,
    const thrift::PrefixEntries& prefixEntries,
    bool hasBgp,
    AreaLinkStates const& areaLinkStates,
    PrefixState const& prefixState,
    thrift::PrefixForwardingAlgorithm algo) {
  auto& clk = tEcmpClock;
  int64_t tk = nowNs();
  auto lap = [&](int i) {
    const int64_t n = nowNs();
    clk.ns[i] += n - tk;
    tk = n;
  };
  RibUnicastEntry entry(prefix);
  bool selfNodeContained = false;
  // the chosen paths as link-id spans of their area's flat kth-path memo
  struct PathRef {
    const LinkState* ls;
    const uint32_t* first;
    const uint32_t* last;
    size_t size() const { return (size_t)(last - first); }
  };
  std::vector<PathRef> paths;
  // LinkState::pathAInPathB on link ids: links of one area are equal iff
  // their ids are; links of different areas compare by value
  auto sameLink = [](const PathRef& a, uint32_t la, const PathRef& b, uint32_t lb) {
    return a.ls == b.ls ? la == lb : a.ls->linkOfId(la) == b.ls->linkOfId(lb);
  };
  auto aInB = [&](const PathRef& a, const PathRef& b) {
    if (a.size() > b.size()) {
      return false;
    }
    for (size_t start = 0; start + a.size() <= b.size(); ++start) {
      size_t k = 0;
      while (k < a.size() && sameLink(a, a.first[k], b, b.first[start + k])) {
        ++k;
      }
      if (k == a.size()) {
        return true;
      }
    }
    return false;
  };

  for (const auto& [_, ls] : areaLinkStates) {
    for (const auto& node : best.nodes) {
      if (node == myNodeName) {
        selfNodeContained = true;
        continue;
      }
      const auto& first = ls.kthPathIds(myNodeName, node, 1);
      for (size_t i = 0; i < first.size(); ++i) {
        paths.push_back({&ls, first.begin(i), first.end(i)});
      }
    }
    if (algo == thrift::PrefixForwardingAlgorithm::KSP2_ED_ECMP) {
      // drop second paths that contain a first path (anycast double spray)
      const size_t firstPaths = paths.size();
      for (const auto& node : best.nodes) {
        const auto& second = ls.kthPathIds(myNodeName, node, 2);
        for (size_t j = 0; j < second.size(); ++j) {
          const PathRef sec{&ls, second.begin(j), second.end(j)};
          bool contained = false;
          for (size_t i = 0; i < firstPaths && !contained; ++i) {
            contained = aInB(paths[i], sec);
          }
          if (!contained) {
            paths.push_back(sec);
          }
        }
      }
    }
  }
  lap(5);
  if (paths.empty()) {
    return;
  }

  // one next hop per (path, area): the path's cost and its label stack --
  // the node labels of the hops after the first (PHP), last hop on top of
  // the destination's prepend label (Decision.cpp:1000-1047)
  const bool isV4Prefix = prefix.prefixAddress.addr.size() == 4;
  std::vector<int32_t> hopLabels;
  // one area (the fabric): walk the paths by node id -- labels from the
  // per-build array, hop metrics from the device CSR -- instead of a name
  // lookup in the adjacency databases per hop (same values: the engine's
  // metrics are the links' metrics, ksp2Labels_ the databases' labels)
  const bool byId = ksp2Fast_.ok && areaLinkStates.size() == 1;
  // one next hop per path and area at most: no rehash while they go in
  entry.nexthops.reserve(paths.size() * areaLinkStates.size());
  std::vector<std::pair<uint32_t, const thrift::PrefixEntry*>> destCache;
  for (const auto& path : paths) {
    if (path.size() == 0) {
      throw std::logic_error("selectKsp2: empty path");
    }
    const Link& firstLink = path.ls->linkOfId(path.first[0]);
    if (byId && path.ls == ksp2Fast_.ls) {
      const auto& area = *ksp2Fast_.area;
      Metric cost = 0;
      uint32_t at = ksp2Fast_.me;
      hopLabels.clear();
      bool ok = true;
      for (const uint32_t* l = path.first; l != path.last && ok; ++l) {
        uint32_t to = 0;
        LinkStateMetric w = 0;
        ok = path.ls->linkHop(*l, at, to, w);
        cost += w;
        at = to;
        hopLabels.push_back(ok ? ksp2Fast_.labels[at] : 0);
      }
      if (ok) {
        const thrift::PrefixEntry* destEntry = nullptr;
        for (const auto& [id, e] : destCache) {
          if (id == at) {
            destEntry = e;
          }
        }
        if (!destEntry) {
          destEntry = &prefixEntries.at(path.ls->nodeNameOf(at)).at(area);
          destCache.emplace_back(at, destEntry);
        }
        std::vector<int32_t> labels;
        labels.reserve(hopLabels.size());
        if (destEntry->prependLabel) {
          labels.push_back(*destEntry->prependLabel); // bottom of stack
        }
        for (size_t h = hopLabels.size(); h-- > 1;) {
          labels.push_back(hopLabels[h]);
        }
        std::optional<thrift::MplsAction> action;
        if (!labels.empty()) {
          action = createMplsAction(thrift::MplsActionCode::PUSH, std::nullopt, std::move(labels));
        }
        entry.nexthops.insert(createNextHop(
            isV4Prefix ? firstLink.getNhV4FromNode(myNodeName)
                       : firstLink.getNhV6FromNode(myNodeName),
            firstLink.getIfaceFromNode(myNodeName), (int32_t)cost, action, true,
            firstLink.getArea()));
        continue;
      }
    }
    for (const auto& [area, ls] : areaLinkStates) {
      const auto& adjDbs = ls.getAdjacencyDatabases();
      Metric cost = 0;
      const std::string* at = &myNodeName;
      hopLabels.clear();
      for (const uint32_t* l = path.first; l != path.last; ++l) {
        const Link& link = path.ls->linkOfId(*l);
        cost += link.getMetricFromNode(*at);
        at = &link.getOtherNodeName(*at);
        hopLabels.push_back(adjDbs.at(*at).nodeLabel);
      }
      const auto& destEntry = prefixEntries.at(*at).at(area);
      std::vector<int32_t> labels;
      labels.reserve(hopLabels.size());
      if (destEntry.prependLabel) {
        labels.push_back(*destEntry.prependLabel); // bottom of stack
      }
      for (size_t h = hopLabels.size(); h-- > 1;) {
        labels.push_back(hopLabels[h]);
      }
      std::optional<thrift::MplsAction> action;
      if (!labels.empty()) {
        action = createMplsAction(thrift::MplsActionCode::PUSH, std::nullopt, std::move(labels));
      }
      entry.nexthops.insert(createNextHop(
          isV4Prefix ? firstLink.getNhV4FromNode(myNodeName)
                     : firstLink.getNhV6FromNode(myNodeName),
          firstLink.getIfaceFromNode(myNodeName), (int32_t)cost, action, true,
          firstLink.getArea()));
    }
  }

  lap(6);
  int staticNexthops = 0;
  if (selfNodeContained) {
    const auto& mine = prefixEntries.at(myNodeName);
    if (mine.size() != 1) {
      throw std::logic_error("selectKsp2: MPLS can only be originated to one area");
    }
    const int32_t label = mine.begin()->second.prependLabel.value();
    auto it = staticRoutes_.mplsRoutes.find(label);
    if (it != staticRoutes_.mplsRoutes.end()) {
      for (const auto& nh : it->second) {
        ++staticNexthops;
        entry.nexthops.insert(
            createNextHop(nh.address, std::nullopt, 0, std::nullopt, true, mine.begin()->first));
      }
    }
  }

  const auto minNextHop = getMinNextHopThreshold(best, prefixEntries);
  const int64_t dynamicNextHops = (int64_t)entry.nexthops.size() - staticNexthops;
  if (minNextHop && *minNextHop > dynamicNextHops) {
    return; // not enough next hops for this prefix
  }
  if (hasBgp) {
    auto bestNextHop = prefixState.getLoopbackVias(
        {best.bestNode}, prefix.prefixAddress.addr.size() == 4, best.bestIgpMetric);
    if (bestNextHop.size() == 1) {
      entry.bestNexthop = bestNextHop.at(0);
      entry.bestPrefixEntry = prefixEntries.at(best.bestNode).at(best.bestArea);
      entry.doNotInstall = bgpDryRun_;
    }
  }
  unicastEntries.emplace(prefix, std::move(entry));
  lap(7);
}

std::pair<Metric, NextHopNodes> SpfSolver::SpfSolverImpl::getNextHopsWithMetric(
    const std::string& myNodeName,
    const std::set<std::string>& dstNodeNames,
    bool perDestination,
    AreaLinkStates const& areaLinkStates) {
  NextHopNodes nextHopNodes;
  Metric shortestMetric = std::numeric_limits<Metric>::max();

  for (const auto& [areaName, ls] : areaLinkStates) {
    const SpfRead mine = myRead(myNodeName, areaName, ls);
    // closest announcers in this area
    Metric areaMin = std::numeric_limits<Metric>::max();
    std::vector<const std::string*> minCostNodes;
    for (const auto& dst : dstNodeNames) {
      const auto d = mine.metric(dst);
      if (!d) {
        continue;
      }
      if (areaMin >= *d) {
        if (areaMin > *d) {
          areaMin = *d;
          minCostNodes.clear();
        }
        minCostNodes.push_back(&dst);
      }
    }
    if (shortestMetric < areaMin) {
      continue;
    }
    if (shortestMetric > areaMin) {
      shortestMetric = areaMin;
      nextHopNodes.clear();
    }
    if (minCostNodes.empty()) {
      continue;
    }
    for (const std::string* dst : minCostNodes) {
      const std::string_view dstRef = perDestination ? std::string_view(*dst) : kNoDestName;
      mine.forEachNextHopWithMetric(*dst, [&](const std::string& nh, Metric toNh) {
        nextHopNodes[std::make_pair(std::string_view(nh), dstRef)] = shortestMetric - toNh;
      });
    }
    if (computeLfaPaths_) {
      if (const MyLinks* mls = cachedLinks(myNodeName, areaName)) {
        // RFC 5286 loop-free alternates through every up neighbour (per-build
        // neighbour views; each destination's id looked up once)
        std::vector<std::pair<const std::string*, std::optional<uint32_t>>> dsts;
        dsts.reserve(dstNodeNames.size());
        for (const auto& dst : dstNodeNames) {
          dsts.emplace_back(&dst, ls.nodeId(dst));
        }
        for (const LfaNbr& ln : mls->lfa) {
          if (!ln.toHere) {
            throw std::out_of_range("LFA: neighbour cannot reach " + myNodeName);
          }
          for (const auto& [dst, id] : dsts) {
            const auto dNbr = ln.read.metricById(id, *dst);
            if (!dNbr) {
              continue;
            }
            if (*dNbr < shortestMetric + *ln.toHere) {
              auto key = std::make_pair(
                  std::string_view(*ln.nbr),
                  perDestination ? std::string_view(*dst) : std::string_view(kNoDestName));
              auto it = nextHopNodes.find(key);
              if (it == nextHopNodes.end()) {
                nextHopNodes.emplace(std::move(key), *dNbr);
              } else if (it->second > *dNbr) {
                it->second = *dNbr;
              }
            }
          }
        }
        continue;
      }
      // RFC 5286 loop-free alternates through every up neighbour
      for (const auto& link : ls.linksFromNode(myNodeName)) {
        if (!link->isUp()) {
          continue;
        }
        const std::string& nbr = link->getOtherNodeName(myNodeName);
        SpfRead fromNbr(ls, nbr);
        const auto nbrToHere = fromNbr.metric(myNodeName);
        if (!nbrToHere) {
          throw std::out_of_range("LFA: neighbour cannot reach " + myNodeName);
        }
        for (const auto& dst : dstNodeNames) {
          const auto dNbr = fromNbr.metric(dst);
          if (!dNbr) {
            continue;
          }
          if (*dNbr < shortestMetric + *nbrToHere) {
            auto key = std::make_pair(
                std::string_view(nbr),
                perDestination ? std::string_view(dst) : std::string_view(kNoDestName));
            auto it = nextHopNodes.find(key);
            if (it == nextHopNodes.end()) {
              nextHopNodes.emplace(std::move(key), *dNbr);
            } else if (it->second > *dNbr) {
              it->second = *dNbr;
            }
          }
        }
      }
    }
  }
  return {shortestMetric, std::move(nextHopNodes)};
}

std::unordered_set<thrift::NextHopThrift> SpfSolver::SpfSolverImpl::getNextHopsThrift(
    const std::string& myNodeName,
    const std::set<std::string>& dstNodeNames,
    bool isV4,
    bool perDestination,
    Metric minMetric,
    const NextHopNodes& nextHopNodes,
    std::optional<int32_t> swapLabel,
    AreaLinkStates const& areaLinkStates,
    const std::set<std::string>& prefixAreas) const {
  if (nextHopNodes.empty()) {
    throw std::logic_error("getNextHopsThrift: no next-hop nodes");
  }
  static const std::set<std::string> kNoDest{std::string()};
  std::unordered_set<thrift::NextHopThrift> nextHops;
  nextHops.reserve(nextHopNodes.size() * 2);
  for (const auto& [area, ls] : areaLinkStates) {
    if (!prefixAreas.count(area)) {
      continue;
    }
    // every (up link of myNode, destination) pair whose (neighbour, destination)
    // is a next-hop node: walk the next-hop nodes and the links to each
    const MyLinks& mls = myLinks(myNodeName, area, ls);
    const auto& dests = perDestination ? dstNodeNames : kNoDest;
    for (auto search = nextHopNodes.begin(); search != nextHopNodes.end(); ++search) {
      const std::string_view dstView = search->first.second;
      auto dIt = dests.find(std::string(dstView));
      if (dIt == dests.end()) {
        continue;
      }
      const std::string& dstNode = *dIt;
      auto byNbr = mls.byNbr.find(search->first.first);
      if (byNbr == mls.byNbr.end()) {
        continue;
      }
      for (const uint32_t li : byNbr->second) {
        const MyLink& ml = mls.links[li];
        if (!ml.up) {
          continue;
        }
        const Link* link = ml.link;
        const std::string& nbr = *ml.nbr;
        // do not reach dstNode through another destination
        if (!dstNode.empty() && dstNodeNames.count(nbr) && nbr != dstNode) {
          continue;
        }
        const Metric distOverLink = ml.metric + search->second;
        if (!computeLfaPaths_ && distOverLink != minMetric) {
          continue; // only shortest paths without LFA
        }
        std::optional<thrift::MplsAction> action;
        if (swapLabel) {
          const bool nbrIsDst = dstNodeNames.count(nbr) > 0;
          action = createMplsAction(
              nbrIsDst ? thrift::MplsActionCode::PHP : thrift::MplsActionCode::SWAP,
              nbrIsDst ? std::nullopt : swapLabel);
        }
        if (!dstNode.empty() && dstNode != nbr) {
          const int32_t dstLabel = ls.getAdjacencyDatabases().at(dstNode).nodeLabel;
          if (!isMplsLabelValid(dstLabel)) {
            continue;
          }
          if (action) {
            throw std::logic_error("getNextHopsThrift: conflicting MPLS actions");
          }
          action = createMplsAction(
              thrift::MplsActionCode::PUSH, std::nullopt, std::vector<int32_t>{dstLabel});
        }
        nextHops.insert(createNextHop(
            isV4 ? *ml.nhV4 : *ml.nhV6, *ml.iface, (int32_t)distOverLink, action, false,
            link->getArea()));
      }
    }
  }
  return nextHops;
}

// ------------------------------------------------------------- SpfSolver

SpfSolver::SpfSolver(
    const std::string& myNodeName,
    bool enableV4,
    bool computeLfaPaths,
    bool enableOrderedFib,
    bool bgpDryRun,
    bool bgpUseIgpMetric)
    : impl_(std::make_unique<SpfSolverImpl>(
          myNodeName, enableV4, computeLfaPaths, enableOrderedFib, bgpDryRun,
          bgpUseIgpMetric)) {}

SpfSolver::~SpfSolver() = default;

bool SpfSolver::staticRoutesUpdated() { return impl_->staticRoutesUpdated(); }

void SpfSolver::pushRoutesDeltaUpdates(thrift::RouteDatabaseDelta& d) {
  impl_->pushRoutesDeltaUpdates(d);
}

std::optional<DecisionRouteUpdate> SpfSolver::processStaticRouteUpdates() {
  return impl_->processStaticRouteUpdates();
}

thrift::StaticRoutes const& SpfSolver::getStaticRoutes() { return impl_->getStaticRoutes(); }

std::optional<DecisionRouteDb> SpfSolver::buildRouteDbPartial(
    const std::string& myNodeName,
    std::unordered_map<std::string, LinkState> const& areaLinkStates,
    PrefixState const& prefixState,
    const std::unordered_set<thrift::IpPrefix>& skipUnicast,
    bool withMpls) {
  impl_->skipPrefixes_ = &skipUnicast;
  impl_->skipMpls_ = !withMpls;
  struct Reset {
    SpfSolverImpl* i;
    ~Reset() {
      i->skipPrefixes_ = nullptr;
      i->skipMpls_ = false;
    }
  } reset{impl_.get()};
  return impl_->buildRouteDb(myNodeName, areaLinkStates, prefixState);
}

std::optional<DecisionRouteDb> SpfSolver::buildRouteDb(
    const std::string& myNodeName,
    std::unordered_map<std::string, LinkState> const& areaLinkStates,
    PrefixState const& prefixState) {
  return impl_->buildRouteDb(myNodeName, areaLinkStates, prefixState);
}

} // namespace openr
