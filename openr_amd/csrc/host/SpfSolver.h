// SpfSolver.h — RouteDb generation for one node on top of the MI355X
// LinkState (drop-in for SpfSolver in openr/decision/Decision.h:212-254 and
// the RouteDb types of RibEntry.h:21-124, RouteUpdate.h:21-48,
// Decision.h:46-86).
#pragma once

#include <memory>
#include <optional>
#include <set>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "LinkState.h"
#include "PrefixState.h"
#include "Types.h"

namespace openr {

struct RibEntry {
  std::unordered_set<thrift::NextHopThrift> nexthops;
  RibEntry() = default;
  explicit RibEntry(std::unordered_set<thrift::NextHopThrift> nh) : nexthops(std::move(nh)) {}
  bool operator==(const RibEntry& other) const { return nexthops == other.nexthops; }
};

struct RibUnicastEntry : RibEntry {
  thrift::IpPrefix prefix; // folly::CIDRNetwork in the reference
  thrift::PrefixEntry bestPrefixEntry;
  std::string bestArea;
  bool doNotInstall{false};
  std::optional<thrift::NextHopThrift> bestNexthop;

  explicit RibUnicastEntry(const thrift::IpPrefix& p) : prefix(p) {}
  RibUnicastEntry(
      const thrift::IpPrefix& p,
      std::unordered_set<thrift::NextHopThrift> nh,
      thrift::PrefixEntry best = {},
      const std::string& area = "",
      bool dni = false,
      std::optional<thrift::NextHopThrift> bestNh = std::nullopt)
      : RibEntry(std::move(nh)),
        prefix(p),
        bestPrefixEntry(std::move(best)),
        bestArea(area),
        doNotInstall(dni),
        bestNexthop(std::move(bestNh)) {}

  bool operator==(const RibUnicastEntry& o) const {
    return prefix == o.prefix && bestPrefixEntry == o.bestPrefixEntry &&
        bestNexthop == o.bestNexthop && doNotInstall == o.doNotInstall &&
        RibEntry::operator==(o);
  }
  thrift::UnicastRoute toThrift() const;
};

struct RibMplsEntry : RibEntry {
  int32_t label{0};
  explicit RibMplsEntry(int32_t l) : label(l) {}
  RibMplsEntry(int32_t l, std::unordered_set<thrift::NextHopThrift> nh)
      : RibEntry(std::move(nh)), label(l) {}
  static RibMplsEntry fromThrift(const thrift::MplsRoute& r) {
    return RibMplsEntry(
        r.topLabel,
        std::unordered_set<thrift::NextHopThrift>(r.nextHops.begin(), r.nextHops.end()));
  }
  bool operator==(const RibMplsEntry& o) const {
    return label == o.label && RibEntry::operator==(o);
  }
  thrift::MplsRoute toThrift() const;
};

struct DecisionRouteDb {
  std::unordered_map<thrift::IpPrefix, RibUnicastEntry> unicastEntries;
  std::unordered_map<int32_t, RibMplsEntry> mplsEntries;
  thrift::RouteDatabase toThrift() const;
  // route shards buildRouteDb used (Parallel.h routeShards): releaseRouteDb
  // frees with the same split (0 = derive it from the route count)
  unsigned unicastShards{0}, mplsShards{0};
};

struct DecisionRouteUpdate {
  std::vector<RibUnicastEntry> unicastRoutesToUpdate;
  std::vector<thrift::IpPrefix> unicastRoutesToDelete;
  std::vector<RibMplsEntry> mplsRoutesToUpdate;
  std::vector<int32_t> mplsRoutesToDelete;
};

// Drop a RouteDb with its payload freed on the host worker pool: the
// Decision thread replaces its RouteDb on every rebuild (Decision.cpp:
// 1803-1804) and freeing ~10^5 next hops one by one costs more than the
// build itself on the fabric (time exported as decision.route_release_us).
void releaseRouteDb(DecisionRouteDb&& db);

// old vs new RouteDb -> delta (reference: Decision.cpp:47-85)
DecisionRouteUpdate getRouteDelta(const DecisionRouteDb& newDb, const DecisionRouteDb& oldDb);

struct BestPathCalResult {
  bool success{false};
  std::string bestNode;
  std::string bestArea;
  std::set<std::string> nodes;
  std::set<std::string> areas;
  std::optional<int64_t> bestIgpMetric;
  std::optional<thrift::MetricVector> bestVector;
};

class SpfSolver {
 public:
  SpfSolver(
      const std::string& myNodeName,
      bool enableV4,
      bool computeLfaPaths,
      bool enableOrderedFib = false,
      bool bgpDryRun = false,
      bool bgpUseIgpMetric = false);
  ~SpfSolver();
  SpfSolver(SpfSolver const&) = delete;
  SpfSolver& operator=(SpfSolver const&) = delete;

  bool staticRoutesUpdated();
  void pushRoutesDeltaUpdates(thrift::RouteDatabaseDelta& staticRoutesDelta);
  std::optional<DecisionRouteUpdate> processStaticRouteUpdates();
  thrift::StaticRoutes const& getStaticRoutes();

  // nullopt iff myNodeName is in no area (Decision.cpp:296-302)
  std::optional<DecisionRouteDb> buildRouteDb(
      const std::string& myNodeName,
      std::unordered_map<std::string, LinkState> const& areaLinkStates,
      PrefixState const& prefixState);

  // buildRouteDb without the unicast prefixes of `skipUnicast` and, with
  // withMpls = false, without MPLS routes: the host share of a RouteDb whose
  // other routes come from a device route table (AllAreasRouteTable)
  std::optional<DecisionRouteDb> buildRouteDbPartial(
      const std::string& myNodeName,
      std::unordered_map<std::string, LinkState> const& areaLinkStates,
      PrefixState const& prefixState,
      const std::unordered_set<thrift::IpPrefix>& skipUnicast,
      bool withMpls);

  class SpfSolverImpl;

 private:
  std::unique_ptr<SpfSolverImpl> impl_;
};

} // namespace openr
