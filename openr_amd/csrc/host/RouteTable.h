// RouteTable.h — the unicast RouteDb of EVERY node of an area, on the device
// (SURVEY.md §8(f) row 1).
//
// The reference builds one node's RouteDb at a time on the Decision thread
// (SpfSolverImpl::buildRouteDb, openr/decision/Decision.cpp:291-542); views
// of other nodes' routes (ctrl getRouteDbComputed, OpenrCtrlHandler.cpp:
// 411-416; breeze `decision routes --nodes`, commands/decision.py:48-363)
// call it again per node.  AllNodesRouteTable runs ONE all-sources SPF with
// next hops over the area graph and spf_route_table_kernel over every
// eligible prefix, so the routes of any node are a row read away.
//
// Scope (what the kernel restates, include/openr_spf.h): prefixes advertised
// in this area only, no BGP entries, forwarding type IP with algorithm
// SP_ECMP (Decision.cpp:395-412), v4 prefixes only with enableV4, LFA off —
// i.e. SpfSolverImpl::selectEcmpOpenr.  routes(node) equals the unicast
// entries SpfSolver::buildRouteDb(node) produces for those prefixes
// (tests/test_route_table.py).
//
// The table owns its device graph, query and rows (a snapshot): it stays
// valid across later LinkState changes and answers for the topology it was
// built from.
#pragma once

#include <memory>
#include <string>
#include <unordered_map>
#include <vector>

#include "LinkState.h"
#include "PrefixState.h"
#include "SpfSolver.h"
#include "openr_spf.h"

namespace openr {

class AllNodesRouteTable {
 public:
  AllNodesRouteTable(const LinkState& ls, const PrefixState& ps, bool enableV4 = true);
  ~AllNodesRouteTable();
  AllNodesRouteTable(const AllNodesRouteTable&) = delete;
  AllNodesRouteTable& operator=(const AllNodesRouteTable&) = delete;

  size_t numNodes() const { return names_.size(); }
  size_t numPrefixes() const { return prefixes_.size(); }
  // device time of the all-sources SPF (+ next hops) and of the route kernel
  float spfMs() const { return spfMs_; }
  float routeMs() const { return routeMs_; }
  // routes present in the table (metric != no-route), over all nodes
  uint64_t countRoutes() const;

  // The unicast routes of `node` (empty if the node is not in the area).
  std::unordered_map<thrift::IpPrefix, RibUnicastEntry> routes(const std::string& node) const;

  // Network-wide route delta against an older table over the same graph
  // layout and prefixes (spf_route_table_diff): per node (id order, see
  // nodeName) the number of prefixes whose route changed.  Throws
  // std::invalid_argument when the layouts differ.
  std::vector<uint32_t> diff(const AllNodesRouteTable& older);
  // The unicast part of getRouteDelta(routes(node), older.routes(node))
  // (Decision.cpp:47-85) from the last diff: changed routes materialised,
  // vanished ones deleted.
  DecisionRouteUpdate delta(const std::string& node) const;
  const std::string& nodeName(uint32_t id) const { return names_.at(id); }

 private:
  struct Row {
    std::vector<uint32_t> metric, best;
    std::vector<uint64_t> links;
    size_t W = 0;
  };
  Row fetchRow(uint32_t i) const;
  RibUnicastEntry materialise(const std::string& node, uint32_t i, const Row& r, size_t p) const;

  struct Announcer {
    uint32_t id;
    thrift::PrefixEntry entry;
  };
  std::string area_;
  bool enableV4_;
  std::vector<std::string> names_;
  std::unordered_map<std::string, uint32_t> ids_;
  std::vector<uint32_t> row_;                 // CSR row offsets of the snapshot
  std::vector<std::shared_ptr<Link>> halfLink_; // half-edge -> Link
  std::vector<thrift::IpPrefix> prefixes_;
  std::vector<std::vector<Announcer>> announcers_;
  spf_graph* graph_{nullptr};
  spf_query* query_{nullptr};
  spf_route_table* table_{nullptr};
  float spfMs_{0}, routeMs_{0};
  bool diffed_{false};
};

} // namespace openr
