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
// MPLS (Decision.cpp:415-534, this area, LFA off): every (node label, owner)
// pair is one more column of the same kernel pass -- a pseudo-prefix
// announced by the owner alone, so its cell is getNextHopsWithMetric(node,
// {owner}) -- and mplsRoutes(node) turns the cells into POP_AND_LOOKUP (own
// label) / PHP (next hop is the owner) / SWAP routes with the reference's
// collision rule (the smallest-named owner the node itself is or reaches),
// then adds the PHP routes of the node's adjacency labels (a node label
// keeps its entry when an adjacency label repeats it).
//
// The table owns its device graph, query and rows (a snapshot): it stays
// valid across later LinkState changes and answers for the topology it was
// built from.
#pragma once

#include <map>
#include <memory>
#include <optional>
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
  // computeLfa: SpfSolver's computeLfaPaths (loop-free alternates as extra
  // next hops with their own metrics, Decision.cpp:1146-1175)
  AllNodesRouteTable(
      const LinkState& ls, const PrefixState& ps, bool enableV4 = true, bool computeLfa = false);
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
  // The MPLS routes of `node` (node labels + adjacency labels, see above).
  std::unordered_map<int32_t, RibMplsEntry> mplsRoutes(const std::string& node) const;
  size_t numLabelColumns() const { return owners_.size(); }

  // Network-wide route delta against an older table over the same graph
  // layout, prefixes and node labels (spf_route_table_diff): per node (id
  // order, see nodeName) the number of changed columns -- unicast prefixes
  // and node-label columns (changedSplit separates them).  Throws
  // std::invalid_argument when the layouts differ.
  std::vector<uint32_t> diff(const AllNodesRouteTable& older);
  // (changed unicast prefixes, changed node-label columns) of `node` from
  // the last diff
  std::pair<uint32_t, uint32_t> changedSplit(const std::string& node) const;
  // getRouteDelta({routes, mplsRoutes}(node), the same of `older`)
  // (Decision.cpp:47-85) from the last diff: changed routes materialised,
  // vanished ones deleted.  MPLS candidates are the labels of changed label
  // columns and the node's adjacency labels, compared entry by entry against
  // `older` (which must outlive this call).
  DecisionRouteUpdate delta(const std::string& node) const;
  const std::string& nodeName(uint32_t id) const { return names_.at(id); }

 private:
  struct Row {
    std::vector<uint32_t> metric, best;
    std::vector<uint64_t> links;
    std::vector<uint32_t> lmet; // LFA: per-link metrics [cols][deg]
    size_t W = 0, deg = 0;
    // metric of link j of cell p (LFA: its own, else the cell's)
    uint32_t linkMetric(size_t p, uint32_t j) const {
      return lmet.empty() ? metric[p] : lmet[p * deg + j];
    }
  };
  Row fetchRow(uint32_t i) const;
  RibUnicastEntry materialise(const std::string& node, uint32_t i, const Row& r, size_t p) const;
  // the MPLS entry of `label` at node i: the node-label winner, else the
  // first adjacency label of that value
  std::optional<RibMplsEntry> mplsEntry(uint32_t i, const Row& r, int32_t label) const;
  std::optional<RibMplsEntry> nodeLabelEntry(uint32_t i, const Row& r, int32_t label) const;

  struct Announcer {
    uint32_t id;
    thrift::PrefixEntry entry;
  };
  std::string area_;
  bool enableV4_;
  bool lfa_;
  std::vector<std::string> names_;
  std::unordered_map<std::string, uint32_t> ids_;
  std::vector<uint32_t> row_;                 // CSR row offsets of the snapshot
  std::vector<std::shared_ptr<Link>> halfLink_; // half-edge -> Link
  std::vector<thrift::IpPrefix> prefixes_;
  std::vector<std::vector<Announcer>> announcers_;
  // node-label columns: column prefixes_.size() + k is owners_[k]
  struct LabelOwner {
    int32_t label;
    uint32_t id;
  };
  std::vector<LabelOwner> owners_;
  std::map<int32_t, std::vector<uint32_t>> labelCols_; // label -> owner columns by name
  // adjacency labels of every node, linksFromNode order (values copied)
  struct AdjLabel {
    int32_t label;
    thrift::BinaryAddress nhV6;
    std::string iface;
    int32_t metric;
    std::string area;
  };
  std::vector<std::vector<AdjLabel>> adjLabels_;
  const AllNodesRouteTable* older_{nullptr};
  spf_graph* graph_{nullptr};
  spf_query* query_{nullptr};
  spf_route_table* table_{nullptr};
  float spfMs_{0}, routeMs_{0};
  bool diffed_{false};
};

} // namespace openr
