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
#include <unordered_set>
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
  // borderNodes (multi-area, see AllAreasRouteTable): non-null selects the
  // prefixes this area's table can serve for its interior nodes -- entries
  // in this area, none of them by a border node; the announcers are the
  // in-area entries (for an interior node every other area's announcer is
  // unreachable, Decision.cpp:555-579)
  // bgpColumns (round 6, AllAreasRouteTable without bgpUseIgpMetric): BGP
  // prefixes on the device too.  With no IGP metric in the vector and every
  // in-graph announcer reachable from every node, the metric-vector
  // selection (runBestPathSelectionBgp, Decision.cpp:714-803) has the same
  // winners for every node, so it runs once on the host and the kernel takes
  // the winners (drained filter applied) as the column's announcers; a node
  // among them gets no route (selectEcmpBgp :805-866).  bestPrefixEntry,
  // bestArea and the loopback next hop are the selection's; doNotInstall =
  // bgpDryRun.  A prefix with an announcer some node cannot reach stays on
  // the host.  diff() refuses tables with BGP columns.
  AllNodesRouteTable(
      const LinkState& ls, const PrefixState& ps, bool enableV4 = true, bool computeLfa = false,
      const std::unordered_set<std::string>* borderNodes = nullptr, bool bgpColumns = false,
      bool bgpDryRun = false);
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
  // the unicast prefixes the kernel serves (routes() covers exactly these)
  const std::vector<thrift::IpPrefix>& prefixes() const { return prefixes_; }
  // BGP prefixes among them (bgpColumns)
  size_t numBgpPrefixes() const { return nbgp_; }

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
  // a BGP column's host-side selection (bgpColumns)
  struct BgpSel {
    thrift::PrefixEntry bestEntry;
    std::string bestArea;
    std::optional<thrift::NextHopThrift> bestNexthop; // nullopt: no route anywhere
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
  std::vector<std::optional<BgpSel>> bgp_; // per prefix (set: a BGP column)
  size_t nbgp_{0};
  bool bgpDryRun_{false};
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

// Every node's COMPLETE RouteDb over all areas (SURVEY §8(f) row 1 beyond
// one area and IGP prefixes): routeDb(node) == SpfSolver::buildRouteDb(node)
// (Decision.cpp:291-542) for any configuration -- multi-area, BGP,
// SR-MPLS / KSP2.  Device share: one AllNodesRouteTable per area (all-sources
// SPF + spf_route_table_kernel) serves the IP / SP_ECMP Open/R prefixes of
// the area's interior nodes (single area: every node, MPLS node labels
// included); the host share is SpfSolver::buildRouteDbPartial over the
// same LinkStates for what the kernel does not restate: border nodes (in two
// or more areas: cross-area ECMP and drain rules), BGP prefixes (metric-
// vector best path, Decision.cpp:714-866), SR-MPLS prefixes, prefixes a
// border node announces, and the multi-area MPLS routes.  With
// prefetchAll, every area's all-sources SPF views are computed in one
// device batch up front, so the host share runs no SPF per node.
class AllAreasRouteTable {
 public:
  AllAreasRouteTable(
      const std::unordered_map<std::string, LinkState>& areas, const PrefixState& ps,
      bool enableV4 = true, bool computeLfa = false, bool bgpDryRun = false,
      bool bgpUseIgpMetric = false, bool prefetchAll = true);
  ~AllAreasRouteTable();
  // nullopt iff `node` is in no area (Decision.cpp:296-302)
  std::optional<DecisionRouteDb> routeDb(const std::string& node) const;
  // routes of the last routeDb() call that came from a device table / the host
  size_t lastTableRoutes() const { return lastTable_; }
  size_t lastHostRoutes() const { return lastHost_; }
  bool isBorder(const std::string& node) const { return border_.count(node) > 0; }
  size_t numTables() const { return tables_.size(); }
  // BGP prefixes the device tables serve (round 6; AllNodesRouteTable
  // bgpColumns)
  size_t numBgpDevicePrefixes() const {
    size_t n = 0;
    for (const auto& [_, t] : tables_) {
      n += t->numBgpPrefixes();
    }
    return n;
  }

 private:
  const std::unordered_map<std::string, LinkState>& areas_;
  const PrefixState& ps_;
  bool enableV4_, lfa_, bgpDryRun_, bgpIgp_;
  std::unordered_set<std::string> border_;
  std::unordered_map<std::string, std::string> home_; // interior node -> its area
  std::map<std::string, std::unique_ptr<AllNodesRouteTable>> tables_;
  std::map<std::string, std::unordered_set<thrift::IpPrefix>> served_;
  std::map<std::string, bool> rest_; // area -> some prefix is left to the host
  mutable size_t lastTable_{0}, lastHost_{0};
};

} // namespace openr
