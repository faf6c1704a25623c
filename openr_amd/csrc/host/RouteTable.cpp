// RouteTable.cpp — AllNodesRouteTable (see RouteTable.h).

#include "RouteTable.h"

#include <algorithm>
#include <chrono>
#include <set>
#include <stdexcept>

#include "Engine.h"
#include "Parallel.h"
#include "Util.h"

namespace openr {

namespace {
int64_t usSince(std::chrono::steady_clock::time_point t0) {
  return std::chrono::duration_cast<std::chrono::microseconds>(
             std::chrono::steady_clock::now() - t0)
      .count();
}

[[noreturn]] void tableFailure(const char* what, int status) {
  throw std::runtime_error(
      std::string("openr_spf: ") + what + ": " + spf_error_string(status) + " (" +
      spf_last_error_detail() + ")");
}
} // namespace

AllNodesRouteTable::AllNodesRouteTable(
    const LinkState& ls, const PrefixState& ps, bool enableV4, bool computeLfa,
    const std::unordered_set<std::string>* borderNodes, bool bgpColumns, bool bgpDryRun)
    : area_(ls.getArea()), enableV4_(enableV4), lfa_(computeLfa), bgpDryRun_(bgpDryRun) {
  auto tp = std::chrono::steady_clock::now();
  LinkState::Engine& eng = ls.engine();
  Counters::add("decision.route_table_engine_us", usSince(tp));
  tp = std::chrono::steady_clock::now();
  if (eng.exact) {
    throw std::invalid_argument(
        "AllNodesRouteTable: metric 0 / 64-bit sums need the exact kernel");
  }
  names_ = eng.names;
  ids_ = eng.ids;
  row_ = eng.row;
  halfLink_.resize(eng.col.size());
  for (size_t e = 0; e < eng.col.size(); ++e) {
    halfLink_[e] = eng.links[eng.linkId[e]];
  }
  // own snapshot of the device graph (the table outlives LinkState changes)
  // and the all-sources query, first: BGP columns check reachability on it
  spf_graph_desc d{};
  d.num_nodes = (uint32_t)eng.names.size();
  d.num_edges = (uint32_t)eng.col.size();
  d.row_ptr = eng.row.data();
  d.col = eng.col.data();
  d.metric = eng.metric.data();
  d.link_id = eng.linkId.data();
  d.rev = eng.rev.data();
  d.node_overloaded = eng.overloaded.data();
  d.num_links = (uint32_t)eng.links.size();
  d.device = getSpfDevice();
  if (int s = spf_graph_create(&d, &graph_); s != SPF_OK) {
    tableFailure("spf_graph_create", s);
  }
  Counters::add("decision.route_table_graph_us", usSince(tp));
  auto cleanup = [&](const char* what, int st) {
    spf_route_table_destroy(table_);
    spf_query_destroy(query_);
    spf_graph_destroy(graph_);
    table_ = nullptr;
    query_ = nullptr;
    graph_ = nullptr;
    tableFailure(what, st);
  };
  try {
    tp = std::chrono::steady_clock::now();
    std::vector<uint32_t> src(d.num_nodes);
    for (uint32_t i = 0; i < d.num_nodes; ++i) {
      src[i] = i;
    }
    spf_query_desc qd{};
    qd.num_queries = d.num_nodes;
    qd.sources = src.data();
    qd.flags = SPF_F_NEXTHOPS;
    int s = SPF_OK;
    if ((s = spf_query_create(graph_, &qd, &query_)) != SPF_OK) {
      cleanup("spf_query_create", s);
    }
    if ((s = spf_query_run(query_)) != SPF_OK) {
      cleanup("spf_query_run", s);
    }
    Counters::add("decision.route_table_query_us", usSince(tp));
    tp = std::chrono::steady_clock::now();
    // eligible prefixes (Decision.cpp:313-412 restricted to selectEcmpOpenr,
    // and with bgpColumns selectEcmpBgp)
    std::vector<uint32_t> annOff{0}, ann;
    {
      // eligibility and announcers per prefix on the host pool (read-only
      // PrefixState lookups), kept in the map's iteration order
      std::vector<std::pair<const thrift::IpPrefix*, const thrift::PrefixEntries*>> items;
      items.reserve(ps.prefixes().size());
      for (const auto& [prefix, entries] : ps.prefixes()) {
        items.emplace_back(&prefix, &entries);
      }
      std::vector<uint8_t> keep(items.size(), 0);
      std::vector<std::vector<Announcer>> anns(items.size());
      std::vector<std::optional<BgpSel>> sels(items.size());
      // BGP candidates: every in-graph announcer (the selection assumes each
      // is reachable from every node; checked below)
      std::vector<std::vector<uint32_t>> bgpAll(items.size());
      parallelFor(items.size(), hostThreads(items.size(), 256), [&](size_t i, unsigned) {
        const auto& prefix = *items[i].first;
        const auto& entries = *items[i].second;
        bool otherArea = false, bgp = false, nonBgp = false, missingMv = false, inArea = false,
             borderAnn = false;
        for (const auto& [node, byArea] : entries) {
          for (const auto& [area, entry] : byArea) {
            otherArea |= area != area_;
            inArea |= area == area_;
            borderAnn |= area == area_ && borderNodes && borderNodes->count(node);
            const bool isBgp = entry.type == thrift::PrefixType::BGP;
            bgp |= isBgp;
            nonBgp |= !isBgp;
            missingMv |= isBgp && !entry.mv.has_value();
          }
        }
        if ((bgp && !bgpColumns) || (bgp && (nonBgp || missingMv)) || entries.empty() ||
            (otherArea && !borderNodes) || !inArea || borderAnn) {
          return;
        }
        if (prefix.prefixAddress.addr.size() == 4 && !enableV4_) {
          return;
        }
        if (getPrefixForwardingType(entries) != thrift::PrefixForwardingType::IP ||
            getPrefixForwardingAlgorithm(entries) != thrift::PrefixForwardingAlgorithm::SP_ECMP) {
          return;
        }
        if (!bgp) {
          for (const auto& [node, byArea] : entries) {
            auto it = ids_.find(node);
            auto ea = byArea.find(area_);
            if (it == ids_.end() || ea == byArea.end()) {
              continue; // not in the graph / announced in another area: never reachable
            }
            anns[i].push_back(Announcer{it->second, ea->second});
          }
          keep[i] = 1;
          return;
        }
        if (otherArea) {
          return; // (interior-node tables of several areas: BGP stays on the host)
        }
        // runBestPathSelectionBgp (Decision.cpp:714-803) without the IGP
        // cost, every in-graph announcer reachable: entries in map order
        namespace mvu = MetricVectorUtils;
        std::optional<thrift::MetricVector> bestVector;
        std::set<std::string> winners;
        std::string bestNode, bestArea;
        for (const auto& [node, byArea] : entries) {
          for (const auto& [area, entry] : byArea) {
            auto it = ids_.find(node);
            if (it == ids_.end()) {
              continue; // not in the graph: unreachable from every node
            }
            bgpAll[i].push_back(it->second);
            const thrift::MetricVector& mvIn = entry.mv.value();
            if (mvu::getMetricEntityByType(mvIn, mvu::kOpenrIgpCostType)) {
              continue;
            }
            thrift::MetricVector mv = mvIn;
            mvu::CompareResult cmp = mvu::CompareResult::WINNER;
            if (bestVector) {
              cmp = mvu::compareMetricVectors(mv, *bestVector);
            }
            switch (cmp) {
            case mvu::CompareResult::WINNER:
              winners.clear();
              [[fallthrough]];
            case mvu::CompareResult::TIE_WINNER:
              bestVector = std::move(mv);
              bestNode = node;
              bestArea = area;
              [[fallthrough]];
            case mvu::CompareResult::TIE_LOOSER:
              winners.insert(node);
              break;
            case mvu::CompareResult::TIE:
            case mvu::CompareResult::ERROR:
              // cannot order: no route at any node
              sels[i] = BgpSel{};
              keep[i] = 2;
              return;
            default:
              break;
            }
          }
        }
        BgpSel sel;
        if (!winners.empty()) {
          // maybeFilterDrainedNodes (Decision.cpp:651-666)
          std::set<std::string> undrained;
          for (const auto& w : winners) {
            if (!ls.isNodeOverloaded(w)) {
              undrained.insert(w);
            }
          }
          const auto& use = undrained.empty() ? winners : undrained;
          auto vias = ps.getLoopbackVias({bestNode}, prefix.prefixAddress.addr.size() == 4,
                                         std::nullopt);
          if (vias.size() == 1) {
            sel.bestEntry = entries.at(bestNode).at(bestArea);
            sel.bestArea = bestArea;
            sel.bestNexthop = vias.at(0);
            for (const auto& w : use) {
              anns[i].push_back(Announcer{ids_.at(w), entries.at(w).at(area_)});
            }
          }
        }
        sels[i] = std::move(sel);
        keep[i] = 2;
      }, 64);
      // BGP columns need every in-graph announcer reachable from every node:
      // reachability is symmetric here (links are up in both directions and a
      // path's interior nodes are the same either way), so the announcer's
      // own row answers for every node
      std::unordered_map<uint32_t, bool> reachesAll;
      std::vector<uint32_t> rowBuf(d.num_nodes);
      for (size_t i = 0; i < items.size(); ++i) {
        if (keep[i] != 2) {
          continue;
        }
        for (const uint32_t a : bgpAll[i]) {
          auto it = reachesAll.find(a);
          if (it == reachesAll.end()) {
            if (int st = spf_query_fetch_rows(query_, a, 1, rowBuf.data(), (size_t)d.num_nodes * 4,
                                              0);
                st != SPF_OK) {
              cleanup("spf_query_fetch_rows", st);
            }
            const bool all = std::all_of(rowBuf.begin(), rowBuf.end(),
                                         [](uint32_t x) { return x != 0xFFFFFFFFu; });
            it = reachesAll.emplace(a, all).first;
          }
          if (!it->second) {
            keep[i] = 0; // some node does not reach this announcer: the host path
            break;
          }
        }
      }
      for (size_t i = 0; i < items.size(); ++i) {
        if (keep[i]) {
          prefixes_.push_back(*items[i].first);
          announcers_.push_back(std::move(anns[i]));
          bgp_.push_back(keep[i] == 2 ? std::move(sels[i]) : std::nullopt);
          nbgp_ += keep[i] == 2;
        }
      }
    }
    // prefix order: by first announcer id, so neighbouring lanes of the
    // kernel read neighbouring distance / next-hop mask words of a row
    {
      std::vector<uint32_t> order(prefixes_.size());
      for (uint32_t i = 0; i < order.size(); ++i) {
        order[i] = i;
      }
      auto key = [&](uint32_t i) {
        return announcers_[i].empty() ? 0xFFFFFFFFu : announcers_[i][0].id;
      };
      std::stable_sort(order.begin(), order.end(),
                       [&](uint32_t x, uint32_t y) { return key(x) < key(y); });
      std::vector<thrift::IpPrefix> px;
      std::vector<std::vector<Announcer>> ax;
      std::vector<std::optional<BgpSel>> bx;
      px.reserve(order.size());
      ax.reserve(order.size());
      bx.reserve(order.size());
      for (uint32_t i : order) {
        px.push_back(std::move(prefixes_[i]));
        ax.push_back(std::move(announcers_[i]));
        bx.push_back(std::move(bgp_[i]));
      }
      prefixes_ = std::move(px);
      announcers_ = std::move(ax);
      bgp_ = std::move(bx);
      for (const auto& as : announcers_) {
        for (const auto& a : as) {
          ann.push_back(a.id);
        }
        annOff.push_back((uint32_t)ann.size());
      }
    }
    Counters::add("decision.route_table_prefixes_us", usSince(tp));
    // node-label columns (Decision.cpp:415-481): one pseudo-prefix per (valid
    // label, owner in the graph), owners of a label by name; the cell of node
    // s is getNextHopsWithMetric(s, {owner}) with LFA off
    {
      // (label, owner id) sorted: labels ascending, owners by name (ids are
      // name ranks) -- the order of a label -> sorted names map, without one
      std::vector<std::pair<int32_t, uint32_t>> lab;
      lab.reserve(names_.size());
      for (const auto& [node, db] : ls.getAdjacencyDatabases()) {
        if (db.nodeLabel == 0 || !isMplsLabelValid(db.nodeLabel)) {
          continue;
        }
        auto it = ids_.find(node);
        if (it != ids_.end()) {
          lab.emplace_back(db.nodeLabel, it->second);
        }
      }
      std::sort(lab.begin(), lab.end());
      for (size_t i = 0; i < lab.size();) {
        auto& cols =
            labelCols_.emplace_hint(labelCols_.end(), lab[i].first, std::vector<uint32_t>{})
                ->second;
        size_t j = i;
        for (; j < lab.size() && lab[j].first == lab[i].first; ++j) {
          cols.push_back((uint32_t)(prefixes_.size() + owners_.size()));
          owners_.push_back(LabelOwner{lab[j].first, lab[j].second});
          ann.push_back(lab[j].second);
          annOff.push_back((uint32_t)ann.size());
        }
        i = j;
      }
    }
    Counters::add("decision.route_table_labels_us", usSince(tp));
    // adjacency labels of every node (Decision.cpp:511-534), values copied
    // (independent per node: read-only LinkState lookups on the host pool)
    adjLabels_.resize(names_.size());
    parallelFor(names_.size(), hostThreads(names_.size(), 256), [&](size_t i, unsigned) {
      for (const auto& link : ls.linksFromNode(names_[i])) {
        const int32_t label = link->getAdjLabelFromNode(names_[i]);
        if (label == 0 || !isMplsLabelValid(label)) {
          continue;
        }
        adjLabels_[i].push_back(AdjLabel{
            label, link->getNhV6FromNode(names_[i]), link->getIfaceFromNode(names_[i]),
            (int32_t)link->getMetricFromNode(names_[i]), link->getArea()});
      }
    }, 64);
    Counters::add("decision.route_table_host_us", usSince(tp));
    tp = std::chrono::steady_clock::now();
    if ((s = spf_route_table_create_ex(
             query_, (uint32_t)(prefixes_.size() + owners_.size()), annOff.data(),
             ann.empty() ? nullptr : ann.data(), lfa_ ? SPF_RT_LFA : 0u, &table_)) != SPF_OK) {
      cleanup("spf_route_table_create", s);
    }
    Counters::add("decision.route_table_create_us", usSince(tp));
    tp = std::chrono::steady_clock::now();
    if ((s = spf_route_table_run(table_)) != SPF_OK) {
      cleanup("spf_route_table_run", s);
    }
    if ((s = spf_query_elapsed_ms(query_, &spfMs_)) != SPF_OK ||
        (s = spf_route_table_elapsed_ms(table_, &routeMs_)) != SPF_OK) {
      cleanup("elapsed", s);
    }
  } catch (...) {
    // (cleanup already released the handles when it threw)
    spf_route_table_destroy(table_);
    spf_query_destroy(query_);
    spf_graph_destroy(graph_);
    table_ = nullptr;
    query_ = nullptr;
    graph_ = nullptr;
    throw;
  }
  Counters::add("decision.route_table_run_us", usSince(tp));
  Counters::add("decision.route_table_builds", 1);
}

AllNodesRouteTable::~AllNodesRouteTable() {
  const auto tp = std::chrono::steady_clock::now();
  spf_route_table_destroy(table_);
  spf_query_destroy(query_);
  spf_graph_destroy(graph_);
  Counters::add("decision.route_table_destroy_us", usSince(tp));
}

uint64_t AllNodesRouteTable::countRoutes() const {
  uint64_t n = 0;
  const size_t C = prefixes_.size() + owners_.size();
  std::vector<uint32_t> metric(C), best(C);
  std::vector<uint64_t> links;
  for (uint32_t i = 0; i < names_.size(); ++i) {
    const int w = spf_route_table_link_words(table_, i);
    links.resize(std::max<size_t>(1, C * (size_t)std::max(w, 0)));
    if (int s = spf_route_table_fetch(table_, i, metric.data(), best.data(), links.data());
        s != SPF_OK) {
      tableFailure("spf_route_table_fetch", s);
    }
    for (size_t p = 0; p < prefixes_.size(); ++p) {
      n += metric[p] != 0xFFFFFFFFu;
    }
  }
  return n;
}

AllNodesRouteTable::Row AllNodesRouteTable::fetchRow(uint32_t i) const {
  Row r;
  const int w = spf_route_table_link_words(table_, i);
  if (w < 0) {
    tableFailure("spf_route_table_link_words", w);
  }
  const size_t P = prefixes_.size() + owners_.size();
  r.W = (size_t)w;
  r.metric.resize(P);
  r.best.resize(P);
  r.links.resize(std::max<size_t>(1, P * r.W));
  if (int s = spf_route_table_fetch(table_, i, r.metric.data(), r.best.data(), r.links.data());
      s != SPF_OK) {
    tableFailure("spf_route_table_fetch", s);
  }
  if (lfa_) {
    r.deg = row_[i + 1] - row_[i];
    r.lmet.resize(std::max<size_t>(1, P * r.deg));
    if (int s = spf_route_table_fetch_link_metrics(table_, i, r.lmet.data()); s != SPF_OK) {
      tableFailure("spf_route_table_fetch_link_metrics", s);
    }
  }
  return r;
}

RibUnicastEntry AllNodesRouteTable::materialise(
    const std::string& node, uint32_t i, const Row& r, size_t p) const {
  const bool isV4 = prefixes_[p].prefixAddress.addr.size() == 4;
  const uint32_t e0 = row_[i];
  std::unordered_set<thrift::NextHopThrift> nhs;
  for (size_t k = 0; k < r.W; ++k) {
    uint64_t m = r.links[p * r.W + k];
    while (m) {
      const uint32_t j = (uint32_t)(k * 64 + __builtin_ctzll(m));
      m &= m - 1;
      const Link& l = *halfLink_[e0 + j];
      nhs.insert(createNextHop(
          isV4 ? l.getNhV4FromNode(node) : l.getNhV6FromNode(node), l.getIfaceFromNode(node),
          (int32_t)r.linkMetric(p, j), std::nullopt, false, l.getArea()));
    }
  }
  if (bgp_[p]) {
    // selectEcmpBgp (Decision.cpp:805-866): the host-side selection's best
    const BgpSel& b = *bgp_[p];
    return RibUnicastEntry(prefixes_[p], std::move(nhs), b.bestEntry, b.bestArea, bgpDryRun_,
                           b.bestNexthop);
  }
  const thrift::PrefixEntry* bestEntry = nullptr;
  for (const auto& a : announcers_[p]) {
    if (a.id == r.best[p]) {
      bestEntry = &a.entry;
    }
  }
  if (!bestEntry) {
    throw std::logic_error("AllNodesRouteTable: best announcer not in the prefix");
  }
  return RibUnicastEntry(prefixes_[p], std::move(nhs), *bestEntry, area_);
}

std::unordered_map<thrift::IpPrefix, RibUnicastEntry> AllNodesRouteTable::routes(
    const std::string& node) const {
  std::unordered_map<thrift::IpPrefix, RibUnicastEntry> out;
  auto it = ids_.find(node);
  if (it == ids_.end() || prefixes_.empty()) {
    return out;
  }
  const Row r = fetchRow(it->second);
  for (size_t p = 0; p < prefixes_.size(); ++p) {
    if (r.metric[p] != 0xFFFFFFFFu) {
      out.emplace(prefixes_[p], materialise(node, it->second, r, p));
    }
  }
  return out;
}

std::optional<RibMplsEntry> AllNodesRouteTable::nodeLabelEntry(
    uint32_t i, const Row& r, int32_t label) const {
  auto lc = labelCols_.find(label);
  if (lc == labelCols_.end()) {
    return std::nullopt;
  }
  // the smallest-named owner that is this node (POP_AND_LOOKUP) or that it
  // reaches (an unreachable owner inserts nothing and blocks nothing)
  for (const uint32_t col : lc->second) {
    const LabelOwner& o = owners_[col - prefixes_.size()];
    if (o.id == i) {
      thrift::NextHopThrift nh;
      nh.address.addr = std::string(16, '\0'); // "::"
      nh.area = area_;
      nh.mplsAction = createMplsAction(thrift::MplsActionCode::POP_AND_LOOKUP);
      return RibMplsEntry(label, {nh});
    }
    if (r.metric[col] == 0xFFFFFFFFu) {
      continue;
    }
    const std::string& node = names_[i];
    const std::string& owner = names_[o.id];
    const uint32_t e0 = row_[i];
    std::unordered_set<thrift::NextHopThrift> nhs;
    for (size_t k = 0; k < r.W; ++k) {
      uint64_t m = r.links[col * r.W + k];
      while (m) {
        const uint32_t j = (uint32_t)(k * 64 + __builtin_ctzll(m));
        m &= m - 1;
        const Link& l = *halfLink_[e0 + j];
        const bool php = l.getOtherNodeName(node) == owner;
        nhs.insert(createNextHop(
            l.getNhV6FromNode(node), l.getIfaceFromNode(node), (int32_t)r.linkMetric(col, j),
            createMplsAction(
                php ? thrift::MplsActionCode::PHP : thrift::MplsActionCode::SWAP,
                php ? std::nullopt : std::optional<int32_t>(label)),
            false, l.getArea()));
      }
    }
    return RibMplsEntry(label, std::move(nhs));
  }
  return std::nullopt;
}

std::optional<RibMplsEntry> AllNodesRouteTable::mplsEntry(
    uint32_t i, const Row& r, int32_t label) const {
  if (auto e = nodeLabelEntry(i, r, label)) {
    return e;
  }
  for (const AdjLabel& a : adjLabels_[i]) {
    if (a.label == label) {
      return RibMplsEntry(
          label,
          {createNextHop(a.nhV6, a.iface, a.metric, createMplsAction(thrift::MplsActionCode::PHP),
                         false, a.area)});
    }
  }
  return std::nullopt;
}

std::unordered_map<int32_t, RibMplsEntry> AllNodesRouteTable::mplsRoutes(
    const std::string& node) const {
  std::unordered_map<int32_t, RibMplsEntry> out;
  auto it = ids_.find(node);
  if (it == ids_.end()) {
    return out;
  }
  const uint32_t i = it->second;
  const Row r = owners_.empty() ? Row{} : fetchRow(i);
  for (const auto& [label, cols] : labelCols_) {
    if (auto e = nodeLabelEntry(i, r, label)) {
      out.emplace(label, std::move(*e));
    }
  }
  for (const AdjLabel& a : adjLabels_[i]) {
    if (!out.count(a.label)) {
      out.emplace(a.label, *mplsEntry(i, r, a.label));
    }
  }
  return out;
}

std::vector<uint32_t> AllNodesRouteTable::diff(const AllNodesRouteTable& older) {
  bool sameOwners = older.owners_.size() == owners_.size();
  for (size_t k = 0; sameOwners && k < owners_.size(); ++k) {
    sameOwners = older.owners_[k].label == owners_[k].label && older.owners_[k].id == owners_[k].id;
  }
  if (nbgp_ || older.nbgp_) {
    throw std::invalid_argument(
        "AllNodesRouteTable::diff: tables with BGP columns (AllAreasRouteTable) are not diffed");
  }
  if (older.names_ != names_ || older.prefixes_ != prefixes_ || older.row_ != row_ ||
      !sameOwners || older.lfa_ != lfa_) {
    throw std::invalid_argument(
        "AllNodesRouteTable::diff: different nodes, prefixes, node labels or links");
  }
  std::vector<uint32_t> changed(names_.size());
  if (int s = spf_route_table_diff(older.table_, table_, changed.data()); s != SPF_OK) {
    if (s == SPF_E_UNSUPPORTED) {
      throw std::invalid_argument(std::string("AllNodesRouteTable::diff: ") +
                                  spf_last_error_detail());
    }
    tableFailure("spf_route_table_diff", s);
  }
  diffed_ = true;
  older_ = &older;
  return changed;
}

std::pair<uint32_t, uint32_t> AllNodesRouteTable::changedSplit(const std::string& node) const {
  if (!diffed_) {
    throw std::logic_error("AllNodesRouteTable::changedSplit: no diff has run");
  }
  auto it = ids_.find(node);
  const size_t P = prefixes_.size(), C = P + owners_.size();
  if (it == ids_.end() || !C) {
    return {0, 0};
  }
  std::vector<uint64_t> bits((C + 63) / 64);
  if (int s = spf_route_table_changed(table_, it->second, bits.data()); s != SPF_OK) {
    tableFailure("spf_route_table_changed", s);
  }
  uint32_t uni = 0, lab = 0;
  for (size_t k = 0; k < bits.size(); ++k) {
    uint64_t m = bits[k];
    while (m) {
      const size_t p = k * 64 + __builtin_ctzll(m);
      m &= m - 1;
      (p < P ? uni : lab) += 1;
    }
  }
  return {uni, lab};
}

DecisionRouteUpdate AllNodesRouteTable::delta(const std::string& node) const {
  DecisionRouteUpdate u;
  auto it = ids_.find(node);
  if (!diffed_) {
    throw std::logic_error("AllNodesRouteTable::delta: no diff has run");
  }
  if (it == ids_.end()) {
    return u;
  }
  const uint32_t i = it->second;
  const size_t P = prefixes_.size(), C = P + owners_.size();
  std::vector<uint64_t> bits((C + 63) / 64);
  if (C) {
    if (int s = spf_route_table_changed(table_, i, bits.data()); s != SPF_OK) {
      tableFailure("spf_route_table_changed", s);
    }
  }
  bool any = false;
  for (uint64_t b : bits) {
    any |= b != 0;
  }
  // MPLS candidates: labels of changed label columns + adjacency labels
  std::set<int32_t> labels;
  for (const AdjLabel& a : adjLabels_[i]) {
    labels.insert(a.label);
  }
  for (const AdjLabel& a : older_->adjLabels_[i]) {
    labels.insert(a.label);
  }
  if (!any && labels.empty()) {
    return u;
  }
  const Row r = C ? fetchRow(i) : Row{};
  for (size_t k = 0; k < bits.size(); ++k) {
    uint64_t m = bits[k];
    while (m) {
      const size_t p = k * 64 + __builtin_ctzll(m);
      m &= m - 1;
      if (p >= P) {
        labels.insert(owners_[p - P].label);
      } else if (r.metric[p] == 0xFFFFFFFFu) {
        u.unicastRoutesToDelete.push_back(prefixes_[p]);
      } else {
        u.unicastRoutesToUpdate.push_back(materialise(node, i, r, p));
      }
    }
  }
  if (!labels.empty()) {
    const Row o = C ? older_->fetchRow(i) : Row{};
    for (const int32_t label : labels) {
      auto ne = mplsEntry(i, r, label);
      auto oe = older_->mplsEntry(i, o, label);
      if (ne && (!oe || !(*oe == *ne))) {
        u.mplsRoutesToUpdate.push_back(std::move(*ne));
      } else if (!ne && oe) {
        u.mplsRoutesToDelete.push_back(label);
      }
    }
  }
  return u;
}

AllAreasRouteTable::AllAreasRouteTable(
    const std::unordered_map<std::string, LinkState>& areas, const PrefixState& ps,
    bool enableV4, bool computeLfa, bool bgpDryRun, bool bgpUseIgpMetric, bool prefetchAll)
    : areas_(areas),
      ps_(ps),
      enableV4_(enableV4),
      lfa_(computeLfa),
      bgpDryRun_(bgpDryRun),
      bgpIgp_(bgpUseIgpMetric) {
  // nodes of every area (hasNode, LinkState.h) -> border nodes (>= 2 areas)
  std::unordered_map<std::string, std::vector<std::string>> areasOf;
  for (const auto& [area, ls] : areas_) {
    for (const auto& [node, _] : ls.getAdjacencyDatabases()) {
      if (ls.hasNode(node)) {
        areasOf[node].push_back(area);
      }
    }
  }
  for (const auto& [node, as] : areasOf) {
    if (as.size() > 1) {
      border_.insert(node);
    } else {
      home_[node] = as.front();
    }
  }
  const bool multi = areas_.size() > 1;
  for (const auto& [area, ls] : areas_) {
    if (ls.engine().exact) {
      continue; // metric 0 / 64-bit sums: this area stays on the host path
    }
    // BGP prefixes join the device table when the selection cannot depend
    // on the node (no IGP cost in the metric vector)
    auto t = std::make_unique<AllNodesRouteTable>(ls, ps, enableV4, computeLfa,
                                                  multi ? &border_ : nullptr, !bgpUseIgpMetric &&
                                                  std::getenv("OPENR_RT_BGP_HOST") == nullptr,
                                                  bgpDryRun);
    auto& served = served_[area];
    for (const auto& p : t->prefixes()) {
      served.insert(p);
    }
    rest_[area] = served.size() < ps.prefixes().size();
    tables_[area] = std::move(t);
    if (prefetchAll) {
      // the host share then reads resident rows only (one batch per area)
      std::vector<std::string> all;
      for (const auto& [node, as] : areasOf) {
        if (std::find(as.begin(), as.end(), area) != as.end()) {
          all.push_back(node);
        }
      }
      ls.prefetchSpf(all, true);
    }
  }
}

AllAreasRouteTable::~AllAreasRouteTable() = default;

std::optional<DecisionRouteDb> AllAreasRouteTable::routeDb(const std::string& node) const {
  lastTable_ = lastHost_ = 0;
  bool known = false;
  for (const auto& [_, ls] : areas_) {
    known |= ls.hasNode(node);
  }
  if (!known) {
    return std::nullopt;
  }
  SpfSolver solver(node, enableV4_, lfa_, false, bgpDryRun_, bgpIgp_);
  const auto h = home_.find(node);
  const auto t = h == home_.end() ? tables_.end() : tables_.find(h->second);
  if (t == tables_.end()) {
    // border node (or an area the kernel does not take): the host path
    auto db = solver.buildRouteDb(node, areas_, ps_);
    if (db) {
      lastHost_ = db->unicastEntries.size() + db->mplsEntries.size();
    }
    return db;
  }
  const bool single = areas_.size() == 1;
  DecisionRouteDb db;
  db.unicastEntries = t->second->routes(node);
  if (single) {
    db.mplsEntries = t->second->mplsRoutes(node);
  }
  lastTable_ = db.unicastEntries.size() + db.mplsEntries.size();
  if (!single || rest_.at(h->second)) {
    auto part = solver.buildRouteDbPartial(node, areas_, ps_, served_.at(h->second), !single);
    if (part) {
      lastHost_ = part->unicastEntries.size() + (single ? 0 : part->mplsEntries.size());
      for (auto& [p, e] : part->unicastEntries) {
        db.unicastEntries.emplace(p, std::move(e));
      }
      if (!single) {
        db.mplsEntries = std::move(part->mplsEntries);
      }
    }
  }
  return db;
}

} // namespace openr
