// bindings.cpp — pybind11 surface of the C++ LinkState / SpfSolver /
// PrefixState re-implementation (module openr_amd._openr_spf).  Inputs are
// the Python thrift mirrors of openr_amd/thrift.py (read by attribute);
// outputs are canonical tuples/dicts so tests can compare against the oracle
// and the reference's known answers.

#include <pybind11/pybind11.h>

#include <chrono>
#include <pybind11/stl.h>

#include "../host/AllSourcesTable.h"
#include "../host/LinkState.h"
#include "../host/PrefixState.h"
#include "../host/Publication.h"
#include "../host/RouteTable.h"
#include "../host/SpfSolver.h"
#include "../host/Util.h"
#include "convert.h"
#include "openr_spf.h"

namespace py = pybind11;
using namespace openr;

using namespace openr_py;

namespace {

py::dict routeDbToPy(const DecisionRouteDb& db) {
  py::dict unicast, mpls;
  for (const auto& [prefix, e] : db.unicastEntries) {
    py::dict d;
    d["nexthops"] = nextHopSet(e.nexthops);
    d["bestArea"] = e.bestArea;
    d["doNotInstall"] = e.doNotInstall;
    d["bestNexthop"] = e.bestNexthop ? py::object(nextHopKey(*e.bestNexthop)) : py::none();
    d["bestPrefixEntry"] = prefixEntryKey(e.bestPrefixEntry);
    unicast[prefixKey(prefix)] = d;
  }
  for (const auto& [label, e] : db.mplsEntries) {
    mpls[py::int_(label)] = nextHopSet(e.nexthops);
  }
  py::dict out;
  out["unicast"] = unicast;
  out["mpls"] = mpls;
  return out;
}

py::tuple linkKey(const Link& l) {
  const auto& n = l.orderedNames();
  return py::make_tuple(
      py::make_tuple(n.first.first, n.first.second),
      py::make_tuple(n.second.first, n.second.second));
}

py::dict spfResultToPy(const LinkState::SpfResult& res) {
  py::dict out;
  for (const auto& [name, r] : res) {
    py::list paths;
    for (const auto& pl : r.pathLinks()) {
      paths.append(py::make_tuple(linkKey(*pl.link), pl.prevNode));
    }
    py::set nhs;
    for (const auto& h : r.nextHops()) {
      nhs.add(py::str(h));
    }
    out[py::str(name)] = py::make_tuple(r.metric(), py::frozenset(nhs), paths);
  }
  return out;
}

py::tuple changeToPy(const LinkState::LinkStateChange& c) {
  return py::make_tuple(c.topologyChanged, c.linkAttributesChanged, c.nodeLabelChanged);
}

// holder with a deleted copy so pybind11 never instantiates map copies
struct AreaMapHolder {
  std::unordered_map<std::string, LinkState> map;
  AreaMapHolder() = default;
  AreaMapHolder(const AreaMapHolder&) = delete;
};

py::object pyAddr(py::module_& T, const thrift::BinaryAddress& a) {
  return T.attr("BinaryAddress")(py::bytes(a.addr), a.ifName ? py::object(py::str(*a.ifName)) : py::none());
}

py::object pyAdjDb(const thrift::AdjacencyDatabase& db) {
  py::module_ T = py::module_::import("openr_amd.thrift");
  py::list adjs;
  for (const auto& a : db.adjacencies) {
    adjs.append(T.attr("Adjacency")(a.otherNodeName, a.ifName, pyAddr(T, a.nextHopV6),
                                    pyAddr(T, a.nextHopV4), a.metric, a.adjLabel, a.isOverloaded,
                                    a.rtt, a.timestamp, a.weight, a.otherIfName));
  }
  return T.attr("AdjacencyDatabase")(db.thisNodeName, db.isOverloaded, adjs, db.nodeLabel, db.area);
}

py::object pyPrefixDb(const thrift::PrefixDatabase& db) {
  py::module_ T = py::module_::import("openr_amd.thrift");
  py::list entries;
  for (const auto& e : db.prefixEntries) {
    py::object mv = py::none();
    if (e.mv) {
      py::list ms;
      for (const auto& me : e.mv->metrics) {
        ms.append(T.attr("MetricEntity")(me.type, me.priority, (int)me.op, me.isBestPathTieBreaker,
                                         py::cast(me.metric)));
      }
      mv = T.attr("MetricVector")(e.mv->version, ms);
    }
    entries.append(T.attr("PrefixEntry")(
        T.attr("IpPrefix")(pyAddr(T, e.prefix.prefixAddress), e.prefix.prefixLength), (int)e.type,
        e.data ? py::object(py::bytes(*e.data)) : py::none(), (int)e.forwardingType,
        (int)e.forwardingAlgorithm, e.ephemeral ? py::object(py::bool_(*e.ephemeral)) : py::none(), mv,
        e.minNexthop ? py::object(py::int_(*e.minNexthop)) : py::none(),
        e.prependLabel ? py::object(py::int_(*e.prependLabel)) : py::none()));
  }
  return T.attr("PrefixDatabase")(db.thisNodeName, entries, db.deletePrefix, db.area);
}

thrift::Publication toPublication(const std::string& area, py::dict keyVals, py::list expired) {
  thrift::Publication pub;
  pub.area = area;
  for (auto kv : keyVals) {
    thrift::Value v;
    if (!kv.second.is_none()) {
      v.value = kv.second.cast<std::string>();
    } else {
      v.ttlVersion = 1;
    }
    pub.keyVals.emplace(kv.first.cast<std::string>(), std::move(v));
  }
  for (auto k : expired) {
    pub.expiredKeys.push_back(k.cast<std::string>());
  }
  return pub;
}

py::dict pendingToPy(const PendingUpdates& p) {
  py::dict d;
  py::set prefixes;
  for (const auto& x : p.updatedPrefixes) {
    prefixes.add(prefixKey(x));
  }
  d["needsFullRebuild"] = p.needsFullRebuild;
  d["updatedPrefixes"] = prefixes;
  d["count"] = p.count;
  d["needsRouteUpdate"] = p.needsRouteUpdate();
  return d;
}

} // namespace

PYBIND11_MODULE(_openr_spf, m) {
  m.doc() = "MI355X Decision SPF engine: LinkState / SpfSolver / PrefixState";

  m.def("device_count", &spf_device_count);
  m.def("set_spf_device", &setSpfDevice);
  m.def("get_spf_device", &getSpfDevice);
  m.def("set_spf_devices", &setSpfDevices);
  m.def("set_cluster_min_sources", &setClusterMinSources);
  m.def("cluster_min_sources", &clusterMinSources);
  m.def("get_spf_devices", &getSpfDevices);
  m.def("get_counters", [] {
    py::dict d;
    for (const auto& [k, v] : Counters::snapshot()) {
      d[py::str(k)] = v;
    }
    return d;
  });
  m.def("reset_counters", &Counters::reset);
  // fb303-exported names (decision.spf_runs.count, decision.spf_ms.avg, ...)
  m.def("get_fb303_counters", [] {
    py::dict d;
    for (const auto& [k, v] : Counters::fb303Snapshot()) {
      d[py::str(k)] = v;
    }
    return d;
  });

  // HoldableValue<bool> / HoldableValue<LinkStateMetric> (LinkState.h:36-58)
  py::class_<HoldableValue<bool>>(m, "HoldableValueBool")
      .def(py::init<bool>())
      .def("value", [](const HoldableValue<bool>& h) { return h.value(); })
      .def("hasHold", &HoldableValue<bool>::hasHold)
      .def("decrementTtl", &HoldableValue<bool>::decrementTtl)
      .def("updateValue", &HoldableValue<bool>::updateValue);
  py::class_<HoldableValue<LinkStateMetric>>(m, "HoldableValueMetric")
      .def(py::init<LinkStateMetric>())
      .def("value", [](const HoldableValue<LinkStateMetric>& h) { return h.value(); })
      .def("hasHold", &HoldableValue<LinkStateMetric>::hasHold)
      .def("decrementTtl", &HoldableValue<LinkStateMetric>::decrementTtl)
      .def("updateValue", &HoldableValue<LinkStateMetric>::updateValue);

  py::class_<Link, std::shared_ptr<Link>>(m, "Link")
      .def(py::init<std::string, std::string, std::string, std::string, std::string>())
      .def_static("fromAdjacencies",
                  [](const std::string& area, const std::string& n1, py::handle a1,
                     const std::string& n2, py::handle a2) {
                    return std::make_shared<Link>(area, n1, toAdjacency(a1), n2, toAdjacency(a2));
                  })
      .def("setMetricFromNode", &Link::setMetricFromNode)
      .def("setOverloadFromNode", &Link::setOverloadFromNode)
      .def("key", [](const Link& l) { return linkKey(l); })
      .def("getArea", &Link::getArea)
      .def("getOtherNodeName", &Link::getOtherNodeName)
      .def("firstNodeName", &Link::firstNodeName)
      .def("secondNodeName", &Link::secondNodeName)
      .def("getIfaceFromNode", &Link::getIfaceFromNode)
      .def("getMetricFromNode", &Link::getMetricFromNode)
      .def("getAdjLabelFromNode", &Link::getAdjLabelFromNode)
      .def("getOverloadFromNode", &Link::getOverloadFromNode)
      .def("isUp", &Link::isUp)
      .def("hasHolds", &Link::hasHolds)
      .def("toString", &Link::toString)
      .def("directionalToString", &Link::directionalToString)
      .def_readonly("hash", &Link::hash)
      .def("__eq__", [](const Link& a, const Link& b) { return a == b; })
      .def("__lt__", [](const Link& a, const Link& b) { return a < b; })
      .def("__hash__", [](const Link& l) { return l.hash; })
      .def("__repr__", &Link::toString);

  py::class_<LinkState>(m, "LinkState")
      .def(py::init<std::string>())
      .def("getArea", &LinkState::getArea)
      .def(
          "updateAdjacencyDatabase",
          [](LinkState& ls, py::handle db, uint64_t up, uint64_t down) {
            return changeToPy(ls.updateAdjacencyDatabase(toAdjDb(db), up, down));
          },
          py::arg("adjDb"), py::arg("holdUpTtl") = 0, py::arg("holdDownTtl") = 0)
      .def("deleteAdjacencyDatabase",
           [](LinkState& ls, const std::string& n) { return changeToPy(ls.deleteAdjacencyDatabase(n)); })
      .def("decrementHolds", [](LinkState& ls) { return changeToPy(ls.decrementHolds()); })
      .def("hasHolds", &LinkState::hasHolds)
      .def("hasNode", &LinkState::hasNode)
      .def("numLinks", &LinkState::numLinks)
      .def("numNodes", &LinkState::numNodes)
      .def("isNodeOverloaded", &LinkState::isNodeOverloaded)
      .def("linksFromNode",
           [](const LinkState& ls, const std::string& n) {
             py::list out;
             for (const auto& l : ls.linksFromNode(n)) {
               out.append(py::cast(l));
             }
             return out;
           })
      .def(
          "getSpfResult",
          [](const LinkState& ls, const std::string& node, bool useLinkMetric) {
            return spfResultToPy(ls.getSpfResult(node, useLinkMetric));
          },
          py::arg("node"), py::arg("useLinkMetric") = true)
      .def(
          "runSpfBatch",
          [](const LinkState& ls, const std::string& src, py::list ignoreSets, bool useLinkMetric) {
            std::vector<LinkState::LinkSet> sets;
            for (auto lst : ignoreSets) {
              LinkState::LinkSet set;
              for (auto l : lst) {
                set.insert(l.cast<std::shared_ptr<Link>>());
              }
              sets.push_back(std::move(set));
            }
            std::unique_ptr<LinkState::SpfBatch> b;
            {
              py::gil_scoped_release rel;
              b = ls.runSpfBatch(src, sets, useLinkMetric);
            }
            return b;
          },
          py::arg("src"), py::arg("linksToIgnore"), py::arg("useLinkMetric") = true,
          py::keep_alive<0, 1>())
      .def(
          "getKthPaths",
          [](const LinkState& ls, const std::string& s, const std::string& d, size_t k) {
            py::list out;
            for (const auto& path : ls.getKthPaths(s, d, k)) {
              py::list p;
              for (const auto& l : path) {
                p.append(py::cast(l));
              }
              out.append(p);
            }
            return out;
          })
      .def("getMetricFromAToB", &LinkState::getMetricFromAToB, py::arg("a"), py::arg("b"),
           py::arg("useLinkMetric") = true)
      .def("getHopsFromAToB", &LinkState::getHopsFromAToB)
      .def("getMaxHopsToNode", &LinkState::getMaxHopsToNode)
      .def("prefetchSpf", &LinkState::prefetchSpf, py::arg("nodes"), py::arg("useLinkMetric") = true)
      .def("prefetchKthPaths", &LinkState::prefetchKthPaths)
      .def("lastDeviceMs", &LinkState::lastDeviceMs)
      .def("numGraphNodes", &LinkState::numGraphNodes)
      .def("invalidate", &LinkState::invalidate)
      .def_static("pathAInPathB", [](py::list a, py::list b) {
        LinkState::Path pa, pb;
        for (auto x : a) pa.push_back(x.cast<std::shared_ptr<Link>>());
        for (auto x : b) pb.push_back(x.cast<std::shared_ptr<Link>>());
        return LinkState::pathAInPathB(pa, pb);
      });

  py::class_<LinkState::SpfBatch>(m, "SpfBatch")
      .def("size", &LinkState::SpfBatch::size)
      .def("__len__", &LinkState::SpfBatch::size)
      .def("result", [](const LinkState::SpfBatch& b, size_t i) { return spfResultToPy(b.result(i)); })
      .def("metric", [](const LinkState::SpfBatch& b, size_t i, uint32_t nodeId) -> py::object {
        const auto& v = b.view(i);
        if (!v.reached(nodeId)) {
          return py::none();
        }
        return py::int_(v.dist[nodeId]);
      });

  // std::unordered_map<std::string, LinkState> as the reference tests build it
  py::class_<AreaMapHolder>(m, "AreaLinkStates")
      .def(py::init<>())
      .def(
          "add",
          [](AreaMapHolder& am, const std::string& area) -> LinkState& {
            return am.map.emplace(area, LinkState(area)).first->second;
          },
          py::return_value_policy::reference_internal)
      .def(
          "__getitem__",
          [](AreaMapHolder& am, const std::string& area) -> LinkState& { return am.map.at(area); },
          py::return_value_policy::reference_internal)
      .def("areas",
           [](const AreaMapHolder& am) {
             std::vector<std::string> out;
             for (const auto& kv : am.map) out.push_back(kv.first);
             return out;
           })
      .def("__len__", [](const AreaMapHolder& am) { return am.map.size(); });

  py::class_<AllAreasRouteTable>(m, "AllAreasRouteTable")
      .def(py::init([](const AreaMapHolder& areas, const PrefixState& ps, bool enableV4, bool lfa,
                       bool bgpDryRun, bool bgpUseIgpMetric, bool prefetchAll) {
             return std::make_unique<AllAreasRouteTable>(areas.map, ps, enableV4, lfa, bgpDryRun,
                                                         bgpUseIgpMetric, prefetchAll);
           }),
           py::arg("areas"), py::arg("prefix_state"), py::arg("enable_v4") = true,
           py::arg("lfa") = false, py::arg("bgp_dry_run") = false,
           py::arg("bgp_use_igp_metric") = false, py::arg("prefetch_all") = true,
           py::keep_alive<1, 2>(), py::keep_alive<1, 3>())
      .def("route_db", [](const AllAreasRouteTable& t, const std::string& node) -> py::object {
        auto db = t.routeDb(node);
        if (!db) {
          return py::none();
        }
        return routeDbToPy(*db);
      })
      .def_property_readonly("last_table_routes", &AllAreasRouteTable::lastTableRoutes)
      .def_property_readonly("last_host_routes", &AllAreasRouteTable::lastHostRoutes)
      .def_property_readonly("num_tables", &AllAreasRouteTable::numTables)
      .def_property_readonly("bgp_device_prefixes", &AllAreasRouteTable::numBgpDevicePrefixes)
      .def("is_border", &AllAreasRouteTable::isBorder);

  py::class_<AllSourcesTable>(m, "AllSourcesTable")
      .def(py::init([](const AreaMapHolder& areas, const std::string& area, std::vector<int> devices,
                       bool nexthops) {
             return std::make_unique<AllSourcesTable>(areas.map.at(area), devices, nexthops);
           }),
           py::arg("areas"), py::arg("area"), py::arg("devices") = std::vector<int>{},
           py::arg("nexthops") = false)
      .def_property_readonly("num_nodes", &AllSourcesTable::numNodes)
      .def_property_readonly("num_devices", &AllSourcesTable::numDevices)
      .def_property_readonly("node_names", &AllSourcesTable::nodeNames)
      .def_property_readonly("last_spf_ms", &AllSourcesTable::lastSpfMs)
      .def("recompute", &AllSourcesTable::recompute)
      .def("update", [](AllSourcesTable& t, const AreaMapHolder& areas, const std::string& area) {
        const auto st = t.update(areas.map.at(area));
        py::dict d;
        d["deltas"] = st.deltas;
        d["affected"] = st.affected;
        d["graph_patched"] = st.graphPatched;
        d["relaxed"] = st.relaxed;
        d["diff_ms"] = st.diffMs;
        d["graph_ms"] = st.graphMs;
        d["screen_ms"] = st.screenMs;
        d["spf_ms"] = st.spfMs;
        d["nexthops_ms"] = st.nextHopsMs;
        d["wall_ms"] = st.wallMs;
        return d;
      })
      .def("row", &AllSourcesTable::row)
      .def("distance", &AllSourcesTable::distance)
      .def("next_hops", &AllSourcesTable::nextHops)
      .def_property_readonly("has_next_hops", &AllSourcesTable::hasNextHops);

  py::class_<AllNodesRouteTable>(m, "AllNodesRouteTable")
      .def(py::init([](const AreaMapHolder& areas, const std::string& area, const PrefixState& ps,
                       bool enableV4, bool lfa) {
             return std::make_unique<AllNodesRouteTable>(areas.map.at(area), ps, enableV4, lfa);
           }),
           py::arg("areas"), py::arg("area"), py::arg("prefix_state"), py::arg("enable_v4") = true,
           py::arg("lfa") = false, py::keep_alive<1, 2>())
      .def_property_readonly("num_nodes", &AllNodesRouteTable::numNodes)
      .def_property_readonly("num_prefixes", &AllNodesRouteTable::numPrefixes)
      .def_property_readonly("spf_ms", &AllNodesRouteTable::spfMs)
      .def_property_readonly("route_ms", &AllNodesRouteTable::routeMs)
      .def("count_routes", &AllNodesRouteTable::countRoutes)
      .def("routes", [](const AllNodesRouteTable& t, const std::string& node) {
        DecisionRouteDb db;
        db.unicastEntries = t.routes(node);
        py::dict all = routeDbToPy(db);
        py::object unicast = all["unicast"]; // owned before `all` goes away
        return unicast;
      })
      .def_property_readonly("num_label_columns", &AllNodesRouteTable::numLabelColumns)
      .def("mpls_routes", [](const AllNodesRouteTable& t, const std::string& node) {
        DecisionRouteDb db;
        db.mplsEntries = t.mplsRoutes(node);
        py::dict all = routeDbToPy(db);
        py::object mpls = all["mpls"];
        return mpls;
      })
      .def("delta_mpls", [](const AllNodesRouteTable& t, const std::string& node) {
        // (updated MPLS routes as mpls_routes() renders them, deleted labels)
        const DecisionRouteUpdate u = t.delta(node);
        DecisionRouteDb db;
        for (const auto& e : u.mplsRoutesToUpdate) {
          db.mplsEntries.emplace(e.label, e);
        }
        py::dict all = routeDbToPy(db);
        py::object upd = all["mpls"];
        py::list del;
        for (int32_t l : u.mplsRoutesToDelete) {
          del.append(l);
        }
        return py::make_tuple(upd, del);
      })
      .def("diff", &AllNodesRouteTable::diff, py::arg("older"), py::keep_alive<1, 2>())
      .def("node_name", &AllNodesRouteTable::nodeName)
      .def("changed_split", &AllNodesRouteTable::changedSplit)
      .def("delta", [](const AllNodesRouteTable& t, const std::string& node) {
        // (updated unicast routes as routes() renders them, deleted prefixes)
        const DecisionRouteUpdate u = t.delta(node);
        DecisionRouteDb db;
        for (const auto& e : u.unicastRoutesToUpdate) {
          db.unicastEntries.emplace(e.prefix, e);
        }
        py::dict all = routeDbToPy(db);
        py::object upd = all["unicast"];
        py::list del;
        for (const auto& p : u.unicastRoutesToDelete) {
          del.append(prefixKey(p));
        }
        return py::make_tuple(upd, del);
      })
      .def("routes_timed", [](const AllNodesRouteTable& t, const std::string& node) {
        // fetch + materialise the node's routes in C++, no Python conversion
        const auto t0 = std::chrono::steady_clock::now();
        auto r = t.routes(node);
        const double us = std::chrono::duration<double, std::micro>(
                              std::chrono::steady_clock::now() - t0)
                              .count();
        return py::make_tuple((long)r.size(), us);
      });

  // CompactProtocol blobs and Decision::processPublication
  m.def("compact_encode_adj_db", [](py::handle db) { return py::bytes(compact::encode(toAdjDb(db))); });
  m.def(
      "compact_encode_prefix_db",
      [](py::handle db, py::object areaStacks) {
        if (areaStacks.is_none()) {
          return py::bytes(compact::encode(toPrefixDb(db)));
        }
        auto st = areaStacks.cast<std::vector<std::vector<std::string>>>();
        return py::bytes(compact::encode(toPrefixDb(db), &st));
      },
      py::arg("db"), py::arg("area_stacks") = py::none());
  m.def("compact_decode_adj_db", [](py::bytes b) {
    try {
      return pyAdjDb(compact::decodeAdjacencyDatabase(std::string(b)));
    } catch (const compact::DecodeError& e) {
      throw py::value_error(e.what());
    }
  });
  m.def("compact_decode_prefix_db", [](py::bytes b) {
    try {
      auto w = compact::decodePrefixDatabase(std::string(b));
      return py::make_tuple(pyPrefixDb(w.db), py::cast(w.areaStacks),
                            w.perPrefixKey ? py::object(py::bool_(*w.perPrefixKey)) : py::none());
    } catch (const compact::DecodeError& e) {
      throw py::value_error(e.what());
    }
  });
  m.def("parse_prefix_key", [](const std::string& key) -> py::object {
    auto k = parsePrefixKey(key);
    if (!k) {
      return py::none();
    }
    return py::make_tuple(k->node, k->area, prefixKey(k->prefix));
  });
  m.def("get_node_name_from_key", &getNodeNameFromKey);

  py::class_<PublicationIngest>(m, "PublicationIngest")
      .def(py::init<std::string, bool>(), py::arg("my_node_name"), py::arg("enable_ordered_fib") = false)
      .def(
          "processPublication",
          [](PublicationIngest& d, AreaMapHolder& areas, PrefixState& ps, const std::string& area,
             py::dict keyVals, py::list expiredKeys) {
            const auto pub = toPublication(area, keyVals, expiredKeys);
            try {
              return pendingToPy(d.processPublication(pub, areas.map, ps));
            } catch (const CheckFailure& e) {
              throw std::runtime_error(e.what());
            }
          },
          py::arg("areas"), py::arg("prefix_state"), py::arg("area"), py::arg("key_vals"),
          py::arg("expired_keys") = py::list())
      .def(
          "processPublicationTimed",
          [](PublicationIngest& d, AreaMapHolder& areas, PrefixState& ps, const std::string& area,
             py::dict keyVals, py::list expiredKeys) {
            // (count, microseconds of processPublication alone: decode + LinkState /
            // PrefixState updates, the publication already in C++ form)
            const auto pub = toPublication(area, keyVals, expiredKeys);
            const auto t0 = std::chrono::steady_clock::now();
            const auto& p = d.processPublication(pub, areas.map, ps);
            const double us = std::chrono::duration<double, std::micro>(
                                  std::chrono::steady_clock::now() - t0)
                                  .count();
            return py::make_tuple(p.count, us);
          },
          py::arg("areas"), py::arg("prefix_state"), py::arg("area"), py::arg("key_vals"),
          py::arg("expired_keys") = py::list())
      .def("pending", [](PublicationIngest& d) { return pendingToPy(d.pending()); })
      .def("resetPending", [](PublicationIngest& d) { d.pending().reset(); });

  py::class_<PrefixState>(m, "PrefixState")
      .def(py::init<>())
      .def("updatePrefixDatabase",
           [](PrefixState& ps, py::handle db) {
             py::set out;
             for (const auto& p : ps.updatePrefixDatabase(toPrefixDb(db))) {
               out.add(prefixKey(p));
             }
             return out;
           })
      .def("prefixes",
           [](const PrefixState& ps) {
             py::dict out;
             for (const auto& [p, byNode] : ps.prefixes()) {
               py::dict nodes;
               for (const auto& [node, byArea] : byNode) {
                 py::dict areas;
                 for (const auto& [area, e] : byArea) {
                   areas[py::str(area)] = prefixEntryKey(e);
                 }
                 nodes[py::str(node)] = areas;
               }
               out[prefixKey(p)] = nodes;
             }
             return out;
           })
      .def("getLoopbackVias",
           [](const PrefixState& ps, std::vector<std::string> nodes, bool isV4,
              std::optional<int64_t> igp) {
             std::unordered_set<std::string> s(nodes.begin(), nodes.end());
             py::list out;
             for (const auto& nh : ps.getLoopbackVias(s, isV4, igp)) {
               out.append(nextHopKey(nh));
             }
             return out;
           });

  py::class_<DecisionRouteDb>(m, "DecisionRouteDb")
      .def(py::init<>())
      .def("to_dict", [](const DecisionRouteDb& db) { return routeDbToPy(db); });
  // getRouteDelta (Decision.cpp:47-85) on the host RouteDbs
  // Fib's best-next-hop filters (Util.cpp:473-531): NextHopThrift objects in,
  // canonical next-hop tuples out, input order kept
  m.def("getBestNextHopsUnicast", [](py::iterable nhs) {
    std::vector<openr::thrift::NextHopThrift> v;
    for (auto nh : nhs) {
      v.push_back(toNextHop(nh));
    }
    py::list out;
    for (const auto& nh : openr::getBestNextHopsUnicast(v)) {
      out.append(nextHopKey(nh));
    }
    return out;
  });
  m.def("getBestNextHopsMpls", [](py::iterable nhs) {
    std::vector<openr::thrift::NextHopThrift> v;
    for (auto nh : nhs) {
      v.push_back(toNextHop(nh));
    }
    py::list out;
    for (const auto& nh : openr::getBestNextHopsMpls(v)) {
      out.append(nextHopKey(nh));
    }
    return out;
  });
  m.def("getRouteDelta", [](const DecisionRouteDb& newDb, const DecisionRouteDb& oldDb) {
    const DecisionRouteUpdate u = getRouteDelta(newDb, oldDb);
    DecisionRouteDb upd;
    for (const auto& e : u.unicastRoutesToUpdate) {
      upd.unicastEntries.emplace(e.prefix, e);
    }
    for (const auto& e : u.mplsRoutesToUpdate) {
      upd.mplsEntries.emplace(e.label, e);
    }
    py::dict all = routeDbToPy(upd);
    py::list udel, mdel;
    for (const auto& p : u.unicastRoutesToDelete) {
      udel.append(prefixKey(p));
    }
    for (const auto l : u.mplsRoutesToDelete) {
      mdel.append(py::int_(l));
    }
    py::dict out;
    out["unicastRoutesToUpdate"] = all["unicast"];
    out["unicastRoutesToDelete"] = udel;
    out["mplsRoutesToUpdate"] = all["mpls"];
    out["mplsRoutesToDelete"] = mdel;
    return out;
  });

  py::class_<SpfSolver>(m, "SpfSolver")
      .def(py::init<std::string, bool, bool, bool, bool, bool>(), py::arg("myNodeName"),
           py::arg("enableV4"), py::arg("computeLfaPaths"), py::arg("enableOrderedFib") = false,
           py::arg("bgpDryRun") = false, py::arg("bgpUseIgpMetric") = false)
      .def("buildRouteDb",
           [](SpfSolver& s, const std::string& node, const AreaMapHolder& areas,
              const PrefixState& ps) -> py::object {
             auto db = s.buildRouteDb(node, areas.map, ps);
             if (!db) {
               return py::none();
             }
             return routeDbToPy(*db);
           })
      .def("buildRouteDbTimed",
           [](SpfSolver& s, const std::string& node, const AreaMapHolder& areas,
              const PrefixState& ps) {
             // RouteDb build timed in C++ (no Python conversion of the
             // routes); the release of the RouteDb (Decision drops the old
             // one on every rebuild) is timed separately
             const auto t0 = std::chrono::steady_clock::now();
             auto db = s.buildRouteDb(node, areas.map, ps);
             const auto t1 = std::chrono::steady_clock::now();
             const double us = std::chrono::duration<double, std::micro>(t1 - t0).count();
             long nu = -1, nm = -1;
             if (db) {
               nu = (long)db->unicastEntries.size();
               nm = (long)db->mplsEntries.size();
             }
             if (db) {
               releaseRouteDb(std::move(*db));
             }
             db.reset();
             const double freeUs = std::chrono::duration<double, std::micro>(
                                       std::chrono::steady_clock::now() - t1)
                                       .count();
             return py::make_tuple(nu, nm, us, freeUs);
           })
      .def("buildRouteDbObject",
           [](SpfSolver& s, const std::string& node, const AreaMapHolder& areas,
              const PrefixState& ps) -> py::object {
             auto db = s.buildRouteDb(node, areas.map, ps);
             if (!db) {
               return py::none();
             }
             return py::cast(std::move(*db));
           })
      .def("staticRoutesUpdated", &SpfSolver::staticRoutesUpdated)
      .def("pushRoutesDeltaUpdates",
           [](SpfSolver& s, py::list toUpdate, std::vector<int32_t> toDelete) {
             thrift::RouteDatabaseDelta d;
             for (auto r : toUpdate) {
               thrift::MplsRoute mr;
               mr.topLabel = r.attr("topLabel").cast<int32_t>();
               for (auto nh : r.attr("nextHops")) {
                 mr.nextHops.push_back(toNextHop(nh));
               }
               d.mplsRoutesToUpdate.push_back(std::move(mr));
             }
             d.mplsRoutesToDelete = std::move(toDelete);
             s.pushRoutesDeltaUpdates(d);
           })
      .def("processStaticRouteUpdates", [](SpfSolver& s) -> py::object {
        auto u = s.processStaticRouteUpdates();
        if (!u) {
          return py::none();
        }
        py::dict upd;
        for (const auto& e : u->mplsRoutesToUpdate) {
          upd[py::int_(e.label)] = nextHopSet(e.nexthops);
        }
        return py::make_tuple(upd, py::cast(u->mplsRoutesToDelete));
      });
}
