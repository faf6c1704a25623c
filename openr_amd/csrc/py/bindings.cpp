// bindings.cpp — pybind11 surface of the C++ LinkState / SpfSolver /
// PrefixState re-implementation (module openr_amd._openr_spf).  Inputs are
// the Python thrift mirrors of openr_amd/thrift.py (read by attribute);
// outputs are canonical tuples/dicts so tests can compare against the oracle
// and the reference's known answers.

#include <pybind11/pybind11.h>

#include <chrono>
#include <pybind11/stl.h>

#include "../host/LinkState.h"
#include "../host/PrefixState.h"
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

py::tuple changeToPy(const LinkState::LinkStateChange& c) {
  return py::make_tuple(c.topologyChanged, c.linkAttributesChanged, c.nodeLabelChanged);
}

// holder with a deleted copy so pybind11 never instantiates map copies
struct AreaMapHolder {
  std::unordered_map<std::string, LinkState> map;
  AreaMapHolder() = default;
  AreaMapHolder(const AreaMapHolder&) = delete;
};

} // namespace

PYBIND11_MODULE(_openr_spf, m) {
  m.doc() = "MI355X Decision SPF engine: LinkState / SpfSolver / PrefixState";

  m.def("device_count", &spf_device_count);
  m.def("set_spf_device", &setSpfDevice);
  m.def("get_spf_device", &getSpfDevice);
  m.def("get_counters", [] {
    py::dict d;
    for (const auto& [k, v] : Counters::snapshot()) {
      d[py::str(k)] = v;
    }
    return d;
  });
  m.def("reset_counters", &Counters::reset);

  py::class_<Link, std::shared_ptr<Link>>(m, "Link")
      .def(py::init<std::string, std::string, std::string, std::string, std::string>())
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
            py::dict out;
            for (const auto& [name, r] : ls.getSpfResult(node, useLinkMetric)) {
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
          },
          py::arg("node"), py::arg("useLinkMetric") = true)
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

  py::class_<AllNodesRouteTable>(m, "AllNodesRouteTable")
      .def(py::init([](const AreaMapHolder& areas, const std::string& area, const PrefixState& ps,
                       bool enableV4) {
             return std::make_unique<AllNodesRouteTable>(areas.map.at(area), ps, enableV4);
           }),
           py::arg("areas"), py::arg("area"), py::arg("prefix_state"), py::arg("enable_v4") = true,
           py::keep_alive<1, 2>())
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
      .def("diff", &AllNodesRouteTable::diff, py::arg("older"))
      .def("node_name", &AllNodesRouteTable::nodeName)
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
