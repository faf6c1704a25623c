// convert.h — Python thrift mirrors (openr_amd/thrift.py) <-> the C++ structs
// of host/Types.h, and the canonical output tuples shared by the product
// module (_openr_spf) and the oracle module (oracle/_oracle_ref).  Plumbing
// only: no SPF or RouteDb logic lives here.
#pragma once

#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <optional>
#include <string>
#include <unordered_set>

#include "../host/Types.h"

namespace py = pybind11;

namespace openr_py {

template <class T>
inline std::optional<T> optAttr(py::handle o, const char* name) {
  py::object v = o.attr(name);
  if (v.is_none()) {
    return std::nullopt;
  }
  return v.cast<T>();
}

inline std::string bytesAttr(py::handle o, const char* name) {
  py::object v = o.attr(name);
  if (py::isinstance<py::bytes>(v)) {
    return v.cast<std::string>();
  }
  return py::bytes(v).cast<std::string>();
}

inline openr::thrift::BinaryAddress toBinaryAddress(py::handle o) {
  openr::thrift::BinaryAddress a;
  a.addr = bytesAttr(o, "addr");
  a.ifName = optAttr<std::string>(o, "ifName");
  return a;
}

inline openr::thrift::IpPrefix toIpPrefix(py::handle o) {
  openr::thrift::IpPrefix p;
  p.prefixAddress = toBinaryAddress(o.attr("prefixAddress"));
  p.prefixLength = o.attr("prefixLength").cast<int16_t>();
  return p;
}

inline openr::thrift::Adjacency toAdjacency(py::handle o) {
  openr::thrift::Adjacency a;
  a.otherNodeName = o.attr("otherNodeName").cast<std::string>();
  a.ifName = o.attr("ifName").cast<std::string>();
  a.nextHopV6 = toBinaryAddress(o.attr("nextHopV6"));
  a.nextHopV4 = toBinaryAddress(o.attr("nextHopV4"));
  a.metric = o.attr("metric").cast<int32_t>();
  a.adjLabel = o.attr("adjLabel").cast<int32_t>();
  a.isOverloaded = o.attr("isOverloaded").cast<bool>();
  a.rtt = o.attr("rtt").cast<int32_t>();
  a.timestamp = o.attr("timestamp").cast<int64_t>();
  a.weight = o.attr("weight").cast<int64_t>();
  a.otherIfName = o.attr("otherIfName").cast<std::string>();
  return a;
}

inline openr::thrift::AdjacencyDatabase toAdjDb(py::handle o) {
  openr::thrift::AdjacencyDatabase db;
  db.thisNodeName = o.attr("thisNodeName").cast<std::string>();
  db.isOverloaded = o.attr("isOverloaded").cast<bool>();
  for (auto adj : o.attr("adjacencies")) {
    db.adjacencies.push_back(toAdjacency(adj));
  }
  db.nodeLabel = o.attr("nodeLabel").cast<int32_t>();
  db.area = o.attr("area").cast<std::string>();
  return db;
}

inline openr::thrift::MetricVector toMetricVector(py::handle o) {
  openr::thrift::MetricVector mv;
  mv.version = o.attr("version").cast<int64_t>();
  for (auto e : o.attr("metrics")) {
    openr::thrift::MetricEntity me;
    me.type = e.attr("type").cast<int64_t>();
    me.priority = e.attr("priority").cast<int64_t>();
    me.op = (openr::thrift::CompareType)e.attr("op").cast<int32_t>();
    me.isBestPathTieBreaker = e.attr("isBestPathTieBreaker").cast<bool>();
    me.metric = e.attr("metric").cast<std::vector<int64_t>>();
    mv.metrics.push_back(std::move(me));
  }
  return mv;
}

inline openr::thrift::PrefixEntry toPrefixEntry(py::handle o) {
  openr::thrift::PrefixEntry e;
  e.prefix = toIpPrefix(o.attr("prefix"));
  e.type = (openr::thrift::PrefixType)o.attr("type").cast<int32_t>();
  if (!o.attr("data").is_none()) {
    e.data = bytesAttr(o, "data");
  }
  e.forwardingType = (openr::thrift::PrefixForwardingType)o.attr("forwardingType").cast<int32_t>();
  e.forwardingAlgorithm =
      (openr::thrift::PrefixForwardingAlgorithm)o.attr("forwardingAlgorithm").cast<int32_t>();
  e.ephemeral = optAttr<bool>(o, "ephemeral");
  if (!o.attr("mv").is_none()) {
    e.mv = toMetricVector(o.attr("mv"));
  }
  e.minNexthop = optAttr<int64_t>(o, "minNexthop");
  e.prependLabel = optAttr<int32_t>(o, "prependLabel");
  return e;
}

inline openr::thrift::PrefixDatabase toPrefixDb(py::handle o) {
  openr::thrift::PrefixDatabase db;
  db.thisNodeName = o.attr("thisNodeName").cast<std::string>();
  for (auto e : o.attr("prefixEntries")) {
    db.prefixEntries.push_back(toPrefixEntry(e));
  }
  db.deletePrefix = o.attr("deletePrefix").cast<bool>();
  db.area = o.attr("area").cast<std::string>();
  return db;
}

inline openr::thrift::MplsAction toMplsAction(py::handle o) {
  openr::thrift::MplsAction a;
  a.action = (openr::thrift::MplsActionCode)o.attr("action").cast<int32_t>();
  a.swapLabel = optAttr<int32_t>(o, "swapLabel");
  a.pushLabels = optAttr<std::vector<int32_t>>(o, "pushLabels");
  return a;
}

inline openr::thrift::NextHopThrift toNextHop(py::handle o) {
  openr::thrift::NextHopThrift nh;
  nh.address = toBinaryAddress(o.attr("address"));
  nh.weight = o.attr("weight").cast<int32_t>();
  if (!o.attr("mplsAction").is_none()) {
    nh.mplsAction = toMplsAction(o.attr("mplsAction"));
  }
  nh.metric = o.attr("metric").cast<int32_t>();
  nh.useNonShortestRoute = o.attr("useNonShortestRoute").cast<bool>();
  nh.area = optAttr<std::string>(o, "area");
  return nh;
}

// ---- outputs: canonical tuples (see NextHopThrift.key() in thrift.py)

inline py::object optOut(const std::optional<std::string>& s) {
  return s ? py::object(py::str(*s)) : py::none();
}

inline py::tuple mplsKey(const openr::thrift::MplsAction& a) {
  return py::make_tuple(
      (int)a.action, a.swapLabel ? py::object(py::int_(*a.swapLabel)) : py::none(),
      a.pushLabels ? py::object(py::tuple(py::cast(*a.pushLabels))) : py::none());
}

inline py::tuple nextHopKey(const openr::thrift::NextHopThrift& nh) {
  return py::make_tuple(
      py::bytes(nh.address.addr), optOut(nh.address.ifName), nh.weight,
      nh.mplsAction ? py::object(mplsKey(*nh.mplsAction)) : py::none(), nh.metric,
      nh.useNonShortestRoute, optOut(nh.area));
}

inline py::tuple prefixKey(const openr::thrift::IpPrefix& p) {
  return py::make_tuple(py::bytes(p.prefixAddress.addr), p.prefixLength);
}

inline py::tuple prefixEntryKey(const openr::thrift::PrefixEntry& e) {
  py::object mv = py::none();
  if (e.mv) {
    py::list ents;
    for (const auto& me : e.mv->metrics) {
      ents.append(py::make_tuple(
          me.type, me.priority, (int)me.op, me.isBestPathTieBreaker, py::tuple(py::cast(me.metric))));
    }
    mv = py::make_tuple(e.mv->version, py::tuple(ents));
  }
  return py::make_tuple(
      prefixKey(e.prefix), (int)e.type,
      e.data ? py::object(py::bytes(*e.data)) : py::none(), (int)e.forwardingType,
      (int)e.forwardingAlgorithm, e.ephemeral ? py::object(py::bool_(*e.ephemeral)) : py::none(),
      mv, e.minNexthop ? py::object(py::int_(*e.minNexthop)) : py::none(),
      e.prependLabel ? py::object(py::int_(*e.prependLabel)) : py::none());
}

inline py::frozenset nextHopSet(const std::unordered_set<openr::thrift::NextHopThrift>& s) {
  py::set out;
  for (const auto& nh : s) {
    out.add(nextHopKey(nh));
  }
  return py::frozenset(out);
}

} // namespace openr_py
