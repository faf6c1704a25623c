// LinkState.cpp — graph bookkeeping of the reference LinkState
// (openr/decision/LinkState.cpp) on top of the MI355X SPF engine.
//
// Graph maintenance (links exist only when both ends advertise each other,
// HoldableValue holds, change flags) follows the reference semantics line by
// line because its outputs are asserted by the reference tests.  Shortest
// paths come from libopenr_spf (include/openr_spf.h): the up-link graph is
// flattened once per topology version into a device CSR whose node ids are
// name ranks and whose rows list links in linksFromNode() iteration order.

#include "LinkState.h"
#include "FollyHash.h"
#include "Engine.h"

#include <atomic>
#include <chrono>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <map>
#include <mutex>
#include <shared_mutex>
#include <stdexcept>
#include <thread>

#include "Parallel.h"

#include "openr_spf.h"

namespace openr {

// ------------------------------------------------------------------ counters

namespace {
std::mutex& counterMutex() {
  static std::mutex m;
  return m;
}
std::unordered_map<std::string, int64_t>& counterMap() {
  static std::unordered_map<std::string, int64_t> m;
  return m;
}
std::unordered_map<std::string, int64_t>& sampleMap() {
  static std::unordered_map<std::string, int64_t> m;
  return m;
}
enum class ExportType { COUNT, SUM, AVG };
// the export types the reference registers (Decision.cpp:105-127)
const std::unordered_map<std::string, ExportType>& exportTypes() {
  static const std::unordered_map<std::string, ExportType> m = {
      {"decision.adj_db_update", ExportType::COUNT},
      {"decision.incompatible_forwarding_type", ExportType::COUNT},
      {"decision.missing_loopback_addr", ExportType::SUM},
      {"decision.no_route_to_label", ExportType::COUNT},
      {"decision.no_route_to_prefix", ExportType::COUNT},
      {"decision.path_build_ms", ExportType::AVG},
      {"decision.prefix_db_update", ExportType::COUNT},
      {"decision.route_build_ms", ExportType::AVG},
      {"decision.route_build_runs", ExportType::COUNT},
      {"decision.skipped_mpls_route", ExportType::COUNT},
      {"decision.duplicate_node_label", ExportType::COUNT},
      {"decision.skipped_unicast_route", ExportType::COUNT},
      {"decision.spf_ms", ExportType::AVG},
      {"decision.spf_runs", ExportType::COUNT},
      {"decision.errors", ExportType::COUNT},
  };
  return m;
}
int& spfDevice() {
  static int d = 0;
  return d;
}
} // namespace

void Counters::add(const std::string& key, int64_t v) {
  std::lock_guard<std::mutex> g(counterMutex());
  counterMap()[key] += v;
  ++sampleMap()[key];
}
void Counters::addSamples(const std::string& key, int64_t sum, int64_t samples) {
  std::lock_guard<std::mutex> g(counterMutex());
  counterMap()[key] += sum;
  sampleMap()[key] += samples;
}
int64_t Counters::samples(const std::string& key) {
  std::lock_guard<std::mutex> g(counterMutex());
  auto it = sampleMap().find(key);
  return it == sampleMap().end() ? 0 : it->second;
}
std::unordered_map<std::string, int64_t> Counters::fb303Snapshot() {
  std::lock_guard<std::mutex> g(counterMutex());
  std::unordered_map<std::string, int64_t> out;
  for (const auto& [key, sum] : counterMap()) {
    auto t = exportTypes().find(key);
    if (t == exportTypes().end()) {
      continue; // engine-internal timing keys are not fb303 stats
    }
    const int64_t n = sampleMap()[key];
    const char* suffix = t->second == ExportType::COUNT ? ".count"
        : t->second == ExportType::SUM                  ? ".sum"
                                                         : ".avg";
    const int64_t value = t->second == ExportType::COUNT ? n
        : t->second == ExportType::SUM                   ? sum
                                                         : (n ? sum / n : 0);
    for (const char* window : {"", ".60", ".600", ".3600"}) {
      out[key + suffix + window] = value;
    }
  }
  return out;
}
int64_t Counters::get(const std::string& key) {
  std::lock_guard<std::mutex> g(counterMutex());
  auto it = counterMap().find(key);
  return it == counterMap().end() ? 0 : it->second;
}
std::unordered_map<std::string, int64_t> Counters::snapshot() {
  std::lock_guard<std::mutex> g(counterMutex());
  return counterMap();
}
void Counters::reset() {
  std::lock_guard<std::mutex> g(counterMutex());
  counterMap().clear();
  sampleMap().clear();
}

void setSpfDevice(int device) { spfDevice() = device; }
int getSpfDevice() { return spfDevice(); }

namespace {
struct ClusterState {
  std::mutex mu;
  std::vector<int> devices;
  // not destroyed at process exit: RCCL / HIP teardown from a static
  // destructor can run after the runtime's own exit handlers
  spf_cluster* cluster{nullptr};
  // bumped whenever the device set changes: an Engine's cluster graph of an
  // older generation is rebuilt for the new devices
  uint64_t gen{1};
};
ClusterState& clusterState() {
  static ClusterState s;
  return s;
}
} // namespace

void setSpfDevices(const std::vector<int>& devices) {
  auto& cs = clusterState();
  std::lock_guard<std::mutex> g(cs.mu);
  if (cs.devices == devices) {
    return;
  }
  if (cs.cluster) {
    spf_cluster_destroy(cs.cluster);
    cs.cluster = nullptr;
  }
  cs.devices = devices;
  ++cs.gen;
}

namespace {
std::atomic<size_t>& clusterMin() {
  static std::atomic<size_t> n{kClusterMinSources};
  return n;
}
} // namespace
void setClusterMinSources(size_t n) { clusterMin().store(std::max<size_t>(1, n)); }
size_t clusterMinSources() { return clusterMin().load(); }

std::vector<int> getSpfDevices() {
  auto& cs = clusterState();
  std::lock_guard<std::mutex> g(cs.mu);
  return cs.devices;
}

// --------------------------------------------------------------- hashing

namespace {
// Link::hash = folly's std::hash<pair<pair<string,string>, pair<string,string>>>
// (FollyHash.h): it feeds Link::operator< and the bucket order of every
// LinkSet, and that order picks the parallel link a KSP2 trace takes
// (DecisionTest.cpp:3276-3279, 3694-3696, 3726-3727).
using follyhash::hash128to64;
inline size_t hashStrPair(const std::pair<std::string, std::string>& p) {
  return follyhash::hashStringPair(p);
}
} // namespace

size_t LinkState::KthKeyHash::operator()(const KthKey& key) const {
  return hash128to64(
      hash128to64(std::hash<std::string>()(key.src), std::hash<std::string>()(key.dst)),
      key.k);
}

// ---------------------------------------------------------- HoldableValue

template <class T>
HoldableValue<T>::HoldableValue(T val) : val_(val) {}

template <class T>
void HoldableValue<T>::operator=(T val) {
  val_ = val;
  heldVal_.reset();
  holdTtl_ = 0;
}

template <class T>
const T& HoldableValue<T>::value() const {
  if (heldVal_) {
    return *heldVal_;
  }
  return val_;
}

template <class T>
bool HoldableValue<T>::hasHold() const {
  return heldVal_.has_value();
}

template <class T>
bool HoldableValue<T>::decrementTtl() {
  if (!heldVal_) {
    return false;
  }
  if (--holdTtl_ != 0) {
    return false;
  }
  heldVal_.reset();
  return true;
}

template <class T>
bool HoldableValue<T>::updateValue(
    T val, LinkStateMetric holdUpTtl, LinkStateMetric holdDownTtl) {
  if (val == val_) {
    return false; // same value: no-op
  }
  if (heldVal_) {
    // a second change while holding falls back to an immediate update
    heldVal_.reset();
    holdTtl_ = 0;
  } else {
    holdTtl_ = isChangeBringingUp(val) ? holdUpTtl : holdDownTtl;
    if (holdTtl_ != 0) {
      heldVal_ = val_;
    }
  }
  val_ = val;
  return !heldVal_.has_value();
}

template <>
bool HoldableValue<bool>::isChangeBringingUp(bool val) {
  // clearing an overload brings the element up
  return val_ && !val;
}

template <>
bool HoldableValue<LinkStateMetric>::isChangeBringingUp(LinkStateMetric val) {
  // a metric decrease attracts traffic
  return val < val_;
}

template class HoldableValue<LinkStateMetric>;
template class HoldableValue<bool>;

// --------------------------------------------------------------------- Link

Link::Link(
    const std::string& area,
    const std::string& nodeName1,
    const std::string& if1,
    const std::string& nodeName2,
    const std::string& if2)
    : area_(area),
      n1_(nodeName1),
      n2_(nodeName2),
      if1_(if1),
      if2_(if2),
      orderedNames_(std::minmax(std::make_pair(n1_, if1_), std::make_pair(n2_, if2_))),
      hash(hash128to64(hashStrPair(orderedNames_.first), hashStrPair(orderedNames_.second))) {}

Link::Link(
    const std::string& area,
    const std::string& nodeName1,
    const thrift::Adjacency& adj1,
    const std::string& nodeName2,
    const thrift::Adjacency& adj2)
    : Link(area, nodeName1, adj1.ifName, nodeName2, adj2.ifName) {
  // an i32 metric widens to the uint64 LinkStateMetric (negative -> huge)
  metric1_ = static_cast<LinkStateMetric>(static_cast<int64_t>(adj1.metric));
  metric2_ = static_cast<LinkStateMetric>(static_cast<int64_t>(adj2.metric));
  overload1_ = adj1.isOverloaded;
  overload2_ = adj2.isOverloaded;
  adjLabel1_ = adj1.adjLabel;
  adjLabel2_ = adj2.adjLabel;
  nhV41_ = adj1.nextHopV4;
  nhV42_ = adj2.nextHopV4;
  nhV61_ = adj1.nextHopV6;
  nhV62_ = adj2.nextHopV6;
}

namespace {
[[noreturn]] void badNode(const std::string& nodeName) {
  throw std::invalid_argument(nodeName);
}
} // namespace

#define LINK_SIDE(nodeName, a, b) \
  ((nodeName) == n1_ ? (a) : ((nodeName) == n2_ ? (b) : (badNode(nodeName), (a))))

const std::string& Link::getOtherNodeName(const std::string& nodeName) const {
  return LINK_SIDE(nodeName, n2_, n1_);
}
const std::string& Link::firstNodeName() const { return orderedNames_.first.first; }
const std::string& Link::secondNodeName() const { return orderedNames_.second.first; }
const std::string& Link::getIfaceFromNode(const std::string& nodeName) const {
  return LINK_SIDE(nodeName, if1_, if2_);
}
LinkStateMetric Link::getMetricFromNode(const std::string& nodeName) const {
  return LINK_SIDE(nodeName, metric1_, metric2_).value();
}
int32_t Link::getAdjLabelFromNode(const std::string& nodeName) const {
  return LINK_SIDE(nodeName, adjLabel1_, adjLabel2_);
}
bool Link::getOverloadFromNode(const std::string& nodeName) const {
  return LINK_SIDE(nodeName, overload1_, overload2_).value();
}
const thrift::BinaryAddress& Link::getNhV4FromNode(const std::string& nodeName) const {
  return LINK_SIDE(nodeName, nhV41_, nhV42_);
}
const thrift::BinaryAddress& Link::getNhV6FromNode(const std::string& nodeName) const {
  return LINK_SIDE(nodeName, nhV61_, nhV62_);
}
void Link::setNhV4FromNode(const std::string& nodeName, const thrift::BinaryAddress& nhV4) {
  LINK_SIDE(nodeName, nhV41_, nhV42_) = nhV4;
}
void Link::setNhV6FromNode(const std::string& nodeName, const thrift::BinaryAddress& nhV6) {
  LINK_SIDE(nodeName, nhV61_, nhV62_) = nhV6;
}
bool Link::setMetricFromNode(
    const std::string& nodeName,
    LinkStateMetric d,
    LinkStateMetric holdUpTtl,
    LinkStateMetric holdDownTtl) {
  return LINK_SIDE(nodeName, metric1_, metric2_).updateValue(d, holdUpTtl, holdDownTtl);
}
void Link::setAdjLabelFromNode(const std::string& nodeName, int32_t adjLabel) {
  LINK_SIDE(nodeName, adjLabel1_, adjLabel2_) = adjLabel;
}
bool Link::setOverloadFromNode(
    const std::string& nodeName,
    bool overload,
    LinkStateMetric holdUpTtl,
    LinkStateMetric holdDownTtl) {
  const bool upBefore = isUp();
  LINK_SIDE(nodeName, overload1_, overload2_).updateValue(overload, holdUpTtl, holdDownTtl);
  // only a change of isUp() is a topology change (no simplex overloads)
  return upBefore != isUp();
}
#undef LINK_SIDE

void Link::setHoldUpTtl(LinkStateMetric ttl) { holdUpTtl_ = ttl; }

bool Link::isUp() const {
  return holdUpTtl_ == 0 && !overload1_.value() && !overload2_.value();
}

bool Link::decrementHolds() {
  bool expired = false;
  if (holdUpTtl_ != 0) {
    --holdUpTtl_;
    expired |= holdUpTtl_ == 0;
  }
  expired |= metric1_.decrementTtl();
  expired |= metric2_.decrementTtl();
  expired |= overload1_.decrementTtl();
  expired |= overload2_.decrementTtl();
  return expired;
}

bool Link::hasHolds() const {
  return holdUpTtl_ != 0 || metric1_.hasHold() || metric2_.hasHold() ||
      overload1_.hasHold() || overload2_.hasHold();
}

bool Link::operator<(const Link& other) const {
  // hash first, then names (LinkState.cpp:347-353)
  if (hash != other.hash) {
    return hash < other.hash;
  }
  return orderedNames_ < other.orderedNames_;
}

bool Link::operator==(const Link& other) const {
  return hash == other.hash && orderedNames_ == other.orderedNames_;
}

std::string Link::toString() const {
  return area_ + " - " + n1_ + "%" + if1_ + " <---> " + n2_ + "%" + if2_;
}

std::string Link::directionalToString(const std::string& fromNode) const {
  const auto& to = getOtherNodeName(fromNode);
  return area_ + " - " + fromNode + "%" + getIfaceFromNode(fromNode) + " ---> " +
      to + "%" + getIfaceFromNode(to);
}

// ------------------------------------------------------------------ engine

// struct LinkState::Engine: Engine.h (shared with RouteTable.cpp)

namespace {

[[noreturn]] void engineFailure(const char* what, int status) {
  throw std::runtime_error(
      std::string("openr_spf: ") + what + ": " + spf_error_string(status) + " (" +
      spf_last_error_detail() + ")");
}

// Flatten the up links into the device CSR.  Rows follow linksFromNode()
// iteration order (the reference's relaxation order).
void buildGraph(
    LinkState::Engine& eng,
    const std::unordered_map<std::string, LinkState::LinkSet>& linkMap,
    const std::unordered_map<std::string, thrift::AdjacencyDatabase>& adjDbs,
    const LinkState& ls) {
  eng.names.clear();
  eng.names.reserve(adjDbs.size() + linkMap.size());
  for (const auto& kv : adjDbs) {
    eng.names.push_back(kv.first);
  }
  for (const auto& kv : linkMap) {
    if (!adjDbs.count(kv.first)) {
      eng.names.push_back(kv.first);
    }
  }
  std::sort(eng.names.begin(), eng.names.end());
  const uint32_t V = (uint32_t)eng.names.size();
  eng.ids.clear();
  eng.ids.reserve(V * 2);
  for (uint32_t i = 0; i < V; ++i) {
    eng.ids.emplace(eng.names[i], i);
  }
  eng.row.assign(V + 1, 0);
  eng.col.clear();
  eng.linkId.clear();
  eng.metric.clear();
  eng.links.clear();
  eng.overloaded.assign(V, 0);
  // half-edge slots per link: [0] = from firstNodeName, [1] = from second
  auto& halves = eng.halves;
  halves.clear();
  // Link ids without hashing, on the host pool.  Ids are name ranks, so a
  // link's side-0 half (from firstNodeName, the smaller name) is the one met
  // first in row order: link ids number the side-0 halves in CSR order (the
  // order a serial walk would give).  Pass A counts each row's up links and
  // side-0 halves, pass B fills the rows and tags each link with its id
  // (Link::engineEpoch / engineId, per build), pass C completes the side-1
  // halves from the tags: each half's other endpoint is the node holding the
  // other half, so no name -> id lookup per half-edge.
  static std::atomic<uint64_t> epochs{0};
  const uint64_t epoch = eng.epoch = ++epochs;
  const unsigned nt = hostThreads(V, 256);
  std::vector<const LinkState::LinkSet*> sets(V, nullptr);
  std::vector<uint32_t> firstBase(V + 1, 0);
  parallelFor(V, nt, [&](size_t u, unsigned) {
    const std::string& name = eng.names[u];
    eng.overloaded[u] = ls.isNodeOverloaded(name) ? 1 : 0;
    auto it = linkMap.find(name);
    if (it == linkMap.end()) {
      return;
    }
    sets[u] = &it->second;
    uint32_t d = 0, f = 0;
    for (const auto& link : it->second) {
      if (link->isUp()) {
        ++d;
        f += name == link->firstNodeName() ? 1u : 0u;
      }
    }
    eng.row[u + 1] = d;
    firstBase[u + 1] = f;
  }, 64);
  for (uint32_t u = 0; u < V; ++u) {
    eng.row[u + 1] += eng.row[u];
    firstBase[u + 1] += firstBase[u];
  }
  const uint32_t E0 = eng.row[V], L0 = firstBase[V];
  eng.col.assign(E0, ~0u);
  eng.linkId.assign(E0, ~0u);
  eng.metric.assign(E0, 0);
  eng.links.assign(L0, nullptr);
  halves.assign(L0, {~0u, ~0u});
  std::vector<uint32_t> firstNode(L0);
  std::vector<const std::shared_ptr<Link>*> halfLink(E0); // the row's set element
  parallelFor(V, nt, [&](size_t u, unsigned) {
    if (!sets[u]) {
      return;
    }
    const std::string& name = eng.names[u];
    uint32_t e = eng.row[u], lid = firstBase[u];
    for (const auto& link : *sets[u]) {
      if (!link->isUp()) {
        continue;
      }
      eng.metric[e] = link->getMetricFromNode(name);
      halfLink[e] = &link;
      if (name == link->firstNodeName()) {
        link->engineEpoch = epoch;
        link->engineId = lid;
        eng.links[lid] = link;
        halves[lid][0] = e;
        firstNode[lid] = (uint32_t)u;
        eng.linkId[e] = lid++;
      }
      ++e;
    }
  }, 64);
  parallelFor(V, nt, [&](size_t u, unsigned) {
    for (uint32_t e = eng.row[u]; e < eng.row[u + 1]; ++e) {
      const Link* link = halfLink[e]->get();
      if (eng.linkId[e] != ~0u || link->engineEpoch != epoch) {
        continue; // side 0, or a link its side-0 endpoint does not list
      }
      const uint32_t lid = link->engineId;
      eng.linkId[e] = lid;
      eng.col[e] = firstNode[lid];
      halves[lid][1] = e;
      eng.col[halves[lid][0]] = (uint32_t)u;
    }
  }, 64);
  // halves the passes could not pair (not expected: linkMap lists every
  // link under both endpoints) resolve by name
  for (uint32_t u = 0; u < V; ++u) {
    for (uint32_t e = eng.row[u]; e < eng.row[u + 1]; ++e) {
      const std::shared_ptr<Link>& link = *halfLink[e];
      if (eng.linkId[e] == ~0u) {
        const uint32_t lid = (uint32_t)eng.links.size();
        link->engineEpoch = epoch;
        link->engineId = lid;
        eng.links.push_back(link);
        halves.push_back({~0u, ~0u});
        halves[lid][eng.names[u] == link->firstNodeName() ? 0 : 1] = e;
        eng.linkId[e] = lid;
      }
      if (eng.col[e] == ~0u) {
        eng.col[e] = eng.ids.at(link->getOtherNodeName(eng.names[u]));
      }
    }
  }
  const uint32_t E = (uint32_t)eng.col.size();
  eng.rev.assign(E, 0);
  for (uint32_t e = 0; e < E; ++e) {
    const auto& h = halves[eng.linkId[e]];
    eng.rev[e] = h[0] == e ? h[1] : h[0];
  }
  spf_graph_desc d{};
  d.num_nodes = V;
  d.num_edges = E;
  d.row_ptr = eng.row.data();
  d.col = eng.col.data();
  d.metric = eng.metric.data();
  d.link_id = eng.linkId.data();
  d.rev = eng.rev.data();
  d.node_overloaded = eng.overloaded.data();
  d.num_links = (uint32_t)eng.links.size();
  d.device = getSpfDevice();
  eng.retireGraph(); // (refused while a query over it lives: kept, freed later)
  if (V > 0) {
    const auto tc = std::chrono::steady_clock::now();
    const int s = spf_graph_create(&d, &eng.graph);
    Counters::add(
        "decision.graph_upload_us",
        std::chrono::duration_cast<std::chrono::microseconds>(
            std::chrono::steady_clock::now() - tc)
            .count());
    if (s != SPF_OK) {
      engineFailure("spf_graph_create", s);
    }
    eng.exact = spf_graph_needs_exact(eng.graph) != 0;
  }
  eng.built = true;
}

// One device batch; returns one SpfView per source.
std::vector<std::unique_ptr<SpfView>> runBatch(
    LinkState::Engine& eng,
    const std::vector<uint32_t>& sources,
    bool useLinkMetric,
    bool wantNextHops,
    const std::vector<std::vector<uint32_t>>* ignore) {
  std::vector<std::unique_ptr<SpfView>> out;
  if (sources.empty()) {
    return out;
  }
  const auto tBatch = std::chrono::steady_clock::now();
  struct BatchTimer {
    std::chrono::steady_clock::time_point t0;
    ~BatchTimer() {
      Counters::add(
          "decision.spf_batch_us",
          std::chrono::duration_cast<std::chrono::microseconds>(
              std::chrono::steady_clock::now() - t0)
              .count());
    }
  } batchTimer{tBatch};
  const bool exact = eng.exact && useLinkMetric;
  uint32_t flags = 0;
  if (!useLinkMetric) {
    flags |= SPF_F_UNIT_METRIC;
  }
  if (wantNextHops) {
    flags |= SPF_F_NEXTHOPS;
  }
  if (exact) {
    flags |= SPF_F_ORDER;
  }
  std::vector<uint32_t> ioff, ilinks;
  spf_query_desc qd{};
  qd.num_queries = (uint32_t)sources.size();
  qd.sources = sources.data();
  qd.flags = flags;
  if (ignore) {
    ioff.push_back(0);
    for (const auto& l : *ignore) {
      ilinks.insert(ilinks.end(), l.begin(), l.end());
      ioff.push_back((uint32_t)ilinks.size());
    }
    qd.ignore_offsets = ioff.data();
    qd.ignore_links = ilinks.data();
  }
  const char* cacheEnv = std::getenv("OPENR_LS_QUERY_CACHE"); // (read per batch: A/B)
  const bool cacheQuery = !(cacheEnv && std::atoi(cacheEnv) == 0);
  // (small areas only: on the fabric the reuse bought nothing on the RouteDb
  // loops and cost 4-6 ms on the KSP2 loop, A/B/A/B on one box, r06aw)
  const bool reuse = cacheQuery && !ignore && eng.names.size() <= 4096;
  spf_query* q = nullptr;
  int s = SPF_OK;
  if (reuse && eng.lastQuery && eng.lastFlags == flags && eng.lastSources == sources) {
    q = eng.lastQuery;
    Counters::add("decision.spf_query_reuses", 1);
  } else {
    if (reuse) {
      eng.dropQuery();
    }
    if ((s = spf_query_create(eng.graph, &qd, &q)) != SPF_OK) {
      engineFailure("spf_query_create", s);
    }
  }
  // a cached query outlives the batch; any other is destroyed on return
  struct Guard {
    spf_query* q;
    ~Guard() {
      if (q) {
        spf_query_destroy(q);
      }
    }
  } guard{reuse ? nullptr : q};
  if (reuse && !eng.lastQuery) {
    eng.lastQuery = q;
    eng.lastSources = sources;
    eng.lastFlags = flags;
  }
  if ((s = spf_query_run(q)) != SPF_OK || (s = spf_query_sync(q)) != SPF_OK) {
    if (q == eng.lastQuery) {
      eng.dropQuery();
    }
    engineFailure("spf_query_run", s);
  }
  spf_query_elapsed_ms(q, &eng.lastMs);
  Counters::add("decision.spf_device_us", (int64_t)(eng.lastMs * 1000.0f));
  {
    // decision.spf_ms (LinkState.cpp:875-878): one AVG sample of whole
    // milliseconds per SPF; a batch's SPFs share its wall time
    const double batchMs = std::chrono::duration<double, std::milli>(
                               std::chrono::steady_clock::now() - tBatch)
                               .count();
    const int64_t perSpf = (int64_t)(batchMs / (double)sources.size());
    for (size_t i = 0; i < sources.size(); ++i) {
      Counters::add("decision.spf_ms", perSpf);
    }
  }
  const uint32_t V = (uint32_t)eng.names.size();
  const uint32_t nq = (uint32_t)sources.size();
  out.resize(nq);
  // 32-bit rows (every fast plan) and next-hop masks come back in one
  // transfer each; the per-view expansion runs on the host worker pool
  std::shared_ptr<std::vector<uint32_t>> rows32;
  std::vector<uint64_t> masks;
  std::vector<uint64_t> maskOff(nq + 1, 0);
  std::vector<uint32_t> words(nq, 1);
  if (!exact && nq > 1) {
    const size_t need = (size_t)nq * V;
    if (eng.rowBlock && eng.rowBlock.use_count() == 1 && eng.rowBlock->size() >= need) {
      rows32 = eng.rowBlock; // no live view reads it: overwrite in place
    } else {
      rows32 = std::make_shared<std::vector<uint32_t>>(need);
      if (!eng.rowBlock || eng.rowBlock.use_count() > 1 || eng.rowBlock->size() < need) {
        eng.rowBlock = rows32;
      }
    }
  }
  if (wantNextHops) {
    for (uint32_t i = 0; i < nq; ++i) {
      words[i] = (uint32_t)spf_query_nh_words(q, i);
      maskOff[i + 1] = maskOff[i] + (uint64_t)V * words[i];
    }
    if (nq > 1) {
      masks.resize(maskOff[nq]);
    }
  }
  // rows and masks in one call: one synchronisation for both transfers
  if (rows32 || !masks.empty()) {
    if ((s = spf_query_fetch_host(q, 0, nq, rows32 ? rows32->data() : nullptr, (size_t)V * 4,
                                  masks.empty() ? nullptr : masks.data())) != SPF_OK) {
      engineFailure("spf_query_fetch_host", s);
    }
  }
  auto fill = [&](size_t i, unsigned) {
    auto view = std::make_unique<SpfView>();
    view->src = sources[i];
    view->useLinkMetric = useLinkMetric;
    view->exact = exact;
    if (rows32) {
      view->dist.share32(rows32, i * V, V);
    } else if (int st = spf_query_dist(q, (uint32_t)i, view->dist.resize64(V)); st != SPF_OK) {
      engineFailure("spf_query_dist", st);
    }
    if (wantNextHops) {
      view->words = words[i];
      if (!masks.empty()) {
        view->nh.assign(masks.begin() + maskOff[i], masks.begin() + maskOff[i + 1]);
      } else {
        view->nh.resize((size_t)V * view->words);
        if (int st = spf_query_nexthops(q, (uint32_t)i, view->nh.data()); st != SPF_OK) {
          engineFailure("spf_query_nexthops", st);
        }
      }
      const int nn = spf_graph_num_nbrs(eng.graph, sources[i]);
      view->nbrs.resize(std::max(nn, 0));
      if (nn > 0) {
        spf_graph_nbrs(eng.graph, sources[i], view->nbrs.data());
      }
    }
    if (exact) {
      // wide plan: compare (dist, key); literal replay: settle ranks
      view->okey.resize(V);
      int st = spf_query_order_keys(q, (uint32_t)i, view->okey.data());
      if (st == SPF_E_UNSUPPORTED) {
        view->okey.clear();
        view->order.resize(V);
        st = spf_query_order(q, (uint32_t)i, view->order.data());
      }
      if (st != SPF_OK) {
        engineFailure("spf_query_order", st);
      }
    }
    if (ignore) {
      view->ignored = (*ignore)[i];
    }
    out[i] = std::move(view);
  };
  // the single-row reads of the exact plan go through the ABI (one thread)
  parallelFor(nq, exact ? 1u : hostThreads(nq, 32), fill, 8);
  return out;
}

// The multi-GPU fan-out of one batch (setSpfDevices): the queries are split
// over the cluster's devices in one spf_table run over the engine's
// persistent cluster graph (one upload per device per topology, patched in
// place by patchMemo), each block with its slice of the ignore lists, and
// every block comes back to the host from the device that computed it.  Same
// views as runBatch (32-bit rows shared from one block, next-hop masks).
// Returns no views when a block's plan keeps 64-bit rows (a source with more
// than 1,024 neighbours, SPF_E_UNSUPPORTED from the row fetch): the caller
// runs the batch on its single device instead.
std::vector<std::unique_ptr<SpfView>> runBatchCluster(
    LinkState::Engine& eng, const std::vector<uint32_t>& sources, bool useLinkMetric,
    bool wantNextHops, const std::vector<std::vector<uint32_t>>* ignore) {
  const auto tBatch = std::chrono::steady_clock::now();
  auto& cs = clusterState();
  std::lock_guard<std::mutex> g(cs.mu);
  if (!cs.cluster) {
    const int s = spf_cluster_create_local(
        (uint32_t)cs.devices.size(), cs.devices.data(), &cs.cluster);
    if (s != SPF_OK) {
      throw std::runtime_error(
          std::string("MI355X SPF engine failure in spf_cluster_create_local: ") +
          spf_error_string(s) + " (" + spf_cluster_last_error() + ")");
    }
  }
  const uint32_t V = (uint32_t)eng.names.size();
  const uint32_t nq = (uint32_t)sources.size();
  spf_table* t = nullptr;
  auto check = [&](int s, const char* what) {
    if (s != SPF_OK) {
      if (t) {
        spf_table_destroy(t);
      }
      throw std::runtime_error(
          std::string("MI355X SPF engine failure in ") + what + ": " + spf_error_string(s) +
          " (" + spf_cluster_last_error() + " / " + spf_last_error_detail() + ")");
    }
  };
  if (eng.cgraph && eng.cgraphGen != cs.gen) {
    spf_cgraph_destroy(eng.cgraph); // built for another device set
    eng.cgraph = nullptr;
  }
  if (!eng.cgraph) {
    spf_graph_desc d{};
    d.num_nodes = V;
    d.num_edges = (uint32_t)eng.col.size();
    d.row_ptr = eng.row.data();
    d.col = eng.col.data();
    d.metric = eng.metric.data();
    d.link_id = eng.linkId.data();
    d.rev = eng.rev.data();
    d.node_overloaded = eng.overloaded.data();
    d.num_links = (uint32_t)eng.links.size();
    const auto tc = std::chrono::steady_clock::now();
    check(spf_cgraph_create(cs.cluster, &d, &eng.cgraph), "spf_cgraph_create");
    eng.cgraphGen = cs.gen;
    Counters::add("decision.cluster_graph_uploads", 1);
    Counters::add("decision.cluster_graph_upload_us",
                  std::chrono::duration_cast<std::chrono::microseconds>(
                      std::chrono::steady_clock::now() - tc)
                      .count());
  }
  std::vector<uint32_t> ioff, ilinks;
  spf_query_desc qd{};
  qd.num_queries = nq;
  qd.sources = sources.data();
  qd.flags = (wantNextHops ? SPF_F_NEXTHOPS : 0u) | (useLinkMetric ? 0u : SPF_F_UNIT_METRIC);
  if (ignore) {
    ioff.push_back(0);
    for (const auto& l : *ignore) {
      ilinks.insert(ilinks.end(), l.begin(), l.end());
      ioff.push_back((uint32_t)ilinks.size());
    }
    qd.ignore_offsets = ioff.data();
    qd.ignore_links = ilinks.data();
  }
  check(spf_table_create_q(eng.cgraph, &qd, 0, &t), "spf_table_create_q");
  check(spf_table_run(t), "spf_table_run");
  check(spf_table_sync(t), "spf_table_sync");
  float cm = 0, gm = 0;
  check(spf_table_elapsed_ms(t, &cm, &gm), "spf_table_elapsed_ms");
  auto rows32 = std::make_shared<std::vector<uint32_t>>((size_t)nq * V);
  if (const int s = spf_table_fetch_rows(t, 0, nq, rows32->data()); s == SPF_E_UNSUPPORTED) {
    // 64-bit rows in some block: the caller's single-device path runs the
    // batch again and charges its own device time (not this run's)
    spf_table_destroy(t);
    Counters::add("decision.spf_cluster_fallbacks", 1);
    return {};
  } else {
    check(s, "spf_table_fetch_rows");
  }
  eng.lastMs = cm + gm;
  Counters::add("decision.spf_device_us", (int64_t)(eng.lastMs * 1000.0f));
  Counters::add("decision.spf_cluster_batches", 1);
  std::vector<uint32_t> words(nq, 1);
  std::vector<uint64_t> maskOff(nq + 1, 0);
  std::vector<uint64_t> masks;
  if (wantNextHops) {
    for (uint32_t i = 0; i < nq; ++i) {
      words[i] = (uint32_t)spf_table_nh_words(t, i);
      maskOff[i + 1] = maskOff[i] + (uint64_t)V * words[i];
    }
    masks.resize(maskOff[nq]);
    check(spf_table_fetch_nexthops(t, 0, nq, masks.data()), "spf_table_fetch_nexthops");
  }
  spf_table_destroy(t);
  t = nullptr;
  std::vector<std::unique_ptr<SpfView>> out(nq);
  parallelFor(nq, hostThreads(nq, 32), [&](size_t i, unsigned) {
    auto view = std::make_unique<SpfView>();
    view->src = sources[i];
    view->useLinkMetric = useLinkMetric;
    view->dist.share32(rows32, i * V, V);
    if (wantNextHops) {
      view->words = words[i];
      view->nh.assign(masks.begin() + maskOff[i], masks.begin() + maskOff[i + 1]);
      const int nn = spf_graph_num_nbrs(eng.graph, sources[i]);
      view->nbrs.resize(std::max(nn, 0));
      if (nn > 0) {
        spf_graph_nbrs(eng.graph, sources[i], view->nbrs.data());
      }
    }
    if (ignore) {
      view->ignored = (*ignore)[i];
    }
    out[i] = std::move(view);
  }, 8);
  const double batchMs = std::chrono::duration<double, std::milli>(
                             std::chrono::steady_clock::now() - tBatch)
                             .count();
  Counters::add("decision.spf_batch_us", (int64_t)(batchMs * 1000.0));
  for (uint32_t i = 0; i < nq; ++i) {
    Counters::add("decision.spf_ms", (int64_t)(batchMs / (double)nq));
  }
  return out;
}

// One device batch on the fan-out devices when they are configured and the
// batch is big enough (kClusterMinSources) on a 32-bit plan, else (or when a
// block needs 64-bit rows) on the area's own device.  Caller holds devMu.
std::vector<std::unique_ptr<SpfView>> runBatchAuto(
    LinkState::Engine& eng, const std::vector<uint32_t>& sources, bool useLinkMetric,
    bool wantNextHops, const std::vector<std::vector<uint32_t>>* ignore) {
  if (sources.size() >= clusterMinSources() && !(eng.exact && useLinkMetric) &&
      !getSpfDevices().empty()) {
    auto views = runBatchCluster(eng, sources, useLinkMetric, wantNextHops, ignore);
    if (!views.empty()) {
      return views;
    }
  }
  return runBatch(eng, sources, useLinkMetric, wantNextHops, ignore);
}

// KSP2 second passes with their traces on the device (getKthPaths k = 2,
// LinkState.cpp:760-789): one ignore-list SPF per destination, then
// spf_query_trace_paths / spf_table_trace_paths over the rows where they lie,
// so only link-id paths come back (no 4*V-byte row per destination).  count[i]
// = SPF_TRACE_OVERFLOW marks a query the device could not trace: its row is
// returned in rows[i] for the host trace.  Caller holds devMu; the batch is
// 32-bit (the caller checks !eng.exact).
struct DeviceTraces {
  std::vector<uint32_t> count, linkCount; // per query (count: SPF_TRACE_OVERFLOW)
  std::vector<uint32_t> links, ends;      // packed (spf_query_trace_fetch)
  std::vector<std::unique_ptr<SpfView>> rows; // overflowed queries only
  bool unsupported = false; // 64-bit rows in some block: use runBatchAuto
};

// default (OPENR_KSP2_DEVICE_TRACE=0 traces on the host pool instead): the
// cursor DFS (spf_trace_cursor_kernel) keeps one pathLinks cursor per node in
// device scratch; the round-3 kernel re-scanned a node's in-edges per step
// and overflowed 632 of the fabric's 9,975 traces to the host (profiles/r03d)
bool deviceTraceEnabled() {
  const char* e = std::getenv("OPENR_KSP2_DEVICE_TRACE");
  return !e || std::atoi(e) != 0;
}

DeviceTraces traceSecondPasses(
    LinkState::Engine& eng, const std::vector<uint32_t>& sources,
    const std::vector<uint32_t>& dests, const std::vector<std::vector<uint32_t>>& lists) {
  const auto tBatch = std::chrono::steady_clock::now();
  const uint32_t V = (uint32_t)eng.names.size();
  const uint32_t nq = (uint32_t)sources.size();
  DeviceTraces out;
  out.count.assign(nq, 0);
  out.linkCount.assign(nq, 0);
  out.rows.resize(nq);
  auto sizeOutputs = [&] {
    size_t nl = 0, np = 0;
    for (uint32_t i = 0; i < nq; ++i) {
      if (out.count[i] != SPF_TRACE_OVERFLOW) {
        nl += out.linkCount[i];
        np += out.count[i];
      }
    }
    out.links.resize(nl);
    out.ends.resize(np);
  };
  std::vector<uint32_t> ioff{0}, ilinks;
  for (const auto& l : lists) {
    ilinks.insert(ilinks.end(), l.begin(), l.end());
    ioff.push_back((uint32_t)ilinks.size());
  }
  spf_query_desc qd{};
  qd.num_queries = nq;
  qd.sources = sources.data();
  qd.flags = 0; // link metrics, distances only: a trace reads no masks
  qd.ignore_offsets = ioff.data();
  qd.ignore_links = ilinks.data();
  auto rowView = [&](size_t i, const std::shared_ptr<std::vector<uint32_t>>& row) {
    auto view = std::make_unique<SpfView>();
    view->src = sources[i];
    view->useLinkMetric = true;
    view->dist.share32(row, 0, V);
    view->ignored = lists[i];
    return view;
  };
  const bool cluster = nq >= clusterMinSources() && !getSpfDevices().empty();
  if (cluster) {
    auto& cs = clusterState();
    std::lock_guard<std::mutex> g(cs.mu);
    if (!cs.cluster) {
      const int c = spf_cluster_create_local(
          (uint32_t)cs.devices.size(), cs.devices.data(), &cs.cluster);
      if (c != SPF_OK) {
        engineFailure("spf_cluster_create_local", c);
      }
    }
    if (eng.cgraph && eng.cgraphGen != cs.gen) {
      spf_cgraph_destroy(eng.cgraph);
      eng.cgraph = nullptr;
    }
    if (!eng.cgraph) {
      spf_graph_desc d{};
      d.num_nodes = V;
      d.num_edges = (uint32_t)eng.col.size();
      d.row_ptr = eng.row.data();
      d.col = eng.col.data();
      d.metric = eng.metric.data();
      d.link_id = eng.linkId.data();
      d.rev = eng.rev.data();
      d.node_overloaded = eng.overloaded.data();
      d.num_links = (uint32_t)eng.links.size();
      if (const int c = spf_cgraph_create(cs.cluster, &d, &eng.cgraph); c != SPF_OK) {
        engineFailure("spf_cgraph_create", c);
      }
      eng.cgraphGen = cs.gen;
      Counters::add("decision.cluster_graph_uploads", 1);
    }
    spf_table* t = nullptr;
    int st = spf_table_create_q(eng.cgraph, &qd, 0, &t);
    struct TGuard {
      spf_table* t;
      ~TGuard() {
        if (t) {
          spf_table_destroy(t);
        }
      }
    } tg{t};
    if (st == SPF_OK && (st = spf_table_run(t)) == SPF_OK && (st = spf_table_sync(t)) == SPF_OK) {
      float cm = 0, gm = 0;
      spf_table_elapsed_ms(t, &cm, &gm);
      eng.lastMs = cm + gm;
      Counters::add("decision.spf_device_us", (int64_t)(eng.lastMs * 1000.0f));
      const auto tTr = std::chrono::steady_clock::now();
      st = spf_table_trace_paths(t, dests.data(), out.count.data(), out.linkCount.data());
      if (st == SPF_E_UNSUPPORTED) {
        out.unsupported = true;
        return out;
      }
      if (st == SPF_OK) {
        sizeOutputs();
        st = spf_table_trace_fetch(t, out.links.data(), out.ends.data());
      }
      Counters::add("decision.kth2_device_trace_us",
                    std::chrono::duration_cast<std::chrono::microseconds>(
                        std::chrono::steady_clock::now() - tTr)
                        .count());
    }
    if (st != SPF_OK) {
      engineFailure("spf_table (KSP2 device traces)", st);
    }
    Counters::add("decision.spf_cluster_batches", 1);
    for (uint32_t i = 0; i < nq; ++i) {
      if (out.count[i] == SPF_TRACE_OVERFLOW) {
        auto row = std::make_shared<std::vector<uint32_t>>(V);
        if (const int c = spf_table_fetch_rows(t, i, 1, row->data()); c != SPF_OK) {
          engineFailure("spf_table_fetch_rows", c);
        }
        out.rows[i] = rowView(i, row);
      }
    }
  } else {
    spf_query* q = nullptr;
    int s = spf_query_create(eng.graph, &qd, &q);
    if (s != SPF_OK) {
      engineFailure("spf_query_create", s);
    }
    struct Guard {
      spf_query* q;
      ~Guard() { spf_query_destroy(q); }
    } guard{q};
    if ((s = spf_query_run(q)) != SPF_OK || (s = spf_query_sync(q)) != SPF_OK) {
      engineFailure("spf_query_run", s);
    }
    spf_query_elapsed_ms(q, &eng.lastMs);
    Counters::add("decision.spf_device_us", (int64_t)(eng.lastMs * 1000.0f));
    const auto tTr = std::chrono::steady_clock::now();
    s = spf_query_trace_paths(q, 0, nq, dests.data(), out.count.data(), out.linkCount.data());
    if (s == SPF_E_UNSUPPORTED) {
      out.unsupported = true;
      return out;
    }
    if (s != SPF_OK) {
      engineFailure("spf_query_trace_paths", s);
    }
    sizeOutputs();
    if ((s = spf_query_trace_fetch(q, out.links.data(), out.ends.data())) != SPF_OK) {
      engineFailure("spf_query_trace_fetch", s);
    }
    Counters::add("decision.kth2_device_trace_us",
                  std::chrono::duration_cast<std::chrono::microseconds>(
                      std::chrono::steady_clock::now() - tTr)
                      .count());
    for (uint32_t i = 0; i < nq; ++i) {
      if (out.count[i] == SPF_TRACE_OVERFLOW) {
        auto row = std::make_shared<std::vector<uint32_t>>(V);
        if ((s = spf_query_fetch_rows(q, i, 1, row->data(), (size_t)V * 4, 0)) != SPF_OK) {
          engineFailure("spf_query_fetch_rows", s);
        }
        out.rows[i] = rowView(i, row);
      }
    }
  }
  const double batchMs =
      std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tBatch)
          .count();
  Counters::add("decision.spf_batch_us", (int64_t)(batchMs * 1000.0));
  for (uint32_t i = 0; i < nq; ++i) {
    Counters::add("decision.spf_ms", (int64_t)(batchMs / (double)nq));
  }
  return out;
}

// Predecessors of v in the reference's pathLinks order: usable in-links whose
// tail is the source or transit, is settled before v and is tight; sorted by
// the tail's settle rank, then by the tail's linksFromNode() order.
void pathLinksOf(
    const LinkState::Engine& eng,
    const SpfView& view,
    uint32_t v,
    std::vector<std::pair<uint32_t /* half-edge u->v */, uint32_t /* u */>>& out) {
  out.clear();
  if (!view.reached(v) || v == view.src) {
    return;
  }
  const uint64_t dv = view.dist[v];
  for (uint32_t e = eng.row[v]; e < eng.row[v + 1]; ++e) {
    const uint32_t u = eng.col[e];
    if (!view.reached(u)) {
      continue;
    }
    if (u != view.src && eng.overloaded[u]) {
      continue;
    }
    if (!view.ignored.empty() &&
        std::binary_search(view.ignored.begin(), view.ignored.end(), eng.linkId[e])) {
      continue;
    }
    const uint32_t eu = eng.rev[e]; // the half-edge u->v
    const uint64_t w = view.useLinkMetric ? eng.metric[eu] : 1ull;
    if (view.dist[u] + w != dv) {
      continue;
    }
    if (!view.settlesBefore(u, v)) {
      continue;
    }
    out.emplace_back(eu, u);
  }
  std::sort(out.begin(), out.end(), [&](const auto& a, const auto& b) {
    const uint32_t ua = a.second, ub = b.second;
    if (ua != ub) {
      return view.settlesBefore(ua, ub);
    }
    return a.first < b.first; // row-u position = linksFromNode(u) order
  });
}

} // namespace

namespace {

// OPENR_SPF_MEMO_SCREEN=0: drop the whole memo on every change (the
// reference's behaviour, LinkState.cpp:712-715)
bool memoScreenEnabled() {
  static const bool on = [] {
    const char* e = getenv("OPENR_SPF_MEMO_SCREEN");
    return !(e && atoi(e) == 0);
  }();
  return on;
}

// The table screen rule (spf_table_screen) on one host view:
// the view keeps its distances AND next hops exactly unless some delta in
// scope of its source is a tight edge that disappears or an edge at least as
// good as the current distance of its head.
bool screenHit(const SpfView& view, const std::vector<spf_edge_delta>& ds) {
  const uint32_t s = view.src;
  for (const auto& d : ds) {
    if ((d.scope == SPF_SCOPE_TAIL_ONLY && s != d.tail) ||
        (d.scope == SPF_SCOPE_NOT_TAIL && s == d.tail)) {
      continue;
    }
    const uint64_t du = view.dist[d.tail];
    if (du == SpfView::kUnreachable) {
      continue;
    }
    const uint64_t dv = view.dist[d.head];
    const uint64_t c = du + (view.useLinkMetric ? d.metric : 1ull);
    if (d.kind == SPF_DELTA_REMOVED ? c == dv : (dv == SpfView::kUnreachable || c <= dv)) {
      return true;
    }
  }
  return false;
}

// keep the views of `memo` the deltas cannot touch, drop the rest
template <class Map>
void screenMemo(Map& memo, Map& into, const std::vector<spf_edge_delta>& ds) {
  int64_t kept = 0, dropped = 0;
  for (auto& [id, view] : memo) {
    if (view && !screenHit(*view, ds)) {
      into.emplace(id, std::move(view));
      ++kept;
    } else {
      ++dropped;
    }
  }
  memo.clear();
  Counters::add("decision.spf_memo_kept", kept);
  Counters::add("decision.spf_memo_dropped", dropped);
}

spf_graph_desc engineDesc(const LinkState::Engine& eng, const uint64_t* metric) {
  spf_graph_desc d{};
  d.num_nodes = (uint32_t)eng.names.size();
  d.num_edges = (uint32_t)eng.col.size();
  d.row_ptr = eng.row.data();
  d.col = eng.col.data();
  d.metric = metric;
  d.link_id = eng.linkId.data();
  d.rev = eng.rev.data();
  d.node_overloaded = eng.overloaded.data();
  d.num_links = (uint32_t)eng.links.size();
  return d;
}

// Memo views of a retired engine that survive a structural change: same
// nodes (ids = name ranks), deltas = spf_graph_diff of the two CSRs (unit
// metrics for the hop-count memo), the screen rule per view.
void adoptScreenedViews(LinkState::Engine& old, LinkState::Engine& neu) {
  if (old.names != neu.names || old.exact || neu.exact) {
    return;
  }
  for (int k = 0; k < 2; ++k) {
    if (old.memo[k].empty()) {
      continue;
    }
    const std::vector<uint64_t> onesOld(old.col.size(), 1), onesNew(neu.col.size(), 1);
    const spf_graph_desc a = engineDesc(old, k ? old.metric.data() : onesOld.data());
    const spf_graph_desc b = engineDesc(neu, k ? neu.metric.data() : onesNew.data());
    uint32_t n = 0;
    if (spf_graph_diff(&a, &b, nullptr, 0, &n) != SPF_OK) {
      return;
    }
    std::vector<spf_edge_delta> ds(n);
    if (n && spf_graph_diff(&a, &b, ds.data(), n, &n) != SPF_OK) {
      return;
    }
    screenMemo(old.memo[k], neu.memo[k], ds);
  }
}

} // namespace

LinkState::Engine& LinkState::engine() const {
  if (!engine_) {
    engine_ = std::make_unique<Engine>();
  }
  if (!engine_->built) {
    const auto t0 = std::chrono::steady_clock::now();
    buildGraph(*engine_, linkMap_, adjacencyDatabases_, *this);
    Counters::add(
        "decision.graph_build_us",
        std::chrono::duration_cast<std::chrono::microseconds>(
            std::chrono::steady_clock::now() - t0)
            .count());
    if (retired_) {
      adoptScreenedViews(*retired_, *engine_);
      retired_.reset();
    }
  }
  return *engine_;
}

// ---------------------------------------------------------------- LinkState

LinkState::LinkState(const std::string& area) : area_(area) {}
LinkState::~LinkState() {
  if (kthReaper_.joinable()) {
    kthReaper_.join();
  }
}
LinkState::LinkState(LinkState&& o) noexcept
    : area_(o.area_),
      linkMap_(std::move(o.linkMap_)),
      allLinks_(std::move(o.allLinks_)),
      nodeOverloads_(std::move(o.nodeOverloads_)),
      adjacencyDatabases_(std::move(o.adjacencyDatabases_)),
      spfResultsMetric_(std::move(o.spfResultsMetric_)),
      spfResultsHops_(std::move(o.spfResultsHops_)),
      kth_(std::move(o.kth_)),
      kthReaper_(std::move(o.kthReaper_)),
      kthFill_(std::move(o.kthFill_)),
      engine_(std::move(o.engine_)),
      retired_(std::move(o.retired_)),
      topoGen_(o.topoGen_) {}

size_t LinkState::LinkPtrHash::operator()(const std::shared_ptr<Link>& l) const {
  return l->hash;
}
bool LinkState::LinkPtrLess::operator()(
    const std::shared_ptr<Link>& lhs, const std::shared_ptr<Link>& rhs) const {
  return *lhs < *rhs;
}
bool LinkState::LinkPtrEqual::operator()(
    const std::shared_ptr<Link>& lhs, const std::shared_ptr<Link>& rhs) const {
  return *lhs == *rhs;
}

void LinkState::clearKthMemo() const {
  // the stripes hold one entry per (src, dst, k) a KSP2 build filled (20k on
  // the fabric, two vectors each, allocated by the build's worker threads):
  // the filled memo is swapped for an empty one at once and freed by a
  // reaper thread, off the update path (freeing it here took 24 ms of every
  // KSP2 topology update, most of it in malloc arena locks).  Nothing reads
  // the old memo any more (updates and builds do not overlap); the next
  // clear and the destructor join the reaper first.
  size_t n = 0;
  for (auto& stripe : *kth_) {
    n += stripe.ids.size() + stripe.paths.size();
  }
  if (n == 0) {
    return;
  }
  auto old = std::move(kth_);
  kth_ = std::make_unique<std::array<KthStripe, kKthStripes>>();
  if (kthReaper_.joinable()) {
    kthReaper_.join();
  }
  static const bool inlineFree = std::getenv("OPENR_KTH_FREE_INLINE") != nullptr;
  if (inlineFree) {
    old.reset();
    return;
  }
  kthReaper_ = std::thread([o = std::move(old)]() mutable { o.reset(); });
}

void LinkState::clearMemo() const {
  ++topoGen_;
  spfResultsMetric_.clear();
  spfResultsHops_.clear();
  clearKthMemo();
  if (engine_) {
    // a built engine retires with its memo: the next graph build keeps the
    // views no edge delta can touch (selective invalidation, SURVEY §8(f)
    // row 2); the reference drops them all (LinkState.cpp:712-715)
    if (engine_->built && memoScreenEnabled()) {
      retired_ = std::move(engine_);
    }
    engine_.reset(); // drop the device graph: the topology changed
  }
}

// Drop the device graph and every memoized result, retired ones included
// (nothing is screened or adopted by the next build).
void LinkState::invalidate() const {
  clearMemo();
  retired_.reset();
  engine_.reset();
}

// Topology change that keeps the set of up links: drop every SPF memo but
// keep the device graph, patching node transit bits / link metrics in place
// (incremental CSR deltas instead of a full rebuild).
void LinkState::patchMemo(
    const std::vector<std::string>& transitNodes,
    const std::vector<std::pair<std::shared_ptr<Link>, std::string>>& metricPatches) const {
  if (!engine_ || !engine_->built || !engine_->graph) {
    clearMemo();
    return;
  }
  auto& eng = *engine_;
  ++topoGen_;
  std::vector<uint32_t> edges;
  std::vector<uint64_t> metrics;
  for (const auto& [link, from] : metricPatches) {
    const uint32_t li = eng.linkIdOf(link.get());
    if (li == ~0u) {
      clearMemo(); // not an up link of the device graph: rebuild
      return;
    }
    const auto& h = eng.halves[li];
    const uint32_t e = from == link->firstNodeName() ? h[0] : h[1];
    if (e == ~0u) {
      clearMemo();
      return;
    }
    edges.push_back(e);
    metrics.push_back(link->getMetricFromNode(from));
  }
  // edge deltas of this patch for the memo screen (metric memo / hop memo),
  // taken before the host mirrors change: a metric change is its half-edge
  // REMOVED at the old and ADDED at the new metric; a transit flip of x is
  // every out-edge of x REMOVED / ADDED for sources other than x
  std::vector<spf_edge_delta> dMetric, dHops;
  std::unordered_map<uint32_t, uint64_t> newMetric;
  for (size_t i = 0; i < edges.size(); ++i) {
    newMetric[edges[i]] = metrics[i];
    const uint32_t e = edges[i];
    const uint32_t u = eng.col[eng.rev[e]], v = eng.col[e];
    dMetric.push_back({u, v, eng.metric[e], SPF_DELTA_REMOVED, SPF_SCOPE_ALL});
    dMetric.push_back({u, v, metrics[i], SPF_DELTA_ADDED, SPF_SCOPE_ALL});
  }
  bool transit = false;
  for (const auto& n : transitNodes) {
    auto it = eng.ids.find(n);
    if (it == eng.ids.end()) {
      continue; // not in the graph: no transit bit to flip
    }
    const uint32_t x = it->second;
    const uint8_t ov = isNodeOverloaded(n) ? 1 : 0;
    if (eng.overloaded[x] != ov) {
      transit = true;
      const uint32_t kind = ov ? SPF_DELTA_REMOVED : SPF_DELTA_ADDED;
      for (uint32_t e = eng.row[x]; e < eng.row[x + 1]; ++e) {
        auto nm = newMetric.find(e);
        const uint64_t w = ov || nm == newMetric.end() ? eng.metric[e] : nm->second;
        dMetric.push_back({x, eng.col[e], w, kind, SPF_SCOPE_NOT_TAIL});
        dHops.push_back({x, eng.col[e], 1, kind, SPF_SCOPE_NOT_TAIL});
      }
    }
    eng.overloaded[x] = ov;
  }
  const auto tClear = std::chrono::steady_clock::now();
  spfResultsMetric_.clear();
  spfResultsHops_.clear();
  clearKthMemo();
  Counters::add("decision.kth_memo_clear_us",
                std::chrono::duration_cast<std::chrono::microseconds>(
                    std::chrono::steady_clock::now() - tClear)
                    .count());
  if (memoScreenEnabled() && !eng.exact) {
    for (int k = 0; k < 2; ++k) {
      std::remove_reference_t<decltype(eng.memo[0])> keep;
      screenMemo(eng.memo[k], keep, k ? dMetric : dHops);
      eng.memo[k] = std::move(keep);
    }
  }
  for (auto& m : eng.memo) {
    if (!memoScreenEnabled() || eng.exact) {
      m.clear();
    }
  }
  for (auto& m : eng.prefetched) {
    m.clear();
  }
  eng.kthPrefetch.clear();
  eng.isolated.clear();
  const auto t0 = std::chrono::steady_clock::now();
  // The host mirrors (eng.overloaded, eng.metric) were / are updated before
  // the device upload: if an upload fails, drop the whole engine so the next
  // access rebuilds the device graph from linkMap_ instead of comparing
  // against mirrors that no longer describe the device state.
  try {
    if (transit) {
      const int s = spf_graph_set_transit(eng.graph, eng.overloaded.data());
      if (s != SPF_OK) {
        engineFailure("spf_graph_set_transit", s);
      }
      if (eng.cgraph) {
        const int c = spf_cgraph_set_transit(eng.cgraph, eng.overloaded.data());
        if (c != SPF_OK) {
          engineFailure("spf_cgraph_set_transit", c);
        }
      }
    }
    if (!edges.empty()) {
      for (size_t i = 0; i < edges.size(); ++i) {
        eng.metric[edges[i]] = metrics[i];
      }
      eng.dropQuery(); // (plans read the metrics: uniform, widths, buckets)
      const int s = spf_graph_patch_metrics(
          eng.graph, (uint32_t)edges.size(), edges.data(), metrics.data());
      if (s != SPF_OK) {
        engineFailure("spf_graph_patch_metrics", s);
      }
      if (eng.cgraph) {
        const int c = spf_cgraph_patch_metrics(
            eng.cgraph, (uint32_t)edges.size(), edges.data(), metrics.data());
        if (c != SPF_OK) {
          engineFailure("spf_cgraph_patch_metrics", c);
        }
      }
    }
    // metrics and transit bits both feed the 32-bit row bound (refresh_exact)
    eng.exact = spf_graph_needs_exact(eng.graph) != 0;
  } catch (...) {
    clearMemo();
    throw;
  }
  Counters::add("decision.graph_patches", 1);
  Counters::add(
      "decision.graph_patch_us",
      std::chrono::duration_cast<std::chrono::microseconds>(
          std::chrono::steady_clock::now() - t0)
          .count());
}

// Link flaps in place (SURVEY §8(f) row 2 for the product LinkState): the
// links whose up-ness flipped change the rows of their endpoints only, so
// those rows are rebuilt from linkMap_ and every other row is copied (node
// ids are name ranks and the node set is unchanged).  Link ids of links that
// stay are kept (a removed link's id is freed, a new link takes a free id or
// the next one), so the Link tags stay valid; half-edge indices of the kept
// rows shift by their row's offset change.  The device graph is rebuilt in
// place from the spliced arrays (spf_graph_update); SPF memos survive where no edge delta can touch
// them (the same screen as patchMemo).  Returns false (nothing changed) when
// a link's endpoint is not a node of the graph, or the engine is not built.
bool LinkState::patchStructure(
    const std::vector<std::shared_ptr<Link>>& down,
    const std::vector<std::shared_ptr<Link>>& up,
    const std::vector<std::string>& transitNodes,
    const std::vector<std::pair<std::shared_ptr<Link>, std::string>>& metricPatches) const {
  static const bool enabled = [] {
    const char* e = std::getenv("OPENR_LS_INPLACE_LINKS");
    return !(e && std::atoi(e) == 0);
  }();
  if (!enabled || !engine_ || !engine_->built || !engine_->graph) {
    return false;
  }
  const auto t0 = std::chrono::steady_clock::now();
  // OPENR_LS_SPLICE_TIMING=1: phase times of the splice on stderr (diagnostics)
  static const bool splTiming = [] {
    const char* e = std::getenv("OPENR_LS_SPLICE_TIMING");
    return e && std::atoi(e) != 0;
  }();
  auto tp = t0;
  auto mark = [&](const char* what) {
    if (splTiming) {
      const auto t = std::chrono::steady_clock::now();
      std::fprintf(stderr, "[patchStructure] %-10s %8.3f ms\n", what,
                   std::chrono::duration<double, std::milli>(t - tp).count());
      tp = t;
    }
  };
  auto& eng = *engine_;
  const uint32_t V = (uint32_t)eng.names.size();
  std::vector<uint8_t> aff(V, 0);
  auto nodeOf = [&](const std::string& n) -> uint32_t {
    auto it = eng.ids.find(n);
    return it == eng.ids.end() ? ~0u : it->second;
  };
  for (const auto& l : down) {
    const uint32_t a = nodeOf(l->firstNodeName()), b = nodeOf(l->secondNodeName());
    if (a == ~0u || b == ~0u || eng.linkIdOf(l.get()) == ~0u) {
      return false;
    }
    aff[a] = aff[b] = 1;
  }
  for (const auto& l : up) {
    const uint32_t a = nodeOf(l->firstNodeName()), b = nodeOf(l->secondNodeName());
    if (a == ~0u || b == ~0u || eng.linkIdOf(l.get()) != ~0u || !l->isUp()) {
      return false;
    }
    aff[a] = aff[b] = 1;
  }
  // new rows of the affected nodes, in linksFromNode order (up links only)
  std::vector<uint32_t> affNodes;
  for (uint32_t u = 0; u < V; ++u) {
    if (aff[u]) {
      affNodes.push_back(u);
    }
  }
  std::vector<std::vector<const std::shared_ptr<Link>*>> affRows(affNodes.size());
  // the retired arrays of the last splice are reused (no fresh pages)
  std::vector<uint32_t> newRow = std::move(eng.spareRow);
  newRow.assign(V + 1, 0);
  {
    size_t k = 0;
    for (uint32_t u = 0; u < V; ++u) {
      uint32_t d = eng.row[u + 1] - eng.row[u];
      if (aff[u]) {
        for (const auto& link : linksFromNode(eng.names[u])) {
          if (link->isUp()) {
            affRows[k].push_back(&link);
          }
        }
        d = (uint32_t)affRows[k++].size();
      }
      newRow[u + 1] = newRow[u] + d;
    }
  }
  const uint32_t E = newRow[V];
  mark("rows");
  // link ids: freed for the links going down, taken for the ones coming up.
  // eng.links is not copied (a copy of ~100k shared_ptrs is two atomic
  // refcount updates per link, ~2 ms on the fabric): which ids are alive is a
  // byte per id, and the id -> Link changes are applied at the commit.  The
  // byte and halves arrays of the last splice are reused (no fresh pages).
  std::vector<uint8_t> alive = std::move(eng.spareAlive);
  alive.resize(eng.links.size());
  std::vector<std::array<uint32_t, 2>> halves = std::move(eng.spareHalves);
  halves.resize(eng.halves.size());
  {
    // one parallel pass: the alive bytes, and the halves moved to the new
    // CSR.  Only the affected rows change length, so a kept half-edge e moves
    // by the summed length change of the affected rows before it (a few
    // ranges: no per-edge lookup of its tail); a half in an affected row is
    // re-set below.
    std::vector<std::array<uint32_t, 3>> rng; // old [begin, end), shift after it
    int64_t cum = 0;
    for (uint32_t u : affNodes) {
      cum += (int64_t)(newRow[u + 1] - newRow[u]) - (int64_t)(eng.row[u + 1] - eng.row[u]);
      rng.push_back({eng.row[u], eng.row[u + 1], (uint32_t)cum});
    }
    auto moved = [&](uint32_t e) -> uint32_t {
      uint32_t d = 0;
      for (const auto& r : rng) {
        if (e < r[0]) {
          break;
        }
        if (e < r[1]) {
          return ~0u;
        }
        d = r[2];
      }
      return e + d; // modular: a negative shift wraps back
    };
    constexpr size_t kLB = 16384;
    const size_t nl = std::max(eng.links.size(), eng.halves.size());
    parallelFor((nl + kLB - 1) / kLB, hostThreads(nl, 1u << 14), [&](size_t b, unsigned) {
      const size_t i1 = std::min(nl, (b + 1) * kLB);
      for (size_t i = b * kLB; i < i1; ++i) {
        if (i < eng.links.size()) {
          alive[i] = eng.links[i] != nullptr;
        }
        if (i < eng.halves.size()) {
          const auto& h = eng.halves[i];
          halves[i] = {h[0] == ~0u ? ~0u : moved(h[0]), h[1] == ~0u ? ~0u : moved(h[1])};
        }
      }
    }, 1);
  }
  std::vector<std::pair<uint32_t, std::shared_ptr<Link>>> linkSets; // applied at the commit
  mark("ids");
  std::vector<uint32_t> freeIds = eng.freeIds;
  std::vector<spf_edge_delta> dMetric, dHops;
  for (const auto& l : down) {
    const uint32_t lid = eng.linkIdOf(l.get());
    for (int s = 0; s < 2; ++s) {
      const uint32_t e = eng.halves[lid][s];
      if (e != ~0u) {
        const uint32_t u = eng.col[eng.rev[e]], v = eng.col[e];
        dMetric.push_back({u, v, eng.metric[e], SPF_DELTA_REMOVED, SPF_SCOPE_ALL});
        dHops.push_back({u, v, 1, SPF_DELTA_REMOVED, SPF_SCOPE_ALL});
      }
    }
    alive[lid] = 0;
    linkSets.emplace_back(lid, nullptr);
    halves[lid] = {~0u, ~0u};
    freeIds.push_back(lid);
  }
  std::sort(freeIds.begin(), freeIds.end(), std::greater<uint32_t>());
  std::unordered_map<const Link*, uint32_t> upIds;
  for (const auto& l : up) {
    uint32_t lid;
    if (!freeIds.empty()) {
      lid = freeIds.back();
      freeIds.pop_back();
    } else {
      lid = (uint32_t)alive.size();
      alive.push_back(0);
      halves.push_back({~0u, ~0u});
    }
    alive[lid] = 1;
    linkSets.emplace_back(lid, l);
    upIds.emplace(l.get(), lid);
  }
  auto idOf = [&](const Link* l) {
    auto it = upIds.find(l);
    return it != upIds.end() ? it->second : eng.linkIdOf(l);
  };
  // the copies and scatters below run in blocks on the host pool (one
  // writer per element: a kept half / row / link id belongs to one block);
  // node blocks are small because a fabric's high-degree rows are adjacent
  constexpr size_t kBlk = 4096, kNodeBlk = 256;
  const unsigned nth = hostThreads(eng.col.size(), 1u << 15);
  mark("shift");
  std::vector<uint32_t> col = std::move(eng.spareCol), linkId = std::move(eng.spareLinkId);
  std::vector<uint64_t> metric = std::move(eng.spareMetric);
  col.resize(E);
  linkId.resize(E);
  metric.resize(E);
  parallelFor((V + kNodeBlk - 1) / kNodeBlk, nth, [&](size_t b, unsigned) {
    const uint32_t u1 = (uint32_t)std::min<size_t>(V, (b + 1) * kNodeBlk);
    for (uint32_t u = (uint32_t)(b * kNodeBlk); u < u1; ++u) {
      if (!aff[u]) {
        const uint32_t a = eng.row[u], z = eng.row[u + 1], o = newRow[u];
        std::copy(eng.col.begin() + a, eng.col.begin() + z, col.begin() + o);
        std::copy(eng.linkId.begin() + a, eng.linkId.begin() + z, linkId.begin() + o);
        std::copy(eng.metric.begin() + a, eng.metric.begin() + z, metric.begin() + o);
      }
    }
  }, 1);
  {
    size_t k = 0;
    for (uint32_t u : affNodes) {
      const std::string& name = eng.names[u];
      uint32_t e = newRow[u];
      for (const auto* lp : affRows[k++]) {
        const Link* link = lp->get();
        const uint32_t lid = idOf(link);
        const uint32_t v = nodeOf(link->getOtherNodeName(name));
        if (lid == ~0u || v == ~0u) {
          return false; // an up link the graph does not know: rebuild
        }
        col[e] = v;
        linkId[e] = lid;
        metric[e] = link->getMetricFromNode(name);
        halves[lid][name == link->firstNodeName() ? 0 : 1] = e;
        ++e;
      }
    }
  }
  mark("copy");
  std::vector<uint32_t> rev = std::move(eng.spareRev);
  rev.assign(E, ~0u);
  std::atomic<bool> oneHalf{false};
  parallelFor((halves.size() + kBlk - 1) / kBlk, nth, [&](size_t b, unsigned) {
    const size_t l1 = std::min(halves.size(), (b + 1) * kBlk);
    for (size_t lid = b * kBlk; lid < l1; ++lid) {
      const auto& h = halves[lid];
      if (!alive[lid]) {
        continue;
      }
      if (h[0] == ~0u || h[1] == ~0u) {
        oneHalf.store(true, std::memory_order_relaxed);
        return;
      }
      rev[h[0]] = h[1];
      rev[h[1]] = h[0];
    }
  }, 1);
  if (oneHalf.load()) {
    eng.spareRev = std::move(rev);
    return false; // a link with one half: rebuild
  }
  for (const auto& l : up) {
    const auto& h = halves[upIds.at(l.get())];
    for (int s = 0; s < 2; ++s) {
      const uint32_t e = h[s];
      dMetric.push_back({col[rev[e]], col[e], metric[e], SPF_DELTA_ADDED, SPF_SCOPE_ALL});
      dHops.push_back({col[rev[e]], col[e], 1, SPF_DELTA_ADDED, SPF_SCOPE_ALL});
    }
  }
  // metric patches of the same update.  The REMOVED delta must carry the
  // metric the memoized rows were computed with: an affected row was rebuilt
  // from linkMap_ above, where Link::setMetricFromNode has already run, so
  // metric[e] may hold the new value; the old one is in the retired arrays
  // (eng.metric at the link's old half-edge).
  for (const auto& [link, from] : metricPatches) {
    const int side = from == link->firstNodeName() ? 0 : 1;
    const uint64_t w = link->getMetricFromNode(from);
    if (const auto it = upIds.find(link.get()); it != upIds.end()) {
      // came up in this update: its ADDED delta above has the new metric
      const uint32_t e = halves[it->second][side];
      if (e == ~0u) {
        return false;
      }
      metric[e] = w;
      continue;
    }
    const uint32_t lid = eng.linkIdOf(link.get());
    if (lid == ~0u || lid >= eng.halves.size()) {
      return false;
    }
    const uint32_t eOld = eng.halves[lid][side], e = halves[lid][side];
    if (eOld == ~0u || e == ~0u) {
      return false;
    }
    const uint64_t wOld = eng.metric[eOld];
    if (wOld != w) {
      dMetric.push_back({col[rev[e]], col[e], wOld, SPF_DELTA_REMOVED, SPF_SCOPE_ALL});
      dMetric.push_back({col[rev[e]], col[e], w, SPF_DELTA_ADDED, SPF_SCOPE_ALL});
    }
    metric[e] = w;
  }
  std::vector<uint8_t> overloaded = eng.overloaded;
  for (const auto& n : transitNodes) {
    const uint32_t x = nodeOf(n);
    if (x == ~0u) {
      continue;
    }
    const uint8_t ov = isNodeOverloaded(n) ? 1 : 0;
    if (overloaded[x] != ov) {
      const uint32_t kind = ov ? SPF_DELTA_REMOVED : SPF_DELTA_ADDED;
      for (uint32_t e = newRow[x]; e < newRow[x + 1]; ++e) {
        dMetric.push_back({x, col[e], metric[e], kind, SPF_SCOPE_NOT_TAIL});
        dHops.push_back({x, col[e], 1, kind, SPF_SCOPE_NOT_TAIL});
      }
    }
    overloaded[x] = ov;
  }
  // the new device graph first: on failure nothing of the engine changed
  spf_graph_desc d{};
  d.num_nodes = V;
  d.num_edges = E;
  d.row_ptr = newRow.data();
  d.col = col.data();
  d.metric = metric.data();
  d.link_id = linkId.data();
  d.rev = rev.data();
  d.node_overloaded = overloaded.data();
  d.num_links = (uint32_t)alive.size();
  d.device = getSpfDevice();
  // the device graph is rebuilt in place (same handle, stream and buffers:
  // spf_graph_update).  A failed update leaves it unusable: it is retired
  // (Engine::retireGraph), and the caller's clearMemo() retires the engine,
  // whose next build creates a fresh graph
  mark("rev+rest");
  const auto tu = std::chrono::steady_clock::now();
  Counters::add("decision.graph_splice_us",
                std::chrono::duration_cast<std::chrono::microseconds>(tu - t0).count());
  eng.dropQuery(); // (the splice changes rows, neighbour lists and plans)
  if (spf_graph_update(eng.graph, &d) != SPF_OK) {
    // the handle is never nulled while the ABI still refuses to free it
    // (live queries): retireGraph keeps it for a later destroy
    eng.retireGraph();
    return false;
  }
  Counters::add("decision.graph_update_us",
                std::chrono::duration_cast<std::chrono::microseconds>(
                    std::chrono::steady_clock::now() - tu)
                    .count());
  // commit
  ++topoGen_;
  spfResultsMetric_.clear();
  spfResultsHops_.clear();
  clearKthMemo();
  for (const auto& l : down) {
    l->engineEpoch = 0;
  }
  for (const auto& [l, lid] : upIds) {
    l->engineEpoch = eng.epoch;
    l->engineId = lid;
  }
  if (eng.cgraph) {
    spf_cgraph_destroy(eng.cgraph);
    eng.cgraph = nullptr;
    eng.cgraphGen = 0;
  }
  std::swap(eng.row, newRow);
  std::swap(eng.col, col);
  std::swap(eng.linkId, linkId);
  std::swap(eng.metric, metric);
  std::swap(eng.rev, rev);
  eng.spareRow = std::move(newRow);
  eng.spareCol = std::move(col);
  eng.spareLinkId = std::move(linkId);
  eng.spareMetric = std::move(metric);
  eng.spareRev = std::move(rev);
  eng.overloaded = std::move(overloaded);
  if (eng.links.size() < alive.size()) {
    eng.links.resize(alive.size());
  }
  for (auto& [lid, l] : linkSets) {
    eng.links[lid] = std::move(l); // in order: a freed id taken again ends up set
  }
  eng.spareHalves = std::move(eng.halves);
  eng.halves = std::move(halves);
  eng.spareAlive = std::move(alive);
  eng.freeIds = std::move(freeIds);
  eng.exact = spf_graph_needs_exact(eng.graph) != 0;
  if (memoScreenEnabled() && !eng.exact) {
    const auto ts = std::chrono::steady_clock::now();
    for (int k = 0; k < 2; ++k) {
      std::remove_reference_t<decltype(eng.memo[0])> keep;
      screenMemo(eng.memo[k], keep, k ? dMetric : dHops);
      eng.memo[k] = std::move(keep);
    }
    Counters::add("decision.graph_memo_screen_us",
                  std::chrono::duration_cast<std::chrono::microseconds>(
                      std::chrono::steady_clock::now() - ts)
                      .count());
  } else {
    eng.memo[0].clear();
    eng.memo[1].clear();
  }
  for (auto& m : eng.prefetched) {
    m.clear();
  }
  eng.kthPrefetch.clear();
  eng.isolated.clear();
  Counters::add("decision.graph_inplace_link_patches", 1);
  Counters::add("decision.graph_patch_us",
                std::chrono::duration_cast<std::chrono::microseconds>(
                    std::chrono::steady_clock::now() - t0)
                    .count());
  return true;
}

void LinkState::addLink(std::shared_ptr<Link> link) {
  if (!linkMap_[link->firstNodeName()].insert(link).second ||
      !linkMap_[link->secondNodeName()].insert(link).second ||
      !allLinks_.insert(link).second) {
    throw CheckFailure("addLink: duplicate link " + link->toString());
  }
}

void LinkState::removeLink(std::shared_ptr<Link> link) {
  if (!linkMap_.at(link->firstNodeName()).erase(link) ||
      !linkMap_.at(link->secondNodeName()).erase(link) || !allLinks_.erase(link)) {
    throw CheckFailure("removeLink: missing link " + link->toString());
  }
}

void LinkState::removeNode(const std::string& nodeName) {
  auto it = linkMap_.find(nodeName);
  if (it == linkMap_.end()) {
    return; // an empty adjacency database created no links
  }
  for (const auto& link : it->second) {
    if (!linkMap_.at(link->getOtherNodeName(nodeName)).erase(link) ||
        !allLinks_.erase(link)) {
      throw CheckFailure("removeNode: inconsistent link set");
    }
  }
  linkMap_.erase(it);
  nodeOverloads_.erase(nodeName);
}

const LinkState::LinkSet& LinkState::linksFromNode(const std::string& nodeName) const {
  static const LinkSet kEmpty;
  auto it = linkMap_.find(nodeName);
  return it == linkMap_.end() ? kEmpty : it->second;
}

std::vector<std::shared_ptr<Link>> LinkState::orderedLinksFromNode(
    const std::string& nodeName) const {
  const auto& set = linksFromNode(nodeName);
  std::vector<std::shared_ptr<Link>> links(set.begin(), set.end());
  std::sort(links.begin(), links.end(), LinkPtrLess{});
  return links;
}

bool LinkState::updateNodeOverloaded(
    const std::string& nodeName,
    bool isOverloaded,
    LinkStateMetric holdUpTtl,
    LinkStateMetric holdDownTtl) {
  auto it = nodeOverloads_.find(nodeName);
  if (it == nodeOverloads_.end()) {
    // a new node is not a topology change by itself
    nodeOverloads_.emplace(nodeName, HoldableValue<bool>{isOverloaded});
    return false;
  }
  return it->second.updateValue(isOverloaded, holdUpTtl, holdDownTtl);
}

bool LinkState::isNodeOverloaded(const std::string& nodeName) const {
  auto it = nodeOverloads_.find(nodeName);
  return it != nodeOverloads_.end() && it->second.value();
}

LinkState::LinkStateChange LinkState::decrementHolds() {
  LinkStateChange change;
  for (const auto& link : allLinks_) {
    change.topologyChanged |= link->decrementHolds();
  }
  for (auto& kv : nodeOverloads_) {
    change.topologyChanged |= kv.second.decrementTtl();
  }
  if (change.topologyChanged) {
    clearMemo();
  }
  return change;
}

bool LinkState::hasHolds() const {
  for (const auto& link : allLinks_) {
    if (link->hasHolds()) {
      return true;
    }
  }
  for (const auto& kv : nodeOverloads_) {
    if (kv.second.hasHold()) {
      return true;
    }
  }
  return false;
}

std::shared_ptr<Link> LinkState::maybeMakeLink(
    const std::string& nodeName, const thrift::Adjacency& adj) const {
  // bidirectional only: the neighbour must advertise the mirror adjacency
  auto it = adjacencyDatabases_.find(adj.otherNodeName);
  if (it == adjacencyDatabases_.end()) {
    return nullptr;
  }
  for (const auto& mirror : it->second.adjacencies) {
    if (mirror.otherNodeName == nodeName && mirror.ifName == adj.otherIfName &&
        mirror.otherIfName == adj.ifName) {
      return std::make_shared<Link>(area_, nodeName, adj, adj.otherNodeName, mirror);
    }
  }
  return nullptr;
}

std::vector<std::shared_ptr<Link>> LinkState::getOrderedLinkSet(
    const thrift::AdjacencyDatabase& adjDb) const {
  std::vector<std::shared_ptr<Link>> links;
  links.reserve(adjDb.adjacencies.size());
  for (const auto& adj : adjDb.adjacencies) {
    if (auto link = maybeMakeLink(adjDb.thisNodeName, adj)) {
      links.push_back(std::move(link));
    }
  }
  std::sort(links.begin(), links.end(), LinkPtrLess{});
  return links;
}

LinkState::LinkStateChange LinkState::updateAdjacencyDatabase(
    thrift::AdjacencyDatabase const& newDb,
    LinkStateMetric holdUpTtl,
    LinkStateMetric holdDownTtl) {
  return updateAdjacencyDatabase(thrift::AdjacencyDatabase(newDb), holdUpTtl, holdDownTtl);
}

LinkState::LinkStateChange LinkState::updateAdjacencyDatabase(
    thrift::AdjacencyDatabase&& db,
    LinkStateMetric holdUpTtl,
    LinkStateMetric holdDownTtl) {
  LinkStateChange change;
  // the database moves into adjacencyDatabases_ (a decoded publication is
  // not copied a second time); newDb refers to the stored one
  auto slot = adjacencyDatabases_.try_emplace(db.thisNodeName).first;
  const std::string& nodeName = slot->first;
  thrift::AdjacencyDatabase priorDb(std::move(slot->second));
  slot->second = std::move(db);
  const thrift::AdjacencyDatabase& newDb = slot->second;

  // both sides sorted by Link::operator< so one merge pass finds the diff
  const auto oldLinks = orderedLinksFromNode(nodeName);
  const auto newLinks = getOrderedLinkSet(newDb);

  const bool transitChanged =
      updateNodeOverloaded(nodeName, newDb.isOverloaded, holdUpTtl, holdDownTtl);
  change.topologyChanged |= transitChanged;
  change.nodeLabelChanged = priorDb.nodeLabel != newDb.nodeLabel;
  // what the device graph needs: a rebuild when the set of up links changes,
  // else in-place transit / metric patches
  bool structural = false;
  std::vector<std::pair<std::shared_ptr<Link>, std::string>> metricPatches;
  std::vector<std::shared_ptr<Link>> downLinks, upLinks; // up-ness flips

  size_t ni = 0, oi = 0;
  while (ni < newLinks.size() || oi < oldLinks.size()) {
    const bool haveNew = ni < newLinks.size(), haveOld = oi < oldLinks.size();
    if (haveNew && (!haveOld || *newLinks[ni] < *oldLinks[oi])) {
      // link appears: keep it held down for holdUpTtl
      newLinks[ni]->setHoldUpTtl(holdUpTtl);
      change.topologyChanged |= newLinks[ni]->isUp();
      structural |= newLinks[ni]->isUp();
      if (newLinks[ni]->isUp()) {
        upLinks.push_back(newLinks[ni]);
      }
      addLink(newLinks[ni]);
      ++ni;
      continue;
    }
    if (haveOld && (!haveNew || *oldLinks[oi] < *newLinks[ni])) {
      // link disappears (a held or overloaded link was not carrying traffic)
      change.topologyChanged |= oldLinks[oi]->isUp();
      structural |= oldLinks[oi]->isUp();
      if (oldLinks[oi]->isUp()) {
        downLinks.push_back(oldLinks[oi]);
      }
      removeLink(oldLinks[oi]);
      ++oi;
      continue;
    }
    // same link: fold attribute changes into the existing Link object
    const Link& fresh = *newLinks[ni];
    Link& cur = *oldLinks[oi];
    const bool wasUp = cur.isUp();
    const LinkStateMetric oldMetric = cur.getMetricFromNode(nodeName);
    if (fresh.getMetricFromNode(nodeName) != cur.getMetricFromNode(nodeName)) {
      change.topologyChanged |= cur.setMetricFromNode(
          nodeName, fresh.getMetricFromNode(nodeName), holdUpTtl, holdDownTtl);
    }
    if (fresh.getOverloadFromNode(nodeName) != cur.getOverloadFromNode(nodeName)) {
      change.topologyChanged |= cur.setOverloadFromNode(
          nodeName, fresh.getOverloadFromNode(nodeName), holdUpTtl, holdDownTtl);
    }
    if (cur.isUp() != wasUp) {
      structural = true;
      (wasUp ? downLinks : upLinks).push_back(oldLinks[oi]);
    } else if (wasUp && cur.getMetricFromNode(nodeName) != oldMetric) {
      metricPatches.emplace_back(oldLinks[oi], nodeName);
    }
    if (fresh.getAdjLabelFromNode(nodeName) != cur.getAdjLabelFromNode(nodeName)) {
      change.linkAttributesChanged = true;
      cur.setAdjLabelFromNode(nodeName, fresh.getAdjLabelFromNode(nodeName));
    }
    if (fresh.getNhV4FromNode(nodeName) != cur.getNhV4FromNode(nodeName)) {
      change.linkAttributesChanged = true;
      cur.setNhV4FromNode(nodeName, fresh.getNhV4FromNode(nodeName));
    }
    if (fresh.getNhV6FromNode(nodeName) != cur.getNhV6FromNode(nodeName)) {
      change.linkAttributesChanged = true;
      cur.setNhV6FromNode(nodeName, fresh.getNhV6FromNode(nodeName));
    }
    ++ni;
    ++oi;
  }
  if (change.topologyChanged) {
    if (structural) {
      if (!patchStructure(
              downLinks, upLinks,
              transitChanged ? std::vector<std::string>{nodeName} : std::vector<std::string>{},
              metricPatches)) {
        clearMemo();
      }
    } else {
      patchMemo(
          transitChanged ? std::vector<std::string>{nodeName} : std::vector<std::string>{},
          metricPatches);
    }
  }
  return change;
}

LinkState::LinkStateChange LinkState::deleteAdjacencyDatabase(const std::string& nodeName) {
  LinkStateChange change;
  auto it = adjacencyDatabases_.find(nodeName);
  if (it != adjacencyDatabases_.end()) {
    removeNode(nodeName);
    adjacencyDatabases_.erase(it);
    clearMemo();
    change.topologyChanged = true;
  }
  return change;
}

bool LinkState::pathAInPathB(Path const& a, Path const& b) {
  if (a.size() > b.size()) {
    return false;
  }
  for (size_t start = 0; start + a.size() <= b.size(); ++start) {
    size_t k = 0;
    while (k < a.size() && *a[k] == *b[start + k]) {
      ++k;
    }
    if (k == a.size()) {
      return true;
    }
  }
  return false;
}

// ---------------------------------------------------------- SPF accessors

bool LinkState::linkHop(
    uint32_t linkId, uint32_t from, uint32_t& to, LinkStateMetric& metric) const {
  const auto& eng = engine();
  if (linkId >= eng.halves.size()) {
    return false;
  }
  const auto& h = eng.halves[linkId];
  if (h[0] == ~0u || h[1] == ~0u) {
    return false;
  }
  const uint32_t first = eng.col[h[1]], second = eng.col[h[0]];
  if (from == first) {
    to = second;
    metric = eng.metric[h[0]];
    return true;
  }
  if (from == second) {
    to = first;
    metric = eng.metric[h[1]];
    return true;
  }
  return false;
}

std::optional<uint32_t> LinkState::nodeId(const std::string& name) const {
  auto& eng = engine();
  auto it = eng.ids.find(name);
  if (it == eng.ids.end()) {
    return std::nullopt;
  }
  return it->second;
}

const std::string& LinkState::nodeNameOf(uint32_t id) const {
  return engine().names.at(id);
}

const std::vector<std::string>& LinkState::nodeNames() const {
  return engine().names;
}

uint32_t LinkState::numGraphNodes() const {
  return (uint32_t)engine().names.size();
}

float LinkState::lastDeviceMs() const {
  return engine_ ? engine_->lastMs : 0.0f;
}

const SpfView& LinkState::spfView(const std::string& node, bool useLinkMetric) const {
  auto& eng = engine();
  auto idIt = eng.ids.find(node);
  auto& memo = eng.memo[useLinkMetric ? 1 : 0];
  {
    std::shared_lock<std::shared_mutex> rd(eng.viewMu);
    if (idIt == eng.ids.end()) {
      auto it = eng.isolated.find(node);
      if (it != eng.isolated.end()) {
        return *it->second;
      }
    } else {
      auto it = memo.find(idIt->second);
      if (it != memo.end()) {
        return *it->second;
      }
    }
  }
  std::unique_lock<std::shared_mutex> wr(eng.viewMu);
  if (idIt == eng.ids.end()) {
    // unknown source: the reference result holds only the source itself
    auto& slot = eng.isolated[node];
    if (!slot) {
      slot = std::make_unique<SpfView>();
      slot->src = ~0u;
      slot->useLinkMetric = useLinkMetric;
      Counters::add("decision.spf_runs", 1);
    }
    return *slot;
  }
  const uint32_t id = idIt->second;
  auto it = memo.find(id);
  if (it != memo.end()) {
    return *it->second;
  }
  auto& pre = eng.prefetched[useLinkMetric ? 1 : 0];
  std::unique_ptr<SpfView> view;
  auto pit = pre.find(id);
  if (pit != pre.end()) {
    view = std::move(pit->second);
    pre.erase(pit);
  } else {
    const auto t0 = std::chrono::steady_clock::now();
    std::lock_guard<std::mutex> dev(eng.devMu);
    auto batch = runBatch(eng, {id}, useLinkMetric, true, nullptr);
    view = std::move(batch.front());
    Counters::add(
        "decision.spf_us",
        std::chrono::duration_cast<std::chrono::microseconds>(
            std::chrono::steady_clock::now() - t0)
            .count());
  }
  Counters::add("decision.spf_runs", 1);
  return *memo.emplace(id, std::move(view)).first->second;
}

void LinkState::prefetchSpf(const std::vector<std::string>& nodes, bool useLinkMetric) const {
  auto& eng = engine();
  std::unique_lock<std::shared_mutex> wr(eng.viewMu);
  std::lock_guard<std::mutex> dev(eng.devMu);
  auto& memo = eng.memo[useLinkMetric ? 1 : 0];
  auto& pre = eng.prefetched[useLinkMetric ? 1 : 0];
  std::vector<uint32_t> todo;
  std::unordered_set<uint32_t> seen;
  for (const auto& n : nodes) {
    auto it = eng.ids.find(n);
    if (it == eng.ids.end()) {
      continue;
    }
    const uint32_t id = it->second;
    if (memo.count(id) || pre.count(id) || !seen.insert(id).second) {
      continue;
    }
    todo.push_back(id);
  }
  if (todo.empty()) {
    return;
  }
  // the multi-GPU fan-out for big batches on the fast (32-bit) plans
  auto views = runBatchAuto(eng, todo, useLinkMetric, true, nullptr);
  for (size_t i = 0; i < todo.size(); ++i) {
    pre.emplace(todo[i], std::move(views[i]));
  }
}

LinkState::SpfResult const& LinkState::getSpfResult(
    const std::string& nodeName, bool useLinkMetric) const {
  auto& cache = useLinkMetric ? spfResultsMetric_ : spfResultsHops_;
  auto it = cache.find(nodeName);
  if (it != cache.end()) {
    return it->second;
  }
  const SpfView& view = spfView(nodeName, useLinkMetric);
  return cache.emplace(nodeName, materialize(view, nodeName)).first->second;
}

LinkState::SpfResult LinkState::materialize(const SpfView& view, const std::string& srcName) const {
  const auto& eng = *engine_;
  SpfResult res;
  if (view.src == ~0u) {
    res.emplace(srcName, NodeSpfResult(0));
    return res;
  }
  std::vector<std::pair<uint32_t, uint32_t>> preds;
  const uint32_t V = (uint32_t)eng.names.size();
  res.reserve(V);
  for (uint32_t v = 0; v < V; ++v) {
    if (!view.reached(v)) {
      continue;
    }
    NodeSpfResult r(view.dist[v]);
    pathLinksOf(eng, view, v, preds);
    for (const auto& [eu, u] : preds) {
      r.addPath(eng.links[eng.linkId[eu]], eng.names[u]);
    }
    view.forEachNextHop(v, [&](uint32_t h) { r.addNextHop(eng.names[h]); });
    res.emplace(eng.names[v], std::move(r));
  }
  return res;
}

std::unique_ptr<LinkState::SpfBatch> LinkState::runSpfBatch(
    const std::string& src, const std::vector<LinkSet>& linksToIgnore, bool useLinkMetric) const {
  auto& eng = engine();
  auto batch = std::make_unique<SpfBatch>();
  batch->ls_ = this;
  batch->gen_ = topoGen_;
  batch->src_ = src;
  const size_t nq = linksToIgnore.size();
  // one COUNT sample per SPF, as the reference's per-runSpf addStatValue
  Counters::addSamples("decision.spf_runs", (int64_t)nq, (int64_t)nq);
  auto sid = eng.ids.find(src);
  if (sid == eng.ids.end()) {
    // unknown source: every result holds only the source itself
    for (size_t i = 0; i < nq; ++i) {
      auto v = std::make_unique<SpfView>();
      v->src = ~0u;
      v->useLinkMetric = useLinkMetric;
      batch->views_.push_back(std::move(v));
    }
    return batch;
  }
  // ignore lists as sorted device link ids (links that are not up links of
  // this area cannot be relaxed anyway)
  std::vector<std::vector<uint32_t>> lists(nq);
  for (size_t i = 0; i < nq; ++i) {
    for (const auto& link : linksToIgnore[i]) {
      uint32_t li = eng.linkIdOf(link.get());
      if (li == ~0u) {
        // an equal Link object of this LinkState (the caller may hold a copy)
        auto own = allLinks_.find(link);
        if (own != allLinks_.end()) {
          li = eng.linkIdOf(own->get());
        }
      }
      if (li != ~0u) {
        lists[i].push_back(li);
      }
    }
    std::sort(lists[i].begin(), lists[i].end());
    lists[i].erase(std::unique(lists[i].begin(), lists[i].end()), lists[i].end());
  }
  std::vector<uint32_t> sources(nq, sid->second);
  {
    std::lock_guard<std::mutex> dev(eng.devMu);
    batch->views_ = runBatchAuto(eng, sources, useLinkMetric, true, &lists);
  }
  return batch;
}

LinkState::SpfResult LinkState::SpfBatch::result(size_t i) const {
  if (!ls_ || ls_->topoGen_ != gen_ || !ls_->engine_) {
    throw std::logic_error("SpfBatch::result: the topology changed since the batch ran");
  }
  return ls_->materialize(*views_.at(i), src_);
}

std::optional<LinkStateMetric> LinkState::getMetricFromAToB(
    std::string const& a, std::string const& b, bool useLinkMetric) const {
  if (a == b) {
    return 0;
  }
  const SpfView& view = spfView(a, useLinkMetric);
  if (view.src == ~0u) {
    return std::nullopt;
  }
  auto it = engine_->ids.find(b);
  if (it == engine_->ids.end() || !view.reached(it->second)) {
    return std::nullopt;
  }
  return view.dist[it->second];
}

LinkStateMetric LinkState::getMaxHopsToNode(const std::string& nodeName) const {
  const SpfView& view = spfView(nodeName, false);
  LinkStateMetric best = 0;
  for (size_t v = 0; v < view.dist.size(); ++v) {
    const uint64_t d = view.dist[v];
    if (d != SpfView::kUnreachable) {
      best = std::max(best, d);
    }
  }
  return best;
}

// The reference's greedy edge-disjoint DFS (traceOnePath, LinkState.cpp:
// 398-419), with two memos that keep its result and order exactly:
//  * preds: pathLinksOf(v) depends on the SPF result and v only, so it is
//    computed once per node per SPF view -- and kept across the getKthPaths
//    calls of one thread that trace over the same view (every k = 1 trace of
//    one source reads the source's own SPF), keyed by (view serial, topology
//    generation, engine).  A k = 2 trace runs over an ignore-list SPF that
//    differs from the source's own SPF at few nodes: pathLinksOf(v) reads
//    dist[v], the in-neighbours' dist and the ignore list at v only, so every
//    node whose dist, in-neighbours' dist and in-links all match the
//    source's SPF takes the source view's (cached) predecessors;
//  * dead: a node whose search failed has had every predecessor link
//    inserted into linksToIgnore (the loop only stops early on success, and
//    links are never removed), so any later search from it fails with no
//    side effect — return at once.  This turns the final, exhaustive search
//    of every call from O(visits x degree) into O(DAG).
// The reference's visited LinkSet (shared by the successive traces of one
// getKthPaths call, LinkState.cpp:776-786) is a link-id stamp array here:
// same membership, no hashing or allocation per link.
struct LinkState::TraceMemo {
  using Preds = std::vector<std::pair<uint32_t, uint32_t>>;
  // pathLinksOf of one view, per node, valid while stamp[v] == epoch
  struct PredCache {
    std::vector<uint32_t> stamp;
    std::vector<Preds> preds;
    uint32_t epoch = 0;
    uint64_t serial = 0, gen = 0;
    const void* eng = nullptr;
    void bind(uint32_t V, const SpfView& view, uint64_t g, const void* e) {
      if (stamp.size() != V) {
        stamp.assign(V, 0);
        preds.assign(V, {});
        epoch = 0;
        eng = nullptr;
      }
      if (view.serial != serial || g != gen || e != eng) {
        serial = view.serial;
        gen = g;
        eng = e;
        if (++epoch == 0) {
          std::fill(stamp.begin(), stamp.end(), 0);
          epoch = 1;
        }
      }
    }
    const Preds& get(const LinkState::Engine& en, const SpfView& view, uint32_t v) {
      if (stamp[v] != epoch) {
        pathLinksOf(en, view, v, preds[v]);
        stamp[v] = epoch;
      }
      return preds[v];
    }
  };
  PredCache own;  // the traced view
  PredCache base; // the source's own SPF (k >= 2 traces)
  const SpfView* baseView = nullptr;
  std::vector<uint32_t> visited; // == epoch: link id taken by some trace
  std::vector<uint32_t> dead;    // == epoch: search from v failed
  std::vector<uint32_t> changed; // == epoch: v does not take base's preds
  uint32_t epoch = 0;
  void reset(uint32_t V, uint32_t L, const SpfView& view, uint64_t gen, const void* eng) {
    if (visited.size() != L || dead.size() != V) {
      visited.assign(L, 0);
      dead.assign(V, 0);
      changed.assign(V, 0);
      epoch = 0;
    }
    own.bind(V, view, gen, eng);
    baseView = nullptr;
    if (++epoch == 0) {
      std::fill(visited.begin(), visited.end(), 0);
      std::fill(dead.begin(), dead.end(), 0);
      std::fill(changed.begin(), changed.end(), 0);
      epoch = 1;
    }
  }
  // trace `view` (an ignore-list SPF of the same source) with the source's
  // own SPF `src` as the base: mark the nodes whose predecessors may differ
  void useBase(const LinkState::Engine& en, const SpfView& view, const SpfView& src,
               uint64_t gen) {
    const uint32_t V = (uint32_t)dead.size();
    base.bind(V, src, gen, &en);
    baseView = &src;
    auto mark = [&](uint32_t x) {
      changed[x] = epoch;
      for (uint32_t e = en.row[x]; e < en.row[x + 1]; ++e) {
        changed[en.col[e]] = epoch; // x is an in-neighbour of col[e]
      }
    };
    const uint32_t* a = view.dist.raw32();
    const uint32_t* b = src.dist.raw32();
    if (a && b) {
      // the rows differ at few nodes: skip equal 256-byte chunks (memcmp)
      constexpr uint32_t kChunk = 64;
      for (uint32_t x0 = 0; x0 < V; x0 += kChunk) {
        const uint32_t n = std::min(kChunk, V - x0);
        if (std::memcmp(a + x0, b + x0, (size_t)n * sizeof(uint32_t)) == 0) {
          continue;
        }
        for (uint32_t x = x0; x < x0 + n; ++x) {
          if (a[x] != b[x]) {
            mark(x);
          }
        }
      }
    } else {
      for (uint32_t x = 0; x < V; ++x) {
        if (view.dist[x] != src.dist[x]) {
          mark(x);
        }
      }
    }
    for (const uint32_t lid : view.ignored) {
      for (const uint32_t h : en.halves[lid]) {
        if (h != ~0u) {
          changed[en.col[h]] = epoch;
          changed[en.col[en.rev[h]]] = epoch;
        }
      }
    }
  }
  const Preds& preds(const LinkState::Engine& en, const SpfView& view, uint32_t v) {
    if (baseView && changed[v] != epoch) {
      return base.get(en, *baseView, v);
    }
    return own.get(en, view, v);
  }
  bool take(uint32_t lid) {
    if (visited[lid] == epoch) {
      return false;
    }
    visited[lid] = epoch;
    return true;
  }
};

bool LinkState::traceOnePath(
    uint32_t src, uint32_t dest, const SpfView& result, TraceMemo& memo,
    std::vector<uint32_t>& links) const {
  // appends the path's links (src -> dest order) on success only
  if (src == dest) {
    return true;
  }
  if (memo.dead[dest] == memo.epoch) {
    return false;
  }
  const auto& eng = *engine_;
  const auto& preds = memo.preds(eng, result, dest);
  for (size_t i = 0; i < preds.size(); ++i) {
    const auto [eu, u] = preds[i];
    const uint32_t lid = eng.linkId[eu];
    if (memo.take(lid) && traceOnePath(src, u, result, memo, links)) {
      links.push_back(lid);
      return true;
    }
  }
  memo.dead[dest] = memo.epoch;
  return false;
}

const Link& LinkState::linkOfId(uint32_t id) const {
  return *engine().links.at(id);
}

const LinkState::KthPathIds& LinkState::kthPathIds(
    const std::string& src, const std::string& dest, size_t k) const {
  if (k < 1) {
    throw std::invalid_argument("getKthPaths: k must be >= 1");
  }
  KthKey key{src, dest, k};
  KthStripe& stripe = kthStripe(key);
  auto lookup = [&]() -> const KthPathIds* {
    std::shared_lock<std::shared_mutex> rd(stripe.mu);
    auto found = stripe.ids.find(key);
    return found == stripe.ids.end() ? nullptr : &found->second;
  };
  if (auto hit = lookup()) {
    return *hit;
  }
  // linksToIgnore of the reference (LinkState.cpp:766-775): the sorted ids
  // of the links on the paths of ranks < k.  Filled BEFORE this key's fill
  // lock is taken, so a fill never holds a lock while it recurses (every
  // k >= 3 shares one fill lock; k = 4 recursing into k = 3 under it would
  // lock it twice on one thread).
  std::vector<uint32_t> ign;
  for (size_t i = 1; i < k; ++i) {
    const auto& lower = kthPathIds(src, dest, i);
    ign.insert(ign.end(), lower.links.begin(), lower.links.end());
  }
  // once-only fill: concurrent callers of the same key wait for the first
  std::mutex& fillMu = k == 1 ? kthFill_->k1[KthKeyHash{}(key) % KthFillLocks::kStripes]
      : k == 2 ? kthFill_->k2[KthKeyHash{}(key) % KthFillLocks::kStripes]
               : kthFill_->kN;
  std::lock_guard<std::mutex> fill(fillMu);
  if (auto hit = lookup()) {
    return *hit;
  }
  auto& eng = engine();
  const bool anyLink = !ign.empty();
  std::sort(ign.begin(), ign.end());
  ign.erase(std::unique(ign.begin(), ign.end()), ign.end());
  KthPathIds paths;
  const SpfView* res = nullptr;
  std::unique_ptr<SpfView> second;
  if (!anyLink) {
    res = &spfView(src, true);
  } else {
    auto sid = eng.ids.find(src);
    if (sid != eng.ids.end()) {
      auto did = eng.ids.find(dest);
      if (did != eng.ids.end()) {
        // only this key's fill holder takes its prefetched view, and
        // kthPrefetch changes shape only under the exclusive lock: moving the
        // view out (the emptied entry stays) needs the shared lock alone
        std::shared_lock<std::shared_mutex> rd(eng.viewMu);
        auto pit = eng.kthPrefetch.find({sid->second, did->second});
        if (pit != eng.kthPrefetch.end() && pit->second && pit->second->ignored == ign) {
          second = std::move(pit->second);
        }
      }
      if (!second) {
        std::vector<std::vector<uint32_t>> lists{ign};
        std::lock_guard<std::mutex> dev(eng.devMu);
        second = std::move(runBatch(eng, {sid->second}, true, false, &lists).front());
      }
      res = second.get();
    }
    Counters::add("decision.spf_runs", 1);
  }
  const auto tTrace = std::chrono::steady_clock::now();
  if (res && res->src != ~0u) {
    auto did = eng.ids.find(dest);
    if (did != eng.ids.end() && res->reached(did->second)) {
      thread_local TraceMemo memo;
      memo.reset((uint32_t)eng.names.size(), (uint32_t)eng.links.size(), *res, topoGen_, &eng);
      if (second && !second->exact && second->okey.empty() && second->useLinkMetric) {
        // the source's own SPF, if memoized (looking it up runs nothing)
        const SpfView* own = nullptr;
        {
          std::shared_lock<std::shared_mutex> rd(eng.viewMu);
          auto it = eng.memo[1].find(res->src);
          if (it != eng.memo[1].end()) {
            own = it->second.get();
          }
        }
        if (own && !own->exact && own->okey.empty() && own->useLinkMetric &&
            own->ignored.empty() &&
            own->src == res->src && own->dist.size() == res->dist.size()) {
          const auto tBase = std::chrono::steady_clock::now();
          memo.useBase(eng, *res, *own, topoGen_);
          Counters::add("decision.kth2_base_us",
                        std::chrono::duration_cast<std::chrono::microseconds>(
                            std::chrono::steady_clock::now() - tBase)
                            .count());
        }
      }
      // successive traces until one fails or is empty (src == dest)
      for (;;) {
        const size_t before = paths.links.size();
        if (!traceOnePath(res->src, did->second, *res, memo, paths.links) ||
            paths.links.size() == before) {
          break;
        }
        paths.off.push_back((uint32_t)paths.links.size());
      }
    }
  }
  if (k >= 2) {
    // summed over the calling threads
    Counters::add("decision.kth2_trace_us",
                  std::chrono::duration_cast<std::chrono::microseconds>(
                      std::chrono::steady_clock::now() - tTrace)
                      .count());
  }
  std::unique_lock<std::shared_mutex> wr(stripe.mu);
  return stripe.ids.emplace(std::move(key), std::move(paths)).first->second;
}

std::vector<LinkState::Path> const& LinkState::getKthPaths(
    const std::string& src, const std::string& dest, size_t k) const {
  const KthPathIds& ids = kthPathIds(src, dest, k);
  KthKey key{src, dest, k};
  KthStripe& stripe = kthStripe(key);
  {
    std::shared_lock<std::shared_mutex> rd(stripe.mu);
    auto found = stripe.paths.find(key);
    if (found != stripe.paths.end()) {
      return found->second;
    }
  }
  const auto& eng = engine();
  std::vector<Path> paths(ids.size());
  for (size_t i = 0; i < ids.size(); ++i) {
    for (const uint32_t* l = ids.begin(i); l != ids.end(i); ++l) {
      paths[i].push_back(eng.links[*l]);
    }
  }
  std::unique_lock<std::shared_mutex> wr(stripe.mu);
  return stripe.paths.emplace(std::move(key), std::move(paths)).first->second;
}

void LinkState::prefetchKthPaths(
    const std::string& src, const std::vector<std::string>& dests) const {
  const auto tAll = std::chrono::steady_clock::now();
  auto& eng = engine();
  auto sid = eng.ids.find(src);
  if (sid == eng.ids.end()) {
    return;
  }
  // destinations whose second pass is still to run: the name and memo
  // lookups on the host pool (~230 ns each serially: 2.3 ms for the
  // fabric's 9,975), then the duplicates dropped in order
  std::vector<std::pair<const std::string*, uint32_t>> todo;
  {
    std::shared_lock<std::shared_mutex> rv(eng.viewMu); // (held for the workers too)
    const size_t n = dests.size();
    std::vector<uint32_t> idOf(n, ~0u); // ~0u: unknown node, or nothing to run
    parallelFor(n, hostThreads(n, 256), [&](size_t i, unsigned) {
      const auto& d = dests[i];
      auto did = eng.ids.find(d);
      if (did == eng.ids.end()) {
        return;
      }
      const KthKey k2{src, d, 2};
      KthStripe& stripe = kthStripe(k2);
      bool known;
      {
        std::shared_lock<std::shared_mutex> rk(stripe.mu);
        known = stripe.ids.count(k2) > 0;
      }
      auto pf = eng.kthPrefetch.find({sid->second, did->second});
      if (!known && !(pf != eng.kthPrefetch.end() && pf->second)) {
        idOf[i] = did->second;
      }
    }, 64);
    std::vector<uint8_t> seen(eng.names.size(), 0);
    for (size_t i = 0; i < n; ++i) {
      if (idOf[i] != ~0u && !seen[idOf[i]]) {
        seen[idOf[i]] = 1;
        todo.emplace_back(&dests[i], idOf[i]);
      }
    }
  }
  if (todo.empty()) {
    return;
  }
  Counters::add("decision.kth_todo_us", std::chrono::duration_cast<std::chrono::microseconds>(
                                            std::chrono::steady_clock::now() - tAll)
                                            .count());
  spfView(src, true); // every k = 1 trace reads the source's own SPF
  // k = 1 paths of every destination (independent traces over the same
  // row: host worker pool), then their links as the ignore lists
  std::vector<std::vector<uint32_t>> ignAll(todo.size());
  const auto tTrace = std::chrono::steady_clock::now();
  parallelFor(todo.size(), hostThreads(todo.size(), 32), [&](size_t i, unsigned) {
    auto& ign = ignAll[i];
    ign = kthPathIds(src, *todo[i].first, 1).links;
    std::sort(ign.begin(), ign.end());
    ign.erase(std::unique(ign.begin(), ign.end()), ign.end());
  });
  Counters::add("decision.kth_trace_us",
                std::chrono::duration_cast<std::chrono::microseconds>(
                    std::chrono::steady_clock::now() - tTrace)
                    .count());
  std::vector<uint32_t> sources;
  std::vector<uint32_t> dstIds;
  std::vector<std::vector<uint32_t>> lists;
  for (size_t i = 0; i < todo.size(); ++i) {
    if (ignAll[i].empty()) {
      continue;
    }
    sources.push_back(sid->second);
    dstIds.push_back(todo[i].second);
    lists.push_back(std::move(ignAll[i]));
  }
  if (sources.empty()) {
    return;
  }
  std::vector<std::unique_ptr<SpfView>> views;
  bool traced = false;
  if (!eng.exact && deviceTraceEnabled()) {
    // second passes AND their traces on the device (fanned out by
    // destination when devices are configured): the (src, dst, 2) memo
    // entries are filled here, as the fill in kthPathIds would (one counted
    // runSpf each, LinkState.cpp:776-777); overflowed traces keep their row
    // for the host trace
    DeviceTraces tr;
    const auto tDev = std::chrono::steady_clock::now();
    {
      std::lock_guard<std::mutex> dev(eng.devMu);
      tr = traceSecondPasses(eng, sources, dstIds, lists);
    }
    const auto tFill = std::chrono::steady_clock::now();
    Counters::add("decision.kth_lists_us",
                  std::chrono::duration_cast<std::chrono::microseconds>(tDev - tTrace).count());
    traced = !tr.unsupported;
    if (!traced) {
      tr.count.clear();
    }
    // the (src, dst, 2) entries: offsets serially, then one host-pool task
    // per memo stripe (9,975 fills on the fabric; serially they were ~15 ms)
    struct Fill {
      const std::string* dst;
      size_t i, lo, po;
    };
    std::vector<std::vector<Fill>> byStripe(kKthStripes);
    size_t j = 0, lo = 0, po = 0;
    uint64_t overflowed = 0;
    for (size_t i = 0; i < tr.count.size(); ++i) {
      if (tr.count[i] == SPF_TRACE_OVERFLOW) {
        ++overflowed;
        continue;
      }
      while (todo[j].second != dstIds[i]) {
        ++j; // todo and dstIds are in the same order (dstIds skips entries)
      }
      const std::string* dstName = todo[j].first;
      const size_t st = KthKeyHash{}(KthKey{src, *dstName, 2}) % kKthStripes;
      byStripe[st].push_back({dstName, i, lo, po});
      lo += tr.linkCount[i];
      po += tr.count[i];
    }
    std::atomic<int64_t> filled{0};
    parallelFor(kKthStripes, hostThreads(tr.count.size(), 256), [&](size_t st, unsigned) {
      KthStripe& stripe = (*kth_)[st];
      int64_t n = 0;
      std::unique_lock<std::shared_mutex> wr(stripe.mu);
      for (const Fill& f : byStripe[st]) {
        KthPathIds paths;
        const uint32_t* L = tr.links.data() + f.lo;
        const uint32_t* E = tr.ends.data() + f.po;
        paths.links.assign(L, L + tr.linkCount[f.i]);
        paths.off.reserve(tr.count[f.i] + 1);
        for (uint32_t p = 0; p < tr.count[f.i]; ++p) {
          paths.off.push_back(E[p]);
        }
        n += stripe.ids.emplace(KthKey{src, *f.dst, 2}, std::move(paths)).second ? 1 : 0;
      }
      filled += n;
    }, 1);
    // one COUNT sample per SPF, as the per-entry add(1) of the fill
    Counters::addSamples("decision.spf_runs", filled.load(), filled.load());
    Counters::add("decision.kth_fill_us", std::chrono::duration_cast<std::chrono::microseconds>(
                                              std::chrono::steady_clock::now() - tFill)
                                              .count());
    if (traced) {
      views = std::move(tr.rows);
      Counters::add("decision.kth2_device_traces", (int64_t)(tr.count.size() - overflowed));
      Counters::add("decision.kth2_device_overflows", (int64_t)overflowed);
    }
  }
  if (!traced) {
    // the second passes of many destinations: fanned out by destination
    // when devices are configured (distances only: a trace reads no masks)
    std::lock_guard<std::mutex> dev(eng.devMu);
    views = runBatchAuto(eng, sources, true, false, &lists);
  }
  std::unique_lock<std::shared_mutex> wr(eng.viewMu);
  for (size_t i = 0; i < views.size(); ++i) {
    if (views[i]) {
      eng.kthPrefetch[{sid->second, dstIds[i]}] = std::move(views[i]);
    }
  }
}

} // namespace openr

size_t std::hash<openr::LinkState::LinkSet>::operator()(
    openr::LinkState::LinkSet const& set) const {
  size_t h = 0;
  for (const auto& link : set) {
    h ^= link->hash; // order independent
  }
  return h;
}

bool std::equal_to<openr::LinkState::LinkSet>::operator()(
    openr::LinkState::LinkSet const& a, openr::LinkState::LinkSet const& b) const {
  if (a.size() != b.size()) {
    return false;
  }
  for (const auto& l : a) {
    if (!b.count(l)) {
      return false;
    }
  }
  return true;
}
