// Types.h — plain-C++ equivalents of the fbthrift structs the Decision SPF
// path reads and writes.  Field names, defaults and optional-ness follow the
// IDL so that code written against the reference's generated types compiles
// against these unchanged:
//   Adjacency / AdjacencyDatabase        openr/if/Lsdb.thrift:70-128
//   MetricEntity / MetricVector           openr/if/Lsdb.thrift:183-213
//   PrefixEntry / PrefixDatabase          openr/if/Lsdb.thrift:271-352
//   MplsAction / BinaryAddress / IpPrefix /
//   NextHopThrift / MplsRoute / UnicastRoute  openr/if/Network.thrift:46-133
//   RouteDatabase                         openr/if/Fib.thrift:18-32
//   PrefixEntries                         openr/if/Decision.thrift:32-37
// Generated-code conventions kept: `==` over all fields (an optional equals
// another when both are unset or both set and equal) and lexicographic `<`.
#pragma once

#include <cstdint>
#include <cstring>
#include <functional>
#include <new>
#include <ostream>
#include <string_view>
#include <map>
#include <optional>
#include <set>
#include <stdexcept>
#include <string>
#include <tuple>
#include <unordered_map>
#include <unordered_set>
#include <vector>

namespace openr {

// String value with the bytes inline up to 30 characters (heap beyond): the
// IPv6 next-hop addresses (16 bytes) and interface names ("if_3-172-45_2-
// 172-0", 19) of every NextHopThrift would each be one heap block in a
// std::string (15-byte SSO), and a fabric RouteDb holds ~1.6M of them, built
// per build and freed per release.  Same bytes, comparisons and std::hash
// value as the std::string it replaces; converts to std::string implicitly.
class SmallString {
 public:
  static constexpr size_t kInline = 30;
  SmallString() noexcept { buf_[0] = 0; n_ = 0; }
  SmallString(const char* p, size_t n) { init(p, n); }
  SmallString(const char* p) : SmallString(p, std::strlen(p)) {} // NOLINT
  SmallString(const std::string& s) : SmallString(s.data(), s.size()) {} // NOLINT
  SmallString(std::string_view s) : SmallString(s.data(), s.size()) {} // NOLINT
  SmallString(size_t n, char c) {
    init(nullptr, n);
    std::memset(mut(), c, n);
  }
  SmallString(const SmallString& o) {
    if (o.n_ != kHeap) {
      std::memcpy(this, &o, sizeof(SmallString));
    } else {
      init(o.data(), o.size());
    }
  }
  SmallString(SmallString&& o) noexcept {
    std::memcpy(this, &o, sizeof(SmallString));
    o.buf_[0] = 0;
    o.n_ = 0;
  }
  SmallString& operator=(const SmallString& o) {
    if (this != &o) {
      release();
      new (this) SmallString(o);
    }
    return *this;
  }
  SmallString& operator=(SmallString&& o) noexcept {
    if (this != &o) {
      release();
      new (this) SmallString(std::move(o));
    }
    return *this;
  }
  SmallString& operator=(const std::string& s) {
    release();
    init(s.data(), s.size());
    return *this;
  }
  SmallString& operator=(const char* p) {
    // p may point into this string's own buffer (s = s.c_str()): copy first
    SmallString tmp(p, std::strlen(p));
    return *this = std::move(tmp);
  }
  ~SmallString() { release(); }

  size_t size() const noexcept { return n_ == kHeap ? heapLen() : n_; }
  size_t length() const noexcept { return size(); }
  bool empty() const noexcept { return size() == 0; }
  const char* data() const noexcept { return n_ == kHeap ? heapPtr() : buf_; }
  const char* c_str() const noexcept { return data(); }
  const char* begin() const noexcept { return data(); }
  const char* end() const noexcept { return data() + size(); }
  char operator[](size_t i) const { return data()[i]; }
  char& operator[](size_t i) { return mut()[i]; }
  std::string_view view() const noexcept { return {data(), size()}; }
  std::string str() const { return std::string(data(), size()); }
  operator std::string() const { return str(); } // NOLINT
  int compare(const SmallString& o) const noexcept { return view().compare(o.view()); }
  SmallString& assign(const char* p, size_t n) {
    SmallString t(p, n);
    return *this = std::move(t);
  }

  friend bool operator==(const SmallString& a, const SmallString& b) noexcept {
    return a.view() == b.view();
  }
  friend bool operator!=(const SmallString& a, const SmallString& b) noexcept { return !(a == b); }
  friend bool operator<(const SmallString& a, const SmallString& b) noexcept {
    return a.view() < b.view();
  }
  friend bool operator==(const SmallString& a, const std::string& b) noexcept {
    return a.view() == std::string_view(b);
  }
  friend bool operator==(const std::string& a, const SmallString& b) noexcept { return b == a; }
  friend bool operator!=(const SmallString& a, const std::string& b) noexcept { return !(a == b); }
  friend bool operator!=(const std::string& a, const SmallString& b) noexcept { return !(b == a); }
  friend bool operator==(const SmallString& a, const char* b) noexcept {
    return a.view() == std::string_view(b);
  }
  friend bool operator!=(const SmallString& a, const char* b) noexcept { return !(a == b); }
  friend std::string operator+(const std::string& a, const SmallString& b) {
    return a + b.str();
  }
  friend std::string operator+(const SmallString& a, const std::string& b) {
    return a.str() + b;
  }
  friend std::string operator+(const char* a, const SmallString& b) { return a + b.str(); }
  friend std::string operator+(const SmallString& a, const char* b) { return a.str() + b; }

 private:
  static constexpr uint8_t kHeap = 255;
  char buf_[31]; // inline bytes + NUL, or {char* ptr; size_t len} when n_ == kHeap
  uint8_t n_;
  const char* heapPtr() const noexcept {
    const char* p;
    std::memcpy(&p, buf_, sizeof p);
    return p;
  }
  size_t heapLen() const noexcept {
    size_t n;
    std::memcpy(&n, buf_ + sizeof(char*), sizeof n);
    return n;
  }
  char* mut() noexcept { return n_ == kHeap ? const_cast<char*>(heapPtr()) : buf_; }
  void init(const char* p, size_t n) {
    if (n <= kInline) {
      if (p) {
        std::memcpy(buf_, p, n);
      }
      buf_[n] = 0;
      n_ = (uint8_t)n;
      return;
    }
    char* h = new char[n + 1];
    if (p) {
      std::memcpy(h, p, n);
    }
    h[n] = 0;
    std::memcpy(buf_, &h, sizeof h);
    std::memcpy(buf_ + sizeof(char*), &n, sizeof n);
    n_ = kHeap;
  }
  void release() noexcept {
    if (n_ == kHeap) {
      delete[] heapPtr();
      n_ = 0;
      buf_[0] = 0;
    }
  }
};

inline std::ostream& operator<<(std::ostream& os, const SmallString& s) { return os << s.view(); }

// A reference CHECK on the path failed (glog CHECK aborts the daemon there,
// e.g. LinkState.cpp:423-433; thrown here and never swallowed as a
// per-key or per-prefix error).
struct CheckFailure : std::logic_error {
  using std::logic_error::logic_error;
};

namespace thrift {

enum class PrefixType : int32_t {
  LOOPBACK = 1,
  DEFAULT = 2,
  BGP = 3,
  PREFIX_ALLOCATOR = 4,
  BREEZE = 5,
  RIB = 6,
  TYPE_1 = 21,
  TYPE_2 = 22,
  TYPE_3 = 23,
  TYPE_4 = 24,
  TYPE_5 = 25,
};

enum class PrefixForwardingType : int32_t { IP = 0, SR_MPLS = 1 };
enum class PrefixForwardingAlgorithm : int32_t { SP_ECMP = 0, KSP2_ED_ECMP = 1 };
enum class MplsActionCode : int32_t {
  PUSH = 0,
  SWAP = 1,
  PHP = 2,
  POP_AND_LOOKUP = 3,
  NOOP = 4,
};
enum class CompareType : int32_t {
  WIN_IF_PRESENT = 1,
  WIN_IF_NOT_PRESENT = 2,
  IGNORE_IF_NOT_PRESENT = 3,
};

struct BinaryAddress {
  SmallString addr; // 4 / 16 raw bytes
  std::optional<SmallString> ifName;
  auto tie() const { return std::tie(addr, ifName); }
  bool operator==(const BinaryAddress& o) const { return tie() == o.tie(); }
  bool operator!=(const BinaryAddress& o) const { return !(*this == o); }
  bool operator<(const BinaryAddress& o) const { return tie() < o.tie(); }
};

struct IpPrefix {
  BinaryAddress prefixAddress;
  int16_t prefixLength{0};
  auto tie() const { return std::tie(prefixAddress, prefixLength); }
  bool operator==(const IpPrefix& o) const { return tie() == o.tie(); }
  bool operator!=(const IpPrefix& o) const { return !(*this == o); }
  bool operator<(const IpPrefix& o) const { return tie() < o.tie(); }
};

struct MplsAction {
  MplsActionCode action{MplsActionCode::PUSH};
  std::optional<int32_t> swapLabel;
  std::optional<std::vector<int32_t>> pushLabels;
  auto tie() const { return std::tie(action, swapLabel, pushLabels); }
  bool operator==(const MplsAction& o) const { return tie() == o.tie(); }
  bool operator!=(const MplsAction& o) const { return !(*this == o); }
  bool operator<(const MplsAction& o) const { return tie() < o.tie(); }
};

struct NextHopThrift {
  BinaryAddress address;
  int32_t weight{0};
  std::optional<MplsAction> mplsAction;
  int32_t metric{0};
  bool useNonShortestRoute{false};
  std::optional<std::string> area;
  auto tie() const {
    return std::tie(
        address, weight, mplsAction, metric, useNonShortestRoute, area);
  }
  bool operator==(const NextHopThrift& o) const { return tie() == o.tie(); }
  bool operator!=(const NextHopThrift& o) const { return !(*this == o); }
  bool operator<(const NextHopThrift& o) const { return tie() < o.tie(); }
};

struct Adjacency {
  std::string otherNodeName;
  std::string ifName;
  BinaryAddress nextHopV6;
  BinaryAddress nextHopV4;
  int32_t metric{0};
  int32_t adjLabel{0};
  bool isOverloaded{false};
  int32_t rtt{0};
  int64_t timestamp{0};
  int64_t weight{1};
  std::string otherIfName;
  auto tie() const {
    return std::tie(
        otherNodeName, ifName, nextHopV6, nextHopV4, metric, adjLabel,
        isOverloaded, rtt, timestamp, weight, otherIfName);
  }
  bool operator==(const Adjacency& o) const { return tie() == o.tie(); }
  bool operator!=(const Adjacency& o) const { return !(*this == o); }
};

struct AdjacencyDatabase {
  std::string thisNodeName;
  bool isOverloaded{false};
  std::vector<Adjacency> adjacencies;
  int32_t nodeLabel{0};
  std::string area;
  auto tie() const {
    return std::tie(thisNodeName, isOverloaded, adjacencies, nodeLabel, area);
  }
  bool operator==(const AdjacencyDatabase& o) const { return tie() == o.tie(); }
};

struct MetricEntity {
  int64_t type{0};
  int64_t priority{0};
  CompareType op{CompareType::WIN_IF_PRESENT};
  bool isBestPathTieBreaker{false};
  std::vector<int64_t> metric;
  auto tie() const {
    return std::tie(type, priority, op, isBestPathTieBreaker, metric);
  }
  bool operator==(const MetricEntity& o) const { return tie() == o.tie(); }
  bool operator<(const MetricEntity& o) const { return tie() < o.tie(); }
};

struct MetricVector {
  int64_t version{0};
  std::vector<MetricEntity> metrics;
  auto tie() const { return std::tie(version, metrics); }
  bool operator==(const MetricVector& o) const { return tie() == o.tie(); }
  bool operator<(const MetricVector& o) const { return tie() < o.tie(); }
};

struct PrefixEntry {
  IpPrefix prefix;
  PrefixType type{PrefixType::LOOPBACK};
  std::optional<std::string> data;
  PrefixForwardingType forwardingType{PrefixForwardingType::IP};
  PrefixForwardingAlgorithm forwardingAlgorithm{
      PrefixForwardingAlgorithm::SP_ECMP};
  std::optional<bool> ephemeral;
  std::optional<MetricVector> mv;
  std::optional<int64_t> minNexthop;
  std::optional<int32_t> prependLabel;
  auto tie() const {
    return std::tie(
        prefix, type, data, forwardingType, forwardingAlgorithm, ephemeral, mv,
        minNexthop, prependLabel);
  }
  bool operator==(const PrefixEntry& o) const { return tie() == o.tie(); }
  bool operator!=(const PrefixEntry& o) const { return !(*this == o); }
};

struct PrefixDatabase {
  std::string thisNodeName;
  std::vector<PrefixEntry> prefixEntries;
  bool deletePrefix{false};
  std::string area{"0"};
};

using PrefixEntriesByAreaId = std::map<std::string /* area */, PrefixEntry>;
using PrefixEntries = std::map<std::string /* node */, PrefixEntriesByAreaId>;

struct UnicastRoute {
  IpPrefix dest;
  std::vector<NextHopThrift> nextHops;
  std::optional<PrefixType> prefixType;
  std::optional<std::string> data;
  bool doNotInstall{false};
  std::optional<NextHopThrift> bestNexthop;
};

struct MplsRoute {
  int32_t topLabel{0};
  std::vector<NextHopThrift> nextHops;
};

struct RouteDatabase {
  std::string thisNodeName;
  std::vector<UnicastRoute> unicastRoutes;
  std::vector<MplsRoute> mplsRoutes;
};

struct StaticRoutes {
  std::unordered_map<int32_t, std::vector<NextHopThrift>> mplsRoutes;
};

struct RouteDatabaseDelta {
  std::vector<MplsRoute> mplsRoutesToUpdate;
  std::vector<int32_t> mplsRoutesToDelete;
};

inline const std::string&
kDefaultArea() {
  static const std::string area{"0"};
  return area;
}

} // namespace thrift

namespace detail {
inline size_t
mix(size_t seed, size_t v) {
  // boost-style combine; only bucket placement depends on it
  return seed ^ (v + 0x9e3779b97f4a7c15ull + (seed << 6) + (seed >> 2));
}
} // namespace detail
} // namespace openr

namespace std {
template <>
struct hash<openr::SmallString> {
  size_t operator()(const openr::SmallString& s) const noexcept {
    return std::hash<std::string_view>()(s.view()); // == std::hash<std::string>
  }
};
template <>
struct hash<openr::thrift::BinaryAddress> {
  size_t operator()(const openr::thrift::BinaryAddress& a) const {
    size_t h = std::hash<openr::SmallString>()(a.addr);
    if (a.ifName) {
      h = openr::detail::mix(h, std::hash<openr::SmallString>()(*a.ifName));
    }
    return h;
  }
};
template <>
struct hash<openr::thrift::IpPrefix> {
  size_t operator()(const openr::thrift::IpPrefix& p) const {
    return openr::detail::mix(
        std::hash<openr::thrift::BinaryAddress>()(p.prefixAddress),
        (size_t)p.prefixLength);
  }
};
template <>
struct hash<openr::thrift::MplsAction> {
  size_t operator()(const openr::thrift::MplsAction& a) const {
    size_t h = (size_t)a.action;
    if (a.swapLabel) {
      h = openr::detail::mix(h, (size_t)*a.swapLabel);
    }
    if (a.pushLabels) {
      for (auto l : *a.pushLabels) {
        h = openr::detail::mix(h, (size_t)l);
      }
    }
    return h;
  }
};
template <>
struct hash<openr::thrift::NextHopThrift> {
  size_t operator()(const openr::thrift::NextHopThrift& n) const {
    size_t h = std::hash<openr::thrift::BinaryAddress>()(n.address);
    h = openr::detail::mix(h, (size_t)n.weight);
    h = openr::detail::mix(h, (size_t)n.metric);
    if (n.mplsAction) {
      h = openr::detail::mix(
          h, std::hash<openr::thrift::MplsAction>()(*n.mplsAction));
    }
    return h;
  }
};
} // namespace std
