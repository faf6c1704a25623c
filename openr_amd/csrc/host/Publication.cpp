// Publication.cpp — CompactProtocol reader / writer for the Decision path's
// structs and Decision::processPublication.  See Publication.h.
//
// Wire format (fbthrift CompactProtocol, the serializer Decision uses):
//   field header  one byte (id delta << 4 | type) when 0 < delta <= 15, else
//                 the type byte followed by the zigzag-varint i16 field id;
//                 booleans live in the type nibble (1 true, 2 false); 0 = stop
//   i16/i32/i64   zigzag varint; double 8 bytes; binary/string varint length
//   list/set      one byte (size << 4 | elem type) when size < 15, else
//                 0xF0 | elem type followed by a varint size
//   map           varint size, then (key type << 4 | value type) if size > 0
// Unknown fields, and known ids carrying an unexpected type, are skipped.
#include "Publication.h"

#include <arpa/inet.h>

#include <cstring>

namespace openr {
namespace compact {
namespace {

enum : uint8_t {
  kStop = 0,
  kTrue = 1,
  kFalse = 2,
  kByte = 3,
  kI16 = 4,
  kI32 = 5,
  kI64 = 6,
  kDouble = 7,
  kBinary = 8,
  kList = 9,
  kSet = 10,
  kMap = 11,
  kStruct = 12,
};

constexpr int kMaxDepth = 64;

class Reader {
 public:
  explicit Reader(std::string_view b)
      : p_(reinterpret_cast<const uint8_t*>(b.data())), end_(p_ + b.size()) {}

  uint8_t byte() {
    if (p_ >= end_) {
      throw DecodeError("truncated input");
    }
    return *p_++;
  }
  uint64_t varint() {
    uint64_t r = 0;
    for (int s = 0; s < 64; s += 7) {
      const uint8_t b = byte();
      r |= (uint64_t)(b & 0x7f) << s;
      if (!(b & 0x80)) {
        return r;
      }
    }
    throw DecodeError("varint longer than 10 bytes");
  }
  int64_t zz() {
    const uint64_t v = varint();
    return (int64_t)(v >> 1) ^ -(int64_t)(v & 1);
  }
  std::string binary() {
    const uint64_t n = varint();
    if (n > (uint64_t)(end_ - p_)) {
      throw DecodeError("binary length past the end");
    }
    std::string s(reinterpret_cast<const char*>(p_), n);
    p_ += n;
    return s;
  }
  // next field of the current struct; false at its stop byte
  bool field(int16_t& last, int16_t& id, uint8_t& type) {
    const uint8_t b = byte();
    if (b == kStop) {
      return false;
    }
    type = b & 0x0f;
    const uint8_t d = b >> 4;
    id = d ? (int16_t)(last + d) : (int16_t)zz();
    last = id;
    return true;
  }
  // list / set header: element type and size
  uint32_t list(uint8_t& et) {
    const uint8_t b = byte();
    et = b & 0x0f;
    uint64_t n = b >> 4;
    if (n == 15) {
      n = varint();
    }
    if (n > (uint64_t)(end_ - p_)) { // every element takes >= 1 byte
      throw DecodeError("list size past the end");
    }
    return (uint32_t)n;
  }
  void skip(uint8_t type, int depth) {
    if (depth > kMaxDepth) {
      throw DecodeError("nesting too deep");
    }
    switch (type) {
    case kTrue:
    case kFalse:
    case kByte:
      byte(); // booleans inside containers take one byte
      return;
    case kI16:
    case kI32:
    case kI64:
      varint();
      return;
    case kDouble:
      for (int i = 0; i < 8; ++i) {
        byte();
      }
      return;
    case kBinary:
      binary();
      return;
    case kList:
    case kSet: {
      uint8_t et;
      const uint32_t n = list(et);
      for (uint32_t i = 0; i < n; ++i) {
        skip(et, depth + 1);
      }
      return;
    }
    case kMap: {
      const uint64_t n = varint();
      if (n == 0) {
        return;
      }
      const uint8_t kv = byte();
      for (uint64_t i = 0; i < n; ++i) {
        skip(kv >> 4, depth + 1);
        skip(kv & 0x0f, depth + 1);
      }
      return;
    }
    case kStruct: {
      int16_t last = 0, id;
      uint8_t t;
      while (field(last, id, t)) {
        skip(t, depth + 1);
      }
      return;
    }
    default:
      throw DecodeError("unknown wire type " + std::to_string(type));
    }
  }
  bool done() const { return p_ == end_; }

 private:
  const uint8_t* p_;
  const uint8_t* end_;
};

bool isBool(uint8_t t) { return t == kTrue || t == kFalse; }

// generic struct walk: fn(id, type) returns true when it consumed the field
template <class Fn>
void readStruct(Reader& r, int depth, Fn&& fn) {
  if (depth > kMaxDepth) {
    throw DecodeError("nesting too deep");
  }
  int16_t last = 0, id;
  uint8_t t;
  while (r.field(last, id, t)) {
    if (!fn(id, t)) {
      r.skip(t, depth + 1);
    }
  }
}

int32_t i32(Reader& r) {
  const int64_t v = r.zz();
  if (v < INT32_MIN || v > INT32_MAX) {
    throw DecodeError("i32 out of range");
  }
  return (int32_t)v;
}

thrift::BinaryAddress readAddr(Reader& r, int depth) {
  thrift::BinaryAddress a;
  readStruct(r, depth, [&](int16_t id, uint8_t t) {
    if (id == 1 && t == kBinary) {
      a.addr = r.binary();
    } else if (id == 3 && t == kBinary) {
      a.ifName = r.binary();
    } else {
      return false;
    }
    return true;
  });
  return a;
}

thrift::IpPrefix readPrefix(Reader& r, int depth) {
  thrift::IpPrefix p;
  readStruct(r, depth, [&](int16_t id, uint8_t t) {
    if (id == 1 && t == kStruct) {
      p.prefixAddress = readAddr(r, depth + 1);
    } else if (id == 2 && t == kI16) {
      p.prefixLength = (int16_t)r.zz();
    } else {
      return false;
    }
    return true;
  });
  return p;
}

thrift::Adjacency readAdj(Reader& r, int depth) {
  thrift::Adjacency a;
  readStruct(r, depth, [&](int16_t id, uint8_t t) {
    switch (id) {
    case 1:
      if (t != kBinary) return false;
      a.otherNodeName = r.binary();
      return true;
    case 2:
      if (t != kBinary) return false;
      a.ifName = r.binary();
      return true;
    case 3:
      if (t != kStruct) return false;
      a.nextHopV6 = readAddr(r, depth + 1);
      return true;
    case 5:
      if (t != kStruct) return false;
      a.nextHopV4 = readAddr(r, depth + 1);
      return true;
    case 4:
      if (t != kI32) return false;
      a.metric = i32(r);
      return true;
    case 6:
      if (t != kI32) return false;
      a.adjLabel = i32(r);
      return true;
    case 7:
      if (!isBool(t)) return false;
      a.isOverloaded = t == kTrue;
      return true;
    case 8:
      if (t != kI32) return false;
      a.rtt = i32(r);
      return true;
    case 9:
      if (t != kI64) return false;
      a.timestamp = r.zz();
      return true;
    case 10:
      if (t != kI64) return false;
      a.weight = r.zz();
      return true;
    case 11:
      if (t != kBinary) return false;
      a.otherIfName = r.binary();
      return true;
    default:
      return false;
    }
  });
  return a;
}

thrift::MetricVector readMv(Reader& r, int depth) {
  thrift::MetricVector mv;
  readStruct(r, depth, [&](int16_t id, uint8_t t) {
    if (id == 1 && t == kI64) {
      mv.version = r.zz();
      return true;
    }
    if (id == 2 && t == kList) {
      uint8_t et;
      const uint32_t n = r.list(et);
      for (uint32_t i = 0; i < n; ++i) {
        if (et != kStruct) {
          r.skip(et, depth + 1);
          continue;
        }
        thrift::MetricEntity me;
        readStruct(r, depth + 1, [&](int16_t fid, uint8_t ft) {
          switch (fid) {
          case 1:
            if (ft != kI64) return false;
            me.type = r.zz();
            return true;
          case 2:
            if (ft != kI64) return false;
            me.priority = r.zz();
            return true;
          case 3:
            if (ft != kI32) return false;
            me.op = (thrift::CompareType)i32(r);
            return true;
          case 4:
            if (!isBool(ft)) return false;
            me.isBestPathTieBreaker = ft == kTrue;
            return true;
          case 5: {
            if (ft != kList) return false;
            uint8_t mt;
            const uint32_t m = r.list(mt);
            for (uint32_t j = 0; j < m; ++j) {
              if (mt == kI64) {
                me.metric.push_back(r.zz());
              } else {
                r.skip(mt, depth + 2);
              }
            }
            return true;
          }
          default:
            return false;
          }
        });
        mv.metrics.push_back(std::move(me));
      }
      return true;
    }
    return false;
  });
  return mv;
}

thrift::PrefixEntry readPrefixEntry(Reader& r, int depth, std::vector<std::string>& areaStack) {
  thrift::PrefixEntry e;
  readStruct(r, depth, [&](int16_t id, uint8_t t) {
    switch (id) {
    case 1:
      if (t != kStruct) return false;
      e.prefix = readPrefix(r, depth + 1);
      return true;
    case 2:
      if (t != kI32) return false;
      e.type = (thrift::PrefixType)i32(r);
      return true;
    case 3:
      if (t != kBinary) return false;
      e.data = r.binary();
      return true;
    case 4:
      if (t != kI32) return false;
      e.forwardingType = (thrift::PrefixForwardingType)i32(r);
      return true;
    case 7:
      if (t != kI32) return false;
      e.forwardingAlgorithm = (thrift::PrefixForwardingAlgorithm)i32(r);
      return true;
    case 5:
      if (!isBool(t)) return false;
      e.ephemeral = t == kTrue;
      return true;
    case 6:
      if (t != kStruct) return false;
      e.mv = readMv(r, depth + 1);
      return true;
    case 8:
      if (t != kI64) return false;
      e.minNexthop = r.zz();
      return true;
    case 9:
      if (t != kI32) return false;
      e.prependLabel = i32(r);
      return true;
    case 12: {
      if (t != kList) return false;
      uint8_t et;
      const uint32_t n = r.list(et);
      for (uint32_t i = 0; i < n; ++i) {
        if (et == kBinary) {
          areaStack.push_back(r.binary());
        } else {
          r.skip(et, depth + 1);
        }
      }
      return true;
    }
    default:
      return false; // 10 metrics, 11 tags: not on this path
    }
  });
  return e;
}

// ---------------------------------------------------------------- writer

class Writer {
 public:
  std::string out;

  void byte(uint8_t b) { out.push_back((char)b); }
  void varint(uint64_t v) {
    while (v >= 0x80) {
      byte((uint8_t)(v | 0x80));
      v >>= 7;
    }
    byte((uint8_t)v);
  }
  void zz(int64_t v) { varint(((uint64_t)v << 1) ^ (uint64_t)(v >> 63)); }
  void binary(const std::string& s) {
    varint(s.size());
    out.append(s);
  }
  void field(int16_t id, uint8_t type) {
    const int d = id - last_.back();
    if (d > 0 && d <= 15) {
      byte((uint8_t)(d << 4 | type));
    } else {
      byte(type);
      zz(id);
    }
    last_.back() = id;
  }
  void boolField(int16_t id, bool v) { field(id, v ? kTrue : kFalse); }
  void listHeader(uint32_t n, uint8_t et) {
    if (n < 15) {
      byte((uint8_t)(n << 4 | et));
    } else {
      byte((uint8_t)(0xF0 | et));
      varint(n);
    }
  }
  void begin() { last_.push_back(0); }
  void end() {
    byte(kStop);
    last_.pop_back();
  }

 private:
  std::vector<int16_t> last_{0};
};

void writeAddr(Writer& w, const thrift::BinaryAddress& a) {
  w.begin();
  w.field(1, kBinary);
  w.binary(a.addr);
  if (a.ifName) {
    w.field(3, kBinary);
    w.binary(*a.ifName);
  }
  w.end();
}

void writePrefix(Writer& w, const thrift::IpPrefix& p) {
  w.begin();
  w.field(1, kStruct);
  writeAddr(w, p.prefixAddress);
  w.field(2, kI16);
  w.zz(p.prefixLength);
  w.end();
}

// fields in IDL declaration order, as fbthrift's generated writers emit them
void writeAdj(Writer& w, const thrift::Adjacency& a) {
  w.begin();
  w.field(1, kBinary);
  w.binary(a.otherNodeName);
  w.field(2, kBinary);
  w.binary(a.ifName);
  w.field(3, kStruct);
  writeAddr(w, a.nextHopV6);
  w.field(5, kStruct);
  writeAddr(w, a.nextHopV4);
  w.field(4, kI32);
  w.zz(a.metric);
  w.field(6, kI32);
  w.zz(a.adjLabel);
  w.boolField(7, a.isOverloaded);
  w.field(8, kI32);
  w.zz(a.rtt);
  w.field(9, kI64);
  w.zz(a.timestamp);
  w.field(10, kI64);
  w.zz(a.weight);
  w.field(11, kBinary);
  w.binary(a.otherIfName);
  w.end();
}

void writeMv(Writer& w, const thrift::MetricVector& mv) {
  w.begin();
  w.field(1, kI64);
  w.zz(mv.version);
  w.field(2, kList);
  w.listHeader((uint32_t)mv.metrics.size(), kStruct);
  for (const auto& me : mv.metrics) {
    w.begin();
    w.field(1, kI64);
    w.zz(me.type);
    w.field(2, kI64);
    w.zz(me.priority);
    w.field(3, kI32);
    w.zz((int32_t)me.op);
    w.boolField(4, me.isBestPathTieBreaker);
    w.field(5, kList);
    w.listHeader((uint32_t)me.metric.size(), kI64);
    for (int64_t m : me.metric) {
      w.zz(m);
    }
    w.end();
  }
  w.end();
}

void writePrefixEntry(Writer& w, const thrift::PrefixEntry& e, const std::vector<std::string>* areaStack) {
  w.begin();
  w.field(1, kStruct);
  writePrefix(w, e.prefix);
  w.field(2, kI32);
  w.zz((int32_t)e.type);
  if (e.data) {
    w.field(3, kBinary);
    w.binary(*e.data);
  }
  w.field(4, kI32);
  w.zz((int32_t)e.forwardingType);
  w.field(7, kI32);
  w.zz((int32_t)e.forwardingAlgorithm);
  if (e.ephemeral) {
    w.boolField(5, *e.ephemeral);
  }
  if (e.mv) {
    w.field(6, kStruct);
    writeMv(w, *e.mv);
  }
  if (e.minNexthop) {
    w.field(8, kI64);
    w.zz(*e.minNexthop);
  }
  if (e.prependLabel) {
    w.field(9, kI32);
    w.zz(*e.prependLabel);
  }
  w.field(12, kList);
  w.listHeader(areaStack ? (uint32_t)areaStack->size() : 0, kBinary);
  if (areaStack) {
    for (const auto& a : *areaStack) {
      w.binary(a);
    }
  }
  w.end();
}

} // namespace

thrift::AdjacencyDatabase decodeAdjacencyDatabase(std::string_view bytes) {
  Reader r(bytes);
  thrift::AdjacencyDatabase db;
  readStruct(r, 0, [&](int16_t id, uint8_t t) {
    switch (id) {
    case 1:
      if (t != kBinary) return false;
      db.thisNodeName = r.binary();
      return true;
    case 2:
      if (!isBool(t)) return false;
      db.isOverloaded = t == kTrue;
      return true;
    case 3: {
      if (t != kList) return false;
      uint8_t et;
      const uint32_t n = r.list(et);
      db.adjacencies.reserve(n);
      for (uint32_t i = 0; i < n; ++i) {
        if (et == kStruct) {
          db.adjacencies.push_back(readAdj(r, 1));
        } else {
          r.skip(et, 1);
        }
      }
      return true;
    }
    case 4:
      if (t != kI32) return false;
      db.nodeLabel = i32(r);
      return true;
    case 6:
      if (t != kBinary) return false;
      db.area = r.binary();
      return true;
    default:
      return false; // 5 perfEvents
    }
  });
  if (!r.done()) {
    throw DecodeError("trailing bytes after AdjacencyDatabase");
  }
  return db;
}

PrefixDbWire decodePrefixDatabase(std::string_view bytes) {
  Reader r(bytes);
  PrefixDbWire w;
  readStruct(r, 0, [&](int16_t id, uint8_t t) {
    switch (id) {
    case 1:
      if (t != kBinary) return false;
      w.db.thisNodeName = r.binary();
      return true;
    case 3: {
      if (t != kList) return false;
      uint8_t et;
      const uint32_t n = r.list(et);
      for (uint32_t i = 0; i < n; ++i) {
        if (et != kStruct) {
          r.skip(et, 1);
          continue;
        }
        w.areaStacks.emplace_back();
        w.db.prefixEntries.push_back(readPrefixEntry(r, 1, w.areaStacks.back()));
      }
      return true;
    }
    case 5:
      if (!isBool(t)) return false;
      w.db.deletePrefix = t == kTrue;
      return true;
    case 6:
      if (!isBool(t)) return false;
      w.perPrefixKey = t == kTrue;
      return true;
    case 7:
      if (t != kBinary) return false;
      w.db.area = r.binary();
      return true;
    default:
      return false; // 4 perfEvents
    }
  });
  if (!r.done()) {
    throw DecodeError("trailing bytes after PrefixDatabase");
  }
  return w;
}

std::string encode(const thrift::AdjacencyDatabase& db) {
  Writer w;
  w.field(1, kBinary);
  w.binary(db.thisNodeName);
  w.boolField(2, db.isOverloaded);
  w.field(3, kList);
  w.listHeader((uint32_t)db.adjacencies.size(), kStruct);
  for (const auto& a : db.adjacencies) {
    writeAdj(w, a);
  }
  w.field(4, kI32);
  w.zz(db.nodeLabel);
  w.field(6, kBinary);
  w.binary(db.area);
  w.byte(kStop);
  return std::move(w.out);
}

std::string encode(
    const thrift::PrefixDatabase& db, const std::vector<std::vector<std::string>>* areaStacks) {
  Writer w;
  w.field(1, kBinary);
  w.binary(db.thisNodeName);
  w.field(3, kList);
  w.listHeader((uint32_t)db.prefixEntries.size(), kStruct);
  for (size_t i = 0; i < db.prefixEntries.size(); ++i) {
    writePrefixEntry(w, db.prefixEntries[i],
                     areaStacks && i < areaStacks->size() ? &(*areaStacks)[i] : nullptr);
  }
  w.boolField(5, db.deletePrefix);
  w.field(7, kBinary);
  w.binary(db.area);
  w.byte(kStop);
  return std::move(w.out);
}

} // namespace compact

std::string getNodeNameFromKey(const std::string& key) {
  const size_t a = key.find(':');
  if (a == std::string::npos) {
    return "";
  }
  const size_t b = key.find(':', a + 1);
  return key.substr(a + 1, b == std::string::npos ? std::string::npos : b - a - 1);
}

std::optional<PrefixKeyParts> parsePrefixKey(const std::string& key) {
  // ^prefix:([A-Za-z0-9._-]+):([A-Za-z0-9]+):\[([0-9a-fA-F.:]+)/([0-9]{1,3})\]$
  static const std::string marker = "prefix:";
  if (key.compare(0, marker.size(), marker) != 0) {
    return std::nullopt;
  }
  auto isNode = [](char c) { return isalnum((unsigned char)c) || c == '.' || c == '-' || c == '_'; };
  auto isArea = [](char c) { return isalnum((unsigned char)c) != 0; };
  auto isIp = [](char c) { return isxdigit((unsigned char)c) || c == '.' || c == ':'; };
  size_t i = marker.size();
  auto run = [&](auto&& pred) {
    const size_t s = i;
    while (i < key.size() && pred(key[i])) {
      ++i;
    }
    return key.substr(s, i - s);
  };
  PrefixKeyParts out;
  out.node = run(isNode);
  if (out.node.empty() || i >= key.size() || key[i++] != ':') {
    return std::nullopt;
  }
  out.area = run(isArea);
  if (out.area.empty() || i + 1 >= key.size() || key[i] != ':' || key[i + 1] != '[') {
    return std::nullopt;
  }
  i += 2;
  // the IP class includes ':' — RE2 backtracks to the last '/'; a '/' cannot
  // occur inside the class, so the run ends exactly there
  const std::string ip = run(isIp);
  if (ip.empty() || i >= key.size() || key[i++] != '/') {
    return std::nullopt;
  }
  const std::string plen = run([](char c) { return isdigit((unsigned char)c) != 0; });
  if (plen.empty() || plen.size() > 3 || i + 1 != key.size() || key[i] != ']') {
    return std::nullopt;
  }
  // folly::IPAddress::createNetwork(ip/plen): parse, range-check, mask
  unsigned char buf[16];
  size_t bytes = 0;
  if (inet_pton(AF_INET, ip.c_str(), buf) == 1) {
    bytes = 4;
  } else if (inet_pton(AF_INET6, ip.c_str(), buf) == 1) {
    bytes = 16;
  } else {
    return std::nullopt;
  }
  const int len = std::stoi(plen);
  if (len > (int)bytes * 8) {
    return std::nullopt;
  }
  for (size_t b = 0; b < bytes; ++b) {
    const int keep = std::max(0, std::min(8, len - (int)b * 8));
    buf[b] &= (unsigned char)(0xFF00 >> keep);
  }
  out.prefix.prefixAddress.addr.assign(reinterpret_cast<char*>(buf), bytes);
  out.prefix.prefixLength = (int16_t)len;
  return out;
}

std::optional<thrift::PrefixDatabase> PublicationIngest::updateNodePrefixDatabase(
    const std::string& key, const compact::PrefixDbWire& wire,
    const std::unordered_map<std::string, LinkState>& areaLinkStates) {
  // Decision.cpp:1585-1629
  const auto& prefixDb = wire.db;
  const auto& nodeName = prefixDb.thisNodeName;
  if (auto pk = parsePrefixKey(key)) {
    if (prefixDb.deletePrefix) {
      perPrefixPrefixEntries_[nodeName].erase(pk->prefix);
    } else {
      if (prefixDb.prefixEntries.size() != 1) {
        throw CheckFailure("per-prefix key " + key + " must carry exactly one entry");
      }
      const auto& areaStack = wire.areaStacks.at(0);
      // self-redistributed route reflection (re-originated by me)
      if (nodeName == myNodeName_ && !areaStack.empty() && areaLinkStates.count(areaStack[0])) {
        return std::nullopt;
      }
      perPrefixPrefixEntries_[nodeName][pk->prefix] = prefixDb.prefixEntries[0];
    }
  } else {
    auto& full = fullDbPrefixEntries_[nodeName];
    full.clear();
    for (const auto& e : prefixDb.prefixEntries) {
      full[e.prefix] = e;
    }
  }
  thrift::PrefixDatabase out;
  out.thisNodeName = nodeName;
  auto& per = perPrefixPrefixEntries_[nodeName];
  out.prefixEntries.reserve(per.size());
  for (const auto& kv : per) {
    out.prefixEntries.push_back(kv.second);
  }
  for (const auto& kv : fullDbPrefixEntries_[nodeName]) {
    if (!per.count(kv.first)) {
      out.prefixEntries.push_back(kv.second);
    }
  }
  return out;
}

const PendingUpdates& PublicationIngest::processPublication(
    const thrift::Publication& pub,
    std::unordered_map<std::string, LinkState>& areaLinkStates,
    PrefixState& prefixState) {
  // Decision.cpp:1631-1763
  if (pub.area.empty()) {
    throw std::invalid_argument("publication without an area");
  }
  const std::string& area = pub.area;
  auto it = areaLinkStates.find(area);
  if (it == areaLinkStates.end()) {
    it = areaLinkStates.emplace(area, LinkState(area)).first;
  }
  LinkState& als = it->second;
  if (pub.keyVals.empty() && pub.expiredKeys.empty()) {
    return pending_;
  }
  auto applyLs = [&](const std::string& node, const LinkState::LinkStateChange& c) {
    pending_.needsFullRebuild |= c.topologyChanged || c.nodeLabelChanged ||
        (c.linkAttributesChanged && node == myNodeName_);
    ++pending_.count;
  };
  auto applyPs = [&](std::unordered_set<thrift::IpPrefix>&& c) {
    pending_.updatedPrefixes.merge(c);
    ++pending_.count;
  };
  static const std::string kAdj = "adj:", kPrefix = "prefix:";
  for (const auto& [key, val] : pub.keyVals) {
    const std::string nodeName = getNodeNameFromKey(key);
    if (!val.value) {
      continue; // TTL refresh
    }
    // Only deserialisation failures are per-key errors (the reference logs
    // them and moves on, Decision.cpp:1718-1721).  Everything after a
    // successful decode -- CHECK failures, engine / device errors, bad_alloc --
    // propagates: the reference aborts on those (Decision.cpp:1392-1404) and a
    // half-applied update must never be counted as a decode error.
    if (key.compare(0, kAdj.size(), kAdj) == 0) {
      thrift::AdjacencyDatabase db;
      try {
        db = compact::decodeAdjacencyDatabase(*val.value);
      } catch (const compact::DecodeError&) {
        Counters::add("decision.publication_decode_errors", 1);
        continue;
      }
      db.area = area;
      if (nodeName != db.thisNodeName) {
        throw CheckFailure("CHECK_EQ(nodeName, adjacencyDb.thisNodeName) failed: " +
                               nodeName + " vs " + db.thisNodeName);
      }
      LinkStateMetric holdUp = 0, holdDown = 0;
      if (enableOrderedFib_) {
        if (auto h = als.getHopsFromAToB(myNodeName_, db.thisNodeName)) {
          holdUp = *h;
          holdDown = als.getMaxHopsToNode(db.thisNodeName) - holdUp;
        }
      }
      Counters::add("decision.adj_db_update", 1);
      const std::string node = db.thisNodeName;
      applyLs(node, als.updateAdjacencyDatabase(std::move(db), holdUp, holdDown));
      continue;
    }
    if (key.compare(0, kPrefix.size(), kPrefix) == 0) {
      compact::PrefixDbWire wire;
      try {
        wire = compact::decodePrefixDatabase(*val.value);
      } catch (const compact::DecodeError&) {
        Counters::add("decision.publication_decode_errors", 1);
        continue;
      }
      if (nodeName != wire.db.thisNodeName) {
        throw CheckFailure("CHECK_EQ(nodeName, prefixDb.thisNodeName) failed: " +
                               nodeName + " vs " + wire.db.thisNodeName);
      }
      auto nodeDb = updateNodePrefixDatabase(key, wire, areaLinkStates);
      if (!nodeDb) {
        continue;
      }
      nodeDb->area = area;
      Counters::add("decision.prefix_db_update", 1);
      applyPs(prefixState.updatePrefixDatabase(*nodeDb));
      continue;
    }
    // fibtime: keys only feed Decision's fib-time estimate (not this path)
  }
  for (const auto& key : pub.expiredKeys) {
    const std::string nodeName = getNodeNameFromKey(key);
    if (key.compare(0, kAdj.size(), kAdj) == 0) {
      applyLs(nodeName, als.deleteAdjacencyDatabase(nodeName));
      continue;
    }
    if (key.compare(0, kPrefix.size(), kPrefix) == 0) {
      compact::PrefixDbWire del;
      del.db.thisNodeName = nodeName;
      del.db.deletePrefix = true;
      auto nodeDb = updateNodePrefixDatabase(key, del, areaLinkStates);
      if (!nodeDb) {
        continue;
      }
      nodeDb->area = area;
      applyPs(prefixState.updatePrefixDatabase(*nodeDb));
    }
  }
  return pending_;
}

} // namespace openr
