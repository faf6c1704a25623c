// Publication.h — the step before the SPF path:
// Decision::processPublication (openr/decision/Decision.cpp:1631-1763) turns
// a KvStore publication of "adj:<node>" / "prefix:<node>[:<area>:[<prefix>]]"
// keys into LinkState / PrefixState updates.  The values are fbthrift
// CompactProtocol blobs (fbzmq::util::readThriftObjStr with Decision's
// CompactSerializer, Decision.cpp:1665-1666, 1693-1694).
//
// This file restates that wire format for the structs on the path
// (Lsdb.thrift:70-128 AdjacencyDatabase / Adjacency, :183-213 MetricVector,
// :271-352 PrefixEntry / PrefixDatabase, Network.thrift:54-62 BinaryAddress /
// IpPrefix) as a direct reader (no generated code, no intermediate objects),
// plus the writer the bench and tests use to make publications, and the
// Decision members processPublication touches (per-prefix / full-db prefix
// entries, pending-update bookkeeping, Decision.h:105-160, 384-400).
#pragma once

#include <cstdint>
#include <optional>
#include <stdexcept>
#include <string>
#include <string_view>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "LinkState.h"
#include "PrefixState.h"
#include "Types.h"

namespace openr {
namespace thrift {

// KvStore.thrift:20-43 Value
struct Value {
  int64_t version{0};
  std::string originatorId;
  std::optional<std::string> value; // unset = TTL refresh only
  int64_t ttl{0};
  int64_t ttlVersion{0};
  std::optional<int64_t> hash;
};

// KvStore.thrift:228-249 Publication (the fields Decision reads)
struct Publication {
  std::unordered_map<std::string, Value> keyVals;
  std::vector<std::string> expiredKeys;
  std::string area{"0"};
};

} // namespace thrift

namespace compact {

// Malformed input (truncated, bad varint, nesting too deep, wrong length).
struct DecodeError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

// A decoded PrefixDatabase plus the PrefixEntry fields the SPF path's types
// do not carry but updateNodePrefixDatabase reads (area_stack, field 12).
struct PrefixDbWire {
  thrift::PrefixDatabase db;
  std::vector<std::vector<std::string>> areaStacks; // per prefix entry
  std::optional<bool> perPrefixKey;
};

thrift::AdjacencyDatabase decodeAdjacencyDatabase(std::string_view bytes);
PrefixDbWire decodePrefixDatabase(std::string_view bytes);

std::string encode(const thrift::AdjacencyDatabase& db);
std::string encode(
    const thrift::PrefixDatabase& db,
    const std::vector<std::vector<std::string>>* areaStacks = nullptr);

} // namespace compact

// Decision's pending-update state (Decision.h:105-160).
struct PendingUpdates {
  bool needsFullRebuild{false};
  std::unordered_set<thrift::IpPrefix> updatedPrefixes;
  uint64_t count{0};
  bool needsRouteUpdate() const { return needsFullRebuild || !updatedPrefixes.empty(); }
  void reset() {
    needsFullRebuild = false;
    updatedPrefixes.clear();
    count = 0;
  }
};

// The Decision members processPublication reads and writes, without the
// event loop around them.  Counters: decision.adj_db_update,
// decision.prefix_db_update (as the reference), decision.publication_decode_errors
// (the reference only logs those, Decision.cpp:1718-1721).
class PublicationIngest {
 public:
  PublicationIngest(std::string myNodeName, bool enableOrderedFib = false)
      : myNodeName_(std::move(myNodeName)), enableOrderedFib_(enableOrderedFib) {}

  // Decision::processPublication (Decision.cpp:1631-1763).  Areas missing
  // from `areaLinkStates` are created.  Returns the updates applied so far
  // (cleared by the caller after a route rebuild, like pendingUpdates_).
  const PendingUpdates& processPublication(
      const thrift::Publication& pub,
      std::unordered_map<std::string, LinkState>& areaLinkStates,
      PrefixState& prefixState);

  PendingUpdates& pending() { return pending_; }

 private:
  std::optional<thrift::PrefixDatabase> updateNodePrefixDatabase(
      const std::string& key, const compact::PrefixDbWire& wire,
      const std::unordered_map<std::string, LinkState>& areaLinkStates);

  std::string myNodeName_;
  bool enableOrderedFib_;
  PendingUpdates pending_;
  // Decision.h:390-396
  std::unordered_map<std::string, std::unordered_map<thrift::IpPrefix, thrift::PrefixEntry>>
      perPrefixPrefixEntries_, fullDbPrefixEntries_;
};

// getNodeNameFromKey (openr/common/Util.cpp:1037-1044): the field after the
// first ':' ("" when there is none).
std::string getNodeNameFromKey(const std::string& key);

// PrefixKey::fromStr (openr/common/Util.cpp:68-88): "prefix:<node>:<area>:
// [<ip>/<len>]" -> (node, area, masked prefix); nullopt for any other form.
struct PrefixKeyParts {
  std::string node, area;
  thrift::IpPrefix prefix;
};
std::optional<PrefixKeyParts> parsePrefixKey(const std::string& key);

} // namespace openr
