// PrefixState.h — prefix -> {node -> {area -> PrefixEntry}} bookkeeping, the
// host-side input of RouteDb generation (reference:
// openr/decision/PrefixState.h:20-63, PrefixState.cpp:19-164).  Stays on the
// CPU: it is string/prefix bookkeeping with no SPF arithmetic.
#pragma once

#include <optional>
#include <set>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "Types.h"

namespace openr {

class PrefixState {
 public:
  std::unordered_map<thrift::IpPrefix, thrift::PrefixEntries> const& prefixes() const {
    return prefixes_;
  }

  void deleteLoopbackPrefix(thrift::IpPrefix const& prefix, const std::string& nodename);

  // prefixes whose advertisement changed (added, withdrawn or modified)
  std::unordered_set<thrift::IpPrefix> updatePrefixDatabase(
      thrift::PrefixDatabase const& prefixDb);

  std::unordered_map<std::string, thrift::PrefixDatabase> getPrefixDatabases() const;

  std::vector<thrift::NextHopThrift> getLoopbackVias(
      std::unordered_set<std::string> const& nodes,
      bool const isV4,
      std::optional<int64_t> const& igpMetric) const;

  std::unordered_map<std::string, thrift::BinaryAddress> const& getNodeHostLoopbacksV4() const {
    return nodeHostLoopbacksV4_;
  }
  std::unordered_map<std::string, thrift::BinaryAddress> const& getNodeHostLoopbacksV6() const {
    return nodeHostLoopbacksV6_;
  }

 private:
  std::unordered_map<thrift::IpPrefix, thrift::PrefixEntries> prefixes_;
  std::unordered_map<std::string, std::unordered_map<std::string, std::set<thrift::IpPrefix>>>
      nodeToPrefixes_;
  std::unordered_map<std::string, thrift::BinaryAddress> nodeHostLoopbacksV4_;
  std::unordered_map<std::string, thrift::BinaryAddress> nodeHostLoopbacksV6_;
};

} // namespace openr
