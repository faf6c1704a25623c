// PrefixState.cpp — see PrefixState.h (reference: PrefixState.cpp:19-164).

#include "PrefixState.h"

#include "Util.h"

namespace openr {

namespace {
// a host loopback is a /32 (v4) or /128 (v6) LOOPBACK prefix
bool isHostPrefix(const thrift::IpPrefix& p, size_t bytes, int bits) {
  return p.prefixAddress.addr.size() == bytes && p.prefixLength == bits;
}
} // namespace

void PrefixState::deleteLoopbackPrefix(
    thrift::IpPrefix const& prefix, const std::string& nodeName) {
  auto drop = [&](std::unordered_map<std::string, thrift::BinaryAddress>& m) {
    auto it = m.find(nodeName);
    if (it != m.end() && it->second == prefix.prefixAddress) {
      m.erase(it);
    }
  };
  if (isHostPrefix(prefix, 4, 32)) {
    drop(nodeHostLoopbacksV4_);
  }
  if (isHostPrefix(prefix, 16, 128)) {
    drop(nodeHostLoopbacksV6_);
  }
}

std::unordered_set<thrift::IpPrefix> PrefixState::updatePrefixDatabase(
    thrift::PrefixDatabase const& prefixDb) {
  std::unordered_set<thrift::IpPrefix> changed;
  const std::string& nodeName = prefixDb.thisNodeName;
  const std::string& area = prefixDb.area;

  const std::set<thrift::IpPrefix> oldSet = nodeToPrefixes_[nodeName][area];
  auto& newSet = nodeToPrefixes_[nodeName][area];
  newSet.clear();
  for (const auto& entry : prefixDb.prefixEntries) {
    newSet.insert(entry.prefix);
  }

  // withdrawals first
  for (const auto& prefix : oldSet) {
    if (newSet.count(prefix)) {
      continue;
    }
    auto& byNode = prefixes_.at(prefix);
    auto nodeIt = byNode.find(nodeName);
    if (nodeIt == byNode.end()) {
      continue; // duplicate withdraw
    }
    nodeIt->second.erase(area);
    if (nodeIt->second.empty()) {
      byNode.erase(nodeIt);
    }
    if (byNode.empty()) {
      prefixes_.erase(prefix);
    }
    deleteLoopbackPrefix(prefix, nodeName);
    changed.insert(prefix);
  }

  // announcements / updates
  for (const auto& entry : prefixDb.prefixEntries) {
    auto& byNode = prefixes_[entry.prefix];
    auto nodeIt = byNode.find(nodeName);
    if (nodeIt != byNode.end()) {
      auto areaIt = nodeIt->second.find(area);
      if (areaIt != nodeIt->second.end() && areaIt->second == entry) {
        continue; // unchanged
      }
    }
    byNode[nodeName][area] = entry;
    changed.insert(entry.prefix);
    if (entry.type == thrift::PrefixType::LOOPBACK) {
      if (isHostPrefix(entry.prefix, 4, 32)) {
        nodeHostLoopbacksV4_[nodeName] = entry.prefix.prefixAddress;
      }
      if (isHostPrefix(entry.prefix, 16, 128)) {
        nodeHostLoopbacksV6_[nodeName] = entry.prefix.prefixAddress;
      }
    }
  }

  if (newSet.empty()) {
    nodeToPrefixes_.erase(nodeName);
  }
  return changed;
}

std::unordered_map<std::string, thrift::PrefixDatabase> PrefixState::getPrefixDatabases()
    const {
  std::unordered_map<std::string, thrift::PrefixDatabase> dbs;
  for (const auto& [node, byArea] : nodeToPrefixes_) {
    for (const auto& [area, prefixes] : byArea) {
      thrift::PrefixDatabase db;
      db.thisNodeName = node;
      db.area = area;
      for (const auto& prefix : prefixes) {
        db.prefixEntries.push_back(prefixes_.at(prefix).at(node).at(area));
      }
      dbs.emplace(node, std::move(db));
    }
  }
  return dbs;
}

std::vector<thrift::NextHopThrift> PrefixState::getLoopbackVias(
    std::unordered_set<std::string> const& nodes,
    bool const isV4,
    std::optional<int64_t> const& igpMetric) const {
  std::vector<thrift::NextHopThrift> vias;
  vias.reserve(nodes.size());
  const auto& loopbacks = isV4 ? nodeHostLoopbacksV4_ : nodeHostLoopbacksV6_;
  for (const auto& node : nodes) {
    auto it = loopbacks.find(node);
    if (it != loopbacks.end()) {
      vias.push_back(createNextHop(
          it->second, std::nullopt, (int32_t)igpMetric.value_or(0)));
    }
  }
  return vias;
}

} // namespace openr
