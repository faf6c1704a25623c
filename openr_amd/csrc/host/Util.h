// Util.h — the openr/common helpers the SPF/RouteDb path calls
// (reference: openr/common/Util.h:285-530, Util.cpp:635-703, 914-976,
// 1051-1228).  Header-only.
#pragma once

#include <algorithm>
#include <limits>
#include <optional>
#include <stdexcept>
#include <string>
#include <vector>

#include "Types.h"

namespace openr {

// 20-bit MPLS label (Util.h:303-306)
inline bool isMplsLabelValid(int32_t const mplsLabel) {
  return (mplsLabel & 0xfff00000) == 0;
}

// The reference CHECK-fails on malformed actions (Util.cpp:673-703); here the
// same conditions raise, so a bad label never reaches a route silently.
inline void checkMplsAction(thrift::MplsAction const& a) {
  auto bad = [](const char* why) { throw std::logic_error(std::string("checkMplsAction: ") + why); };
  switch (a.action) {
  case thrift::MplsActionCode::PUSH:
    if (a.swapLabel || !a.pushLabels || a.pushLabels->empty()) {
      bad("PUSH needs push labels only");
    }
    for (auto l : *a.pushLabels) {
      if (!isMplsLabelValid(l)) {
        bad("invalid push label");
      }
    }
    break;
  case thrift::MplsActionCode::SWAP:
    if (!a.swapLabel || !isMplsLabelValid(*a.swapLabel) || a.pushLabels) {
      bad("SWAP needs one valid swap label");
    }
    break;
  case thrift::MplsActionCode::PHP:
  case thrift::MplsActionCode::POP_AND_LOOKUP:
    if (a.swapLabel || a.pushLabels) {
      bad("PHP/POP take no labels");
    }
    break;
  default:
    bad("unknown action code");
  }
}

inline thrift::MplsAction createMplsAction(
    thrift::MplsActionCode code,
    std::optional<int32_t> swapLabel = std::nullopt,
    std::optional<std::vector<int32_t>> pushLabels = std::nullopt) {
  thrift::MplsAction a;
  a.action = code;
  a.swapLabel = swapLabel;
  a.pushLabels = std::move(pushLabels);
  checkMplsAction(a);
  return a;
}

// metric narrows to int32 exactly as the reference signature does
// (Util.cpp:914-930)
inline thrift::NextHopThrift createNextHop(
    thrift::BinaryAddress addr,
    std::optional<std::string> ifName = std::nullopt,
    int32_t metric = 0,
    std::optional<thrift::MplsAction> mplsAction = std::nullopt,
    bool useNonShortestRoute = false,
    const std::string& area = thrift::kDefaultArea()) {
  thrift::NextHopThrift nh;
  nh.address = std::move(addr);
  nh.address.ifName = std::move(ifName);
  nh.metric = metric;
  nh.mplsAction = std::move(mplsAction);
  nh.useNonShortestRoute = useNonShortestRoute;
  nh.area = area;
  return nh;
}

// Fib's programmed subset of a unicast route's next hops (Util.cpp:473-495):
// those at the minimum metric, plus any marked useNonShortestRoute; input
// order kept.
inline std::vector<thrift::NextHopThrift> getBestNextHopsUnicast(
    const std::vector<thrift::NextHopThrift>& allNextHops) {
  if (allNextHops.size() <= 1) {
    return allNextHops;
  }
  int32_t minCost = std::numeric_limits<int32_t>::max();
  for (const auto& nh : allNextHops) {
    minCost = std::min(minCost, nh.metric);
  }
  std::vector<thrift::NextHopThrift> best;
  for (const auto& nh : allNextHops) {
    if (nh.metric == minCost || nh.useNonShortestRoute) {
      best.push_back(nh);
    }
  }
  return best;
}

// The MPLS counterpart (Util.cpp:497-531): minimum metric, and among the
// next hops reaching it PHP is preferred over SWAP; PUSH and POP_AND_LOOKUP
// are invalid in a multi-next-hop label route (the reference CHECKs).
inline std::vector<thrift::NextHopThrift> getBestNextHopsMpls(
    const std::vector<thrift::NextHopThrift>& allNextHops) {
  if (allNextHops.size() <= 1) {
    return allNextHops;
  }
  int32_t minCost = std::numeric_limits<int32_t>::max();
  thrift::MplsActionCode code = thrift::MplsActionCode::SWAP;
  for (const auto& nh : allNextHops) {
    if (!nh.mplsAction) {
      throw CheckFailure("getBestNextHopsMpls: next hop without an MPLS action");
    }
    if (nh.mplsAction->action == thrift::MplsActionCode::PUSH ||
        nh.mplsAction->action == thrift::MplsActionCode::POP_AND_LOOKUP) {
      throw CheckFailure("getBestNextHopsMpls: PUSH / POP_AND_LOOKUP in a label route");
    }
    if (nh.metric <= minCost) {
      minCost = nh.metric;
      if (nh.mplsAction->action == thrift::MplsActionCode::PHP) {
        code = thrift::MplsActionCode::PHP;
      }
    }
  }
  std::vector<thrift::NextHopThrift> best;
  for (const auto& nh : allNextHops) {
    if (nh.metric == minCost && nh.mplsAction->action == code) {
      best.push_back(nh);
    }
  }
  return best;
}

// IP wins over SR_MPLS when advertisers disagree (Util.cpp:635-652)
inline thrift::PrefixForwardingType getPrefixForwardingType(
    const thrift::PrefixEntries& entries) {
  for (const auto& [node, byArea] : entries) {
    for (const auto& [area, e] : byArea) {
      if (e.forwardingType == thrift::PrefixForwardingType::IP) {
        return thrift::PrefixForwardingType::IP;
      }
    }
  }
  return entries.empty() ? thrift::PrefixForwardingType::IP
                         : thrift::PrefixForwardingType::SR_MPLS;
}

// SP_ECMP wins over KSP2_ED_ECMP (Util.cpp:654-671)
inline thrift::PrefixForwardingAlgorithm getPrefixForwardingAlgorithm(
    const thrift::PrefixEntries& entries) {
  for (const auto& [node, byArea] : entries) {
    for (const auto& [area, e] : byArea) {
      if (e.forwardingAlgorithm == thrift::PrefixForwardingAlgorithm::SP_ECMP) {
        return thrift::PrefixForwardingAlgorithm::SP_ECMP;
      }
    }
  }
  return entries.empty() ? thrift::PrefixForwardingAlgorithm::SP_ECMP
                         : thrift::PrefixForwardingAlgorithm::KSP2_ED_ECMP;
}

// BGP metric-vector best path (Util.cpp:1051-1228)
namespace MetricVectorUtils {

enum class CompareResult { WINNER, TIE_WINNER, TIE, TIE_LOOSER, LOOSER, ERROR };

constexpr int64_t kOpenrIgpCostType = 9;        // MetricEntityType::OPENR_IGP_COST
constexpr int64_t kOpenrIgpCostPriority = 3500; // MetricEntityPriority::OPENR_IGP_COST

inline std::optional<thrift::MetricEntity> getMetricEntityByType(
    const thrift::MetricVector& mv, int64_t type) {
  for (const auto& me : mv.metrics) {
    if (me.type == type) {
      return me;
    }
  }
  return std::nullopt;
}

inline thrift::MetricEntity createMetricEntity(
    int64_t type,
    int64_t priority,
    thrift::CompareType op,
    bool isBestPathTieBreaker,
    const std::vector<int64_t>& metric) {
  thrift::MetricEntity me;
  me.type = type;
  me.priority = priority;
  me.op = op;
  me.isBestPathTieBreaker = isBestPathTieBreaker;
  me.metric = metric;
  return me;
}

inline CompareResult flip(CompareResult r) {
  switch (r) {
  case CompareResult::WINNER:
    return CompareResult::LOOSER;
  case CompareResult::TIE_WINNER:
    return CompareResult::TIE_LOOSER;
  case CompareResult::TIE_LOOSER:
    return CompareResult::TIE_WINNER;
  case CompareResult::LOOSER:
    return CompareResult::WINNER;
  default:
    return r; // TIE, ERROR
  }
}

inline bool isDecisive(CompareResult r) {
  return r == CompareResult::WINNER || r == CompareResult::LOOSER ||
      r == CompareResult::ERROR;
}

inline CompareResult compareMetrics(
    const std::vector<int64_t>& l, const std::vector<int64_t>& r, bool tieBreaker) {
  if (l.size() != r.size()) {
    return CompareResult::ERROR;
  }
  for (size_t i = 0; i < l.size(); ++i) {
    if (l[i] > r[i]) {
      return tieBreaker ? CompareResult::TIE_WINNER : CompareResult::WINNER;
    }
    if (l[i] < r[i]) {
      return tieBreaker ? CompareResult::TIE_LOOSER : CompareResult::LOOSER;
    }
  }
  return CompareResult::TIE;
}

inline CompareResult resultForLoner(const thrift::MetricEntity& e) {
  if (e.op == thrift::CompareType::WIN_IF_PRESENT) {
    return e.isBestPathTieBreaker ? CompareResult::TIE_WINNER : CompareResult::WINNER;
  }
  if (e.op == thrift::CompareType::WIN_IF_NOT_PRESENT) {
    return e.isBestPathTieBreaker ? CompareResult::TIE_LOOSER : CompareResult::LOOSER;
  }
  return CompareResult::TIE; // IGNORE_IF_NOT_PRESENT
}

inline void maybeUpdate(CompareResult& target, CompareResult update) {
  if (isDecisive(update) || target == CompareResult::TIE) {
    target = update;
  }
}

// The reference sorts the (copied) vectors in place by decreasing priority
// with std::sort when they are not already sorted.
inline void sortByPriority(std::vector<thrift::MetricEntity>& m) {
  bool sorted = true;
  for (size_t i = 1; i < m.size(); ++i) {
    if (m[i].priority > m[i - 1].priority) {
      sorted = false;
      break;
    }
  }
  if (!sorted) {
    std::sort(m.begin(), m.end(), [](const thrift::MetricEntity& a, const thrift::MetricEntity& b) {
      return a.priority > b.priority;
    });
  }
}

inline CompareResult compareMetricVectors(thrift::MetricVector& l, thrift::MetricVector& r) {
  if (l.version != r.version) {
    return CompareResult::ERROR;
  }
  sortByPriority(l.metrics);
  sortByPriority(r.metrics);
  CompareResult result = CompareResult::TIE;
  size_t li = 0, ri = 0;
  const auto& L = l.metrics;
  const auto& R = r.metrics;
  while (!isDecisive(result) && li < L.size() && ri < R.size()) {
    if (L[li].type == R[ri].type) {
      if (L[li].isBestPathTieBreaker != R[ri].isBestPathTieBreaker) {
        maybeUpdate(result, CompareResult::ERROR);
      } else {
        maybeUpdate(result, compareMetrics(L[li].metric, R[ri].metric, L[li].isBestPathTieBreaker));
      }
      ++li;
      ++ri;
    } else if (L[li].priority > R[ri].priority) {
      maybeUpdate(result, resultForLoner(L[li]));
      ++li;
    } else if (L[li].priority < R[ri].priority) {
      maybeUpdate(result, flip(resultForLoner(R[ri])));
      ++ri;
    } else {
      maybeUpdate(result, CompareResult::ERROR); // same priority, other type
    }
  }
  while (!isDecisive(result) && li < L.size()) {
    maybeUpdate(result, resultForLoner(L[li++]));
  }
  while (!isDecisive(result) && ri < R.size()) {
    maybeUpdate(result, flip(resultForLoner(R[ri++])));
  }
  return result;
}

} // namespace MetricVectorUtils

} // namespace openr
