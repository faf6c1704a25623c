// decision_consumer.cpp — a standalone C++ program that uses the drop-in the
// way Open/R's Decision does (Decision::rebuildRoutes, Decision.cpp:
// 1803-1804): AdjacencyDatabases into a per-area LinkState, PrefixDatabases
// into PrefixState, SpfSolver::buildRouteDb for one node.  No pybind, no
// torch: it links only libopenr_decision.so (the host layer) and
// libopenr_spf.so (the C ABI), built by the recipe in INTEGRATION.md.
//
// Topology: a 4-node ring 1-2-4-3-1, metric 10 everywhere, node labels
// 101..104, one /128 loopback per node.  Prints node "1"'s RouteDb as sorted
// text lines (unicast: prefix, next-hop interface + metric; MPLS: label,
// action, interface) and exits 0.  Without a usable MI355X the engine has no
// CPU path: the LinkState raises and the program exits 3.
#include <algorithm>
#include <cstdio>
#include <exception>
#include <string>
#include <unordered_map>
#include <vector>

#include "LinkState.h"
#include "PrefixState.h"
#include "SpfSolver.h"
#include "openr_spf.h"

using namespace openr;

namespace {

thrift::BinaryAddress v6(int host) {
  thrift::BinaryAddress a;
  a.addr = std::string(16, '\0');
  a.addr[0] = (char)0xfe;
  a.addr[1] = (char)0x80;
  a.addr[15] = (char)host;
  return a;
}

thrift::IpPrefix loopback(int node) {
  thrift::IpPrefix p;
  p.prefixAddress.addr = std::string(16, '\0');
  p.prefixAddress.addr[0] = (char)0xfc;
  p.prefixAddress.addr[15] = (char)node;
  p.prefixLength = 128;
  return p;
}

thrift::Adjacency adj(int me, int other) {
  thrift::Adjacency a;
  a.otherNodeName = std::to_string(other);
  a.ifName = "if_" + std::to_string(me) + "_" + std::to_string(other);
  a.otherIfName = "if_" + std::to_string(other) + "_" + std::to_string(me);
  a.nextHopV6 = v6(other);
  a.metric = 10;
  return a;
}

std::string hopText(const thrift::NextHopThrift& nh) {
  std::string s = nh.address.ifName.value_or("?") + " metric " + std::to_string(nh.metric);
  if (nh.mplsAction) {
    static const char* names[] = {"PUSH", "SWAP", "PHP", "POP_AND_LOOKUP", "NOOP"};
    s += std::string(" ") + names[(int)nh.mplsAction->action];
    if (nh.mplsAction->swapLabel) {
      s += " " + std::to_string(*nh.mplsAction->swapLabel);
    }
  }
  return s;
}

} // namespace

int main() {
  const std::vector<std::pair<int, int>> ring = {{1, 2}, {2, 4}, {4, 3}, {3, 1}};
  std::unordered_map<std::string, LinkState> areas;
  areas.emplace("0", LinkState("0"));
  PrefixState prefixes;
  try {
    for (int n = 1; n <= 4; ++n) {
      thrift::AdjacencyDatabase db;
      db.thisNodeName = std::to_string(n);
      db.nodeLabel = 100 + n;
      db.area = "0";
      for (auto [a, b] : ring) {
        if (a == n) db.adjacencies.push_back(adj(a, b));
        if (b == n) db.adjacencies.push_back(adj(b, a));
      }
      areas.at("0").updateAdjacencyDatabase(db);
      thrift::PrefixDatabase pdb;
      pdb.thisNodeName = db.thisNodeName;
      thrift::PrefixEntry e;
      e.prefix = loopback(n);
      pdb.prefixEntries.push_back(e);
      prefixes.updatePrefixDatabase(pdb);
    }
    SpfSolver solver("1", false, false);
    auto db = solver.buildRouteDb("1", areas, prefixes);
    if (!db) {
      std::fprintf(stderr, "node 1 is in no area\n");
      return 1;
    }
    std::vector<std::string> lines;
    for (const auto& [prefix, entry] : db->unicastEntries) {
      for (const auto& nh : entry.nexthops) {
        lines.push_back("unicast fc00::" + std::to_string((int)(unsigned char)prefix.prefixAddress.addr[15]) +
                        "/128 via " + hopText(nh));
      }
    }
    for (const auto& [label, entry] : db->mplsEntries) {
      for (const auto& nh : entry.nexthops) {
        lines.push_back("mpls " + std::to_string(label) + " via " + hopText(nh));
      }
    }
    std::sort(lines.begin(), lines.end());
    for (const auto& l : lines) {
      std::printf("%s\n", l.c_str());
    }
    std::printf("spf_runs %lld\n", (long long)Counters::get("decision.spf_runs"));
    return 0;
  } catch (const std::exception& ex) {
    std::fprintf(stderr, "engine unavailable: %s\n", ex.what());
    return spf_device_count() > 0 ? 2 : 3;
  }
}
