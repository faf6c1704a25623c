// AllSourcesTable.cpp — see AllSourcesTable.h.
#include "AllSourcesTable.h"

#include <algorithm>
#include <chrono>
#include <stdexcept>

#include "Engine.h"

namespace openr {
namespace {

using Clock = std::chrono::steady_clock;

double msSince(Clock::time_point t) {
  return std::chrono::duration<double, std::milli>(Clock::now() - t).count();
}

void check(int s, const char* what) {
  if (s != SPF_OK) {
    throw std::runtime_error(std::string("MI355X SPF engine failure in ") + what + ": " +
                             spf_error_string(s) + " (" + spf_last_error_detail() + ")");
  }
}

} // namespace

spf_graph_desc AllSourcesTable::Csr::desc(int device) const {
  spf_graph_desc d{};
  d.num_nodes = (uint32_t)overloaded.size();
  d.num_edges = (uint32_t)col.size();
  d.row_ptr = row.data();
  d.col = col.data();
  d.metric = metric.data();
  d.link_id = linkId.data();
  d.rev = rev.data();
  d.node_overloaded = overloaded.data();
  d.num_links = numLinks;
  d.device = device;
  return d;
}

AllSourcesTable::Csr AllSourcesTable::snapshot(const LinkState& ls) const {
  LinkState::Engine& eng = ls.engine(); // builds the flat CSR if needed
  Csr c;
  c.row = eng.row;
  c.col = eng.col;
  c.linkId = eng.linkId;
  c.rev = eng.rev;
  c.metric = eng.metric;
  c.overloaded = eng.overloaded;
  c.numLinks = (uint32_t)eng.links.size();
  if (eng.names != names_ && !names_.empty()) {
    throw std::invalid_argument("AllSourcesTable::update: the node set changed, rebuild the table");
  }
  return c;
}

AllSourcesTable::AllSourcesTable(const LinkState& ls, std::vector<int> devices)
    : AllSourcesTable(ls, std::move(devices), false) {}

AllSourcesTable::AllSourcesTable(const LinkState& ls, std::vector<int> devices, bool withNextHops)
    : withNh_(withNextHops) {
  LinkState::Engine& eng = ls.engine();
  if (eng.exact) {
    throw std::invalid_argument(
        "AllSourcesTable: metric 0 / 64-bit sums need 64-bit rows (the exact kernels)");
  }
  names_ = eng.names;
  ids_ = eng.ids;
  cur_ = snapshot(ls);
  if (devices.empty()) {
    devices = getSpfDevices();
  }
  if (devices.empty()) {
    devices = {0};
  }
  const uint32_t V = (uint32_t)names_.size();
  const uint32_t n = (uint32_t)devices.size();
  // contiguous source blocks (spf_table_layout's split: n / world each, the
  // first n % world one more)
  uint32_t first = 0;
  try {
    for (uint32_t r = 0; r < n; ++r) {
      Block b;
      b.device = devices[r];
      b.first = first;
      b.count = V / n + (r < V % n ? 1 : 0);
      first += b.count;
      b.sources.resize(b.count);
      for (uint32_t i = 0; i < b.count; ++i) {
        b.sources[i] = b.first + i;
      }
      blocks_.push_back(std::move(b));
    }
    buildGraphs(cur_);
    for (auto& b : blocks_) {
      setHalo(b); // (allocates the rows)
    }
    recompute();
    if (withNh_) {
      for (auto& b : blocks_) {
        refreshMasks(b, {});
      }
    }
  } catch (...) {
    for (auto& b : blocks_) {
      if (b.graph) {
        spf_graph_destroy(b.graph);
      }
      spf_device_free(b.device, b.rows);
      spf_device_free(b.device, b.masks);
    }
    throw;
  }
}

bool AllSourcesTable::setHalo(Block& b) {
  const uint32_t V = (uint32_t)names_.size();
  std::vector<uint32_t> srcs(b.sources.begin(), b.sources.begin() + b.count);
  if (withNh_ && blocks_.size() > 1) {
    std::vector<uint8_t> mark(V, 0);
    for (uint32_t i = 0; i < b.count; ++i) {
      const uint32_t u = b.first + i;
      for (uint32_t e = layRow_[u]; e < layRow_[u + 1]; ++e) {
        const uint32_t f = layCol_[e];
        if (f < b.first || f >= b.first + b.count) {
          mark[f] = 1;
        }
      }
    }
    for (uint32_t f = 0; f < V; ++f) {
      if (mark[f]) {
        srcs.push_back(f);
      }
    }
  }
  const bool changed = srcs != b.sources || !b.rows;
  if (!changed) {
    return false;
  }
  b.sources = std::move(srcs);
  if (b.sources.size() > b.rowCap || !b.rows) {
    spf_device_free(b.device, b.rows);
    b.rows = nullptr;
    b.rowCap = 0;
    void* p = nullptr;
    check(spf_device_alloc(b.device, std::max<size_t>(b.sources.size(), 1) * V * 4, &p),
          "spf_device_alloc");
    b.rows = static_cast<uint32_t*>(p);
    b.rowCap = std::max<size_t>(b.sources.size(), 1);
  }
  if (withNh_) {
    b.rowOf.assign(V, -1);
    for (uint32_t r = 0; r < b.sources.size(); ++r) {
      b.rowOf[b.sources[r]] = (int32_t)r;
    }
  }
  return true;
}

void AllSourcesTable::refreshMasks(Block& b, const std::vector<uint32_t>& idx) {
  const uint32_t V = (uint32_t)names_.size();
  if (!b.count) {
    return;
  }
  if (idx.empty()) {
    // layout from the graph's current distinct-neighbour lists
    b.maskWords.assign(b.count, 1);
    b.maskOff.assign(b.count + 1, 0);
    for (uint32_t i = 0; i < b.count; ++i) {
      const int nb = spf_graph_num_nbrs(b.graph, b.first + i);
      check(nb < 0 ? nb : SPF_OK, "spf_graph_num_nbrs");
      b.maskWords[i] = std::max<uint32_t>(1, ((uint32_t)nb + 63) / 64);
      b.maskOff[i + 1] = b.maskOff[i] + (uint64_t)V * b.maskWords[i];
    }
    const size_t bytes = std::max<size_t>(b.maskOff[b.count], 1) * 8;
    if (bytes > b.maskBytes) {
      spf_device_free(b.device, b.masks);
      b.masks = nullptr;
      b.maskBytes = 0;
      void* p = nullptr;
      check(spf_device_alloc(b.device, bytes, &p), "spf_device_alloc");
      b.masks = static_cast<uint64_t*>(p);
      b.maskBytes = bytes;
    }
    std::vector<uint32_t> own(b.count);
    for (uint32_t i = 0; i < b.count; ++i) {
      own[i] = b.first + i;
    }
    check(spf_table_nexthops(b.graph, b.rows, V, b.rowOf.data(), b.count, own.data(), b.masks,
                             b.maskOff.data()),
          "spf_table_nexthops");
    return;
  }
  std::vector<uint32_t> srcs(idx.size());
  std::vector<uint64_t> off(idx.size());
  for (size_t k = 0; k < idx.size(); ++k) {
    srcs[k] = b.sources[idx[k]];
    off[k] = b.maskOff[idx[k]];
  }
  check(spf_table_nexthops(b.graph, b.rows, V, b.rowOf.data(), (uint32_t)srcs.size(), srcs.data(),
                           b.masks, off.data()),
        "spf_table_nexthops");
}

AllSourcesTable::~AllSourcesTable() {
  for (auto& b : blocks_) {
    if (b.graph) {
      spf_graph_destroy(b.graph);
    }
    spf_device_free(b.device, b.rows);
    spf_device_free(b.device, b.masks);
  }
}

void AllSourcesTable::buildGraphs(const Csr& c) {
  for (auto& b : blocks_) {
    spf_graph* g = nullptr;
    const spf_graph_desc d = c.desc(b.device);
    check(spf_graph_create(&d, &g), "spf_graph_create");
    if (b.graph) {
      spf_graph_destroy(b.graph);
    }
    b.graph = g;
  }
  layRow_ = c.row;
  layCol_ = c.col;
  layRev_ = c.rev;
  layUp_.assign(c.col.size(), 1);
  layW_ = c.metric;
}

// rows of `idx` (block-local row indices) recomputed: one batch query; the
// whole block lands in place (fetch_rows), a subset is scattered
void AllSourcesTable::computeBlock(Block& b, const std::vector<uint32_t>& idx, bool scatter) {
  if (idx.empty()) {
    return;
  }
  const uint32_t V = (uint32_t)names_.size();
  std::vector<uint32_t> srcs(idx.size());
  for (size_t i = 0; i < idx.size(); ++i) {
    srcs[i] = b.sources[idx[i]];
  }
  spf_query_desc qd{};
  qd.num_queries = (uint32_t)srcs.size();
  qd.sources = srcs.data();
  qd.flags = 0;
  spf_query* q = nullptr;
  check(spf_query_create(b.graph, &qd, &q), "spf_query_create");
  struct Guard {
    spf_query* q;
    ~Guard() { spf_query_destroy(q); }
  } guard{q};
  check(spf_query_run(q), "spf_query_run");
  if (scatter) {
    check(spf_query_scatter_rows(q, idx.data(), b.rows, (size_t)V * 4), "spf_query_scatter_rows");
  } else {
    check(spf_query_fetch_rows(q, 0, qd.num_queries, b.rows, (size_t)V * 4, 1),
          "spf_query_fetch_rows");
  }
  check(spf_query_sync(q), "spf_query_sync");
  float ms = 0;
  spf_query_elapsed_ms(q, &ms);
  lastSpfMs_ = std::max(lastSpfMs_, (double)ms);
}

void AllSourcesTable::recompute() {
  lastSpfMs_ = 0;
  for (auto& b : blocks_) {
    std::vector<uint32_t> all(b.sources.size());
    for (uint32_t i = 0; i < all.size(); ++i) {
      all[i] = i;
    }
    computeBlock(b, all, false);
  }
}

// Link-set deltas onto the resident layout (the C++ form of
// allsources.ShardedAllSources._links_in_place): a REMOVED half-edge
// (tail, head, metric) is an up slot going down, an ADDED one a down slot
// (tail, head) coming back up.  Slots are chosen as LINK PAIRS — the pull
// kernels read a slot's head with win[e] = the metric of its reverse half
// rev[e], so both halves of a link must be up or down together: an added
// half-edge takes the slot a removed delta of this update took down (a
// metric change), else a slot whose other half this pass brought up, else
// any down slot, and a result whose touched slots disagree with their
// reverse halves (parallel links matched across links) is refused.  false:
// rebuild (a new link, unpairable halves, a metric 0 / past 2^31 - 1).
bool AllSourcesTable::linksInPlace(
    const std::vector<spf_edge_delta>& deltas, std::vector<uint32_t>& edges,
    std::vector<uint8_t>& up, std::vector<uint64_t>& w) {
  std::vector<uint8_t> lu = layUp_;
  std::vector<uint64_t> lw = layW_;
  // 1: touched by a REMOVED delta, 2: brought up by an ADDED one
  std::vector<uint8_t> touched(layCol_.size(), 0);
  for (int pass = 0; pass < 2; ++pass) { // REMOVED first (a metric change is both)
    const uint32_t kind = pass == 0 ? SPF_DELTA_REMOVED : SPF_DELTA_ADDED;
    for (const auto& d : deltas) {
      if (d.scope == SPF_SCOPE_NOT_TAIL || d.kind != kind) {
        continue; // transit flips are set_transit's
      }
      if (d.metric == 0 || d.metric > 0x7FFFFFFFull) {
        return false;
      }
      uint32_t hit = ~0u;
      int rank = 3;
      for (uint32_t e = layRow_[d.tail]; e < layRow_[d.tail + 1]; ++e) {
        if (layCol_[e] != d.head) {
          continue;
        }
        if (kind == SPF_DELTA_REMOVED) {
          if (lu[e] && lw[e] == d.metric) {
            hit = e;
            break;
          }
          continue;
        }
        if (lu[e]) {
          continue;
        }
        const int r = (touched[e] & 1u) ? 0 : ((touched[layRev_[e]] & 2u) && lu[layRev_[e]]) ? 1 : 2;
        if (r < rank) {
          rank = r;
          hit = e;
        }
      }
      if (hit == ~0u) {
        return false;
      }
      lu[hit] = kind == SPF_DELTA_ADDED;
      if (kind == SPF_DELTA_ADDED) {
        lw[hit] = d.metric;
      }
      touched[hit] |= kind == SPF_DELTA_REMOVED ? 1u : 2u;
    }
  }
  edges.clear();
  up.clear();
  w.clear();
  for (uint32_t e = 0; e < touched.size(); ++e) {
    if (touched[e]) {
      if (lu[e] != lu[layRev_[e]]) {
        return false; // the halves of a link disagree
      }
      edges.push_back(e);
      up.push_back(lu[e]);
      w.push_back(lw[e]);
    }
  }
  layUp_ = std::move(lu);
  layW_ = std::move(lw);
  return true;
}

AllSourcesTable::UpdateStats AllSourcesTable::update(const LinkState& ls) {
  UpdateStats st;
  const auto t0 = Clock::now();
  if (ls.engine().exact) {
    throw std::invalid_argument("AllSourcesTable::update: the new topology needs 64-bit rows");
  }
  Csr nc = snapshot(ls);
  if (stale_) {
    // a failed update patched the graphs but left the old rows: start over
    buildGraphs(nc);
    cur_ = std::move(nc);
    if (spf_graph_needs_exact(blocks_.front().graph)) {
      throw std::invalid_argument("AllSourcesTable::update: the new topology needs 64-bit rows");
    }
    for (auto& b : blocks_) {
      setHalo(b);
    }
    recompute();
    if (withNh_) {
      for (auto& b : blocks_) {
        refreshMasks(b, {});
      }
    }
    stale_ = false;
    st.affected = (uint32_t)names_.size();
    st.spfMs = lastSpfMs_;
    st.wallMs = msSince(t0);
    return st;
  }
  const uint32_t V = (uint32_t)names_.size();
  // edge deltas
  std::vector<spf_edge_delta> deltas;
  {
    const spf_graph_desc a = cur_.desc(0), b = nc.desc(0);
    uint32_t n = 0;
    check(spf_graph_diff(&a, &b, nullptr, 0, &n), "spf_graph_diff");
    deltas.resize(n);
    if (n) {
      check(spf_graph_diff(&a, &b, deltas.data(), n, &n), "spf_graph_diff");
    }
  }
  st.deltas = (uint32_t)deltas.size();
  st.diffMs = msSince(t0);
  // device graphs: in place when the link set is the layout's, or links went
  // down / came back up; rebuilt for a new link
  const auto tg = Clock::now();
  const bool sameLinks = nc.row == cur_.row && nc.col == cur_.col && nc.linkId == cur_.linkId &&
                         nc.rev == cur_.rev;
  const bool layoutIsCur = std::all_of(layUp_.begin(), layUp_.end(), [](uint8_t x) { return x; }) &&
                           layRow_ == cur_.row && layCol_ == cur_.col;
  const bool transit = nc.overloaded != cur_.overloaded;
  std::vector<uint32_t> edges;
  std::vector<uint8_t> up;
  std::vector<uint64_t> w;
  bool linkSetChanged = true; // next hops: neighbour lists (mask bits) may move
  if (sameLinks && layoutIsCur) {
    linkSetChanged = false;
    std::vector<uint32_t> ch;
    std::vector<uint64_t> cm;
    for (uint32_t e = 0; e < nc.metric.size(); ++e) {
      if (nc.metric[e] != cur_.metric[e]) {
        ch.push_back(e);
        cm.push_back(nc.metric[e]);
      }
    }
    for (auto& b : blocks_) {
      if (!ch.empty()) {
        check(spf_graph_patch_metrics(b.graph, (uint32_t)ch.size(), ch.data(), cm.data()),
              "spf_graph_patch_metrics");
      }
      if (transit) {
        check(spf_graph_set_transit(b.graph, nc.overloaded.data()), "spf_graph_set_transit");
      }
    }
    layW_ = nc.metric;
    st.graphPatched = true;
  } else if (linksInPlace(deltas, edges, up, w)) {
    for (auto& b : blocks_) {
      if (!edges.empty()) {
        check(spf_graph_set_edges(b.graph, (uint32_t)edges.size(), edges.data(), up.data(),
                                  w.data()),
              "spf_graph_set_edges");
      }
      if (transit) {
        check(spf_graph_set_transit(b.graph, nc.overloaded.data()), "spf_graph_set_transit");
      }
    }
    st.graphPatched = true;
  } else {
    buildGraphs(nc);
  }
  cur_ = std::move(nc);
  st.graphMs = msSince(tg);
  if (spf_graph_needs_exact(blocks_.front().graph)) {
    stale_ = true;
    throw std::invalid_argument("AllSourcesTable::update: the new topology needs 64-bit rows");
  }
  // screen, then repair (or recompute) the affected rows of each block (its
  // halo rows included); a block whose halo a rebuilt layout changed is
  // recomputed whole
  lastSpfMs_ = 0;
  bool anyRelaxed = false, anyRecomputed = false;
  std::vector<std::vector<uint32_t>> hitRows(blocks_.size()); // own rows repaired, per block
  std::vector<uint8_t> fresh(blocks_.size(), 0);
  if (!st.graphPatched) {
    for (size_t k = 0; k < blocks_.size(); ++k) {
      if (setHalo(blocks_[k])) {
        std::vector<uint32_t> all(blocks_[k].sources.size());
        for (uint32_t i = 0; i < all.size(); ++i) {
          all[i] = i;
        }
        computeBlock(blocks_[k], all, false);
        fresh[k] = 1;
        anyRecomputed = true;
      }
    }
  }
  for (size_t k = 0; k < blocks_.size(); ++k) {
    Block& b = blocks_[k];
    const uint32_t nr = (uint32_t)b.sources.size();
    if (!nr || deltas.empty() || fresh[k]) {
      continue;
    }
    const auto ts = Clock::now();
    std::vector<uint8_t> hit(nr, 0);
    check(spf_table_screen(b.graph, b.rows, V, nr, b.sources.data(), deltas.data(),
                           (uint32_t)deltas.size(), hit.data()),
          "spf_table_screen");
    st.screenMs += msSince(ts);
    std::vector<uint32_t> idx, srcs;
    for (uint32_t i = 0; i < nr; ++i) {
      if (hit[i]) {
        idx.push_back(i);
        srcs.push_back(b.sources[i]);
        if (i < b.count) {
          ++st.affected; // own rows (halo rows repeat another block's)
          hitRows[k].push_back(i);
        }
      }
    }
    if (idx.empty()) {
      continue;
    }
    const auto tr = Clock::now();
    const int s = spf_table_repair(b.graph, b.rows, V, (uint32_t)idx.size(), srcs.data(),
                                   idx.data(), deltas.data(), (uint32_t)deltas.size());
    if (s == SPF_OK) {
      anyRelaxed = true;
    } else if (s == SPF_E_UNSUPPORTED) {
      computeBlock(b, idx, true);
      anyRecomputed = true;
    } else {
      check(s, "spf_table_repair");
    }
    st.spfMs += msSince(tr);
  }
  st.relaxed = anyRelaxed && !anyRecomputed;
  if (withNh_ && !deltas.empty()) {
    // a source the screen passed keeps its masks (defined by its tight edges
    // alone) unless its neighbour list moved; a link-set change may move any
    // (the neighbours' rows it reads are the block's halo, repaired above)
    const auto tn = Clock::now();
    for (size_t k = 0; k < blocks_.size(); ++k) {
      if (linkSetChanged || fresh[k]) {
        refreshMasks(blocks_[k], {});
      } else if (!hitRows[k].empty()) {
        refreshMasks(blocks_[k], hitRows[k]);
      }
    }
    st.nextHopsMs = msSince(tn);
  }
  st.wallMs = msSince(t0);
  return st;
}

std::vector<std::string> AllSourcesTable::nextHops(const std::string& src,
                                                   const std::string& dst) const {
  if (!withNh_) {
    throw std::logic_error("AllSourcesTable::nextHops: table built without next hops");
  }
  if (stale_) {
    throw std::logic_error("AllSourcesTable::nextHops: the last update() failed, the rows are stale");
  }
  const auto s = ids_.find(src), d = ids_.find(dst);
  if (s == ids_.end() || d == ids_.end()) {
    throw std::out_of_range("AllSourcesTable::nextHops: unknown node");
  }
  const Block* bp = nullptr;
  for (const auto& x : blocks_) {
    if (s->second >= x.first && s->second < x.first + x.count) {
      bp = &x;
    }
  }
  if (!bp) {
    throw std::out_of_range("AllSourcesTable::nextHops: no block holds " + src);
  }
  const Block& b = *bp;
  const uint32_t i = s->second - b.first;
  const uint32_t V = (uint32_t)names_.size(), W = b.maskWords[i];
  std::vector<uint64_t> m(W);
  check(spf_device_memcpy(b.device, m.data(), b.masks + b.maskOff[i] + (size_t)d->second * W,
                          (size_t)W * 8, SPF_COPY_D2H),
        "spf_device_memcpy");
  const int nn = spf_graph_num_nbrs(b.graph, s->second);
  check(nn < 0 ? nn : SPF_OK, "spf_graph_num_nbrs");
  std::vector<uint32_t> nb(std::max(nn, 0));
  if (nn > 0) {
    check(spf_graph_nbrs(b.graph, s->second, nb.data()), "spf_graph_nbrs");
  }
  std::vector<std::string> out;
  for (uint32_t w = 0; w < W; ++w) {
    for (uint64_t x = m[w]; x; x &= x - 1) {
      const uint32_t bit = w * 64 + (uint32_t)__builtin_ctzll(x);
      if (bit < nb.size()) {
        out.push_back(names_[nb[bit]]);
      }
    }
  }
  (void)V;
  std::sort(out.begin(), out.end());
  return out;
}

std::vector<uint32_t> AllSourcesTable::row(const std::string& src) const {
  if (stale_) {
    throw std::logic_error("AllSourcesTable::row: the last update() failed, the rows are stale");
  }
  const auto it = ids_.find(src);
  if (it == ids_.end()) {
    throw std::out_of_range("AllSourcesTable::row: unknown node " + src);
  }
  const uint32_t V = (uint32_t)names_.size();
  for (const auto& b : blocks_) {
    if (it->second >= b.first && it->second < b.first + b.count) {
      std::vector<uint32_t> out(V);
      check(spf_device_memcpy(b.device, out.data(), b.rows + (size_t)(it->second - b.first) * V,
                              (size_t)V * 4, SPF_COPY_D2H),
            "spf_device_memcpy");
      return out;
    }
  }
  throw std::out_of_range("AllSourcesTable::row: no block holds " + src);
}

std::optional<uint64_t> AllSourcesTable::distance(const std::string& src,
                                                  const std::string& dst) const {
  const auto dit = ids_.find(dst);
  if (dit == ids_.end()) {
    return std::nullopt;
  }
  const uint32_t d = row(src)[dit->second];
  return d == 0xFFFFFFFFu ? std::nullopt : std::optional<uint64_t>(d);
}

} // namespace openr
