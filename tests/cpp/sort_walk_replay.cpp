// Host replay of the device sort's reuse walk (svscope_amd/csrc/poa_fold.hip
// dfs_sort): for every fold of a POA task, the walk over the previous rank
// order's segments (64-rank windows over the segment-start bit plane, exactly
// as the kernel does it) followed by the root scan of the new ids, checked
// against spoa's full DFS order (the oracle's Graph::topological_sort).
// Test tooling only (it links the CPU oracle).
//
//   g++ -O2 -std=c++17 -o /tmp/sort_walk_replay tests/cpp/sort_walk_replay.cpp
//   /tmp/sort_walk_replay SEQS.txt SEED TRIALS
//
// SEQS.txt: one sequence per line (a task's reads in order).  Trial 0 folds
// them all; trials 1.. fold random thirds of them (consensus-like subsets).
// Prints the DFS examinations the walk still runs and the ranks it copies.
#include "../../oracle/spoa_oracle.cpp"
#include <fstream>
#include <iostream>
#include <random>
using namespace oracle;
struct Prev { std::vector<uint32_t> r2n, col; std::vector<uint8_t> seg; size_t V = 0; };
static bool walk_sort(Graph& g, Prev& pv, const std::vector<uint8_t>& chg, uint64_t& exams, uint64_t& copies) {
  const uint32_t V = g.nodes.size(), V0 = pv.V;
  std::vector<uint8_t> done(V, 0), ign(V, 0);
  std::vector<uint32_t> r2n, col(V, 0xFFFFFFFF); std::vector<uint8_t> nseg;
  uint32_t ncol = 0;
  auto emit = [&](uint32_t v) { r2n.push_back(v); col[v] = ncol; nseg.push_back(0); };
  auto run_root = [&](uint32_t root) {
    nseg.push_back(0); nseg.pop_back();
    size_t start = r2n.size();
    Node* rn = g.nodes[root].get();
    // fast path: all tails and aligned below root; no done bits set
    bool fast = rn->inedges.size() <= 3;
    for (Edge* e : rn->inedges) fast = fast && e->tail->id < root;
    for (Node* a : rn->aligned) fast = fast && a->id < root;
    auto isdone = [&](uint32_t v) { return v < root || done[v]; };
    if (fast) { emit(root); for (Node* a : rn->aligned) emit(a->id); ++ncol; }
    else {
      std::vector<uint32_t> st{root};
      while (!st.empty()) {
        uint32_t cur = st.back(); ++exams; Node* c = g.nodes[cur].get();
        if (done[cur]) { st.pop_back(); continue; }
        bool ok = true;
        for (Edge* e : c->inedges) if (!isdone(e->tail->id)) { st.push_back(e->tail->id); ok = false; }
        if (!ign[cur]) for (Node* a : c->aligned) if (!isdone(a->id)) { st.push_back(a->id); ign[a->id] = 1; ok = false; }
        if (ok) { done[cur] = 1; if (!ign[cur]) { emit(cur); for (Node* a : c->aligned) emit(a->id); ++ncol; } st.pop_back(); }
      }
    }
    if (r2n.size() > start) nseg[start] = 1; else { std::cerr << "root emitted nothing\n"; }
  };
  // exact port of the device walk (64-rank windows over bit planes)
  std::vector<uint32_t> segw((V0 + 31) / 32 + 2, 0);
  for (uint32_t k = 0; k < V0; ++k) if (pv.seg[k]) segw[k >> 5] |= 1u << (k & 31);
  auto seg_window = [&](uint32_t p) -> uint64_t {
    uint32_t a = p >> 5, s = p & 31;
    uint64_t lo = segw[a] | ((uint64_t)segw[a + 1] << 32), hi = segw[a + 2];
    uint64_t m = s ? (lo >> s) | (hi << (64 - s)) : lo;
    uint32_t left = V0 - p;
    if (left < 64) m = (m & ((1ull << left) - 1)) | (1ull << left);
    return m;
  };
  auto next_start = [&](uint32_t q) -> uint32_t {
    while (q < V0) { uint32_t w = segw[q >> 5] >> (q & 31); if (w) return std::min(q + (uint32_t)__builtin_ctz(w), V0); q = (q | 31) + 1; }
    return V0;
  };
  auto bad_of = [&](uint32_t v) { return chg[v] || done[v]; };
  auto copy_chunk = [&](const uint32_t* nd, uint32_t k, uint32_t c0, uint64_t st) {
    for (uint32_t l = 0; l < k; ++l) { uint32_t v = nd[l]; r2n.push_back(v); col[v] = ncol + pv.col[v] - c0; done[v] = 1; nseg.push_back((st >> l) & 1); }
    return pv.col[nd[k - 1]];
  };
  uint32_t p = 0;
  while (p < V0) {
    uint32_t nd[64]; bool in[64];
    for (int l = 0; l < 64; ++l) { in[l] = p + l < V0; nd[l] = in[l] ? pv.r2n[p + l] : 0; }
    uint64_t sm = seg_window(p), bad = 0;
    for (int l = 0; l < 64; ++l) if (in[l] && bad_of(nd[l])) bad |= 1ull << l;
    uint64_t upto = bad ? (2ull << __builtin_ctzll(bad)) - 1 : ~0ull;
    uint64_t ends = sm & upto & ~1ull;
    if (ends) {
      uint32_t k = 63 - __builtin_clzll(ends);
      uint32_t c0 = pv.col[nd[0]];
      uint32_t cl = copy_chunk(nd, k, c0, sm);
      ncol += cl + 1 - c0; copies += k; p += k; continue;
    }
    uint64_t rest = sm & ~1ull;
    uint32_t e = rest ? p + __builtin_ctzll(rest) : next_start(p + 64);
    uint32_t n0 = std::min(e - p, 64u);
    uint32_t r = 0xFFFFFFFF; for (uint32_t l = 0; l < n0; ++l) r = std::min(r, nd[l]);
    bool clean = (bad & (n0 < 64 ? (1ull << n0) - 1 : ~0ull)) == 0;
    for (uint32_t c = p + 64; c < e; c += 64) for (uint32_t l = 0; l < 64 && c + l < e; ++l) { uint32_t v = pv.r2n[c + l]; if (bad_of(v)) clean = false; r = std::min(r, v); }
    if (clean) {
      uint32_t c0 = pv.col[nd[0]], cl = c0;
      for (uint32_t c = p; c < e; c += 64) { uint32_t ch[64]; uint32_t k = std::min(e - c, 64u); for (uint32_t l = 0; l < k; ++l) ch[l] = pv.r2n[c + l]; cl = copy_chunk(ch, k, c0, c == p ? 1 : 0); }
      ncol += cl + 1 - c0; copies += e - p; p = e; continue;
    }
    p = e;
    if (done[r]) continue;
    run_root(r);
  }
  // new ids (or all ids)
  for (uint32_t v = V0; v < V; ++v) if (!done[v]) {
    // done-by-emission check: fast-path roots have no done bit but are emitted
    bool emitted = col[v] != 0xFFFFFFFF;
    if (!emitted) run_root(v);
  }
  if (r2n.size() != V) { std::cerr << "count " << r2n.size() << " != " << V << "\n"; return false; }
  for (uint32_t i = 0; i < V; ++i) if (r2n[i] != g.rank_to_node[i]->id) { std::cerr << "order differs at " << i << "\n"; return false; }
  pv.r2n = r2n; pv.col = col; pv.seg = nseg; pv.V = V;
  return true;
}
int main(int argc, char** argv) {
  std::ifstream f(argv[1]); std::vector<std::string> all; std::string l;
  while (std::getline(f, l)) if (!l.empty()) all.push_back(l);
  std::mt19937 rng(atoi(argv[2]));
  int trials = atoi(argv[3]);
  Params P{5, -4, -8, -6, -10, -4};
  uint64_t ex = 0, cp = 0;
  for (int t = 0; t < trials; ++t) {
    std::vector<std::string> seqs;
    if (t == 0) seqs = all;
    else { for (auto& s : all) if (rng() % 3 == 0) seqs.push_back(s); if (seqs.empty()) continue; }
    Graph g; Prev pv; Stats stt;
    for (size_t s = 0; s < seqs.size(); ++s) {
      std::vector<size_t> indeg, alc;
      for (auto& n : g.nodes) { indeg.push_back(n->inedges.size()); alc.push_back(n->aligned.size()); }
      auto aln = align_nw_convex(seqs[s], g, P, &stt);
      g.add_alignment(aln, seqs[s]);
      std::vector<uint8_t> ch(g.nodes.size(), 1);
      for (size_t v = 0; v < indeg.size(); ++v) ch[v] = g.nodes[v]->inedges.size() != indeg[v] || g.nodes[v]->aligned.size() != alc[v];
      if (s == 0) { pv.V = g.nodes.size(); pv.r2n.clear(); pv.col.clear(); pv.seg.assign(pv.V, 1);
        for (auto* nd : g.rank_to_node) pv.r2n.push_back(nd->id);
        pv.col.resize(pv.V); for (uint32_t i = 0; i < pv.V; ++i) pv.col[pv.r2n[i]] = i; continue; }
      if (!walk_sort(g, pv, ch, ex, cp)) { std::cerr << "trial " << t << " fold " << s << " failed\n"; return 1; }
    }
  }
  std::printf("ok: exams %lu copied ranks %lu\n", ex, cp);
}
