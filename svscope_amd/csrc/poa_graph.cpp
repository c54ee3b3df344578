// Flat-array POA graph: host half of the batched MI355X POA engine.
// See poa_graph.hpp for the semantic contract (spoa 4.x Graph behaviour).
#include "poa_graph.hpp"

#include <algorithm>
#include <climits>
#include <cstdlib>
#include <stdexcept>

namespace svs {

static constexpr uint32_t kNone = 0xFFFFFFFFu;

uint32_t PoaGraph::new_node(char b) {
  const uint32_t id = static_cast<uint32_t>(base_.size());
  base_.push_back(b);
  in_.emplace_back();
  out_.emplace_back();
  aligned_.emplace_back();
  cov_.push_back(0);
  cov_last_.push_back(0);
  return id;
}

void PoaGraph::link(uint32_t tail, uint32_t head, int64_t w, uint32_t seq_id) {
  const uint32_t tag = seq_id + 1;
  for (uint32_t x : {tail, head}) {
    if (cov_last_[x] != tag) { cov_last_[x] = tag; ++cov_[x]; }
  }
  for (uint32_t e : out_[tail]) {
    if (e_head_[e] == head) { e_w_[e] += w; return; }
  }
  const uint32_t e = static_cast<uint32_t>(e_tail_.size());
  e_tail_.push_back(tail);
  e_head_.push_back(head);
  e_w_.push_back(w);
  out_[tail].push_back(e);
  in_[head].push_back(e);
}

uint32_t PoaGraph::chain(const std::string& s, uint32_t b, uint32_t e, std::vector<uint32_t>* path) {
  if (b == e) return kNone;
  const uint32_t sid = static_cast<uint32_t>(paths_.size());
  uint32_t prev = new_node(s[b]);
  path->push_back(prev);
  for (uint32_t i = b + 1; i < e; ++i) {
    const uint32_t cur = new_node(s[i]);
    link(prev, cur, 2, sid);
    path->push_back(cur);
    prev = cur;
  }
  return (*path)[0];
}

void PoaGraph::add_alignment_ranks(const std::vector<int32_t>& rank_pairs, const std::string& seq) {
  std::vector<std::pair<int32_t, int32_t>> np;
  np.reserve(rank_pairs.size() / 2);
  for (size_t k = 0; k + 1 < rank_pairs.size(); k += 2) {
    const int32_t r = rank_pairs[k];
    np.emplace_back(r < 0 ? -1 : static_cast<int32_t>(rank_to_node_.at(static_cast<size_t>(r))),
                    rank_pairs[k + 1]);
  }
  add_alignment_nodes(np, seq);
}

void PoaGraph::add_alignment_nodes(const std::vector<std::pair<int32_t, int32_t>>& aln,
                                   const std::string& seq) {
  if (seq.empty()) return;
  const uint32_t sid = static_cast<uint32_t>(paths_.size());
  std::vector<uint32_t> path;
  path.reserve(seq.size());
  if (aln.empty()) {
    chain(seq, 0, static_cast<uint32_t>(seq.size()), &path);
    paths_.push_back(std::move(path));
    sort_ranks();
    return;
  }
  int32_t first = -1, last = -1;
  for (const auto& p : aln) {
    if (p.second == -1) continue;
    if (p.second < 0 || p.second >= static_cast<int32_t>(seq.size()))
      throw std::runtime_error("alignment position out of range");
    if (first == -1) first = p.second;
    last = p.second;
  }
  if (first == -1) throw std::runtime_error("alignment consumes no sequence");
  // spoa creates the prefix chain, then the suffix chain, then the middle.
  chain(seq, 0, static_cast<uint32_t>(first), &path);
  uint32_t prev = path.empty() ? kNone : path.back();
  std::vector<uint32_t> suffix;
  const uint32_t suffix_head =
      chain(seq, static_cast<uint32_t>(last) + 1, static_cast<uint32_t>(seq.size()), &suffix);
  for (const auto& p : aln) {
    if (p.second == -1) continue;
    const char letter = seq[static_cast<size_t>(p.second)];
    uint32_t cur = kNone;
    if (p.first == -1) {
      cur = new_node(letter);
    } else {
      const uint32_t n = static_cast<uint32_t>(p.first);
      if (base_[n] == letter) {
        cur = n;
      } else {
        for (uint32_t a : aligned_[n])
          if (base_[a] == letter) { cur = a; break; }
        if (cur == kNone) {
          cur = new_node(letter);
          for (uint32_t a : aligned_[n]) {
            aligned_[a].push_back(cur);
            aligned_[cur].push_back(a);
          }
          aligned_[n].push_back(cur);
          aligned_[cur].push_back(n);
        }
      }
    }
    if (prev != kNone) link(prev, cur, 2, sid);
    path.push_back(cur);
    prev = cur;
  }
  if (suffix_head != kNone) {
    link(prev, suffix_head, 2, sid);
    path.insert(path.end(), suffix.begin(), suffix.end());
  }
  paths_.push_back(std::move(path));
  sort_ranks();
}

void PoaGraph::sort_ranks() {
  // spoa's DFS topological sort (aligned groups kept contiguous), with the
  // mark / ignored flags in one byte array and a raw stack: the same visit
  // order as the textbook form, fewer instructions per visit
  const uint32_t n = num_nodes();
  rank_to_node_.resize(n);
  uint32_t* __restrict__ order = rank_to_node_.data();
  uint32_t cnt = 0;
  static thread_local std::vector<uint8_t> flags;  // bits 0-1: 0 new, 1 open, 2 done; bit 2: ignored
  static thread_local std::vector<uint32_t> stack;
  flags.assign(n, 0);
  if (stack.size() < e_tail_.size() + 2 * static_cast<size_t>(n) + 64) stack.resize(e_tail_.size() + 2 * n + 64);
  uint8_t* __restrict__ fl = flags.data();
  uint32_t* stk = stack.data();
  const uint32_t* __restrict__ etail = e_tail_.data();
  seg_start_.assign(n, 0);
  for (uint32_t root = 0; root < n; ++root) {
    if (fl[root] != 0) continue;
    if (cnt < n) seg_start_[cnt] = 1;
    size_t sp = 0;
    stk[sp++] = root;
    while (sp != 0) {
      const uint32_t cur = stk[sp - 1];
      if ((fl[cur] & 3) == 2) {
        --sp;
        continue;
      }
      bool ready = true;
      const NodeList& al = aligned_[cur];
      if (sp + in_[cur].size() + al.size() + 1 > stack.size()) {
        stack.resize(2 * stack.size());
        stk = stack.data();
      }
      for (uint32_t e : in_[cur]) {
        const uint32_t t = etail[e];
        if ((fl[t] & 3) != 2) { stk[sp++] = t; ready = false; }
      }
      if (!(fl[cur] & 4)) {
        for (uint32_t a : al) {
          if ((fl[a] & 3) != 2) { stk[sp++] = a; fl[a] |= 4; ready = false; }
        }
      }
      if (ready) {
        fl[cur] = static_cast<uint8_t>((fl[cur] & 4) | 2);
        if (!(fl[cur] & 4)) {
          order[cnt++] = cur;
          for (uint32_t a : al) order[cnt++] = a;
        }
        --sp;
      } else {
        fl[cur] = static_cast<uint8_t>((fl[cur] & 4) | 1);
      }
    }
  }
  rank_to_node_.resize(cnt);
  node_to_rank_.resize(n);
  uint32_t* __restrict__ n2r = node_to_rank_.data();
  for (uint32_t r = 0; r < cnt; ++r) n2r[order[r]] = r;
}

void PoaGraph::export_rows(RowTables* t) const {
  const uint32_t V = num_nodes();
  t->info.resize(V);
  t->slot.resize(V);
  t->pstart.resize(V + 1);
  t->pred_row.clear();
  t->pred_slot.clear();
  t->max_preds = 0;
  static thread_local std::vector<uint32_t> last_use, free_slots;
  last_use.resize(V);
  free_slots.clear();
  uint32_t np = 0;
  for (uint32_t r = 0; r < V; ++r) {
    const uint32_t node = rank_to_node_[r];
    t->info[r] = static_cast<uint8_t>(base_[node]) | (out_[node].empty() ? 0x100u : 0u);
    t->pstart[r] = np;
    last_use[r] = r;
    for (uint32_t e : in_[node]) {
      const uint32_t pr = node_to_rank_[e_tail_[e]];
      t->pred_row.push_back(pr + 1);
      last_use[pr] = std::max(last_use[pr], r);
      ++np;
    }
    t->max_preds = std::max<uint32_t>(t->max_preds, static_cast<uint32_t>(in_[node].size()));
  }
  t->pstart[V] = np;
  t->n_rows = V;
  t->n_edges = np;
  t->pred_slot.resize(np);
  // Row-pool slot assignment: a row lives from its computation until its last
  // successor has been computed; slot 0 holds the virtual row 0 for the whole job.
  uint32_t next = 1;
  for (uint32_t r = 0; r < V; ++r) {
    uint32_t s;
    if (free_slots.empty()) {
      s = next++;
    } else {
      s = free_slots.back();
      free_slots.pop_back();
    }
    t->slot[r] = s;
    for (uint32_t k = t->pstart[r]; k < t->pstart[r + 1]; ++k) {
      const uint32_t pr = t->pred_row[k] - 1;
      t->pred_slot[k] = t->slot[pr];
    }
    for (uint32_t k = t->pstart[r]; k < t->pstart[r + 1]; ++k) {
      const uint32_t pr = t->pred_row[k] - 1;
      if (last_use[pr] == r) free_slots.push_back(t->slot[pr]);
    }
    if (last_use[r] == r) free_slots.push_back(s);
  }
  t->n_slots = next;
}

void PoaGraph::export_strip_rows(RowTables* t) const { export_strip_rows(t, nullptr); }

void PoaGraph::export_strip_rows(RowTables* t, const int32_t* gaps) const {
  const uint32_t V = num_nodes();
  const uint32_t E = static_cast<uint32_t>(e_tail_.size());  // every edge is one in-edge entry
  t->info.clear();
  t->slot.clear();
  t->pstart.resize(V + 1);
  t->pred_row.resize(E);
  t->pred_slot.resize(E);
  t->rec.resize(static_cast<size_t>(V) * kRecWords);
  if (gaps) t->col0.resize(3 * static_cast<size_t>(V));
  const StripDst dst{t->rec.data(), t->pstart.data(), t->pred_row.data(), t->pred_slot.data(),
                     gaps ? t->col0.data() : nullptr};
  export_strip_rows(t, gaps, &dst);
}

void PoaGraph::export_strip_rows(RowTables* t, const int32_t* gaps, const StripDst* dst) const {
  const uint32_t V = num_nodes();
  const uint32_t E = static_cast<uint32_t>(e_tail_.size());
  t->n_rows = V;
  t->n_edges = E;
  t->lite = false;
  static thread_local std::vector<uint32_t> lds_last, slot, free_slots, dmin, dmax;
  lds_last.assign(V, 0);
  slot.resize(V);
  free_slots.clear();
  uint32_t* __restrict__ pred_row = dst->pred_row;
  uint32_t* __restrict__ pstart = dst->pstart;
  uint32_t* __restrict__ last = lds_last.data();
  const uint32_t* __restrict__ n2r = node_to_rank_.data();
  const uint32_t* __restrict__ etail = e_tail_.data();
  // pass 1 (ranks forward): in-edge rows (CSR), per row the last row that
  // reads it through the pool (an in-edge from the row just above does not),
  // and with gaps = {g, e, q, c} the column-0 values (fill_col0, fused)
  int32_t* __restrict__ c0 = gaps ? dst->col0 : nullptr;
  uint32_t k = 0, max_preds = 0;
  for (uint32_t r = 0; r < V; ++r) {
    const NodeList& in = in_[rank_to_node_[r]];
    pstart[r] = k;
    max_preds = std::max(max_preds, in.size());
    int32_t F0 = INT32_MIN + 1024, O0 = INT32_MIN + 1024;
    for (uint32_t e : in) {
      const uint32_t pr = n2r[etail[e]];
      pred_row[k++] = pr + 1;
      if (pr + 1 != r && last[pr] < r + 1) last[pr] = r + 1;
      if (c0) {
        F0 = std::max(F0, c0[3 * pr + 1]);
        O0 = std::max(O0, c0[3 * pr + 2]);
      }
    }
    if (c0) {
      if (in.empty()) {
        F0 = gaps[0];
        O0 = gaps[2];
      } else {
        F0 += gaps[1];
        O0 += gaps[3];
      }
      c0[3 * r] = std::max(F0, O0);
      c0[3 * r + 1] = F0;
      c0[3 * r + 2] = O0;
    }
  }
  pstart[V] = k;
  t->max_preds = max_preds;
  // pass 2 (forward): pool slots (a slot is free again after its row's last
  // reader) and row records w0, w1, w3
  uint32_t* __restrict__ pslot = dst->pred_slot;
  uint32_t* __restrict__ rec = dst->rec;
  // slot 0: virtual row 0.  Test hook: SVS_POA_TEST_WIDE_SLOTS=<n> numbers the
  // slots of graphs with >= n rows from 40 up, so that jobs with slot indices
  // past the pruning kernel's 31 liveness bits share launches with pruned ones.
  // (read per call, ~1 us against the export's ~0.3 ms: tests set it mid-process)
  const char* wide_env = std::getenv("SVS_POA_TEST_WIDE_SLOTS");
  const uint32_t wide_rows = wide_env ? static_cast<uint32_t>(std::strtoul(wide_env, nullptr, 10)) : 0u;
  uint32_t next = (wide_rows != 0 && V >= wide_rows) ? 40 : 1;
  for (uint32_t r = 0; r < V; ++r) {
    const uint32_t node = rank_to_node_[r];
    const bool store = last[r] != 0;
    uint32_t own = kNoSlot;
    if (store) {
      if (free_slots.empty()) {
        own = next++;
      } else {
        own = free_slots.back();
        free_slots.pop_back();
      }
    }
    slot[r] = own;
    const uint32_t a = pstart[r], b = pstart[r + 1];
    uint32_t* w = rec + static_cast<size_t>(r) * kRecWords;
    w[0] = static_cast<uint8_t>(base_[node]) | (out_[node].empty() ? 0x100u : 0u) | (store ? 0x200u : 0u) |
           (std::min<uint32_t>(b - a, 63u) << 10) | (own << 16);  // in-degree 63: >= 63 (pstart has it)
    uint32_t w1 = 0, w3 = 0;  // a source's in-edge comes from the virtual row 0 (slot 0)
    for (uint32_t x = a; x < b; ++x) {
      const uint32_t pr = pred_row[x] - 1;
      const uint32_t ps = (pr + 1 == r) ? kNoSlot : slot[pr];
      pslot[x] = ps;
      if (x - a < kInlinePreds) w1 |= ps << (16 * (x - a));
      if (pr + 1 != r && last[pr] == r + 1) {
        free_slots.push_back(ps);
        // the pruning kernel's liveness bits: slots 0..30 (bit 31 is its
        // register row; slots >= 31 have no bit and count as always alive)
        if (ps < 31) w3 |= 1u << ps;
      }
    }
    w[1] = w1;
    w[3] = w3;
  }
  t->n_slots = next;
  // pass 3 (backward): fewest / most nodes on a path to a sink; every out-edge
  // leads to a higher rank, so a row is final when the scan reaches it and
  // pushes its values to its in-edge rows
  dmin.assign(V, 0xFFFFFFFFu);
  dmax.assign(V, 0);
  uint32_t* __restrict__ lo = dmin.data();
  uint32_t* __restrict__ hi = dmax.data();
  for (uint32_t r = V; r-- > 0;) {
    if (lo[r] == 0xFFFFFFFFu) lo[r] = 0;  // a sink
    const uint32_t l1 = lo[r] + 1, h1 = hi[r] + 1;
    for (uint32_t x = pstart[r]; x < pstart[r + 1]; ++x) {
      const uint32_t p = pred_row[x] - 1;
      lo[p] = std::min(lo[p], l1);
      hi[p] = std::max(hi[p], h1);
    }
    rec[static_cast<size_t>(r) * kRecWords + 2] = std::min(lo[r], 0xFFFFu) | (std::min(hi[r], 0xFFFFu) << 16);
  }
}

void PoaGraph::export_strip_lite(RowTables* t, const StripLiteDst* dst) const {
  const uint32_t V = num_nodes();
  t->n_rows = V;
  t->n_edges = static_cast<uint32_t>(e_tail_.size());
  t->lite = true;
  static thread_local std::vector<uint32_t> lds_last;
  lds_last.assign(V, 0);
  uint32_t* __restrict__ pstart = dst->pstart;
  uint32_t* __restrict__ pred_row = dst->pred_row;
  uint32_t* __restrict__ info = dst->info;
  uint32_t* __restrict__ last = lds_last.data();
  const uint32_t* __restrict__ n2r = node_to_rank_.data();
  const uint32_t* __restrict__ etail = e_tail_.data();
  // pass 1 of export_strip_rows: in-edge rows, per row its last pool reader
  uint32_t k = 0, max_preds = 0;
  for (uint32_t r = 0; r < V; ++r) {
    const uint32_t node = rank_to_node_[r];
    const NodeList& in = in_[node];
    pstart[r] = k;
    max_preds = std::max(max_preds, in.size());
    for (uint32_t e : in) {
      const uint32_t pr = n2r[etail[e]];
      pred_row[k++] = pr + 1;
      if (pr + 1 != r && last[pr] < r + 1) last[pr] = r + 1;
    }
    info[r] = static_cast<uint8_t>(base_[node]) | (out_[node].empty() ? 0x100u : 0u) |
              (std::min<uint32_t>(static_cast<uint32_t>(in.size()), 63u) << 10);
  }
  pstart[V] = k;
  t->max_preds = max_preds;
  // the planner's free-list size, replayed: store bits, last-read flags and
  // the slot count of export_strip_rows' pass 2
  const char* wide_env = std::getenv("SVS_POA_TEST_WIDE_SLOTS");
  const uint32_t wide_rows = wide_env ? static_cast<uint32_t>(std::strtoul(wide_env, nullptr, 10)) : 0u;
  uint32_t next = (wide_rows != 0 && V >= wide_rows) ? 40 : 1, nfree = 0;
  t->slot_base = next;
  for (uint32_t r = 0; r < V; ++r) {
    if (last[r] != 0) {
      info[r] |= 0x200u;
      if (nfree) --nfree;
      else ++next;
    }
    for (uint32_t x = pstart[r]; x < pstart[r + 1]; ++x) {
      const uint32_t pr = pred_row[x] - 1;
      if (pr + 1 != r && last[pr] == r + 1) {
        pred_row[x] |= 0x80000000u;
        ++nfree;
      }
    }
  }
  t->n_slots = next;
}

void fill_col0(RowTables* t, int32_t g, int32_t e, int32_t q, int32_t c) {
  const size_t V = t->pstart.empty() ? 0 : t->pstart.size() - 1;
  t->col0.resize(3 * V);
  for (size_t r = 0; r < V; ++r) {
    int32_t F0, O0;
    if (t->pstart[r] == t->pstart[r + 1]) {
      F0 = g;
      O0 = q;
    } else {
      F0 = INT32_MIN + 1024;
      O0 = INT32_MIN + 1024;
      for (uint32_t k = t->pstart[r]; k < t->pstart[r + 1]; ++k) {
        const size_t p = t->pred_row[k] - 1;
        F0 = std::max(F0, t->col0[3 * p + 1]);
        O0 = std::max(O0, t->col0[3 * p + 2]);
      }
      F0 += e;
      O0 += c;
    }
    t->col0[3 * r] = std::max(F0, O0);
    t->col0[3 * r + 1] = F0;
    t->col0[3 * r + 2] = O0;
  }
}

std::vector<std::string> PoaGraph::msa() const {
  std::vector<uint32_t> col(num_nodes(), 0);
  uint32_t ncol = 0;
  for (size_t r = 0; r < rank_to_node_.size(); ++r) {
    const uint32_t node = rank_to_node_[r];
    col[node] = ncol;
    for (size_t k = 0; k < aligned_[node].size(); ++k) col[rank_to_node_[++r]] = ncol;
    ++ncol;
  }
  std::vector<std::string> rows;
  rows.reserve(paths_.size());
  for (const auto& p : paths_) {
    std::string row(ncol, '-');
    for (uint32_t node : p) row[col[node]] = base_[node];
    rows.push_back(std::move(row));
  }
  return rows;
}

uint32_t PoaGraph::branch_complete(uint32_t rank, std::vector<int64_t>& score, std::vector<int64_t>& pred) {
  const uint32_t start = rank_to_node_[rank];
  for (uint32_t e : out_[start])
    for (uint32_t f : in_[e_head_[e]])
      if (e_tail_[f] != start) score[e_tail_[f]] = -1;
  int64_t best = -1;
  for (uint32_t r = rank + 1; r < rank_to_node_.size(); ++r) {
    const uint32_t n = rank_to_node_[r];
    score[n] = -1;
    pred[n] = -1;
    for (uint32_t e : in_[n]) {
      const uint32_t t = e_tail_[e];
      if (score[t] == -1) continue;
      if (score[n] < e_w_[e] || (score[n] == e_w_[e] && score[pred[n]] <= score[t])) {
        score[n] = e_w_[e];
        pred[n] = t;
      }
    }
    if (pred[n] != -1) score[n] += score[pred[n]];
    if (best == -1 || score[best] < score[n]) best = n;
  }
  return static_cast<uint32_t>(best);
}

std::string PoaGraph::consensus(int32_t min_coverage) {
  std::string out;
  if (rank_to_node_.empty()) return out;
  const uint32_t n = num_nodes();
  std::vector<int64_t> score(n, -1), pred(n, -1);
  int64_t best = -1;
  for (uint32_t node : rank_to_node_) {
    for (uint32_t e : in_[node]) {
      const uint32_t t = e_tail_[e];
      if (score[node] < e_w_[e] || (score[node] == e_w_[e] && score[pred[node]] <= score[t])) {
        score[node] = e_w_[e];
        pred[node] = t;
      }
    }
    if (pred[node] != -1) score[node] += score[pred[node]];
    if (best == -1 || score[best] < score[node]) best = node;
  }
  while (!out_[static_cast<uint32_t>(best)].empty())
    best = branch_complete(node_to_rank_[static_cast<uint32_t>(best)], score, pred);
  std::vector<uint32_t> path;
  for (int64_t x = best; x != -1; x = pred[x]) path.push_back(static_cast<uint32_t>(x));
  for (auto it = path.rbegin(); it != path.rend(); ++it)
    if (min_coverage <= 0 || static_cast<int32_t>(cov_[*it]) >= min_coverage) out += base_[*it];
  return out;
}

}  // namespace svs
