// Flat-array partial-order graph used by the batched MI355X POA engine.
//
// Semantics follow spoa 4.x Graph (the library behind `poa(seqs, 1)` at
// /root/reference/src/DataScanner.py:206,213 and DecisionMaker.py:160,171):
// AddAlignment with aligned-node merging, DFS topological sort with aligned
// groups kept contiguous, MSA columns from rank groups, heaviest-bundle
// consensus.  The representation is built for batched device export: every
// node/edge lives in flat vectors, each sequence keeps its node path (used for
// the MSA instead of edge-label walks) and export_rows() writes the
// rank-ordered row tables the HIP DP kernel consumes.
#pragma once
#include <algorithm>
#include <cstdint>
#include <string>
#include <vector>

namespace svs {

// One DP row table for a single read-vs-graph alignment job (host side).
struct RowTables {
  std::vector<uint32_t> info;    // per rank row: bits 0-7 base, bit 8 sink
  std::vector<uint32_t> slot;    // per rank row: pool slot (>=1; slot 0 = virtual row 0)
  std::vector<uint32_t> pstart;  // n_rows + 1 CSR offsets into pred_row/pred_slot
  std::vector<uint32_t> pred_row;   // 1-based DP row of each in-edge tail (insertion order)
  std::vector<uint32_t> pred_slot;  // pool slot of that row
  std::vector<int32_t> col0;        // per rank row: H, F, O of DP column 0 (fill_col0)
  uint32_t n_slots = 1;
  uint32_t max_preds = 0;
  uint32_t n_rows = 0, n_edges = 0;  // set by export_strip_rows (also when it writes to a StripDst)
  uint32_t slot_base = 1;             // first pool slot the planner hands out (export_strip_lite)
  bool lite = false;                  // written by export_strip_lite (the device completes the tables)
  // Strip-kernel tables (export_strip_rows): kRecWords words per row
  //   w0: base | sink << 8 | store << 9 | np << 10 | own pool slot << 16
  //       (kNoSlot: not stored)
  //   w1: 16-bit pool slots of in-edges 0 and 1 (rows with at most
  //       kInlinePreds in-edges), kNoSlot = "the row just above" (kept in
  //       registers); rows with more in-edges read all slots from
  //       pred_slot[pstart[r] + k]
  //   w2: dmin | dmax << 16: fewest / most nodes on a path from the row's
  //       node (exclusive) to a sink (inclusive), clamped to 0xFFFF; they
  //       bound the score any alignment can still gain below the row (the
  //       kernel's exact pruning, poa_strip.hip)
  //   w3: bit p set for each slot p < 32 whose last reader is this row; the
  //       pruning kernel clears their liveness after it
  std::vector<uint32_t> rec;
};

// Adjacency list of one node: up to four entries inline, more on the heap.
// Nearly every node has one or two in/out edges and no aligned partner, so a
// graph of thousands of nodes costs a handful of allocations instead of one or
// two per list (those made folding and releasing graphs allocator-bound).
class NodeList {
 public:
  NodeList() = default;
  NodeList(const NodeList& o) { assign(o); }
  NodeList(NodeList&& o) noexcept { steal(o); }
  NodeList& operator=(const NodeList& o) {
    if (this != &o) { release(); assign(o); }
    return *this;
  }
  NodeList& operator=(NodeList&& o) noexcept {
    if (this != &o) { release(); steal(o); }
    return *this;
  }
  ~NodeList() { release(); }

  uint32_t size() const { return n_; }
  bool empty() const { return n_ == 0; }
  const uint32_t* begin() const { return data(); }
  const uint32_t* end() const { return data() + n_; }
  uint32_t operator[](size_t i) const { return data()[i]; }
  void push_back(uint32_t v) {
    if (n_ == cap_) grow();
    data()[n_++] = v;
  }

 private:
  static constexpr uint32_t kInline = 4;
  bool on_heap() const { return cap_ > kInline; }
  uint32_t* data() { return on_heap() ? u_.heap : u_.inl; }
  const uint32_t* data() const { return on_heap() ? u_.heap : u_.inl; }
  void grow() {
    const uint32_t cap = cap_ * 2;
    uint32_t* h = new uint32_t[cap];
    std::copy(data(), data() + n_, h);
    release_heap();
    u_.heap = h;
    cap_ = cap;
  }
  void release_heap() {
    if (on_heap()) delete[] u_.heap;
  }
  void release() {
    release_heap();
    n_ = 0;
    cap_ = kInline;
  }
  void assign(const NodeList& o) {
    n_ = 0;
    cap_ = kInline;
    if (o.n_ > kInline) {
      u_.heap = new uint32_t[o.cap_];
      cap_ = o.cap_;
    }
    std::copy(o.begin(), o.end(), data());
    n_ = o.n_;
  }
  void steal(NodeList& o) {
    n_ = o.n_;
    cap_ = o.cap_;
    if (o.on_heap()) u_.heap = o.u_.heap;
    else std::copy(o.u_.inl, o.u_.inl + o.n_, u_.inl);
    o.n_ = 0;
    o.cap_ = kInline;
  }
  uint32_t n_ = 0, cap_ = kInline;
  union {
    uint32_t inl[kInline];
    uint32_t* heap;
  } u_;
};

constexpr uint32_t kRecWords = 4;
constexpr uint32_t kInlinePreds = 2;
constexpr uint32_t kNoSlot = 0xFFFF;

// One strip job's tables as one contiguous block of the launch's staging
// buffer (byte offsets from the block start; the block starts at a multiple of
// 48 so that the 12-B column-0 triples and the 16-B records both index it):
// col0 (12 V), records (16 V), pstart (4 (V+1)), pred_row (4 E), pred_slot
// (4 E), then the read: one zero pad byte, the read, zeros up to ls + 64.
struct StripBlock {
  size_t col0, rec, pstart, pred_row, pred_slot, seq, bytes;
  size_t info;  // strip_block_lite only
};
inline StripBlock strip_block_layout(uint32_t V, uint32_t E, uint32_t ls) {
  StripBlock b{};
  size_t o = 0;
  b.col0 = o;
  o = (o + 12ull * V + 15) / 16 * 16;
  b.rec = o;
  o += 16ull * V;
  b.pstart = o;
  o += 4ull * (V + 1);
  b.pred_row = o;
  o += 4ull * E;
  b.pred_slot = o;
  o += 4ull * E;
  b.seq = o + 1;
  o += ls + 64;
  b.bytes = (o + 47) / 48 * 48;
  return b;
}

// The same block for a job whose row records, in-edge slots and column 0 the
// device derives (poa_prep.hip): pstart, pred_row (bit 31: this in-edge is its
// tail row's last pool read), per row base | sink << 8 | store << 9 |
// in-degree << 10, then the read.
inline StripBlock strip_block_lite(uint32_t V, uint32_t E, uint32_t ls) {
  StripBlock b{};
  size_t o = 0;
  b.pstart = o;
  o += 4ull * (V + 1);
  b.pred_row = o;
  o += 4ull * E;
  b.info = o;
  o += 4ull * V;
  b.seq = o + 1;
  o += ls + 64;
  b.bytes = (o + 47) / 48 * 48;
  return b;
}
// Device-side output region of such a job: column 0 (12 V), records (16 V),
// in-edge slots (4 E, rounded to 16 B), then the device planner's scratch
// (3 words per row, rows rounded to 4); starts at a multiple of 48.
inline StripBlock strip_prep_out_layout(uint32_t V, uint32_t E) {
  StripBlock b{};
  size_t o = 0;
  b.col0 = o;
  o = (o + 12ull * V + 15) / 16 * 16;
  b.rec = o;
  o += 16ull * V;
  b.pred_slot = o;
  o += 4ull * ((E + 3u) & ~3u);
  o += 12ull * ((V + 3u) & ~3u);
  b.bytes = (o + 47) / 48 * 48;
  return b;
}

// Destinations for export_strip_lite.
struct StripLiteDst {
  uint32_t* pstart;
  uint32_t* pred_row;
  uint32_t* info;
};

// Raw destinations for export_strip_rows (a StripBlock in pinned staging).
struct StripDst {
  uint32_t* rec;
  uint32_t* pstart;
  uint32_t* pred_row;
  uint32_t* pred_slot;
  int32_t* col0;
};

// Column 0 of the NW matrix depends only on the graph (gap runs down the
// in-edges, spoa Initialize): F0 = max_p F0[p] + e (g for sources), O0 likewise
// with q/c, H0 = max(F0, O0).  Computed once per job on the host.
void fill_col0(RowTables* t, int32_t g, int32_t e, int32_t q, int32_t c);

class PoaGraph {
 public:
  uint32_t num_nodes() const { return static_cast<uint32_t>(base_.size()); }
  uint32_t num_edges() const { return static_cast<uint32_t>(e_tail_.size()); }
  uint32_t num_sequences() const { return static_cast<uint32_t>(paths_.size()); }
  bool empty() const { return base_.empty(); }
  size_t in_degree(uint32_t v) const { return in_[v].size(); }
  size_t aligned_count(uint32_t v) const { return aligned_[v].size(); }

  // pairs are (rank-row index 0-based or -1, sequence position or -1), in
  // forward order.  Node identity is resolved through the CURRENT rank order.
  void add_alignment_ranks(const std::vector<int32_t>& rank_pairs, const std::string& seq);
  // pairs are (node id or -1, position or -1); empty => fresh chain.
  void add_alignment_nodes(const std::vector<std::pair<int32_t, int32_t>>& node_pairs,
                           const std::string& seq);

  void export_rows(RowTables* t) const;
  // Tables for the strip-major kernel: a row is stored in the pool only if a
  // successor other than the next row reads it; an in-edge from the row just
  // above is served from registers.  Fills rec, pstart, pred_row, pred_slot,
  // n_slots, max_preds (info/slot are left empty).
  void export_strip_rows(RowTables* t) const;
  // the same, also filling col0 as fill_col0(t, gaps[0..3] = g, e, q, c) does
  void export_strip_rows(RowTables* t, const int32_t* gaps) const;
  // the same, writing the tables to dst instead of t's vectors (which are left
  // untouched); t gets n_rows, n_edges, n_slots and max_preds
  void export_strip_rows(RowTables* t, const int32_t* gaps, const StripDst* dst) const;
  // Pass 1 of export_strip_rows only, for the device planner (poa_prep.hip):
  // CSR in-edge rows with the last-read flag, per row words, and t's n_rows,
  // n_edges, max_preds, slot_base and n_slots (the count the planner reaches).
  void export_strip_lite(RowTables* t, const StripLiteDst* dst) const;
  std::vector<std::string> msa() const;
  std::string consensus(int32_t min_coverage);

  const std::vector<uint32_t>& rank_to_node() const { return rank_to_node_; }
  // by rank: 1 where a DFS root's segment of the order starts (the device
  // sort's reuse plane, checked by SVS_POA_VERIFY_GRAPH)
  const std::vector<uint8_t>& segment_starts() const { return seg_start_; }

 private:
  uint32_t new_node(char b);
  void link(uint32_t tail, uint32_t head, int64_t w, uint32_t seq_id);
  uint32_t chain(const std::string& s, uint32_t b, uint32_t e, std::vector<uint32_t>* path);
  void sort_ranks();
  uint32_t branch_complete(uint32_t rank, std::vector<int64_t>& score, std::vector<int64_t>& pred);

  std::vector<char> base_;
  std::vector<NodeList> in_;    // edge ids into node, insertion order
  std::vector<NodeList> out_;   // edge ids out of node
  std::vector<NodeList> aligned_;
  std::vector<uint32_t> cov_, cov_last_;     // distinct sequences touching a node's edges
  std::vector<uint32_t> e_tail_, e_head_;
  std::vector<int64_t> e_w_;
  std::vector<std::vector<uint32_t>> paths_;
  std::vector<uint32_t> rank_to_node_, node_to_rank_;
  std::vector<uint8_t> seg_start_;
};

}  // namespace svs
