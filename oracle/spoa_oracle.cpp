// ============================================================================
// ORACLE — TEST INFRASTRUCTURE ONLY.  Never linked into, called by, or shipped
// with the svscope_amd product path.  Only tests/, __graft_entry__.smoke() and
// bench.py's cpu_baseline leg may load this library, and only as the checker.
//
// What it is: a plain CPU restatement of the partial-order-alignment semantics
// the reference reaches through `from spoa import poa` (pyspoa 0.2.1 -> spoa
// 4.x, README.md:19).  The reference calls it as `poa(list_of_str, 1)` at
//   /root/reference/src/DataScanner.py:206,213   (window MSA)
//   /root/reference/src/DecisionMaker.py:160,171 (per-cluster consensus)
// pyspoa/spoa are NOT vendored in /root/reference and are not installed in
// this image, so this file restates spoa's published algorithm (SISD engine,
// AlignmentType kNW=1, convex gap subtype chosen by spoa for the pyspoa
// defaults m=5 n=-4 g=-8 e=-6 q=-10 c=-4):
//   * Needleman-Wunsch of each sequence against the growing graph, rows in
//     topological rank order, 5 DP planes H/E/F/O/Q (E,Q horizontal; F,O
//     vertical; gap(l) = max(g+(l-1)e, q+(l-1)c));
//   * spoa's backtrack check order (diagonal over in-edges in insertion order,
//     then vertical F/H+g/O/H+q, then horizontal E/H+g/Q/H+q, gap-run walks);
//   * Graph::AddAlignment with aligned-node merging, edge labels/weights;
//   * Graph::TopologicalSort (DFS with aligned-node grouping);
//   * GenerateMultipleSequenceAlignment (empty sequences produce no row);
//   * heaviest-bundle consensus with branch completion.
// PARITY STATUS: the restatement is pinned against the fixtures under
// tests/golden/ (hand-checked small cases); it could not be pinned against
// pyspoa itself (absent, no network) => "parity unpinned" vs pyspoa, see
// DESIGN.md §Oracle.
//
// Structure is intentionally the textbook pointer graph (Node/Edge objects,
// full int32 matrices) — the product engine (svscope_amd/csrc) is a separate
// flat-array + HIP implementation, so agreement between the two is evidence.
// ============================================================================
#include <algorithm>
#include <climits>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <stack>
#include <stdexcept>
#include <string>
#include <unordered_set>
#include <utility>
#include <vector>

namespace oracle {

constexpr int32_t kNegInf = INT32_MIN + 1024;  // spoa's kNegativeInfinity

struct Node;
struct Edge {
  Node* tail;
  Node* head;
  std::vector<uint32_t> labels;
  int64_t weight;
};
struct Node {
  uint32_t id;
  char base;
  std::vector<Edge*> inedges;
  std::vector<Edge*> outedges;
  std::vector<Node*> aligned;
  Node* successor(uint32_t label) const {
    for (Edge* e : outedges)
      for (uint32_t l : e->labels)
        if (l == label) return e->head;
    return nullptr;
  }
  uint32_t coverage() const {
    std::unordered_set<uint32_t> s;
    for (Edge* e : inedges) s.insert(e->labels.begin(), e->labels.end());
    for (Edge* e : outedges) s.insert(e->labels.begin(), e->labels.end());
    return static_cast<uint32_t>(s.size());
  }
};

using Alignment = std::vector<std::pair<int32_t, int32_t>>;  // (node id | -1, seq pos | -1)

class Graph {
 public:
  std::vector<std::unique_ptr<Node>> nodes;
  std::vector<std::unique_ptr<Edge>> edges;
  std::vector<Node*> rank_to_node;
  std::vector<Node*> sequences;  // begin node of every non-empty sequence
  std::vector<Node*> consensus;

  Node* add_node(char b) {
    nodes.emplace_back(new Node());
    nodes.back()->id = static_cast<uint32_t>(nodes.size() - 1);
    nodes.back()->base = b;
    return nodes.back().get();
  }
  void add_edge(Node* tail, Node* head, int64_t w) {
    for (Edge* e : tail->outedges) {
      if (e->head == head) {
        e->labels.push_back(static_cast<uint32_t>(sequences.size()));
        e->weight += w;
        return;
      }
    }
    edges.emplace_back(new Edge{tail, head, {static_cast<uint32_t>(sequences.size())}, w});
    tail->outedges.push_back(edges.back().get());
    head->inedges.push_back(edges.back().get());
  }
  // AddSequence(sequence, weights, begin, end): a fresh chain, weight w_i + w_{i+1}
  Node* add_chain(const std::string& s, uint32_t b, uint32_t e) {
    if (b == e) return nullptr;
    Node* first = add_node(s[b]);
    Node* prev = first;
    for (uint32_t i = b + 1; i < e; ++i) {
      Node* cur = add_node(s[i]);
      add_edge(prev, cur, 2);
      prev = cur;
    }
    return first;
  }

  void add_alignment(const Alignment& aln, const std::string& s) {
    if (s.empty()) return;
    if (aln.empty()) {
      sequences.push_back(add_chain(s, 0, static_cast<uint32_t>(s.size())));
      topological_sort();
      return;
    }
    std::vector<uint32_t> valid;
    for (auto& p : aln)
      if (p.second != -1) valid.push_back(static_cast<uint32_t>(p.second));
    if (valid.empty()) throw std::runtime_error("alignment consumes no sequence");
    Node* begin = add_chain(s, 0, valid.front());
    Node* prev = begin ? nodes.back().get() : nullptr;
    Node* last = add_chain(s, valid.back() + 1, static_cast<uint32_t>(s.size()));
    for (auto& p : aln) {
      if (p.second == -1) continue;
      char letter = s[p.second];
      Node* cur = nullptr;
      if (p.first == -1) {
        cur = add_node(letter);
      } else {
        Node* n = nodes[p.first].get();
        if (n->base == letter) {
          cur = n;
        } else {
          for (Node* a : n->aligned)
            if (a->base == letter) { cur = a; break; }
          if (!cur) {
            cur = add_node(letter);
            for (Node* a : n->aligned) {
              a->aligned.push_back(cur);
              cur->aligned.push_back(a);
            }
            n->aligned.push_back(cur);
            cur->aligned.push_back(n);
          }
        }
      }
      if (!begin) begin = cur;
      if (prev) add_edge(prev, cur, 2);
      prev = cur;
    }
    if (last) add_edge(prev, last, 2);
    sequences.push_back(begin);
    topological_sort();
  }

  void topological_sort() {
    rank_to_node.clear();
    std::vector<uint8_t> mark(nodes.size(), 0);
    std::vector<uint8_t> ignored(nodes.size(), 0);
    std::stack<Node*> st;
    for (auto& up : nodes) {
      if (mark[up->id] != 0) continue;
      st.push(up.get());
      while (!st.empty()) {
        Node* cur = st.top();
        bool ok = true;
        if (mark[cur->id] != 2) {
          for (Edge* e : cur->inedges)
            if (mark[e->tail->id] != 2) { st.push(e->tail); ok = false; }
          if (!ignored[cur->id]) {
            for (Node* a : cur->aligned)
              if (mark[a->id] != 2) { st.push(a); ignored[a->id] = 1; ok = false; }
          }
          if (ok) {
            mark[cur->id] = 2;
            if (!ignored[cur->id]) {
              rank_to_node.push_back(cur);
              for (Node* a : cur->aligned) rank_to_node.push_back(a);
            }
          } else {
            mark[cur->id] = 1;
          }
        }
        if (ok) st.pop();
      }
    }
  }

  std::vector<std::string> msa() const {
    std::vector<uint32_t> col(nodes.size(), 0);
    uint32_t c = 0;
    for (size_t i = 0; i < rank_to_node.size(); ++i) {
      Node* n = rank_to_node[i];
      col[n->id] = c;
      for (size_t k = 0; k < n->aligned.size(); ++k) col[rank_to_node[++i]->id] = c;
      ++c;
    }
    std::vector<std::string> out;
    for (uint32_t s = 0; s < sequences.size(); ++s) {
      std::string row(c, '-');
      for (Node* n = sequences[s]; n; n = n->successor(s)) row[col[n->id]] = n->base;
      out.push_back(row);
    }
    return out;
  }

  Node* branch_completion(uint32_t rank, std::vector<int64_t>& score, std::vector<Node*>& pred) {
    Node* start = rank_to_node[rank];
    for (Edge* e : start->outedges)
      for (Edge* f : e->head->inedges)
        if (f->tail != start) score[f->tail->id] = -1;
    Node* best = nullptr;
    for (size_t r = rank + 1; r < rank_to_node.size(); ++r) {
      Node* n = rank_to_node[r];
      score[n->id] = -1;
      pred[n->id] = nullptr;
      for (Edge* e : n->inedges) {
        if (score[e->tail->id] == -1) continue;
        if (score[n->id] < e->weight ||
            (score[n->id] == e->weight && score[pred[n->id]->id] <= score[e->tail->id])) {
          score[n->id] = e->weight;
          pred[n->id] = e->tail;
        }
      }
      if (pred[n->id]) score[n->id] += score[pred[n->id]->id];
      if (!best || score[best->id] < score[n->id]) best = n;
    }
    return best;
  }

  void heaviest_bundle() {
    consensus.clear();
    if (rank_to_node.empty()) return;
    std::vector<Node*> pred(nodes.size(), nullptr);
    std::vector<int64_t> score(nodes.size(), -1);
    Node* best = nullptr;
    for (Node* n : rank_to_node) {
      for (Edge* e : n->inedges) {
        if (score[n->id] < e->weight ||
            (score[n->id] == e->weight && score[pred[n->id]->id] <= score[e->tail->id])) {
          score[n->id] = e->weight;
          pred[n->id] = e->tail;
        }
      }
      if (pred[n->id]) score[n->id] += score[pred[n->id]->id];
      if (!best || score[best->id] < score[n->id]) best = n;
    }
    if (!best->outedges.empty()) {
      std::vector<uint32_t> rank(nodes.size(), 0);
      for (uint32_t i = 0; i < rank_to_node.size(); ++i) rank[rank_to_node[i]->id] = i;
      while (!best->outedges.empty()) best = branch_completion(rank[best->id], score, pred);
    }
    while (pred[best->id]) {
      consensus.push_back(best);
      best = pred[best->id];
    }
    consensus.push_back(best);
    std::reverse(consensus.begin(), consensus.end());
  }

  std::string consensus_string(int32_t min_coverage) {
    heaviest_bundle();
    std::string s;
    for (Node* n : consensus)
      if (min_coverage <= 0 || static_cast<int32_t>(n->coverage()) >= min_coverage) s += n->base;
    return s;
  }
};

struct Params { int32_t m, n, g, e, q, c; };

struct Stats {
  uint64_t cells = 0;      // sum over alignments of (|V|+1)*(L+1)
  uint32_t max_nodes = 0;  // largest graph aligned against
};

// spoa SisdAlignmentEngine::Initialize + Convex, AlignmentType::kNW.
Alignment align_nw_convex(const std::string& seq, const Graph& g, const Params& P, Stats* st) {
  if (g.nodes.empty() || seq.empty()) return {};
  const uint64_t W = seq.size() + 1;
  const uint64_t Hh = g.nodes.size() + 1;
  if (st) {
    st->cells += W * Hh;
    st->max_nodes = std::max<uint32_t>(st->max_nodes, static_cast<uint32_t>(g.nodes.size()));
  }
  std::vector<int32_t> H(W * Hh), E(W * Hh), F(W * Hh), O(W * Hh), Q(W * Hh);
  std::vector<uint32_t> rank(g.nodes.size());
  for (uint32_t i = 0; i < g.rank_to_node.size(); ++i) rank[g.rank_to_node[i]->id] = i;
  auto prof = [&](const Node* n, uint64_t j) -> int32_t { return n->base == seq[j - 1] ? P.m : P.n; };
  // ---- Initialize (convex, falls through affine) ----
  O[0] = 0; Q[0] = 0;
  for (uint64_t j = 1; j < W; ++j) { O[j] = kNegInf; Q[j] = P.q + static_cast<int32_t>(j - 1) * P.c; }
  for (uint64_t i = 1; i < Hh; ++i) {
    const Node* n = g.rank_to_node[i - 1];
    int32_t pen = n->inedges.empty() ? P.q - P.c : kNegInf;
    for (Edge* e : n->inedges) pen = std::max(pen, O[(rank[e->tail->id] + 1) * W]);
    O[i * W] = pen + P.c;
    Q[i * W] = kNegInf;
  }
  F[0] = 0; E[0] = 0;
  for (uint64_t j = 1; j < W; ++j) { F[j] = kNegInf; E[j] = P.g + static_cast<int32_t>(j - 1) * P.e; }
  for (uint64_t i = 1; i < Hh; ++i) {
    const Node* n = g.rank_to_node[i - 1];
    int32_t pen = n->inedges.empty() ? P.g - P.e : kNegInf;
    for (Edge* e : n->inedges) pen = std::max(pen, F[(rank[e->tail->id] + 1) * W]);
    F[i * W] = pen + P.e;
    E[i * W] = kNegInf;
  }
  H[0] = 0;
  for (uint64_t j = 1; j < W; ++j) H[j] = std::max(Q[j], E[j]);
  for (uint64_t i = 1; i < Hh; ++i) H[i * W] = std::max(O[i * W], F[i * W]);

  // ---- fill ----
  int32_t max_score = kNegInf;
  uint64_t max_i = 0, max_j = 0;
  for (const Node* n : g.rank_to_node) {
    const uint64_t i = rank[n->id] + 1;
    int32_t* Hr = &H[i * W]; int32_t* Fr = &F[i * W]; int32_t* Or = &O[i * W];
    uint64_t pi = n->inedges.empty() ? 0 : rank[n->inedges[0]->tail->id] + 1;
    const int32_t* Hp = &H[pi * W]; const int32_t* Fp = &F[pi * W]; const int32_t* Op = &O[pi * W];
    for (uint64_t j = 1; j < W; ++j) {
      Fr[j] = std::max(Hp[j] + P.g, Fp[j] + P.e);
      Or[j] = std::max(Hp[j] + P.q, Op[j] + P.c);
      Hr[j] = Hp[j - 1] + prof(n, j);
    }
    for (size_t p = 1; p < n->inedges.size(); ++p) {
      pi = rank[n->inedges[p]->tail->id] + 1;
      Hp = &H[pi * W]; Fp = &F[pi * W]; Op = &O[pi * W];
      for (uint64_t j = 1; j < W; ++j) {
        Fr[j] = std::max(Fr[j], std::max(Hp[j] + P.g, Fp[j] + P.e));
        Or[j] = std::max(Or[j], std::max(Hp[j] + P.q, Op[j] + P.c));
        Hr[j] = std::max(Hr[j], Hp[j - 1] + prof(n, j));
      }
    }
    int32_t* Er = &E[i * W]; int32_t* Qr = &Q[i * W];
    for (uint64_t j = 1; j < W; ++j) {
      Er[j] = std::max(Hr[j - 1] + P.g, Er[j - 1] + P.e);
      Qr[j] = std::max(Hr[j - 1] + P.q, Qr[j - 1] + P.c);
      Hr[j] = std::max(Hr[j], std::max(Fr[j], Or[j]));
      Hr[j] = std::max(Hr[j], std::max(Er[j], Qr[j]));
    }
    if (n->outedges.empty() && max_score < Hr[W - 1]) {
      max_score = Hr[W - 1]; max_i = i; max_j = W - 1;
    }
  }
  if (max_i == 0 && max_j == 0) return {};

  // ---- backtrack ----
  Alignment aln;
  uint64_t i = max_i, j = max_j, prev_i = 0, prev_j = 0;
  auto at = [&](const std::vector<int32_t>& M, uint64_t r, uint64_t col) { return M[r * W + col]; };
  while (!(i == 0 && j == 0)) {
    const int32_t Hij = at(H, i, j);
    bool found = false, ext_left = false, ext_up = false;
    if (i != 0 && j != 0) {
      const Node* n = g.rank_to_node[i - 1];
      const int32_t mc = prof(n, j);
      uint64_t pi = n->inedges.empty() ? 0 : rank[n->inedges[0]->tail->id] + 1;
      if (Hij == at(H, pi, j - 1) + mc) {
        prev_i = pi; prev_j = j - 1; found = true;
      } else {
        for (size_t p = 1; p < n->inedges.size(); ++p) {
          pi = rank[n->inedges[p]->tail->id] + 1;
          if (Hij == at(H, pi, j - 1) + mc) { prev_i = pi; prev_j = j - 1; found = true; break; }
        }
      }
    }
    if (!found && i != 0) {
      const Node* n = g.rank_to_node[i - 1];
      uint64_t pi = n->inedges.empty() ? 0 : rank[n->inedges[0]->tail->id] + 1;
      auto up_ok = [&](uint64_t r) {
        return (ext_up = Hij == at(F, r, j) + P.e) || Hij == at(H, r, j) + P.g ||
               (ext_up = Hij == at(O, r, j) + P.c) || Hij == at(H, r, j) + P.q;
      };
      if (up_ok(pi)) {
        prev_i = pi; prev_j = j; found = true;
      } else {
        for (size_t p = 1; p < n->inedges.size(); ++p) {
          pi = rank[n->inedges[p]->tail->id] + 1;
          if (up_ok(pi)) { prev_i = pi; prev_j = j; found = true; break; }
        }
      }
    }
    if (!found && j != 0) {
      if ((ext_left = Hij == at(E, i, j - 1) + P.e) || Hij == at(H, i, j - 1) + P.g ||
          (ext_left = Hij == at(Q, i, j - 1) + P.c) || Hij == at(H, i, j - 1) + P.q) {
        prev_i = i; prev_j = j - 1; found = true;
      }
    }
    if (!found) throw std::runtime_error("oracle backtrack: no predecessor");
    aln.emplace_back(i == prev_i ? -1 : static_cast<int32_t>(g.rank_to_node[i - 1]->id),
                     j == prev_j ? -1 : static_cast<int32_t>(j - 1));
    i = prev_i; j = prev_j;
    if (ext_left) {
      while (true) {
        aln.emplace_back(-1, static_cast<int32_t>(j - 1));
        --j;
        if (at(H, i, j) + P.g == at(E, i, j + 1) || at(H, i, j) + P.q == at(Q, i, j + 1)) break;
      }
    } else if (ext_up) {
      while (true) {
        bool stop = false;
        prev_i = 0;
        for (Edge* e : g.rank_to_node[i - 1]->inedges) {
          const uint64_t pi = rank[e->tail->id] + 1;
          if ((stop = at(F, i, j) == at(H, pi, j) + P.g) || at(F, i, j) == at(F, pi, j) + P.e ||
              (stop = at(O, i, j) == at(H, pi, j) + P.q) || at(O, i, j) == at(O, pi, j) + P.c) {
            prev_i = pi;
            break;
          }
        }
        aln.emplace_back(static_cast<int32_t>(g.rank_to_node[i - 1]->id), -1);
        i = prev_i;
        if (stop || i == 0) break;
      }
    }
  }
  std::reverse(aln.begin(), aln.end());
  return aln;
}

}  // namespace oracle

// ----------------------------------------------------------------------------
// C ABI for ctypes (tests / cpu_baseline only).
// ----------------------------------------------------------------------------
struct OracleResult {
  std::string consensus;
  std::vector<std::string> msa;
  std::vector<uint32_t> rank_ids;  // final topological order (node ids)
  oracle::Stats stats;
  std::string error;
};

extern "C" {

// Runs pyspoa-equivalent poa(seqs, algorithm=1) on n sequences.
// Returns an opaque handle (never NULL); check oracle_error().
void* oracle_poa(int n, const char* const* seqs, const int* lens, int algorithm,
                 int m, int mis, int g, int e, int q, int c, int min_coverage) {
  auto* r = new OracleResult();
  try {
    if (algorithm != 1) throw std::runtime_error("oracle supports AlignmentType kNW (1) only");
    if (!(g < e && !(g <= q || e >= c))) throw std::runtime_error("oracle supports the convex gap subtype only");
    oracle::Params P{m, mis, g, e, q, c};
    oracle::Graph graph;
    for (int s = 0; s < n; ++s) {
      std::string seq(seqs[s], static_cast<size_t>(lens[s]));
      auto aln = oracle::align_nw_convex(seq, graph, P, &r->stats);
      graph.add_alignment(aln, seq);
    }
    r->consensus = graph.consensus_string(min_coverage);
    r->msa = graph.msa();
    for (auto* nd : graph.rank_to_node) r->rank_ids.push_back(nd->id);
  } catch (const std::exception& ex) {
    r->error = ex.what();
  }
  return r;
}

const char* oracle_error(void* h) {
  auto* r = static_cast<OracleResult*>(h);
  return r->error.empty() ? nullptr : r->error.c_str();
}
int oracle_consensus_len(void* h) { return static_cast<int>(static_cast<OracleResult*>(h)->consensus.size()); }
const char* oracle_consensus(void* h) { return static_cast<OracleResult*>(h)->consensus.c_str(); }
int oracle_msa_rows(void* h) { return static_cast<int>(static_cast<OracleResult*>(h)->msa.size()); }
int oracle_msa_cols(void* h) {
  auto* r = static_cast<OracleResult*>(h);
  return r->msa.empty() ? 0 : static_cast<int>(r->msa[0].size());
}
const char* oracle_msa_row(void* h, int i) { return static_cast<OracleResult*>(h)->msa[i].c_str(); }
unsigned long long oracle_cells(void* h) { return static_cast<OracleResult*>(h)->stats.cells; }
int oracle_max_nodes(void* h) { return static_cast<int>(static_cast<OracleResult*>(h)->stats.max_nodes); }
void oracle_free(void* h) { delete static_cast<OracleResult*>(h); }

}  // extern "C"
