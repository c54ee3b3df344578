// ORACLE — test infrastructure only (tests/, __graft_entry__.smoke(), the
// cpu_baseline leg of probes).  Never linked into libsvscope_hip.
//
// C++ twin of oracle/pairwise2_oracle.py: the reference's AligmentScore
// (/root/reference/src/PairwiseCompare.py:19-30) =
//   Bio.pairwise2.align.globalms(som, ger, match, mismatch, open, extend)[0]
//   -> format_alignment(...).split('\n')[1][cutoff:len-cutoff]
//   -> (length, count('|')).
// Biopython's pairwise2 (third party, not vendored, not installed here) is
// restated from the published module (1.72..1.81): _make_score_matrix_fast
// (score matrix, 5-bit trace: 1 row-open, 2 diagonal, 4 col-open, 8 row-extend,
// 16 col-extend), _recover_alignments (DFS over an explicit stack, lowest trace
// bit first, col_gap forbids a seqA gap right after a seqB gap),
// _find_gap_open (scans back to the border, pushing every cell where the gap
// could have opened), _finish_backtrace.  Global alignment, end gaps
// penalised, penalize_extend_when_opening = False.  Only the first recovered
// alignment is followed to completion (it is element [0] of pairwise2's list).
//
// The full int32 score matrix and byte trace matrix are kept, like pairwise2,
// on purpose: the product's kernel stores 4-bit score differences instead.
#include <cstdint>
#include <cstring>
#include <vector>

namespace {

int affine(int length, int open, int extend) {
  if (length <= 0) return 0;
  return open + extend * length - extend;  // penalize_extend_when_opening False
}

// A DFS state; like pairwise2's (ali_seqA, ali_seqB, ...) tuples it owns a
// copy of the match-line flags traced so far (in traceback order).
struct State {
  int row, col;
  bool col_gap;
  int trace;
  std::vector<uint8_t> flag;  // 1 = '|'
};

struct Aligner {
  const char* A;
  const char* B;
  int la, lb;
  int match, mismatch, open, extend;
  std::vector<int32_t> S;
  std::vector<uint8_t> T;
  long long steps = 0;

  int& s(int r, int c) { return S[(size_t)r * (lb + 1) + c]; }
  uint8_t& t(int r, int c) { return T[(size_t)r * (lb + 1) + c]; }

  void fill() {
    S.assign((size_t)(la + 1) * (lb + 1), 0);
    T.assign((size_t)(la + 1) * (lb + 1), 0);  // border traces: None (falsy)
    const int first_gap = affine(1, open, extend);
    for (int i = 0; i <= la; ++i) s(i, 0) = affine(i, open, extend);
    for (int j = 0; j <= lb; ++j) s(0, j) = affine(j, open, extend);
    std::vector<int> col_score(lb + 1, 0);
    for (int j = 1; j <= lb; ++j) col_score[j] = affine(j, 2 * open, extend);
    for (int r = 1; r <= la; ++r) {
      int row_score = affine(r, 2 * open, extend);
      for (int c = 1; c <= lb; ++c) {
        const int nogap = s(r - 1, c - 1) + (A[r - 1] == B[c - 1] ? match : mismatch);
        const int row_open = s(r, c - 1) + first_gap;
        const int row_extend = row_score + extend;
        row_score = row_open > row_extend ? row_open : row_extend;
        const int col_open = s(r - 1, c) + first_gap;
        const int col_extend = col_score[c] + extend;
        col_score[c] = col_open > col_extend ? col_open : col_extend;
        int best = nogap;
        if (col_score[c] > best) best = col_score[c];
        if (row_score > best) best = row_score;
        s(r, c) = best;
        int rt = (row_open == row_score ? 1 : 0) + (row_extend == row_score ? 8 : 0);
        int ct = (col_open == col_score[c] ? 4 : 0) + (col_extend == col_score[c] ? 16 : 0);
        int tr = 0;
        if (nogap == best) tr += 2;
        if (row_score == best) tr += rt;
        if (col_score[c] == best) tr += ct;
        t(r, c) = (uint8_t)tr;
      }
    }
  }

  // returns false when no alignment was recovered
  bool first_alignment(std::vector<uint8_t>* out) {
    std::vector<State> stack;
    stack.push_back({la, lb, false, t(la, lb), {}});
    while (!stack.empty()) {
      State st = stack.back();
      stack.pop_back();
      int row = st.row, col = st.col, trace = st.trace;
      std::vector<uint8_t> flag = std::move(st.flag);
      bool col_gap = st.col_gap, dead = false;
      while ((row > 0 || col > 0) && !dead) {
        ++steps;
        State cache{row, col, col_gap, 0, flag};
        if (!trace) {
          if (col && col_gap) {
            dead = true;
          } else {  // _finish_backtrace: the rest against gaps
            // a '-' in a sequence against a gap still prints '|' (a == b)
            for (int k = row - 1; k >= 0; --k) flag.push_back(A[k] == '-');
            for (int k = col - 1; k >= 0; --k) flag.push_back(B[k] == '-');
          }
          break;
        } else if (trace % 2 == 1) {
          trace -= 1;
          if (col_gap) {
            dead = true;
          } else {
            col -= 1;
            flag.push_back(B[col] == '-');
            col_gap = false;
          }
        } else if (trace % 4 == 2) {
          trace -= 2;
          row -= 1;
          col -= 1;
          flag.push_back(A[row] == B[col]);
          col_gap = false;
        } else if (trace % 8 == 4) {
          trace -= 4;
          row -= 1;
          flag.push_back(A[row] == '-');
          col_gap = true;
        } else if (trace == 8 || trace == 24) {
          trace -= 8;
          if (col_gap) {
            dead = true;
          } else {
            col_gap = false;
            dead = gap_open(row, col, flag, col_gap, stack, /*horizontal=*/true);
          }
        } else if (trace == 16) {
          trace -= 16;
          col_gap = true;
          dead = gap_open(row, col, flag, col_gap, stack, /*horizontal=*/false);
        }
        if (trace) {
          cache.trace = trace;
          stack.push_back(std::move(cache));
        }
        trace = t(row, col);
      }
      if (!dead) {
        *out = std::move(flag);
        return true;
      }
    }
    return false;
  }

  // _find_gap_open: walks back along the row (horizontal) or column to the
  // border; pushes every cell (n > 0) where opening the gap gives the score.
  bool gap_open(int& row, int& col, std::vector<uint8_t>& flag, bool col_gap, std::vector<State>& stack,
                bool horizontal) {
    bool dead = false;
    const int target_score = s(row, col);
    const int target = horizontal ? col : row;
    for (int n = 0; n < target; ++n) {
      if (horizontal) {
        col -= 1;
        flag.push_back(B[col] == '-');
      } else {
        row -= 1;
        flag.push_back(A[row] == '-');
      }
      const int actual = s(row, col) + affine(n + 1, open, extend);
      if (actual == target_score && n > 0) {
        if (!t(row, col)) break;
        stack.push_back({row, col, col_gap, t(row, col), flag});
      }
      if (!t(row, col)) dead = true;
    }
    return dead;
  }
};

}  // namespace

extern "C" {

// Returns 0 and writes len(TD_alig) and count('|') of the first alignment's
// trimmed match line; -1 when pairwise2 would return no alignment (an empty
// sequence: the reference then raises IndexError on [0]).
int oracle_aligment_counts(const char* a, int la, const char* b, int lb, int match, int mismatch, int open,
                           int extend, int cutoff, int* out_len, int* out_match, long long* out_steps) {
  if (la <= 0 || lb <= 0) return -1;
  Aligner al{a, b, la, lb, match, mismatch, open, extend, {}, {}, 0};
  al.fill();
  std::vector<uint8_t> flag;
  if (!al.first_alignment(&flag)) return -2;
  const int nc = (int)flag.size();
  // the flags are in traceback order (alignment reversed); trimming is symmetric
  const int lo = cutoff, hi = nc - cutoff;
  int len = hi > lo ? hi - lo : 0, m = 0;
  for (int k = lo; k < hi; ++k) m += flag[k];
  *out_len = len;
  *out_match = m;
  if (out_steps) *out_steps = al.steps;
  return 0;
}

}  // extern "C"
