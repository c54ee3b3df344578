// MisScore traceback: the first alignment Biopython's pairwise2 recovers for
// globalms(som, ger, 1, 0, -1, -1), replayed from 4-bit score differences.
//
// Reference: /root/reference/src/PairwiseCompare.py:19-30 (AligmentScore), on
// top of Bio.pairwise2 (third party; restated in oracle/pairwise2_oracle.py,
// whose header cites the functions it follows).
//
// Why 4 bits per cell are enough.  With match 1, mismatch 0 and linear gaps
// (open = extend = -1, penalize_extend_when_opening False) pairwise2's
// on-the-fly row score is E[r][c] = H[r][c-1] - 1 and its col score is
// F[r][c] = H[r-1][c] - 1 exactly (an extension E[r][c-1] - 1 never beats the
// opening, because E <= H).  Let dh = H[r][c] - H[r][c-1] and
// dv = H[r][c] - H[r-1][c]; both lie in [-1, 2].  The five trace bits of
// _make_score_matrix_fast follow from them:
//   2  (diagonal)   H[r-1][c-1] + s == H[r][c]  <=>  dh(r,c) + dv(r,c-1) == s
//   1  (row open)   E == H                      <=>  dh(r,c) == -1
//   8  (row extend) E == H and E[r][c-1] == H[r][c-1]
//                                               <=>  dh(r,c) == -1, c >= 2, dh(r,c-1) == -1
//   4  (col open)   dv(r,c) == -1
//   16 (col extend) dv(r,c) == -1, r >= 2, dv(r-1,c) == -1
// with dv(r,0) = -1 (H[r][0] = -r).  _find_gap_open's test
// H[row][c'] + gap(col - c') == H[row][col] becomes "every dh in (c', col] is
// -1", so the scan back to the border stops where that run ends: past it no
// cell can match and the walked path is dead.
//
// The DFS below follows pairwise2's _recover_alignments step for step (the
// lowest remaining trace bit first, the rest pushed as an alternative; col_gap
// forbids a seqA gap right after a seqB gap; _finish_backtrace at a border)
// and stops at the first alignment that completes, which is element [0] of
// pairwise2's list.  It only keeps counters of the match line
// (format_alignment's '|' where the two aligned characters are equal, so a
// '-' in a sequence opposite a gap also counts) plus the first and the last
// 64 flags, enough for AligmentScore's cutoff <= 64.
//
// Shared by the HIP kernel (misscore_kernels.hip) and the CPU emulator of the
// tests (tests/cpp/misscore_emu.cpp): the includer defines SVS_MS_FN.
#pragma once
#include <cstdint>

#ifndef SVS_MS_FN
#error "define SVS_MS_FN (function qualifiers) before including misscore_tb.hpp"
#endif

namespace svs {

// One DFS state (pairwise2's in_process tuple, with counters for strings).
struct MsState {
  int32_t row, col;
  int32_t trace;    // remaining trace bits
  int32_t col_gap;  // the last move was a gap in seqB
  int32_t nc, nm;   // match-line columns so far and '|' among them
  uint64_t front;   // flags of match-line positions 0..63 in traceback order
  uint64_t recent;  // the last 64 flags, bit 0 = the latest
};

// MsResult::status
constexpr int32_t kMsOk = 0;
constexpr int32_t kMsStepLimit = 1;     // traceback exceeded its step budget
constexpr int32_t kMsStackFull = 2;     // DFS stack capacity exceeded
constexpr int32_t kMsNoAlignment = 3;   // every path dead (pairwise2 retries transposed)
constexpr int32_t kMsEmpty = 4;         // an empty sequence: pairwise2 returns []

struct MsResult {
  int32_t status;
  int32_t cols;        // len(match line)
  int32_t matches;     // count('|')
  int32_t trim_len;    // len(alig[cutoff:len-cutoff])
  int32_t trim_match;  // its count('|')
  int32_t max_depth;   // deepest stack use
  int64_t steps;       // DFS steps
};

SVS_MS_FN void ms_put(MsState& s, uint32_t f) {
  if (s.nc < 64) s.front |= static_cast<uint64_t>(f) << s.nc;
  s.recent = (s.recent << 1) | f;
  s.nc += 1;
  s.nm += static_cast<int32_t>(f);
}

SVS_MS_FN int32_t ms_dh(uint32_t nib) { return static_cast<int32_t>(nib & 3u) - 1; }
SVS_MS_FN int32_t ms_dv(uint32_t nib) { return static_cast<int32_t>(nib >> 2) - 1; }

// Trace bits of cell (r, c); 0 on the borders (pairwise2 leaves them None).
template <class Env>
SVS_MS_FN int32_t ms_trace(Env& env, int32_t r, int32_t c) {
  if (r == 0 || c == 0) return 0;
  const uint32_t n = env.nib(r, c);
  const int32_t dh = ms_dh(n), dv = ms_dv(n);
  int32_t dvl = -1, dhl = 0;
  if (c >= 2) {
    const uint32_t nl = env.nib(r, c - 1);
    dvl = ms_dv(nl);
    dhl = ms_dh(nl);
  }
  const int32_t s = env.a(r - 1) == env.b(c - 1) ? 1 : 0;
  int32_t t = (dh + dvl == s) ? 2 : 0;
  if (dh == -1) t |= (dhl == -1) ? 9 : 1;
  if (dv == -1) t |= (r >= 2 && ms_dv(env.nib(r - 1, c)) == -1) ? 20 : 4;
  return t;
}

// _find_gap_open along the row (horizontal, a gap in seqA) or the column.
// Pushes every cell where the gap could have opened (n > 0); returns dead.
template <class Env>
SVS_MS_FN bool ms_gap_open(Env& env, MsState& cur, bool horizontal, int32_t& depth, bool& overflow) {
  const int32_t target = horizontal ? cur.col : cur.row;
  for (int32_t n = 0; n < target; ++n) {
    // the cell this step leaves must continue the run of -1 differences
    const uint32_t nib = env.nib(cur.row, cur.col);
    const bool run = (horizontal ? ms_dh(nib) : ms_dv(nib)) == -1;
    if (horizontal) {
      cur.col -= 1;
      ms_put(cur, env.b(cur.col) == '-');
    } else {
      cur.row -= 1;
      ms_put(cur, env.a(cur.row) == '-');
    }
    if (!run) return true;  // no later cell can match: walked to the border, dead
    if (n > 0) {
      const bool border = horizontal ? cur.col == 0 : cur.row == 0;
      if (border) return false;  // pairwise2 breaks here and finishes the path
      MsState alt = cur;
      alt.trace = ms_trace(env, cur.row, cur.col);
      alt.col_gap = horizontal ? 0 : 1;
      if (!env.push(alt)) {
        overflow = true;
        return true;
      }
      if (++depth > env.max_depth) env.max_depth = depth;
    }
    if (horizontal ? cur.col == 0 : cur.row == 0) return true;
  }
  return true;
}

template <class Env>
SVS_MS_FN MsResult ms_first_alignment(Env& env, int32_t la, int32_t lb, int32_t cutoff, int64_t max_steps) {
  MsResult res{};
  res.status = kMsNoAlignment;
  if (la <= 0 || lb <= 0) {
    res.status = kMsEmpty;
    return res;
  }
  int32_t depth = 0;
  bool overflow = false;
  env.max_depth = 0;
  {
    MsState st{};
    st.row = la;
    st.col = lb;
    st.trace = ms_trace(env, la, lb);
    env.push(st);
    depth = 1;
  }
  int64_t steps = 0;
  MsState cur{};
  while (depth > 0) {
    env.pop(cur);
    --depth;
    int32_t trace = cur.trace;
    bool dead = false;
    while ((cur.row > 0 || cur.col > 0) && !dead) {
      if (++steps > max_steps) {
        res.status = kMsStepLimit;
        res.steps = steps;
        return res;
      }
      MsState cache = cur;
      if (!trace) {
        if (cur.col && cur.col_gap) {
          dead = true;
        } else {  // _finish_backtrace: the rest of one sequence against gaps
          for (int32_t k = cur.row - 1; k >= 0; --k) ms_put(cur, env.a(k) == '-');
          for (int32_t k = cur.col - 1; k >= 0; --k) ms_put(cur, env.b(k) == '-');
        }
        break;
      } else if (trace & 1) {
        trace -= 1;
        if (cur.col_gap) {
          dead = true;
        } else {
          cur.col -= 1;
          ms_put(cur, env.b(cur.col) == '-');
          cur.col_gap = 0;
        }
      } else if (trace & 2) {
        trace -= 2;
        cur.row -= 1;
        cur.col -= 1;
        ms_put(cur, env.a(cur.row) == env.b(cur.col));
        cur.col_gap = 0;
      } else if (trace & 4) {
        trace -= 4;
        cur.row -= 1;
        ms_put(cur, env.a(cur.row) == '-');
        cur.col_gap = 1;
      } else if (trace & 8) {
        trace -= 8;
        if (cur.col_gap) {
          dead = true;
        } else {
          cur.col_gap = 0;
          dead = ms_gap_open(env, cur, true, depth, overflow);
        }
      } else {  // trace == 16
        trace -= 16;
        cur.col_gap = 1;
        dead = ms_gap_open(env, cur, false, depth, overflow);
      }
      if (overflow) {
        res.status = kMsStackFull;
        return res;
      }
      if (trace) {
        cache.trace = trace;
        if (!env.push(cache)) {
          res.status = kMsStackFull;
          return res;
        }
        if (++depth > env.max_depth) env.max_depth = depth;
      }
      trace = ms_trace(env, cur.row, cur.col);
    }
    if (!dead) {
      res.status = kMsOk;
      res.cols = cur.nc;
      res.matches = cur.nm;
      res.steps = steps;
      res.max_depth = env.max_depth;
      if (cutoff <= 0) {
        res.trim_len = cur.nc;
        res.trim_match = cur.nm;
      } else if (cur.nc - cutoff <= cutoff) {
        res.trim_len = 0;
        res.trim_match = 0;
      } else {
        const uint64_t mask = cutoff >= 64 ? ~0ull : ((1ull << cutoff) - 1);
        res.trim_len = cur.nc - 2 * cutoff;
        res.trim_match = cur.nm - __builtin_popcountll(cur.front & mask) - __builtin_popcountll(cur.recent & mask);
      }
      return res;
    }
  }
  res.steps = steps;
  return res;
}

}  // namespace svs
