// TEST INFRASTRUCTURE: scalar CPU emulation of the strip kernel (svscope_amd/csrc/poa_strip.hip) and of
// a row-major sweep over the host planner's export_rows tables
// (lanes become a loop) driven by the product's host graph engine
// (poa_graph.cpp).  Lets the CPU test suite check the kernel's two-scan
// recurrence, traceback codes and code-driven traceback against the oracle
// without a GPU.  Not part of the product library.
#include <algorithm>
#include <chrono>
#include <climits>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../svscope_amd/csrc/poa_graph.hpp"

namespace {
constexpr int32_t NEG_INF = INT32_MIN + 1024;
constexpr int32_t VNEG = INT32_MIN / 2;
struct Score { int32_t m, n, g, e, q, c; };

int32_t r0e(const Score& P, int32_t j) { return j == 0 ? 0 : P.g + (j - 1) * P.e; }
int32_t r0q(const Score& P, int32_t j) { return j == 0 ? 0 : P.q + (j - 1) * P.c; }
int32_t r0h(const Score& P, int32_t j) { return j == 0 ? 0 : std::max(r0q(P, j), r0e(P, j)); }

std::vector<int32_t> emu_traceback(const svs::RowTables& T, const std::vector<uint16_t>& tb, uint64_t LS, int32_t L,
                                   int32_t best_row, const Score& P) {
  std::vector<int32_t> out;
  auto tbc = [&](int32_t row, int32_t col) -> uint32_t { return tb[static_cast<uint64_t>(row - 1) * LS + col]; };
  auto pred_of = [&](int32_t row, uint32_t k) -> int32_t {
    const uint32_t a = T.pstart[row - 1], b = T.pstart[row];
    return b == a ? 0 : static_cast<int32_t>(T.pred_row[a + k]);
  };
  int32_t i = best_row, jj = L;
  while (!(i == 0 && jj == 0)) {
    int32_t pi = i, pj = jj;
    bool el = false, eu = false;
    if (i == 0) {
      const int32_t Hij = r0h(P, jj);
      const bool a = Hij == r0e(P, jj - 1) + P.e, b = Hij == r0h(P, jj - 1) + P.g;
      const bool c = Hij == r0q(P, jj - 1) + P.c, d = Hij == r0h(P, jj - 1) + P.q;
      if (!(a || b || c || d)) throw std::runtime_error("emu: row0 no move");
      el = a || (!b && c);
      pj = jj - 1;
    } else {
      const uint32_t code = tbc(i, jj), t = code & 3u, k = (code >> 3) & 31u;
      if (t == 0) { pi = pred_of(i, k); pj = jj - 1; }
      else if (t == 1) { pi = pred_of(i, k); eu = (code >> 2) & 1u; }
      else if (t == 2) { pj = jj - 1; el = (code >> 2) & 1u; }
      else throw std::runtime_error("emu: no move");
    }
    out.push_back(pi == i ? -1 : i - 1);
    out.push_back(pj == jj ? -1 : jj - 1);
    i = pi; jj = pj;
    if (el) {
      while (true) {
        out.push_back(-1); out.push_back(jj - 1); --jj;
        const bool stop = i == 0 ? (r0h(P, jj) + P.g == r0e(P, jj + 1) || r0h(P, jj) + P.q == r0q(P, jj + 1))
                                 : ((tbc(i, jj + 1) >> 8) & 1u);
        if (stop) break;
      }
    } else if (eu) {
      while (true) {
        const uint32_t code = tbc(i, jj), k = (code >> 10) & 31u;
        const bool stop = (code >> 9) & 1u;
        const int32_t nxt = k == 31u ? 0 : pred_of(i, k);
        out.push_back(i - 1); out.push_back(-1);
        i = nxt;
        if (stop || i == 0) break;
      }
    }
  }
  std::vector<int32_t> fwd(out.size());
  const size_t n = out.size() / 2;
  for (size_t k = 0; k < n; ++k) { fwd[2 * k] = out[2 * (n - 1 - k)]; fwd[2 * k + 1] = out[2 * (n - 1 - k) + 1]; }
  return fwd;
}

// returns forward rank pairs
std::vector<int32_t> emu_align(const svs::RowTables& T, const std::string& seq, const Score& P) {
  const int32_t L = static_cast<int32_t>(seq.size());
  const uint64_t LS = (static_cast<uint64_t>(L) + 1 + 63) / 64 * 64;
  const uint32_t V = static_cast<uint32_t>(T.info.size());
  std::vector<int32_t> pl(static_cast<size_t>(T.n_slots) * 3 * LS);
  std::vector<uint16_t> tb(static_cast<size_t>(V) * LS);
  for (int32_t j = 0; j <= L; ++j) {
    pl[j] = r0h(P, j);
    pl[LS + j] = j == 0 ? 0 : NEG_INF;
    pl[2 * LS + j] = j == 0 ? 0 : NEG_INF;
  }
  const int32_t nstrips = (L + 1 + 63) >> 6;
  int32_t best = NEG_INF, best_row = 0;
  int32_t Hpre[64], Fv[64], Ov[64], Q[64], E[64], H[64], x[64], y[64], pHpre[64], pQ[64], pE[64], pH[64];
  for (uint32_t r = 0; r < V; ++r) {
    const uint8_t nb = T.info[r] & 0xFF;
    const bool sink = (T.info[r] >> 8) & 1;
    const uint64_t so = static_cast<uint64_t>(T.slot[r]) * 3 * LS;
    const uint32_t p0 = T.pstart[r], np = T.pstart[r + 1] - p0, npass = np ? np : 1;
    const int32_t F0 = T.col0[3 * r + 1], O0 = T.col0[3 * r + 2];
    const int32_t H0 = std::max(F0, O0);
    int32_t run1 = VNEG, run2 = VNEG, cHpre = H0, cQ = NEG_INF, cE = NEG_INF, cH = H0;
    for (int32_t s = 0; s < nstrips; ++s) {
      auto pslot = [&](uint32_t k) -> uint64_t {
        return np == 0 ? 0 : static_cast<uint64_t>(T.pred_slot[p0 + k]) * 3 * LS;
      };
      for (int l = 0; l < 64; ++l) {
        const int32_t j = s * 64 + l;
        const bool valid = j <= L, c0 = j == 0, inner = valid && !c0;
        const int32_t mc = (inner && static_cast<uint8_t>(seq[j - 1]) == nb) ? P.m : P.n;
        int32_t F = VNEG, O = VNEG, Hd = VNEG;
        if (inner) {
          for (uint32_t k = 0; k < npass; ++k) {
            const uint64_t ps = pslot(k);
            F = std::max(F, std::max(pl[ps + j] + P.g, pl[ps + LS + j] + P.e));
            O = std::max(O, std::max(pl[ps + j] + P.q, pl[ps + 2 * LS + j] + P.c));
            Hd = std::max(Hd, pl[ps + j - 1] + mc);
          }
        } else if (c0) { F = F0; O = O0; }
        Fv[l] = F; Ov[l] = O;
        Hpre[l] = c0 ? H0 : std::max(Hd, std::max(F, O));
      }
      // carry-independent scans (kernel v3 formulation)
      int32_t P1[64], P2[64];
      for (int l = 0; l < 64; ++l) pHpre[l] = l == 0 ? cHpre : Hpre[l - 1];
      for (int l = 0; l < 64; ++l) {
        const int32_t j = s * 64 + l; const bool inner = j <= L && j != 0;
        P1[l] = inner ? pHpre[l] + P.q - j * P.c : VNEG;
      }
      for (int l = 1; l < 64; ++l) P1[l] = std::max(P1[l], P1[l - 1]);
      for (int l = 0; l < 64; ++l) {
        const int32_t j = s * 64 + l; const bool inner = j <= L && j != 0;
        const int32_t qloc = l > 0 ? P1[l - 1] + (j - 1) * P.c : VNEG;
        P2[l] = inner ? std::max(pHpre[l], qloc) + P.g - j * P.e : VNEG;
      }
      for (int l = 1; l < 64; ++l) P2[l] = std::max(P2[l], P2[l - 1]);
      const int32_t j0 = s * 64;
      const int32_t T1 = s > 0 ? cQ + P.g - j0 * P.e : VNEG;
      for (int l = 0; l < 64; ++l) {
        const int32_t j = s * 64 + l; const bool inner = j <= L && j != 0;
        const int32_t T2 = l > 0 ? run1 + (j - 1) * P.c + P.g - j * P.e : VNEG;
        pQ[l] = 0;
        Q[l] = inner ? j * P.c + std::max(P1[l], run1) : NEG_INF;
        E[l] = inner ? j * P.e + std::max(std::max(P2[l], run2), std::max(T1, T2)) : NEG_INF;
        H[l] = inner ? std::max(Hpre[l], std::max(E[l], Q[l])) : H0;
      }
      {
        const int32_t jl = j0 + 63;
        const int32_t T2l = run1 + (jl - 1) * P.c + P.g - jl * P.e;
        run2 = std::max(std::max(run2, P2[63]), std::max(T1, T2l));
        run1 = std::max(run1, P1[63]);
      }
      for (int l = 0; l < 64; ++l) pQ[l] = l == 0 ? cQ : Q[l - 1];
      for (int l = 0; l < 64; ++l) { pE[l] = l == 0 ? cE : E[l - 1]; pH[l] = l == 0 ? cH : H[l - 1]; }
      for (int l = 0; l < 64; ++l) {
        const int32_t j = s * 64 + l;
        const bool valid = j <= L, c0 = j == 0, inner = valid && !c0;
        if (!valid) continue;
        const int32_t mc = (inner && static_cast<uint8_t>(seq[j - 1]) == nb) ? P.m : P.n;
        uint32_t dk = 31, uk = 31, ue = 0, ck = 31, cs = 0;
        for (uint32_t k = 0; k < npass; ++k) {
          const uint64_t ps = pslot(k);
          const int32_t hpm = inner ? pl[ps + j - 1] : 0, hp = pl[ps + j], fp = pl[ps + LS + j], op = pl[ps + 2 * LS + j];
          if (inner && dk == 31 && H[l] == hpm + mc) dk = k;
          if (uk == 31) {
            const bool a = H[l] == fp + P.e, b = H[l] == hp + P.g, c = H[l] == op + P.c, d = H[l] == hp + P.q;
            if (a || b || c || d) { uk = k; ue = (a || (!b && c)) ? 1 : 0; }
          }
          if (np != 0 && ck == 31) {
            const bool a = Fv[l] == hp + P.g, b = Fv[l] == fp + P.e, c = Ov[l] == hp + P.q, d = Ov[l] == op + P.c;
            if (a || b || c || d) { ck = k; cs = (a || (!b && c)) ? 1 : 0; }
          }
        }
        uint32_t code;
        if (dk != 31) code = dk << 3;
        else if (uk != 31) code = 1u | (ue << 2) | (uk << 3);
        else {
          const bool a = inner && H[l] == pE[l] + P.e, b = inner && H[l] == pH[l] + P.g;
          const bool c = inner && H[l] == pQ[l] + P.c, d = inner && H[l] == pH[l] + P.q;
          code = (a || b || c || d) ? (2u | ((a || (!b && c)) ? 4u : 0u)) : 3u;
        }
        const bool lbit = inner && (pH[l] + P.g == E[l] || pH[l] + P.q == Q[l]);
        code |= (lbit ? 1u : 0u) << 8;
        code |= cs << 9;
        code |= ck << 10;
        tb[static_cast<uint64_t>(r) * LS + j] = static_cast<uint16_t>(code);
        if (sink && j == L && H[l] > best) { best = H[l]; best_row = static_cast<int32_t>(r) + 1; }
      }
      // stores after all lanes read this strip's pred values (row slots differ from pred slots)
      for (int l = 0; l < 64; ++l) {
        const int32_t j = s * 64 + l;
        if (j > L) continue;
        pl[so + j] = H[l];
        pl[so + LS + j] = j == 0 ? F0 : Fv[l];
        pl[so + 2 * LS + j] = j == 0 ? O0 : Ov[l];
      }
      cHpre = Hpre[63]; cQ = Q[63]; cE = E[63]; cH = H[63];
    }
  }
  return emu_traceback(T, tb, LS, L, best_row, P);
}

// Strip-major emulation of poa_strip.hip on the export_strip_rows tables:
// per strip, a 64-column pool with the planner's slots, register pass-through
// for in-edges from the row just above, per-slot boundary H, and the per-row
// carries handed from strip to strip.
// Exact pruning (poa_strip.hip): with lb <= the optimum, a strip row is
// skipped when none of its inputs is alive, and a computed row whose every
// cell has H + ub < lb is marked dead; *retry is set when the best sink score
// falls below lb (the bound did not hold: the caller re-runs with no pruning).
struct StripPrune {
  int32_t lb = INT32_MIN / 2;  // no pruning
  bool retry = false;
  int32_t best = 0;  // best sink score at column L (the optimum when lb held)
  uint64_t rows_done = 0, rows_all = 0;
  uint64_t rows_slow_skip = 0;  // rows skipped one by one (not inside a fast_forward jump)
};

int32_t upper_suffix(const Score& P, int32_t rr, uint32_t w2) {
  const int32_t dmin = static_cast<int32_t>(w2 & 0xFFFF), dmax = static_cast<int32_t>(w2 >> 16);
  const int32_t cg = std::max(std::max(P.g, P.e), std::max(P.q, P.c));
  if (std::getenv("EMU_LOOSE")) return P.m * rr;
  return P.m * rr + cg * std::max(0, dmin - rr) - (P.m - cg) * std::max(0, rr - dmax);
}

std::vector<int32_t> emu_align_strip(const svs::RowTables& T, const std::string& seq, const Score& P,
                                     StripPrune* prune = nullptr) {
  StripPrune none;
  StripPrune& PR = prune ? *prune : none;
  const bool on = prune != nullptr;
  const int32_t L = static_cast<int32_t>(seq.size());
  const uint64_t LS = (static_cast<uint64_t>(L) + 1 + 63) / 64 * 64;
  const uint32_t V = static_cast<uint32_t>(T.pstart.size() - 1);
  const int32_t nstrips = static_cast<int32_t>(LS >> 6);
  std::vector<int32_t> pool(static_cast<size_t>(T.n_slots) * 192, 0x7eadbeef), slot_ch(T.n_slots, 0x7eadbeef);
  std::vector<int32_t> bnd(static_cast<size_t>(V) * 4 * 2, 0);
  std::vector<uint16_t> tb(static_cast<size_t>(V) * LS);
  std::vector<uint8_t> written(T.n_slots, 0);
  int32_t best = NEG_INF, best_row = 0;
  for (int32_t s = 0; s < nstrips; ++s) {
    const bool FIRST = s == 0;
    const int32_t j0 = s * 64;
    int32_t* bin = bnd.data() + static_cast<size_t>((s + 1) & 1) * V * 4;
    int32_t* bout = bnd.data() + static_cast<size_t>(s & 1) * V * 4;
    std::fill(written.begin(), written.end(), 0);
    for (int l = 0; l < 64; ++l) {
      const int32_t j = j0 + l;
      const uint32_t tF = static_cast<uint32_t>(P.e - P.g + 1), tO = static_cast<uint32_t>(P.c - P.q + 1);
      const int32_t h0 = r0h(P, j), fo = j == 0 ? 0 : NEG_INF;
      pool[l] = h0;
      pool[64 + l] = h0 - static_cast<int32_t>(std::min(static_cast<uint32_t>(h0) - static_cast<uint32_t>(fo), tF));
      pool[128 + l] = h0 - static_cast<int32_t>(std::min(static_cast<uint32_t>(h0) - static_cast<uint32_t>(fo), tO));
    }
    slot_ch[0] = FIRST ? 0 : r0h(P, j0 - 1);
    written[0] = 1;
    std::vector<uint8_t> slot_alive(T.n_slots, 0);
    // the virtual row 0: alive when row0_h + m (L - j) reaches lb at j0-1
    slot_alive[0] = FIRST || !on || static_cast<int64_t>(r0h(P, j0 - 1)) + P.m * (L - j0 + 1) >= PR.lb;
    bool reg_alive = false;
    int32_t pHv[64], pFv[64], pOv[64], pcH = 0;
    for (uint32_t r = 0; r < V; ++r) {
      const uint32_t* w = T.rec.data() + static_cast<size_t>(r) * svs::kRecWords;
      const uint32_t nb = w[0] & 0xFF, np = (w[0] >> 10) & 31;
      const bool sink = (w[0] >> 8) & 1, store = (w[0] >> 9) & 1;
      const uint32_t own = w[0] >> 16;
      PR.rows_all += 1;
      // the kernel's freed-slot bits (w3) and its fast_forward condition
      auto clear_freed = [&]() {
        for (uint32_t f = 0; f < 32 && f < slot_alive.size(); ++f)
          if ((w[3] >> f) & 1u) slot_alive[f] = 0;
      };
      bool dead_state = !reg_alive;
      for (size_t k = 1; k < slot_alive.size(); ++k) dead_state = dead_state && !slot_alive[k];
      if (on && dead_state) {
        // the kernel's fast_forward: rows passed over, then every slot but the
        // virtual row's reset to VNEG (idempotent here, row by row)
        for (uint32_t p = 1; p < T.n_slots; ++p) {
          for (int l = 0; l < 192; ++l) pool[p * 192 + l] = VNEG;
          slot_ch[p] = VNEG;
          written[p] = 1;
        }
        for (int l = 0; l < 64; ++l) { pHv[l] = VNEG; pFv[l] = VNEG; pOv[l] = VNEG; }
        pcH = VNEG;
      }
      if (on) {
        // skip: no live input (carry from strip s-1 / strip 0's column-0 cell,
        // or an in-edge row's slot in this strip; a source reads slot 0)
        const bool carry_alive = FIRST ? static_cast<int64_t>(T.col0[3 * r]) + upper_suffix(P, L, w[2]) >= PR.lb
                                       : bin[4 * r + 3] > VNEG / 2;
        bool pred_alive = np == 0 && slot_alive[0];
        for (uint32_t k = 0; k < np; ++k) {
          const uint32_t ps = np <= svs::kInlinePreds ? (w[1] >> (16 * k)) & 0xFFFF : T.pred_slot[T.pstart[r] + k];
          pred_alive = pred_alive || (ps == svs::kNoSlot ? reg_alive : slot_alive[ps] != 0);
        }
        if (!carry_alive && !pred_alive) {
          if (store) {
            for (int l = 0; l < 192; ++l) pool[own * 192 + l] = VNEG;
            slot_ch[own] = VNEG;
            written[own] = 1;
            slot_alive[own] = 0;
          }
          clear_freed();
          for (int l = 0; l < 64; ++l) { pHv[l] = VNEG; pFv[l] = VNEG; pOv[l] = VNEG; }
          pcH = VNEG;
          reg_alive = false;
          for (int x = 0; x < 4; ++x) bout[4 * r + x] = VNEG;
          if (!dead_state) PR.rows_slow_skip += 1;
          continue;
        }
      }
      PR.rows_done += 1;
      int32_t run1, run2, cHpre, cQ, cE, cH, H0 = 0, F0 = 0, O0 = 0;
      if (FIRST) {
        H0 = T.col0[3 * r]; F0 = T.col0[3 * r + 1]; O0 = T.col0[3 * r + 2];
        run1 = VNEG; run2 = VNEG; cHpre = H0; cQ = NEG_INF; cE = NEG_INF; cH = H0;
      } else {
        run1 = bin[4 * r]; run2 = bin[4 * r + 1]; cHpre = bin[4 * r + 2]; cH = bin[4 * r + 3];
        cQ = (j0 - 1) * P.c + run1; cE = (j0 - 1) * P.e + run2;
      }
      const int32_t cH_in = cH;
      const uint32_t npass = np ? np : 1;
      auto slot_of = [&](uint32_t k) -> uint32_t {
        if (np == 0) return 0;
        if (np <= svs::kInlinePreds) return (w[1] >> (16 * k)) & 0xFFFF;
        return T.pred_slot[T.pstart[r] + k];
      };
      auto vals = [&](uint32_t k, int l, int32_t& hp, int32_t& fp, int32_t& op, int32_t& hpm) {
        const uint32_t ps = slot_of(k);
        int32_t fill;
        if (ps == svs::kNoSlot) {
          if (r == 0) throw std::runtime_error("emu strip: register in-edge on row 0");
          hp = pHv[l]; fp = pFv[l]; op = pOv[l]; fill = pcH;
          hpm = l == 0 ? fill : pHv[l - 1];
        } else {
          if (!written[ps]) throw std::runtime_error("emu strip: read of an unwritten pool slot");
          hp = pool[ps * 192 + l]; fp = pool[ps * 192 + 64 + l]; op = pool[ps * 192 + 128 + l]; fill = slot_ch[ps];
          hpm = l == 0 ? fill : pool[ps * 192 + l - 1];
        }
      };
      int32_t Hpre[64], Fv[64], Ov[64], Hd[64];
      for (int l = 0; l < 64; ++l) {
        const int32_t j = j0 + l;
        const bool c0 = FIRST && l == 0;
        const int32_t mc = static_cast<uint8_t>(j >= 1 && j <= L ? seq[j - 1] : 0) == nb ? P.m : P.n;
        int32_t F = VNEG, O = VNEG, D = VNEG;
        for (uint32_t k = 0; k < npass; ++k) {
          int32_t hp, fp, op, hpm;
          vals(k, l, hp, fp, op, hpm);
          // no floor: a dead in-edge (VNEG) gives VNEG + g etc., as in the kernel
          const int32_t f = std::max(hp + P.g, fp + P.e), o = std::max(hp + P.q, op + P.c), d = (c0 ? 0 : hpm) + mc;
          F = k == 0 ? f : std::max(F, f);
          O = k == 0 ? o : std::max(O, o);
          D = k == 0 ? d : std::max(D, d);
        }
        if (c0) { F = F0; O = O0; }
        Fv[l] = F; Ov[l] = O; Hd[l] = D;
        Hpre[l] = c0 ? H0 : std::max(D, std::max(F, O));
      }
      int32_t P1[64], P2[64], Q[64], E[64], H[64], pHp[64];
      for (int l = 0; l < 64; ++l) pHp[l] = l == 0 ? cHpre : Hpre[l - 1];
      auto inner_of = [&](int l) { const int32_t j = j0 + l; return FIRST ? (l != 0 && j <= L) : true; };
      for (int l = 0; l < 64; ++l) P1[l] = inner_of(l) ? pHp[l] + P.q - (j0 + l) * P.c : VNEG;
      for (int l = 1; l < 64; ++l) P1[l] = std::max(P1[l], P1[l - 1]);
      for (int l = 0; l < 64; ++l) {
        const int32_t j = j0 + l;
        const int32_t p1m = l > 0 ? P1[l - 1] : VNEG;
        P2[l] = inner_of(l) ? std::max(pHp[l], p1m + (j - 1) * P.c) + P.g - j * P.e : VNEG;
      }
      for (int l = 1; l < 64; ++l) P2[l] = std::max(P2[l], P2[l - 1]);
      const int32_t T1 = j0 > 0 ? cQ + P.g - j0 * P.e : VNEG;
      for (int l = 0; l < 64; ++l) {
        const int32_t j = j0 + l;
        const int32_t T2 = l > 0 ? run1 + (j - 1) * P.c + P.g - j * P.e : VNEG;
        Q[l] = inner_of(l) ? j * P.c + std::max(P1[l], run1) : NEG_INF;
        E[l] = inner_of(l) ? j * P.e + std::max(std::max(P2[l], run2), std::max(T1, T2)) : NEG_INF;
        H[l] = inner_of(l) ? std::max(Hpre[l], std::max(E[l], Q[l])) : H0;
      }
      int32_t pQ[64], pE[64], pH[64];
      for (int l = 0; l < 64; ++l) {
        pQ[l] = l == 0 ? cQ : Q[l - 1]; pE[l] = l == 0 ? cE : E[l - 1]; pH[l] = l == 0 ? cH : H[l - 1];
      }
      {
        const int32_t jl = j0 + 63;
        const int32_t T2l = run1 + (jl - 1) * P.c + P.g - jl * P.e;
        run2 = std::max(std::max(run2, P2[63]), std::max(T1, T2l));
        run1 = std::max(run1, P1[63]);
        cQ = jl * P.c + run1; cE = jl * P.e + run2; cHpre = Hpre[63];
        cH = std::max(cHpre, std::max(cE, cQ));
      }
      for (int l = 0; l < 64; ++l) {
        const int32_t j = j0 + l;
        const bool c0 = FIRST && l == 0;
        const bool inner = inner_of(l);
        const int32_t mc = static_cast<uint8_t>(j >= 1 && j <= L ? seq[j - 1] : 0) == nb ? P.m : P.n;
        uint32_t dk = 31, uk = 31, ue = 0, ck = 31, cs = 0;
        for (uint32_t k = 0; k < npass; ++k) {
          int32_t hp, fp, op, hpm;
          vals(k, l, hp, fp, op, hpm);
          if (c0) hpm = 0;
          if (inner && dk == 31 && H[l] == hpm + mc) dk = k;
          if (uk == 31) {
            const bool a = H[l] == fp + P.e, b = H[l] == hp + P.g, c = H[l] == op + P.c, d = H[l] == hp + P.q;
            if (a || b || c || d) { uk = k; ue = (a || (!b && c)) ? 1 : 0; }
          }
          if (np != 0 && ck == 31) {
            const bool a = Fv[l] == hp + P.g, b = Fv[l] == fp + P.e, c = Ov[l] == hp + P.q, d = Ov[l] == op + P.c;
            if (a || b || c || d) { ck = k; cs = (a || (!b && c)) ? 1 : 0; }
          }
        }
        uint32_t code;
        if (dk != 31) code = dk << 3;
        else if (uk != 31) code = 1u | (ue << 2) | (uk << 3);
        else {
          const bool a = inner && H[l] == pE[l] + P.e, b = inner && H[l] == pH[l] + P.g;
          const bool c = inner && H[l] == pQ[l] + P.c, d = inner && H[l] == pH[l] + P.q;
          code = (a || b || c || d) ? (2u | ((a || (!b && c)) ? 4u : 0u)) : 3u;
        }
        const bool lbit = inner && (pH[l] + P.g == E[l] || pH[l] + P.q == Q[l]);
        code |= (lbit ? 1u : 0u) << 8;
        code |= cs << 9;
        code |= ck << 10;
        if (np <= 1) {
          // the kernel's fast-path formula (identities H==max(F,O), H==max(E,Q))
          int32_t hp, fp, op, hpm;
          vals(0, l, hp, fp, op, hpm);
          if (c0) hpm = 0;
          const bool dg = inner && H[l] == hpm + mc;
          const bool up = H[l] == std::max(Fv[l], Ov[l]);
          const bool ua = H[l] == fp + P.e, ub = H[l] == hp + P.g, uc = H[l] == op + P.c;
          const bool lf = inner && H[l] == std::max(E[l], Q[l]);
          const bool la = H[l] == pE[l] + P.e, lb = H[l] == pH[l] + P.g, lc = H[l] == pQ[l] + P.c;
          const bool va = Fv[l] == hp + P.g, vb = Fv[l] == fp + P.e, vc = Ov[l] == hp + P.q;
          uint32_t c2 = dg ? 0u : (up ? ((ua || (!ub && uc)) ? 5u : 1u) : (lf ? ((la || (!lb && lc)) ? 6u : 2u) : 3u));
          c2 |= lbit ? 0x100u : 0u;
          if (np != 0) c2 |= (va || (!vb && vc)) ? 0x200u : 0u;
          else c2 |= 31u << 10;
          if (c2 != code) {
            char buf[512];
            snprintf(buf, sizeof buf, "emu strip: fast-path code formula differs (code %x fast %x np %u r %u l %d s %d H %d F %d O %d E %d Q %d hp %d fp %d op %d hpm %d pE %d pH %d pQ %d lb %d)",
                     code, c2, np, r, l, s, H[l], Fv[l], Ov[l], E[l], Q[l], hp, fp, op, hpm, pE[l], pH[l], pQ[l], PR.lb);
            throw std::runtime_error(buf);
          }
        }
        if (np == 2 && !FIRST) {
          // the kernel's two-in-edge formula
          int32_t hp0, fp0, op0, hm0, hp1, fp1, op1, hm1;
          vals(0, l, hp0, fp0, op0, hm0);
          vals(1, l, hp1, fp1, op1, hm1);
          const int32_t F0k = std::max(hp0 + P.g, fp0 + P.e), O0k = std::max(hp0 + P.q, op0 + P.c);
          const int32_t F1k = std::max(hp1 + P.g, fp1 + P.e), O1k = std::max(hp1 + P.q, op1 + P.c);
          const int32_t Fr = Fv[l], Or = Ov[l], Hh = H[l];
          const bool up0 = Hh == std::max(F0k, O0k), up1 = Hh == std::max(F1k, O1k);
          const int32_t hpu = up0 ? hp0 : hp1, fpu = up0 ? fp0 : fp1, opu = up0 ? op0 : op1;
          const bool ua = Hh == fpu + P.e, ub = Hh == hpu + P.g, uc = Hh == opu + P.c;
          const bool ch0 = Fr == F0k || Or == O0k;
          const int32_t hpc = ch0 ? hp0 : hp1, fpc = ch0 ? fp0 : fp1;
          const bool va = Fr == hpc + P.g, vb = Fr == fpc + P.e, vc = Or == hpc + P.q;
          const bool lf = Hh == std::max(E[l], Q[l]);
          const bool la = Hh == pE[l] + P.e, lb = Hh == pH[l] + P.g, lc = Hh == pQ[l] + P.c;
          const uint32_t upc = ((ua || (!ub && uc)) ? 5u : 1u) | (up0 ? 0u : 8u);
          const uint32_t lfc = (la || (!lb && lc)) ? 6u : 2u;
          uint32_t c2 = Hh == hm0 + mc ? 0u : (Hh == hm1 + mc ? 8u : (up0 || up1 ? upc : (lf ? lfc : 3u)));
          c2 |= lbit ? 0x100u : 0u;
          c2 |= ((va || (!vb && vc)) ? 0x200u : 0u) | (ch0 ? 0u : (1u << 10));
          if (c2 != code) throw std::runtime_error("emu strip: two-in-edge code formula differs");
        }
        tb[static_cast<uint64_t>(r) * LS + j] = static_cast<uint16_t>(code);
        if (sink && j == L && H[l] > best) { best = H[l]; best_row = static_cast<int32_t>(r) + 1; }
      }
      bool any_alive = false;
      for (int l = 0; l < 64; ++l) {
        const int32_t j = j0 + l;
        if (j <= L && static_cast<int64_t>(H[l]) + upper_suffix(P, L - j, w[2]) >= PR.lb) any_alive = true;
      }
      const bool carry_in_alive = FIRST ? false : cH_in > VNEG / 2;
      const bool out_alive = any_alive || carry_in_alive;
      reg_alive = out_alive;
      if (store && on) slot_alive[own] = out_alive;
      if (on) clear_freed();
      if (store) {
        if (own == svs::kNoSlot || own == 0 || own >= T.n_slots) throw std::runtime_error("emu strip: bad own slot");
        // the kernel keeps F, O as distances to H clamped at e-g+1 / c-q+1
        const uint32_t tF = static_cast<uint32_t>(P.e - P.g + 1), tO = static_cast<uint32_t>(P.c - P.q + 1);
        for (int l = 0; l < 64; ++l) {
          const uint32_t dF = std::min(static_cast<uint32_t>(H[l]) - static_cast<uint32_t>(Fv[l]), tF);
          const uint32_t dO = std::min(static_cast<uint32_t>(H[l]) - static_cast<uint32_t>(Ov[l]), tO);
          pool[own * 192 + l] = H[l];
          pool[own * 192 + 64 + l] = H[l] - static_cast<int32_t>(dF);
          pool[own * 192 + 128 + l] = H[l] - static_cast<int32_t>(dO);
        }
        slot_ch[own] = cH_in;
        written[own] = 1;
      }
      for (int l = 0; l < 64; ++l) { pHv[l] = H[l]; pFv[l] = Fv[l]; pOv[l] = Ov[l]; }
      pcH = cH_in;
      if (any_alive || !on) {
        bout[4 * r] = run1; bout[4 * r + 1] = run2; bout[4 * r + 2] = cHpre; bout[4 * r + 3] = cH;
      } else {
        for (int x = 0; x < 4; ++x) bout[4 * r + x] = VNEG;
      }
    }
  }
  PR.best = best;
  if (best < PR.lb) {
    PR.retry = true;
    return {};
  }
  return emu_traceback(T, tb, LS, L, best_row, P);
}

struct EmuResult {
  std::string consensus, error;
  std::vector<std::string> msa;
  uint32_t max_slots = 0;
  double graph_ms = 0, dp_ms = 0;
  // row-structure counters over every exported table (tools/row_stats.py)
  uint64_t rows = 0, np0 = 0, np1 = 0, np2 = 0, pred_prev = 0, must_store = 0, slot_sum = 0, tables = 0;
  uint64_t rows_done = 0, rows_all = 0, rows_slow = 0;  // strip rows computed / total / skipped one by one under EMU_PRUNE
};

void row_stats(const svs::RowTables& T, EmuResult* r) {
  const size_t R = T.info.size();
  std::vector<uint8_t> store(R + 1, 0);
  for (size_t i = 0; i < R; ++i) {
    const uint32_t a = T.pstart[i], b = T.pstart[i + 1], np = b - a;
    r->rows += 1;
    if (np == 0) r->np0 += 1; else if (np == 1) r->np1 += 1; else r->np2 += 1;
    for (uint32_t k = a; k < b; ++k) {
      const uint32_t p = T.pred_row[k];  // 1-based
      if (p == i) r->pred_prev += 1;     // pred is the row just above (row i is 1-based i+1)
      else if (p >= 1) store[p] = 1;
    }
  }
  for (size_t i = 1; i <= R; ++i) r->must_store += store[i];
  r->slot_sum += T.n_slots;
  r->tables += 1;
}
}  // namespace

extern "C" {
void* emu_poa(int n, const char* const* seqs, const int* lens, int m, int mis, int g, int e, int q, int c) {
  auto* r = new EmuResult();
  try {
    Score P{m, mis, g, e, q, c};
    svs::PoaGraph graph;
    svs::RowTables T;
    for (int s = 0; s < n; ++s) {
      std::string seq(seqs[s], static_cast<size_t>(lens[s]));
      if (seq.empty()) continue;
      if (graph.empty()) { graph.add_alignment_nodes({}, seq); continue; }
      auto t0 = std::chrono::steady_clock::now();
      const bool strip = std::getenv("EMU_STRIP") != nullptr;
      if (strip) graph.export_strip_rows(&T);
      else graph.export_rows(&T);
      svs::fill_col0(&T, P.g, P.e, P.q, P.c);
      auto t1 = std::chrono::steady_clock::now();
      r->max_slots = std::max(r->max_slots, T.n_slots);
      if (!strip) row_stats(T, r);
      std::vector<int32_t> aln;
      const char* pm = std::getenv("EMU_PRUNE");
      if (strip && pm) {
        // exactness check of the pruning: with lb = the optimum (the tightest
        // valid bound) the alignment must not change; with lb above it the
        // kernel must ask for a retry
        StripPrune full;
        aln = emu_align_strip(T, seq, P, &full);
        StripPrune tight;
        tight.lb = full.best - std::atoi(pm);
        const auto aln2 = emu_align_strip(T, seq, P, &tight);
        if (tight.retry || aln2 != aln) throw std::runtime_error("emu strip: pruned alignment differs");
        StripPrune over;
        over.lb = full.best + 1;
        emu_align_strip(T, seq, P, &over);
        if (!over.retry) throw std::runtime_error("emu strip: lb above the optimum not detected");
        r->rows_done += tight.rows_done;
        r->rows_all += tight.rows_all;
        r->rows_slow += tight.rows_slow_skip;
      } else {
        aln = strip ? emu_align_strip(T, seq, P) : emu_align(T, seq, P);
      }
      auto t2 = std::chrono::steady_clock::now();
      if (const char* rec = std::getenv("EMU_RECORD")) {
        // alignments for tests/cpp/host_bench.cpp: length-prefixed sequence and rank pairs
        if (FILE* f = std::fopen(rec, "ab")) {
          const uint32_t ls = static_cast<uint32_t>(seq.size()), la = static_cast<uint32_t>(aln.size());
          std::fwrite(&ls, 4, 1, f);
          std::fwrite(seq.data(), 1, ls, f);
          std::fwrite(&la, 4, 1, f);
          std::fwrite(aln.data(), 4, la, f);
          std::fclose(f);
        }
      }
      graph.add_alignment_ranks(aln, seq);
      auto t3 = std::chrono::steady_clock::now();
      r->graph_ms += std::chrono::duration<double, std::milli>((t1 - t0) + (t3 - t2)).count();
      r->dp_ms += std::chrono::duration<double, std::milli>(t2 - t1).count();
    }
    r->consensus = graph.consensus(-1);
    r->msa = graph.msa();
  } catch (const std::exception& ex) { r->error = ex.what(); }
  return r;
}
const char* emu_error(void* h) { auto* r = static_cast<EmuResult*>(h); return r->error.empty() ? nullptr : r->error.c_str(); }
const char* emu_consensus(void* h) { return static_cast<EmuResult*>(h)->consensus.c_str(); }
int emu_msa_rows(void* h) { return static_cast<int>(static_cast<EmuResult*>(h)->msa.size()); }
const char* emu_msa_row(void* h, int i) { return static_cast<EmuResult*>(h)->msa[i].c_str(); }
int emu_max_slots(void* h) { return static_cast<int>(static_cast<EmuResult*>(h)->max_slots); }
void emu_row_stats(void* h, uint64_t* out) {
  auto* r = static_cast<EmuResult*>(h);
  const uint64_t v[8] = {r->rows, r->np0, r->np1, r->np2, r->pred_prev, r->must_store, r->slot_sum, r->tables};
  for (int i = 0; i < 8; ++i) out[i] = v[i];
}
void emu_prune_rows(void* h, uint64_t* out) {
  auto* r = static_cast<EmuResult*>(h);
  out[0] = r->rows_done;
  out[1] = r->rows_all;
  out[2] = r->rows_slow;
}
void emu_free(void* h) { delete static_cast<EmuResult*>(h); }
double emu_graph_ms(void* h) { return static_cast<EmuResult*>(h)->graph_ms; }
}
