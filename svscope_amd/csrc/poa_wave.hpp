// Wave-level building blocks shared by the POA kernels (gfx950, wave64):
// DPP prefix-max scans, lane shifts, the two-scan convex horizontal-gap
// recurrence of one 64-column strip, traceback-code assembly and the lane-0
// traceback that replays spoa's backtrack order over the 16-bit codes.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

#include "svs_device.hpp"

namespace svs {

#define SVS_NEG_INF (INT32_MIN + 1024)
#define SVS_VNEG (INT32_MIN / 2)

__device__ __forceinline__ int32_t imax(int32_t a, int32_t b) { return a > b ? a : b; }

// One step of an inclusive prefix-max scan: x = max(x, x[src lane]) as a
// DPP-combined v_max_i32_dpp.  Lanes with no source (row_shr at a row's start)
// or in a masked row read the identity INT32_MIN, so they keep x.  Written
// with the builtin so that the compiler sees the DPP read-after-write hazard
// (2 wait states on gfx950) and fills it with independent work instead of a
// fixed s_nop.
template <int CTRL, int ROW_MASK>
__device__ __forceinline__ int32_t dpp_max_step(int32_t x) {
  return imax(x, __builtin_amdgcn_update_dpp(static_cast<int32_t>(INT32_MIN), x, CTRL, ROW_MASK, 0xF, false));
}

// Inclusive prefix max over the 64 lanes of a wave: row_shr 1/2/4/8 within
// each 16-lane row, then row_bcast15 (rows 1, 3) and row_bcast31 (rows 2, 3).
__device__ __forceinline__ int32_t wave_prefix_max(int32_t x) {
  x = dpp_max_step<0x111, 0xF>(x);
  x = dpp_max_step<0x112, 0xF>(x);
  x = dpp_max_step<0x114, 0xF>(x);
  x = dpp_max_step<0x118, 0xF>(x);
  x = dpp_max_step<0x142, 0xA>(x);
  x = dpp_max_step<0x143, 0xC>(x);
  return x;
}

// Two independent inclusive prefix-max scans, written step by step so that
// the compiler interleaves the two dependency chains (each step of one scan
// covers a wait state of the other).
__device__ __forceinline__ void wave_prefix_max2(int32_t& a, int32_t& b) {
  a = dpp_max_step<0x111, 0xF>(a);
  b = dpp_max_step<0x111, 0xF>(b);
  a = dpp_max_step<0x112, 0xF>(a);
  b = dpp_max_step<0x112, 0xF>(b);
  a = dpp_max_step<0x114, 0xF>(a);
  b = dpp_max_step<0x114, 0xF>(b);
  a = dpp_max_step<0x118, 0xF>(a);
  b = dpp_max_step<0x118, 0xF>(b);
  a = dpp_max_step<0x142, 0xA>(a);
  b = dpp_max_step<0x142, 0xA>(b);
  a = dpp_max_step<0x143, 0xC>(a);
  b = dpp_max_step<0x143, 0xC>(b);
}

// lane l <- x[l-1]; lane 0 <- fill (wave-uniform).  DPP wave_shr:1.
__device__ __forceinline__ int32_t wave_shr1(int32_t x, int32_t fill, int /*lane*/) {
  return __builtin_amdgcn_update_dpp(fill, x, 0x138, 0xF, 0xF, false);
}

__device__ __forceinline__ int32_t readlane63(int32_t x) {
  return __builtin_amdgcn_readlane(x, 63);
}

// Row-0 (virtual source row) values, spoa Initialize for kNW convex.
__device__ __forceinline__ int32_t row0_e(const PoaScore& P, int32_t j) { return j == 0 ? 0 : P.g + (j - 1) * P.e; }
__device__ __forceinline__ int32_t row0_q(const PoaScore& P, int32_t j) { return j == 0 ? 0 : P.q + (j - 1) * P.c; }
__device__ __forceinline__ int32_t row0_h(const PoaScore& P, int32_t j) {
  return j == 0 ? 0 : imax(row0_q(P, j), row0_e(P, j));
}

// Cross-strip state of one row sweep (all wave-uniform scalars).
struct StripCarry {
  int32_t run1, run2;  // running maxima of the Q / E scan terms over earlier columns
  int32_t cHpre, cQ, cE, cH;  // Hpre, Q, E, H at the previous strip's last column
};

// Horizontal-gap scans of one 64-column strip.  Both prefix scans depend only
// on this strip's Hpre (not on earlier strips), so the long DPP chains of
// strip s+1 can overlap strip s; earlier strips enter through a few scalar
// maxima (exact for e <= c, checked on host):
//   P1[j] = max_{j0<=k<=j} (Hpre[k-1] + q - k c)
//   Q[j]  = j c + max(P1[j], run1)
//   P2[j] = max_{j0<=k<=j} (max(Hpre[k-1], Qloc[k-1]) + g - k e),  Qloc[k-1] = (k-1) c + P1[k-1]
//   E[j]  = j e + max(P2[j], run2, cQ + g - j0 e, run1 + (j-1) c + g - j e)
__device__ __forceinline__ void strip_gaps(const PoaScore& P, int lane, int32_t j, int32_t j0, bool inner,
                                           int32_t Hpre, int32_t H0, StripCarry& cr, int32_t& Q, int32_t& E,
                                           int32_t& H, int32_t& prevQ, int32_t& prevE, int32_t& prevH) {
  const int32_t pH = wave_shr1(Hpre, cr.cHpre, lane);
  int32_t p1 = inner ? pH + P.q - j * P.c : SVS_VNEG;
  p1 = wave_prefix_max(p1);
  const int32_t p1m = wave_shr1(p1, SVS_VNEG, lane);
  int32_t p2 = inner ? imax(pH, p1m + (j - 1) * P.c) + P.g - j * P.e : SVS_VNEG;
  p2 = wave_prefix_max(p2);
  const int32_t T1 = j0 > 0 ? cr.cQ + P.g - j0 * P.e : SVS_VNEG;
  const int32_t T2 = lane > 0 ? cr.run1 + (j - 1) * P.c + P.g - j * P.e : SVS_VNEG;
  Q = inner ? j * P.c + imax(p1, cr.run1) : SVS_NEG_INF;
  E = inner ? j * P.e + imax(imax(p2, cr.run2), imax(T1, T2)) : SVS_NEG_INF;
  H = inner ? imax(Hpre, imax(E, Q)) : H0;
  prevQ = wave_shr1(Q, cr.cQ, lane);
  prevE = wave_shr1(E, cr.cE, lane);
  prevH = wave_shr1(H, cr.cH, lane);
  // carries for the next strip, from carry-free lane-63 values
  const int32_t jl = j0 + 63;
  const int32_t p1l = readlane63(p1), p2l = readlane63(p2), hl = readlane63(Hpre);
  const int32_t T2l = cr.run1 + (jl - 1) * P.c + P.g - jl * P.e;
  cr.run2 = imax(imax(cr.run2, p2l), imax(T1, T2l));
  cr.run1 = imax(cr.run1, p1l);
  cr.cQ = jl * P.c + cr.run1;
  cr.cE = jl * P.e + cr.run2;
  cr.cHpre = hl;
  cr.cH = imax(hl, imax(cr.cE, cr.cQ));
}

// Traceback code of one DP cell (the strip kernel writes one per evaluated
// cell, the backtrack below reads nothing else).  Narrow (uint16, graphs
// whose nodes have at most 31 in-edges):
//   bits 0-1  main move: 0 diagonal, 1 up, 2 left, 3 none
//   bit  2    extend flag of the main move (extend_up / extend_left)
//   bits 3-7  in-edge index of the main move (diag/up)
//   bit  8    left-gap run opened here:  H[j-1]+g==E[j] || H[j-1]+q==Q[j]
//   bit  9    up-gap run stop flag
//   bits 10-14 in-edge index continuing an up-gap run (31 = none)
// Wide (uint32, up to 4094 in-edges: large windows): in-edge indices of 12
// bits at 3-14 and 17-28 (4095 = none), the flags at bits 15 and 16.
template <class CodeT> struct TbFmt;
template <> struct TbFmt<uint16_t> {
  static constexpr uint32_t kMask = 31, kLBit = 8, kStop = 9, kUc = 10, kMaxPreds = 31;
};
template <> struct TbFmt<uint32_t> {
  static constexpr uint32_t kMask = 4095, kLBit = 15, kStop = 16, kUc = 17, kMaxPreds = 4094;
};

// Assembly from the per-in-edge tests (branch-free selects); kMask = none.
template <class F>
__device__ __forceinline__ uint32_t assemble_code(uint32_t diag_k, uint32_t up_k, uint32_t up_ext, bool left_ok,
                                                  bool left_ext, bool lbit, uint32_t uc_k, uint32_t uc_stop) {
  const uint32_t left = left_ok ? (2u | (left_ext ? 4u : 0u)) : 3u;
  const uint32_t up = 1u | (up_ext << 2) | (up_k << 3);
  uint32_t code = up_k != F::kMask ? up : left;
  code = diag_k != F::kMask ? (diag_k << 3) : code;
  return code | ((lbit ? 1u : 0u) << F::kLBit) | (uc_stop << F::kStop) | (uc_k << F::kUc);
}

// Lane-0 traceback (spoa SisdAlignmentEngine backtrack order, kNW convex)
// from (best_row, L) to (0, 0); writes (row, pos) pairs in reverse into out.
// tbc(row, col): traceback code of DP cell (row >= 1); pred_of(row, k): 1-based
// DP row of in-edge k of row `row` (0 = virtual row 0); emit(n, a, b) stores
// pair n.  Returns the pair count, or -1 for an inconsistent path.  Control
// flow depends only on its arguments and on tbc / pred_of results, so a whole
// wave may run it in lockstep (the strip kernel's tile-cached codes).
template <class F, class Tbc, class PredOf, class Emit>
__device__ int32_t poa_traceback(const PoaScore& P, uint32_t V, int32_t L, int32_t best_row, Tbc tbc,
                                 PredOf pred_of, Emit emit) {
  const int64_t cap = static_cast<int64_t>(V) + L + 1;
  int64_t n = 0;
  int32_t i = best_row, jj = L;
  bool ok = best_row > 0 || V == 0;
  while (ok && !(i == 0 && jj == 0)) {
    int32_t pi = i, pj = jj;
    bool el = false, eu = false;
    if (i == 0) {
      const int32_t Hij = row0_h(P, jj);
      const bool a = Hij == row0_e(P, jj - 1) + P.e, b = Hij == row0_h(P, jj - 1) + P.g;
      const bool c = Hij == row0_q(P, jj - 1) + P.c, d = Hij == row0_h(P, jj - 1) + P.q;
      if (!(a || b || c || d)) { ok = false; break; }
      el = a || (!b && c);
      pj = jj - 1;
    } else {
      const uint32_t code = tbc(i, jj);
      const uint32_t t = code & 3u, k = (code >> 3) & F::kMask;
      if (t == 0) { pi = pred_of(i, k); pj = jj - 1; }
      else if (t == 1) { pi = pred_of(i, k); eu = (code >> 2) & 1u; }
      else if (t == 2) { pj = jj - 1; el = (code >> 2) & 1u; }
      else { ok = false; break; }
    }
    if (n >= cap) { ok = false; break; }
    emit(n, (pi == i) ? -1 : i - 1, (pj == jj) ? -1 : jj - 1);
    ++n;
    i = pi;
    jj = pj;
    if (el) {
      while (true) {
        if (n >= cap || jj <= 0) { ok = false; break; }
        emit(n, -1, jj - 1);
        ++n;
        --jj;
        bool stop;
        if (i == 0) {
          stop = row0_h(P, jj) + P.g == row0_e(P, jj + 1) || row0_h(P, jj) + P.q == row0_q(P, jj + 1);
        } else {
          stop = (tbc(i, jj + 1) >> F::kLBit) & 1u;
        }
        if (stop) break;
      }
    } else if (eu) {
      while (true) {
        if (n >= cap || i <= 0) { ok = false; break; }
        const uint32_t code = tbc(i, jj);
        const uint32_t k = (code >> F::kUc) & F::kMask;
        const bool stop = (code >> F::kStop) & 1u;
        const int32_t nxt = (k == F::kMask) ? 0 : pred_of(i, k);
        emit(n, i - 1, -1);
        ++n;
        i = nxt;
        if (stop || i == 0) break;
      }
    }
  }
  return ok ? static_cast<int32_t>(n) : -1;
}

}  // namespace svs
