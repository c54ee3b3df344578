// MI355X (gfx950) POA alignment kernel: Needleman-Wunsch of one read against a
// partial-order graph with spoa's convex gap model, plus traceback, for a
// batch of independent (window, read) jobs.
//
// Replaces the DP + backtrack of spoa's SisdAlignmentEngine (kNW, convex),
// reached by the reference through `poa(seqs, 1)` at
// /root/reference/src/DataScanner.py:206,213 and DecisionMaker.py:160,171.
//
// Mapping (CDNA4-first, not a translation of spoa's SIMD engine):
//  * one 64-lane wave per job; four independent jobs per 256-thread block;
//  * graph rows in topological rank order; each row is swept in strips of 64
//    columns, lane l owning column 64*s + l, so every pool/traceback access is
//    a coalesced 256-B (int32) / 128-B (uint16) wave access;
//  * the sequential horizontal recurrences E (g,e) and Q (q,c) are rewritten
//    as two wave-wide prefix-max scans (DPP row_shr + row_bcast), exact for
//    parameters satisfying g<=e, q<=c, g<=c, e<=c, g+q<=2c (checked on host):
//        Q[j] = j*c + max_{k<=j} (Hpre[k-1] + q - k*c)
//        E[j] = j*e + max_{k<=j} (max(Hpre,Q)[k-1] + g - k*e)
//    where Hpre = max(diagonal, F, O) over all in-edges;
//  * H/F/O rows live in a small per-job row pool (slots recycled by the host
//    planner once a row's last successor is done) instead of full matrices;
//  * per cell only a 16-bit traceback code is written to HBM: it records the
//    outcome of every comparison spoa's backtrack makes at that cell, so the
//    backtrack replays spoa's exact tie-break order without the score planes.
//
// Traceback code layout (uint16):
//   bits 0-1  main move: 0 diagonal, 1 up, 2 left, 3 none
//   bit  2    extend flag of the main move (extend_up / extend_left)
//   bits 3-7  in-edge index of the main move (diag/up)
//   bit  8    left-gap run opened here:  H[j-1]+g==E[j] || H[j-1]+q==Q[j]
//   bit  9    up-gap run stop flag
//   bits 10-14 in-edge index continuing an up-gap run (31 = none)
#include <hip/hip_runtime.h>
#include <cstdint>
#include <type_traits>

#include "poa_wave.hpp"
#include "svs_device.hpp"

namespace svs {

constexpr int kRing = 8;        // carry ring depth between column-chunk waves
constexpr int kMaxSlots = 64;   // row-pool slots tracked in LDS (host checks)
constexpr long kSpinLimit = 1l << 26;

// Per-job LDS state when WPJ waves share one job (WPJ > 1).
struct JobLds {
  StripCarry ring[3][kRing];   // wave w -> w+1: carries after w's chunk, per row
  int32_t done[4];             // rows whose carry wave w has published
  int32_t cons[4];             // rows whose carry wave w has consumed
  int32_t bnd[4][kMaxSlots];   // per pool slot: H at column 64*sb(w) - 1 (owned by wave w-1)
  int32_t best[4], best_row[4];
  int32_t err;
};

__device__ __forceinline__ int32_t lds_acquire(int32_t* p) {
  return __builtin_amdgcn_readfirstlane(__hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP));
}
__device__ __forceinline__ void lds_release(int32_t* p, int32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// Bounded wait until *p >= target; sets *err and gives up after kSpinLimit polls.
__device__ __forceinline__ void lds_wait_ge(int32_t* p, int32_t target, int32_t* err) {
  long n = 0;
  while (lds_acquire(p) < target) {
    __builtin_amdgcn_s_sleep(1);
    if (++n > kSpinLimit) { __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); return; }
  }
}

// One job = one read against one graph, swept by WPJ waves of a 256-thread
// block: wave `sub` owns strips [sb, se) of every row.  Row r of wave sub
// starts once wave sub-1 has published its carries for row r, so the waves of
// a job run as a row-skewed pipeline; pool columns and traceback codes are
// private to their wave, and the one value read across a chunk boundary,
// H[pred][64*sb-1], is kept per pool slot in LDS.
template <int WPJ>
__global__ __launch_bounds__(256) void poa_nw_convex_kernel(
    const PoaJob* __restrict__ jobs, int n_jobs, PoaScore P,
    const uint32_t* __restrict__ row_info, const uint32_t* __restrict__ row_slot,
    const uint32_t* __restrict__ row_pstart, const uint32_t* __restrict__ pred_row,
    const uint32_t* __restrict__ pred_slot, const int32_t* __restrict__ col0,
    const uint8_t* __restrict__ seqs, uint16_t* __restrict__ tb, int32_t* __restrict__ pool,
    int32_t* __restrict__ aln, int32_t* __restrict__ aln_len) {
  constexpr int JPB = 4 / WPJ;  // jobs per block
  __shared__ JobLds lds_all[WPJ > 1 ? JPB : 1];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int sub = wave % WPJ;
  JobLds& S = lds_all[WPJ > 1 ? wave / WPJ : 0];
  const int job_id = __builtin_amdgcn_readfirstlane(blockIdx.x * JPB + wave / WPJ);
  const bool active = job_id < n_jobs;
  PoaJob J{};
  if (active) J = jobs[job_id];
  const int32_t L = static_cast<int32_t>(J.len);
  const uint64_t LS = J.ls;
  const uint32_t V = J.n_rows;
  const uint8_t* __restrict__ seq = seqs + J.seq_off;
  int32_t* __restrict__ pl = pool + J.pool_off;
  uint16_t* __restrict__ tbj = tb + J.tb_off;
  const uint32_t* __restrict__ rinfo = row_info + J.row_off;
  const uint32_t* __restrict__ rslot = row_slot + J.row_off;
  const int32_t* __restrict__ rc0 = col0 + 3ull * J.row_off;
  const uint32_t* __restrict__ rps = row_pstart + J.pstart_off;
  const uint32_t* __restrict__ prow = pred_row + J.pred_off;
  const uint32_t* __restrict__ pslot = pred_slot + J.pred_off;
  const int32_t nstrips = static_cast<int32_t>(LS >> 6);  // LS = 64 * ceil((L+1)/64)
  const int32_t chunk = (nstrips + WPJ - 1) / WPJ;
  const int32_t sb = min(nstrips, sub * chunk), se = min(nstrips, sb + chunk);
  const __amdgpu_buffer_rsrc_t pool_rsrc =
      __builtin_amdgcn_make_buffer_rsrc(pl, 0, static_cast<int32_t>(J.n_slots * 3u * J.ls * 4u), 0x00020000);
  const __amdgpu_buffer_rsrc_t tb_rsrc = __builtin_amdgcn_make_buffer_rsrc(
      tbj, 0, static_cast<int32_t>(static_cast<uint64_t>(V) * J.ls * 2u), 0x00020000);
  // seq_rsrc byte offset b addresses seq[b - 1] (the zero pad byte precedes the read)
  const __amdgpu_buffer_rsrc_t seq_rsrc =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(seq) - 1, 0, static_cast<int32_t>(J.ls + 1), 0x00020000);
  const uint32_t lane4 = static_cast<uint32_t>(lane) * 4u, lane2 = static_cast<uint32_t>(lane) * 2u;
  const uint32_t LS4 = static_cast<uint32_t>(LS) * 4u;

  if (active) {
    // virtual row 0 -> slot 0 (planes H, F, O at offsets 0, LS, 2LS), own columns
    for (int32_t j = sb * 64 + lane; j < se * 64; j += 64) {
      pl[j] = row0_h(P, j);
      pl[LS + j] = j == 0 ? 0 : SVS_NEG_INF;
      pl[2 * LS + j] = j == 0 ? 0 : SVS_NEG_INF;
    }
  }
  if (WPJ > 1) {
    if (lane == 0) {
      S.done[sub] = 0;
      S.cons[sub] = 0;
      if (sub > 0) S.bnd[sub][0] = row0_h(P, sb * 64 - 1);
      if (sub == 0) S.err = 0;
      S.best[sub] = SVS_NEG_INF;
      S.best_row[sub] = 0;
    }
    __syncthreads();
  }

  int32_t best = SVS_NEG_INF;  // meaningful on the lane owning column L
  int32_t best_row = 0;

  for (uint32_t r = 0; active && r < V; ++r) {
    const uint32_t info = rinfo[r];
    const uint8_t nb = static_cast<uint8_t>(info & 0xFF);
    const bool sink = (info >> 8) & 1;
    const uint32_t rs = rslot[r];
    const uint64_t so = static_cast<uint64_t>(rs) * 3 * LS;
    const uint32_t p0 = rps[r];
    const uint32_t np = rps[r + 1] - p0;
    const int32_t H0 = rc0[3 * r], F0 = rc0[3 * r + 1], O0 = rc0[3 * r + 2];

    StripCarry cr{SVS_VNEG, SVS_VNEG, H0, SVS_NEG_INF, SVS_NEG_INF, H0};
    if (WPJ > 1 && sub > 0) {
      lds_wait_ge(&S.done[sub - 1], static_cast<int32_t>(r) + 1, &S.err);
      const StripCarry& in = S.ring[sub - 1][r % kRing];
      cr.run1 = __builtin_amdgcn_readfirstlane(in.run1);
      cr.run2 = __builtin_amdgcn_readfirstlane(in.run2);
      cr.cHpre = __builtin_amdgcn_readfirstlane(in.cHpre);
      cr.cQ = __builtin_amdgcn_readfirstlane(in.cQ);
      cr.cE = __builtin_amdgcn_readfirstlane(in.cE);
      cr.cH = __builtin_amdgcn_readfirstlane(in.cH);
      if (lane == 0) {
        lds_release(&S.cons[sub], static_cast<int32_t>(r) + 1);
        S.bnd[sub][rs] = cr.cH;  // H[r][64*sb - 1] for later successors of r
      }
    }

    if (np <= 1 && sb < se) {
      // ---- fast path: zero or one in-edge (the common POA row) ----
      // Three statically named load sets (loop unrolled x3): set k holds strip
      // s and is reloaded with strip s+3 right after its last use, so no waits
      // on loads in flight.  Buffer loads past a buffer end return 0.
      const uint32_t ps = np == 0 ? 0u : pslot[p0];
      const uint32_t ps4 = ps * 3u * static_cast<uint32_t>(LS) * 4u;
      struct Ld { int32_t hp, fp, op; uint8_t rc; };
      auto load = [&](Ld& d, int32_t st) {
        const uint32_t o4 = static_cast<uint32_t>(st) << 8;
        d.hp = __builtin_amdgcn_raw_buffer_load_b32(pool_rsrc, lane4, ps4 + o4, 0);
        d.fp = __builtin_amdgcn_raw_buffer_load_b32(pool_rsrc, lane4, ps4 + LS4 + o4, 0);
        d.op = __builtin_amdgcn_raw_buffer_load_b32(pool_rsrc, lane4, ps4 + 2 * LS4 + o4, 0);
        d.rc = __builtin_amdgcn_raw_buffer_load_b8(seq_rsrc, static_cast<uint32_t>(lane),
                                                   static_cast<uint32_t>(st) << 6, 0);
      };
      // chunk starting at strip 0: strip 0 (masks for column 0 / validity) runs
      // first from its own load set Z; the unrolled loop then always starts at A
      const int32_t s1 = sb == 0 ? 1 : sb;
      Ld Z, A, B, C;
      if (sb == 0) load(Z, 0);
      load(A, s1);
      load(B, s1 + 1);
      load(C, s1 + 2);
      int32_t cHp = (WPJ > 1 && sub > 0) ? S.bnd[sub][ps] : 0;
      if (WPJ > 1) cHp = __builtin_amdgcn_readfirstlane(cHp);
      const uint32_t so4 = static_cast<uint32_t>(so) * 4u;
      const uint32_t tro2 = r * static_cast<uint32_t>(LS) * 2u;
      auto step = [&](auto first_tag, int32_t s, Ld& d) {
        constexpr bool FIRST = decltype(first_tag)::value;
        const int32_t j0 = s << 6;
        const int32_t j = j0 + lane;
        // strips >= 1 need no masks: lanes past L compute row padding that
        // no valid column ever reads (scans only propagate towards higher j)
        const bool c0 = FIRST && lane == 0;
        const bool inner = FIRST ? (lane != 0 && j <= L) : true;
        const int32_t hp = d.hp, fp = d.fp, op = d.op;
        const int32_t hpm = wave_shr1(hp, cHp, lane);
        const int32_t mc = d.rc == nb ? P.m : P.n;
        int32_t F = imax(hp + P.g, fp + P.e);
        int32_t O = imax(hp + P.q, op + P.c);
        int32_t Hpre = imax(hpm + mc, imax(F, O));
        if (FIRST) {
          F = c0 ? F0 : F;
          O = c0 ? O0 : O;
          Hpre = c0 ? H0 : Hpre;
        }
        int32_t Q, E, H, prevQ, prevE, prevH;
        strip_gaps(P, lane, j, j0, inner, Hpre, H0, cr, Q, E, H, prevQ, prevE, prevH);

        const bool dg = inner && H == hpm + mc;
        const bool ua = H == fp + P.e, ub = H == hp + P.g, uc = H == op + P.c, ud = H == hp + P.q;
        const bool va = F == hp + P.g, vb = F == fp + P.e, vc = O == hp + P.q, vd = O == op + P.c;
        const bool vm = np != 0 && (va || vb || vc || vd);
        const bool la = inner && H == prevE + P.e, lb = inner && H == prevH + P.g;
        const bool lc = inner && H == prevQ + P.c, ld = inner && H == prevH + P.q;
        const bool lbit = inner && (prevH + P.g == E || prevH + P.q == Q);
        const uint32_t code =
            assemble_code(dg ? 0u : 31u, (ua || ub || uc || ud) ? 0u : 31u, (ua || (!ub && uc)) ? 1u : 0u,
                          la || lb || lc || ld, la || (!lb && lc), lbit, vm ? 0u : 31u,
                          (vm && (va || (!vb && vc))) ? 1u : 0u);
        cHp = readlane63(hp);
        load(d, s + 3);
        const uint32_t j04 = static_cast<uint32_t>(j0) * 4u;
        __builtin_amdgcn_raw_buffer_store_b16(static_cast<uint16_t>(code), tb_rsrc, lane2,
                                              tro2 + static_cast<uint32_t>(j0) * 2u, 0);
        __builtin_amdgcn_raw_buffer_store_b32(H, pool_rsrc, lane4, so4 + j04, 0);
        __builtin_amdgcn_raw_buffer_store_b32(F, pool_rsrc, lane4, so4 + LS4 + j04, 0);
        __builtin_amdgcn_raw_buffer_store_b32(O, pool_rsrc, lane4, so4 + 2 * LS4 + j04, 0);
        if (sink && j == L && H > best) { best = H; best_row = static_cast<int32_t>(r) + 1; }
      };
      using TrueT = std::integral_constant<bool, true>;
      using FalseT = std::integral_constant<bool, false>;
      if (sb == 0) step(TrueT{}, 0, Z);
      for (int32_t s = s1; s < se; s += 3) {
        step(FalseT{}, s, A);
        if (s + 1 >= se) break;
        step(FalseT{}, s + 1, B);
        if (s + 2 >= se) break;
        step(FalseT{}, s + 2, C);
      }
    } else if (sb < se) {
      // ---- general path: two or more in-edges ----
      for (int32_t s = sb; s < se; ++s) {
        const int32_t j = (s << 6) + lane;
        const bool valid = j <= L;
        const bool c0 = j == 0;
        const bool inner = valid && !c0;
        const bool edge = WPJ > 1 && s == sb && sb > 0 && lane == 0;  // H[p][j-1] owned by wave sub-1
        const int32_t mc = (inner && seq[j - 1] == nb) ? P.m : P.n;

        int32_t F = SVS_VNEG, O = SVS_VNEG, Hd = SVS_VNEG;
        int32_t hpm0 = 0, hp0 = 0, fp0 = 0, op0 = 0;  // first in-edge kept in registers
        for (uint32_t k = 0; k < np; ++k) {
          const uint32_t psk = pslot[p0 + k];
          const uint64_t ps = static_cast<uint64_t>(psk) * 3 * LS;
          const int32_t hpm = c0 ? 0 : (edge ? S.bnd[sub][psk] : pl[ps + j - 1]);
          const int32_t hp = pl[ps + j];
          const int32_t fp = pl[ps + LS + j];
          const int32_t op = pl[ps + 2 * LS + j];
          if (k == 0) { hpm0 = hpm; hp0 = hp; fp0 = fp; op0 = op; }
          F = imax(F, imax(hp + P.g, fp + P.e));
          O = imax(O, imax(hp + P.q, op + P.c));
          Hd = imax(Hd, hpm + mc);
        }
        if (c0) { F = F0; O = O0; }
        const int32_t Hpre = c0 ? H0 : imax(Hd, imax(F, O));
        int32_t Q, E, H, prevQ, prevE, prevH;
        strip_gaps(P, lane, j, s << 6, inner, Hpre, H0, cr, Q, E, H, prevQ, prevE, prevH);

        uint32_t diag_k = 31, up_k = 31, up_ext = 0, uc_k = 31, uc_stop = 0;
        for (uint32_t k = 0; k < np; ++k) {
          int32_t hpm, hp, fp, op;
          if (k == 0) {
            hpm = hpm0; hp = hp0; fp = fp0; op = op0;
          } else {
            const uint32_t psk = pslot[p0 + k];
            const uint64_t ps = static_cast<uint64_t>(psk) * 3 * LS;
            hpm = c0 ? 0 : (edge ? S.bnd[sub][psk] : pl[ps + j - 1]);
            hp = pl[ps + j];
            fp = pl[ps + LS + j];
            op = pl[ps + 2 * LS + j];
          }
          if (inner && diag_k == 31 && H == hpm + mc) diag_k = k;
          if (up_k == 31) {
            const bool a = H == fp + P.e, b = H == hp + P.g, c = H == op + P.c, d = H == hp + P.q;
            if (a || b || c || d) { up_k = k; up_ext = (a || (!b && c)) ? 1u : 0u; }
          }
          if (uc_k == 31) {
            const bool a = F == hp + P.g, b = F == fp + P.e, c = O == hp + P.q, d = O == op + P.c;
            if (a || b || c || d) { uc_k = k; uc_stop = (a || (!b && c)) ? 1u : 0u; }
          }
        }
        const bool la = inner && H == prevE + P.e, lb = inner && H == prevH + P.g;
        const bool lc = inner && H == prevQ + P.c, ld = inner && H == prevH + P.q;
        const bool lbit = inner && (prevH + P.g == E || prevH + P.q == Q);
        const uint32_t code = assemble_code(diag_k, up_k, up_ext, la || lb || lc || ld, la || (!lb && lc), lbit, uc_k,
                                            uc_stop);
        if (valid) tbj[static_cast<uint64_t>(r) * LS + j] = static_cast<uint16_t>(code);
        pl[so + j] = H;
        pl[so + LS + j] = F;
        pl[so + 2 * LS + j] = O;
        if (sink && j == L && H > best) { best = H; best_row = static_cast<int32_t>(r) + 1; }
      }
    }

    if (WPJ > 1 && sub < WPJ - 1) {
      // publish this row's carries once the consumer has freed the ring slot
      lds_wait_ge(&S.cons[sub + 1], static_cast<int32_t>(r) + 1 - kRing, &S.err);
      if (lane == 0) {
        StripCarry& out = S.ring[sub][r % kRing];
        out = cr;
        lds_release(&S.done[sub], static_cast<int32_t>(r) + 1);
      }
    }
  }

  if (WPJ > 1) {
    // gather the sink maximum (lane owning column L of the owning wave) and
    // make every wave's traceback codes visible to wave 0
    const int owner_lane = L & 63;
    const int32_t b = __shfl(best, owner_lane, 64), br = __shfl(best_row, owner_lane, 64);
    if (lane == 0 && sb * 64 <= L && L < se * 64) {
      S.best[sub] = b;
      S.best_row[sub] = br;
    }
    __syncthreads();
    if (!active || sub != 0) return;
    int32_t bb = SVS_NEG_INF, bbr = 0;
    for (int w = 0; w < WPJ; ++w)
      if (S.best_row[w] != 0) { bb = S.best[w]; bbr = S.best_row[w]; }
    (void)bb;
    best_row = bbr;
    if (S.err) {
      if (lane == 0) aln_len[job_id] = -1;
      return;
    }
  } else {
    if (!active) return;
  }

  if (WPJ == 1) {
    // Make the wave's traceback-code stores visible to its own lane 0.
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    best_row = __shfl(best_row, L & 63, 64);
  }
  if (lane != 0) return;

  // ---- traceback (spoa backtrack order), lane 0 ----
  auto tbc = [&](int32_t row, int32_t col) -> uint32_t { return tbj[static_cast<uint64_t>(row - 1) * LS + col]; };
  auto pred_of = [&](int32_t row, uint32_t k) -> int32_t {
    const uint32_t a = rps[row - 1], b = rps[row];
    return (b == a) ? 0 : static_cast<int32_t>(prow[a + k]);
  };
  int32_t* __restrict__ out = aln + 2 * J.aln_off;
  auto emit = [&](int64_t n, int32_t a, int32_t b) {
    out[2 * n] = a;
    out[2 * n + 1] = b;
  };
  aln_len[job_id] = poa_traceback(P, V, L, best_row, tbc, pred_of, emit);
}

hipError_t launch_poa_nw_convex(const PoaLaunch& a, hipStream_t stream) {
  if (a.n_jobs <= 0) return hipSuccess;
  const int wpj = a.waves_per_job;
  const int jpb = 4 / wpj;
  const int blocks = (a.n_jobs + jpb - 1) / jpb;
#define SVS_LAUNCH(W)                                                                                     \
  hipLaunchKernelGGL(poa_nw_convex_kernel<W>, dim3(blocks), dim3(256), 0, stream, a.jobs, a.n_jobs, a.score, \
                     a.row_info, a.row_slot, a.row_pstart, a.pred_row, a.pred_slot, a.col0, a.seqs, a.tb,     \
                     a.pool, a.aln, a.aln_len)
  if (wpj == 4) SVS_LAUNCH(4);
  else if (wpj == 2) SVS_LAUNCH(2);
  else SVS_LAUNCH(1);
#undef SVS_LAUNCH
  return hipGetLastError();
}

// ---- self-test kernels for the wave primitives (used by the GPU tests) ----
__global__ void wave_scan_selftest_kernel(const int32_t* in, int32_t* out_scan, int32_t* out_shift) {
  const int lane = threadIdx.x & 63;
  const int32_t x = in[blockIdx.x * 64 + lane];
  out_scan[blockIdx.x * 64 + lane] = wave_prefix_max(x);
  out_shift[blockIdx.x * 64 + lane] = wave_shr1(x, -7, lane);
}

hipError_t launch_wave_selftest(const int32_t* in, int32_t* scan, int32_t* shift, int n_waves,
                                hipStream_t stream) {
  hipLaunchKernelGGL(wave_scan_selftest_kernel, dim3(n_waves), dim3(64), 0, stream, in, scan, shift);
  return hipGetLastError();
}

}  // namespace svs
