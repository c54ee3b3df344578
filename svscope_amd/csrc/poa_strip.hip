// MI355X (gfx950) POA alignment kernel, strip-major: Needleman-Wunsch of one
// read against a partial-order graph with spoa's convex gap model, plus the
// traceback, for a batch of independent (graph, read) jobs.
//
// Replaces the DP + backtrack of spoa's SisdAlignmentEngine (kNW, convex)
// reached by the reference through `poa(seqs, 1)` at
// /root/reference/src/DataScanner.py:206,213 and DecisionMaker.py:160,171.
//
// Mapping (one job = one workgroup of WPJ waves, WPJ in 1..8):
//  * the DP matrix is swept strip by strip: strip s = columns 64s .. 64s+63,
//    lane l owning column 64s + l; within a strip all graph rows are visited in
//    rank order;
//  * the row pool (H, F, O of rows that a later, non-adjacent row still reads)
//    only spans the current strip, so it lives in LDS: n_slots x 768 B per
//    wave (config-3 windows need <= 13 slots); an in-edge from the row just
//    above is served from registers and that row is not stored at all when no
//    other row reads it (export_strip_rows plans slots and liveness);
//  * the only state carried from strip s-1 to strip s is per row: the two
//    scan carries, Hpre and H at the strip's last column (16 B), written once
//    by lane 0 and read back as a uniform load by the wave sweeping strip s,
//    prefetched two rows ahead; row records (16 B) are prefetched the same
//    way.  With WPJ > 1 the waves of a job sweep consecutive strips as a
//    row-skewed pipeline (LDS progress counters);
//  * per cell only the 16-bit traceback code goes to HBM (coalesced 128 B per
//    strip row); the backtrack is the same lane-0 replay of spoa's order as in
//    the row-major kernel (poa_wave.hpp).
// HBM traffic per DP cell: 2 B traceback + ~0.5 B carries (vs ~25 B for the
// row-major kernel's global pool), and no global load on the row-to-row
// dependency chain.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <algorithm>
#include <type_traits>
#include <cstdio>
#include <vector>

#include "poa_graph.hpp"
#include "poa_wave.hpp"
#include "svs_device.hpp"

namespace svs {

namespace {

// Global-memory (address space 1) views of the job's tables: loads through
// them are global_load (vmcnt only) instead of flat loads, which also count in
// lgkmcnt and so made every LDS-pool wait of a row wait for the carries
// prefetched for a later row as well.
#define GLB __attribute__((address_space(1)))
template <class T> __device__ __forceinline__ const GLB T* glb(const T* p) { return (const GLB T*)(p); }
// The job's row tables (records, in-edges, column 0) are written by earlier
// kernels and only read here: through the constant address space, a load at a
// wave-uniform address is a scalar load straight into SGPRs (no vector load,
// no v_readfirstlane per word), which the compiler cannot prove for pointers
// it reads from the job descriptor.  SVS_TABLES_GLOBAL=1 (development builds)
// keeps them global.
#ifndef SVS_TABLES_GLOBAL
#define TBL __attribute__((address_space(4)))
#else
#define TBL GLB
#endif
template <class T> __device__ __forceinline__ const TBL T* tbl(const T* p) { return (const TBL T*)(p); }

// One pool slot: 65 int32 Hx = H at columns j0-1 .. j0+63 (so a successor
// reads H[j] at Hx[l+1] and its diagonal H[j-1] at Hx[l], with no lane shift),
// then 64 uint16 D = dF | dO << 8 with dF = min(H - F, tF), dO = min(H - O, tO)
// (see pack_fo).
constexpr int kSlotInts = 65 + 32;
static_assert(kSlotInts * 4 == kStripSlotBytes, "pool slot size");

// F and O enter the recurrence only through F + e (against H + g) and O + c
// (against H + q), and F, O <= H.  So F matters only while H - F <= e - g and
// O only while H - O <= c - q; storing the distance to H clamped at
// tF = e - g + 1 and tO = c - q + 1 keeps every max and every equality test of
// the recurrence and the traceback codes exact (a clamped F' = H - tF gives
// F' + e = H + g - 1, below the H + g it is compared with, just like the true
// F).  Halves the pool in LDS, so twice the waves fit on a CU.
//
// The clamp itself is 255 (one literal operand, no SGPR): any clamp T >= tF
// keeps F' + e < H + g (tF, tO <= 255 host-checked), and below it the stored
// distance is the true one.
__device__ __forceinline__ uint32_t pack_fo(int32_t H, int32_t F, int32_t O) {
  const uint32_t dF = min(static_cast<uint32_t>(H) - static_cast<uint32_t>(F), 255u);
  const uint32_t dO = min(static_cast<uint32_t>(H) - static_cast<uint32_t>(O), 255u);
  return dF | (dO << 8);
}

// d = (lane > 0 ? a[lane-1] : d) + b, one DPP-combined VALU op (wave_shr:1
// leaves lane 0 unwritten; the caller preloads d with lane 0's value).  Kept
// in asm: the builtin form needs a separate move of d into the destination
// (update_dpp's "old" is not the identity of the add), one VALU more per call.
__device__ __forceinline__ int32_t shr1_add(int32_t d, int32_t a, int32_t b) {
  asm volatile("s_nop 1\n\tv_add_u32_dpp %0, %1, %2 wave_shr:1 row_mask:0xf bank_mask:0xf" : "+v"(d) : "v"(a), "v"(b));
  return d;
}
// d = (lane > 0 ? a[lane-1] : 0) + b: wave_shr:1 with bound_ctrl (lane 0
// reads zero), which the compiler folds into one v_add_u32_dpp.
__device__ __forceinline__ int32_t shr1_add_bc(int32_t a, int32_t b) {
  return __builtin_amdgcn_update_dpp(0, a, 0x138, 0xF, 0xF, true) + b;
}

// Lane constants of one strip (columns j = j0 + lane, j0 > 0) for the
// horizontal-gap scans of strip_gaps_nf.
struct StripConst {
  int32_t qjc;  // q - j c
  int32_t k1;   // (g - j e) - (q - j c)
  int32_t k2;   // (j-1) c + g - j e; lane 0: VNEG + that
  int32_t t2b;  // (j-1) c + g - j e; lane 0: VNEG
  int32_t jc, je, ve, vc;
};

typedef int32_t svs_i32x4 __attribute__((ext_vector_type(4)));

struct GapOut {
  int32_t Q, E, H, prevH, prevEe, prevQc;  // prevEe = E[j-1] + e, prevQc = Q[j-1] + c
};

// strip_gaps (poa_wave.hpp) for a strip after the first: every lane is an
// inner column, and the lane shifts that feed an addition are DPP-combined
// adds (P1's input Hpre[j-1] + q - jc, P2's P1[j-1] + (j-1)c + g - je, and the
// E[j-1] + e / Q[j-1] + c terms of the traceback tests).  Same values.
//
// The P2 scan of strip_gaps, scan(max(B[k], P1[k-1] + f(k))) with
// B[k] = Hpre[k-1] + g - k e and f(k) = (k-1) c + g - k e, equals
// max(scan(B)[j], P1[j-1] + f(j)): P1 is a prefix max and f is non-decreasing
// (f(k+1) - f(k) = c - e >= 0, checked on host), so the P1 term's own prefix
// max is its last value.  The scans of A (P1's input) and B are therefore
// independent and run interleaved (wave_prefix_max2).
//
// strip_gaps_tail is everything after the two scans (p1, u scanned).
__device__ __forceinline__ void strip_gaps_tail(const PoaScore& P, int32_t j0, int32_t Hpre, const StripConst& K,
                                                int32_t p1, int32_t u, StripCarry& cr, GapOut& o);
__device__ __forceinline__ void strip_gaps_nf(const PoaScore& P, int32_t j0, int32_t Hpre, const StripConst& K,
                                              StripCarry& cr, GapOut& o) {
  int32_t p1 = shr1_add(cr.cHpre + K.qjc, Hpre, K.qjc);
  int32_t u = p1 + K.k1;  // Hpre[j-1] + g - j e
  wave_prefix_max2(p1, u);
  strip_gaps_tail(P, j0, Hpre, K, p1, u, cr, o);
}
__device__ __forceinline__ void strip_gaps_tail(const PoaScore& P, int32_t j0, int32_t Hpre, const StripConst& K,
                                                int32_t p1, int32_t u, StripCarry& cr, GapOut& o) {
  const int32_t p2 = imax(u, shr1_add_bc(p1, K.k2));
  const int32_t T1 = cr.cQ + P.g - j0 * P.e;
  const int32_t T2 = cr.run1 + K.t2b;
  o.Q = K.jc + imax(p1, cr.run1);
  o.E = K.je + imax(imax(p2, imax(cr.run2, T1)), T2);
  o.H = imax(Hpre, imax(o.E, o.Q));
  o.prevEe = shr1_add(cr.cE + P.e, o.E, K.ve);
  o.prevQc = shr1_add(cr.cQ + P.c, o.Q, K.vc);
  o.prevH = wave_shr1(o.H, cr.cH, 0);
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

// Prefetched inputs of one row: its record and its carries into this strip
// (strip 0: column-0 values H0, F0, O0 from fill_col0).
struct RowIn {
  uint32_t w0, w1, w2, w3;
  int32_t b0, b1, b2, b3;
};

__device__ __forceinline__ uint32_t pred_slot_of(const RowIn& d, uint32_t k, const TBL uint32_t* __restrict__ spill) {
  if (k >= kInlinePreds) return spill[k];
  return (d.w1 >> (16 * k)) & 0xFFFFu;
}

}  // namespace

// Publishing a wave's carry progress.  The consumer reads the carries with
// scalar loads (bndr below), and those reach L2 beside the vector path: the
// workgroup-scope release of the progress store orders this wave's carry
// stores only for vector loads of the same CU (it emits no vmcnt wait), so a
// scalar load issued right after the consumer sees the progress could reach
// L2 before the store and cache a stale line (seen as a rare misalignment on
// a one-row graph, where the consumer spins on the strip's only line).
// Every publication therefore waits for this wave's vector memory
// operations first (tests/test_poa_gpu.py::test_short_graph_strip_handoff:
// 2-19 of 1500 one-row-graph alignments per kernel instance moved without
// it, profiles/r04_j4).  It costs nothing measurable (MSA probe kernel time
// 2714 vs 2728 ms without it); deferring the publication by a row or more so
// that the wait finds the stores landed costs 3 % (with or without the
// wait: the lag or the extra scalar state in the row loop).  gfx9 s_waitcnt
// field layout (gfx950 is a gfx9 target; gfx10+ encode the fields
// differently and count stores apart): vmcnt [3:0] and [15:14], expcnt
// [6:4], lgkmcnt [11:8]; kVmcnt0 is vmcnt(0) with the others at maximum.
//
// What the handoff relies on besides the wait: a published unit is whole
// 128-B carry lines (8 rows x 16 B), so a consumer's scalar load never shares
// a cache line with a carry its producer has not yet stored.  Strip blocks are
// VP = round_up(V, 8) rows (a multiple of 128 B) and every job's carry region
// starts 256-B aligned (bnd_off; svs_poa_engine.cpp check_carry_aligned and
// check_carry_base throw before a launch where it would not).
#if defined(__HIP_DEVICE_COMPILE__) && !defined(__gfx950__)
#error "poa_strip.hip is written for gfx950 (the s_waitcnt encoding below is gfx9's)"
#endif
constexpr int kVmcnt0 = (0x7 << 4) | (0xF << 8);  // vmcnt 0, expcnt 7, lgkmcnt 15
static_assert(kVmcnt0 == 0x0F70, "gfx9 s_waitcnt vmcnt(0) encoding");
static_assert(kCarryLineRows * 16 == 128, "a carry publication unit is one 128-B line");
__device__ __forceinline__ void wait_vm_stores() { __builtin_amdgcn_s_waitcnt(kVmcnt0); }


// Bounded LDS-flag wait (workgroup scope); sets *err after kStripSpinLimit polls.
// Nap schedule of the progress polls: the first SVS_POLL_N polls sleep
// SVS_POLL_S1 x 64 cycles, later ones SVS_POLL_S2 x 64.  A consumer that
// caught up with its producer waits for the next 8-row line, thousands of
// cycles: polling often only takes issue slots from the computing waves
// (profiles/r02_v42: 8/1/4 -> always 8 is 1.5 % less kernel time).
#ifndef SVS_POLL_N
#define SVS_POLL_N 0
#define SVS_POLL_S1 8
#define SVS_POLL_S2 8
#endif
constexpr long kStripSpinLimit = 1l << 26;

// SVS_STRIP_PROF (development builds, tools/build_variant.py): per wave, the
// shader clocks spent waiting for the producing wave's progress, in
// fast_forward, in sweeps, in the traceback and at the job's final barrier,
// and the wave's lifetime, summed over the launch into svs_strip_prof
// (tools/poa_probe.py reads them through svs_debug_strip_prof).
#ifdef SVS_STRIP_PROF
__device__ unsigned long long svs_strip_prof[10];
#define SVS_SP_T() __builtin_amdgcn_s_memtime()
#define SVS_SP_DECL uint64_t sp_acc[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0}; const uint64_t sp_t0 = SVS_SP_T()
#define SVS_SP(i, stmt)                  \
  do {                                   \
    const uint64_t sp_a = SVS_SP_T();    \
    stmt;                                \
    sp_acc[i] += SVS_SP_T() - sp_a;      \
  } while (0)
#else
#define SVS_SP_DECL
#define SVS_SP(i, stmt) stmt
#endif
__device__ __forceinline__ int32_t strip_wait_ge(int32_t* flag, int32_t target, int32_t* err) {
  long n = 0;
  int32_t v;
  while ((v = __builtin_amdgcn_readfirstlane(
              __hip_atomic_load(flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP))) < target) {
    if (n < SVS_POLL_N) __builtin_amdgcn_s_sleep(SVS_POLL_S1);
    else __builtin_amdgcn_s_sleep(SVS_POLL_S2);
    if (++n > kStripSpinLimit) {
      __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      return target;
    }
  }
  return v;
}

// WPJ waves per job (one job per workgroup): wave w sweeps strips w, w+WPJ,
// ...; strip s reads the carries wave (w-1) mod WPJ left for strip s-1, which
// it publishes every 8 rows through an LDS progress counter (workgroup-scope
// release / acquire), so the waves form a row-skewed pipeline over strips.
//
// (A dual sweep, two strips per wave over the same rows, was measured slower
// in round 4 and removed: DESIGN §4.1.)
template <bool LDSP, int WPJ, bool PRUNE, class CodeT>
// The pruning variant is held to 72 VGPRs (a few spills to scratch in cold
// paths): its workgroups still fill a CU 6 waves per SIMD deep (LDS-bound),
// and the 80 registers per SIMD left over take the one-wave fold kernels
// that run beside it (poa_fold.hip) without displacing a DP workgroup:
// 232 vs 225 windows/s at 80 VGPRs (profiles/r03_v28); 80 beat the natural 86
// in round 1 (profiles/r01_v36).  SVS_PRUNE_OCC overrides it in development
// builds.
#ifndef SVS_PRUNE_OCC
#define SVS_PRUNE_OCC 7
#endif
#define SVS_PRUNE_ATTR __attribute__((amdgpu_waves_per_eu(PRUNE ? SVS_PRUNE_OCC : 1)))
// SVS_WG_TIMES (development builds, tools/build_variant.py): the kernel body
// becomes a device function and the kernel records each wave's start and end
// (s_memrealtime, 100 MHz) into svs_wg_times, dumped at session close
// (tools/dp_occupancy.py reads the dump)
#ifdef SVS_WG_TIMES
__device__ __forceinline__ void poa_strip_body(
#else
__global__ __launch_bounds__(64 * WPJ) SVS_PRUNE_ATTR void poa_strip_kernel(
#endif
    const PoaJob* __restrict__ jobs, int n_jobs, PoaScore Parg,
    CodeT* __restrict__ tb, int32_t* __restrict__ bnd_all, const int32_t* __restrict__ bnd_rd,
    int32_t* __restrict__ gpool, int32_t* __restrict__ aln, int32_t* __restrict__ aln_len, uint32_t lds_slots) {
  extern __shared__ int32_t lds[];
  using TF = TbFmt<CodeT>;
  const PoaScore P = Parg;
  SVS_SP_DECL;
  __shared__ int32_t prog[WPJ];  // per wave: strip * (V + 1) + rows done, carries published
  __shared__ int32_t s_err;
  __shared__ int32_t s_brow[WPJ], s_best[WPJ];
  __shared__ uint32_t s_rows[WPJ];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x) >> 6);
  const int job_id = blockIdx.x;
  if (job_id >= n_jobs) return;
  const PoaJob J = jobs[job_id];
  const int32_t L = static_cast<int32_t>(J.len);
  const uint32_t LS = J.ls;
  const uint32_t V = J.n_rows;
  const uint32_t VP = (V + 7) & ~7u;  // carry rows per strip, padded to whole 128-B lines
  // 64-column strips
  const int32_t nstrips = static_cast<int32_t>(LS >> 6);
  auto strip_of = [](int32_t j) -> int32_t { return j >> 6; };
  auto lane_of = [](int32_t j) -> int32_t { return j & 63; };
  constexpr int kStride = kSlotInts;
  const uint32_t nslot = LDSP ? lds_slots : J.n_slots;
  int32_t* __restrict__ pool;  // this wave's pool: nslot x {H, F, O} x 64, then nslot boundary H
  if constexpr (LDSP) pool = lds + static_cast<uint32_t>(wave) * nslot * kStride;
  else pool = gpool + J.pool_off + static_cast<uint64_t>(wave) * ((nslot * kSlotInts + 63) / 64 * 64);
  CodeT* __restrict__ tbj = tb + J.tb_off;
  const TBL uint32_t* __restrict__ rec = tbl(J.rec);
  const TBL uint32_t* __restrict__ rps = tbl(J.pstart);
  const TBL uint32_t* __restrict__ prow = tbl(J.pred);
  const TBL uint32_t* __restrict__ pslot = tbl(J.pslot);
  const TBL int32_t* __restrict__ rc0 = tbl(J.col0);
  const GLB uint8_t* __restrict__ seq = glb(J.seq);
  int32_t* __restrict__ bnd = bnd_all + J.bnd_off;
  // The same carry buffer, read-only: loads through it are uniform and never
  // clobbered by this kernel's stores (those go through bnd), so they become
  // scalar-cache loads.  Safe because every carry line is written once per
  // launch, by whole 128-B lines (strip blocks padded to 8 rows), and read only
  // after its producer has finished the line (progress is published at
  // multiples of 8 rows) and waited for its stores to land (wait_vm_stores:
  // the release alone does not order them for scalar loads).
  const GLB int32_t* __restrict__ bndr = glb(bnd_rd) + J.bnd_off;

  int32_t best = SVS_NEG_INF;  // meaningful on the lane owning column L
  int32_t best_row = 0;
  // Exact pruning (J.lb != kNoPrune).  With ub(cell) an upper bound of the
  // score any completion of an alignment through the cell can still add
  // (every remaining read base matched, the fewest excess gaps the paths from
  // the row's node to a sink allow: m rr + cg max(0, dmin - rr)
  // - (m - cg) max(0, rr - dmax)), a cell with H + ub < lb cannot lie on an
  // alignment scoring >= lb, and ub never grows along a move, so every cell
  // whose maximum comes from such a cell is dead too.  Per strip, a row is
  // alive when some cell of it at columns j0-1 .. j0+63 is (its computed cells,
  // or the carry from strip s-1; in strip 0 the column-0 cell).  A row none of
  // whose inputs (carry / column-0 cell, in-edge rows) is alive is not
  // computed: its slot, registers and carry to strip s+1 become VNEG.  When
  // nothing in the strip is alive the sweep jumps ahead 64 rows at a time to
  // the next row with an alive input (fast_forward), then resets every pool
  // slot to VNEG.  Alive cells keep their exact values and traceback codes: a
  // dead input (VNEG, or the real values of a computed dead row) has every term
  // below an alive cell's maximum.  If the best
  // sink score reaches lb, lb <= the optimum, every cell of every optimal path
  // was computed and the traceback is spoa's; otherwise the job returns
  // kPruneRetry and the host runs it again with no bound.
  const int32_t lb = J.lb;
  // the pruning variant prunes every job of its launch (a job without a bound
  // gets kPruneAll, a bound below every real score: nothing is pruned)
  constexpr bool prune = PRUNE;
  const int32_t cg = imax(imax(P.g, P.e), imax(P.q, P.c));  // best per-base gap score (<= 0, host-checked)
  uint32_t rows_done = 0;

  auto sweep = [&](auto first_tag, int32_t s) {
    constexpr bool FIRST = decltype(first_tag)::value;
    const int32_t j0 = s << 6;
    const int32_t j = j0 + lane;
    const uint8_t rc = seq[j - 1];  // seq[-1] is a zero pad byte (column 0)
    // The read base is waited for here, once per strip.  Left to the compiler,
    // the wait sat at its first use inside the row loop: a load from before the
    // loop is still "pending" at the loop header (the waitcnt pass merges the
    // preheader's state), and with the row's code and carry stores counted on
    // the same vmcnt it became a vmcnt(0) on every computed row, each row
    // waiting for the previous row's stores to be acknowledged.
    wait_vm_stores();
    CodeT* __restrict__ tbl = tbj + j;  // this lane's column of the traceback codes
    const GLB int32_t* __restrict__ bin = bndr + static_cast<uint64_t>(s > 0 ? s - 1 : 0) * VP * 4;
    int32_t* __restrict__ bout = bnd + static_cast<uint64_t>(s) * VP * 4;
    const int32_t pw = (wave + WPJ - 1) % WPJ;          // producer of strip s-1
    const int32_t need0 = (s - 1) * static_cast<int32_t>(V + 1);
    int32_t avail = -1;                                  // producer progress seen so far
    const bool write_bnd = s + 1 < nstrips;
    // rows left until the next whole 8-row carry line, where progress is
    // published (the strip's last row after the row loop): a countdown
    // instead of a test of r per row
    uint32_t pub_left = 8;
    // pruning state of this strip: slot liveness bits (slots < 64, host-checked;
    // slot 0 = the virtual row 0, alive when row0_h + m (L - j) reaches lb at
    // some column j0-1 .. j0+63, i.e. at j0-1: it decreases along j), and the
    // register row's liveness
    // bit p < 31: slot p alive (pruning: < 31 slots, host-checked); bit 31: the
    // register row (the row just above) alive
    constexpr uint32_t kRegBit = 1u << 31;
    uint32_t alive = (FIRST || !prune || row0_h(P, j0 - 1) + P.m * (L - j0 + 1) >= lb) ? 1u : 0u;
    const int32_t rrem = L - j;              // read bases after column j
    // lanes past column L are never alive for a real bound: their m rr term
    // is VNEG/2, so H + ub stays below -5e8 while prune_bound keeps real
    // bounds >= -1e8 (no overflow: H >= VNEG - gaps); a kPruneAll job may see
    // them alive, which only keeps rows it computes anyway.  The liveness
    // ballot then needs no rrem >= 0 lane mask
    const int32_t mrr = rrem >= 0 ? P.m * rrem : SVS_VNEG / 2;
    // every lane tracks its own sink maximum; only the lane of column L in
    // the last strip (which owns L, swept last by its wave) is read
    best = SVS_NEG_INF;
    best_row = 0;
    // m rr + cg max(0, dmin - rr) - (m - cg) max(0, rr - dmax) as
    // m rr + d (d >= 0 ? cg : m - cg) with d = clamp(rr, dmin, dmax) - rr
    auto ub_of = [&](uint32_t w2, int32_t rr, int32_t mr) -> int32_t {
      const int32_t dmin = static_cast<int32_t>(w2 & 0xFFFFu), dmax = static_cast<int32_t>(w2 >> 16);
      const int32_t d = min(imax(rr, dmin), dmax) - rr;
      // 24-bit multiply (full rate; v_mul_lo_u32 is quarter rate): |d| < 2^16
      // and the scores are host-checked to a few thousand
      return mr + __mul24(d, d >= 0 ? cg : P.m - cg);
    };
    StripConst K;
    if (!FIRST) {
      const int32_t ge = P.g - j * P.e, c1 = (j - 1) * P.c;
      K.qjc = P.q - j * P.c;
      K.k1 = ge - K.qjc;
      K.k2 = lane == 0 ? SVS_VNEG + c1 + ge : c1 + ge;
      K.t2b = lane == 0 ? SVS_VNEG : c1 + ge;
      K.jc = j * P.c;
      K.je = j * P.e;
      K.ve = P.e;
      K.vc = P.c;
    }
    // virtual row 0 in slot 0
    {
      const int32_t h0 = row0_h(P, j), fo0 = j == 0 ? 0 : SVS_NEG_INF;
      pool[lane + 1] = h0;
      if (lane == 0) pool[0] = FIRST ? 0 : row0_h(P, j0 - 1);
      reinterpret_cast<uint16_t*>(pool + 65)[lane] = static_cast<uint16_t>(pack_fo(h0, fo0, fo0));
    }
    __builtin_amdgcn_wave_barrier();

    auto fetch = [&](RowIn& d, uint32_t r) {
      const uint32_t rr = r < V ? r : V - 1;
      // 32-bit byte offsets off the job's bases (a job has < 2^28 rows), so
      // that the scalar loads take them as their SGPR offset (an index scaled
      // in 64 bits cost four more SALU per load)
      const TBL uint32_t* w = reinterpret_cast<const TBL uint32_t*>(reinterpret_cast<const TBL char*>(rec) + (rr << 4));
      d.w0 = w[0];
      d.w1 = w[1];
      if constexpr (PRUNE) {
        // path lengths and released slots, read after the DP: prefetched with
        // the rest of the record instead of a dependent load in the row step
        d.w2 = w[2];
        d.w3 = w[3];
      }
      if (FIRST) {
        d.b0 = rc0[3 * rr];
        d.b1 = rc0[3 * rr + 1];
        d.b2 = rc0[3 * rr + 2];
        d.b3 = 0;
      } else {
        if (WPJ > 1) {
          const int32_t need = need0 + static_cast<int32_t>(rr) + 1;
          if (avail < need) {
            SVS_SP(0, avail = strip_wait_ge(&prog[pw], need, &s_err));
          }
        }
        const svs_i32x4 v = *reinterpret_cast<const GLB svs_i32x4*>(reinterpret_cast<const GLB char*>(bin) + (rr << 4));
        d.b0 = v.x; d.b1 = v.y; d.b2 = v.z; d.b3 = v.w;
      }
    };

    int32_t pH = 0, pF = 0, pO = 0, pHm = 0;  // the row just above (registers); pHm = its H[j-1]
    auto step = [&](uint32_t r, const RowIn& d) {
      const uint32_t w0 = __builtin_amdgcn_readfirstlane(d.w0);
      const uint32_t nb = w0 & 0xFFu;
      const bool sink = (w0 >> 8) & 1u;
      const bool store = (w0 >> 9) & 1u;
      // in-degree: 6 bits of w0 (63: at least 63); launches with wide codes
      // count it from pstart
      const uint32_t np = sizeof(CodeT) == 4 ? rps[r + 1] - rps[r] : (w0 >> 10) & 63u;
      const uint32_t own = w0 >> 16;
      // slots >= 31 have no liveness bit (only jobs without a bound of their
      // own, kPruneAll, have them): always alive
      auto slot_alive = [&](uint32_t ps) -> bool {
        if (ps == kNoSlot) return (alive >> 31) != 0;
        return ps >= 31u || ((alive >> ps) & 1u) != 0;
      };
      const uint32_t own_bit = (store && own < 31u) ? 1u << own : 0u;
      auto publish = [&]() {
        if (WPJ > 1 && write_bnd && --pub_left == 0) {
          pub_left = 8;
          // every lane stores the same value: no exec-mask branch, and the
          // countdown stays a scalar
          wait_vm_stores();
          __hip_atomic_store(&prog[wave], s * static_cast<int32_t>(V + 1) + static_cast<int32_t>(r) + 1,
                             __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
      };
      const int32_t cH_in = FIRST ? SVS_VNEG : __builtin_amdgcn_readfirstlane(d.b3);
      if (prune) {
        // the row's own input: the carry (strip 0: the column-0 cell)
        bool live;
        if (FIRST) {
          const int32_t h0 = __builtin_amdgcn_readfirstlane(d.b0);
          live = h0 + ub_of(__builtin_amdgcn_readfirstlane(d.w2), L, P.m * L) >= lb;
        } else {
          live = cH_in > SVS_VNEG / 2;
        }
        if (!live) {
          const uint32_t wp = __builtin_amdgcn_readfirstlane(d.w1);
          live = slot_alive(wp & 0xFFFFu) || (np >= 2 && slot_alive(wp >> 16));
          if (!live && np > kInlinePreds) {
            const TBL uint32_t* __restrict__ spill = pslot + rps[r];
            for (uint32_t k = kInlinePreds; k < np && !live; ++k)
              live = slot_alive(__builtin_amdgcn_readfirstlane(spill[k]));
          }
        }
        if (!live) {
          // no alive input: the row's cells are all dead, never computed
          if (store) {
            int32_t* q = pool + own * kStride;
            q[lane + 1] = SVS_VNEG;
            q[lane] = SVS_VNEG;
            reinterpret_cast<uint16_t*>(q + 65)[lane] = 0;  // F = O = H = VNEG
          }
          // own slot dead, slots whose last reader this row is (w3) released
          alive &= ~(__builtin_amdgcn_readfirstlane(d.w3) | own_bit | kRegBit);
          pH = pF = pO = pHm = SVS_VNEG;
          if (write_bnd && lane == 0)
            *reinterpret_cast<int4*>(reinterpret_cast<char*>(bout) + (r << 4)) = make_int4(SVS_VNEG, SVS_VNEG, SVS_VNEG, SVS_VNEG);
          publish();
          return;
        }
      }
      if constexpr (PRUNE) ++rows_done;
      // the row's path lengths (w2) and released slots (w3), needed after the DP
      uint2 w2w3 = make_uint2(0, 0);
      if constexpr (PRUNE)
        w2w3 = make_uint2(__builtin_amdgcn_readfirstlane(d.w2), __builtin_amdgcn_readfirstlane(d.w3));
      int32_t H0 = 0, F0 = 0, O0 = 0;
      StripCarry cr;
      if (FIRST) {
        H0 = __builtin_amdgcn_readfirstlane(d.b0);
        F0 = __builtin_amdgcn_readfirstlane(d.b1);
        O0 = __builtin_amdgcn_readfirstlane(d.b2);
        cr = StripCarry{SVS_VNEG, SVS_VNEG, H0, SVS_NEG_INF, SVS_NEG_INF, H0};
      } else {
        const int32_t jl = j0 - 1;
        cr.run1 = __builtin_amdgcn_readfirstlane(d.b0);
        cr.run2 = __builtin_amdgcn_readfirstlane(d.b1);
        cr.cHpre = __builtin_amdgcn_readfirstlane(d.b2);
        cr.cH = __builtin_amdgcn_readfirstlane(d.b3);
        cr.cQ = jl * P.c + cr.run1;
        cr.cE = jl * P.e + cr.run2;
      }
      const bool c0 = FIRST && lane == 0;
      const bool inner = FIRST ? (lane != 0 && j <= L) : true;
      const int32_t mc = rc == nb ? P.m : P.n;
      // in-edge k: H, F, O at column j and H at column j-1
      // (pool reads are nontemporal loads so that the compiler cannot merge them
      // with the register case into a select of pointers, which would force the
      // registers into scratch and every pool read onto the flat path)
      auto pred_vals = [&](uint32_t ps, int32_t& hp, int32_t& fp, int32_t& op, int32_t& hpm) {
        if (ps == kNoSlot) {
          hp = pH; fp = pF; op = pO; hpm = pHm;
        } else {
          const int32_t* q = pool + ps * kStride;
          hpm = __builtin_nontemporal_load(q + lane);
          hp = __builtin_nontemporal_load(q + lane + 1);
          const uint32_t dd = __builtin_nontemporal_load(reinterpret_cast<const uint16_t*>(q + 65) + lane);
          fp = hp - static_cast<int32_t>(dd & 0xFFu);
          op = hp - static_cast<int32_t>((dd >> 8) & 0xFFu);
        }
      };
      int32_t H, F, O, Q, E, prevH, prevEe, prevQc;  // prevEe = E[j-1] + e, prevQc = Q[j-1] + c
      uint32_t code;
      auto gaps = [&](int32_t Hpre, bool inner_) {
        if (FIRST) {
          int32_t prevQ, prevE;
          strip_gaps(P, lane, j, j0, inner_, Hpre, H0, cr, Q, E, H, prevQ, prevE, prevH);
          prevEe = prevE + P.e;
          prevQc = prevQ + P.c;
        } else {
          GapOut o;
          strip_gaps_nf(P, j0, Hpre, K, cr, o);
          Q = o.Q; E = o.E; H = o.H; prevH = o.prevH; prevEe = o.prevEe; prevQc = o.prevQc;
        }
      };
      if (np <= 1) {
        const uint32_t ps = __builtin_amdgcn_readfirstlane(d.w1) & 0xFFFFu;  // np == 0: slot 0 (virtual row)
        int32_t hp, fp, op, hpm;
        pred_vals(ps, hp, fp, op, hpm);
        {
        F = imax(hp + P.g, fp + P.e);
        O = imax(hp + P.q, op + P.c);
        int32_t Hpre = imax(hpm + mc, imax(F, O));
        if (FIRST) {
          F = c0 ? F0 : F;
          O = c0 ? O0 : O;
          Hpre = c0 ? H0 : Hpre;
        }
        gaps(Hpre, inner);
        // One in-edge: F = max(hp+g, fp+e) and O = max(hp+q, op+c), so "some
        // up move fits" (H equals one of the four) is H == max(F, O); likewise
        // E = max(prevE+e, prevH+g), Q = max(prevQ+c, prevH+q) make "some left
        // move fits" H == max(E, Q); and F always equals hp+g or fp+e, so the
        // up-chain in-edge is 0 whenever there is an in-edge.  Same codes as
        // assemble_code over the individual tests, fewer instructions.
        const bool dg = inner && H == hpm + mc;
        const bool up = H == imax(F, O);
        const bool ua = H == fp + P.e, ub = H == hp + P.g, uc = H == op + P.c;
        const bool lf = inner && H == imax(E, Q);
        const bool la = H == prevEe, lb = H == prevH + P.g, lc = H == prevQc;
        const bool lbit = inner && (prevH + P.g == E || prevH + P.q == Q);
        const bool va = F == hp + P.g, vb = F == fp + P.e, vc = O == hp + P.q;
        const uint32_t upc = (ua || (!ub && uc)) ? 5u : 1u;
        const uint32_t lfc = (la || (!lb && lc)) ? 6u : 2u;
        code = dg ? 0u : (up ? upc : (lf ? lfc : 3u));
        code |= lbit ? 1u << TF::kLBit : 0u;
        if (np != 0) code |= (va || (!vb && vc)) ? 1u << TF::kStop : 0u;
        else code |= TF::kMask << TF::kUc;
        }
      } else if (!FIRST && np == 2) {
        // Two in-edges (the common merge row), both kept in registers between
        // the DP and the code tests.  Per in-edge k, Fk = max(hp+g, fp+e) and
        // Ok = max(hp+q, op+c): "an up move to k fits" is H == max(Fk, Ok), and
        // "k continues the up-gap run" is F == Fk || O == Ok (F, O, H bound
        // every term from above off column 0, so these equal the four-way
        // tests of the generic loop below).
        const uint32_t w2 = __builtin_amdgcn_readfirstlane(d.w1);
        int32_t hp0, fp0, op0, hm0, hp1, fp1, op1, hm1;
        pred_vals(w2 & 0xFFFFu, hp0, fp0, op0, hm0);
        pred_vals(w2 >> 16, hp1, fp1, op1, hm1);
        const int32_t F0k = imax(hp0 + P.g, fp0 + P.e), O0k = imax(hp0 + P.q, op0 + P.c);
        const int32_t F1k = imax(hp1 + P.g, fp1 + P.e), O1k = imax(hp1 + P.q, op1 + P.c);
        F = imax(F0k, F1k);
        O = imax(O0k, O1k);
        const int32_t D0 = hm0 + mc, D1 = hm1 + mc;
        const int32_t Hpre = imax(imax(D0, D1), imax(F, O));
        gaps(Hpre, true);
        const bool up0 = H == imax(F0k, O0k), up1 = H == imax(F1k, O1k);
        const int32_t hpu = up0 ? hp0 : hp1, fpu = up0 ? fp0 : fp1, opu = up0 ? op0 : op1;
        const bool ua = H == fpu + P.e, ub = H == hpu + P.g, uc = H == opu + P.c;
        const bool ch0 = F == F0k || O == O0k;
        const int32_t hpc = ch0 ? hp0 : hp1, fpc = ch0 ? fp0 : fp1;
        const bool va = F == hpc + P.g, vb = F == fpc + P.e, vc = O == hpc + P.q;
        const bool lf = H == imax(E, Q);
        const bool la = H == prevEe, lb = H == prevH + P.g, lc = H == prevQc;
        const bool lbit = prevH + P.g == E || prevH + P.q == Q;
        const uint32_t upc = ((ua || (!ub && uc)) ? 5u : 1u) | (up0 ? 0u : 8u);
        const uint32_t lfc = (la || (!lb && lc)) ? 6u : 2u;
        code = H == D0 ? 0u : (H == D1 ? 8u : (up0 || up1 ? upc : (lf ? lfc : 3u)));
        code |= lbit ? 1u << TF::kLBit : 0u;
        code |= ((va || (!vb && vc)) ? 1u << TF::kStop : 0u) | (ch0 ? 0u : (1u << TF::kUc));
      } else {
        const TBL uint32_t* __restrict__ spill = pslot + rps[r];
        F = SVS_VNEG;
        O = SVS_VNEG;
        int32_t Hd = SVS_VNEG;
        for (uint32_t k = 0; k < np; ++k) {
          int32_t hp, fp, op, hpm;
          pred_vals(__builtin_amdgcn_readfirstlane(pred_slot_of(d, k, spill)), hp, fp, op, hpm);
          if (FIRST) hpm = c0 ? 0 : hpm;
          F = imax(F, imax(hp + P.g, fp + P.e));
          O = imax(O, imax(hp + P.q, op + P.c));
          Hd = imax(Hd, hpm + mc);
        }
        if (c0) { F = F0; O = O0; }
        const int32_t Hpre = c0 ? H0 : imax(Hd, imax(F, O));
        gaps(Hpre, inner);
        uint32_t diag_k = TF::kMask, up_k = TF::kMask, up_ext = 0, uc_k = TF::kMask, uc_stop = 0;
        for (uint32_t k = 0; k < np; ++k) {
          int32_t hp, fp, op, hpm;
          pred_vals(__builtin_amdgcn_readfirstlane(pred_slot_of(d, k, spill)), hp, fp, op, hpm);
          if (FIRST) hpm = c0 ? 0 : hpm;
          if (inner && diag_k == TF::kMask && H == hpm + mc) diag_k = k;
          if (up_k == TF::kMask) {
            const bool a = H == fp + P.e, b = H == hp + P.g, c = H == op + P.c, dd = H == hp + P.q;
            if (a || b || c || dd) { up_k = k; up_ext = (a || (!b && c)) ? 1u : 0u; }
          }
          if (uc_k == TF::kMask) {
            const bool a = F == hp + P.g, b = F == fp + P.e, c = O == hp + P.q, dd = O == op + P.c;
            if (a || b || c || dd) { uc_k = k; uc_stop = (a || (!b && c)) ? 1u : 0u; }
          }
        }
        const bool la = inner && H == prevEe, lb = inner && H == prevH + P.g;
        const bool lc = inner && H == prevQc, ld = inner && H == prevH + P.q;
        const bool lbit = inner && (prevH + P.g == E || prevH + P.q == Q);
        code = assemble_code<TF>(diag_k, up_k, up_ext, la || lb || lc || ld, la || (!lb && lc), lbit, uc_k, uc_stop);
      }
      // 32-bit row offset off this lane's column: the host keeps n_rows x ls
      // below 2^31 per job
      tbl[r * LS] = static_cast<CodeT>(code);
      bool any_alive = true;
      if (prune) {
        const int32_t ub = ub_of(w2w3.x, rrem, mrr);
        any_alive = __builtin_amdgcn_ballot_w64(H + ub >= lb) != 0;
        const bool out_alive = any_alive || cH_in > SVS_VNEG / 2;
        const uint32_t ob = own_bit | kRegBit;
        alive = ((alive & ~ob) | (out_alive ? ob : 0u)) & ~w2w3.y;
      }
      if (store) {
        // Hx[l+1] = H[l], then Hx[l] = prevH[l] (= H[l-1], lane 0: H[j0-1]);
        // the two full-wave writes agree wherever they overlap
        int32_t* q = pool + own * kStride;
        q[lane + 1] = H;
        q[lane] = prevH;
        reinterpret_cast<uint16_t*>(q + 65)[lane] = static_cast<uint16_t>(pack_fo(H, F, O));
      }
      pH = H;
      pF = F;
      pO = O;
      pHm = prevH;
      if (write_bnd && lane == 0) {
        *reinterpret_cast<int4*>(reinterpret_cast<char*>(bout) + (r << 4)) =
            any_alive ? make_int4(cr.run1, cr.run2, cr.cHpre, cr.cH) : make_int4(SVS_VNEG, SVS_VNEG, SVS_VNEG, SVS_VNEG);
      }
      publish();
      if (sink) {
        const bool u = H > best;
        best = u ? H : best;
        best_row = u ? static_cast<int32_t>(r) + 1 : best_row;
      }
    };

    // Pruning: with no slot (but the virtual row's) and not the register row
    // alive, the next rows are alive only through their carry (strip 0: the
    // column-0 cell) or, while the virtual row is, as sources (no in-edge).
    // Scans 64 rows per step with one load per lane, hands VNEG carries on for
    // the rows it passes, and returns the first row with such an input (or V).
    auto fast_forward = [&](uint32_t r) -> uint32_t {
      while (r < V) {
        uint32_t lim = min(64u, V - r);  // rows this step may look at
        if (!FIRST && WPJ > 1) {
          // only rows strip s-1 has finished (whole 8-row lines); a full chunk
          // is not waited for, so the scan keeps pace with its producer
          const int32_t least = need0 + static_cast<int32_t>(min(V, r + 8));
          if (avail < least) {
            SVS_SP(8, avail = strip_wait_ge(&prog[pw], least, &s_err));
          }
          lim = min(lim, static_cast<uint32_t>(min(static_cast<int32_t>(V), avail - need0)) - r);
        }
        const uint32_t rr = r + static_cast<uint32_t>(lane);
        const bool in = static_cast<uint32_t>(lane) < lim;
        bool cand = false;
        if (FIRST) {
          if (in) {
            const uint32_t w2 = rec[static_cast<uint64_t>(rr) * kRecWords + 2];
            cand = rc0[3 * rr] + ub_of(w2, L, P.m * L) >= lb;
          }
        } else {
          if (in) cand = __builtin_nontemporal_load(bin + 4ull * rr + 3) > SVS_VNEG / 2;
        }
        if ((alive & 1u) && in) cand = cand || ((rec[static_cast<uint64_t>(rr) * kRecWords] >> 10) & 63u) == 0;
        const uint64_t m = __builtin_amdgcn_ballot_w64(cand);
        const uint32_t n = m ? static_cast<uint32_t>(__builtin_ctzll(m)) : lim;
        if (write_bnd && static_cast<uint32_t>(lane) < n)
          *reinterpret_cast<int4*>(bout + 4ull * rr) = make_int4(SVS_VNEG, SVS_VNEG, SVS_VNEG, SVS_VNEG);
        r += n;
        if (m) break;
      }
      // rows passed over left stale pool slots: every slot but the virtual row's to VNEG
      for (uint32_t p = 1; p < nslot; ++p) {
        int32_t* q = pool + p * kStride;
        q[lane + 1] = SVS_VNEG;
        if (lane == 0) q[0] = SVS_VNEG;
        reinterpret_cast<uint16_t*>(q + 65)[lane] = 0;
      }
      pH = pF = pO = pHm = SVS_VNEG;
      // carries of every row before r are stored: publish whole 8-row lines
      if (WPJ > 1 && write_bnd) {
        wait_vm_stores();
        if (lane == 0) {
          const uint32_t done = r >= V ? V : (r & ~7u);
          __hip_atomic_store(&prog[wave], s * static_cast<int32_t>(V + 1) + static_cast<int32_t>(done),
                             __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
      }
      return r;
    };
    auto dead_strip = [&]() { return (alive & ~1u) == 0; };

#ifndef SVS_TWO_SETS
    // One prefetch set, refilled for the next row as soon as a row is done.
    // The row tables and carries are scalar loads, and a scalar load is only
    // waited for with lgkmcnt(0), which waits for every scalar load (they
    // return out of order) and LDS operation in flight: a second set loaded a
    // row further ahead was waited for at the next row's start all the same,
    // and its 8 SGPRs pushed more live values into spill lanes.
    RowIn A;
    uint32_t r = 0;
    if (prune) SVS_SP(1, r = fast_forward(0));
    pub_left = 8u - (r & 7u);
    fetch(A, r);
    while (r < V) {
      step(r, A);
      if (prune && dead_strip()) {
        SVS_SP(1, r = fast_forward(r + 1));
        pub_left = 8u - (r & 7u);
        fetch(A, r);
        continue;
      }
      ++r;
      fetch(A, r);
    }
#else
    // rows in pairs with two statically named prefetch sets (no waits on
    // loads still in flight when a set is refilled)
    RowIn A, B;
    uint32_t r = 0;
    if (prune) SVS_SP(1, r = fast_forward(0));
    pub_left = 8u - (r & 7u);
    fetch(A, r);
    fetch(B, r + 1);
    while (r < V) {
      step(r, A);
      if (prune && dead_strip()) {
        SVS_SP(1, r = fast_forward(r + 1));
        pub_left = 8u - (r & 7u);
        fetch(A, r);
        fetch(B, r + 1);
        continue;
      }
      fetch(A, r + 2);
      if (r + 1 >= V) break;
      step(r + 1, B);
      if (prune && dead_strip()) {
        SVS_SP(1, r = fast_forward(r + 2));
        pub_left = 8u - (r & 7u);
        fetch(A, r);
        fetch(B, r + 1);
        continue;
      }
      fetch(B, r + 3);
      r += 2;
    }
#endif
    // this strip's boundary stores must land before the next strip reads
    // them; then the strip's last rows (V not a multiple of 8) are published:
    // every carry is stored
    __builtin_amdgcn_s_waitcnt(0);
    if (WPJ > 1 && write_bnd && lane == 0)
      __hip_atomic_store(&prog[wave], s * static_cast<int32_t>(V + 1) + static_cast<int32_t>(V), __ATOMIC_RELEASE,
                         __HIP_MEMORY_SCOPE_WORKGROUP);
    __builtin_amdgcn_wave_barrier();
  };


  if (WPJ > 1) {
    if (lane == 0) {
      prog[wave] = -1;
      if (wave == 0) s_err = 0;
    }
    __syncthreads();
  }
  if (V > 0) {
    using TrueT = std::integral_constant<bool, true>;
    using FalseT = std::integral_constant<bool, false>;
    for (int32_t s = wave; s < nstrips; s += WPJ) {
      if (s == 0) SVS_SP(2, sweep(TrueT{}, 0));
      else SVS_SP(2, sweep(FalseT{}, s));
    }
  }

  // the owner of column L's strip holds the sink maximum; every wave's
  // traceback-code stores must be visible to wave 0's lane 0
  best_row = __shfl(best_row, lane_of(L), 64);
  best = __shfl(best, lane_of(L), 64);
  // the wave that swept column L's strip
  const int32_t sink_wave = strip_of(L) % WPJ;
  if (WPJ > 1) {
    if (lane == 0) {
      s_rows[wave] = rows_done;
      if (sink_wave == wave) {
        s_brow[wave] = best_row;
        s_best[wave] = best;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    SVS_SP(4, __syncthreads());
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
#ifdef SVS_STRIP_PROF
    if (wave != 0 && lane == 0) {
      atomicAdd(&svs_strip_prof[0], sp_acc[0]);
      atomicAdd(&svs_strip_prof[1], sp_acc[1]);
      atomicAdd(&svs_strip_prof[2], sp_acc[2]);
      atomicAdd(&svs_strip_prof[4], sp_acc[4]);
      atomicAdd(&svs_strip_prof[5], SVS_SP_T() - sp_t0);
      atomicAdd(&svs_strip_prof[7], 1ull);
      atomicAdd(&svs_strip_prof[8], sp_acc[8]);
    }
#endif
    if (wave != 0) return;
    best_row = s_brow[sink_wave];
    best = s_best[sink_wave];
    rows_done = 0;
    for (int w = 0; w < WPJ; ++w) rows_done += s_rows[w];
    if (s_err) {
      if (lane == 0) aln_len[job_id] = -1;
      return;
    }
  } else {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    __builtin_amdgcn_wave_barrier();
  }
  // Traceback by the whole of wave 0 in lockstep (every value it branches on
  // is uniform).  Codes come from 16 x 16 tiles (rows r-15..r, columns
  // c-15..c, four gathers per lane issued together) and in-edge rows 0 and 1
  // from 64-row tiles, so the path pays one HBM round trip per tile instead of
  // one or two per step.
  best_row = __builtin_amdgcn_readfirstlane(best_row);
  best = __builtin_amdgcn_readfirstlane(best);
  if constexpr (!PRUNE) rows_done = V * (LS >> 6);  // in 64-column strip rows
  if (lane == 0) {
    aln_len[n_jobs + job_id] = best;
    aln_len[2 * n_jobs + job_id] = static_cast<int32_t>(rows_done);
  }
  if (prune && best < lb) {
    if (lane == 0) aln_len[job_id] = kPruneRetry;
    return;
  }
  int32_t t_r = INT32_MIN / 2, t_c = INT32_MIN / 2, p_r = INT32_MIN / 2;
  uint32_t t0 = 0, t1 = 0, t2 = 0, t3 = 0;  // element e = 64 v + lane: (t_r - e / 16, t_c - e % 16)
  int32_t pn = 0, p0 = 0, p1 = 0;           // lane l: in-edge count and in-edges 0, 1 of row p_r - l
  auto tbc = [&](int32_t row, int32_t col) -> uint32_t {
    const uint32_t dr = static_cast<uint32_t>(t_r - row), dc = static_cast<uint32_t>(t_c - col);
    if (dr >= 16u || dc >= 16u) {
      t_r = row;
      t_c = col;
      const int32_t cc = col - (lane & 15), r0 = row - (lane >> 4);
      auto ld = [&](int32_t rr) -> uint32_t {
        return (rr >= 1 && cc >= 0) ? tbj[static_cast<uint64_t>(rr - 1) * LS + cc] : 0u;
      };
      t0 = ld(r0);
      t1 = ld(r0 - 4);
      t2 = ld(r0 - 8);
      t3 = ld(r0 - 12);
      return __builtin_amdgcn_readfirstlane(t0);
    }
    const uint32_t e = dr * 16 + dc, l = e & 63u, v = e >> 6;
    const uint32_t x0 = __builtin_amdgcn_readlane(t0, l), x1 = __builtin_amdgcn_readlane(t1, l);
    const uint32_t x2 = __builtin_amdgcn_readlane(t2, l), x3 = __builtin_amdgcn_readlane(t3, l);
    return v == 0 ? x0 : (v == 1 ? x1 : (v == 2 ? x2 : x3));
  };
  auto pred_of = [&](int32_t row, uint32_t k) -> int32_t {
    if (k >= 2) {
      const uint32_t a = rps[row - 1], b = rps[row];
      return (b == a) ? 0 : static_cast<int32_t>(prow[a + k] & 0x7FFFFFFFu);  // bit 31: export_strip_lite's flag
    }
    if (static_cast<uint32_t>(p_r - row) >= 64u) {
      p_r = row;
      const int32_t rr = row - lane;
      uint32_t a = 0, b = 0;
      if (rr >= 1) { a = rps[rr - 1]; b = rps[rr]; }
      pn = static_cast<int32_t>(b - a);
      p0 = pn > 0 ? static_cast<int32_t>(prow[a] & 0x7FFFFFFFu) : 0;
      p1 = pn > 1 ? static_cast<int32_t>(prow[a + 1] & 0x7FFFFFFFu) : 0;
    }
    const uint32_t l = static_cast<uint32_t>(p_r - row);
    const int32_t n = __builtin_amdgcn_readlane(pn, l);
    const int32_t x = __builtin_amdgcn_readlane(k == 0 ? p0 : p1, l);
    return n == 0 ? 0 : x;
  };
  int32_t* __restrict__ out = aln + 2 * J.aln_off;
  auto emit = [&](int64_t n, int32_t a, int32_t b) {
    if (lane == 0) {
      out[2 * n] = a;
      out[2 * n + 1] = b;
    }
  };
  int32_t nout;
  SVS_SP(3, nout = poa_traceback<TF>(P, V, L, best_row, tbc, pred_of, emit));
  if (lane == 0) aln_len[job_id] = nout;
#ifdef SVS_STRIP_PROF
  if (lane == 0) {
    for (int i = 0; i < 5; ++i) atomicAdd(&svs_strip_prof[i], sp_acc[i]);
    atomicAdd(&svs_strip_prof[5], SVS_SP_T() - sp_t0);
    atomicAdd(&svs_strip_prof[6], static_cast<unsigned long long>(rows_done));
    atomicAdd(&svs_strip_prof[7], 1ull);
    atomicAdd(&svs_strip_prof[8], sp_acc[8]);
  }
#endif
}

#ifdef SVS_WG_TIMES
constexpr unsigned kWgTimesCap = 1u << 23;
__device__ unsigned long long svs_wg_times[kWgTimesCap][8];
__device__ unsigned int svs_wg_n;
template <bool LDSP, int WPJ, bool PRUNE, class CodeT>
__global__ __launch_bounds__(64 * WPJ) SVS_PRUNE_ATTR void poa_strip_kernel(
    const PoaJob* __restrict__ jobs, int n_jobs, PoaScore Parg,
    CodeT* __restrict__ tb, int32_t* __restrict__ bnd_all, const int32_t* __restrict__ bnd_rd,
    int32_t* __restrict__ gpool, int32_t* __restrict__ aln, int32_t* __restrict__ aln_len, uint32_t lds_slots) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  poa_strip_body<LDSP, WPJ, PRUNE, CodeT>(jobs, n_jobs, Parg, tb, bnd_all, bnd_rd, gpool, aln, aln_len, lds_slots);
  const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
  if ((threadIdx.x & 63) == 0) {
    const unsigned i = atomicAdd(&svs_wg_n, 1u);
    if (i < kWgTimesCap) {
      svs_wg_times[i][0] = t0;
      svs_wg_times[i][1] = t1;
      svs_wg_times[i][2] = (static_cast<unsigned long long>(blockIdx.x) << 32) | (threadIdx.x >> 6);
      svs_wg_times[i][3] = (static_cast<unsigned long long>(reinterpret_cast<uintptr_t>(jobs)) & 0xFFFFFFFFFFFFull) |
                           (static_cast<unsigned long long>(WPJ) << 56) | (static_cast<unsigned long long>(n_jobs >> 4) << 48);
      // the job's rows and read length; wave 0 (which ends with the
      // traceback): the strip rows the job computed and its best score
      const PoaJob& J = jobs[blockIdx.x];
      const bool w0 = threadIdx.x < 64 && static_cast<int>(blockIdx.x) < n_jobs;
      svs_wg_times[i][4] = J.n_rows;
      svs_wg_times[i][5] = J.len;
      svs_wg_times[i][6] = w0 ? static_cast<unsigned long long>(static_cast<uint32_t>(aln_len[2 * n_jobs + blockIdx.x])) : 0ull;
      svs_wg_times[i][7] = w0 ? static_cast<unsigned long long>(static_cast<uint32_t>(J.lb)) : 0ull;
    }
  }
}
#endif

hipError_t launch_poa_strip(const PoaLaunch& a, hipStream_t stream) {
  if (a.n_jobs <= 0) return hipSuccess;
  const int w = a.waves_per_job;
  const bool lds_pool = a.lds_slots > 0;
  const size_t lds = lds_pool ? static_cast<size_t>(w) * a.lds_slots * kStripSlotBytes : 0;
#define SVS_STRIP4(LP, W, PR, CT)                                                                          \
  hipLaunchKernelGGL((poa_strip_kernel<LP, W, PR, CT>), dim3(a.n_jobs), dim3(64 * W), lds, stream, a.jobs, \
                     a.n_jobs, a.score, static_cast<CT*>(a.tb), a.bnd, a.bnd, a.pool, a.aln, a.aln_len,     \
                     a.lds_slots)
#define SVS_STRIP3(LP, W, PR)              \
  do {                                     \
    if (a.wide) {                          \
      SVS_STRIP4(LP, W, PR, uint32_t);     \
    } else {                               \
      SVS_STRIP4(LP, W, PR, uint16_t);     \
    }                                      \
  } while (0)
#define SVS_STRIP(LP, W)              \
  do {                                \
    if (a.prune) {                    \
      SVS_STRIP3(LP, W, true);        \
    } else {                          \
      SVS_STRIP3(LP, W, false);       \
    }                                 \
  } while (0)
  // the engine's choices: 1, 2, 4, 8 waves per job (16 with the pool in LDS)
  if (lds_pool) {
    switch (w) {
      case 16: SVS_STRIP(true, 16); break;
      case 8: SVS_STRIP(true, 8); break;
      case 4: SVS_STRIP(true, 4); break;
      case 2: SVS_STRIP(true, 2); break;
      case 1: SVS_STRIP(true, 1); break;
      default: return hipErrorInvalidValue;
    }
  } else {
    switch (w) {
      case 8: SVS_STRIP(false, 8); break;
      case 4: SVS_STRIP(false, 4); break;
      case 2: SVS_STRIP(false, 2); break;
      case 1: SVS_STRIP(false, 1); break;
      default: return hipErrorInvalidValue;
    }
  }
#undef SVS_STRIP
#undef SVS_STRIP3
#undef SVS_STRIP4
  return hipGetLastError();
}

// Primitive self-test (tests/test_poa_gpu.py): per wave, the DPP inclusive
// prefix max and the wave_shr1 lane shift the strip kernel's scans are built of.
__global__ void wave_scan_selftest_kernel(const int32_t* in, int32_t* out_scan, int32_t* out_shift) {
  const int lane = threadIdx.x & 63;
  const int32_t x = in[blockIdx.x * 64 + lane];
  out_scan[blockIdx.x * 64 + lane] = wave_prefix_max(x);
  out_shift[blockIdx.x * 64 + lane] = wave_shr1(x, -7, lane);
}

// SVS_STRIP_PROF builds: the counters above (out[10]); reset = 1 zeroes them.
// Other builds report zeros.
extern "C" int svs_debug_strip_prof(unsigned long long* out, int reset) {
#ifdef SVS_STRIP_PROF
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(svs_strip_prof), 10 * sizeof(unsigned long long)) != hipSuccess) return -3;
  if (reset) {
    unsigned long long z[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(svs_strip_prof), z, sizeof(z)) != hipSuccess) return -3;
  }
#else
  (void)reset;
  for (int i = 0; i < 10; ++i) out[i] = 0;
#endif
  return 0;
}

// SVS_WG_TIMES builds: writes the recorded wave times (n x 8 uint64) to path
// and resets the count; other builds write nothing.
extern "C" int svs_debug_wg_times_dump(const char* path) {
#ifdef SVS_WG_TIMES
  unsigned n = 0;
  if (hipDeviceSynchronize() != hipSuccess) return -3;
  if (hipMemcpyFromSymbol(&n, HIP_SYMBOL(svs_wg_n), sizeof(n)) != hipSuccess) return -3;
  n = std::min(n, kWgTimesCap);
  std::vector<unsigned long long> h(static_cast<size_t>(n) * 8);
  if (n && hipMemcpyFromSymbol(h.data(), HIP_SYMBOL(svs_wg_times), h.size() * 8) != hipSuccess) return -3;
  FILE* f = std::fopen(path, "wb");
  if (!f) return -1;
  std::fwrite(h.data(), 8, h.size(), f);
  std::fclose(f);
  const unsigned z = 0;
  if (hipMemcpyToSymbol(HIP_SYMBOL(svs_wg_n), &z, sizeof(z)) != hipSuccess) return -3;
  return static_cast<int>(n);
#else
  (void)path;
  return 0;
#endif
}

hipError_t launch_wave_selftest(const int32_t* in, int32_t* scan, int32_t* shift, int n_waves,
                                hipStream_t stream) {
  hipLaunchKernelGGL(wave_scan_selftest_kernel, dim3(n_waves), dim3(64), 0, stream, in, scan, shift);
  return hipGetLastError();
}

}  // namespace svs
