// MisScore on gfx950: Biopython pairwise2.align.globalms(som, ger, 1, 0, -1, -1)[0]
// and its match-line counts for many (somatic, germline) consensus pairs
// (reference: /root/reference/src/PairwiseCompare.py:19-30 AligmentScore,
// called by CalculateMisscore :54-64 for every pair of a Raw.bed row).
//
// Two kernels per launch:
//
// misscore_fill_kernel — one wave per pair.  The DP matrix (rows = som,
// columns = ger) is swept in 64-column strips; inside a strip lane k owns
// column c0 + k and works one row behind lane k - 1 (a diagonal wavefront),
// so each step is one DPP lane shift plus a max3:
//   H[r][c] = max(H[r-1][c-1] + (a == b), max(H[r-1][c], H[r][c-1]) - 1)
// (linear gaps: pairwise2's row/col scores equal H - 1 of the left/upper
// cell, see misscore_tb.hpp).  Only the two score differences
// dh = H[r][c] - H[r][c-1] and dv = H[r][c] - H[r-1][c] leave the kernel, two
// bits each, eight rows of one column per 32-bit word:
//   word index = (strip * n_groups + (t - 1) / 8) * 64 + lane,
//   nibble     = (t - 1) % 8,  t = r + lane (the step that computed the cell),
// so all 64 lanes close a word on the same step: one coalesced 256-B store
// every 8 steps.
// 0.5 B per cell of HBM writes instead of pairwise2's int score + trace.
// The H column at a strip's right edge is handed to the next strip through a
// per-pair carry vector (one int32 per row, in place, 64 rows per coalesced
// load/store, loaded one 64-step chunk ahead); the A characters stream in the
// same way.  The 64 steps of a chunk are unrolled, so lane selects are
// immediates and stores sit at fixed positions.
//
// misscore_traceback_kernel — one lane per pair replays pairwise2's DFS
// (misscore_tb.hpp) over the nibbles with an explicit stack in HBM.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>

#define SVS_MS_FN __device__ __forceinline__
#include "misscore_device.hpp"

namespace svs {

namespace {

// lane l <- x[l-1]; lane 0 <- fill.  DPP wave_shr:1 (bound_ctrl off keeps old).
__device__ __forceinline__ int32_t shr1(int32_t x, int32_t fill) {
  return __builtin_amdgcn_update_dpp(fill, x, 0x138, 0xF, 0xF, false);
}
// lane l <- x[l+1] (lane 63 keeps x).  DPP wave_shl:1.
__device__ __forceinline__ int32_t shl1(int32_t x) { return __builtin_amdgcn_update_dpp(x, x, 0x130, 0xF, 0xF, false); }
// lane l <- x[l-1], lane 0 <- x[63].  DPP wave_ror:1.
__device__ __forceinline__ int32_t ror1(int32_t x) { return __builtin_amdgcn_update_dpp(x, x, 0x13C, 0xF, 0xF, false); }

__global__ __launch_bounds__(256) void misscore_fill_kernel(const MsPair* __restrict__ pairs,
                                                            const int32_t* __restrict__ solo, int n_solo,
                                                            const uint8_t* __restrict__ seqs,
                                                            uint32_t* __restrict__ nib, int32_t* __restrict__ carry) {
  const int sid = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (sid >= n_solo) return;
  const int lane = threadIdx.x & 63;
  const MsPair P = pairs[solo[sid]];
  const int32_t la = P.la, lb = P.lb;
  const int32_t n_chunks = ms_chunks(la);
  const int32_t n_strips = (lb + 63) >> 6;
  const uint8_t* A = seqs + P.a_off;
  const uint8_t* B = seqs + P.b_off;
  int32_t* cr = carry + P.carry_off;  // cr[r - 1] = H[r][c0 - 1] of the current strip
  for (int32_t s = 0; s < n_strips; ++s) {
    const int32_t c = s * 64 + lane + 1;
    const bool col_ok = c <= lb;
    const int32_t bc = col_ok ? static_cast<int32_t>(B[c - 1]) : -1;
    const bool last = s == n_strips - 1;
    int32_t h = -c;           // H[r-1][c]: row 0 is -c
    int32_t diag = -(c - 1);  // H[r-1][c-1]
    int32_t ach = 0;          // A[r-1] of this lane's row
    int32_t cout = 0;         // H of lane 63's rows in this chunk (lane j: step 63 - j)
    uint32_t* out = nib + P.nib_off + static_cast<uint64_t>(s) * n_chunks * 8 * 64 + lane;
    // chunk 0: rows 1..64 (lane j holds row 1 + j)
    int32_t nxt_c, nxt_a;
    {
      const int32_t rr = 1 + lane;
      const bool ok = rr <= la;
      nxt_c = s == 0 ? -rr : (ok ? cr[rr - 1] : 0);
      nxt_a = ok ? static_cast<int32_t>(A[rr - 1]) : 0;
    }
    for (int32_t ch = 0; ch < n_chunks; ++ch) {
      int32_t cc = nxt_c, ca = nxt_a;  // lane 0 holds this step's left H / A character
      {  // prefetch the next chunk's left column and A characters
        const int32_t rr = 64 * (ch + 1) + 1 + lane;
        const bool ok = rr <= la;
        nxt_c = s == 0 ? -rr : (ok ? cr[rr - 1] : 0);
        nxt_a = ok ? static_cast<int32_t>(A[rr - 1]) : 0;
      }
      // step t = 64 ch + u + 1; lane k is at row r = t - k
      const int32_t rm1_base = 64 * ch - lane;  // r - 1 at u = 0
      uint32_t acc = 0;
#pragma unroll
      for (int32_t u = 0; u < 64; ++u) {
        const int32_t left = shr1(h, cc);  // lane 0 keeps cc (its left neighbour)
        ach = shr1(ach, ca);
        cc = shl1(cc);
        ca = shl1(ca);
        const int32_t sc = ach == bc ? 1 : 0;
        const int32_t hn = max(diag + sc, max(h, left) - 1);
        const bool act = static_cast<uint32_t>(rm1_base + u) < static_cast<uint32_t>(la);
        const uint32_t code = static_cast<uint32_t>(hn - left + 1) | (static_cast<uint32_t>(hn - h + 1) << 2);
        acc |= (act ? code : 0u) << ((u & 7) * 4);
        diag = act ? left : diag;
        h = act ? hn : h;
        if ((u & 7) == 7) {  // every lane closes an 8-step group together
          if (col_ok) out[static_cast<uint64_t>(ch * 8 + (u >> 3)) * 64] = acc;
          acc = 0;
        }
        // history of lane 63's H: lane j ends with the value of step 63 - j
        cout = shr1(cout, ror1(h));
      }
      if (!last) {  // lane 63's rows of this chunk: step u = 63 - lane, row t - 63 = 64 ch + u - 62
        const int32_t row = 64 * ch + 1 - lane;
        if (row >= 1 && row <= la) cr[row - 1] = cout;
      }
    }
    // the next strip reads the carries this wave just wrote
    __threadfence_block();
  }
}

typedef short s16x2 __attribute__((ext_vector_type(2)));
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ s16x2 as_s(int32_t x) { return __builtin_bit_cast(s16x2, x); }
__device__ __forceinline__ int32_t as_i(s16x2 v) { return __builtin_bit_cast(int32_t, v); }
__device__ __forceinline__ int32_t as_i(u16x2 v) { return __builtin_bit_cast(int32_t, v); }
__device__ __forceinline__ int32_t pack2(int32_t lo, int32_t hi) {
  return static_cast<int32_t>((static_cast<uint32_t>(lo) & 0xFFFFu) | (static_cast<uint32_t>(hi) << 16));
}

// misscore_fill_kernel for two pairs at once (a "duo"): the low 16-bit half of
// every register belongs to pair X, the high half to pair Y, and the step runs
// on packed VOP3P math (v_pk_add/sub/max/min_*16), so one VALU instruction
// advances two cells.  Both pairs sweep max(la) x max(lb); cells outside a
// pair's own matrix are computed but never stored, and they only ever feed
// cells further right or down, outside it too.  Scores fit in 16 bits:
// |H| <= max(la, lb) <= kMsPackedMaxLen (host-checked).  Each 8-step group's
// two 4-step accumulators are split into X's and Y's 32-bit words with
// v_perm, so the nibble layout is the 32-bit kernel's.
__global__ __launch_bounds__(256) void misscore_fill2_kernel(const MsPair* __restrict__ pairs,
                                                             const MsDuo* __restrict__ duos, int n_duos,
                                                             const uint8_t* __restrict__ seqs,
                                                             uint32_t* __restrict__ nib, int32_t* __restrict__ carry) {
  const int did = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (did >= n_duos) return;
  const int lane = threadIdx.x & 63;
  const MsDuo D = duos[did];
  const MsPair X = pairs[D.x];
  const bool has_y = D.y >= 0;
  const MsPair Y = pairs[has_y ? D.y : D.x];
  const int32_t la = max(X.la, Y.la), lb = max(X.lb, Y.lb);
  const int32_t n_chunks = ms_chunks(la);
  const int32_t gx = ms_chunks(X.la) * 8, gy = ms_chunks(Y.la) * 8;  // each pair's own word rows per strip
  const int32_t n_strips = (lb + 63) >> 6;
  const uint8_t* AX = seqs + X.a_off;
  const uint8_t* AY = seqs + Y.a_off;
  const uint8_t* BX = seqs + X.b_off;
  const uint8_t* BY = seqs + Y.b_off;
  int32_t* cr = carry + D.carry_off;  // packed H[r][c0 - 1]
  const u16x2 one = {1, 1};
  for (int32_t s = 0; s < n_strips; ++s) {
    const int32_t c = s * 64 + lane + 1;
    const bool okx = c <= X.lb, oky = has_y && c <= Y.lb;
    // 0x100 never equals a character
    const int32_t bc = pack2(okx ? BX[c - 1] : 0x100, oky ? BY[c - 1] : 0x100);
    const bool last = s == n_strips - 1;
    int32_t h = pack2(-c, -c);
    int32_t diag = pack2(-(c - 1), -(c - 1));
    int32_t ach = 0, cout = 0;
    uint32_t* outx = nib + X.nib_off + static_cast<uint64_t>(s) * gx * 64 + lane;
    uint32_t* outy = nib + Y.nib_off + static_cast<uint64_t>(s) * gy * 64 + lane;
    auto chunk_in = [&](int32_t rr, int32_t& vc, int32_t& va) {
      const bool ok = rr <= la;
      vc = s == 0 ? pack2(-rr, -rr) : (ok ? cr[rr - 1] : 0);
      va = pack2(rr <= X.la ? AX[rr - 1] : 0x200, has_y && rr <= Y.la ? AY[rr - 1] : 0x200);
    };
    int32_t nxt_c, nxt_a;
    chunk_in(1 + lane, nxt_c, nxt_a);
    for (int32_t ch = 0; ch < n_chunks; ++ch) {
      int32_t cc = nxt_c, ca = nxt_a;
      chunk_in(64 * (ch + 1) + 1 + lane, nxt_c, nxt_a);
      const int32_t rm1_base = 64 * ch - lane;
      uint32_t acc0 = 0, acc1 = 0;  // steps 0-3 and 4-7 of the current group, both pairs
#pragma unroll
      for (int32_t u = 0; u < 64; ++u) {
        const int32_t left = shr1(h, cc);
        ach = shr1(ach, ca);
        cc = shl1(cc);
        ca = shl1(ca);
        // per half: 1 where the characters differ, 0 where they match (asm keeps
        // it one v_pk_min_u16: the compiler would otherwise split it into
        // two 16-bit compares and selects)
        int32_t ne;
        asm("v_pk_min_u16 %0, %1, 1 op_sel_hi:[1,0]" : "=v"(ne) : "v"(ach ^ bc));
        const s16x2 dmatch = as_s(diag) + as_s(as_i(one)) - as_s(ne);  // H[r-1][c-1] + (a == b)
        const s16x2 hn = __builtin_elementwise_max(dmatch,
                                                   __builtin_elementwise_max(as_s(h), as_s(left)) - as_s(as_i(one)));
        const bool act = static_cast<uint32_t>(rm1_base + u) < static_cast<uint32_t>(la);
        const s16x2 hn1 = hn + as_s(as_i(one));
        const uint32_t dh1 = static_cast<uint32_t>(as_i(hn1 - as_s(left)));  // 0..3 per half
        const uint32_t dv1 = static_cast<uint32_t>(as_i(hn1 - as_s(h)));
        const uint32_t code = act ? (dh1 | (dv1 << 2)) : 0u;
        if ((u & 4) == 0) acc0 |= code << ((u & 3) * 4);
        else acc1 |= code << ((u & 3) * 4);
        diag = act ? left : diag;
        h = act ? as_i(hn) : h;
        if ((u & 7) == 7) {
          const int32_t g = ch * 8 + (u >> 3);
          if (okx && g < gx) outx[static_cast<uint64_t>(g) * 64] = __builtin_amdgcn_perm(acc1, acc0, 0x05040100u);
          if (oky && g < gy) outy[static_cast<uint64_t>(g) * 64] = __builtin_amdgcn_perm(acc1, acc0, 0x07060302u);
          acc0 = 0;
          acc1 = 0;
        }
        cout = shr1(cout, ror1(h));
      }
      if (!last) {
        const int32_t row = 64 * ch + 1 - lane;
        if (row >= 1 && row <= la) cr[row - 1] = cout;
      }
    }
    __threadfence_block();
  }
}

struct DevEnv {
  const uint32_t* nibs;
  const uint8_t* A;
  const uint8_t* B;
  MsState* stack;
  uint32_t cap;
  uint32_t top;
  int32_t n_groups;
  int32_t max_depth;
  __device__ __forceinline__ uint32_t nib(int32_t r, int32_t c) const {
    // lane k of strip s holds row r at step t = r + k: word (s, (t-1)/8, k), nibble (t-1)%8
    const int32_t k = (c - 1) & 63, t1 = r - 1 + k;
    const uint32_t w = nibs[(static_cast<uint64_t>((c - 1) >> 6) * n_groups + (t1 >> 3)) * 64 + k];
    return (w >> ((t1 & 7) * 4)) & 15u;
  }
  __device__ __forceinline__ uint8_t a(int32_t i) const { return A[i]; }
  __device__ __forceinline__ uint8_t b(int32_t j) const { return B[j]; }
  __device__ __forceinline__ bool push(const MsState& s) {
    if (top >= cap) return false;
    stack[top++] = s;
    return true;
  }
  __device__ __forceinline__ void pop(MsState& s) { s = stack[--top]; }
};

__global__ __launch_bounds__(64) void misscore_traceback_kernel(const MsPair* __restrict__ pairs, int n_pairs,
                                                                const uint8_t* __restrict__ seqs,
                                                                const uint32_t* __restrict__ nib,
                                                                MsState* __restrict__ stack, int32_t cutoff,
                                                                MsResult* __restrict__ out) {
  const int pid = blockIdx.x * 64 + threadIdx.x;
  if (pid >= n_pairs) return;
  const MsPair P = pairs[pid];
  DevEnv env{nib + P.nib_off, seqs + P.a_off, seqs + P.b_off, stack + P.stack_off, P.stack_cap, 0,
             ms_chunks(P.la) * 8, 0};
  const int64_t max_steps = 8ll * (P.la + P.lb) + 4096;
  out[P.out_idx] = ms_first_alignment(env, P.la, P.lb, cutoff, max_steps);
}

// The same DFS with one wave per pair.  Every value the DFS branches on is
// wave-uniform; the wave's lanes only serve as a register cache.  Nibbles come
// from a 32-column x 32-step tile (two words per lane: lane l holds column
// tc - (l & 31), words g0 - (l >> 5) and g0 - 2 - (l >> 5) of that column,
// g0 the word holding row tr), so a path pays one HBM round trip per ~16-32
// steps instead of two or three dependent loads per step.  Characters come
// from 64-wide register windows the same way.  Stack entries are written and
// read back by lane 0 only (a thread sees its own stores) and broadcast.
struct WaveEnv {
  const uint32_t* nibs;
  const uint8_t* A;
  const uint8_t* B;
  MsState* stack;
  uint32_t cap;
  uint32_t top;
  int32_t n_groups;
  int32_t max_depth;
  int32_t lane;
  int32_t tr = -1000000, tc = -1000000;  // tile anchor (row, column)
  uint32_t tw0 = 0, tw1 = 0;
  int32_t ta = -1000000, tb = -1000000;  // character windows: lane l holds A[ta-1-l], B[tb-1-l]
  int32_t wa = 0, wb = 0;
  __device__ __forceinline__ uint32_t word_at(int32_t c, int32_t g) const {
    const int32_t k = (c - 1) & 63;
    return nibs[(static_cast<uint64_t>((c - 1) >> 6) * n_groups + g) * 64 + k];
  }
  __device__ __forceinline__ void load_tile(int32_t r, int32_t c) {
    tr = r;
    tc = c;
    const int32_t cc = c - (lane & 31);
    const int32_t g0 = (r - 1 + ((cc - 1) & 63)) >> 3;
    const int32_t ga = g0 - (lane >> 5), gb = ga - 2;
    tw0 = (cc >= 1 && ga >= 0) ? word_at(cc, ga) : 0u;
    tw1 = (cc >= 1 && gb >= 0) ? word_at(cc, gb) : 0u;
  }
  __device__ __forceinline__ uint32_t nib(int32_t r, int32_t c) {
    const int32_t k = (c - 1) & 63, t1 = r - 1 + k;
    int32_t d = tc - c, dg = ((tr - 1 + k) >> 3) - (t1 >> 3);
    if (static_cast<uint32_t>(d) >= 32u || static_cast<uint32_t>(dg) >= 4u) {
      load_tile(r, c);
      d = 0;
      dg = 0;
    }
    const int32_t l = d + 32 * (dg & 1);
    const uint32_t w = (dg >> 1) ? __builtin_amdgcn_readlane(tw1, l) : __builtin_amdgcn_readlane(tw0, l);
    return (w >> ((t1 & 7) * 4)) & 15u;
  }
  __device__ __forceinline__ uint8_t a(int32_t i) {
    int32_t d = ta - 1 - i;
    if (static_cast<uint32_t>(d) >= 64u) {
      ta = i + 1;
      wa = i - lane >= 0 ? A[i - lane] : 0;
      d = 0;
    }
    return static_cast<uint8_t>(__builtin_amdgcn_readlane(wa, d));
  }
  __device__ __forceinline__ uint8_t b(int32_t j) {
    int32_t d = tb - 1 - j;
    if (static_cast<uint32_t>(d) >= 64u) {
      tb = j + 1;
      wb = j - lane >= 0 ? B[j - lane] : 0;
      d = 0;
    }
    return static_cast<uint8_t>(__builtin_amdgcn_readlane(wb, d));
  }
  __device__ __forceinline__ bool push(const MsState& s) {
    if (top >= cap) return false;
    if (lane == 0) stack[top] = s;
    ++top;
    return true;
  }
  __device__ __forceinline__ void pop(MsState& s) {
    --top;
    MsState v{};
    if (lane == 0) v = stack[top];
    s.row = __builtin_amdgcn_readfirstlane(v.row);
    s.col = __builtin_amdgcn_readfirstlane(v.col);
    s.trace = __builtin_amdgcn_readfirstlane(v.trace);
    s.col_gap = __builtin_amdgcn_readfirstlane(v.col_gap);
    s.nc = __builtin_amdgcn_readfirstlane(v.nc);
    s.nm = __builtin_amdgcn_readfirstlane(v.nm);
    s.front = (static_cast<uint64_t>(static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int32_t>(v.front >> 32)))) << 32) |
              static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int32_t>(v.front)));
    s.recent = (static_cast<uint64_t>(static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int32_t>(v.recent >> 32)))) << 32) |
               static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int32_t>(v.recent)));
  }
};

__global__ __launch_bounds__(64) void misscore_traceback_wave_kernel(const MsPair* __restrict__ pairs, int n_pairs,
                                                                     const uint8_t* __restrict__ seqs,
                                                                     const uint32_t* __restrict__ nib,
                                                                     MsState* __restrict__ stack, int32_t cutoff,
                                                                     MsResult* __restrict__ out) {
  const int pid = blockIdx.x;
  if (pid >= n_pairs) return;
  const MsPair P = pairs[pid];
  WaveEnv env{nib + P.nib_off, seqs + P.a_off, seqs + P.b_off, stack + P.stack_off, P.stack_cap, 0,
              ms_chunks(P.la) * 8, 0, static_cast<int32_t>(threadIdx.x)};
  const int64_t max_steps = 8ll * (P.la + P.lb) + 4096;
  const MsResult r = ms_first_alignment(env, P.la, P.lb, cutoff, max_steps);
  if (threadIdx.x == 0) out[P.out_idx] = r;
}

}  // namespace

hipError_t launch_misscore(const MsPair* pairs, int n_pairs, const MsDuo* duos, int n_duos, const int32_t* solo,
                           int n_solo, const uint8_t* seqs, uint32_t* nib, int32_t* carry, MsState* stack,
                           int32_t cutoff, MsResult* out, hipStream_t stream, hipEvent_t ev_fill_start,
                           hipEvent_t ev_fill_end) {
  if (n_pairs <= 0) return hipSuccess;
  if (ev_fill_start) (void)hipEventRecord(ev_fill_start, stream);
  if (n_duos > 0) misscore_fill2_kernel<<<(n_duos + 3) / 4, 256, 0, stream>>>(pairs, duos, n_duos, seqs, nib, carry);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  if (n_solo > 0) misscore_fill_kernel<<<(n_solo + 3) / 4, 256, 0, stream>>>(pairs, solo, n_solo, seqs, nib, carry);
  e = hipGetLastError();
  if (e != hipSuccess) return e;
  if (ev_fill_end) (void)hipEventRecord(ev_fill_end, stream);
  // SVS_MS_TB=lane: one lane per pair (the first version; kept as a tested variant)
  const char* tbe = std::getenv("SVS_MS_TB");
  if (tbe && tbe[0] == 'l')
    misscore_traceback_kernel<<<(n_pairs + 63) / 64, 64, 0, stream>>>(pairs, n_pairs, seqs, nib, stack, cutoff, out);
  else
    misscore_traceback_wave_kernel<<<n_pairs, 64, 0, stream>>>(pairs, n_pairs, seqs, nib, stack, cutoff, out);
  return hipGetLastError();
}

}  // namespace svs
