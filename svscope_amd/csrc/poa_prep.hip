// MI355X (gfx950) device half of the strip kernel's row export: for the jobs
// whose graph the host exported lite (PoaGraph::export_strip_lite: in-edge
// rows, per-row words, last-read flags), derive what export_strip_rows'
// passes 2 and 3 and the column-0 fill compute on the host (poa_graph.cpp):
// pool slots and row records w0/w1/w3, the in-edge slots, column 0, and the
// path lengths of w2.  The tables come out identical to the host's; the
// engine can check that (SVS_POA_VERIFY_PREP=1, svs_poa_engine.cpp).
//
// Three waves per job, one per pass (a slot is handed out from a LIFO free
// list in rank order; the path lengths are forward and backward DPs over the
// rows).  The two path-length passes (waves 1 and 2) are lane-parallel per
// 64-row chunk (see there); the slot pass runs its row loop in lockstep with
// uniform values:
//  * inputs come in chunks of 64 rows, loaded by all lanes with coalesced
//    loads one chunk ahead, held in VGPRs (lane i = row r0 + i; the chunk's
//    first 128 in-edges likewise) and read with v_readlane;
//  * the chunk in use keeps its per-row words in a VGPR, and so does the chunk
//    before it (the backward pass: the pushes pending for the chunk after
//    it); finished chunks go to a per-job scratch area for the rarer
//    references more than one chunk back;
//  * the free list lives in one VGPR (lane i = entry i) and, past 64
//    entries, in LDS (up to kStripPrepMaxSlots, host-checked); the row
//    outputs of a chunk in VGPR lanes, stored once per chunk.
// No LDS, so the kernel can share CUs with the other group's DP kernel
// (SVS_POA_PREP_STREAM=1).
// Column 0 follows from the fewest-nodes distance sd alone: with e, c <= 0
// (host-checked) F0 = g + sd e and O0 = q + sd c.
#include <hip/hip_runtime.h>
#include <cstdint>

#include "poa_dgraph.hpp"
#include "poa_graph.hpp"
#include "svs_device.hpp"

// Issue priority of the device-graph prep kernel: the fold waves' (3, ahead
// of the DP waves).  It is the last link of its group's chain DP -> fold ->
// next DP, and the sooner that chain ends, the sooner the group's next DP
// launch starts in the other group's tail: 448.7 / 446.9 vs 439.3 / 440.5
// windows/s at the DP waves' priority 0, prep kernel 4.0 vs 6.4 s per run
// (profiles/r05_pp1).  (In round 3, when the chain ended well inside the other
// group's DP launch, 0 was 1 % faster: profiles/r03_em1.)
#ifndef SVS_PREP_PRIO_LEVEL
#define SVS_PREP_PRIO_LEVEL 3
#endif

namespace svs {

namespace {

constexpr uint32_t kChunk = 64;
constexpr uint32_t kRegEdges = 128;  // in-edges of a chunk held in two VGPRs; more spill to LDS

__device__ __forceinline__ uint32_t uni(uint32_t x) { return __builtin_amdgcn_readfirstlane(x); }
__device__ __forceinline__ uint64_t ballot(bool p) { return __builtin_amdgcn_ballot_w64(p); }
__device__ __forceinline__ uint32_t lane_of(uint32_t v, uint32_t l) {
  return static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int32_t>(v), static_cast<int32_t>(l)));
}
// lane l of `old` replaced by v (l uniform): one compare and one select
__device__ __forceinline__ uint32_t set_lane(uint32_t v, uint32_t l, uint32_t old) {
  return (threadIdx.x & 63u) == l ? v : old;
}

// One chunk of rows r0 .. r0 + n - 1 in registers: lane i holds row r0 + i's
// in-edge start and per-row word, and in-edges e0 + i, e0 + 64 + i (further
// in-edges of a chunk are read from memory).  Loaded one chunk ahead.
struct Chunk {
  uint32_t r0, n, e0, e1;
  uint32_t ps, info, ea, eb;
};

// Three waves per job, one per independent sequential pass:
//  wave 0: pool slots (LIFO free list), record words w0, w1, w3, in-edge slots;
//  wave 1: fewest nodes from a source (sd) -> column 0;
//  wave 2: fewest / most nodes to a sink (backwards) -> record word w2.
// Each keeps the words of its current chunk in a VGPR and writes finished
// chunks to a per-job scratch area (`scr`, 3 words per row) that the rare
// references further back read.
// One job's tables: V rows, in-edge CSR (gps, gpr) and per-row words (ginfo)
// in; records, in-edge slots and column 0 out; per-wave scratch after the
// in-edge slots; pool slots handed out from slot_base.
__device__ void strip_prep_job(const PoaScore& P, uint32_t V, uint32_t slot_base, const uint32_t* __restrict__ gps,
                               const uint32_t* __restrict__ gpr, const uint32_t* __restrict__ ginfo,
                               uint32_t* __restrict__ rec, uint32_t* __restrict__ pslot, int32_t* __restrict__ c0,
                               uint32_t* fl_ext, uint32_t* w2l) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wave = uni(threadIdx.x >> 6);
  // this wave's scratch words, one per row (after the job's in-edge slots)
  uint32_t* scr = pslot + ((uni(gps[V]) + 3u) & ~3u) + static_cast<uint64_t>(wave) * ((V + 3u) & ~3u);
  const uint32_t E = uni(gps[V]);

  auto load = [&](uint32_t r0) -> Chunk {
    Chunk c;
    c.r0 = r0;
    c.n = min(kChunk, V - r0);
    c.e0 = uni(gps[r0]);
    c.e1 = uni(gps[r0 + c.n]);
    c.ps = lane < c.n ? gps[r0 + lane] : 0u;
    c.info = lane < c.n ? ginfo[r0 + lane] : 0u;
    c.ea = c.e0 + lane < c.e1 ? gpr[c.e0 + lane] : 0u;
    c.eb = c.e0 + 64 + lane < c.e1 ? gpr[c.e0 + 64 + lane] : 0u;
    return c;
  };
  auto edge = [&](const Chunk& c, uint32_t x) -> uint32_t {
    const uint32_t i = x - c.e0;
    if (i < 64) return lane_of(c.ea, i);
    if (i < kRegEdges) return lane_of(c.eb, i - 64);
    return uni(gpr[x]);
  };
  auto pstart_of = [&](const Chunk& c, uint32_t i) -> uint32_t { return i < c.n ? lane_of(c.ps, i) : c.e1; };
  // scratch is read back by the wave that wrote it, past the vector L1 (which
  // may hold a line from before the store)
  auto ld = [](const uint32_t* p) -> uint32_t {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  };
  auto flush_fence = [&]() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  };
  // a word more than one chunk back (waves 0, 1): the scratch stores of the
  // finished chunks are drained once, at the first such read after them
  bool dirty = false;
  auto far = [&](uint32_t x) -> uint32_t {
    if (dirty) {
      flush_fence();
      dirty = false;
    }
    return uni(ld(scr + x));
  };

  if (wave == 0) {
    // pool slots, record words w0 w1 w3, in-edge slots
    uint32_t next = slot_base, fsp = 0;
    uint32_t fstack = 0;  // free list: lane i = entry i; entries past 64 in LDS (fl_ext)
    uint32_t ebuf = 0, ebase = 0;  // in-edge slots of edges ebase + lane
    uint32_t pwin = 0;             // lane i: pool slot of row r0 - 64 + i (the chunk before)
    Chunk cur = load(0);
    for (;;) {
      const Chunk nxt = cur.r0 + kChunk < V ? load(cur.r0 + kChunk) : cur;
      uint32_t win = 0;  // lane i: pool slot of row r0 + i
      uint32_t ow0 = 0, ow1 = 0, ow3 = 0;
      for (uint32_t i = 0; i < cur.n; ++i) {
        const uint32_t r = cur.r0 + i;
        const uint32_t a = pstart_of(cur, i), b = pstart_of(cur, i + 1);
        const uint32_t inf = lane_of(cur.info, i);
        uint32_t own = kNoSlot;
        if ((inf >> 9) & 1u) {
          if (fsp != 0) {
            --fsp;
            own = fsp < 64 ? lane_of(fstack, fsp) : uni(fl_ext[fsp - 64]);
          } else {
            own = next++;
          }
        }
        uint32_t w1 = 0, w3 = 0;
        for (uint32_t x = a; x < b; ++x) {
          const uint32_t pe = edge(cur, x);
          const uint32_t pr = (pe & 0x7FFFFFFFu) - 1;
          uint32_t ps = kNoSlot;
          if (pr + 1 != r)
            ps = pr >= cur.r0 ? lane_of(win, pr - cur.r0)
                              : (pr + kChunk >= cur.r0 ? lane_of(pwin, pr + kChunk - cur.r0) : far(pr));
          if (x - ebase == 64) {
            pslot[ebase + lane] = ebuf;
            ebase += 64;
          }
          ebuf = set_lane(ps, x - ebase, ebuf);
          if (x - a < kInlinePreds) w1 |= ps << (16 * (x - a));
          if (pe >> 31) {  // this row is the tail row's last pool reader: its slot is free again
            if (fsp < 64) fstack = set_lane(ps, fsp, fstack);
            else if (lane == 0) fl_ext[fsp - 64] = ps;
            ++fsp;
            if (ps < 31u) w3 |= 1u << ps;
          }
        }
        win = set_lane(own, i, win);
        ow0 = set_lane(inf | (own << 16), i, ow0);
        ow1 = set_lane(w1, i, ow1);
        ow3 = set_lane(w3, i, ow3);
      }
      if (lane < cur.n) {
        const uint64_t r = cur.r0 + lane;
        scr[r] = win;
        *reinterpret_cast<uint2*>(rec + 4 * r) = make_uint2(ow0, ow1);
        rec[4 * r + 3] = ow3;
      }
      dirty = true;
      if (cur.r0 + kChunk >= V) break;
      pwin = win;
      cur = nxt;
    }
    if (ebase + lane < E) pslot[ebase + lane] = ebuf;
  } else if (wave == 1) {
    // fewest nodes from a source -> column 0: F0 = g + sd e, O0 = q + sd c.
    // Lane-parallel per chunk (lane i = row r0 + i), vector issue only:
    // sd[r] = min over in-edges p of sd[p] + 1 (a source: 0).  In-edges from
    // earlier chunks are final and fold into a per-row base; the in-edge from
    // the row just above (the rank chain) makes sd a min-plus scan along
    // chain segments, sd[i] = min over k in [start(i), i] of y[k] + i - k;
    // the other in-edges inside the chunk (merge edges) enter y from the
    // previous estimate, and the chunk repeats until nothing changes.  From
    // all-INF estimates every round is an upper bound and every row is final
    // once its in-chunk merge depth is reached, so the fixed point is the
    // sequential DP's value (an unchanged round is that fixed point).
    const int32_t ilane = static_cast<int32_t>(lane);
    uint32_t pwin = 0;  // lane i: sd of row r0 - 64 + i (the chunk before)
    Chunk cur = load(0);
    for (;;) {
      const Chunk nxt = cur.r0 + kChunk < V ? load(cur.r0 + kChunk) : cur;
      const bool in = lane < cur.n;
      const uint32_t a = in ? cur.ps : 0u;
      const uint32_t bn = static_cast<uint32_t>(__shfl(static_cast<int32_t>(cur.ps), min(ilane + 1, 63), 64));
      const uint32_t b = in ? (lane + 1 < cur.n ? bn : cur.e1) : 0u;
      const uint32_t deg = b - a;
      uint32_t maxdeg = deg;
      for (int o = 32; o >= 1; o >>= 1) maxdeg = max(maxdeg, static_cast<uint32_t>(__shfl_xor(static_cast<int32_t>(maxdeg), o, 64)));
      maxdeg = uni(maxdeg);
      uint32_t base = deg == 0 ? 0u : 0x3FFFFFFFu;  // min over in-edges from earlier chunks (+1)
      bool chain = false;                           // in-edge from the row just above, inside the chunk
      uint32_t q = 0xFFFFFFFFu;                     // up to 4 in-chunk merge in-edges (byte = lane, 0xFF none)
      bool ovf = false;                             // more than 4 of them: re-read each round
      for (uint32_t x = 0; x < maxdeg; ++x) {
        const bool has = x < deg;
        const uint32_t pr = has ? (gpr[a + x] & 0x7FFFFFFFu) - 1u : 0u;
        const bool inchunk = has && pr >= cur.r0;
        const bool prevc = has && !inchunk && pr + kChunk >= cur.r0;
        const bool farp = has && !inchunk && !prevc;
        const uint32_t pv = static_cast<uint32_t>(
            __shfl(static_cast<int32_t>(pwin), prevc ? static_cast<int32_t>(pr + kChunk - cur.r0) : ilane, 64));
        if (prevc) base = min(base, pv + 1u);
        if (ballot(farp)) {
          if (dirty) {
            flush_fence();
            dirty = false;
          }
          if (farp) base = min(base, ld(scr + pr) + 1u);
        }
        if (inchunk) {
          if (pr + 1u == cur.r0 + lane) {
            chain = true;
          } else {
            const uint32_t off = pr - cur.r0;
            if ((q >> 24) != 0xFFu) ovf = true;
            else q = (q << 8) | off;
          }
        }
      }
      // chain segments: lane i's segment starts at the last lane <= i without
      // a chain in-edge
      const uint64_t starts = ballot(!chain);
      const uint64_t upto = starts & (lane == 63u ? ~0ull : ((2ull << lane) - 1ull));
      const int32_t seg0 = 63 - static_cast<int32_t>(__builtin_clzll(upto));  // lane 0 is always a start
      uint32_t sd = 0x3FFFFFFFu;
      const bool any_ovf = ballot(ovf) != 0;
      for (;;) {
        uint32_t y = base;
        for (int k = 0; k < 4; ++k) {
          const uint32_t off = (q >> (8 * k)) & 0xFFu;
          const uint32_t v = static_cast<uint32_t>(
              __shfl(static_cast<int32_t>(sd), off != 0xFFu ? static_cast<int32_t>(off) : ilane, 64));
          if (off != 0xFFu) y = min(y, v + 1u);
        }
        if (any_ovf) {
          for (uint32_t x = 0; x < maxdeg; ++x) {
            const bool has = ovf && x < deg;
            const uint32_t pr = has ? (gpr[a + x] & 0x7FFFFFFFu) - 1u : 0u;
            const bool use = has && pr >= cur.r0 && pr + 1u != cur.r0 + lane;
            const uint32_t v = static_cast<uint32_t>(
                __shfl(static_cast<int32_t>(sd), use ? static_cast<int32_t>(pr - cur.r0) : ilane, 64));
            if (use) y = min(y, v + 1u);
          }
        }
        // segmented min-plus scan: z[i] = y[i] - i, prefix min within the segment, + i
        int32_t z = static_cast<int32_t>(y) - ilane;
        for (int d = 1; d < 64; d <<= 1) {
          const int32_t o = __shfl(z, max(ilane - d, 0), 64);
          if (ilane - d >= seg0) z = min(z, o);
        }
        // (capped at the all-INF start: every round is then <= the last)
        const uint32_t nsd = min(static_cast<uint32_t>(z + ilane), 0x3FFFFFFFu);
        const bool changed = ballot(nsd != sd) != 0;
        sd = nsd;
        if (!changed) break;
      }
      const uint32_t win = in ? sd : 0u;  // lane i: sd of row r0 + i
      if (lane < cur.n) {
        const uint64_t r = cur.r0 + lane;
        scr[r] = win;
        const int32_t F0 = P.g + static_cast<int32_t>(win) * P.e, O0 = P.q + static_cast<int32_t>(win) * P.c;
        c0[3 * r] = F0 > O0 ? F0 : O0;
        c0[3 * r + 1] = F0;
        c0[3 * r + 2] = O0;
      }
      dirty = true;
      if (cur.r0 + kChunk >= V) break;
      pwin = win;
      cur = nxt;
    }
  } else {
    // fewest / most nodes to a sink (record word w2: lo = fewest, 0xFFFF for
    // none; hi = most), backwards over chunks of 64 rows, lane-parallel
    // within a chunk (vector issue only).  A row's successors have higher
    // ranks: those in later chunks pushed into this chunk already (the chunk
    // just after through the LDS window plo/phi, older ones through scratch);
    // inside the chunk, the successor just below on the rank chain makes lo
    // (hi) a min-plus (max-plus) suffix scan along chain segments, and the
    // other in-chunk successors push through LDS atomics from the previous
    // round's estimates, until a round changes nothing (lo falls from 0xFFFF
    // and hi rises from 0, each round a bound on the sequential DP's value,
    // so the fixed point is that value).  Every step saturates at 0xFFFF as
    // the sequential min(x + 1, 0xFFFF) does.
    for (uint32_t r = lane; r < V; r += 64) scr[r] = 0xFFFFu;  // lo 0xFFFF (none seen), hi 0
    uint32_t* clo = w2l;        // this chunk's pushes (lo, atomic min)
    uint32_t* chi = w2l + 64;   // (hi, atomic max)
    uint32_t* plo = w2l + 128;  // pushes into the chunk processed next
    uint32_t* phi = w2l + 192;
    plo[lane] = 0xFFFFu;
    phi[lane] = 0u;
    flush_fence();
    const int32_t ilane = static_cast<int32_t>(lane);
    auto lds_fence = [&]() {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    };
    Chunk cur = load((V - 1) / kChunk * kChunk);
    for (;;) {
      const Chunk nxt = cur.r0 > 0 ? load(cur.r0 - kChunk) : cur;
      const bool in = lane < cur.n;
      const uint32_t sv = in ? ld(scr + cur.r0 + lane) : 0xFFFFu;
      const uint32_t blo = in ? min(sv & 0xFFFFu, plo[lane]) : 0xFFFFu;
      const uint32_t bhi = in ? max(sv >> 16, phi[lane]) : 0u;
      lds_fence();
      plo[lane] = 0xFFFFu;
      phi[lane] = 0u;
      const bool sink = in && ((cur.info >> 8) & 1u);
      const uint32_t a = in ? cur.ps : 0u;
      const uint32_t bn = static_cast<uint32_t>(__shfl(static_cast<int32_t>(cur.ps), min(ilane + 1, 63), 64));
      const uint32_t b = in ? (lane + 1 < cur.n ? bn : cur.e1) : 0u;
      const uint32_t deg = b - a;
      uint32_t maxdeg = deg;
      for (int o = 32; o >= 1; o >>= 1) maxdeg = max(maxdeg, static_cast<uint32_t>(__shfl_xor(static_cast<int32_t>(maxdeg), o, 64)));
      maxdeg = uni(maxdeg);
      // in-edges inside the chunk: the rank chain (from the row just above)
      // and up to four merge edges (byte = lane, 0xFF none; more: re-read)
      bool chain_prev = false, ovf = false;
      uint32_t q = 0xFFFFFFFFu;
      for (uint32_t x = 0; x < maxdeg; ++x) {
        const bool has = x < deg;
        const uint32_t pr = has ? (gpr[a + x] & 0x7FFFFFFFu) - 1u : 0u;
        if (has && pr >= cur.r0) {
          if (pr + 1u == cur.r0 + lane) {
            chain_prev = true;
          } else if ((q >> 24) != 0xFFu) {
            ovf = true;
          } else {
            q = (q << 8) | (pr - cur.r0);
          }
        }
      }
      const bool any_ovf = ballot(ovf) != 0;
      // lane i continues its segment into lane i + 1 when row i + 1's chain
      // in-edge comes from row i
      const bool cnext = __shfl(chain_prev ? 1 : 0, min(ilane + 1, 63), 64) != 0 && lane + 1 < cur.n;
      const uint64_t ends = ballot(!cnext);  // lane 63 always ends a segment
      const int32_t seg1 = static_cast<int32_t>(__builtin_ctzll(ends >> lane)) + ilane;
      uint32_t lo = 0xFFFFu, hi = 0u;
      for (;;) {
        clo[lane] = blo;
        chi[lane] = bhi;
        lds_fence();
        const uint32_t l1 = min(lo + 1u, 0xFFFFu), h1 = min(hi + 1u, 0xFFFFu);
        for (int k = 0; k < 4; ++k) {
          const uint32_t off = (q >> (8 * k)) & 0xFFu;
          if (off != 0xFFu) {
            __hip_atomic_fetch_min(clo + off, l1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            __hip_atomic_fetch_max(chi + off, h1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          }
        }
        if (any_ovf) {
          for (uint32_t x = 0; x < maxdeg; ++x) {
            const bool has = ovf && x < deg;
            const uint32_t pr = has ? (gpr[a + x] & 0x7FFFFFFFu) - 1u : 0u;
            if (has && pr >= cur.r0 && pr + 1u != cur.r0 + lane) {
              __hip_atomic_fetch_min(clo + (pr - cur.r0), l1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
              __hip_atomic_fetch_max(chi + (pr - cur.r0), h1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
          }
        }
        lds_fence();
        const uint32_t pl = sink ? 0u : clo[lane], ph = chi[lane];
        // suffix scans over [i, seg1(i)]: lo = min_k pl[k] + k - i, hi = max_k ph[k] + k - i
        int32_t zl = static_cast<int32_t>(pl) + ilane, zh = static_cast<int32_t>(ph) + ilane;
        for (int d = 1; d < 64; d <<= 1) {
          const int32_t ol = __shfl(zl, min(ilane + d, 63), 64), oh = __shfl(zh, min(ilane + d, 63), 64);
          if (ilane + d <= seg1) {
            zl = min(zl, ol);
            zh = max(zh, oh);
          }
        }
        const uint32_t nlo = in ? min(static_cast<uint32_t>(zl - ilane), 0xFFFFu) : 0xFFFFu;
        const uint32_t nhi = in ? min(static_cast<uint32_t>(zh - ilane), 0xFFFFu) : 0u;
        const bool changed = ballot(nlo != lo || nhi != hi) != 0;
        lo = nlo;
        hi = nhi;
        if (!changed) break;
      }
      if (in) rec[4ull * (cur.r0 + lane) + 2] = lo | (hi << 16);
      // pushes out of the chunk: into the chunk processed next (LDS window),
      // and further back (scratch, one at a time)
      const uint32_t l1 = min(lo + 1u, 0xFFFFu), h1 = min(hi + 1u, 0xFFFFu);
      for (uint32_t x = 0; x < maxdeg; ++x) {
        const bool has = x < deg;
        const uint32_t pr = has ? (gpr[a + x] & 0x7FFFFFFFu) - 1u : 0u;
        const bool prevc = has && pr < cur.r0 && pr + kChunk >= cur.r0;
        const bool farp = has && pr + kChunk < cur.r0;
        if (prevc) {
          __hip_atomic_fetch_min(plo + (pr + kChunk - cur.r0), l1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          __hip_atomic_fetch_max(phi + (pr + kChunk - cur.r0), h1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        uint64_t fm = ballot(farp);
        while (fm) {
          const uint32_t l = static_cast<uint32_t>(__builtin_ctzll(fm));
          fm &= fm - 1;
          const uint32_t p = lane_of(pr, l), ql = lane_of(l1, l), qh = lane_of(h1, l);
          const uint32_t pv = uni(ld(scr + p));
          if (lane == 0) scr[p] = min(pv & 0xFFFFu, ql) | (max(pv >> 16, qh) << 16);
          flush_fence();
        }
      }
      lds_fence();
      if (cur.r0 == 0) break;
      cur = nxt;
    }
  }
}

__global__ __launch_bounds__(192) void poa_strip_prep_kernel(const PoaJob* __restrict__ jobs, PoaScore P) {
  __shared__ uint32_t fl_ext[kStripPrepMaxSlots - 64];
  __shared__ uint32_t w2l[4 * 64];
  const PoaJob J = jobs[blockIdx.x];
  if (!(J.prep & 1u)) return;
  strip_prep_job(P, J.n_rows, J.prep >> 1, J.pstart, J.pred, J.info, const_cast<uint32_t*>(J.rec),
                 const_cast<uint32_t*>(J.pslot), const_cast<int32_t*>(J.col0), fl_ext, w2l);
}

// The same for the device-resident graphs (poa_dgraph.hpp): the jobs whose
// fold exported the next alignment's lite tables into their block.
__global__ __launch_bounds__(192) void poa_dgraph_prep_kernel(const FoldJob* __restrict__ jobs, PoaScore P) {
  __builtin_amdgcn_s_setprio(SVS_PREP_PRIO_LEVEL);
  __shared__ uint32_t fl_ext[kStripPrepMaxSlots - 64];
  __shared__ uint32_t w2l[4 * 64];
  const FoldJob J = jobs[blockIdx.x];
  if (!(J.flags & kFoldExport)) return;
  const FoldResult* res = J.result;
  if (uni(static_cast<uint32_t>(res->status)) != static_cast<uint32_t>(kFoldOk)) return;
  const uint32_t V = uni(res->V);
  if (V == 0 || V > kStripPrepMaxRows || uni(res->n_slots) > kStripPrepMaxSlots || uni(res->max_preds) > kMaxInEdges) return;
  const DGraphLayout L = dgraph_layout(J.cv, J.ce);
  uint8_t* b = J.blk;
  strip_prep_job(P, V, 1u, reinterpret_cast<const uint32_t*>(b + L.pstart), reinterpret_cast<const uint32_t*>(b + L.pred),
                 reinterpret_cast<const uint32_t*>(b + L.info), reinterpret_cast<uint32_t*>(b + L.rec),
                 reinterpret_cast<uint32_t*>(b + L.pslot), reinterpret_cast<int32_t*>(b + L.col0), fl_ext, w2l);
}

}  // namespace

size_t strip_prep_scratch_words(uint32_t V) { return 3ull * ((V + 3u) & ~3u); }

hipError_t launch_poa_strip_prep(const PoaJob* jobs, int n_jobs, const PoaScore& score, uint32_t max_rows,
                                 hipStream_t stream) {
  if (n_jobs <= 0) return hipSuccess;
  if (max_rows > kStripPrepMaxRows) return hipErrorInvalidValue;
  hipLaunchKernelGGL(poa_strip_prep_kernel, dim3(n_jobs), dim3(192), 0, stream, jobs, score);
  return hipGetLastError();
}

hipError_t launch_dgraph_prep(const FoldJob* jobs, int n_jobs, const PoaScore& score, hipStream_t stream) {
  if (n_jobs <= 0) return hipSuccess;
  hipLaunchKernelGGL(poa_dgraph_prep_kernel, dim3(n_jobs), dim3(192), 0, stream, jobs, score);
  return hipGetLastError();
}

}  // namespace svs
