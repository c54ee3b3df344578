// MI355X (gfx950) device half of the strip kernel's row export: for the jobs
// whose graph the host exported lite (PoaGraph::export_strip_lite: in-edge
// rows, per-row words, last-read flags), derive what export_strip_rows'
// passes 2 and 3 and the column-0 fill compute on the host (poa_graph.cpp):
// pool slots and row records w0/w1/w3, the in-edge slots, column 0, and the
// path lengths of w2.  The tables come out identical to the host's; the
// engine can check that (SVS_POA_VERIFY_PREP=1, svs_poa_engine.cpp).
//
// One wave per job.  The row loops are sequential, as on the host (a slot is
// handed out from a LIFO free list in rank order; path lengths are a backward
// DP over the rows), so the wave runs them in lockstep with uniform values:
//  * inputs come through LDS, 64 rows (and their in-edges) per chunk, loaded
//    by all lanes with coalesced loads;
//  * per row, one LDS word holds slot | fewest nodes from a source << 16 in
//    the forward pass, then fewest | most nodes to a sink << 16 backwards;
//  * the free list lives in one VGPR (lane i = entry i, <= 64 entries,
//    host-checked), the row outputs of a chunk in VGPR lanes, stored once per
//    chunk.
// Column 0 follows from the fewest-nodes distance sd alone: with e, c <= 0
// (host-checked) F0 = g + sd e and O0 = q + sd c.
#include <hip/hip_runtime.h>
#include <cstdint>

#include "poa_graph.hpp"
#include "svs_device.hpp"

namespace svs {

namespace {

constexpr uint32_t kChunk = 64;
constexpr uint32_t kChunkEdges = kChunk * 31;  // in-degree <= 31 (host-checked)

__device__ __forceinline__ uint32_t uni(uint32_t x) { return __builtin_amdgcn_readfirstlane(x); }
// lane l of `old` replaced by v (l uniform): one compare and one select
__device__ __forceinline__ int32_t set_lane(int32_t v, uint32_t l, int32_t old) {
  return threadIdx.x == l ? v : old;
}

__global__ __launch_bounds__(64) void poa_strip_prep_kernel(const PoaJob* __restrict__ jobs, PoaScore P,
                                                           uint8_t* __restrict__ base) {
  extern __shared__ uint32_t lds[];
  const uint32_t lane = threadIdx.x;
  const PoaJob J = jobs[blockIdx.x];
  if (!(J.prep & 1u)) return;
  const uint32_t V = J.n_rows;
  const uint32_t* __restrict__ gps = reinterpret_cast<const uint32_t*>(base) + J.pstart_off;
  const uint32_t* __restrict__ gpr = reinterpret_cast<const uint32_t*>(base) + J.pred_off;
  const uint32_t* __restrict__ ginfo = reinterpret_cast<const uint32_t*>(base) + J.info_off;
  uint32_t* __restrict__ rec = reinterpret_cast<uint32_t*>(base) + 4ull * J.rec_off;
  uint32_t* __restrict__ pslot = reinterpret_cast<uint32_t*>(base) + J.pslot_off;
  int32_t* __restrict__ c0 = reinterpret_cast<int32_t*>(base) + 3ull * J.row_off;
  uint32_t* state = lds;                         // V words
  uint32_t* cps = lds + ((V + 3u) & ~3u);        // kChunk + 1 words
  uint32_t* cinfo = cps + kChunk + 4;            // kChunk words
  uint32_t* cedge = cinfo + kChunk;              // <= kChunkEdges words

  // rows r0 .. r0 + n - 1 with their in-edges into LDS; returns n
  auto load_chunk = [&](uint32_t r0) -> uint32_t {
    const uint32_t n = min(kChunk, V - r0);
    __syncthreads();  // the previous chunk's reads are done
    if (lane < n) {
      cps[lane] = gps[r0 + lane];
      cinfo[lane] = ginfo[r0 + lane];
    }
    if (lane == 0) cps[n] = gps[r0 + n];
    __syncthreads();
    const uint32_t e0 = uni(cps[0]), e1 = uni(cps[n]);
    for (uint32_t x = e0 + lane; x < e1; x += 64) cedge[x - e0] = gpr[x];
    __syncthreads();
    return n;
  };

  // forward: pool slots, records w0/w1/w3, in-edge slots, column 0
  uint32_t next = J.prep >> 1, fsp = 0;
  int32_t fstack = 0;               // free list: lane i = entry i
  uint32_t sd_prev = 0;             // sd of the row just above
  int32_t ebuf = 0;                 // in-edge slots of edges ebase + lane
  uint32_t ebase = 0;
  for (uint32_t r0 = 0; r0 < V; r0 += kChunk) {
    const uint32_t n = load_chunk(r0);
    const uint32_t e0 = uni(cps[0]);
    int32_t ow0 = 0, ow1 = 0, ow3 = 0, osd = 0;  // rows r0 + lane
    for (uint32_t i = 0; i < n; ++i) {
      const uint32_t r = r0 + i;
      const uint32_t a = uni(cps[i]), b = uni(cps[i + 1]);
      const uint32_t inf = uni(cinfo[i]);
      uint32_t own = kNoSlot;
      if ((inf >> 9) & 1u) {
        if (fsp != 0) {
          --fsp;
          own = uni(static_cast<uint32_t>(__builtin_amdgcn_readlane(fstack, static_cast<int>(fsp))));
        } else {
          own = next++;
        }
      }
      uint32_t w1 = 0, w3 = 0, sd = 0xFFFFu;
      for (uint32_t x = a; x < b; ++x) {
        const uint32_t pe = uni(cedge[x - e0]);
        const uint32_t pr = (pe & 0x7FFFFFFFu) - 1;
        uint32_t ps, sdp;
        if (pr + 1 == r) {
          ps = kNoSlot;
          sdp = sd_prev;
        } else {
          const uint32_t v = uni(state[pr]);
          ps = v & 0xFFFFu;
          sdp = v >> 16;
        }
        if (x - ebase == 64) {
          pslot[ebase + lane] = static_cast<uint32_t>(ebuf);
          ebase += 64;
        }
        ebuf = set_lane(static_cast<int32_t>(ps), x - ebase, ebuf);
        if (x - a < kInlinePreds) w1 |= ps << (16 * (x - a));
        if (pe >> 31) {  // this row is the tail row's last pool reader: its slot is free again
          fstack = set_lane(static_cast<int32_t>(ps), fsp, fstack);
          ++fsp;
          if (ps < 31u) w3 |= 1u << ps;
        }
        sd = min(sd, sdp + 1);
      }
      if (a == b) sd = 0;  // a source
      if (lane == 0) state[r] = own | (sd << 16);
      sd_prev = sd;
      ow0 = set_lane(static_cast<int32_t>(inf | (own << 16)), i, ow0);
      ow1 = set_lane(static_cast<int32_t>(w1), i, ow1);
      ow3 = set_lane(static_cast<int32_t>(w3), i, ow3);
      osd = set_lane(static_cast<int32_t>(sd), i, osd);
    }
    if (lane < n) {
      const uint64_t r = r0 + lane;
      *reinterpret_cast<uint4*>(rec + 4 * r) =
          make_uint4(static_cast<uint32_t>(ow0), static_cast<uint32_t>(ow1), 0u, static_cast<uint32_t>(ow3));
      const int32_t F0 = P.g + osd * P.e, O0 = P.q + osd * P.c;
      c0[3 * r] = F0 > O0 ? F0 : O0;
      c0[3 * r + 1] = F0;
      c0[3 * r + 2] = O0;
    }
  }
  {
    const uint32_t E = uni(gps[V]);
    if (ebase + lane < E) pslot[ebase + lane] = static_cast<uint32_t>(ebuf);
  }

  // backward: fewest / most nodes on a path to a sink (record word w2); every
  // out-edge leads to a higher rank, so a row is final when the scan reaches it
  __syncthreads();
  for (uint32_t r = lane; r < V; r += 64) state[r] = 0xFFFFu;  // lo 0xFFFF (none seen), hi 0
  for (uint32_t r0 = (V - 1) / kChunk * kChunk;; r0 -= kChunk) {
    const uint32_t n = load_chunk(r0);
    const uint32_t e0 = uni(cps[0]);
    int32_t ow2 = 0;
    for (uint32_t i = n; i-- > 0;) {
      const uint32_t r = r0 + i;
      const uint32_t v = uni(state[r]);
      uint32_t lo = v & 0xFFFFu;
      const uint32_t hi = v >> 16;
      if ((uni(cinfo[i]) >> 8) & 1u) lo = 0;  // a sink
      const uint32_t l1 = min(lo + 1, 0xFFFFu), h1 = min(hi + 1, 0xFFFFu);
      const uint32_t a = uni(cps[i]), b = uni(cps[i + 1]);
      for (uint32_t x = a; x < b; ++x) {
        const uint32_t p = (uni(cedge[x - e0]) & 0x7FFFFFFFu) - 1;
        const uint32_t pv = uni(state[p]);
        const uint32_t plo = min(pv & 0xFFFFu, l1), phi = max(pv >> 16, h1);
        if (lane == 0) state[p] = plo | (phi << 16);
      }
      ow2 = set_lane(static_cast<int32_t>(lo | (hi << 16)), i, ow2);
    }
    if (lane < n) rec[4ull * (r0 + lane) + 2] = static_cast<uint32_t>(ow2);
    if (r0 == 0) break;
  }
}

}  // namespace

size_t strip_prep_lds_bytes(uint32_t max_rows) {
  return 4ull * (((max_rows + 3u) & ~3u) + kChunk + 4 + kChunk + kChunkEdges);
}

hipError_t launch_poa_strip_prep(const PoaJob* jobs, int n_jobs, const PoaScore& score, uint8_t* base,
                                 uint32_t max_rows, hipStream_t stream) {
  if (n_jobs <= 0) return hipSuccess;
  if (max_rows > kStripPrepMaxRows) return hipErrorInvalidValue;
  hipLaunchKernelGGL(poa_strip_prep_kernel, dim3(n_jobs), dim3(64), strip_prep_lds_bytes(max_rows), stream, jobs,
                     score, base);
  return hipGetLastError();
}

}  // namespace svs
