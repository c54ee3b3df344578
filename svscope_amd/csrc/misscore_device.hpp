// Device-side descriptors of the MisScore launch, shared by the host engine
// (svs_misscore_engine.cpp) and the HIP kernels (misscore_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#ifndef SVS_MS_FN
#define SVS_MS_FN inline
#endif
#include "misscore_tb.hpp"

namespace svs {

// One (somatic, germline) consensus pair of a launch.
struct MsPair {
  uint64_t nib_off;    // uint32 words into the nibble buffer (n_strips * n_groups * 64)
  uint64_t stack_off;  // MsState entries into the DFS stack buffer
  uint32_t a_off;      // som bytes in the launch's sequence buffer
  uint32_t b_off;      // ger bytes
  int32_t la, lb;      // lengths (>= 1)
  uint32_t carry_off;  // int32 into the carry buffer (la entries)
  uint32_t stack_cap;  // MsState entries
  int32_t out_idx;     // result slot
  int32_t pad;
};

// Two pairs swept together by the packed int16 fill kernel (y = -1: x alone).
struct MsDuo {
  int32_t x, y;        // indices into the launch's MsPair array
  uint32_t carry_off;  // int32 (two int16 halves) into the carry buffer, max(la) entries
  int32_t pad;
};

// Longest sequence the packed int16 fill takes (|H| <= max(la, lb) < 2^15).
constexpr int32_t kMsPackedMaxLen = 30000;

// 64-step chunks of one strip: la + 63 steps (lane 63 trails lane 0 by 63 rows)
__host__ __device__ inline int32_t ms_chunks(int32_t la) { return (la + 63 + 63) / 64; }
inline uint64_t ms_nib_words(int32_t la, int32_t lb) {
  return static_cast<uint64_t>((lb + 63) / 64) * ms_chunks(la) * 8 * 64;
}
inline uint32_t ms_stack_cap(int32_t la, int32_t lb) { return 2u * static_cast<uint32_t>(la + lb) + 256u; }

// Fills the duos with the packed int16 kernel and the pairs listed in solo
// with the int32 kernel, then runs the traceback of every pair.
hipError_t launch_misscore(const MsPair* pairs, int n_pairs, const MsDuo* duos, int n_duos, const int32_t* solo,
                           int n_solo, const uint8_t* seqs, uint32_t* nib, int32_t* carry, MsState* stack,
                           int32_t cutoff, MsResult* out, hipStream_t stream, hipEvent_t ev_fill_start,
                           hipEvent_t ev_fill_end);

}  // namespace svs
