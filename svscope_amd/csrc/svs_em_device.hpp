// Device-side descriptors for the EM kernels (em_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace svs {

struct EmWindow {
  uint64_t x_off;     // bytes into X (row-major n_reads x n_feat, symbols 0..4)
  uint64_t lab_off;   // int32 into labels: (kmax-1) rows of n_reads fcluster labels (1-based)
  uint64_t ws_off;    // doubles into the workspace
  uint64_t outd_off;  // doubles into outd: (kmax-1) BICs then n_reads per-read likelihoods
  uint64_t outi_off;  // int32 into outi: K, best, status, pad, rng_used lo/hi, Rclust[n_reads]
  uint64_t par_off;   // doubles into the optional parameter dump (gamma | pi | theta of the chosen K)
  int32_t n_reads, n_feat, kmax, zero_params;
};

struct EmConfig {
  int32_t n_step;
  int32_t pad;
  double eps;
};

// Windows of up to kEmLdsReads reads keep gamma and the E-step partial sums
// in LDS; larger ones (deep windows: WindowSelection_v8.py:600 keeps a window
// by its span, not its depth) keep them in the workspace.
constexpr int kEmLdsReads = 256;

// theta per K | LT | gamma per K | pi per K | gsum | A | M | lik per K | XT
// (feature-major reads, nf x round_up(n, 64) bytes) | XR (read-major, n x round_up(nf, 16) bytes)
// [| gamma + E-step partials, 2 x n x 16 doubles, for n > kEmLdsReads]
inline uint64_t em_workspace_doubles(int n, int nf, int kmax) {
  const uint64_t nk = static_cast<uint64_t>(kmax - 1);
  return nk * (nk + 1) / 2 * nf * 5 + nk * nf * 5 + nk * (nk + 1) / 2 * n + nk * (nk + 1) / 2 + 16 +
         2ull * n * 16 + nk * n + 8 + static_cast<uint64_t>(nf) * ((n + 63) / 64) * 8 +
         static_cast<uint64_t>(n) * ((nf + 15) / 16) * 2 + 64 + (n > kEmLdsReads ? 2ull * n * 16 + 8 : 0);
}

hipError_t launch_similarity(const EmWindow* wins, int n, const uint8_t* X, const int64_t* s_off, double* S,
                             hipStream_t stream);
hipError_t launch_em_cluster(const EmWindow* wins, int n, const uint8_t* X, const int32_t* labels,
                             const double* rng, uint64_t rng_len, const EmConfig& cfg, double* ws, double* outd,
                             int32_t* outi, hipStream_t stream);
hipError_t launch_em_gather(const EmWindow* wins, int n, const double* ws, const int32_t* outi, double* par,
                            hipStream_t stream);

}  // namespace svs
