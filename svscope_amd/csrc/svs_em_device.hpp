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

// One window's workspace (offsets in doubles from the window's ws_off; XT/XR
// in bytes): theta, LT, gamma, pi, gsum, A, M and lik of every K (K's block at
// sum_{k<K} k or K - 1 strides), the K-parallel path's per-K record (RNG
// draws, overflow flag), XT (feature-major reads, nf x round_up(n, 64) bytes),
// XR (read-major, n x round_up(nf, 16) bytes), and for n > kEmLdsReads each
// K's gamma + E-step partials (2 x n x 16 doubles).
struct EmWsLayout {
  uint64_t theta, lt, gamma, pi, gsum, A, M, lik, spec, big;  // doubles
  uint64_t xt_bytes, xr_rel;                                     // bytes from the window's base; XR after XT
  uint64_t doubles;                                              // total
};
__host__ __device__ inline EmWsLayout em_ws_layout(int n, int nf, int kmax) {
  const uint64_t N = static_cast<uint64_t>(n), F = static_cast<uint64_t>(nf), nk = static_cast<uint64_t>(kmax - 1);
  const uint64_t tri = nk * (nk + 1) / 2;
  EmWsLayout L{};
  uint64_t o = 0;
  L.theta = o; o += tri * F * 5;
  L.lt = o; o += tri * F * 5;
  L.gamma = o; o += tri * N;
  L.pi = o; o += tri;
  L.gsum = o; o += 16 * nk;
  L.A = o; o += 16 * N * nk;
  L.M = o; o += 16 * N * nk;
  L.lik = o; o += N * nk;
  L.spec = o; o += 2 * nk;
  o = (o + 7) / 8 * 8;  // XT on a 64-byte boundary
  L.xt_bytes = o * 8;
  const uint64_t xt = F * ((N + 63) / 64 * 64), xr = N * ((F + 15) / 16 * 16);
  L.xr_rel = xt;
  o += (xt + xr + 63) / 64 * 8;
  L.big = 0;
  if (n > kEmLdsReads) {
    L.big = o;
    o += 32 * N * nk;
  }
  L.doubles = o;
  return L;
}
inline uint64_t em_workspace_doubles(int n, int nf, int kmax) { return em_ws_layout(n, nf, kmax).doubles; }

hipError_t launch_similarity(const EmWindow* wins, int n, const uint8_t* X, const int64_t* s_off, double* S,
                             hipStream_t stream);
// LDS of one EM workgroup (doubles): gamma (n x nk) and the E-step partials
// (slices x n x nk; a window of up to 64 reads splits its features four ways,
// up to 128 two ways); windows past kEmLdsReads keep both in the workspace.
inline uint64_t em_lds_doubles(int n, int nk) {
  if (n > kEmLdsReads) return 0;
  const int chunks = (n + 63) / 64;
  const int slices = chunks <= 4 ? 4 / chunks : 1;
  return static_cast<uint64_t>(n) * nk * (1 + slices);
}
hipError_t launch_em_cluster(const EmWindow* wins, int n, const uint8_t* X, const int32_t* labels,
                             const double* rng, uint64_t rng_len, const EmConfig& cfg, double* ws, double* outd,
                             int32_t* outi, size_t lds_doubles, hipStream_t stream);
// K-parallel EMCluster (em_x_kernel, em_k_kernel over (window, K), em_select_kernel);
// windows whose RNG draws the speculation could not place get outi[3] = 1 and
// go through launch_em_cluster.  max_nk: the largest kmax - 1 of the windows.
hipError_t launch_em_parallel(const EmWindow* wins, int n, int max_nk, const uint8_t* X, const int32_t* labels,
                              const double* rng, uint64_t rng_len, const EmConfig& cfg, double* ws, double* outd,
                              int32_t* outi, size_t lds_doubles, hipStream_t stream);
hipError_t launch_em_gather(const EmWindow* wins, int n, const double* ws, const int32_t* outi, double* par,
                            hipStream_t stream);

}  // namespace svs
