// MI355X kernels for the read-clustering half of the localGraph hot path:
//   * pairwise read similarity   (ReadsCluster.pariwiseDistance, ReadsCluster.py:44-59)
//   * the categorical mixture EM over K = 1..Kmax-1 with BIC model selection
//     (ReadsCluster.EMCluster :221-277 -> EM :190-209, gamma_updating :132-155,
//      pitheta_updating :162-188, loglik :104-122, BIC :211-219)
// One 256-thread workgroup per window; windows are independent, K values are
// sequential inside a window because numpy's global RNG state (dirichlet
// re-initialisation, :185-187) carries from one K to the next.  The RNG is a
// precomputed legacy-MT19937 exponential table (host side, bitwise numpy);
// each window consumes it from offset 0 (per-window reseed contract).
//
// fp64 throughout.  Reduction orders follow numpy where the reference uses
// plain reductions (gamma.sum(axis=0) row by row, the K-wide exp-sum pairwise,
// Rlik.sum() pairwise); the BLAS dot products are summed in feature order.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdlib>

#include "svs_em_device.hpp"

namespace svs {

__device__ __forceinline__ double clip_eps(double x, double eps) {
  return fmin(fmax(x, eps), 1.0 - eps);
}

// numpy pairwise_sum_DOUBLE for n <= 128 (8 accumulators) with the n < 8 path.
__device__ double np_pairwise_small(const double* a, int n, int stride) {
  if (n < 8) {
    double r = 0.0;
    for (int i = 0; i < n; ++i) r += a[i * stride];
    return r;
  }
  double r[8];
  for (int j = 0; j < 8; ++j) r[j] = a[j * stride];
  int i = 8;
  for (; i < n - (n % 8); i += 8)
    for (int j = 0; j < 8; ++j) r[j] += a[(i + j) * stride];
  double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
  for (; i < n; ++i) res += a[i * stride];
  return res;
}

// numpy pairwise sum for n > 128 (iterative form of the recursive split).
__device__ __noinline__ double np_pairwise_large(const double* a, int n) {
  // explicit stack of (offset, length, stage)
  int off[32], len[32];
  double part[32];
  int st[32];
  int sp = 0;
  off[0] = 0; len[0] = n; st[0] = 0;
  double ret = 0.0;
  while (sp >= 0) {
    const int o = off[sp], l = len[sp];
    if (l <= 128) {
      ret = np_pairwise_small(a + o, l, 1);
      --sp;
      // deliver ret to parent
      while (sp >= 0) {
        if (st[sp] == 1) { part[sp] = ret; st[sp] = 2; break; }
        ret = part[sp] + ret;  // st == 2: left + right
        --sp;
      }
      if (sp < 0) break;
      // parent now needs its right half
      int n2 = len[sp] / 2; n2 -= n2 % 8;
      ++sp; off[sp] = off[sp - 1] + n2; len[sp] = len[sp - 1] - n2; st[sp] = 0;
      continue;
    }
    int n2 = l / 2; n2 -= n2 % 8;
    st[sp] = 1;
    ++sp; off[sp] = o; len[sp] = n2; st[sp] = 0;
  }
  return ret;
}

__global__ __launch_bounds__(256) void similarity_kernel(const EmWindow* __restrict__ wins,
                                                         const uint8_t* __restrict__ X,
                                                         const int64_t* __restrict__ s_off,
                                                         double* __restrict__ S) {
  const EmWindow W = wins[blockIdx.x];
  const int N = W.n_reads, nf = W.n_feat;
  const uint8_t* x = X + W.x_off;
  double* s = S + s_off[blockIdx.x];
  const double total = nf == 0 ? 1.0 : static_cast<double>(nf);
  for (int p = threadIdx.x; p < N * N; p += blockDim.x) {
    const int i = p / N, j = p % N;
    if (i == j) { s[p] = 1.0; continue; }
    if (j < i) continue;
    int cnt = 0;
    const uint8_t* a = x + static_cast<int64_t>(i) * nf;
    const uint8_t* b = x + static_cast<int64_t>(j) * nf;
    for (int f = 0; f < nf; ++f) cnt += a[f] == b[f];
    const double v = cnt / total;
    s[p] = v;
    s[j * N + i] = v;
  }
}

__device__ __forceinline__ double np_pairwise(const double* a, int n) {
  return n <= 128 ? np_pairwise_small(a, n, 1) : np_pairwise_large(a, n);
}

// Five named accumulators selected by symbol (avoids a runtime-indexed array).
struct Acc5 {
  double v0 = 0.0, v1 = 0.0, v2 = 0.0, v3 = 0.0, v4 = 0.0;
  __device__ __forceinline__ void add(uint8_t a, double x) {
    v0 += a == 0 ? x : 0.0;
    v1 += a == 1 ? x : 0.0;
    v2 += a == 2 ? x : 0.0;
    v3 += a == 3 ? x : 0.0;
    v4 += a == 4 ? x : 0.0;
  }
};

// numpy's pairwise sum over the K (<= 16) terms exp(clip(M[j] - mi, +-700)).
__device__ __forceinline__ double exp_row_sum(const double* Mi, int K, double mi) {
  auto t = [&](int j) { return exp(fmin(fmax(Mi[j] - mi, -700.0), 700.0)); };
  if (K < 8) {
    double r = 0.0;
    for (int j = 0; j < K; ++j) r += t(j);
    return r;
  }
  double r0 = t(0), r1 = t(1), r2 = t(2), r3 = t(3), r4 = t(4), r5 = t(5), r6 = t(6), r7 = t(7);
  int j = 8;
  if (K == 16) {
    r0 += t(8); r1 += t(9); r2 += t(10); r3 += t(11); r4 += t(12); r5 += t(13); r6 += t(14); r7 += t(15);
    j = 16;
  }
  double res = ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7));
  for (; j < K; ++j) res += t(j);
  return res;
}

struct EmShared {
  int reinit;
  int error;
  uint64_t rng_off;
};

// K = 1..max_C with max_C <= 15 (host check in svs_em_engine.cpp): gamma, A and M rows are 16 wide

// gamma staged for the M-step, E-step partial sums (4/chunks feature slices x
// N reads x K): LDS for windows of up to kEmLdsReads reads, workspace beyond.
struct EmLds {
  double* g;
  double* part;
};

__device__ __forceinline__ int read_pad(int N) { return (N + 63) & ~63; }

// M-step (pitheta_updating :162-188).  One thread per feature f: its 64 read
// symbols come from the feature-major XT row (four 16-B loads), gamma from
// LDS; theta[k][f][a] = sum_i gamma[i,k] [x_if == a] / gsum[k] for every k,
// and LT[(f*5 + a)*K + k] = log(clip(theta)) for the E-step's gathers.
__device__ void m_step(const EmWindow& W, int K, const uint8_t* __restrict__ xt, const double* __restrict__ g,
                       double* __restrict__ pi, double* __restrict__ gsum, double* __restrict__ th,
                       double* __restrict__ lt, const double* __restrict__ rng, uint64_t rng_len, double eps,
                       EmShared* sh, EmLds* L) {
  const int N = W.n_reads, nf = W.n_feat, tid = threadIdx.x;
  if (tid < K) {
    double s = 0.0;
    for (int i = 0; i < N; ++i) s += g[i * K + tid];  // numpy axis-0 reduction: row by row
    gsum[tid] = s;
    pi[tid] = s / N;
  }
  for (int r = tid; r < N * K; r += blockDim.x) L->g[r] = g[r];
  __syncthreads();
  if (tid == 0) {
    int bad = 0;
    for (int k = 0; k < K; ++k) bad |= (pi[k] * N < 1.0) || isnan(pi[k]);
    sh->reinit = bad;
    if (bad) {
      const uint64_t need = static_cast<uint64_t>(K) * nf * 5;
      if (sh->rng_off + need > rng_len) sh->error = 1;
    }
  }
  __syncthreads();
  if (sh->reinit) {
    if (tid < K) pi[tid] = 1.0 / K;
    if (!sh->error) {
      const double* e = rng + sh->rng_off;
      for (int r = tid; r < K * nf; r += blockDim.x) {
        const double e0 = e[5 * r], e1 = e[5 * r + 1], e2 = e[5 * r + 2], e3 = e[5 * r + 3], e4 = e[5 * r + 4];
        const double inv = 1.0 / ((((e0 + e1) + e2) + e3) + e4);
        const double t5[5] = {e0 * inv, e1 * inv, e2 * inv, e3 * inv, e4 * inv};
        double* t = th + 5 * static_cast<int64_t>(r);
        const int k = r / nf, f = r % nf;
        for (int a = 0; a < 5; ++a) {
          t[a] = t5[a];
          lt[(static_cast<int64_t>(f) * 5 + a) * K + k] = log(clip_eps(t5[a], eps));
        }
      }
    }
    __syncthreads();
    if (tid == 0) sh->rng_off += static_cast<uint64_t>(K) * nf * 5;
  } else {
    const int NP = read_pad(N);
    for (int f = tid; f < nf; f += blockDim.x) {
      for (int k = 0; k < K; ++k) {
        Acc5 acc;
        // 16 reads at a time: one 16-B load of the feature row (L1-resident
        // across the k loop), symbols unpacked from registers
        const uint4* row = reinterpret_cast<const uint4*>(xt + static_cast<int64_t>(f) * NP);
        for (int h = 0; h * 16 < N; ++h) {
          const uint4 q = row[h];
          const uint32_t xw[4] = {q.x, q.y, q.z, q.w};
          const double* gc = L->g + (h * 16) * K + k;
#pragma unroll
          for (int i = 0; i < 16; ++i)
            if (h * 16 + i < N) acc.add(static_cast<uint8_t>(xw[i >> 2] >> (8 * (i & 3))), gc[i * K]);
        }
        const double d = gsum[k];
        const double t5[5] = {acc.v0 / d, acc.v1 / d, acc.v2 / d, acc.v3 / d, acc.v4 / d};
        double* t = th + 5 * (static_cast<int64_t>(k) * nf + f);
        for (int a = 0; a < 5; ++a) {
          t[a] = t5[a];
          lt[(static_cast<int64_t>(f) * 5 + a) * K + k] = log(clip_eps(t5[a], eps));
        }
      }
    }
  }
  __syncthreads();
}

// Sum over features [f0, f1) of LT[(f*5 + x_if)*K + k] for one read (its
// padded read-major symbol row xi), k = 0..K-1, into out[0..K-1].
template <int K>
__device__ __forceinline__ void e_accumulate(const uint8_t* __restrict__ xi, const double* __restrict__ lt, int f0,
                                             int f1, double* __restrict__ out) {
  double acc[K];
#pragma unroll
  for (int k = 0; k < K; ++k) acc[k] = 0.0;
  int c = f0;
  for (; c + 16 <= f1; c += 16) {
    const uint4 q = *reinterpret_cast<const uint4*>(xi + c);
    const uint32_t xw[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
    for (int b = 0; b < 16; ++b) {
      const int a = (xw[b >> 2] >> (8 * (b & 3))) & 0xFF;
      const double* row = lt + (static_cast<int64_t>(c + b) * 5 + a) * K;
#pragma unroll
      for (int k = 0; k < K; ++k) acc[k] += row[k];
    }
  }
  for (; c < f1; ++c) {
    const int a = xi[c];
    const double* row = lt + (static_cast<int64_t>(c) * 5 + a) * K;
#pragma unroll
    for (int k = 0; k < K; ++k) acc[k] += row[k];
  }
#pragma unroll
  for (int k = 0; k < K; ++k) out[k] = acc[k];
}

// The same contraction on the matrix cores (SVS_EM_MFMA=1 variant):
// A[i,k] = sum over the 5 nf one-hot columns (f, a) of [x_if == a] LT[(f,a), k],
// a dense (N x 5nf) . (5nf x K) product of v_mfma_f64_16x16x4_f64 tiles, one
// 16-read tile per wave at a time, K padded to 16 columns.  Operand maps
// (gfx950, one f64 per lane): A[i = l&15][kk = l>>4], B[kk = l>>4][j = l&15];
// result D[row = (l>>4) + 4 r][col = l&15], r = 0..3.  Four of every five
// products are with a one-hot zero and K <= 9 of the 16 columns are real:
// the work is ~9x the gather's, kept as the measured alternative
// (DESIGN.md §4.3).
typedef double svs_f64x4 __attribute__((ext_vector_type(4)));
__device__ void e_accumulate_mfma(const EmWindow& W, int K, const uint8_t* __restrict__ xr,
                                  const double* __restrict__ lt, double* __restrict__ out) {
  const int N = W.n_reads, nf = W.n_feat, tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int nfp = (nf + 15) & ~15;
  const int kd = 5 * nf;                       // contraction length
  const int kq = lane >> 4, col = lane & 15;   // this lane's k-slot and A row / B column
  for (int tile = wave; tile * 16 < N; tile += 4) {
    const int i = tile * 16 + col;             // A row (read) of this lane
    const uint8_t* xi = xr + static_cast<int64_t>(i < N ? i : 0) * nfp;
    svs_f64x4 acc = {0.0, 0.0, 0.0, 0.0};
    for (int base = 0; base < kd; base += 4) {
      const int kk = base + kq;                // one-hot column (f, a) = (kk / 5, kk % 5)
      const int f = kk / 5, a = kk - 5 * f;
      const double av = (i < N && kk < kd && xi[f] == a) ? 1.0 : 0.0;
      const double bv = (col < K && kk < kd) ? lt[static_cast<int64_t>(kk) * K + col] : 0.0;
      acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc, 0, 0, 0);
    }
    if (col < K) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = tile * 16 + kq + 4 * r;
        if (row < N) out[row * K + col] = acc[r];
      }
    }
  }
}

// E-step (gamma_updating :132-155) + the feature part of loglik,
// A[i,k] = sum_f log theta'[k,f,x_if].  Lane = read, each of the 4 waves sums
// a quarter of the features (gathers LT rows (f, x_if) of K contiguous
// doubles), then the quarters are added in wave order.
template <bool MFMA, int KC>
__device__ void e_step(const EmWindow& W, int K, const uint8_t* __restrict__ xr, const double* __restrict__ pi,
                       const double* __restrict__ lt, double* __restrict__ A, double* __restrict__ M,
                       double* __restrict__ g, EmLds* L) {
  const int N = W.n_reads, nf = W.n_feat, tid = threadIdx.x;
  if constexpr (MFMA) {
    e_accumulate_mfma(W, K, xr, lt, L->part);
    __syncthreads();
    for (int r = tid; r < N * K; r += blockDim.x) {
      A[r] = L->part[r];
      M[r] = L->part[r] + log(pi[r % K]);
    }
    __syncthreads();
    for (int r = tid; r < N * K; r += blockDim.x) {
      const int i = r / K, I = r % K;
      g[r] = 1.0 / exp_row_sum(M + i * K, K, M[i * K + I]);
    }
    __syncthreads();
    return;
  }
  const int lane = tid & 63, wave = tid >> 6;
  const int NP = read_pad(N), chunks = NP >> 6;       // 64-read chunks
  // up to 4 chunks: every wave one chunk and a 4/chunks share of the
  // features; more: every wave whole reads of chunks wave, wave + 4, ...
  const int slices = chunks <= 4 ? 4 / chunks : 1;    // feature slices per chunk
  // feature slices in whole 16-feature blocks: one 16-B load of the read's
  // symbols, then 16 x K independent LT gathers in flight (K is a template
  // constant so the loads are not split by per-k branches)
  const int nfp = (nf + 15) & ~15;
  const int fs = ((nfp / 16 + slices - 1) / slices) * 16;
  for (int c = chunks <= 4 ? wave % chunks : wave; c < chunks; c += chunks <= 4 ? chunks : 4) {
    const int slice = chunks <= 4 ? wave / chunks : 0;
    const int i = c * 64 + lane;
    if (slice < slices && i < N) {
      const int f0 = slice * fs, f1 = min(nf, f0 + fs);
      const uint8_t* xi = xr + static_cast<int64_t>(i) * nfp;
      double* out = L->part + (slice * N + i) * K;
      // (cases up to KC only: the launch's largest K; the register count of
      // the kernel is that of its largest case)
      switch (K) {
#define SVS_EK(KK) case KK: if constexpr (KK <= KC) e_accumulate<KK>(xi, lt, f0, f1, out); break;
        SVS_EK(1) SVS_EK(2) SVS_EK(3) SVS_EK(4) SVS_EK(5) SVS_EK(6) SVS_EK(7) SVS_EK(8)
        SVS_EK(9) SVS_EK(10) SVS_EK(11) SVS_EK(12) SVS_EK(13) SVS_EK(14) SVS_EK(15)
#undef SVS_EK
        default: break;
      }
    }
    if (chunks <= 4) break;
  }
  __syncthreads();
  for (int r = tid; r < N * K; r += blockDim.x) {
    double a_ik = L->part[r];
    for (int sl = 1; sl < slices; ++sl) a_ik += L->part[sl * N * K + r];
    A[r] = a_ik;
    M[r] = a_ik + log(pi[r % K]);
  }
  __syncthreads();
  for (int r = tid; r < N * K; r += blockDim.x) {
    const int i = r / K, I = r % K;
    g[r] = 1.0 / exp_row_sum(M + i * K, K, M[i * K + I]);
  }
  __syncthreads();
}

// One window's workspace for one K (em_ws_layout): every K has its own
// theta, LT, gamma, pi, gsum, A, M, lik and deep-window scratch, so the K
// values of a window can also run in parallel workgroups (em_k_kernel).
struct EmK {
  double *th, *lt, *g, *pi, *gsum, *A, *M, *lik, *big;
};
__device__ __forceinline__ EmK em_k_ptrs(const EmWindow& W, double* ws, int K) {
  const EmWsLayout L = em_ws_layout(W.n_reads, W.n_feat, W.kmax);
  double* b = ws + W.ws_off;
  const int64_t kk = static_cast<int64_t>(K) * (K - 1) / 2;  // sum_{k<K} k
  const int64_t N = W.n_reads, nf = W.n_feat;
  EmK e;
  e.th = b + L.theta + kk * nf * 5;
  e.lt = b + L.lt + kk * nf * 5;
  e.g = b + L.gamma + kk * N;
  e.pi = b + L.pi + kk;
  e.gsum = b + L.gsum + 16 * (K - 1);
  e.A = b + L.A + 16 * N * (K - 1);
  e.M = b + L.M + 16 * N * (K - 1);
  e.lik = b + L.lik + N * (K - 1);
  e.big = L.big ? b + L.big + 32 * N * (K - 1) : nullptr;
  return e;
}

// feature-major copy of the reads: XT[f][i] (row stride N rounded up to 64),
// pad symbol 5 for i >= N; then the read-major copy with rows padded to 16
// features (16-B aligned loads)
__device__ void em_build_x(const EmWindow& W, const uint8_t* __restrict__ x, uint8_t* __restrict__ xt,
                           uint8_t* __restrict__ xr) {
  const int N = W.n_reads, nf = W.n_feat, tid = threadIdx.x;
  const int NP = read_pad(N);
  for (int64_t r = tid; r < static_cast<int64_t>(nf) * NP; r += blockDim.x) {
    const int f = static_cast<int>(r / NP), i = static_cast<int>(r % NP);
    xt[r] = i < N ? x[static_cast<int64_t>(i) * nf + f] : 5;
  }
  const int nfp = (nf + 15) & ~15;
  for (int64_t r = tid; r < static_cast<int64_t>(N) * nfp; r += blockDim.x) {
    const int i = static_cast<int>(r / nfp), f = static_cast<int>(r % nfp);
    xr[r] = f < nf ? x[static_cast<int64_t>(i) * nf + f] : 0;
  }
}

// EM for one K (EMCluster's loop body :245-256, EM :190-209), NaN retries
// included; the workgroup's RNG position is sh->rng_off.  bic[K-1] is written.
template <bool MFMA, int KC>
__device__ void em_run_k(const EmWindow& W, int K, const EmK& P, const uint8_t* __restrict__ xt,
                         const uint8_t* __restrict__ xr, const int32_t* __restrict__ lab,
                         const double* __restrict__ rng, uint64_t rng_len, const EmConfig& cfg, EmShared* sh,
                         EmLds* lds, double* __restrict__ bic) {
  const int N = W.n_reads, nf = W.n_feat, tid = threadIdx.x;
  const double logN = log(static_cast<double>(N));
  const int32_t* lk = lab + static_cast<int64_t>(K - 1) * N;
  double b0 = NAN;
  for (int tries = 5; isnan(b0) && tries != 0; --tries) {
    for (int r = tid; r < N * K; r += blockDim.x) P.g[r] = (lk[r / K] - 1 == r % K) ? 1.0 : 0.0;
    __syncthreads();
    m_step(W, K, xt, P.g, P.pi, P.gsum, P.th, P.lt, rng, rng_len, cfg.eps, sh, lds);
    e_step<MFMA, KC>(W, K, xr, P.pi, P.lt, P.A, P.M, P.g, lds);
    for (int it = 0; it < cfg.n_step; ++it) {
      m_step(W, K, xt, P.g, P.pi, P.gsum, P.th, P.lt, rng, rng_len, cfg.eps, sh, lds);
      e_step<MFMA, KC>(W, K, xr, P.pi, P.lt, P.A, P.M, P.g, lds);
      for (int i = tid; i < N; i += blockDim.x) {
        double s = 0.0;
        for (int k = 0; k < K; ++k) s += (P.A[i * K + k] + log(clip_eps(P.pi[k], cfg.eps))) * P.g[i * K + k];
        P.lik[i] = s;
      }
      __syncthreads();
    }
    // BIC with ZeroParamNum = 0 decides the NaN retry (EMCluster :249-252)
    const double tot = np_pairwise(P.lik, N);
    b0 = 2.0 * tot - static_cast<double>(K - 1 + static_cast<int64_t>(K) * nf * 4) * logN;
    __syncthreads();
  }
  if (tid == 0) {
    const double tot = np_pairwise(P.lik, N);
    bic[K - 1] = 2.0 * tot - static_cast<double>(K - 1 + static_cast<int64_t>(K) * nf * 4 - W.zero_params) * logN;
  }
  __syncthreads();
}

// Model selection (EMCluster :258-277) by one thread: the best BIC, the K = 1
// rule, labels of the chosen K and its per-read likelihoods.
__device__ void em_select(const EmWindow& W, double* ws, double* __restrict__ outd, int32_t* __restrict__ outi,
                          uint64_t rng_off, bool error) {
  const int N = W.n_reads, nf = W.n_feat, nk = W.kmax - 1;
  double* bic = outd + W.outd_off;  // nk BICs, then N lik of the chosen K
  int32_t* oi = outi + W.outi_off;  // [K, best, status, rerun, rng_used(lo), rng_used(hi), Rclust[N]]
  const double logN = log(static_cast<double>(N));
  int best = -1;
  for (int k = 0; k < nk; ++k)
    if (!isnan(bic[k]) && (best < 0 || bic[k] > bic[best])) best = k;
  int status = error ? 2 : 0;
  if (best < 0) status = 3;  // nanargmax of an all-NaN list (numpy raises)
  int K = best + 1;
  if (status == 0 && K == 1) {
    if (nk < 2) status = 4;  // reference indexes BICList[1] (IndexError)
    else if (bic[0] - bic[1] <= nf * logN) { K = 2; best = 1; }
  }
  oi[0] = K;
  oi[1] = best;
  oi[2] = status;
  oi[3] = 0;
  oi[4] = static_cast<int32_t>(rng_off & 0xFFFFFFFFu);
  oi[5] = static_cast<int32_t>(rng_off >> 32);
  if (status == 0) {
    const EmK P = em_k_ptrs(W, ws, K);
    for (int i = 0; i < N; ++i) {
      int am = 0;
      for (int k = 1; k < K; ++k)
        if (P.g[i * K + k] > P.g[i * K + am]) am = k;
      oi[6 + i] = am;
      bic[nk + i] = P.lik[i];
    }
  }
}

// gamma / E-step partials: LDS, or (deep windows) the K's workspace scratch
__device__ __forceinline__ EmLds em_lds(const EmWindow& W, const EmK& P, double* lds_dyn) {
  const int N = W.n_reads;
  if (N > kEmLdsReads) return EmLds{P.big, P.big + static_cast<int64_t>(N) * 16};
  return EmLds{lds_dyn, lds_dyn + static_cast<int64_t>(N) * (W.kmax - 1)};
}

// The whole EMCluster of a window in one workgroup, K = 1..kmax-1 in order
// with one RNG stream (the reference's order; also the fallback of the
// K-parallel path below).
template <bool MFMA>
__global__ __launch_bounds__(256) void em_cluster_kernel(const EmWindow* __restrict__ wins,
                                                         const uint8_t* __restrict__ X,
                                                         const int32_t* __restrict__ labels,
                                                         const double* __restrict__ rng, uint64_t rng_len,
                                                         EmConfig cfg, double* __restrict__ ws,
                                                         double* __restrict__ outd, int32_t* __restrict__ outi) {
  __shared__ EmShared sh;
  // gamma and the E-step partials of windows up to kEmLdsReads reads, sized by
  // the launch to its largest window (em_lds_doubles): a config-3 window takes
  // 23 KB instead of a fixed 60 KB, so an EM workgroup fits beside the DP
  // kernel's workgroups on a CU instead of displacing one
  extern __shared__ double lds_dyn[];
  const EmWindow W = wins[blockIdx.x];
  const EmWsLayout L = em_ws_layout(W.n_reads, W.n_feat, W.kmax);
  uint8_t* xt = reinterpret_cast<uint8_t*>(ws + W.ws_off) + L.xt_bytes;
  uint8_t* xr = xt + L.xr_rel;
  em_build_x(W, X + W.x_off, xt, xr);
  if (threadIdx.x == 0) { sh.rng_off = 0; sh.error = 0; sh.reinit = 0; }
  __threadfence_block();
  __syncthreads();
  const int nk = W.kmax - 1;
  for (int K = 1; K <= nk; ++K) {
    const EmK P = em_k_ptrs(W, ws, K);
    EmLds lds = em_lds(W, P, lds_dyn);
    em_run_k<MFMA, 15>(W, K, P, xt, xr, labels + W.lab_off, rng, rng_len, cfg, &sh, &lds, outd + W.outd_off);
  }
  if (threadIdx.x == 0) em_select(W, ws, outd, outi, sh.rng_off, sh.error != 0);
}

// K-parallel path.  The K values of a window depend on each other only through
// the RNG stream: K draws from it (a dirichlet re-initialisation) at the
// position the smaller K left it.  em_k_kernel runs every (window, K) in its
// own workgroup from position 0 and records how much it drew; em_select_kernel
// accepts a window when no K drew after an earlier K had drawn (then every
// draw happened at the position the sequential order gives it, and the
// results are the sequential kernel's), and flags the others for a rerun in
// order (oi[3] = 1, em_cluster_kernel on those windows).
__global__ __launch_bounds__(256) void em_x_kernel(const EmWindow* __restrict__ wins, const uint8_t* __restrict__ X,
                                                   double* __restrict__ ws) {
  const EmWindow W = wins[blockIdx.x];
  const EmWsLayout L = em_ws_layout(W.n_reads, W.n_feat, W.kmax);
  uint8_t* xt = reinterpret_cast<uint8_t*>(ws + W.ws_off) + L.xt_bytes;
  em_build_x(W, X + W.x_off, xt, xt + L.xr_rel);
}

// Held to 6 waves per SIMD (80 VGPRs; the gathers' load batches shrink and a
// few values spill to scratch): an EM wave then takes about one DP wave's
// registers (72) instead of 125, and the EM kernel time of the driver's run
// falls from 4.8-5.0 to 3.4-3.5 s with windows/s and the DP busy frac within
// the spread (446.4 vs 444.9 / 441.9 windows/s, frac 0.460 vs 0.453 / 0.456,
// profiles/r06_em2; 5 waves, 96 VGPRs: 3.7-3.9 s, r06_em1).  SVS_EM_OCC
// overrides it in development builds.
#ifndef SVS_EM_OCC
#define SVS_EM_OCC 6
#endif
template <bool MFMA, int KC>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(SVS_EM_OCC))) void em_k_kernel(const EmWindow* __restrict__ wins,
                                                   const int32_t* __restrict__ labels,
                                                   const double* __restrict__ rng, uint64_t rng_len, EmConfig cfg,
                                                   double* __restrict__ ws, double* __restrict__ outd) {
  __shared__ EmShared sh;
  extern __shared__ double lds_dyn[];
  const EmWindow W = wins[blockIdx.x];
  const int K = static_cast<int>(blockIdx.y) + 1;
  if (K > W.kmax - 1) return;
  const EmWsLayout L = em_ws_layout(W.n_reads, W.n_feat, W.kmax);
  const uint8_t* xt = reinterpret_cast<const uint8_t*>(ws + W.ws_off) + L.xt_bytes;
  const EmK P = em_k_ptrs(W, ws, K);
  EmLds lds = em_lds(W, P, lds_dyn);
  if (threadIdx.x == 0) { sh.rng_off = 0; sh.error = 0; sh.reinit = 0; }
  __threadfence_block();
  __syncthreads();
  em_run_k<MFMA, KC>(W, K, P, xt, xt + L.xr_rel, labels + W.lab_off, rng, rng_len, cfg, &sh, &lds, outd + W.outd_off);
  if (threadIdx.x == 0) {
    uint64_t* spec = reinterpret_cast<uint64_t*>(ws + W.ws_off + L.spec) + 2 * (K - 1);
    spec[0] = sh.rng_off;
    spec[1] = static_cast<uint64_t>(sh.error);
  }
}

__global__ __launch_bounds__(64) void em_select_kernel(const EmWindow* __restrict__ wins, int n,
                                                       double* __restrict__ ws, double* __restrict__ outd,
                                                       int32_t* __restrict__ outi) {
  const int w = blockIdx.x * 64 + static_cast<int>(threadIdx.x);
  if (w >= n) return;
  const EmWindow W = wins[w];
  const EmWsLayout L = em_ws_layout(W.n_reads, W.n_feat, W.kmax);
  const uint64_t* spec = reinterpret_cast<const uint64_t*>(ws + W.ws_off + L.spec);
  uint64_t off = 0;
  bool ok = true, error = false;
  for (int K = 1; K <= W.kmax - 1; ++K) {
    const uint64_t used = spec[2 * (K - 1)];
    if (used != 0 && off != 0) ok = false;  // K drew from a position the speculation did not start it at
    error |= spec[2 * (K - 1) + 1] != 0;
    off += used;
  }
  if (!ok) {
    outi[W.outi_off + 3] = 1;
    return;
  }
  em_select(W, ws, outd, outi, off, error);
}

hipError_t launch_similarity(const EmWindow* wins, int n, const uint8_t* X, const int64_t* s_off, double* S,
                             hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(similarity_kernel, dim3(n), dim3(256), 0, stream, wins, X, s_off, S);
  return hipGetLastError();
}

hipError_t launch_em_cluster(const EmWindow* wins, int n, const uint8_t* X, const int32_t* labels,
                             const double* rng, uint64_t rng_len, const EmConfig& cfg, double* ws, double* outd,
                             int32_t* outi, size_t lds_doubles, hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  const size_t lds = lds_doubles * sizeof(double);
  // SVS_EM_MFMA=1: the E-step contraction on v_mfma_f64_16x16x4_f64 (measured
  // alternative, see e_accumulate_mfma); default: the one-hot gather
  const char* me = std::getenv("SVS_EM_MFMA");  // read per launch (a few per batch): tests switch it
  const bool mfma = me && me[0] == '1';
  if (mfma)
    hipLaunchKernelGGL(em_cluster_kernel<true>, dim3(n), dim3(256), lds, stream, wins, X, labels, rng, rng_len, cfg,
                       ws, outd, outi);
  else
    hipLaunchKernelGGL(em_cluster_kernel<false>, dim3(n), dim3(256), lds, stream, wins, X, labels, rng, rng_len, cfg,
                       ws, outd, outi);
  return hipGetLastError();
}

hipError_t launch_em_parallel(const EmWindow* wins, int n, int max_nk, const uint8_t* X, const int32_t* labels,
                              const double* rng, uint64_t rng_len, const EmConfig& cfg, double* ws, double* outd,
                              int32_t* outi, size_t lds_doubles, hipStream_t stream) {
  if (n <= 0 || max_nk <= 0) return hipSuccess;
  const size_t lds = lds_doubles * sizeof(double);
  const char* me = std::getenv("SVS_EM_MFMA");
  const bool mfma = me && me[0] == '1';
  hipLaunchKernelGGL(em_x_kernel, dim3(n), dim3(256), 0, stream, wins, X, ws);
  // the kernel instance whose largest E-step case is the launch's largest K:
  // K <= 9 (the reference's max_C 10) holds 125 VGPRs instead of 154, so an
  // EM wave displaces two DP waves (72 VGPRs) on its SIMD instead of three:
  // EM kernel 5.1 / 5.3 vs 6.0 / 6.6 s per driver run, windows/s within the
  // spread (profiles/r06_c1)
  if (mfma)
    hipLaunchKernelGGL((em_k_kernel<true, 15>), dim3(n, max_nk), dim3(256), lds, stream, wins, labels, rng, rng_len,
                       cfg, ws, outd);
  else if (max_nk <= 9)
    hipLaunchKernelGGL((em_k_kernel<false, 9>), dim3(n, max_nk), dim3(256), lds, stream, wins, labels, rng, rng_len,
                       cfg, ws, outd);
  else
    hipLaunchKernelGGL((em_k_kernel<false, 15>), dim3(n, max_nk), dim3(256), lds, stream, wins, labels, rng, rng_len,
                       cfg, ws, outd);
  hipLaunchKernelGGL(em_select_kernel, dim3((n + 63) / 64), dim3(64), 0, stream, wins, n, ws, outd, outi);
  return hipGetLastError();
}

}  // namespace svs

namespace svs {

// Copies gamma | pi | theta of each window's selected K into the parameter dump
// (only when the caller asks for parameters, e.g. parity tests).
__global__ __launch_bounds__(256) void em_gather_kernel(const EmWindow* __restrict__ wins,
                                                        const double* __restrict__ ws,
                                                        const int32_t* __restrict__ outi,
                                                        double* __restrict__ par) {
  const EmWindow W = wins[blockIdx.x];
  const int32_t* oi = outi + W.outi_off;
  if (oi[2] != 0) return;
  const int K = oi[0], N = W.n_reads, nf = W.n_feat;
  const EmK P = em_k_ptrs(W, const_cast<double*>(ws), K);
  double* p = par + W.par_off;
  for (int64_t r = threadIdx.x; r < static_cast<int64_t>(N) * K; r += blockDim.x) p[r] = P.g[r];
  for (int r = threadIdx.x; r < K; r += blockDim.x) p[static_cast<int64_t>(N) * K + r] = P.pi[r];
  double* t = p + static_cast<int64_t>(N) * K + K;
  for (int64_t r = threadIdx.x; r < static_cast<int64_t>(K) * nf * 5; r += blockDim.x)
    t[r] = P.th[r];
}

hipError_t launch_em_gather(const EmWindow* wins, int n, const double* ws, const int32_t* outi, double* par,
                            hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(em_gather_kernel, dim3(n), dim3(256), 0, stream, wins, ws, outi, par);
  return hipGetLastError();
}

}  // namespace svs
