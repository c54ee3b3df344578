// Host driver of the EM seam (ReadsCluster.EMCluster, /root/reference/src/ReadsCluster.py:221-277).
//
// The reference's only randomness is numpy's legacy global RandomState seeded
// with 2023 at import (ReadsCluster.py:42) and consumed by np.random.dirichlet
// during M-step re-initialisation (:185-187).  numpy's legacy dirichlet with
// alpha = ones(5) draws legacy standard exponentials (-log(1 - u53)) from
// MT19937; this file regenerates that stream bit-for-bit (MT19937 with numpy's
// legacy integer seeding, 53-bit doubles, glibc log) into one device table
// shared by every window.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/svscope.h"
#include "svs_context.hpp"
#include "svs_em_device.hpp"
#include "svs_internal.hpp"
#include "threadpool.hpp"
#include "ward.hpp"

namespace svs {

void legacy_exponentials(uint32_t seed, uint64_t n, double* out) {
  uint32_t mt[624];
  mt[0] = seed;
  for (int i = 1; i < 624; ++i) mt[i] = 1812433253u * (mt[i - 1] ^ (mt[i - 1] >> 30)) + static_cast<uint32_t>(i);
  int pos = 624;
  auto next = [&]() -> uint32_t {
    if (pos >= 624) {
      for (int i = 0; i < 624; ++i) {
        const uint32_t y = (mt[i] & 0x80000000u) | (mt[(i + 1) % 624] & 0x7fffffffu);
        mt[i] = mt[(i + 397) % 624] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
      }
      pos = 0;
    }
    uint32_t y = mt[pos++];
    y ^= y >> 11;
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= y >> 18;
    return y;
  };
  for (uint64_t k = 0; k < n; ++k) {
    const uint32_t a = next() >> 5, b = next() >> 6;
    const double u = (a * 67108864.0 + b) / 9007199254740992.0;
    out[k] = -std::log(1.0 - u);
  }
}

static void ensure_rng(svs_context* ctx, uint32_t seed, uint64_t len) {
  if (ctx->rng_len >= len && ctx->rng_seed == seed) return;
  std::vector<double> tab(len);
  legacy_exponentials(seed, len, tab.data());
  ctx->d_rng.ensure(len * sizeof(double));
  SVS_HIP(hipMemcpy(ctx->d_rng.ptr, tab.data(), len * sizeof(double), hipMemcpyHostToDevice));
  ctx->rng_len = len;
  ctx->rng_seed = seed;
}

static int zero_param_num(const uint8_t* x, int n, int nf) {
  int zeros = 0;
  for (int f = 0; f < nf; ++f) {
    int c[5] = {0, 0, 0, 0, 0};
    for (int i = 0; i < n; ++i) ++c[x[static_cast<int64_t>(i) * nf + f]];
    for (int a = 0; a < 5; ++a) zeros += c[a] == 0;
  }
  return zeros;
}

}  // namespace svs

extern "C" {

int svs_rng_exponential_table(uint32_t seed, int64_t n, double* out) {
  if (n < 0 || (n > 0 && !out)) return SVS_E_INVALID;
  svs::legacy_exponentials(seed, static_cast<uint64_t>(n), out);
  return SVS_OK;
}

}  // extern "C"

namespace svs {

int em_validate(int32_t n_windows, const svs_em_window* wins, const uint8_t* X, std::string* err) {
  if (n_windows < 0 || (n_windows > 0 && (!wins || !X))) { *err = "invalid argument"; return SVS_E_INVALID; }
  for (int32_t w = 0; w < n_windows; ++w) {
    if (wins[w].n_reads < 1 || wins[w].n_feat < 0 || wins[w].x_off < 0) {
      *err = "window " + std::to_string(w) + ": bad shape/offset";
      return SVS_E_INVALID;
    }
    const uint8_t* x = X + wins[w].x_off;
    const int64_t cnt = static_cast<int64_t>(wins[w].n_reads) * wins[w].n_feat;
    for (int64_t k = 0; k < cnt; ++k)
      if (x[k] > 4) { *err = "window " + std::to_string(w) + ": symbol outside 0..4"; return SVS_E_INVALID; }
  }
  return SVS_OK;
}

void run_similarity(svs_context* ctx, int32_t n, const svs_em_window* wins, const uint8_t* X, double* S_out,
                    const int64_t* s_off_in) {
  std::vector<EmWindow> W(n);
  uint64_t xbytes = 0, sdoubles = 0;
  std::vector<int64_t> s_off(n);
  for (int32_t w = 0; w < n; ++w) {
    W[w] = EmWindow{};
    W[w].n_reads = wins[w].n_reads;
    W[w].n_feat = wins[w].n_feat;
    W[w].x_off = xbytes;
    xbytes += static_cast<uint64_t>(wins[w].n_reads) * wins[w].n_feat;
    s_off[w] = static_cast<int64_t>(sdoubles);
    sdoubles += static_cast<uint64_t>(wins[w].n_reads) * wins[w].n_reads;
  }
  const size_t off_w = 0, off_o = (n * sizeof(EmWindow) + 255) / 256 * 256;
  const size_t off_x = off_o + (n * sizeof(int64_t) + 255) / 256 * 256;
  const size_t total = off_x + xbytes;
  ctx->h_em_in.ensure(total);
  char* h = ctx->h_em_in.as<char>();
  std::memcpy(h + off_w, W.data(), n * sizeof(EmWindow));
  std::memcpy(h + off_o, s_off.data(), n * sizeof(int64_t));
  for (int32_t w = 0; w < n; ++w)
    std::memcpy(h + off_x + W[w].x_off, X + wins[w].x_off, static_cast<size_t>(wins[w].n_reads) * wins[w].n_feat);
  ctx->d_em_in.ensure(total);
  ctx->d_em_out.ensure(sdoubles * sizeof(double) + 8);
  char* d = ctx->d_em_in.as<char>();
  SVS_HIP(hipMemcpyAsync(d, h, total, hipMemcpyHostToDevice, ctx->em_stream));
  SVS_HIP(launch_similarity(reinterpret_cast<const EmWindow*>(d + off_w), n, reinterpret_cast<const uint8_t*>(d + off_x),
                            reinterpret_cast<const int64_t*>(d + off_o), ctx->d_em_out.as<double>(), ctx->em_stream));
  ctx->h_em_out.ensure(sdoubles * sizeof(double) + 8);
  SVS_HIP(hipMemcpyAsync(ctx->h_em_out.ptr, ctx->d_em_out.ptr, sdoubles * sizeof(double), hipMemcpyDeviceToHost,
                         ctx->em_stream));
  SVS_HIP(hipStreamSynchronize(ctx->em_stream));
  const double* hs = ctx->h_em_out.as<double>();
  for (int32_t w = 0; w < n; ++w)
    std::memcpy(S_out + s_off_in[w], hs + s_off[w],
                sizeof(double) * static_cast<size_t>(wins[w].n_reads) * wins[w].n_reads);
}

svs_em_result* run_em(svs_context* ctx, int32_t n, const svs_em_window* wins, const uint8_t* X,
                      const int32_t* labels, const svs_em_config& cfg) {
  if (cfg.max_c < 1 || cfg.max_c > 15) throw SvsError(SVS_E_UNSUPPORTED, "max_C must be in 1..15");
  for (int32_t w = 0; w < n; ++w)
    if (wins[w].n_reads > (1 << 16))
      throw SvsError(SVS_E_UNSUPPORTED, "window " + std::to_string(w) + " has more than 65536 reads");
  std::vector<EmWindow> W(n);
  uint64_t xbytes = 0, lab = 0, ws = 0, od = 0, oi = 0, par = 0, lds = 0;
  for (int32_t w = 0; w < n; ++w) {
    EmWindow& e = W[w];
    e.n_reads = wins[w].n_reads;
    e.n_feat = wins[w].n_feat;
    e.kmax = std::min(cfg.max_c + 1, e.n_reads);
    if (e.kmax < 2) throw SvsError(SVS_E_INVALID, "window " + std::to_string(w) + " has fewer than 2 reads");
    e.zero_params = zero_param_num(X + wins[w].x_off, e.n_reads, e.n_feat);
    e.x_off = xbytes;
    e.lab_off = lab;
    e.ws_off = ws;
    e.outd_off = od;
    e.outi_off = oi;
    e.par_off = par;
    const uint64_t N = e.n_reads, nf = e.n_feat, nk = e.kmax - 1;
    xbytes += N * nf;
    lab += nk * N;
    lds = std::max(lds, em_lds_doubles(e.n_reads, static_cast<int>(nk)));
    ws += (em_workspace_doubles(e.n_reads, e.n_feat, e.kmax) + 31) / 32 * 32;
    od += nk + N;
    oi += 6 + N;
    if (cfg.want_params) par += N * nk + nk + nk * nf * 5;
  }
  const size_t off_w = 0;
  const size_t off_l = (n * sizeof(EmWindow) + 255) / 256 * 256;
  const size_t off_x = off_l + (lab * 4 + 255) / 256 * 256;
  const size_t off_r = off_x + (xbytes + 255) / 256 * 256;  // the windows rerun in order (K-parallel path)
  const size_t total = off_r + n * sizeof(EmWindow);
  ctx->h_em_in.ensure(total);
  char* h = ctx->h_em_in.as<char>();
  std::memcpy(h + off_w, W.data(), n * sizeof(EmWindow));
  for (int32_t w = 0; w < n; ++w) {
    const uint64_t N = W[w].n_reads, nk = W[w].kmax - 1;
    std::memcpy(h + off_l + 4 * W[w].lab_off, labels + wins[w].label_off, 4 * N * nk);
    std::memcpy(h + off_x + W[w].x_off, X + wins[w].x_off, N * W[w].n_feat);
  }
  ctx->d_em_in.ensure(total);
  ctx->d_em_ws.ensure(ws * 8 + 64);
  const size_t od_bytes = od * 8, oi_bytes = (oi * 4 + 255) / 256 * 256, par_bytes = par * 8;
  ctx->d_em_out.ensure(od_bytes + oi_bytes + par_bytes + 256);
  ctx->h_em_out.ensure(od_bytes + oi_bytes + par_bytes + 256);
  char* d = ctx->d_em_in.as<char>();
  SVS_HIP(hipMemcpyAsync(d, h, total, hipMemcpyHostToDevice, ctx->em_stream));
  double* d_outd = ctx->d_em_out.as<double>();
  int32_t* d_outi = reinterpret_cast<int32_t*>(ctx->d_em_out.as<char>() + (od_bytes + 255) / 256 * 256);
  double* d_par = reinterpret_cast<double*>(reinterpret_cast<char*>(d_outi) + oi_bytes);
  EmConfig ec{cfg.n_step, 0, cfg.eps};
  int max_nk = 0;
  for (const EmWindow& e : W) max_nk = std::max(max_nk, e.kmax - 1);
  // K-parallel unless SVS_EM_SEQ=1 (em_kernels.hip: windows the speculation
  // cannot place are rerun in order below)
  const char* seq_env = std::getenv("SVS_EM_SEQ");
  const bool parallel = !(seq_env && seq_env[0] == '1');
  auto* res = new svs_em_result();
  try {
    uint64_t want = std::max<uint64_t>(ctx->rng_len, 1ull << 20);
    const size_t outi_at = (od_bytes + 255) / 256 * 256;
    for (int attempt = 0;; ++attempt) {
      ensure_rng(ctx, static_cast<uint32_t>(cfg.seed), want);
      SVS_HIP(hipEventRecord(ctx->ev_start, ctx->em_stream));
      const auto* dW = reinterpret_cast<const EmWindow*>(d + off_w);
      const auto* dX = reinterpret_cast<const uint8_t*>(d + off_x);
      const auto* dL = reinterpret_cast<const int32_t*>(d + off_l);
      if (parallel) {
        SVS_HIP(launch_em_parallel(dW, n, max_nk, dX, dL, ctx->d_rng.as<double>(), ctx->rng_len, ec,
                                   ctx->d_em_ws.as<double>(), d_outd, d_outi, static_cast<size_t>(lds), ctx->em_stream));
        SVS_HIP(hipEventRecord(ctx->ev_mid, ctx->em_stream));
        SVS_HIP(hipMemcpyAsync(ctx->h_em_out.as<char>() + outi_at, d_outi, oi * 4, hipMemcpyDeviceToHost, ctx->em_stream));
        SVS_HIP(hipStreamSynchronize(ctx->em_stream));
        const int32_t* hi = reinterpret_cast<const int32_t*>(ctx->h_em_out.as<char>() + outi_at);
        std::vector<EmWindow> rerun;
        for (int32_t w = 0; w < n; ++w)
          if (hi[W[w].outi_off + 3] == 1) rerun.push_back(W[w]);
        res->em_reruns += static_cast<int64_t>(rerun.size());
        SVS_HIP(hipEventRecord(ctx->ev_rerun, ctx->em_stream));
        if (!rerun.empty()) {
          std::memcpy(h + off_r, rerun.data(), rerun.size() * sizeof(EmWindow));
          SVS_HIP(hipMemcpyAsync(d + off_r, h + off_r, rerun.size() * sizeof(EmWindow), hipMemcpyHostToDevice,
                                 ctx->em_stream));
          SVS_HIP(launch_em_cluster(reinterpret_cast<const EmWindow*>(d + off_r), static_cast<int>(rerun.size()), dX,
                                    dL, ctx->d_rng.as<double>(), ctx->rng_len, ec, ctx->d_em_ws.as<double>(), d_outd,
                                    d_outi, static_cast<size_t>(lds), ctx->em_stream));
        }
      } else {
        SVS_HIP(launch_em_cluster(dW, n, dX, dL, ctx->d_rng.as<double>(), ctx->rng_len, ec, ctx->d_em_ws.as<double>(),
                                  d_outd, d_outi, static_cast<size_t>(lds), ctx->em_stream));
      }
      if (cfg.want_params)
        SVS_HIP(launch_em_gather(reinterpret_cast<const EmWindow*>(d + off_w), n, ctx->d_em_ws.as<double>(), d_outi,
                                 d_par, ctx->em_stream));
      SVS_HIP(hipEventRecord(ctx->ev_stop, ctx->em_stream));
      SVS_HIP(hipMemcpyAsync(ctx->h_em_out.ptr, ctx->d_em_out.ptr,
                             (od_bytes + 255) / 256 * 256 + oi_bytes + par_bytes, hipMemcpyDeviceToHost, ctx->em_stream));
      SVS_HIP(hipStreamSynchronize(ctx->em_stream));
      // kernel time only: in the K-parallel path the host's rerun check
      // between ev_mid and ev_rerun is left out
      float ms = 0.f, ms2 = 0.f;
      if (parallel) {
        SVS_HIP(hipEventElapsedTime(&ms, ctx->ev_start, ctx->ev_mid));
        SVS_HIP(hipEventElapsedTime(&ms2, ctx->ev_rerun, ctx->ev_stop));
      } else {
        SVS_HIP(hipEventElapsedTime(&ms, ctx->ev_start, ctx->ev_stop));
      }
      res->kernel_ms += ms + ms2;
      const int32_t* hi = reinterpret_cast<const int32_t*>(ctx->h_em_out.as<char>() + (od_bytes + 255) / 256 * 256);
      bool overflow = false;
      for (int32_t w = 0; w < n; ++w) overflow |= hi[W[w].outi_off + 2] == 2;
      if (!overflow) break;
      if (attempt >= 6) throw SvsError(SVS_E_INTERNAL, "RNG table growth did not converge");
      want *= 8;  // a window re-initialised more often than the table covers: grow and rerun
    }
    const double* hd = ctx->h_em_out.as<double>();
    const int32_t* hi = reinterpret_cast<const int32_t*>(ctx->h_em_out.as<char>() + (od_bytes + 255) / 256 * 256);
    const double* hp = reinterpret_cast<const double*>(reinterpret_cast<const char*>(hi) + oi_bytes);
    res->w.resize(n);
    for (int32_t w = 0; w < n; ++w) {
      const EmWindow& e = W[w];
      const int32_t* o = hi + e.outi_off;
      const int N = e.n_reads, nk = e.kmax - 1, nf = e.n_feat;
      if (o[2] == 3) throw SvsError(SVS_E_INVALID, "window " + std::to_string(w) + ": all-NaN BIC list (nanargmax)");
      if (o[2] == 4) throw SvsError(SVS_E_INVALID, "window " + std::to_string(w) + ": K=1 rule needs BICList[1]");
      if (o[2] != 0) throw SvsError(SVS_E_INTERNAL, "window " + std::to_string(w) + ": EM kernel status " + std::to_string(o[2]));
      auto& r = res->w[w];
      r.K = o[0];
      r.rng_used = static_cast<int64_t>(static_cast<uint32_t>(o[4])) | (static_cast<int64_t>(o[5]) << 32);
      r.rclust.assign(o + 6, o + 6 + N);
      r.bic.assign(hd + e.outd_off, hd + e.outd_off + nk);
      r.lik.assign(hd + e.outd_off + nk, hd + e.outd_off + nk + N);
      if (cfg.want_params) {
        const double* p = hp + e.par_off;
        const int K = r.K;
        r.gamma.assign(p, p + static_cast<size_t>(N) * K);
        r.pi.assign(p + static_cast<size_t>(N) * K, p + static_cast<size_t>(N) * K + K);
        r.theta.assign(p + static_cast<size_t>(N) * K + K, p + static_cast<size_t>(N) * K + K + static_cast<size_t>(K) * nf * 5);
      }
    }
  } catch (...) {
    delete res;
    throw;
  }
  return res;
}

}  // namespace svs

extern "C" {

int svs_em_result_get(const svs_em_result* r, int32_t window, int32_t field, const void** data, int64_t* count) {
  if (!r || !data || !count || window < 0 || window >= static_cast<int32_t>(r->w.size())) return SVS_E_INVALID;
  const auto& w = r->w[window];
  switch (field) {
    case SVS_EM_K: *data = &w.K; *count = 1; break;
    case SVS_EM_RCLUST: *data = w.rclust.data(); *count = static_cast<int64_t>(w.rclust.size()); break;
    case SVS_EM_BIC: *data = w.bic.data(); *count = static_cast<int64_t>(w.bic.size()); break;
    case SVS_EM_LIK: *data = w.lik.data(); *count = static_cast<int64_t>(w.lik.size()); break;
    case SVS_EM_GAMMA: *data = w.gamma.data(); *count = static_cast<int64_t>(w.gamma.size()); break;
    case SVS_EM_PI: *data = w.pi.data(); *count = static_cast<int64_t>(w.pi.size()); break;
    case SVS_EM_THETA: *data = w.theta.data(); *count = static_cast<int64_t>(w.theta.size()); break;
    case SVS_EM_RNG_USED: *data = &w.rng_used; *count = 1; break;
    default: return SVS_E_INVALID;
  }
  return SVS_OK;
}

int svs_em_result_stats(const svs_em_result* r, double* kernel_ms, int64_t* reruns) {
  if (!r) return SVS_E_INVALID;
  if (kernel_ms) *kernel_ms = r->kernel_ms;
  if (reruns) *reruns = r->em_reruns;
  return SVS_OK;
}

void svs_em_result_free(svs_em_result* r) { delete r; }

}  // extern "C"

namespace svs {

svs_em_result* run_em_cluster(svs_context* ctx, int32_t n, const svs_em_window* wins, const uint8_t* X,
                              const svs_em_config& cfg, ThreadPool* pool) {
  std::vector<svs_em_window> W(wins, wins + n);
  std::vector<int64_t> s_off(n);
  int64_t s_tot = 0, l_tot = 0;
  for (int32_t w = 0; w < n; ++w) {
    const int64_t r = W[w].n_reads;
    s_off[w] = s_tot;
    s_tot += r * r;
    W[w].label_off = l_tot;
    l_tot += (std::min<int64_t>(cfg.max_c + 1, r) - 1) * r;
  }
  std::vector<double> S(static_cast<size_t>(std::max<int64_t>(1, s_tot)));
  std::vector<int32_t> labels(static_cast<size_t>(std::max<int64_t>(1, l_tot)));
  if (n > 0) run_similarity(ctx, n, W.data(), X, S.data(), s_off.data());
  // ward + maxclust per window on the pool (ReadsCluster.py:243, :94)
  auto ward = [&](size_t w) {
    thread_local std::vector<WardMerge> Z;
    const int r = W[w].n_reads;
    ward_linkage(S.data() + s_off[w], r, &Z);
    maxclust_labels(Z, r, std::min(cfg.max_c + 1, r), labels.data() + W[w].label_off);
  };
  if (pool) pool->parallel_for(static_cast<size_t>(n), ward);
  else for (int32_t w = 0; w < n; ++w) ward(static_cast<size_t>(w));
  return run_em(ctx, n, W.data(), X, labels.data(), cfg);
}

}  // namespace svs
