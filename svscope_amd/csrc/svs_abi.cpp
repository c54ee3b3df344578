// extern "C" surface of libsvscope_hip.so (declared in include/svscope.h).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include <sched.h>
#include <thread>
#include <vector>

#include "../../include/svscope.h"
#include "svs_context.hpp"
#include "svs_devarena.hpp"
#include "svs_device.hpp"
#include "svs_internal.hpp"
#include "ward.hpp"

struct svs_poa_result {
  std::vector<std::string> consensus;
  std::vector<std::string> msa_block;
  std::vector<int32_t> rows, cols;
  svs_poa_stats stats{};
};

namespace {
thread_local std::string g_last_error;

int fail(int code, const std::string& msg) {
  g_last_error = msg;
  return code;
}

template <class F>
int guarded(F&& f) {
  try {
    f();
    return SVS_OK;
  } catch (const svs::SvsError& e) {
    return fail(e.code, e.what());
  } catch (const std::bad_alloc&) {
    return fail(SVS_E_NOMEM, "host allocation failed");
  } catch (const std::exception& e) {
    return fail(SVS_E_INTERNAL, e.what());
  }
}

unsigned host_threads() {
  if (const char* s = std::getenv("SVS_HOST_THREADS")) {
    const int v = std::atoi(s);
    if (v > 0) return static_cast<unsigned>(v);
  }
  // the CPUs this process may run on (its affinity mask; svscope_amd/hostcpu.py
  // pins each rank of a multi-GPU run to its slice and sets SVS_HOST_THREADS)
  unsigned hw = std::max(1u, std::thread::hardware_concurrency());
  cpu_set_t set;
  CPU_ZERO(&set);
  if (sched_getaffinity(0, sizeof(set), &set) == 0) hw = std::max(1, CPU_COUNT(&set));
  return std::min(hw, 16u);
}
}  // namespace

extern "C" {

const char* svs_last_error(void) { return g_last_error.c_str(); }

int svs_abi_version(void) { return SVS_ABI_VERSION; }

int svs_device_count(int* out) {
  if (!out) return fail(SVS_E_INVALID, "null out");
  return guarded([&] {
    int n = 0;
    SVS_HIP(hipGetDeviceCount(&n));
    *out = n;
  });
}

int svs_init(int device_ordinal, svs_context** out) {
  if (!out) return fail(SVS_E_INVALID, "null out");
  *out = nullptr;
  svs_context* ctx = nullptr;
  const int rc = guarded([&] {
    int n = 0;
    SVS_HIP(hipGetDeviceCount(&n));
    if (device_ordinal < 0 || device_ordinal >= n)
      throw svs::SvsError(SVS_E_HIP, "no HIP device " + std::to_string(device_ordinal) + " (found " +
                                         std::to_string(n) + ")");
    SVS_HIP(hipSetDevice(device_ordinal));
    ctx = new svs_context();
    ctx->device = device_ordinal;
    SVS_HIP(hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking));
    // (the EM stream at the lowest priority, 1, so that its workgroups only
    // take slots no DP workgroup waits for: windows/s and the DP busy frac
    // within the spread, EM kernel 5.4 vs 4.8-4.9 s, profiles/r06_em2; not kept)
    SVS_HIP(hipStreamCreateWithFlags(&ctx->em_stream, hipStreamNonBlocking));
    SVS_HIP(hipEventCreate(&ctx->ev_start));
    SVS_HIP(hipEventCreate(&ctx->ev_stop));
    SVS_HIP(hipEventCreate(&ctx->ev_mid));
    SVS_HIP(hipEventCreate(&ctx->ev_rerun));
    size_t free_b = 0, total_b = 0;
    SVS_HIP(hipMemGetInfo(&free_b, &total_b));
    // the launches' traceback codes and carries: 5/8 of the free HBM (180 GB
    // of an MI355X), so that a group's launch holds 2048 config-3 alignments
    // (about 40 MB of codes each at the end of a window MSA); the graph arena
    // gets the rest less the carries and 4 GiB (below).  Driver-shape A/B,
    // profiles/r04_h9: 352.5 / 350.9 windows/s at 180 GB and 2048 tasks per
    // group against 334 at half the free HBM and 1792
    size_t budget = free_b / 8 * 5;
    if (const char* s = std::getenv("SVS_DEVICE_BUDGET_GB")) {
      const double gb = std::atof(s);
      if (gb > 0) budget = static_cast<size_t>(gb * (1ull << 30));
    }
    ctx->device_budget = std::max<size_t>(budget, 64ull << 20);
    // the device-resident POA graphs get what the launch buffers leave of the
    // free HBM (the traceback budget, and the carry buffers sized at an eighth
    // of it, svs_poa_engine.cpp), less 4 GiB for the EM and MisScore buffers
    // and HIP itself
    const size_t used = ctx->device_budget + ctx->device_budget / 8 + (4ull << 30);
    const size_t rest = free_b > used ? free_b - used : 0;
    ctx->dgraph_budget = std::max<size_t>(rest, 1ull << 30);
    if (std::getenv("SVS_POA_DEBUG"))
      std::fprintf(stderr, "[svs] context: free %.1f of %.1f GiB, launch budget %.1f GiB, graph arena %.1f GiB\n",
                   free_b / 1073741824.0, total_b / 1073741824.0, ctx->device_budget / 1073741824.0,
                   ctx->dgraph_budget / 1073741824.0);
    ctx->pool = new svs::ThreadPool(host_threads());
  });
  if (rc != SVS_OK) {
    if (ctx) svs_release(ctx);
    return rc;
  }
  *out = ctx;
  return SVS_OK;
}

void svs_release(svs_context* ctx) {
  if (!ctx) return;
  (void)hipSetDevice(ctx->device);
  if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
  if (ctx->em_stream) (void)hipStreamSynchronize(ctx->em_stream);
  ctx->poa_arenas.clear();
  ctx->dgraph_arena.reset();
  for (svs::DeviceBuf* b : {&ctx->d_em_in, &ctx->d_em_ws, &ctx->d_em_out, &ctx->d_rng, &ctx->d_ms_pairs,
                            &ctx->d_ms_seq, &ctx->d_ms_nib, &ctx->d_ms_carry, &ctx->d_ms_stack, &ctx->d_ms_out})
    b->release();
  for (svs::PinnedBuf* b : {&ctx->h_em_in, &ctx->h_em_out}) b->release();
  if (ctx->ev_start) (void)hipEventDestroy(ctx->ev_start);
  if (ctx->ev_stop) (void)hipEventDestroy(ctx->ev_stop);
  if (ctx->ev_mid) (void)hipEventDestroy(ctx->ev_mid);
  if (ctx->ev_rerun) (void)hipEventDestroy(ctx->ev_rerun);
  if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
  if (ctx->em_stream) (void)hipStreamDestroy(ctx->em_stream);
  delete ctx->pool;
  delete ctx;
}

int svs_poa_batch(svs_context* ctx, int32_t n_jobs, const int64_t* job_seq_start,
                  const int64_t* seq_byte_start, const char* seq_bytes, const svs_poa_config* cfg,
                  svs_poa_result** out) {
  if (!ctx || !out || !cfg || n_jobs < 0 || (n_jobs > 0 && (!job_seq_start || !seq_byte_start)))
    return fail(SVS_E_INVALID, "svs_poa_batch: invalid argument");
  *out = nullptr;
  svs_poa_result* res = nullptr;
  const int rc = guarded([&] {
    SVS_HIP(hipSetDevice(ctx->device));
    svs::check_poa_config(*cfg);
    std::vector<svs::PoaTask> tasks(static_cast<size_t>(n_jobs));
    for (int32_t j = 0; j < n_jobs; ++j) {
      const int64_t a = job_seq_start[j], b = job_seq_start[j + 1];
      if (b < a || a < 0) throw svs::SvsError(SVS_E_INVALID, "job_seq_start not monotone");
      for (int64_t s = a; s < b; ++s) {
        const int64_t x = seq_byte_start[s], y = seq_byte_start[s + 1];
        if (y < x || x < 0) throw svs::SvsError(SVS_E_INVALID, "seq_byte_start not monotone");
        if (y > x && !seq_bytes) throw svs::SvsError(SVS_E_INVALID, "null seq_bytes");
        tasks[j].seqs.emplace_back(y > x ? seq_bytes + x : "", static_cast<size_t>(y - x));
      }
    }
    res = new svs_poa_result();
    svs::run_poa_tasks(ctx, tasks, *cfg, res->stats);
    res->consensus.resize(tasks.size());
    res->msa_block.resize(tasks.size());
    res->rows.assign(tasks.size(), 0);
    res->cols.assign(tasks.size(), 0);
    for (size_t j = 0; j < tasks.size(); ++j) {
      res->consensus[j] = std::move(tasks[j].consensus);
      const auto& m = tasks[j].msa;
      res->rows[j] = static_cast<int32_t>(m.size());
      res->cols[j] = m.empty() ? 0 : static_cast<int32_t>(m[0].size());
      std::string& blk = res->msa_block[j];
      blk.reserve(m.size() * (m.empty() ? 0 : m[0].size()));
      for (const auto& row : m) blk += row;
    }
  });
  if (rc != SVS_OK) {
    delete res;
    return rc;
  }
  *out = res;
  return SVS_OK;
}

int svs_poa_result_consensus(const svs_poa_result* r, int32_t job, const char** data, int64_t* len) {
  if (!r || !data || !len || job < 0 || job >= static_cast<int32_t>(r->consensus.size()))
    return fail(SVS_E_INVALID, "svs_poa_result_consensus: invalid argument");
  *data = r->consensus[job].data();
  *len = static_cast<int64_t>(r->consensus[job].size());
  return SVS_OK;
}

int svs_poa_result_msa(const svs_poa_result* r, int32_t job, int32_t* rows, int32_t* cols,
                       const char** data) {
  if (!r || !rows || !cols || !data || job < 0 || job >= static_cast<int32_t>(r->rows.size()))
    return fail(SVS_E_INVALID, "svs_poa_result_msa: invalid argument");
  *rows = r->rows[job];
  *cols = r->cols[job];
  *data = r->msa_block[job].data();
  return SVS_OK;
}

int svs_poa_result_stats(const svs_poa_result* r, svs_poa_stats* out) {
  if (!r || !out) return fail(SVS_E_INVALID, "svs_poa_result_stats: invalid argument");
  *out = r->stats;
  return SVS_OK;
}

void svs_poa_result_free(svs_poa_result* r) { delete r; }

int svs_similarity_batch(svs_context* ctx, int32_t n_windows, const svs_em_window* wins, const uint8_t* X,
                         const int64_t* s_off, double* S) {
  if (!ctx || (n_windows > 0 && (!s_off || !S))) return fail(SVS_E_INVALID, "svs_similarity_batch: invalid argument");
  std::string err;
  const int v = svs::em_validate(n_windows, wins, X, &err);
  if (v != SVS_OK) return fail(v, "svs_similarity_batch: " + err);
  if (n_windows == 0) return SVS_OK;
  return guarded([&] {
    SVS_HIP(hipSetDevice(ctx->device));
    svs::run_similarity(ctx, n_windows, wins, X, S, s_off);
  });
}

int svs_em_batch(svs_context* ctx, int32_t n_windows, const svs_em_window* wins, const uint8_t* X,
                 const int32_t* labels, const svs_em_config* cfg, svs_em_result** out) {
  if (!ctx || !cfg || !out || (n_windows > 0 && !labels)) return fail(SVS_E_INVALID, "svs_em_batch: invalid argument");
  *out = nullptr;
  std::string err;
  const int v = svs::em_validate(n_windows, wins, X, &err);
  if (v != SVS_OK) return fail(v, "svs_em_batch: " + err);
  svs_em_result* res = nullptr;
  const int rc = guarded([&] {
    SVS_HIP(hipSetDevice(ctx->device));
    res = svs::run_em(ctx, n_windows, wins, X, labels, *cfg);
  });
  if (rc == SVS_OK) *out = res;
  return rc;
}

int svs_ward_maxclust_batch(int32_t n_windows, const svs_em_window* wins, const double* S, const int64_t* s_off,
                            int32_t max_c, int32_t* labels) {
  if (n_windows < 0 || (n_windows > 0 && (!wins || !S || !s_off || !labels)) || max_c < 1)
    return fail(SVS_E_INVALID, "svs_ward_maxclust_batch: invalid argument");
  for (int32_t w = 0; w < n_windows; ++w)
    if (wins[w].n_reads < 1 || s_off[w] < 0 || wins[w].label_off < 0)
      return fail(SVS_E_INVALID, "svs_ward_maxclust_batch: window " + std::to_string(w) + " is malformed");
  return guarded([&] {
    std::vector<svs::WardMerge> Z;
    for (int32_t w = 0; w < n_windows; ++w) {
      const int n = wins[w].n_reads;
      svs::ward_linkage(S + s_off[w], n, &Z);
      svs::maxclust_labels(Z, n, std::min(max_c + 1, n), labels + wins[w].label_off);
    }
  });
}

int svs_em_cluster_batch(svs_context* ctx, int32_t n_windows, const svs_em_window* wins, const uint8_t* X,
                         const svs_em_config* cfg, svs_em_result** out) {
  if (!ctx || !cfg || !out) return fail(SVS_E_INVALID, "svs_em_cluster_batch: invalid argument");
  *out = nullptr;
  std::string err;
  const int v = svs::em_validate(n_windows, wins, X, &err);
  if (v != SVS_OK) return fail(v, "svs_em_cluster_batch: " + err);
  if (cfg->max_c < 1) return fail(SVS_E_INVALID, "svs_em_cluster_batch: max_c must be >= 1");
  svs_em_result* res = nullptr;
  const int rc = guarded([&] {
    SVS_HIP(hipSetDevice(ctx->device));
    res = svs::run_em_cluster(ctx, n_windows, wins, X, *cfg, ctx->pool);
  });
  if (rc == SVS_OK) *out = res;
  return rc;
}

static int check_decision_windows(const char* fn, int32_t n_windows, const svs_decision_window* wins,
                                  const int64_t* seq_byte_start, const char* seq_bytes, const char* text,
                                  const uint8_t* is_tlabel) {
  if (n_windows < 0 || (n_windows > 0 && (!wins || !seq_byte_start)))
    return fail(SVS_E_INVALID, std::string(fn) + ": invalid argument");
  for (int32_t w = 0; w < n_windows; ++w) {
    const svs_decision_window& W = wins[w];
    if (W.n_seqs < 1 || W.n_ids < 0 || W.seq_start < 0 || W.flank5_len < 0 || W.flank3_len < 0 || W.tag_off < 0 ||
        ((W.flank5_len || W.flank3_len) && !text) || (W.n_ids && !is_tlabel))
      return fail(SVS_E_INVALID, std::string(fn) + ": window " + std::to_string(w) + " is malformed");
    // every sequence's byte range, checked here on the caller's thread: a bad
    // batch fails its own submit, never the session's worker
    for (int32_t k = 0; k < W.n_seqs; ++k) {
      const int64_t x = seq_byte_start[W.seq_start + k], y = seq_byte_start[W.seq_start + k + 1];
      if (x < 0 || y < x || (y > x && !seq_bytes))
        return fail(SVS_E_INVALID, std::string(fn) + ": window " + std::to_string(w) +
                                       ": seq_byte_start not monotone");
    }
  }
  return SVS_OK;
}

static int check_decision_config(const char* fn, const svs_decision_config* cfg) {
  if (!cfg || cfg->readcutoff < 0 || cfg->em.max_c < 1 || cfg->em.n_step < 1)
    return fail(SVS_E_INVALID, std::string(fn) + ": invalid config");
  return SVS_OK;
}

int svs_decision_batch(svs_context* ctx, int32_t n_windows, const svs_decision_window* wins,
                       const int64_t* seq_byte_start, const char* seq_bytes, const char* text,
                       const uint8_t* is_tlabel, const svs_decision_config* cfg, svs_decision_result** out) {
  if (!ctx || !cfg || !out) return fail(SVS_E_INVALID, "svs_decision_batch: invalid argument");
  *out = nullptr;
  if (int rc = check_decision_windows("svs_decision_batch", n_windows, wins, seq_byte_start, seq_bytes, text,
                                      is_tlabel)) return rc;
  if (int rc = check_decision_config("svs_decision_batch", cfg)) return rc;
  svs_decision_result* res = nullptr;
  const int rc = guarded([&] {
    SVS_HIP(hipSetDevice(ctx->device));
    svs::check_poa_config(cfg->poa);
    res = svs::run_decision(ctx, n_windows, wins, seq_byte_start, seq_bytes, text, is_tlabel, *cfg);
  });
  if (rc == SVS_OK) *out = res;
  return rc;
}

int svs_decision_session_open(svs_context* ctx, const svs_decision_config* cfg, svs_decision_session** out) {
  if (!ctx || !cfg || !out) return fail(SVS_E_INVALID, "svs_decision_session_open: invalid argument");
  *out = nullptr;
  if (int rc = check_decision_config("svs_decision_session_open", cfg)) return rc;
  svs_decision_session* s = nullptr;
  const int rc = guarded([&] {
    SVS_HIP(hipSetDevice(ctx->device));
    s = svs::open_decision_session(ctx, *cfg);
  });
  if (rc == SVS_OK) *out = s;
  return rc;
}

int svs_decision_session_submit(svs_decision_session* s, int32_t n_windows, const svs_decision_window* wins,
                                const int64_t* seq_byte_start, const char* seq_bytes, const char* text,
                                const uint8_t* is_tlabel, int64_t* ticket) {
  if (!s || !ticket) return fail(SVS_E_INVALID, "svs_decision_session_submit: invalid argument");
  if (int rc = check_decision_windows("svs_decision_session_submit", n_windows, wins, seq_byte_start, seq_bytes,
                                      text, is_tlabel))
    return rc;
  return guarded([&] {
    *ticket = svs::submit_decision_batch(s, n_windows, wins, seq_byte_start, seq_bytes, text, is_tlabel);
  });
}

int svs_decision_session_wait(svs_decision_session* s, int64_t ticket, svs_decision_result** out) {
  if (!s || !out) return fail(SVS_E_INVALID, "svs_decision_session_wait: invalid argument");
  *out = nullptr;
  svs_decision_result* r = nullptr;
  const int rc = guarded([&] { r = svs::wait_decision_batch(s, ticket); });
  if (rc == SVS_OK) *out = r;
  return rc;
}

int svs_decision_session_stats(svs_decision_session* s, svs_decision_stats* out) {
  if (!s || !out) return fail(SVS_E_INVALID, "svs_decision_session_stats: invalid argument");
  svs::session_stats(s, out);
  return SVS_OK;
}

int svs_decision_session_close(svs_decision_session* s) {
  if (!s) return SVS_OK;
  return guarded([&] {
    std::exception_ptr e = svs::close_decision_session(s);
    if (e) std::rethrow_exception(e);
  });
}

int svs_decision_result_window(const svs_decision_result* r, int32_t window, int32_t* status, int32_t* K,
                               int32_t* n_som, int32_t* n_germ) {
  if (!r || window < 0 || window >= static_cast<int32_t>(r->w.size()) || !status || !K || !n_som || !n_germ)
    return fail(SVS_E_INVALID, "svs_decision_result_window: invalid argument");
  const auto& w = r->w[window];
  *status = w.status;
  *K = w.K;
  *n_som = static_cast<int32_t>(w.som.size());
  *n_germ = static_cast<int32_t>(w.germ.size());
  return SVS_OK;
}

int svs_decision_result_window_error(const svs_decision_result* r, int32_t window, const char** msg) {
  if (!r || window < 0 || window >= static_cast<int32_t>(r->w.size()) || !msg)
    return fail(SVS_E_INVALID, "svs_decision_result_window_error: invalid argument");
  *msg = r->w[window].error.c_str();
  return SVS_OK;
}

int svs_decision_result_cluster(const svs_decision_result* r, int32_t window, int32_t cluster,
                                const int32_t** ids, int32_t* n_ids, const char** cons, int64_t* cons_len) {
  if (!r || window < 0 || window >= static_cast<int32_t>(r->w.size()) || !ids || !n_ids || !cons || !cons_len)
    return fail(SVS_E_INVALID, "svs_decision_result_cluster: invalid argument");
  const auto& w = r->w[window];
  const int32_t ns = static_cast<int32_t>(w.som.size()), ng = static_cast<int32_t>(w.germ.size());
  if (cluster < 0 || cluster >= ns + ng) return fail(SVS_E_INVALID, "svs_decision_result_cluster: bad cluster");
  const svs::ClusterPlan& p = cluster < ns ? w.som[cluster] : w.germ[cluster - ns];
  *ids = p.ids.data();
  *n_ids = static_cast<int32_t>(p.ids.size());
  *cons = p.consensus.data();
  *cons_len = static_cast<int64_t>(p.consensus.size());
  return SVS_OK;
}

int svs_decision_result_stats(const svs_decision_result* r, svs_decision_stats* out) {
  if (!r || !out) return fail(SVS_E_INVALID, "svs_decision_result_stats: invalid argument");
  *out = r->st;
  return SVS_OK;
}

void svs_decision_result_free(svs_decision_result* r) { delete r; }

int svs_msa_features(int32_t n_rows, int32_t width, const char* msa, const char* flank5, int32_t flank5_len,
                     const char* flank3, int32_t flank3_len, int32_t n_reads, const int32_t* read_lens,
                     int32_t n_ids, int32_t hcutoff, double scutoff, int32_t* rows, int32_t* n_feat,
                     uint8_t* feat, int64_t feat_cap, int32_t* id_map, int32_t* n_map, int64_t id_cap) {
  if (n_rows < 0 || width < 0 || n_reads < 0 || n_ids < 0 || !rows || !n_feat || !n_map ||
      (n_rows * static_cast<int64_t>(width) > 0 && !msa) || (n_reads > 0 && !read_lens) ||
      (flank5_len > 0 && !flank5) || (flank3_len > 0 && !flank3))
    return fail(SVS_E_INVALID, "svs_msa_features: invalid argument");
  *rows = -1;
  return guarded([&] {
    std::vector<std::string> m(n_rows);
    for (int32_t r = 0; r < n_rows; ++r) m[r].assign(msa + static_cast<int64_t>(r) * width, width);
    std::vector<int32_t> lens(read_lens, read_lens + n_reads);
    svs::WindowFeatures f;
    svs::msa_feature_select(m, std::string(flank5 ? flank5 : "", flank5_len),
                            std::string(flank3 ? flank3 : "", flank3_len), lens, n_ids, hcutoff, scutoff, &f);
    *rows = f.rows;
    *n_feat = f.n_feat;
    *n_map = static_cast<int32_t>(f.id_map.size());
    if (static_cast<int64_t>(f.feat.size()) > feat_cap || static_cast<int64_t>(f.id_map.size()) > id_cap ||
        (!f.feat.empty() && !feat) || (!f.id_map.empty() && !id_map))
      throw svs::SvsError(SVS_E_INVALID, "svs_msa_features: output capacity too small");
    if (!f.feat.empty()) std::memcpy(feat, f.feat.data(), f.feat.size());
    if (!f.id_map.empty()) std::memcpy(id_map, f.id_map.data(), 4 * f.id_map.size());
  });
}

int svs_wave_selftest(svs_context* ctx, const int32_t* in, int32_t* scan, int32_t* shift, int32_t n_waves) {
  if (!ctx || !in || !scan || !shift || n_waves <= 0) return fail(SVS_E_INVALID, "svs_wave_selftest: invalid argument");
  return guarded([&] {
    SVS_HIP(hipSetDevice(ctx->device));
    const size_t bytes = static_cast<size_t>(n_waves) * 64 * 4;
    int32_t* d = nullptr;
    SVS_HIP(hipMalloc(&d, 3 * bytes));
    hipError_t e = hipMemcpy(d, in, bytes, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = svs::launch_wave_selftest(d, d + n_waves * 64, d + 2 * n_waves * 64, n_waves, ctx->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    if (e == hipSuccess) e = hipMemcpy(scan, d + n_waves * 64, bytes, hipMemcpyDeviceToHost);
    if (e == hipSuccess) e = hipMemcpy(shift, d + 2 * n_waves * 64, bytes, hipMemcpyDeviceToHost);
    (void)hipFree(d);
    SVS_HIP(e);
  });
}

int svs_aligment_score_batch(svs_context* ctx, int32_t n_pairs, const int32_t* pair_a, const int32_t* pair_b,
                             int32_t n_seqs, const int64_t* seq_byte_start, const char* seq_bytes, int32_t cutoff,
                             int32_t* out_len, int32_t* out_match, int32_t* out_status, svs_misscore_stats* stats) {
  if (!ctx || n_pairs < 0 || n_seqs < 0 ||
      (n_pairs > 0 && (!pair_a || !pair_b || !seq_byte_start || !out_len || !out_match || !out_status)))
    return fail(SVS_E_INVALID, "svs_aligment_score_batch: invalid argument");
  if (cutoff < 0 || cutoff > 64)
    return fail(SVS_E_UNSUPPORTED, "svs_aligment_score_batch: cutoff must be 0..64");
  return guarded([&] {
    for (int32_t s = 0; s < n_seqs; ++s)
      if (seq_byte_start[s] < 0 || seq_byte_start[s + 1] < seq_byte_start[s])
        throw svs::SvsError(SVS_E_INVALID, "seq_byte_start not monotone");
    if (n_seqs > 0 && seq_byte_start[n_seqs] > seq_byte_start[0] && !seq_bytes)
      throw svs::SvsError(SVS_E_INVALID, "null seq_bytes");
    for (int32_t p = 0; p < n_pairs; ++p)
      if (pair_a[p] < 0 || pair_a[p] >= n_seqs || pair_b[p] < 0 || pair_b[p] >= n_seqs)
        throw svs::SvsError(SVS_E_INVALID, "pair " + std::to_string(p) + ": sequence index out of range");
    SVS_HIP(hipSetDevice(ctx->device));
    svs::run_misscore(ctx, n_pairs, pair_a, pair_b, seq_byte_start, seq_bytes, cutoff, out_len, out_match,
                      out_status, stats);
  });
}

}  // extern "C"
