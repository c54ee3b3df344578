// Batched POA engine: lockstep driver over many independent POA jobs (one job
// = one pyspoa `poa(seqs, 1)` call of the reference: a window MSA at
// DataScanner.py:206,213 or a cluster consensus at DecisionMaker.py:160,171).
//
// Step s aligns the s-th sequence of every job at once: the host exports each
// job's rank-ordered row tables, one HIP launch runs every read-vs-graph DP
// (one wave per job) and its traceback, and the host folds the alignments back
// into the graphs in parallel.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "poa_graph.hpp"
#include "svs_context.hpp"
#include "svs_device.hpp"
#include "svs_internal.hpp"

namespace svs {

// ------------------------------------------------------------------ POA driver
static inline uint64_t round_up(uint64_t x, uint64_t a) { return (x + a - 1) / a * a; }

void check_poa_config(const svs_poa_config& c) {
  if (c.algorithm != 1)
    throw SvsError(SVS_E_UNSUPPORTED, "only AlignmentType kNW (algorithm=1) is implemented; the reference "
                                      "always calls poa(seqs, 1)");
  const bool convex = c.g < c.e && !(c.g <= c.q || c.e >= c.c);
  if (!convex) throw SvsError(SVS_E_UNSUPPORTED, "only spoa's convex gap subtype (g<e, g>q, e<c) is implemented");
  // exactness conditions of the two-scan formulation (see poa_kernels.hip)
  if (!(c.g <= c.e && c.q <= c.c && c.g <= c.c && c.e <= c.c && c.g + c.q <= 2 * c.c))
    throw SvsError(SVS_E_UNSUPPORTED, "gap parameters outside the exact scan formulation");
}

namespace {

// Waves per job: enough column-chunk waves to put ~4 waves on each SIMD
// (1024 SIMDs on MI355X), only for jobs wide enough to split (>= 8 strips per
// wave) and pools small enough for the LDS boundary table.
int choose_waves_per_job(const std::vector<PoaJob>& jobs, size_t nj) {
  if (const char* e = std::getenv("SVS_POA_WPJ")) {
    const int w = std::atoi(e);
    if (w == 1 || w == 2 || w == 4) {
      for (size_t k = 0; k < nj; ++k)
        if (w > 1 && jobs[k].n_slots > kPoaMaxSlotsMultiWave) return 1;
      return w;
    }
  }
  uint32_t min_strips = 0xFFFFFFFFu;
  for (size_t k = 0; k < nj; ++k) {
    if (jobs[k].n_slots > kPoaMaxSlotsMultiWave) return 1;
    min_strips = std::min(min_strips, jobs[k].ls / 64);
  }
  int w = 1;
  while (w < 4 && static_cast<size_t>(w) * nj < 4096 && min_strips >= static_cast<uint32_t>(16 * w)) w *= 2;
  return w;
}

}  // namespace

namespace {

using Clock = std::chrono::steady_clock;
double ms_since(Clock::time_point t0) {
  return std::chrono::duration<double, std::milli>(Clock::now() - t0).count();
}

// One launch in flight: the jobs of one task group at one step.
struct Launch {
  std::vector<uint32_t> ids;       // task indices, one job each (tables in PoaTask::rows)
  std::vector<PoaJob> jobs;
  size_t step = 0;
  size_t n_aln = 0;
  PoaArena* arena = nullptr;
};

uint64_t job_bytes(const RowTables& tt, uint64_t L) {
  const uint64_t ls = round_up(L + 1, 64), V = tt.info.size();
  return V * ls * 2 + static_cast<uint64_t>(tt.n_slots) * 3 * ls * 4 + (V + L + 1) * 8;
}

// Packs the launch's tables into the arena's pinned buffer and enqueues
// H2D copy, kernel and D2H copies on the arena's stream (no host wait).
void pack_and_launch(svs_context* ctx, Launch& la, std::vector<PoaTask>& tasks, const PoaScore& score,
                     svs_poa_stats& st, double& host_ms) {
  auto th0 = Clock::now();
  const size_t nj = la.ids.size();
  la.jobs.assign(nj, PoaJob{});
  uint64_t n_rows = 0, n_pstart = 0, n_pred = 0, n_seq = 0, n_tb = 0, n_pool = 0, n_aln = 0;
  uint32_t max_preds = 0;
  for (size_t k = 0; k < nj; ++k) {
    const auto& tt = tasks[la.ids[k]].rows;
    const std::string& s = tasks[la.ids[k]].seqs[la.step];
    PoaJob& J = la.jobs[k];
    J.n_rows = static_cast<uint32_t>(tt.info.size());
    J.len = static_cast<uint32_t>(s.size());
    J.ls = static_cast<uint32_t>(round_up(J.len + 1, 64));
    J.n_slots = tt.n_slots;
    J.row_off = static_cast<uint32_t>(n_rows);
    J.pstart_off = static_cast<uint32_t>(n_pstart);
    J.pred_off = static_cast<uint32_t>(n_pred);
    J.seq_off = static_cast<uint32_t>(n_seq + 1);  // one zero pad byte precedes each read
    J.tb_off = n_tb;
    J.pool_off = n_pool;
    J.aln_off = n_aln;
    n_rows += J.n_rows;
    n_pstart += J.n_rows + 1;
    n_pred += tt.pred_row.size();
    n_seq += J.ls + 64;  // pad byte + read + tail pad
    n_tb += static_cast<uint64_t>(J.n_rows) * J.ls;
    n_pool += static_cast<uint64_t>(J.n_slots) * 3 * J.ls;
    n_aln += static_cast<uint64_t>(J.n_rows) + J.len + 1;
    max_preds = std::max(max_preds, tt.max_preds);
    st.dp_cells += static_cast<uint64_t>(J.n_rows + 1) * (J.len + 1);
  }
  if (max_preds > 31)
    throw SvsError(SVS_E_UNSUPPORTED, "a graph node has more than 31 in-edges (traceback code limit)");
  if (n_rows > 0xFFFFFFFFull || n_pred > 0xFFFFFFFFull || n_seq > 0xFFFFFFFFull)
    throw SvsError(SVS_E_UNSUPPORTED, "batch too large for 32-bit table offsets");
  la.n_aln = n_aln;
  size_t off = 0;
  auto sec = [&](size_t bytes) {
    const size_t o = off;
    off = round_up(off + bytes, 256);
    return o;
  };
  const size_t s_jobs = sec(nj * sizeof(PoaJob));
  const size_t s_info = sec(n_rows * 4), s_slot = sec(n_rows * 4), s_ps = sec(n_pstart * 4);
  const size_t s_col0 = sec(n_rows * 12);
  const size_t s_prow = sec(n_pred * 4), s_pslot = sec(n_pred * 4), s_seq = sec(n_seq + 256);
  PoaArena& A = *la.arena;
  A.h_in.ensure(off);
  char* hs = A.h_in.as<char>();
  std::memcpy(hs + s_jobs, la.jobs.data(), nj * sizeof(PoaJob));
  ctx->pool->parallel_for(nj, [&](size_t k) {
    const auto& tt = tasks[la.ids[k]].rows;
    const PoaJob& J = la.jobs[k];
    std::memcpy(hs + s_info + 4ull * J.row_off, tt.info.data(), 4ull * J.n_rows);
    std::memcpy(hs + s_slot + 4ull * J.row_off, tt.slot.data(), 4ull * J.n_rows);
    std::memcpy(hs + s_ps + 4ull * J.pstart_off, tt.pstart.data(), 4ull * (J.n_rows + 1));
    std::memcpy(hs + s_col0 + 12ull * J.row_off, tt.col0.data(), 12ull * J.n_rows);
    if (!tt.pred_row.empty()) {
      std::memcpy(hs + s_prow + 4ull * J.pred_off, tt.pred_row.data(), 4 * tt.pred_row.size());
      std::memcpy(hs + s_pslot + 4ull * J.pred_off, tt.pred_slot.data(), 4 * tt.pred_slot.size());
    }
    const std::string& s = tasks[la.ids[k]].seqs[la.step];
    std::memset(hs + s_seq + J.seq_off - 1, 0, J.ls + 64);
    std::memcpy(hs + s_seq + J.seq_off, s.data(), s.size());
  });
  host_ms += ms_since(th0);

  A.d_in.ensure(off);
  A.d_tb.ensure(n_tb * 2 + 4096);
  A.d_pool.ensure(n_pool * 4 + 4096);
  A.d_aln.ensure(n_aln * 8);
  A.d_alen.ensure(nj * 4);
  A.h_aln.ensure(n_aln * 8);
  A.h_alen.ensure(nj * 4);
  char* dg = A.d_in.as<char>();
  SVS_HIP(hipMemcpyAsync(dg, hs, off, hipMemcpyHostToDevice, A.stream));
  PoaLaunch pl;
  pl.jobs = reinterpret_cast<const PoaJob*>(dg + s_jobs);
  pl.n_jobs = static_cast<int>(nj);
  pl.score = score;
  pl.row_info = reinterpret_cast<const uint32_t*>(dg + s_info);
  pl.row_slot = reinterpret_cast<const uint32_t*>(dg + s_slot);
  pl.row_pstart = reinterpret_cast<const uint32_t*>(dg + s_ps);
  pl.pred_row = reinterpret_cast<const uint32_t*>(dg + s_prow);
  pl.pred_slot = reinterpret_cast<const uint32_t*>(dg + s_pslot);
  pl.col0 = reinterpret_cast<const int32_t*>(dg + s_col0);
  pl.seqs = reinterpret_cast<const uint8_t*>(dg + s_seq);
  pl.tb = A.d_tb.as<uint16_t>();
  pl.pool = A.d_pool.as<int32_t>();
  pl.aln = A.d_aln.as<int32_t>();
  pl.aln_len = A.d_alen.as<int32_t>();
  pl.waves_per_job = choose_waves_per_job(la.jobs, nj);
  SVS_HIP(hipEventRecord(A.ev0, A.stream));
  SVS_HIP(launch_poa_nw_convex(pl, A.stream));
  SVS_HIP(hipEventRecord(A.ev1, A.stream));
  SVS_HIP(hipMemcpyAsync(A.h_alen.ptr, pl.aln_len, nj * 4, hipMemcpyDeviceToHost, A.stream));
  SVS_HIP(hipMemcpyAsync(A.h_aln.ptr, pl.aln, n_aln * 8, hipMemcpyDeviceToHost, A.stream));
  SVS_HIP(hipEventRecord(A.done, A.stream));
  st.launches += 1;
  st.alignments += nj;
  st.tb_bytes += n_tb * 2;
  st.pool_bytes += n_pool * 4;
  st.h2d_bytes += off;
  st.d2h_bytes += n_aln * 8 + nj * 4;
}

// Waits for the launch and folds its alignments back into the graphs.
void finish(svs_context* ctx, Launch& la, std::vector<PoaTask>& tasks, svs_poa_stats& st, double& host_ms) {
  PoaArena& A = *la.arena;
  SVS_HIP(hipEventSynchronize(A.done));  // the other group's launch may still be queued behind it
  float ms = 0.f;
  SVS_HIP(hipEventElapsedTime(&ms, A.ev0, A.ev1));
  st.kernel_ms += ms;
  auto th0 = Clock::now();
  const int32_t* alen = A.h_alen.as<int32_t>();
  const int32_t* aout = A.h_aln.as<int32_t>();
  ctx->pool->parallel_for(la.ids.size(), [&](size_t k) {
    const int32_t n = alen[k];
    if (n < 0) throw SvsError(SVS_E_INTERNAL, "GPU traceback reported an inconsistent path");
    const int32_t* p = aout + 2 * la.jobs[k].aln_off;
    std::vector<int32_t> fwd(2 * static_cast<size_t>(n));
    for (int32_t x = 0; x < n; ++x) {
      fwd[2 * x] = p[2 * (n - 1 - x)];
      fwd[2 * x + 1] = p[2 * (n - 1 - x) + 1];
    }
    auto& t = tasks[la.ids[k]];
    t.graph.add_alignment_ranks(fwd, t.seqs[la.step]);
  });
  host_ms += ms_since(th0);
}

// Task group: a disjoint subset of the jobs that advances step by step with its
// own arena.  Groups alternate on one in-order stream, so while the GPU runs
// group B's step the host folds group A's alignments and enqueues A's next step.
struct Group {
  std::vector<uint32_t> members;
  size_t step = 0, max_steps = 0;
  Launch la;
  bool pending = false;
};

// Prepares the group's next step with GPU work and launches it (returns false
// when the group is finished).  Steps whose jobs exceed the group's device
// budget run as synchronous sub-launches.
bool advance(svs_context* ctx, Group& g, PoaArena* arena, std::vector<PoaTask>& tasks, const svs_poa_config& cfg,
             const PoaScore& score, size_t budget, svs_poa_stats& st, double& host_ms) {
  std::vector<uint8_t> needs(g.members.size());
  while (g.step < g.max_steps) {
    const size_t step = g.step;
    auto th0 = Clock::now();
    // sequences landing on an empty graph become a fresh chain on the host (no DP)
    ctx->pool->parallel_for(g.members.size(), [&](size_t i) {
      auto& t = tasks[g.members[i]];
      needs[i] = 0;
      if (step >= t.seqs.size() || t.seqs[step].empty()) return;
      if (t.graph.empty()) t.graph.add_alignment_nodes({}, t.seqs[step]);
      else needs[i] = 1;
    });
    std::vector<uint32_t> ids;
    for (size_t i = 0; i < g.members.size(); ++i)
      if (needs[i]) ids.push_back(g.members[i]);
    ++g.step;
    if (ids.empty()) { host_ms += ms_since(th0); continue; }
    ctx->pool->parallel_for(ids.size(), [&](size_t k) {
      auto& t = tasks[ids[k]];
      t.graph.export_rows(&t.rows);
      fill_col0(&t.rows, cfg.g, cfg.e, cfg.q, cfg.c);
    });
    host_ms += ms_since(th0);
    uint64_t total = 0;
    for (size_t k = 0; k < ids.size(); ++k) total += job_bytes(tasks[ids[k]].rows, tasks[ids[k]].seqs[step].size());
    if (total <= budget) {
      g.la.ids = std::move(ids);
      g.la.step = step;
      g.la.arena = arena;
      pack_and_launch(ctx, g.la, tasks, score, st, host_ms);
      g.pending = true;
      return true;
    }
    // over budget: consecutive synchronous sub-launches
    size_t first = 0;
    while (first < ids.size()) {
      size_t last = first;
      uint64_t bytes = 0;
      while (last < ids.size()) {
        const uint64_t b = job_bytes(tasks[ids[last]].rows, tasks[ids[last]].seqs[step].size());
        if (last > first && bytes + b > budget) break;
        bytes += b;
        ++last;
      }
      Launch sub;
      sub.ids.assign(ids.begin() + first, ids.begin() + last);
      sub.step = step;
      sub.arena = arena;
      pack_and_launch(ctx, sub, tasks, score, st, host_ms);
      finish(ctx, sub, tasks, st, host_ms);
      first = last;
    }
  }
  return false;
}

}  // namespace

void run_poa_tasks(svs_context* ctx, std::vector<PoaTask>& tasks, const svs_poa_config& cfg,
                   svs_poa_stats& st) {
  check_poa_config(cfg);
  const auto t_wall0 = Clock::now();
  double host_ms = 0.0;
  const PoaScore score{cfg.m, cfg.n, cfg.g, cfg.e, cfg.q, cfg.c};
  // Two groups once there are enough jobs to keep the GPU busy with half of them.
  const size_t n_groups = tasks.size() >= 64 ? 2 : 1;
  while (ctx->poa_arenas.size() < n_groups) ctx->poa_arenas.emplace_back(new PoaArena(ctx->device, ctx->stream));
  std::vector<Group> groups(n_groups);
  for (size_t i = 0; i < tasks.size(); ++i) {
    Group& g = groups[i % n_groups];
    g.members.push_back(static_cast<uint32_t>(i));
    g.max_steps = std::max(g.max_steps, tasks[i].seqs.size());
  }
  const size_t budget = ctx->device_budget / n_groups;
  try {
    for (size_t gi = 0; gi < n_groups; ++gi)
      advance(ctx, groups[gi], ctx->poa_arenas[gi].get(), tasks, cfg, score, budget, st, host_ms);
    bool any = true;
    while (any) {
      any = false;
      for (size_t gi = 0; gi < n_groups; ++gi) {
        Group& g = groups[gi];
        if (!g.pending) continue;
        finish(ctx, g.la, tasks, st, host_ms);
        g.pending = false;
        advance(ctx, g, ctx->poa_arenas[gi].get(), tasks, cfg, score, budget, st, host_ms);
        any = true;
      }
    }
  } catch (...) {
    for (auto& a : ctx->poa_arenas) (void)hipStreamSynchronize(a->stream);
    throw;
  }
  auto th0 = Clock::now();
  ctx->pool->parallel_for(tasks.size(), [&](size_t i) {
    auto& t = tasks[i];
    t.consensus = t.graph.consensus(cfg.min_coverage);
    if (cfg.genmsa) t.msa = t.graph.msa();
  });
  host_ms += ms_since(th0);
  st.host_graph_ms += host_ms;
  st.wall_ms += ms_since(t_wall0);
}

}  // namespace svs
