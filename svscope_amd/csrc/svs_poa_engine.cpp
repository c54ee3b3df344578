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

struct JobSizes {
  uint64_t tb, pool, aln;
};

struct Section {
  size_t off;
  size_t bytes;
};

}  // namespace

void run_poa_tasks(svs_context* ctx, std::vector<PoaTask>& tasks, const svs_poa_config& cfg,
                   svs_poa_stats& st) {
  check_poa_config(cfg);
  const auto t_wall0 = std::chrono::steady_clock::now();
  double host_ms = 0.0;
  size_t max_steps = 0;
  for (auto& t : tasks) max_steps = std::max(max_steps, t.seqs.size());
  const PoaScore score{cfg.m, cfg.n, cfg.g, cfg.e, cfg.q, cfg.c};

  std::vector<uint8_t> needs(tasks.size());
  std::vector<uint32_t> need;
  std::vector<RowTables> tables;
  for (size_t step = 0; step < max_steps; ++step) {
    auto th0 = std::chrono::steady_clock::now();
    // Sequences landing on an empty graph become a fresh chain on the host (no DP).
    ctx->pool->parallel_for(tasks.size(), [&](size_t i) {
      auto& t = tasks[i];
      needs[i] = 0;
      if (step >= t.seqs.size() || t.seqs[step].empty()) return;
      if (t.graph.empty()) {
        t.graph.add_alignment_nodes({}, t.seqs[step]);
      } else {
        needs[i] = 1;
      }
    });
    need.clear();
    for (size_t i = 0; i < tasks.size(); ++i)
      if (needs[i]) need.push_back(static_cast<uint32_t>(i));
    if (need.empty()) continue;
    tables.resize(need.size());
    ctx->pool->parallel_for(need.size(), [&](size_t k) {
      tasks[need[k]].graph.export_rows(&tables[k]);
      fill_col0(&tables[k], cfg.g, cfg.e, cfg.q, cfg.c);
    });
    host_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - th0).count();

    // Split into launches that fit the device budget.
    size_t first = 0;
    while (first < need.size()) {
      size_t last = first;
      uint64_t bytes = 0;
      while (last < need.size()) {
        const auto& tt = tables[last];
        const uint64_t L = tasks[need[last]].seqs[step].size();
        const uint64_t ls = round_up(L + 1, 64);
        const uint64_t V = tt.info.size();
        const uint64_t b = V * ls * 2 + static_cast<uint64_t>(tt.n_slots) * 3 * ls * 4 + (V + L + 1) * 8;
        if (last > first && bytes + b > ctx->device_budget) break;
        bytes += b;
        ++last;
      }
      const size_t nj = last - first;
      // ---- pack ----
      th0 = std::chrono::steady_clock::now();
      std::vector<PoaJob> jobs(nj);
      uint64_t n_rows = 0, n_pstart = 0, n_pred = 0, n_seq = 0, n_tb = 0, n_pool = 0, n_aln = 0;
      uint32_t max_preds = 0;
      for (size_t k = 0; k < nj; ++k) {
        const auto& tt = tables[first + k];
        const std::string& s = tasks[need[first + k]].seqs[step];
        PoaJob& J = jobs[k];
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
        n_seq += J.ls + 64;  // pad byte + read + tail pad (the kernel prefetches past the read end)
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
      size_t off = 0;
      auto sec = [&](size_t bytes) {
        Section s{off, bytes};
        off = round_up(off + bytes, 256);
        return s;
      };
      const Section s_jobs = sec(nj * sizeof(PoaJob));
      const Section s_info = sec(n_rows * 4), s_slot = sec(n_rows * 4), s_ps = sec(n_pstart * 4);
      const Section s_col0 = sec(n_rows * 12);
      // the kernel's load pipeline reads up to two strips (128 columns) past a row end
      const Section s_prow = sec(n_pred * 4), s_pslot = sec(n_pred * 4), s_seq = sec(n_seq + 256);
      ctx->h_stage.ensure(off);
      char* hs = ctx->h_stage.as<char>();
      std::memcpy(hs + s_jobs.off, jobs.data(), s_jobs.bytes);
      ctx->pool->parallel_for(nj, [&](size_t k) {
        const auto& tt = tables[first + k];
        const PoaJob& J = jobs[k];
        std::memcpy(hs + s_info.off + 4ull * J.row_off, tt.info.data(), 4ull * J.n_rows);
        std::memcpy(hs + s_slot.off + 4ull * J.row_off, tt.slot.data(), 4ull * J.n_rows);
        std::memcpy(hs + s_ps.off + 4ull * J.pstart_off, tt.pstart.data(), 4ull * (J.n_rows + 1));
        std::memcpy(hs + s_col0.off + 12ull * J.row_off, tt.col0.data(), 12ull * J.n_rows);
        if (!tt.pred_row.empty()) {
          std::memcpy(hs + s_prow.off + 4ull * J.pred_off, tt.pred_row.data(), 4 * tt.pred_row.size());
          std::memcpy(hs + s_pslot.off + 4ull * J.pred_off, tt.pred_slot.data(), 4 * tt.pred_slot.size());
        }
        const std::string& s = tasks[need[first + k]].seqs[step];
        std::memset(hs + s_seq.off + J.seq_off - 1, 0, J.ls + 64);
        std::memcpy(hs + s_seq.off + J.seq_off, s.data(), s.size());
      });
      host_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - th0).count();

      // ---- device ----
      ctx->d_row_info.ensure(off);  // one arena holds every input section
      ctx->d_tb.ensure(n_tb * 2 + 4096);
      ctx->d_pool.ensure(n_pool * 4 + 4096);
      ctx->d_aln.ensure(n_aln * 8);
      ctx->d_aln_len.ensure(nj * 4);
      ctx->h_aln.ensure(n_aln * 8);
      ctx->h_aln_len.ensure(nj * 4);
      char* dg = ctx->d_row_info.as<char>();
      SVS_HIP(hipMemcpyAsync(dg, hs, off, hipMemcpyHostToDevice, ctx->stream));
      PoaLaunch la;
      la.jobs = reinterpret_cast<const PoaJob*>(dg + s_jobs.off);
      la.n_jobs = static_cast<int>(nj);
      la.score = score;
      la.row_info = reinterpret_cast<const uint32_t*>(dg + s_info.off);
      la.row_slot = reinterpret_cast<const uint32_t*>(dg + s_slot.off);
      la.row_pstart = reinterpret_cast<const uint32_t*>(dg + s_ps.off);
      la.pred_row = reinterpret_cast<const uint32_t*>(dg + s_prow.off);
      la.pred_slot = reinterpret_cast<const uint32_t*>(dg + s_pslot.off);
      la.col0 = reinterpret_cast<const int32_t*>(dg + s_col0.off);
      la.seqs = reinterpret_cast<const uint8_t*>(dg + s_seq.off);
      la.tb = ctx->d_tb.as<uint16_t>();
      la.pool = ctx->d_pool.as<int32_t>();
      la.aln = ctx->d_aln.as<int32_t>();
      la.aln_len = ctx->d_aln_len.as<int32_t>();
      la.waves_per_job = choose_waves_per_job(jobs, nj);
      SVS_HIP(hipEventRecord(ctx->ev_start, ctx->stream));
      SVS_HIP(launch_poa_nw_convex(la, ctx->stream));
      SVS_HIP(hipEventRecord(ctx->ev_stop, ctx->stream));
      SVS_HIP(hipMemcpyAsync(ctx->h_aln_len.ptr, la.aln_len, nj * 4, hipMemcpyDeviceToHost, ctx->stream));
      SVS_HIP(hipMemcpyAsync(ctx->h_aln.ptr, la.aln, n_aln * 8, hipMemcpyDeviceToHost, ctx->stream));
      SVS_HIP(hipStreamSynchronize(ctx->stream));
      float ms = 0.f;
      SVS_HIP(hipEventElapsedTime(&ms, ctx->ev_start, ctx->ev_stop));
      st.kernel_ms += ms;
      st.launches += 1;
      st.alignments += nj;
      st.tb_bytes += n_tb * 2;
      st.pool_bytes += n_pool * 4;
      st.h2d_bytes += off;
      st.d2h_bytes += n_aln * 8 + nj * 4;

      // ---- fold alignments back into the graphs ----
      th0 = std::chrono::steady_clock::now();
      const int32_t* alen = ctx->h_aln_len.as<int32_t>();
      const int32_t* aout = ctx->h_aln.as<int32_t>();
      ctx->pool->parallel_for(nj, [&](size_t k) {
        const int32_t n = alen[k];
        if (n < 0) throw SvsError(SVS_E_INTERNAL, "GPU traceback reported an inconsistent path");
        const int32_t* p = aout + 2 * jobs[k].aln_off;
        std::vector<int32_t> fwd(2 * static_cast<size_t>(n));
        for (int32_t x = 0; x < n; ++x) {
          fwd[2 * x] = p[2 * (n - 1 - x)];
          fwd[2 * x + 1] = p[2 * (n - 1 - x) + 1];
        }
        auto& t = tasks[need[first + k]];
        t.graph.add_alignment_ranks(fwd, t.seqs[step]);
      });
      host_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - th0).count();
      first = last;
    }
  }
  auto th0 = std::chrono::steady_clock::now();
  ctx->pool->parallel_for(tasks.size(), [&](size_t i) {
    auto& t = tasks[i];
    t.consensus = t.graph.consensus(cfg.min_coverage);
    if (cfg.genmsa) t.msa = t.graph.msa();
  });
  host_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - th0).count();
  st.host_graph_ms += host_ms;
  st.wall_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_wall0).count();
}

}  // namespace svs
