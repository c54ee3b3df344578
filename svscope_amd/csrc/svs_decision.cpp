// Pipelined per-window decision (svs_decision_batch, see include/svscope.h).
//
// One PoaScheduler carries every POA of the batch.  Window MSA tasks are queued
// first; when a window's MSA completes, its feature selection runs on the host
// pool (DataScanner.MSAFeatureSelection), and windows with >= 10 feature
// columns collect for EM.  EM batches run on a worker thread (own HIP stream,
// ward/maxclust serial on that thread) while the POA stream keeps going; their
// labels become consensus tasks that join the same scheduler.  So the GPU sees
// one continuous stream of read-vs-graph launches, and the only drain is at
// the end of the batch.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <chrono>
#include <cstring>
#include <future>
#include <memory>
#include <string>
#include <vector>

#include "features.hpp"
#include "svs_context.hpp"
#include "svs_internal.hpp"
#include "threadpool.hpp"

namespace svs {

namespace {

using Clock = std::chrono::steady_clock;
double ms_since(Clock::time_point t0) { return std::chrono::duration<double, std::milli>(Clock::now() - t0).count(); }

struct EmBatch {
  std::vector<int32_t> windows;
  std::future<std::unique_ptr<svs_em_result>> fut;
  Clock::time_point t0;
};

struct ConsRef {
  int32_t window;
  int32_t cluster;  // index into som (if < n_som) else germ
};

}  // namespace

svs_decision_result* run_decision(svs_context* ctx, int32_t n, const svs_decision_window* wins,
                                  const int64_t* seq_byte_start, const char* seq_bytes, const char* text,
                                  const uint8_t* is_tlabel, const svs_decision_config& cfg) {
  const auto t_wall = Clock::now();
  std::unique_ptr<svs_decision_result> res(new svs_decision_result());
  res->w.resize(n);
  svs_decision_stats& st = res->st;
  std::vector<WindowFeatures> feats(n);
  const size_t em_batch = cfg.em_batch > 0 ? static_cast<size_t>(cfg.em_batch) : 512;
  svs_poa_config pcfg = cfg.poa;
  pcfg.genmsa = 1;

  // inputs
  std::vector<std::vector<int32_t>> read_lens(n);
  std::vector<std::string> f5(n), f3(n);
  PoaScheduler sched(ctx, pcfg, st.poa);
  for (int32_t w = 0; w < n; ++w) {
    const svs_decision_window& W = wins[w];
    PoaTask t;
    t.genmsa = true;
    t.tag = static_cast<uint32_t>(w);
    for (int32_t k = 0; k < W.n_seqs; ++k) {
      const int64_t x = seq_byte_start[W.seq_start + k], y = seq_byte_start[W.seq_start + k + 1];
      if (y < x || x < 0) throw SvsError(SVS_E_INVALID, "seq_byte_start not monotone");
      t.seqs.emplace_back(y > x ? seq_bytes + x : "", static_cast<size_t>(y - x));
      if (k > 0) read_lens[w].push_back(static_cast<int32_t>(y - x));
    }
    f5[w].assign(W.flank5_len ? text + W.flank5_off : "", W.flank5_len);
    f3[w].assign(W.flank3_len ? text + W.flank3_off : "", W.flank3_len);
    sched.add(std::move(t));
  }
  st.msa_tasks = n;
  size_t msa_left = static_cast<size_t>(n);
  std::vector<int32_t> em_ready;
  std::unique_ptr<EmBatch> em;
  std::vector<ConsRef> cons_ref;  // consensus task id - n -> cluster
  // Pruning prior of a window's consensus tasks: their first alignment (read
  // against a one-read graph) has no score rate of its own yet, so it starts
  // from the window's last MSA rate less SVS_POA_CONS_PRIOR (score per read
  // base, default 1.5): two reads differ about twice as much as a read and
  // the reference.  Exact for any value: a bound above the optimum is retried
  // unpruned.  A negative value turns the prior off (the first alignment runs
  // unpruned).
  std::vector<double> msa_rate(static_cast<size_t>(n), 0.0);
  std::vector<uint8_t> msa_has_rate(static_cast<size_t>(n), 0);
  const double cons_prior = [] {
    const char* e = std::getenv("SVS_POA_CONS_PRIOR");
    return e ? std::atof(e) : 1.5;
  }();
  svs_em_config ecfg = cfg.em;
  ecfg.want_params = 0;

  // At most em_batch windows per EM launch, the first launch half that: when
  // every MSA of the batch completes in the same step, the GPU has nothing to
  // run until the first labels arrive, so the first EM launch is kept short.
  auto start_em = [&]() {
    auto b = std::make_unique<EmBatch>();
    const size_t cap = st.em_launches == 0 ? std::max<size_t>(1, em_batch / 2) : em_batch;
    const size_t take = std::min(cap, em_ready.size());
    b->windows.assign(em_ready.begin(), em_ready.begin() + static_cast<std::ptrdiff_t>(take));
    em_ready.erase(em_ready.begin(), em_ready.begin() + static_cast<std::ptrdiff_t>(take));
    b->t0 = Clock::now();
    std::vector<svs_em_window> ew(b->windows.size());
    int64_t xoff = 0;
    for (size_t i = 0; i < b->windows.size(); ++i) {
      const WindowFeatures& f = feats[b->windows[i]];
      ew[i] = svs_em_window{f.rows, f.n_feat, xoff, 0};
      xoff += static_cast<int64_t>(f.rows) * f.n_feat;
    }
    std::vector<uint8_t> X(static_cast<size_t>(std::max<int64_t>(1, xoff)));
    for (size_t i = 0; i < b->windows.size(); ++i) {
      const WindowFeatures& f = feats[b->windows[i]];
      if (!f.feat.empty()) std::memcpy(X.data() + ew[i].x_off, f.feat.data(), f.feat.size());
    }
    const int device = ctx->device;
    b->fut = std::async(std::launch::async, [ctx, device, ecfg, ew = std::move(ew), X = std::move(X)]() {
      SVS_HIP(hipSetDevice(device));
      return std::unique_ptr<svs_em_result>(
          run_em_cluster(ctx, static_cast<int32_t>(ew.size()), ew.data(), X.data(), ecfg, nullptr));
    });
    st.em_launches += 1;
    st.em_windows += static_cast<int64_t>(b->windows.size());
    em = std::move(b);
  };

  // EM results -> labels -> consensus tasks (only for windows that will report)
  auto consume_em = [&]() {
    std::unique_ptr<svs_em_result> r = em->fut.get();
    st.em_wall_ms += ms_since(em->t0);
    st.em_kernel_ms += r->kernel_ms;
    const auto t0 = Clock::now();
    const std::vector<int32_t> ws = std::move(em->windows);
    em.reset();
    ctx->pool->parallel_for(ws.size(), [&](size_t i) {
      const int32_t w = ws[i];
      auto& out = res->w[w];
      out.K = r->w[i].K;
      const bool ok = plan_clusters(feats[w], r->w[i].rclust.data(), is_tlabel + wins[w].tag_off, cfg.readcutoff,
                                    &out.som, &out.germ);
      if (!ok) {
        out.status = SVS_DEC_INDEX_ERROR;
        out.som.clear();
        out.germ.clear();
      } else {
        out.status = (!out.som.empty() && !out.germ.empty()) ? SVS_DEC_EMOUTPUT : SVS_DEC_EM;
      }
      std::vector<uint8_t>().swap(feats[w].feat);
      std::vector<uint8_t>().swap(feats[w].encoded);
    });
    for (int32_t w : ws) {
      auto& out = res->w[w];
      if (out.status != SVS_DEC_EMOUTPUT) continue;  // consensus would not be reported
      const int32_t ns = static_cast<int32_t>(out.som.size());
      for (int32_t c = 0; c < ns + static_cast<int32_t>(out.germ.size()); ++c) {
        ClusterPlan& p = c < ns ? out.som[c] : out.germ[c - ns];
        if (p.reads.empty()) continue;  // all reads empty: "-"
        PoaTask t;
        t.genmsa = false;
        t.tag = static_cast<uint32_t>(cons_ref.size());
        t.seqs = std::move(p.reads);
        if (cons_prior >= 0.0 && msa_has_rate[w]) {
          t.rate = msa_rate[w] - cons_prior;
          t.have_rate = true;
        }
        sched.add(std::move(t));
        cons_ref.push_back(ConsRef{w, c});
        st.consensus_tasks += 1;
      }
    }
    st.labelling_ms += ms_since(t0);
  };

  auto done = [&](const std::vector<uint32_t>& ids) {
    const auto t0 = Clock::now();
    std::vector<uint32_t> msa_ids;
    for (uint32_t id : ids) {
      PoaTask& t = sched.task(id);
      if (t.genmsa) {
        msa_ids.push_back(id);
        msa_rate[t.tag] = t.rate;
        msa_has_rate[t.tag] = t.have_rate ? 1 : 0;
      } else {
        const ConsRef& cr = cons_ref[t.tag];
        auto& out = res->w[cr.window];
        const int32_t ns = static_cast<int32_t>(out.som.size());
        ClusterPlan& p = cr.cluster < ns ? out.som[cr.cluster] : out.germ[cr.cluster - ns];
        p.consensus = std::move(t.consensus);
      }
    }
    ctx->pool->parallel_for(msa_ids.size(), [&](size_t i) {
      PoaTask& t = sched.task(msa_ids[i]);
      const int32_t w = static_cast<int32_t>(t.tag);
      msa_feature_select(t.msa, f5[w], f3[w], read_lens[w], wins[w].n_ids, cfg.hcutoff, cfg.scutoff, &feats[w]);
      std::vector<std::string>().swap(t.msa);
    });
    for (uint32_t id : msa_ids) {
      const int32_t w = static_cast<int32_t>(sched.task(id).tag);
      --msa_left;
      WindowFeatures& f = feats[w];
      if (f.rows != 0 && f.n_feat >= 10 && f.rows >= 3) {
        em_ready.push_back(w);
        continue;
      }
      // EMCluster with < 3 rows reads BICList[1] past its end (ReadsCluster.py:270)
      res->w[w].status = (f.rows != 0 && f.n_feat >= 10) ? SVS_DEC_INDEX_ERROR : SVS_DEC_NO_EM;
      std::vector<uint8_t>().swap(feats[w].feat);
      std::vector<uint8_t>().swap(feats[w].encoded);
    }
    st.features_ms += ms_since(t0);
  };

  auto poll = [&](bool block) {
    if (em && (block || em->fut.wait_for(std::chrono::seconds(0)) == std::future_status::ready)) {
      consume_em();
      block = false;  // new consensus tasks can run while the next EM batch does
    }
    if (!em && !em_ready.empty() && (em_ready.size() >= em_batch || msa_left == 0)) start_em();
    if (em && block) consume_em();
    return em != nullptr || !em_ready.empty();
  };

  try {
    sched.run(done, poll);
  } catch (...) {
    if (em && em->fut.valid()) em->fut.wait();
    throw;
  }
  st.wall_ms = ms_since(t_wall);
  st.poa.wall_ms = st.wall_ms;
  return res.release();
}

}  // namespace svs
