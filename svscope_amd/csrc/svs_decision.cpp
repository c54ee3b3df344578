// Pipelined per-window decision as a streaming session
// (svs_decision_session_*, svs_decision_batch; see include/svscope.h).
//
// A session owns one worker thread and one PoaScheduler that carries every POA
// of every batch submitted to it.  Window MSA tasks are queued as batches
// arrive; when a window's MSA completes, its feature selection runs on the
// host pool (DataScanner.MSAFeatureSelection), and windows with >= 10 feature
// columns collect for EM.  EM batches run on a worker thread (own HIP stream,
// ward/maxclust serial on that thread) while the POA stream keeps going; their
// labels become consensus tasks that join the same scheduler.  Batches never
// drain the GPU between them: the MSA tasks of batch b+1 fill the slots that
// batch b's tail leaves, so the GPU sees one continuous stream of
// read-vs-graph launches for the whole session (the reference runs the same
// windows through a 6-process Pool, SVscope.py:158-165,220-233).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <exception>
#include <future>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <string>
#include <thread>
#include <vector>

#include "features.hpp"
#include "svs_context.hpp"
#include "svs_internal.hpp"
#include "threadpool.hpp"

namespace svs {

namespace {

using Clock = std::chrono::steady_clock;
double ms_since(Clock::time_point t0) { return std::chrono::duration<double, std::milli>(Clock::now() - t0).count(); }

// One submitted batch.  The input arrays are the caller's: they stay valid
// until the batch has been waited for (svs_decision_session_submit).
struct Batch {
  int64_t ticket = 0;
  int32_t n = 0;
  const svs_decision_window* wins = nullptr;
  const int64_t* seq_byte_start = nullptr;
  const char* seq_bytes = nullptr;
  const char* text = nullptr;
  const uint8_t* is_tlabel = nullptr;
  std::unique_ptr<svs_decision_result> res;
  std::vector<WindowFeatures> feats;
  std::vector<std::vector<int32_t>> read_lens;
  std::vector<std::string> f5, f3;
  std::vector<double> msa_rate;
  std::vector<uint8_t> msa_has_rate;
  std::vector<int32_t> cons_left;  // consensus tasks still running, per window
  int32_t left = 0;                // windows not yet complete
  Clock::time_point t0;
  std::vector<PoaTask> built;      // the windows' MSA tasks (prepare_batch), until queued
};

// Builds a submitted batch's window MSA tasks and per-window state, on the
// session's builder thread: a batch's reads are ~100 MB of copies and letter
// checks, 15-60 ms that were spent on the worker thread, which also issues the
// POA launches, so a group whose fold chain ended meanwhile waited for it.
void prepare_batch(Batch& b, const svs_decision_config& cfg, bool device_features_on, ThreadPool* pool) {
  b.t0 = Clock::now();
  b.res.reset(new svs_decision_result());
  b.res->w.resize(b.n);
  b.feats.resize(b.n);
  b.read_lens.resize(b.n);
  b.f5.resize(b.n);
  b.f3.resize(b.n);
  b.msa_rate.assign(b.n, 0.0);
  b.msa_has_rate.assign(b.n, 0);
  b.cons_left.assign(b.n, 0);
  b.left = b.n;
  const uint32_t prio = static_cast<uint32_t>(b.ticket);
  b.built.resize(static_cast<size_t>(b.n));
  pool->parallel_for(static_cast<size_t>(b.n), [&](size_t wi) {
    const int32_t w = static_cast<int32_t>(wi);
    const svs_decision_window& W = b.wins[w];
    PoaTask& t = b.built[wi];
    t.genmsa = true;
    t.prio = prio;
    for (int32_t k = 0; k < W.n_seqs; ++k) {
      const int64_t x = b.seq_byte_start[W.seq_start + k], y = b.seq_byte_start[W.seq_start + k + 1];
      // (ranges checked on submit, check_decision_windows)
      t.seqs.emplace_back(y > x ? b.seq_bytes + x : "", static_cast<size_t>(y - x));
      if (k > 0) b.read_lens[w].push_back(static_cast<int32_t>(y - x));
    }
    b.f5[w].assign(W.flank5_len ? b.text + W.flank5_off : "", W.flank5_len);
    b.f3[w].assign(W.flank3_len ? b.text + W.flank3_off : "", W.flank3_len);
    // the window's feature selection on the device when its graph is there
    // (else, or for a letter SeqEncoder rejects, the host's from the MSA rows)
    t.features = device_features_on;
    try {
      t.feat_params = device_feature_params(t.seqs, b.f5[w], b.f3[w], b.read_lens[w], W.n_ids, cfg.hcutoff,
                                            cfg.scutoff);
    } catch (const SvsError&) {
      t.feat_params.ok = false;
    }
  });
}

struct WinRef {
  Batch* b;
  int32_t w;
};

// What a scheduler task belongs to: a window MSA (cluster < 0) or the
// consensus of one cluster (somatic first, then germline).
struct TaskRef {
  Batch* b = nullptr;
  int32_t w = 0;
  int32_t cluster = -1;
};

struct EmBatch {
  std::vector<WinRef> windows;
  std::future<std::unique_ptr<svs_em_result>> fut;
  Clock::time_point t0;
};

}  // namespace

}  // namespace svs

struct svs_decision_session {
  svs_context* ctx = nullptr;
  svs_decision_config cfg{};
  std::thread worker;
  std::mutex mu;
  std::condition_variable cv_work, cv_done;
  std::deque<std::unique_ptr<svs::Batch>> to_build;            // submitted, tasks not yet built
  std::deque<std::unique_ptr<svs::Batch>> inbox;               // built, not yet queued
  std::map<int64_t, std::unique_ptr<svs::Batch>> in_flight;    // queued in the scheduler
  std::map<int64_t, std::unique_ptr<svs::Batch>> finished;     // complete, not yet waited for
  std::set<int64_t> waited;                                    // tickets already returned by wait
  int64_t next_ticket = 1;
  int64_t building = 0;    // batches submitted and not yet in the inbox
  bool closing = false;
  bool em_signal = false;  // the EM worker finished a launch
  bool device_features_on = true;
  std::exception_ptr error;
  svs_decision_stats published{};  // cumulative statistics, as of the last completed batch
  std::thread builder;
  std::condition_variable cv_build;

  void run();         // worker thread body
  void build_loop();  // builder thread body (prepare_batch)
  // (under mu) nothing submitted is still on its way to the worker
  bool nothing_arriving() const { return inbox.empty() && building == 0; }
};

namespace svs {

namespace {

// The session's pipeline state; lives on the worker thread only.
class Pipeline {
 public:
  explicit Pipeline(svs_decision_session* s)
      : S(s), ctx(s->ctx), cfg(s->cfg), sched(ctx, poa_cfg(s->cfg), st.poa) {
    em_batch = cfg.em_batch > 0 ? static_cast<size_t>(cfg.em_batch) : 512;
    // Pruning prior of a window's consensus tasks: their first alignment (read
    // against a one-read graph) has no score rate of its own yet, so it starts
    // from the window's last MSA rate less SVS_POA_CONS_PRIOR (score per read
    // base, default 1.5): two reads differ about twice as much as a read and
    // the reference.  Exact for any value: a bound above the optimum is retried
    // unpruned.  A negative value turns the prior off (the first alignment runs
    // unpruned).
    const char* e = std::getenv("SVS_POA_CONS_PRIOR");
    cons_prior = e ? std::atof(e) : 1.5;
    ecfg = cfg.em;
    ecfg.want_params = 0;
    t_wall = Clock::now();
  }

  void run() {
    try {
      sched.run([this](const std::vector<uint32_t>& ids) { done(ids); }, [this](bool block) { return poll(block); });
    } catch (...) {
      if (em && em->fut.valid()) em->fut.wait();
      throw;
    }
    publish();
  }

 private:
  static svs_poa_config poa_cfg(const svs_decision_config& c) {
    svs_poa_config p = c.poa;
    p.genmsa = 1;
    return p;
  }

  uint32_t new_ref(const TaskRef& r) {
    if (!free_refs.empty()) {
      const uint32_t k = free_refs.back();
      free_refs.pop_back();
      refs[k] = r;
      return k;
    }
    refs.push_back(r);
    return static_cast<uint32_t>(refs.size() - 1);
  }

  // Queues a built batch's window MSAs in window order (worker thread; the
  // tasks were built by prepare_batch on the builder thread).
  void ingest(std::unique_ptr<Batch> bp) {
    Batch& b = *bp;
    for (int32_t w = 0; w < b.n; ++w) {
      b.built[w].tag = new_ref(TaskRef{&b, w, -1});
      sched.add(std::move(b.built[w]));
    }
    std::vector<PoaTask>().swap(b.built);
    st.msa_tasks += b.n;
    msa_outstanding += static_cast<size_t>(b.n);
    Batch* raw = bp.get();
    {
      std::lock_guard<std::mutex> lk(S->mu);
      S->in_flight.emplace(raw->ticket, std::move(bp));
    }
    if (raw->n == 0) complete_batch(*raw);
  }

  void publish() {
    st.wall_ms = ms_since(t_wall);
    st.poa.wall_ms = st.wall_ms;
    std::lock_guard<std::mutex> lk(S->mu);
    S->published = st;
    S->published.poa.host_graph_ms += sched.host_ms();
  }

  void complete_batch(Batch& b) {
    b.feats.clear();
    b.feats.shrink_to_fit();
    b.res->st = st;
    b.res->st.wall_ms = ms_since(b.t0);
    publish();
    {
      std::lock_guard<std::mutex> lk(S->mu);
      auto it = S->in_flight.find(b.ticket);
      S->finished.emplace(b.ticket, std::move(it->second));
      S->in_flight.erase(it);
    }
    S->cv_done.notify_all();
  }

  void window_complete(Batch& b) {
    if (--b.left == 0) complete_batch(b);
  }

  // At most em_batch windows per EM launch, the first launch half that: when
  // every MSA completes in the same step, the GPU has nothing to run until the
  // first labels arrive, so the first EM launch is kept short.
  void start_em() {
    auto e = std::make_unique<EmBatch>();
    const size_t cap = st.em_launches == 0 ? std::max<size_t>(1, em_batch / 2) : em_batch;
    const size_t take = std::min(cap, em_ready.size());
    e->windows.assign(em_ready.begin(), em_ready.begin() + static_cast<std::ptrdiff_t>(take));
    em_ready.erase(em_ready.begin(), em_ready.begin() + static_cast<std::ptrdiff_t>(take));
    e->t0 = Clock::now();
    std::vector<svs_em_window> ew(e->windows.size());
    int64_t xoff = 0;
    for (size_t i = 0; i < e->windows.size(); ++i) {
      const WindowFeatures& f = e->windows[i].b->feats[e->windows[i].w];
      ew[i] = svs_em_window{f.rows, f.n_feat, xoff, 0};
      xoff += static_cast<int64_t>(f.rows) * f.n_feat;
      // §8(d): sum over K = 1 .. kmax-1 of 41 x 2 N (5 nf) K
      const double kk = std::max(0, std::min(ecfg.max_c + 1, f.rows) - 1);
      st.em_flops += 410.0 * f.rows * f.n_feat * kk * (kk + 1) / 2;
    }
    std::vector<uint8_t> X(static_cast<size_t>(std::max<int64_t>(1, xoff)));
    ctx->pool->parallel_for(e->windows.size(), [&](size_t i) {
      const WindowFeatures& f = e->windows[i].b->feats[e->windows[i].w];
      if (!f.feat.empty()) std::memcpy(X.data() + ew[i].x_off, f.feat.data(), f.feat.size());
    });
    svs_context* c = ctx;
    svs_decision_session* s = S;
    const svs_em_config ec = ecfg;
    e->fut = std::async(std::launch::async, [c, s, ec, ew = std::move(ew), X = std::move(X)]() {
      struct Signal {  // wakes the session worker however the launch ends
        svs_decision_session* s;
        ~Signal() {
          {
            std::lock_guard<std::mutex> lk(s->mu);
            s->em_signal = true;
          }
          s->cv_work.notify_all();
        }
      } sig{s};
      SVS_HIP(hipSetDevice(c->device));
      return std::unique_ptr<svs_em_result>(
          run_em_cluster(c, static_cast<int32_t>(ew.size()), ew.data(), X.data(), ec, nullptr));
    });
    st.em_launches += 1;
    st.em_windows += static_cast<int64_t>(e->windows.size());
    em = std::move(e);
  }

  // EM results -> labels -> consensus tasks (only for windows that will report)
  void consume_em() {
    std::unique_ptr<svs_em_result> r = em->fut.get();
    st.em_wall_ms += ms_since(em->t0);
    st.em_kernel_ms += r->kernel_ms;
    st.em_reruns += r->em_reruns;
    const auto t0 = Clock::now();
    const std::vector<WinRef> ws = std::move(em->windows);
    em.reset();
    ctx->pool->parallel_for(ws.size(), [&](size_t i) {
      Batch& b = *ws[i].b;
      const int32_t w = ws[i].w;
      auto& out = b.res->w[w];
      out.K = r->w[i].K;
      const bool ok = plan_clusters(b.feats[w], r->w[i].rclust.data(), b.is_tlabel + b.wins[w].tag_off,
                                    cfg.readcutoff, &out.som, &out.germ);
      if (!ok) {
        out.status = SVS_DEC_INDEX_ERROR;
        out.som.clear();
        out.germ.clear();
      } else {
        out.status = (!out.som.empty() && !out.germ.empty()) ? SVS_DEC_EMOUTPUT : SVS_DEC_EM;
      }
      std::vector<uint8_t>().swap(b.feats[w].feat);
      std::vector<std::string>().swap(b.feats[w].row_reads);
    });
    for (const WinRef& wr : ws) {
      Batch& b = *wr.b;
      const int32_t w = wr.w;
      auto& out = b.res->w[w];
      int32_t added = 0;
      if (out.status == SVS_DEC_EMOUTPUT) {  // otherwise the consensus would not be reported
        const int32_t ns = static_cast<int32_t>(out.som.size());
        for (int32_t c = 0; c < ns + static_cast<int32_t>(out.germ.size()); ++c) {
          ClusterPlan& p = c < ns ? out.som[c] : out.germ[c - ns];
          if (p.reads.empty()) continue;  // all reads empty: "-"
          PoaTask t;
          t.genmsa = false;
          t.prio = static_cast<uint32_t>(b.ticket);
          t.tag = new_ref(TaskRef{&b, w, c});
          t.seqs = std::move(p.reads);
          if (cons_prior >= 0.0 && b.msa_has_rate[w]) {
            t.rate = b.msa_rate[w] - cons_prior;
            t.have_rate = true;
          }
          sched.add(std::move(t));
          st.consensus_tasks += 1;
          ++added;
        }
      }
      b.cons_left[w] = added;
      if (added == 0) window_complete(b);
    }
    st.labelling_ms += ms_since(t0);
  }

  void done(const std::vector<uint32_t>& ids) {
    const auto t0 = Clock::now();
    std::vector<std::pair<uint32_t, WinRef>> msa_ids;
    for (uint32_t id : ids) {
      PoaTask& t = sched.task(id);
      const TaskRef ref = refs[t.tag];
      free_refs.push_back(t.tag);
      Batch& b = *ref.b;
      if (!t.error.empty()) {
        // past an engine limit: this window fails alone
        auto& out = b.res->w[ref.w];
        if (out.status != SVS_DEC_FAILED) out.error = t.error;
        out.status = SVS_DEC_FAILED;
        if (ref.cluster < 0) {
          --msa_outstanding;
          window_complete(b);
        } else if (--b.cons_left[ref.w] == 0) {
          window_complete(b);
        }
        continue;
      }
      if (ref.cluster < 0) {
        msa_ids.emplace_back(id, WinRef{&b, ref.w});
        b.msa_rate[ref.w] = t.rate;
        b.msa_has_rate[ref.w] = t.have_rate ? 1 : 0;
      } else {
        auto& out = b.res->w[ref.w];
        const int32_t ns = static_cast<int32_t>(out.som.size());
        ClusterPlan& p = ref.cluster < ns ? out.som[ref.cluster] : out.germ[ref.cluster - ns];
        p.consensus = std::move(t.consensus);
        if (--b.cons_left[ref.w] == 0) window_complete(b);
      }
    }
    ctx->pool->parallel_for(msa_ids.size(), [&](size_t i) {
      PoaTask& t = sched.task(msa_ids[i].first);
      Batch& b = *msa_ids[i].second.b;
      const int32_t w = msa_ids[i].second.w;
      if (t.n_feat >= 0) {
        // seqdatamx from the final fold kernel (poa_fold.hip msa_features)
        device_features(t.seqs, b.read_lens[w], b.wins[w].n_ids, t.feat_params, t.n_feat, std::move(t.feat),
                        &b.feats[w]);
        if (!t.msa.empty()) {
          // SVS_POA_VERIFY_GRAPH: the MSA rows came back too; the host's
          // selection from them must be the same
          WindowFeatures h;
          msa_feature_select(t.msa, b.f5[w], b.f3[w], b.read_lens[w], b.wins[w].n_ids, cfg.hcutoff, cfg.scutoff, &h);
          const WindowFeatures& d = b.feats[w];
          if (h.rows != d.rows || h.n_feat != d.n_feat || h.feat != d.feat || h.id_map != d.id_map ||
              h.row_reads != d.row_reads)
            throw SvsError(SVS_E_INTERNAL, "device feature selection differs from the host's (window " +
                                               std::to_string(w) + ": " + std::to_string(d.n_feat) + " vs " +
                                               std::to_string(h.n_feat) + " columns)");
        }
      } else {
        msa_feature_select(t.msa, b.f5[w], b.f3[w], b.read_lens[w], b.wins[w].n_ids, cfg.hcutoff, cfg.scutoff,
                           &b.feats[w]);
      }
      std::vector<std::string>().swap(t.msa);
    });
    for (const auto& m : msa_ids) {
      Batch& b = *m.second.b;
      const int32_t w = m.second.w;
      --msa_outstanding;
      WindowFeatures& f = b.feats[w];
      if (f.rows != 0 && f.n_feat >= 10 && f.rows >= 3) {
        em_ready.push_back(m.second);
        continue;
      }
      // EMCluster with < 3 rows reads BICList[1] past its end (ReadsCluster.py:270)
      b.res->w[w].status = (f.rows != 0 && f.n_feat >= 10) ? SVS_DEC_INDEX_ERROR : SVS_DEC_NO_EM;
      std::vector<uint8_t>().swap(f.feat);
      std::vector<std::string>().swap(f.row_reads);
      window_complete(b);
    }
    st.features_ms += ms_since(t0);
  }

  // Moves submitted batches into the scheduler; true if any arrived.
  bool take_inbox() {
    std::deque<std::unique_ptr<Batch>> got;
    {
      std::lock_guard<std::mutex> lk(S->mu);
      got.swap(S->inbox);
      S->em_signal = false;
    }
    for (auto& b : got) ingest(std::move(b));
    return !got.empty();
  }

  bool em_ready_now() const { return em && em->fut.wait_for(std::chrono::seconds(0)) == std::future_status::ready; }

  // Between launches: new batches, finished EM launches, EM starts.  Returns
  // true while outside work may still add tasks (an open session always may);
  // with block=true (the scheduler is idle) it waits for such work.
  bool poll(bool block) {
    take_inbox();
    if (em && (em_ready_now() || (block && msa_outstanding == 0 && !batches_arriving()))) {
      // blocking on the EM result is only worth it when nothing else can arrive
      consume_em();
      block = false;  // new consensus tasks can run while the next EM batch does
    }
    if (!em && !em_ready.empty() && (em_ready.size() >= em_batch || msa_outstanding == 0)) start_em();
    if (block) {
      std::unique_lock<std::mutex> lk(S->mu);
      // (a closing session still waits for batches its builder has not handed over)
      S->cv_work.wait(lk, [&] { return !S->inbox.empty() || (S->closing && S->building == 0) || S->em_signal; });
      const bool closing = S->closing && S->nothing_arriving();
      lk.unlock();
      take_inbox();
      if (em && (em_ready_now() || closing)) consume_em();
      if (!em && !em_ready.empty() && (em_ready.size() >= em_batch || msa_outstanding == 0)) start_em();
    }
    std::lock_guard<std::mutex> lk(S->mu);
    const bool open = !S->closing || !S->nothing_arriving();
    return open || em != nullptr || !em_ready.empty();
  }

  bool batches_arriving() {
    std::lock_guard<std::mutex> lk(S->mu);
    return !S->nothing_arriving();
  }

  svs_decision_session* S;
  svs_context* ctx;
  const svs_decision_config cfg;
  svs_decision_stats st{};
  PoaScheduler sched;
  size_t em_batch = 512;
  double cons_prior = 1.5;
  svs_em_config ecfg{};
  Clock::time_point t_wall;
  size_t msa_outstanding = 0;  // window MSAs queued or running, all batches
  std::vector<WinRef> em_ready;
  std::unique_ptr<EmBatch> em;
  std::vector<TaskRef> refs;
  std::vector<uint32_t> free_refs;
};

}  // namespace

}  // namespace svs

void svs_decision_session::build_loop() {
  // the builder's own pool: the context's belongs to the worker thread
  // (ThreadPool::parallel_for is not reentrant across threads)
  svs::ThreadPool pool(4);
  for (;;) {
    std::unique_ptr<svs::Batch> b;
    {
      std::unique_lock<std::mutex> lk(mu);
      cv_build.wait(lk, [&] { return !to_build.empty() || closing; });
      if (to_build.empty()) return;  // closing, every batch handed over
      b = std::move(to_build.front());
      to_build.pop_front();
    }
    try {
      svs::prepare_batch(*b, cfg, device_features_on, &pool);
    } catch (...) {
      // the batch is dropped: its waiters see the error
      {
        std::lock_guard<std::mutex> lk(mu);
        if (!error) error = std::current_exception();
        --building;
      }
      cv_work.notify_all();
      cv_done.notify_all();
      continue;
    }
    {
      std::lock_guard<std::mutex> lk(mu);
      inbox.push_back(std::move(b));
      --building;
    }
    cv_work.notify_all();
  }
}

void svs_decision_session::run() {
  try {
    SVS_HIP(hipSetDevice(ctx->device));
    svs::Pipeline p(this);
    p.run();
  } catch (...) {
    std::lock_guard<std::mutex> lk(mu);
    error = std::current_exception();
  }
  cv_done.notify_all();
}

namespace svs {

svs_decision_session* open_decision_session(svs_context* ctx, const svs_decision_config& cfg) {
  check_poa_config(cfg.poa);
  std::unique_ptr<svs_decision_session> s(new svs_decision_session());
  s->ctx = ctx;
  s->cfg = cfg;
  // SVS_DEVICE_FEATURES=0: the window MSA rows come back and the host
  // selects the features (the round-3 path)
  const char* df = std::getenv("SVS_DEVICE_FEATURES");
  s->device_features_on = !(df && std::string(df) == "0");
  svs_decision_session* raw = s.get();
  s->builder = std::thread([raw] { raw->build_loop(); });
  s->worker = std::thread([raw] { raw->run(); });
  return s.release();
}

int64_t submit_decision_batch(svs_decision_session* s, int32_t n, const svs_decision_window* wins,
                              const int64_t* seq_byte_start, const char* seq_bytes, const char* text,
                              const uint8_t* is_tlabel) {
  std::unique_ptr<Batch> b(new Batch());
  b->n = n;
  b->wins = wins;
  b->seq_byte_start = seq_byte_start;
  b->seq_bytes = seq_bytes;
  b->text = text;
  b->is_tlabel = is_tlabel;
  int64_t ticket;
  {
    std::lock_guard<std::mutex> lk(s->mu);
    if (s->error) std::rethrow_exception(s->error);
    if (s->closing) throw SvsError(SVS_E_INVALID, "decision session is closing");
    ticket = s->next_ticket++;
    b->ticket = ticket;
    s->to_build.push_back(std::move(b));
    ++s->building;
  }
  s->cv_build.notify_all();
  return ticket;
}

svs_decision_result* wait_decision_batch(svs_decision_session* s, int64_t ticket) {
  std::unique_lock<std::mutex> lk(s->mu);
  if (ticket <= 0 || ticket >= s->next_ticket) throw SvsError(SVS_E_INVALID, "unknown decision ticket");
  // a ticket is returned once; waiting for it again would never wake
  if (s->waited.count(ticket)) throw SvsError(SVS_E_INVALID, "decision ticket already waited for");
  s->waited.insert(ticket);
  s->cv_done.wait(lk, [&] { return s->error || s->finished.count(ticket) != 0; });
  auto it = s->finished.find(ticket);
  if (it == s->finished.end()) std::rethrow_exception(s->error);
  std::unique_ptr<Batch> b = std::move(it->second);
  s->finished.erase(it);
  return b->res.release();
}

void session_stats(svs_decision_session* s, svs_decision_stats* out) {
  std::lock_guard<std::mutex> lk(s->mu);
  *out = s->published;
}

// Finishes every submitted batch, joins the worker and frees the session.
// Returns the worker's error, if any.
#ifdef SVS_WG_TIMES
extern "C" int svs_debug_wg_times_dump(const char* path);
#endif

std::exception_ptr close_decision_session(svs_decision_session* s) {
  {
    std::lock_guard<std::mutex> lk(s->mu);
    s->closing = true;
  }
  s->cv_build.notify_all();
  s->cv_work.notify_all();
  if (s->builder.joinable()) s->builder.join();
  if (s->worker.joinable()) s->worker.join();
#ifdef SVS_WG_TIMES
  if (const char* p = std::getenv("SVS_WG_TIMES_OUT")) std::fprintf(stderr, "[svs] wg times: %d\n", svs_debug_wg_times_dump(p));
#endif
  std::exception_ptr e = s->error;
  delete s;
  return e;
}

svs_decision_result* run_decision(svs_context* ctx, int32_t n, const svs_decision_window* wins,
                                  const int64_t* seq_byte_start, const char* seq_bytes, const char* text,
                                  const uint8_t* is_tlabel, const svs_decision_config& cfg) {
  svs_decision_session* s = open_decision_session(ctx, cfg);
  svs_decision_result* r = nullptr;
  std::exception_ptr err;
  try {
    r = wait_decision_batch(s, submit_decision_batch(s, n, wins, seq_byte_start, seq_bytes, text, is_tlabel));
  } catch (...) {
    err = std::current_exception();
  }
  std::exception_ptr e2 = close_decision_session(s);
  if (err) {
    delete r;
    std::rethrow_exception(err);
  }
  if (e2) {
    delete r;
    std::rethrow_exception(e2);
  }
  return r;
}

}  // namespace svs
