// Batched POA engine: continuous-batching driver over many independent POA
// tasks (one task = one pyspoa `poa(seqs, 1)` call of the reference: a window
// MSA at DataScanner.py:206,213 or a cluster consensus at DecisionMaker.py:160,171).
//
// Each launch aligns the next sequence of every active task of a group: the
// host exports each task's rank-ordered row tables, one HIP launch runs every
// read-vs-graph DP and its traceback, and the host folds the alignments back
// into the graphs in parallel.  Completed tasks leave after every step and
// queued ones take their place (PoaScheduler).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <cmath>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <functional>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "poa_dgraph.hpp"
#include "poa_graph.hpp"
#include "svs_busy.hpp"
#include "svs_context.hpp"
#include "svs_devarena.hpp"
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
  // exactness conditions of the two-scan formulation (see poa_wave.hpp strip_gaps)
  if (!(c.g <= c.e && c.q <= c.c && c.g <= c.c && c.e <= c.c && c.g + c.q <= 2 * c.c))
    throw SvsError(SVS_E_UNSUPPORTED, "gap parameters outside the exact scan formulation");
  // the strip kernel stores F and O as 8-bit distances to H clamped at e-g+1, c-q+1
  if (c.e - c.g + 1 > 255 || c.c - c.q + 1 > 255)
    throw SvsError(SVS_E_UNSUPPORTED, "gap parameters too far apart for the packed F/O pool");
  // the pruning bound multiplies path-length differences (< 2^16) by scores
  // with 24-bit multiplies
  for (const int32_t x : {c.m, c.n, c.g, c.e, c.q, c.c})
    if (x > 4096 || x < -4096) throw SvsError(SVS_E_UNSUPPORTED, "scores beyond +-4096 are not supported");
}

namespace {

using Clock = std::chrono::steady_clock;
double ms_since(Clock::time_point t0) {
  return std::chrono::duration<double, std::milli>(Clock::now() - t0).count();
}

// One launch in flight: the jobs of one task group (each at its own next sequence).
struct Launch {
  std::vector<uint32_t> ids;       // task ids, one job each (tables in PoaTask::rows)
  std::vector<PoaJob> jobs;
  size_t n_aln = 0;
  PoaArena* arena = nullptr;
  int wpj = 0;
  int gid = 0;
  int code_bytes = 2;    // traceback code width of the launch (4: a node with > 31 in-edges)
  size_t prep_jobs = 0;  // jobs whose tables the device completed (poa_prep.hip)
  int32_t gaps[4] = {0, 0, 0, 0};  // g, e, q, c of the launch (SVS_POA_VERIFY_PREP)
};

// Optional timeline (SVS_POA_TRACE=<file>): one line per host phase and per
// kernel, times in ms from the scheduler's start (kernel times placed on the
// GPU clock through an event recorded on the kernel stream at start).
struct PoaTrace {
  FILE* f = nullptr;
  Clock::time_point t0;
  hipEvent_t e0 = nullptr;
  void open(hipStream_t s) {
    const char* path = std::getenv("SVS_POA_TRACE");
    if (!path) return;
    f = std::fopen(path, "a");
    if (!f) return;
    SVS_HIP(hipEventCreate(&e0));
    SVS_HIP(hipEventRecord(e0, s));
    t0 = Clock::now();
    std::fprintf(f, "# begin\n");
  }
  double at(Clock::time_point t) const { return std::chrono::duration<double, std::milli>(t - t0).count(); }
  void host(const char* what, int g, Clock::time_point a, size_t n) {
    if (f) std::fprintf(f, "host %s %d %.3f %.3f %zu\n", what, g, at(a), at(Clock::now()), n);
  }
  // DP launches also log their kernel instance (prune, wide code flags)
  // and the cells the kernel evaluated (tools/profile_bench_*.sh: per-row
  // counter figures of one instance)
  void kernel(int g, hipEvent_t k0, hipEvent_t k1, size_t n, int wpj, uint64_t cells, int prune = 0, int wide = 0,
              uint64_t computed = 0) {
    if (!f) return;
    float a = 0.f, b = 0.f;
    SVS_HIP(hipEventElapsedTime(&a, e0, k0));
    SVS_HIP(hipEventElapsedTime(&b, e0, k1));
    std::fprintf(f, "kern %d %.3f %.3f %zu %d %llu %d %d %llu\n", g, a, b, n, wpj,
                 static_cast<unsigned long long>(cells), prune, wide, static_cast<unsigned long long>(computed));
  }
  void close() {
    if (!f) return;
    std::fclose(f);
    f = nullptr;
    (void)hipEventDestroy(e0);
  }
};
PoaTrace g_trace;

// Device time during which at least one timed DP launch was running: the
// union of the launches' [ev0, ev1] intervals on the GPU clock, placed through
// an epoch event recorded when the scheduler starts.  With a DP stream per
// task group two launches overlap (one group's first workgroups fill the
// other's tail), so the sum of launch durations (kernel_ms) counts the shared
// time twice; bench.py reports both.
struct DpBusyClock {
  hipEvent_t epoch = nullptr;
  std::map<double, double> iv;  // disjoint merged intervals, start -> end (ms from epoch)
  void start(hipStream_t s) {
    SVS_HIP(hipEventCreate(&epoch));
    SVS_HIP(hipEventRecord(epoch, s));
  }
  void add(hipEvent_t k0, hipEvent_t k1, svs_poa_stats& st) {
    if (!epoch) return;
    float a = 0.f, b = 0.f;
    SVS_HIP(hipEventElapsedTime(&a, epoch, k0));
    SVS_HIP(hipEventElapsedTime(&b, epoch, k1));
    st.kernel_busy_ms += busy_union_add(iv, a, b);
  }
  ~DpBusyClock() {
    if (epoch) (void)hipEventDestroy(epoch);
  }
};

// SVS_POA_STRIP_GLOBAL_POOL=1 keeps the strip kernel's pool in global memory
// even when it fits LDS (tests the path large graphs take).
bool strip_pool_forced_global() {
  const char* e = std::getenv("SVS_POA_STRIP_GLOBAL_POOL");
  return e && std::string(e) == "1";
}

// Exact pruning bound of a strip job (poa_strip.hip): lb = the score per read
// base of the task's last alignment that needed no retry x this read's length,
// less a slack of SVS_POA_PRUNE_SLACK (default 0.025) x m x length.  Any value is exact: a
// bound above the optimum only costs a retry.  The first retry of a read runs
// with the looser slack SVS_POA_PRUNE_RETRY_SLACK (default 0.1; "none": no
// bound), a second one with no bound; each retry of a task multiplies its
// slack by SVS_POA_PRUNE_ADAPT (default 1.5, up to the retry slack).  Values
// from the sweep in profiles/r02_v16, r02_v17.  Off for the first alignment of a task,
// after SVS_POA_PRUNE_MAX_RETRIES (default 16) retries of one task, for graphs
// too long for the 16-bit path lengths of the row records, and for score
// parameters the kernel's upper bound does not cover (SVS_POA_PRUNE=0: off).
struct PruneEnv {
  bool on = true;
  double slack = 0.025;
  bool retry_pruned = true;
  double retry_slack = 0.1;
  int max_retries = 16;
  double adapt = 1.5;  // a task's slack grows by this factor after each retry (SVS_POA_PRUNE_ADAPT)
  PruneEnv() {  // read once per launch, not once per job
    const char* pe = std::getenv("SVS_POA_PRUNE");
    on = !(pe && std::string(pe) == "0");
    const char* se = std::getenv("SVS_POA_PRUNE_SLACK");
    if (se) slack = std::atof(se);
    const char* re = std::getenv("SVS_POA_PRUNE_RETRY_SLACK");
    if (re && std::string(re) == "none") retry_pruned = false;
    else if (re) retry_slack = std::atof(re);
    const char* me = std::getenv("SVS_POA_PRUNE_MAX_RETRIES");
    if (me) max_retries = std::atoi(me);
    const char* ae = std::getenv("SVS_POA_PRUNE_ADAPT");
    if (ae) adapt = std::atof(ae);
  }
};

// The DP kernel's carry handoff publishes whole 128-B carry lines and relies
// on every job's carry region starting 256-B aligned (poa_strip.hip, before
// wait_vm_stores): the region offsets are built as multiples of
// kCarryAlignInts and the buffer base comes from hipMalloc; both are checked
// here rather than assumed.
uint64_t check_carry_aligned(uint64_t off_ints) {
  if (off_ints % kCarryAlignInts)
    throw SvsError(SVS_E_INTERNAL, "DP carry region at int offset " + std::to_string(off_ints) + " is not 256-B aligned");
  return off_ints;
}
void check_carry_base(const int32_t* p) {
  if (reinterpret_cast<uintptr_t>(p) % (kCarryAlignInts * sizeof(int32_t)))
    throw SvsError(SVS_E_INTERNAL, "DP carry buffer base is not 256-B aligned");
}

int32_t prune_bound(const PoaTask& t, const PoaScore& P, uint32_t n_rows, uint32_t len, const PruneEnv& pv) {
  const bool on = pv.on;
  const int32_t cg = std::max(std::max(P.g, P.e), std::max(P.q, P.c));
  if (!on || !t.have_rate || t.n_retries >= pv.max_retries || n_rows > 0xFFFFu || len > (1u << 20)) return kNoPrune;
  if (t.read_retries >= (pv.retry_pruned ? 2 : 1)) return kNoPrune;
  double slack = pv.retry_slack;
  if (t.read_retries == 0) {
    slack = pv.slack;
    for (int k = 0; k < t.n_retries && slack < pv.retry_slack; ++k) slack *= pv.adapt;
    slack = std::min(slack, std::max(pv.slack, pv.retry_slack));
  }
  if (cg > 0 || P.m < P.n || P.m < 0) return kNoPrune;
  const double lb = std::floor(t.rate * len - slack * P.m * len);
  // real bounds stay far above kPruneAll, so that the strip kernel's lanes
  // past column L (ub term VNEG/2) can never reach one (poa_strip.hip)
  if (lb < -1e8 || lb > 1e9) return kNoPrune;
  return static_cast<int32_t>(lb);
}

// LDS words a final fold job may take (64 KiB): above it, or for graphs whose
// scores do not fit, the consensus scores in global memory (poa_fold.hip).
#ifndef SVS_FINAL_LDS_CAP
#define SVS_FINAL_LDS_CAP 16384
#endif

// Kernel selection flags read from the environment once per call site
// (not once per job: getenv scans the whole environment).
struct KernelEnv {
  bool global_pool = strip_pool_forced_global();
};

// Host graphs: strip tables go straight into the group's pinned staging
// buffer (PoaArena::st_*); a table that does not fit stays in the task's
// vectors and is copied in when the launch is packed.  The device completes
// the tables (poa_prep.hip) of graphs it can hold; SVS_POA_VERIFY_PREP=1
// checks them against the host's export after every launch (tests).
bool verify_prep() {
  const char* e = std::getenv("SVS_POA_VERIFY_PREP");
  return e && std::string(e) == "1";
}

// a read in its block: zero pad byte, the read, zeros up to ls + 64 bytes
void write_read(char* p, const std::string& s, uint32_t ls) {
  p[-1] = 0;
  std::memcpy(p, s.data(), s.size());
  std::memset(p + s.size(), 0, ls + 63 - s.size());
}

// Exports the strip tables of t's next step into a fresh block of A's staging
// buffer; false (nothing written) when the buffer is full.
bool export_direct(PoaTask& t, const int32_t* gaps, PoaArena& A) {
  const std::string& s = t.seqs[t.next];
  const uint32_t ls = strip_ls(static_cast<uint32_t>(s.size()));
  const uint32_t V = t.graph.num_nodes(), E = t.graph.num_edges();
  if (V <= kStripPrepMaxRows && gaps[1] <= 0 && gaps[3] <= 0) {
    // host pass 1 only; the device derives the rest (poa_prep.hip)
    const StripBlock b = strip_block_lite(V, E, ls);
    const size_t off = A.st_cur.fetch_add(b.bytes, std::memory_order_relaxed);
    if (off + b.bytes > A.h_in.cap) return false;
    char* base = A.h_in.as<char>() + off;
    const StripLiteDst dst{reinterpret_cast<uint32_t*>(base + b.pstart), reinterpret_cast<uint32_t*>(base + b.pred_row),
                           reinterpret_cast<uint32_t*>(base + b.info)};
    t.graph.export_strip_lite(&t.rows, &dst);
    if (t.rows.n_slots <= kStripPrepMaxSlots && t.rows.max_preds <= kMaxInEdges) {
      write_read(base + b.seq, s, ls);
      t.rows_at = 2;
      t.blk_off = off;
      t.blk_gen = A.st_gen;
      return true;
    }
    // more pool slots or in-edges than the device planner takes: the full
    // tables, in a block of their own
  }
  const StripBlock b = strip_block_layout(V, E, ls);
  const size_t off = A.st_cur.fetch_add(b.bytes, std::memory_order_relaxed);
  if (off + b.bytes > A.h_in.cap) return false;
  char* base = A.h_in.as<char>() + off;
  const StripDst dst{reinterpret_cast<uint32_t*>(base + b.rec), reinterpret_cast<uint32_t*>(base + b.pstart),
                     reinterpret_cast<uint32_t*>(base + b.pred_row), reinterpret_cast<uint32_t*>(base + b.pred_slot),
                     reinterpret_cast<int32_t*>(base + b.col0)};
  t.graph.export_strip_rows(&t.rows, gaps, &dst);
  write_read(base + b.seq, s, ls);
  t.rows_at = 2;
  t.blk_off = off;
  t.blk_gen = A.st_gen;
  return true;
}

// SVS_POA_FORCE_WIDE=1 (tests): every DP launch with 32-bit traceback codes
// (read per launch: tests set it between calls)
bool force_wide() {
  const char* e = std::getenv("SVS_POA_FORCE_WIDE");
  return e && std::atoi(e) != 0;
}

// code_bytes: the launch's traceback code width (4 when some job of it has a
// node with more than 31 in-edges)
uint64_t job_bytes(const RowTables& tt, uint64_t L, const KernelEnv& ke, uint64_t code_bytes) {
  const uint64_t ls = strip_ls(static_cast<uint32_t>(L)), V = tt.n_rows;
  // traceback codes + two strip-boundary carry buffers (+ a global pool when
  // the graph needs more slots than the LDS pool holds)
  const uint64_t pool = (tt.n_slots > kStripMaxLdsSlots || ke.global_pool)
                            ? 8ull * round_up(static_cast<uint64_t>(tt.n_slots) * 97, 64) * 4 : 0;
  return V * ls * code_bytes + round_up(V, 8) * (ls / 64) * 16 + pool + 256 + (V + L + 1) * 8;
}

void verify_prep_tables(const Launch& la, std::deque<PoaTask>& tasks);

// Waves per job of a strip launch: enough strip-pipeline waves to fill the
// CUs, only for reads wide enough to give every wave several strips, and only
// as many as the per-wave LDS pools of one workgroup fit; SVS_POA_WPJ overrides.
int choose_wpj(size_t nj, uint32_t max_slots, uint32_t min_strips, bool lds_pool) {
  int wpj = 1;
  const char* we = std::getenv("SVS_POA_WPJ");
  const int wenv = we ? std::atoi(we) : 0;
  if ((wenv == 1 || wenv == 2 || wenv == 4 || wenv == 8) || (wenv == 16 && lds_pool)) {
    wpj = wenv;
  } else {
    // ~6 waves per SIMD (1024 SIMDs); each wave keeps >= 6 strips.  Measured
    // faster than keeping every workgroup resident (r01_v16): more waves per
    // job shorten each job even when some workgroups start late.
    while (wpj < 8 && static_cast<size_t>(wpj) * nj < 6144 && min_strips >= static_cast<uint32_t>(6 * wpj)) wpj *= 2;
    // the small launches at the end of a batch: 16 waves per job (>= 2 strips
    // each), or the few remaining jobs leave most SIMDs idle
    if (lds_pool && wpj == 8 && nj < 512 && min_strips >= 32u) wpj = 16;
  }
  while (lds_pool && wpj > 1 && static_cast<uint64_t>(wpj) * max_slots * kStripSlotBytes > kStripLdsBytes) wpj /= 2;
  return wpj;
}

void pack_and_launch_strip(svs_context* ctx, Launch& la, std::deque<PoaTask>& tasks, const PoaScore& score,
                           svs_poa_stats& st, double& host_ms) {
  auto th0 = Clock::now();
  const size_t nj = la.ids.size();
  la.jobs.assign(nj, PoaJob{});
  uint64_t n_tb = 0, n_bnd = 0, n_pool = 0, n_aln = 0;
  uint32_t max_preds = 0, max_slots = 1;
  bool any_prune = false;
  PoaArena& A = *la.arena;
  const int32_t gaps[4] = {score.g, score.e, score.q, score.c};
  // tables in an earlier generation of the staging buffer (a retried job, or
  // the over-budget sub-launch path) are exported again
  ctx->pool->parallel_for(nj, [&](size_t k) {
    PoaTask& t = tasks[la.ids[k]];
    if (t.rows_at != 2 || t.blk_gen == A.st_gen) return;
    if (!export_direct(t, gaps, A)) {
      t.graph.export_strip_rows(&t.rows, gaps);
      t.rows_at = 1;
    }
  });
  for (size_t k = 0; k < nj; ++k) max_slots = std::max(max_slots, tasks[la.ids[k]].rows.n_slots);
  const bool lds_pool = max_slots <= kStripMaxLdsSlots && !strip_pool_forced_global();
  auto job_ls = [&](size_t len) -> uint32_t { return strip_ls(static_cast<uint32_t>(len)); };
  uint32_t min_strips = 0xFFFFFFFFu;
  for (size_t k = 0; k < nj; ++k) {
    const uint32_t ls = job_ls(tasks[la.ids[k]].seqs[tasks[la.ids[k]].next].size());
    min_strips = std::min(min_strips, ls / 64);
  }
  const int wpj = choose_wpj(nj, max_slots, min_strips, lds_pool);
  if (std::getenv("SVS_POA_DEBUG"))
    std::fprintf(stderr, "[svs] strip launch: %zu jobs, wpj %d, slots %u\n", nj, wpj, max_slots);
  const PruneEnv penv;
  for (size_t k = 0; k < nj; ++k) {
    const auto& tt = tasks[la.ids[k]].rows;
    const std::string& s = tasks[la.ids[k]].seqs[tasks[la.ids[k]].next];
    PoaJob& J = la.jobs[k];
    J.n_rows = tt.n_rows;
    J.len = static_cast<uint32_t>(s.size());
    J.ls = job_ls(J.len);
    J.n_slots = tt.n_slots;
    if (static_cast<uint64_t>(J.n_rows) * J.ls > 0x7FFFFFFFull)  // the strip kernel's 32-bit code offsets
      throw SvsError(SVS_E_UNSUPPORTED, "a job's traceback matrix exceeds 2^31 cells");
    J.tb_off = n_tb;
    J.bnd_off = check_carry_aligned(n_bnd);
    J.pool_off = n_pool;
    J.aln_off = n_aln;
    J.lb = prune_bound(tasks[la.ids[k]], score, J.n_rows, J.len, penv);
    // the kernel tracks slot liveness in 31 bits; path lengths are 16-bit
    if (J.n_slots > 31 || J.len > kPruneMaxReadLen) J.lb = kNoPrune;
    any_prune = any_prune || J.lb != kNoPrune;
    n_tb += static_cast<uint64_t>(J.n_rows) * J.ls;
    n_bnd += round_up(round_up(J.n_rows, kCarryLineRows) * (J.ls / 64) * 4, kCarryAlignInts);
    if (!lds_pool) n_pool += static_cast<uint64_t>(wpj) * round_up(static_cast<uint64_t>(J.n_slots) * 97, 64);
    n_aln += static_cast<uint64_t>(J.n_rows) + J.len + 1;
    max_preds = std::max(max_preds, tt.max_preds);
    st.dp_cells += static_cast<uint64_t>(J.n_rows + 1) * (J.len + 1);
  }
  if (max_preds > kMaxInEdges)
    throw SvsError(SVS_E_UNSUPPORTED, "a graph node has more than 4094 in-edges (traceback code limit)");
  const bool wide = max_preds > kMaxInEdgesNarrow || force_wide();
  la.code_bytes = wide ? 4 : 2;
  st.wide_launches += wide ? 1 : 0;
  // the pruning variant prunes every job of its launch: the others get no bound
  if (any_prune)
    for (PoaJob& J : la.jobs)
      if (J.lb == kNoPrune) J.lb = kPruneAll;
  la.n_aln = n_aln;
  // every job's tables as one StripBlock in the staging buffer: blocks the
  // fold exported in place, then blocks for tables held in vectors (copied),
  // then the job descriptors
  size_t start = std::min(A.st_cur.load(std::memory_order_relaxed), A.h_in.cap);
  start = round_up(start, 48);
  std::vector<StripBlock> lay(nj);
  std::vector<size_t> boff(nj);
  size_t end = start;
  for (size_t k = 0; k < nj; ++k) {
    const PoaTask& t = tasks[la.ids[k]];
    const uint32_t lsw = strip_ls(la.jobs[k].len);
    lay[k] = (t.rows_at == 2 && t.rows.lite) ? strip_block_lite(t.rows.n_rows, t.rows.n_edges, lsw)
                                              : strip_block_layout(t.rows.n_rows, t.rows.n_edges, lsw);
    if (t.rows_at == 2) {
      boff[k] = t.blk_off;
    } else {
      boff[k] = end;
      end += lay[k].bytes;
    }
  }
  const size_t s_jobs = round_up(end, 256), off = s_jobs + nj * sizeof(PoaJob);
  if (off > A.h_in.cap) A.h_in.grow_keep(off, start);
  A.st_peak = std::max(A.st_peak, off);
  char* hs = A.h_in.as<char>();
  // the device-derived tables of lite jobs: a region after the staging copy
  // in the same device buffer, never copied from the host.  Byte offsets of
  // every table from the buffer's start; pointers once the buffer is sized.
  struct TabOff {
    size_t rec, pstart, pred, pslot, col0, seq, info;
  };
  std::vector<TabOff> to(nj);
  size_t dev_end = round_up(off, 48);
  uint32_t prep_rows = 0;
  size_t n_prep = 0;
  for (size_t k = 0; k < nj; ++k) {
    PoaJob& J = la.jobs[k];
    const PoaTask& t = tasks[la.ids[k]];
    const size_t b = boff[k];
    to[k].pstart = b + lay[k].pstart;
    to[k].pred = b + lay[k].pred_row;
    to[k].seq = b + lay[k].seq;
    if (t.rows_at == 2 && t.rows.lite) {
      const StripBlock o = strip_prep_out_layout(t.rows.n_rows, t.rows.n_edges);
      to[k].info = b + lay[k].info;
      to[k].col0 = dev_end + o.col0;
      to[k].rec = dev_end + o.rec;
      to[k].pslot = dev_end + o.pred_slot;
      J.prep = 1u | (t.rows.slot_base << 1);
      dev_end += o.bytes;
      prep_rows = std::max(prep_rows, t.rows.n_rows);
      ++n_prep;
    } else {
      to[k].info = 0;
      to[k].col0 = b + lay[k].col0;
      to[k].rec = b + lay[k].rec;
      to[k].pslot = b + lay[k].pred_slot;
      J.prep = 0;
    }
  }
  la.prep_jobs = n_prep;
  for (int x = 0; x < 4; ++x) la.gaps[x] = gaps[x];
  ctx->pool->parallel_for(nj, [&](size_t k) {
    const PoaTask& t = tasks[la.ids[k]];
    if (t.rows_at == 2) return;
    const auto& tt = t.rows;
    const PoaJob& J = la.jobs[k];
    char* base = hs + boff[k];
    std::memcpy(base + lay[k].rec, tt.rec.data(), 4ull * kRecWords * J.n_rows);
    std::memcpy(base + lay[k].pstart, tt.pstart.data(), 4ull * (J.n_rows + 1));
    std::memcpy(base + lay[k].col0, tt.col0.data(), 12ull * J.n_rows);
    if (!tt.pred_row.empty()) {
      std::memcpy(base + lay[k].pred_row, tt.pred_row.data(), 4 * tt.pred_row.size());
      std::memcpy(base + lay[k].pred_slot, tt.pred_slot.data(), 4 * tt.pred_slot.size());
    }
    write_read(base + lay[k].seq, t.seqs[t.next], strip_ls(J.len));
  });
  host_ms += ms_since(th0);

  A.d_in.ensure(dev_end);
  // the traceback codes dominate a launch's footprint: sized to the group's
  // budget at the first launch, so it never regrows (and syncs) mid-run
  A.d_tb.ensure(n_tb * la.code_bytes + 4096, ctx->device_budget / 2);
  A.d_pool.ensure((n_bnd + n_pool) * 4 + 4096);
  A.d_aln.ensure(n_aln * 8);
  A.d_alen.ensure(nj * 12);
  A.h_aln.ensure(n_aln * 8);
  A.h_alen.ensure(nj * 12);
  char* dg = A.d_in.as<char>();
  for (size_t k = 0; k < nj; ++k) {
    PoaJob& J = la.jobs[k];
    J.rec = reinterpret_cast<const uint32_t*>(dg + to[k].rec);
    J.pstart = reinterpret_cast<const uint32_t*>(dg + to[k].pstart);
    J.pred = reinterpret_cast<const uint32_t*>(dg + to[k].pred);
    J.pslot = reinterpret_cast<const uint32_t*>(dg + to[k].pslot);
    J.col0 = reinterpret_cast<const int32_t*>(dg + to[k].col0);
    J.seq = reinterpret_cast<const uint8_t*>(dg + to[k].seq);
    J.info = reinterpret_cast<const uint32_t*>(dg + to[k].info);
  }
  std::memcpy(hs + s_jobs, la.jobs.data(), nj * sizeof(PoaJob));
  SVS_HIP(hipMemcpyAsync(dg, hs, off, hipMemcpyHostToDevice, A.copy_stream));
  SVS_HIP(hipEventRecord(A.h2d, A.copy_stream));
  SVS_HIP(hipStreamWaitEvent(A.stream, A.h2d, 0));
  if (n_prep > 0) {
    // on the kernel stream (a stream of its own measured no faster, r02_v28)
    hipStream_t ps = A.stream;
    SVS_HIP(hipEventRecord(A.evp, ps));
    SVS_HIP(launch_poa_strip_prep(reinterpret_cast<const PoaJob*>(dg + s_jobs), static_cast<int>(nj), score,
                                  prep_rows, ps));
    SVS_HIP(hipEventRecord(A.evp1, ps));
    if (verify_prep()) {
      // before the DP kernel reads them: a wrong table fails here, not there
      SVS_HIP(hipStreamSynchronize(ps));
      verify_prep_tables(la, tasks);
    }
  }
  PoaLaunch pl{};
  pl.jobs = reinterpret_cast<const PoaJob*>(dg + s_jobs);
  pl.n_jobs = static_cast<int>(nj);
  pl.score = score;
  pl.tb = A.d_tb.as<char>();
  pl.bnd = A.d_pool.as<int32_t>();
  pl.pool = A.d_pool.as<int32_t>() + n_bnd;
  pl.aln = A.d_aln.as<int32_t>();
  pl.aln_len = A.d_alen.as<int32_t>();
  pl.lds_slots = lds_pool ? max_slots : 0;
  pl.prune = any_prune;
  pl.wide = la.code_bytes == 4;
  pl.waves_per_job = wpj;
  check_carry_base(pl.bnd);
  la.wpj = wpj;
  SVS_HIP(hipEventRecord(A.ev0, A.stream));
  SVS_HIP(launch_poa_strip(pl, A.stream));
  SVS_HIP(hipEventRecord(A.ev1, A.stream));
  SVS_HIP(hipStreamWaitEvent(A.copy_stream, A.ev1, 0));
  SVS_HIP(hipMemcpyAsync(A.h_alen.ptr, pl.aln_len, nj * 12, hipMemcpyDeviceToHost, A.copy_stream));
  SVS_HIP(hipMemcpyAsync(A.h_aln.ptr, pl.aln, n_aln * 8, hipMemcpyDeviceToHost, A.copy_stream));
  SVS_HIP(hipEventRecord(A.done, A.copy_stream));
  st.launches += 1;
  st.alignments += nj;
  st.tb_bytes += n_tb * 2;
  st.pool_bytes += (n_bnd + n_pool) * 4;
  st.h2d_bytes += off;
  st.d2h_bytes += n_aln * 8 + nj * 12;
}

// Readies a task's next step: sequences landing on an empty graph become a
// fresh chain (no DP), empty ones are skipped; then either the row tables of
// the next alignment are exported (returns 1) or, with every sequence in, the
// consensus and MSA are computed (returns 2).
uint8_t prep_task(PoaTask& t, const svs_poa_config& cfg, PoaArena* stage) {
  while (t.next < t.seqs.size()) {
    const std::string& s = t.seqs[t.next];
    if (s.empty()) { ++t.next; continue; }
    if (t.graph.empty()) { t.graph.add_alignment_nodes({}, s); ++t.next; continue; }
    break;
  }
  if (t.next < t.seqs.size()) {
    const int32_t gaps[4] = {cfg.g, cfg.e, cfg.q, cfg.c};
    if (!stage || !export_direct(t, gaps, *stage)) {
      t.graph.export_strip_rows(&t.rows, gaps);
      t.rows_at = 1;
    }
    return 1;
  }
  t.consensus = t.graph.consensus(cfg.min_coverage);
  if (t.genmsa) t.msa = t.graph.msa();
  return 2;
}

// SVS_POA_VERIFY_PREP=1: the device-completed tables of a finished launch
// against the host's full export of the same graphs (still unfolded).
void verify_prep_tables(const Launch& la, std::deque<PoaTask>& tasks) {
  for (size_t k = 0; k < la.ids.size(); ++k) {
    const PoaJob& J = la.jobs[k];
    if (!(J.prep & 1u)) continue;
    PoaTask& t = tasks[la.ids[k]];
    RowTables h;
    t.graph.export_strip_rows(&h, la.gaps);
    const uint32_t V = J.n_rows, E = static_cast<uint32_t>(h.pred_row.size());
    std::vector<uint32_t> rec(4ull * V), ps(E);
    std::vector<int32_t> c0(3ull * V);
    SVS_HIP(hipMemcpy(rec.data(), J.rec, rec.size() * 4, hipMemcpyDeviceToHost));
    if (E) SVS_HIP(hipMemcpy(ps.data(), J.pslot, ps.size() * 4, hipMemcpyDeviceToHost));
    SVS_HIP(hipMemcpy(c0.data(), J.col0, c0.size() * 4, hipMemcpyDeviceToHost));
    if (rec != h.rec || ps != h.pred_slot || c0 != h.col0 || h.n_slots != t.rows.n_slots)
      throw SvsError(SVS_E_INTERNAL, "device strip tables differ from the host export (job " + std::to_string(k) + ")");
  }
}

// Waits for the launch and folds its alignments back into the graphs, each
// task's next step readied right after its fold while its graph is in cache
// (prep_task; PoaTask::prepped).  While
// the launch is still running, `idle` (if given) is called for host work that
// is off the critical path until it returns false.
void finish(svs_context* ctx, Launch& la, std::deque<PoaTask>& tasks, svs_poa_stats& st, double& host_ms,
            const svs_poa_config& cfg, const std::function<bool()>& idle = nullptr, DpBusyClock* busy = nullptr) {
  PoaArena& A = *la.arena;
  const auto tw0 = Clock::now();
  if (idle) {
    for (;;) {
      const hipError_t q = hipEventQuery(A.done);
      if (q == hipSuccess) break;
      if (q != hipErrorNotReady) SVS_HIP(q);
      if (!idle()) break;
    }
  }
  SVS_HIP(hipEventSynchronize(A.done));  // the other group's launch may still be queued behind it
  st.gpu_wait_ms += ms_since(tw0);
  // the launch's staging copy is consumed: a new generation for the next one
  A.st_gen += 1;
  A.st_cur.store(0, std::memory_order_relaxed);
  A.h_in.ensure(A.st_peak + A.st_peak / 4);
  PoaArena* stage = &A;
  float ms = 0.f;
  SVS_HIP(hipEventElapsedTime(&ms, A.ev0, A.ev1));
  st.kernel_ms += ms;
  if (busy) busy->add(A.ev0, A.ev1, st);
  if (la.prep_jobs > 0) {
    float pms = 0.f;
    SVS_HIP(hipEventElapsedTime(&pms, A.evp, A.evp1));
    st.prep_ms += pms;
    st.prep_jobs += la.prep_jobs;
  }
  if (g_trace.f) {
    uint64_t cells = 0;
    for (const PoaJob& J : la.jobs) cells += static_cast<uint64_t>(J.n_rows + 1) * (J.len + 1);
    g_trace.host("wait", la.gid, tw0, la.ids.size());
    g_trace.kernel(la.gid, A.ev0, A.ev1, la.ids.size(), la.wpj, cells);
  }
  auto th0 = Clock::now();
  const int32_t* alen = A.h_alen.as<int32_t>();
  const int32_t* aout = A.h_aln.as<int32_t>();
  const size_t nj = la.ids.size();
  {
    for (size_t k = 0; k < nj; ++k) {
      st.cells_computed += 64ull * static_cast<uint32_t>(alen[2 * nj + k]);
      tasks[la.ids[k]].last_rows = static_cast<uint32_t>(alen[2 * nj + k]);
      if (alen[k] == kPruneRetry) st.prune_retries += 1;
    }
  }
  ctx->pool->parallel_for(nj, [&](size_t k) {
    const int32_t n = alen[k];
    auto& t = tasks[la.ids[k]];
    if (n == kPruneRetry) {
      // the bound was above the optimum: the same sequence again, unpruned
      // (its row tables are still those of this step)
      t.retry = true;
      t.n_retries += 1;
      t.read_retries += 1;
      t.prepped = 1;
      return;
    }
    if (n < 0) throw SvsError(SVS_E_INTERNAL, "GPU traceback reported an inconsistent path");
    {
      const uint32_t len = la.jobs[k].len;
      if (!t.retry && len > 0) {
        t.rate = static_cast<double>(alen[nj + k]) / len;
        t.have_rate = true;
      }
      t.retry = false;
      t.read_retries = 0;
    }
    const int32_t* p = aout + 2 * la.jobs[k].aln_off;
    std::vector<int32_t> fwd(2 * static_cast<size_t>(n));
    for (int32_t x = 0; x < n; ++x) {
      fwd[2 * x] = p[2 * (n - 1 - x)];
      fwd[2 * x + 1] = p[2 * (n - 1 - x) + 1];
    }
    t.graph.add_alignment_ranks(fwd, t.seqs[t.next]);
    ++t.next;
    t.prepped = prep_task(t, cfg, stage);
  });
  host_ms += ms_since(th0);
  g_trace.host("fold", la.gid, th0, la.ids.size());
}

// One launch of the device-resident graphs (poa_dgraph.hpp): DP jobs, then
// the fold jobs (the DP jobs' alignments first, in the same order, then the
// tasks whose first read lands on an empty graph).
struct DevLaunch {
  // fold jobs: first the new tasks' first reads (chains, folded before the DP
  // kernel: their second read is aligned in the same launch), then the DP
  // jobs' alignments in DP-job order
  std::vector<uint32_t> dp_ids, fold_ids, fold_seq;
  size_t n_pre = 0;
  std::vector<PoaJob> jobs;
  std::vector<FoldJob> folds;
  std::vector<uint8_t> moved;                    // fold i's graph moved to a larger block
  std::vector<std::pair<void*, size_t>> old_blocks;  // freed once the launch is done
  std::vector<size_t> cons_off, msa_off;         // fold i's final outputs in the fin buffer
  std::vector<size_t> feat_off;                  // fold i's seqdatamx in the group's h_feat (kFoldFeat)
  size_t n_aln = 0, s_fold = 0, s_res = 0, fin_bytes = 0;
  size_t s_fidx = 0, n_fin = 0;  // the post-DP final folds' indices (from the first post-DP fold)
  size_t fin_copy = 0;  // bytes of the fin buffer copied back (consensus first; MSA rows when wanted)
  int wpj = 0;
  bool timed_dp = false;
  bool prune = false, wide = false;  // the DP kernel instance
  bool split_final = false;          // the final kernel ran on the arena's fin_stream
};

// Task group: a disjoint subset of the active tasks with its own arena.
struct Group {
  std::vector<uint32_t> active;
  Launch la;
  DevLaunch dl;
  std::vector<uint32_t> completed;  // device graphs finished by the last launch
  bool pending = false;
  PoaArena* arena = nullptr;
};

// Device-resident graphs unless SVS_POA_HOST_GRAPH=1 (or a consensus with a
// minimum coverage, which only the host graph implements).
bool device_graphs(const svs_poa_config& c) {
  const char* e = std::getenv("SVS_POA_HOST_GRAPH");
  return !(e && std::string(e) == "1") && c.min_coverage <= 0;
}
// SVS_POA_VERIFY_GRAPH=1: a host PoaGraph of every task replays the device's
// folds; the device's rank order, row tables, consensus and MSA are checked
// against it after every fold (tests).
bool verify_graph() {
  const char* e = std::getenv("SVS_POA_VERIFY_GRAPH");
  return e && std::string(e) == "1";
}
// SVS_POA_FOLD_TIMES: totals of the fold kernels' phase times (FoldResult
// t_*), printed at exit
struct FoldTimes {
  bool on = [] {
    const char* e = std::getenv("SVS_POA_FOLD_TIMES");
    return e && std::atoi(e) != 0;
  }();
  double upd = 0, sort = 0, exp = 0, fin = 0, max_sort = 0, max_fin = 0;
  uint64_t n = 0, n_exp = 0, n_fin = 0, verts = 0, exams = 0, roots = 0, prof[4] = {0, 0, 0, 0};
  void add(const FoldResult& r, uint32_t flags) {
    if (!on) return;
    ++n;
    verts += r.V;
    exams += r.n_exam;
    roots += r.n_roots;
    for (int k = 0; k < 4; ++k) prof[k] += r.prof[k];
    upd += r.t_upd * 1e-5;
    sort += r.t_sort * 1e-5;
    max_sort = std::max(max_sort, r.t_sort * 1e-5);
    if (flags & kFoldExport) {
      ++n_exp;
      exp += r.t_exp * 1e-5;
    }
    if (flags & kFoldFinal) {
      ++n_fin;
      fin += r.t_fin * 1e-5;
      max_fin = std::max(max_fin, r.t_fin * 1e-5);
    }
  }
  ~FoldTimes() {
    if (!on || !n) return;
    std::fprintf(stderr,
                 "[svs] fold times (ms per job): %llu folds, mean V %.0f; update %.3f, sort %.3f (max %.2f); "
                 "%llu exports %.3f; %llu finals %.3f (max %.2f); per fold %.0f DFS examinations, %.0f roots\n",
                 static_cast<unsigned long long>(n), double(verts) / n, upd / n, sort / n, max_sort,
                 static_cast<unsigned long long>(n_exp), n_exp ? exp / n_exp : 0.0,
                 static_cast<unsigned long long>(n_fin), n_fin ? fin / n_fin : 0.0, max_fin, double(exams) / n,
                 double(roots) / n);
#ifdef SVS_FOLD_PROF_UPD
    std::fprintf(stderr, "[svs] update phases per fold (kclk): middle %.0f, edges %.0f, in-list %.0f, out-list %.0f\n",
                 double(prof[0]) * 1.024 / n, double(prof[1]) * 1.024 / n, double(prof[2]) * 1.024 / n,
                 double(prof[3]) * 1.024 / n);
    return;
#endif
    if (prof[0] || prof[1])
      std::fprintf(stderr,
                   "[svs] DFS profile per fold: fast roots %.0f kclk, DFS runs %.0f kclk, %.1f new-node and %.1f "
                   "old-node window loads\n",
                   double(prof[0]) * 1.024 / n, double(prof[1]) * 1.024 / n, double(prof[2]) / n, double(prof[3]) / n);
  }
};
FoldTimes g_fold_times;

bool debug_launches() {
  static const bool on = std::getenv("SVS_POA_DEBUG") != nullptr;
  return on;
}
bool sync_check() {
  const char* e = std::getenv("SVS_POA_SYNC_CHECK");
  return e && std::string(e) == "1";
}
// The final fold kernel runs on a stream of its own, beside the table
// completion of the same launch (a finishing task needs no tables, a
// continuing one no consensus), so the fold chain the group's next DP launch
// waits for is update, sort, then the longer of the two: 427.3 / 429.9 vs
// 418.0 / 419.7 windows/s same box against running it in line
// (profiles/r05_g1; the in-line switch was removed in round 6).

size_t active_jobs_per_group() {
  if (const char* e = std::getenv("SVS_POA_ACTIVE_JOBS")) {
    const long v = std::atol(e);
    if (v > 0) return static_cast<size_t>(v);
  }
  // 2048 tasks per group: with choose_wpj's 4 waves per job a launch holds
  // 8192 waves, more than the 7168 resident at 7 per SIMD (the pruning
  // kernel's 72-VGPR cap), so jobs that end early make room for the rest.
  // Fewer waves per job shorten each job's strip pipeline: at 8 waves per job
  // a wave spends about 30 % of its life waiting for the wave sweeping the
  // strip before it (at 4, 6 %; SVS_STRIP_PROF, profiles/r04_sp1), but a
  // launch then needs more jobs to fill the CUs.  Driver-shape A/B with 10
  // batches in flight: 1536 tasks 296.8 / 297.1, 1792 tasks 301.4 / 310.2 /
  // 311.1 windows/s (profiles/r04_ab5, r04_ab6); after the round-4 DP kernel
  // changes and with the traceback budget at 5/8 of HBM (svs_abi.cpp), 1920
  // 345.1, 2048 352.5 / 350.9, 2176 348.7 (profiles/r04_h9); at half of HBM,
  // 2048 tasks overran the budget and launched in smaller pieces half the
  // time (331.7 / 343.3, r04_h6).
  return 2048;
}

// Two task groups, each with its own arena, DP stream and fold chain: while
// one group folds, the other's DP launch runs.  Three and four groups (the
// same 4096 tasks in flight shared out) made smaller launches, each with its
// own tail: 366.1 / 362.3 and 390.2 vs 447.1 / 440.1 windows/s same box
// (profiles/r05_gr1; the switch was removed in round 6).
constexpr int kMaxGroups = 2;

}  // namespace

struct PoaScheduler::Impl {
  svs_context* ctx;
  svs_poa_config cfg;
  PoaScore score;
  svs_poa_stats& st;
  std::deque<PoaTask> tasks;
  std::deque<uint32_t> queue;
  static constexpr int n_groups = kMaxGroups;
  Group groups[kMaxGroups];
  size_t cap;
  size_t budget;
  double host_ms = 0.0;
  std::vector<uint32_t> graves;  // finished tasks whose storage is not yet released
  std::vector<uint32_t> free_ids;  // released task slots, reused by add()
  bool queue_dirty = false;      // tasks were queued since the last sort

  bool dev;      // device-resident graphs (poa_dgraph.hpp)
  bool verify;   // SVS_POA_VERIFY_GRAPH
  // entries of the sort kernel's DFS stack held in LDS (deeper stacks spill
  // to the task block); SVS_POA_SORT_STACK (>= 64) lowers it in tests so the
  // spill path runs
  uint32_t sort_stack = 1024;
  DevArena* darena = nullptr;

  Impl(svs_context* c, const svs_poa_config& k, svs_poa_stats& s)
      : ctx(c), cfg(k), score{k.m, k.n, k.g, k.e, k.q, k.c}, st(s), cap(active_jobs_per_group()),
        budget(c->device_budget / n_groups), dev(device_graphs(k)), verify(verify_graph()) {
    if (const char* e = std::getenv("SVS_POA_SORT_STACK")) {
      const long v = std::atol(e);
      if (v >= 64 && v <= 1024) sort_stack = static_cast<uint32_t>(v) & ~1u;
    }
    if (const char* e = std::getenv("SVS_POA_TEST_SORT_LDS_WORDS")) {
      const long v = std::atol(e);
      if (v > 0 && static_cast<uint64_t>(v) < kSortLdsWordsMax) sort_lds_max = static_cast<uint64_t>(v);
    }
    if (const char* e = std::getenv("SVS_POA_TEST_MAX_BLOCK_BYTES")) {
      const long long v = std::atoll(e);
      if (v > 0) test_block_cap = static_cast<size_t>(v);
    }
    if (dev) {
      if (!ctx->dgraph_arena) {
        // SVS_POA_TEST_ARENA_BYTES (tests) lowers the limit of a context's
        // graph arena when its first scheduler creates it, so that tasks must
        // wait for blocks other tasks hold (reserve_blocks)
        size_t lim = ctx->dgraph_budget;
        if (const char* e = std::getenv("SVS_POA_TEST_ARENA_BYTES")) {
          const long long v = std::atoll(e);
          if (v > 0) lim = std::min(lim, static_cast<size_t>(v));
        }
        ctx->dgraph_arena.reset(new DevArena(lim));
      }
      darena = ctx->dgraph_arena.get();
    }
    // (both arenas start on the context's stream; the DP streams below)
    while (ctx->poa_arenas.size() < static_cast<size_t>(n_groups))
      ctx->poa_arenas.emplace_back(new PoaArena(ctx->device, ctx->stream));
    for (int g = 0; g < n_groups; ++g) groups[g].arena = ctx->poa_arenas[g].get();
    dp_busy.start(ctx->stream);
    // Each group's DP kernel on a stream of its own (round 5), so that one
    // group's launch starts in the tail of the other's: a launch ends with its
    // longest jobs and leaves CUs idle that the other group's first
    // workgroups now take.  Same-box driver-shape A/B 378.4 / 375.7 vs 362.3 /
    // 361.7 windows/s against both groups on one stream (profiles/r05_a6),
    // 382.1 vs 365.7 (r05_a8); the DP launches' mean event time grows by ~1 %
    // where they overlap.
    for (int g = 0; g < n_groups; ++g) {
      SVS_HIP(hipStreamCreateWithFlags(&own_dp[g], hipStreamNonBlocking));
      groups[g].arena->stream = own_dp[g];
    }
  }
  ~Impl() {
    for (int g = 0; g < n_groups; ++g)
      if (own_dp[g]) {
        (void)hipStreamSynchronize(own_dp[g]);
        groups[g].arena->stream = ctx->stream;
        (void)hipStreamDestroy(own_dp[g]);
      }
  }
  hipStream_t own_dp[kMaxGroups] = {nullptr, nullptr};
  DpBusyClock dp_busy;

  // Moves queued tasks into the group, up to `cap` active tasks; when the
  // other group also has room, at most half of the queue, so that both groups
  // start their share in the same step (staggered starts leave a tail of
  // small launches when the tasks end).
  void refill(Group& g) {
    if (queue.empty() || g.active.size() >= cap) return;
    // longest remaining task first, so the long tasks (germline-cluster
    // consensus) do not form a tail of small launches at the end
    if (queue_dirty) {
      // (within a session: older batches first, so batches complete in order)
      std::stable_sort(queue.begin(), queue.end(), [this](uint32_t a, uint32_t b) {
        if (tasks[a].prio != tasks[b].prio) return tasks[a].prio < tasks[b].prio;
        return tasks[a].seqs.size() - tasks[a].next > tasks[b].seqs.size() - tasks[b].next;
      });
      queue_dirty = false;
    }
    size_t others = 0;  // other groups with room: the queue is shared out among them
    for (int k = 0; k < n_groups; ++k) others += (k != gid(g) && groups[k].active.size() < cap) ? 1u : 0u;
    const size_t room = cap - g.active.size();
    const size_t share = others ? std::max<size_t>(1, (queue.size() + others) / (others + 1)) : queue.size();
    size_t take = std::min(room, share);
    while (take-- > 0 && !queue.empty()) {
      g.active.push_back(queue.front());
      queue.pop_front();
    }
  }

  // ------------------------------------------------ device-resident graphs
  // A task's reads (each as the DP kernel reads it: a zero pad byte, the read,
  // zeros up to ls + 64), the path offsets of its non-empty reads and room for
  // their node paths: one block, uploaded once (through the launch's pinned
  // staging), read by every DP and fold of the task.  layout_static lays the
  // block out (reserve_blocks allocates it); returns the bytes of its host
  // image (reads + path offsets; the paths are written by the folds).
  size_t layout_static(PoaTask& t) {
    const size_t n = t.seqs.size();
    t.seq_at.assign(n, 0);
    size_t o = 64;
    uint32_t n_ne = 0;
    uint64_t path_total = 0;
    t.last_nonempty = 0;
    for (size_t k = 0; k < n; ++k) {
      const uint32_t L = static_cast<uint32_t>(t.seqs[k].size());
      t.seq_at[k] = o;
      o = round_up(o + strip_ls(L) + 64, 64) + 64;
      if (L) {
        ++n_ne;
        path_total += L;
        t.last_nonempty = static_cast<uint32_t>(k) + 1;
      }
    }
    const size_t po = round_up(o, 64), pa = round_up(po + 4ull * (n_ne + 1), 64);
    t.static_bytes = pa + 4 * path_total + 64;
    t.static_po = po;
    return pa;
  }
  // The host image of layout_static's block (`bytes` of it) at h.
  static void write_static(const PoaTask& t, char* h, size_t bytes) {
    const size_t po = static_cast<size_t>(reinterpret_cast<const uint8_t*>(t.d_path_off) - t.d_static);
    std::memset(h, 0, bytes);
    for (size_t k = 0; k < t.seqs.size(); ++k)
      if (!t.seqs[k].empty()) std::memcpy(h + t.seq_at[k], t.seqs[k].data(), t.seqs[k].size());
    uint32_t* poff = reinterpret_cast<uint32_t*>(h + po);
    uint32_t acc = 0, i = 0;
    for (const std::string& q : t.seqs)
      if (!q.empty()) {
        poff[i++] = acc;
        acc += static_cast<uint32_t>(q.size());
      }
    poff[i] = acc;
  }

  // A task past an engine limit completes alone, with no consensus or MSA and
  // the reason in t.error (the decision layer fails its window only).
  void fail_task(Group& g, uint32_t id, std::string why) {
    PoaTask& t = tasks[id];
    t.error = std::move(why);
    t.consensus.clear();
    t.msa.clear();
    release_dev(t);
    g.completed.push_back(id);
  }
  // LDS words of the sort kernel for a graph of n nodes: the done and ignore
  // bit planes, then the DFS stack's LDS part (poa_fold_sort_kernel).  A
  // launch takes the maximum over its folds, so every fold must fit the
  // 160 KiB a workgroup may declare; a graph past it fails alone
  // (advance_dev) instead of failing the launch.
  // (SVS_POA_TEST_SORT_LDS_WORDS lowers the limit in tests)
  static constexpr uint64_t kSortLdsWordsMax = 160 * 1024 / 4 - 64;
  uint64_t sort_lds_max = kSortLdsWordsMax;
  // four bit planes (done, ignored, changed, segment starts) and the stack top
  uint64_t sort_lds_words(uint64_t n) const { return 4 * ((n + 31) / 32) + sort_stack; }
  // SVS_POA_TEST_MAX_BLOCK_BYTES (tests): reserve_blocks treats a block larger
  // than this as past the arena's limit, so that one window fails alone
  size_t test_block_cap = ~size_t(0);

  // the row limit of the device table planner (SVS_POA_TEST_MAX_ROWS lowers it
  // in tests, to fail one window of a batch on purpose)
  static uint32_t planner_max_rows() {
    const char* e = std::getenv("SVS_POA_TEST_MAX_ROWS");
    const long v = e ? std::atol(e) : 0;
    return v > 0 && static_cast<uint64_t>(v) < kStripPrepMaxRows ? static_cast<uint32_t>(v) : kStripPrepMaxRows;
  }

  void release_dev(PoaTask& t) {
    if (t.d_static) darena->free(t.d_static, t.static_bytes);
    if (t.dg.blk) darena->free(t.dg.blk, t.dg_bytes);
    if (t.grow_blk) darena->free(t.grow_blk, t.grow_bytes);
    t.d_static = nullptr;
    t.dg.blk = nullptr;
    t.grow_blk = nullptr;
    t.static_up = false;
  }

  // Device blocks this launch needs, reserved before it is packed: the reads
  // block of each task that starts, the graph block of each first-read chain
  // (sized for the chain and its next read's fold in the same launch), and a
  // larger graph block wherever this launch's fold could overflow the current
  // one.  A task whose block can never fit (larger than the arena's limit, or
  // the test cap) fails alone (fail_task).  A task whose block
  // does not fit only because other tasks hold the arena right now waits for
  // a later launch (whether a window fails must not depend on
  // timing): its chain state is undone (`undo`, saved by advance_dev before it
  // was changed) and it stays active.  Only when nothing could free a block
  // first (no other work in this launch, no launch of the other group in
  // flight) does one task, the one holding the most, give its blocks up and
  // fail; advance_dev then tries the rest again.
  struct ChainUndo {
    uint32_t id;
    DGraphRef dg;
    size_t next;
    uint32_t n_paths, n_slots_next, max_preds_next;
    bool tables_ok;
  };
  void reserve_blocks(Group& g, std::vector<uint32_t>& dp, std::vector<uint32_t>& chain,
                      std::vector<uint32_t>& chain_seq, const std::vector<ChainUndo>& undo) {
    // 1: can never fit, 2: does not fit now
    std::vector<uint8_t> bad(tasks.size(), 0);
    size_t n_bad = 0;
    uint8_t miss = 0;
    auto reserve = [&](size_t bytes) -> uint8_t* {
      if (bytes > test_block_cap || BlockArena::size_class(bytes) > darena->limit()) {
        miss = 1;
        return nullptr;
      }
      miss = 2;
      return static_cast<uint8_t*>(darena->try_alloc(bytes));
    };
    std::vector<uint8_t> is_chain(tasks.size(), 0);
    for (size_t i = 0; i < chain.size(); ++i) {
      const uint32_t id = chain[i];
      PoaTask& t = tasks[id];
      is_chain[id] = 1;
      if (!t.d_static) {
        const size_t pa = layout_static(t);
        t.d_static = reserve(t.static_bytes);
        if (!t.d_static) {
          bad[id] = miss;
          ++n_bad;
          continue;
        }
        t.d_path_off = reinterpret_cast<uint32_t*>(t.d_static + t.static_po);
        t.d_paths = reinterpret_cast<uint32_t*>(t.d_static + pa);
        t.static_up = true;
      }
      const uint32_t len = static_cast<uint32_t>(t.seqs[chain_seq[i]].size());
      const uint32_t nxt = t.next < t.seqs.size() ? static_cast<uint32_t>(t.seqs[t.next].size()) : 0u;
      const uint32_t cv1 = std::max(3 * len, len + 2 * nxt) + 4096;
      const uint32_t ce1 = std::max(4 * len, len + 3 * nxt) + 4096;
      t.dg_bytes = dgraph_layout(cv1, ce1).bytes;
      t.dg.blk = reserve(t.dg_bytes);
      t.dg.cv = cv1;
      t.dg.ce = ce1;
      if (!t.dg.blk) {
        bad[id] = miss;
        ++n_bad;
      }
    }
    for (uint32_t id : dp) {
      PoaTask& t = tasks[id];
      if (is_chain[id] || bad[id]) continue;
      const uint32_t len = static_cast<uint32_t>(t.seqs[t.next].size());
      if (t.dg.V + len > t.dg.cv || t.dg.E + len + 1 > t.dg.ce) {
        // a window MSA of 64 reads x 3 kb ends near 2.2 L nodes and 2.9 L
        // edges: the first block holds that, larger graphs double
        t.grow_cv = std::max<uint32_t>(2 * t.dg.cv, t.dg.V + 3 * len + 4096);
        t.grow_ce = std::max<uint32_t>(2 * t.dg.ce, t.dg.E + 4 * len + 4096);
        t.grow_bytes = dgraph_layout(t.grow_cv, t.grow_ce).bytes;
        t.grow_blk = reserve(t.grow_bytes);
        if (!t.grow_blk) {
          bad[id] = miss;
          ++n_bad;
        }
      }
    }
    if (!n_bad) return;
    auto drop = [&](std::vector<uint32_t>& v, std::vector<uint32_t>* w) {
      size_t o = 0;
      for (size_t i = 0; i < v.size(); ++i)
        if (!bad[v[i]]) {
          if (w) (*w)[o] = (*w)[i];
          v[o++] = v[i];
        }
      v.resize(o);
      if (w) w->resize(o);
    };
    // wait for a later launch where some block can be freed before it
    size_t n_good = 0;
    for (uint32_t id : dp) n_good += bad[id] ? 0u : 1u;
    for (uint32_t id : chain) n_good += bad[id] ? 0u : 1u;
    bool other_in_flight = false;
    for (int k = 0; k < n_groups; ++k) other_in_flight = other_in_flight || (k != gid(g) && groups[k].pending);
    const bool can_wait = n_good > 0 || other_in_flight;
    if (debug_launches())
      std::fprintf(stderr, "[svs] group %d: %zu blocks missing (%zu jobs placed), other group in flight %d, arena %zu of %zu B in use, %zu reserved\n",
                   gid(g), n_bad, n_good, int(other_in_flight), darena->in_use(), darena->limit(), darena->reserved());
    // nothing can free a block first (every task of both groups waits for
    // one): one task gives up its blocks, the one holding the most, and
    // fails; the caller then tries the others again
    uint32_t victim = ~0u;
    if (!can_wait) {
      size_t most = 0;
      for (uint32_t id : g.active)
        if (bad[id] == 2) {
          const PoaTask& t = tasks[id];
          const size_t held = (t.dg.blk ? t.dg_bytes : 0) + (t.d_static && !t.static_up ? t.static_bytes : 0);
          if (victim == ~0u || held > most) {
            victim = id;
            most = held;
          }
        }
    }
    std::vector<uint8_t> waits(tasks.size(), 0);
    for (const ChainUndo& u : undo)
      if (bad[u.id] == 2 && u.id != victim) {
        PoaTask& t = tasks[u.id];
        t.dg = u.dg;
        t.next = u.next;
        t.n_paths = u.n_paths;
        t.n_slots_next = u.n_slots_next;
        t.max_preds_next = u.max_preds_next;
        t.tables_ok = u.tables_ok;
        if (t.static_up && t.d_static) {  // reserved by this call, not yet uploaded: give it back
          darena->free(t.d_static, t.static_bytes);
          t.d_static = nullptr;
          t.d_path_off = t.d_paths = nullptr;
          t.static_up = false;
        }
      }
    for (uint32_t id = 0; id < tasks.size(); ++id) {
      if (!bad[id]) continue;
      if (bad[id] == 2 && id != victim) {
        waits[id] = 1;
        ++st.deferred_tasks;
        continue;
      }
      fail_task(g, id, "the device graph arena is full: this task's graph block would pass its limit of " +
                           std::to_string(darena->limit()) + " bytes (SVS_DEVICE_BUDGET_GB, fewer tasks in flight)");
    }
    drop(dp, nullptr);
    drop(chain, &chain_seq);
    // a waiting task stays active (its blocks so far stay reserved)
    size_t o = 0;
    for (size_t i = 0; i < g.active.size(); ++i)
      if (!bad[g.active[i]] || waits[g.active[i]]) g.active[o++] = g.active[i];
    g.active.resize(o);
  }

  // Prepares the group's next device launch, completing the tasks with nothing
  // left to align, and launches it.
  void advance_dev(Group& g, const DoneFn& done) {
    for (;;) {
      if (!g.completed.empty()) {
        const auto td0 = Clock::now();
        done(g.completed);
        for (uint32_t id : g.completed) graves.push_back(id);
        g_trace.host("done", gid(g), td0, g.completed.size());
        g.completed.clear();
      }
      refill(g);
      if (g.active.empty()) return;
      const auto th0 = Clock::now();
      std::vector<uint32_t> dp, chain, chain_seq, keep, fin;
      // tasks with nothing left to align complete first (every read empty; a
      // finished graph completes in finish_dev), before any task's state is
      // planned for the launch
      for (uint32_t id : g.active) {
        PoaTask& t = tasks[id];
        while (t.next < t.seqs.size() && t.seqs[t.next].empty()) ++t.next;
        if (t.next >= t.seqs.size()) {
          t.consensus.clear();
          t.msa.clear();
          fin.push_back(id);
        } else {
          keep.push_back(id);
        }
      }
      g.active = keep;
      if (!fin.empty()) {
        for (uint32_t id : fin) release_dev(tasks[id]);
        g.completed = fin;
        host_ms += ms_since(th0);
        continue;
      }
      // the next alignment of every task within the DP kernel's limits (a
      // task starting now aligns its second read against its first)
      keep.clear();
      for (uint32_t id : g.active) {
        const PoaTask& t = tasks[id];
        uint64_t rows = t.dg.V, len = t.next < t.seqs.size() ? t.seqs[t.next].size() : 0;
        if (t.dg.V == 0) {
          rows = len;
          size_t k = t.next + 1;
          while (k < t.seqs.size() && t.seqs[k].empty()) ++k;
          len = k < t.seqs.size() ? t.seqs[k].size() : 0;
        }
        const char* why = nullptr;
        if (t.dg.V > 0 && t.max_preds_next > kMaxInEdges)
          why = "a graph node has more than 4094 in-edges (traceback code limit)";
        else if (len > 0 && rows * strip_ls(static_cast<uint32_t>(len)) > 0x7FFFFFFFull)
          why = "an alignment's traceback matrix exceeds 2^31 cells";
        else if (sort_lds_words(rows + len) > sort_lds_max)
          why = "a POA graph too large for the sort kernel's LDS node flags (about 315,000 nodes)";
        if (why) fail_task(g, id, why);
        else keep.push_back(id);
      }
      if (keep.size() != g.active.size()) {
        g.active = keep;
        host_ms += ms_since(th0);
        continue;
      }
      std::vector<ChainUndo> undo;
      for (uint32_t id : g.active) {
        PoaTask& t = tasks[id];
        if (t.dg.V == 0) {
          undo.push_back(ChainUndo{id, t.dg, t.next, t.n_paths, t.n_slots_next, t.max_preds_next, t.tables_ok});
          // the first read becomes a chain before this launch's DP kernel; its
          // tables are known in advance (rows in read order, each reading the
          // row above: one pool slot), so the next read aligns in this launch
          // (deferring it to the next launch, so that the DP kernel need not
          // wait for the chain folds, measured slower: profiles/r05_dc1)
          chain.push_back(id);
          chain_seq.push_back(static_cast<uint32_t>(t.next));
          const uint32_t len = static_cast<uint32_t>(t.seqs[t.next].size());
          t.dg.V = len;
          t.dg.E = len - 1;
          t.dg.par = 1;
          t.n_paths = 1;
          t.n_slots_next = 1;
          t.max_preds_next = len > 1 ? 1 : 0;
          ++t.next;
          while (t.next < t.seqs.size() && t.seqs[t.next].empty()) ++t.next;
          t.tables_ok = t.next < t.seqs.size();
          if (t.tables_ok) dp.push_back(id);
        } else {
          dp.push_back(id);
        }
      }
      host_ms += ms_since(th0);
      // the launch's DP jobs within the group's device budget (longest first;
      // the rest wait for the next launch)
      order_by_cost(dp);
      const KernelEnv ke;
      uint64_t total = 0, code_bytes = force_wide() ? 4 : 2;
      for (uint32_t id : dp)
        if (tasks[id].max_preds_next > kMaxInEdgesNarrow) code_bytes = 4;
      size_t fit = 0;
      for (; fit < dp.size(); ++fit) {
        const PoaTask& t = tasks[dp[fit]];
        const uint64_t b = job_bytes_dev(t, ke, code_bytes);
        if (fit > 0 && total + b > budget) break;
        total += b;
      }
      dp.resize(fit);
      reserve_blocks(g, dp, chain, chain_seq, undo);
      // every task of the launch failed alone (or waits for the other group)
      if (dp.empty() && chain.empty()) {
        if (groups[1 - gid(g)].pending) return;
        continue;
      }
      const auto tp0 = Clock::now();
      pack_and_launch_dev(g, dp, chain, chain_seq);
      g_trace.host("pack", gid(g), tp0, dp.size() + chain.size());
      g.pending = true;
      return;
    }
  }

  uint64_t job_bytes_dev(const PoaTask& t, const KernelEnv& ke, uint64_t code_bytes) const {
    const uint64_t L = t.seqs[t.next].size(), ls = strip_ls(static_cast<uint32_t>(L)), V = t.dg.V;
    const uint64_t pool = (t.n_slots_next > kStripMaxLdsSlots || ke.global_pool)
                              ? 8ull * round_up(static_cast<uint64_t>(t.n_slots_next) * 97, 64) * 4 : 0;
    return V * ls * code_bytes + round_up(V, 8) * (ls / 64) * 16 + pool + 256 + (V + L + 1) * 8;
  }

  void pack_and_launch_dev(Group& g, const std::vector<uint32_t>& dp, const std::vector<uint32_t>& chain,
                           const std::vector<uint32_t>& chain_seq) {
    auto th0 = Clock::now();
    PoaArena& A = *g.arena;
    DevLaunch& D = g.dl;
    D = DevLaunch{};
    D.dp_ids = dp;
    D.n_pre = chain.size();
    D.fold_ids = chain;
    D.fold_ids.insert(D.fold_ids.end(), dp.begin(), dp.end());
    D.fold_seq = chain_seq;
    for (uint32_t id : dp) D.fold_seq.push_back(static_cast<uint32_t>(tasks[id].next));
    const size_t nj = dp.size(), nf = D.fold_ids.size(), npre = D.n_pre;
    // reads of the tasks that start with this launch: blocks planned here,
    // images written straight into the pinned staging below
    std::vector<std::pair<size_t, PoaTask*>> uploads;  // staging offset (from s_up), task
    std::vector<size_t> up_bytes;
    size_t up_total = 0;
    // (the reads blocks and the chains' graph blocks were reserved by
    // reserve_blocks)
    for (uint32_t id : D.fold_ids)
      if (tasks[id].static_up) {
        PoaTask& t = tasks[id];
        t.static_up = false;
        const size_t b = static_cast<size_t>(reinterpret_cast<uint8_t*>(t.d_paths) - t.d_static);
        uploads.emplace_back(up_total, &t);
        up_bytes.push_back(b);
        up_total += round_up(b, 64);
      }
    // DP jobs: the tables the last fold exported, in the task's block
    D.jobs.assign(nj, PoaJob{});
    uint64_t n_tb = 0, n_bnd = 0, n_pool = 0, n_aln = 0;
    uint32_t max_slots = 1, min_strips = 0xFFFFFFFFu;
    bool any_prune = false, wide = force_wide();
    for (uint32_t id : dp) {
      const PoaTask& t = tasks[id];
      if (!t.tables_ok) throw SvsError(SVS_E_INTERNAL, "device graph: no row tables for the next read");
      if (t.max_preds_next > kMaxInEdges)
        throw SvsError(SVS_E_UNSUPPORTED, "a graph node has more than 4094 in-edges (traceback code limit)");
      wide = wide || t.max_preds_next > kMaxInEdgesNarrow;
      max_slots = std::max(max_slots, t.n_slots_next);
      min_strips = std::min(min_strips, strip_ls(static_cast<uint32_t>(t.seqs[t.next].size())) / 64);
    }
    const bool lds_pool = max_slots <= kStripMaxLdsSlots && !strip_pool_forced_global();
    const int wpj = nj ? choose_wpj(nj, max_slots, min_strips, lds_pool) : 1;
    const PruneEnv penv;
    for (size_t k = 0; k < nj; ++k) {
      const PoaTask& t = tasks[dp[k]];
      PoaJob& J = D.jobs[k];
      const DGraphLayout L = dgraph_layout(t.dg.cv, t.dg.ce);
      uint8_t* b = t.dg.blk;
      J.rec = reinterpret_cast<const uint32_t*>(b + L.rec);
      J.pstart = reinterpret_cast<const uint32_t*>(b + L.pstart);
      J.pred = reinterpret_cast<const uint32_t*>(b + L.pred);
      J.pslot = reinterpret_cast<const uint32_t*>(b + L.pslot);
      J.col0 = reinterpret_cast<const int32_t*>(b + L.col0);
      J.seq = t.d_static + t.seq_at[t.next];
      J.info = nullptr;
      J.prep = 0;
      J.n_rows = t.dg.V;
      J.len = static_cast<uint32_t>(t.seqs[t.next].size());
      J.ls = strip_ls(J.len);
      J.n_slots = t.n_slots_next;
      if (static_cast<uint64_t>(J.n_rows) * J.ls > 0x7FFFFFFFull)
        throw SvsError(SVS_E_UNSUPPORTED, "a job's traceback matrix exceeds 2^31 cells");
      J.tb_off = n_tb;
      J.bnd_off = check_carry_aligned(n_bnd);
      J.pool_off = n_pool;
      J.aln_off = n_aln;
      J.lb = prune_bound(t, score, J.n_rows, J.len, penv);
      if (J.n_slots > 31 || J.len > kPruneMaxReadLen) J.lb = kNoPrune;
      any_prune = any_prune || J.lb != kNoPrune;
      n_tb += static_cast<uint64_t>(J.n_rows) * J.ls;
      n_bnd += round_up(round_up(J.n_rows, kCarryLineRows) * (J.ls / 64) * 4, kCarryAlignInts);
      if (!lds_pool) n_pool += static_cast<uint64_t>(wpj) * round_up(static_cast<uint64_t>(J.n_slots) * 97, 64);
      n_aln += static_cast<uint64_t>(J.n_rows) + J.len + 1;
      st.dp_cells += static_cast<uint64_t>(J.n_rows + 1) * (J.len + 1);
    }
    if (any_prune)
      for (PoaJob& J : D.jobs)
        if (J.lb == kNoPrune) J.lb = kPruneAll;
    D.n_aln = n_aln;
    D.wpj = wpj;
    D.prune = any_prune;
    D.wide = wide;
    st.wide_launches += (wide && nj) ? 1 : 0;  // DP launches only (a launch of chains alone runs no DP kernel)
    // (hints: the carries are 16 B per 64 traceback codes, the pairs 8 B per
    // row and read base; sized once for the group's budget instead of growing
    // with the graphs)
    A.d_tb.ensure(n_tb * (wide ? 4 : 2) + 4096, ctx->device_budget / n_groups);
    A.d_pool.ensure((n_bnd + n_pool) * 4 + 4096, ctx->device_budget / (8 * n_groups));
    A.d_aln.ensure(n_aln * 8 + 64, 256ull << 20);
    A.d_alen.ensure(nj * 12 + 64);
    // fold jobs, growing blocks that could not hold this fold
    D.folds.assign(nf, FoldJob{});
    D.moved.assign(nf, 0);
    D.cons_off.assign(nf, 0);
    D.msa_off.assign(nf, 0);
    D.feat_off.assign(nf, 0);
    // the fin buffer: every final fold's consensus, then the MSA rows (their
    // offsets from the MSA part's start until the consensus part is sized);
    // a window MSA of the decision pipeline keeps its rows on the device and
    // writes seqdatamx into the group's h_feat (kFoldFeat)
    size_t fin = 0, fin_msa = 0, feat = 0;
    bool msa_back = false;
    auto final_outputs = [&](size_t i, PoaTask& t, FoldJob& F, size_t bound, uint32_t rows) {
      D.cons_off[i] = fin;
      fin = round_up(fin + bound, 64);
      F.msa_stride = static_cast<uint32_t>(round_up(bound, 64));
      if (!t.genmsa) return;
      D.msa_off[i] = fin_msa;
      fin_msa += static_cast<size_t>(rows) * F.msa_stride;
      if (t.features && t.feat_params.ok) {
        F.flags |= kFoldFeat;
        F.f5_take = t.feat_params.f5_take;
        F.f3_take = t.feat_params.f3_take;
        F.extra = t.feat_params.extra;
        F.cut = t.feat_params.cut;
        D.feat_off[i] = feat;
        feat = round_up(feat + static_cast<size_t>(rows - 1 + F.extra) * F.msa_stride, 64);
      }
      if (!(F.flags & kFoldFeat) || verify) msa_back = true;
    };
    std::vector<std::array<uint64_t, 9>> moves;  // src, cv0, ce0, dst, cv1, ce1, V, E, par
    for (size_t i = 0; i < nf; ++i) {
      PoaTask& t = tasks[D.fold_ids[i]];
      FoldJob& F = D.folds[i];
      const uint32_t si = D.fold_seq[i];
      const uint32_t len = static_cast<uint32_t>(t.seqs[si].size());
      const bool chain_job = i < npre;
      if (chain_job) {
        F.blk = t.dg.blk;
        F.cv = t.dg.cv;
        F.ce = t.dg.ce;
        F.V = 0;
        F.E = 0;
        F.par = 0;
        F.n_paths = 0;
        const bool last = si + 1 >= t.last_nonempty;
        F.flags = kFoldChain | (last ? (kFoldFinal | (t.genmsa ? kFoldMsa : 0u)) : kFoldExport);
        F.seq = t.d_static + t.seq_at[si];
        F.len = len;
        F.paths = t.d_paths;
        F.path_off = t.d_path_off;
        if (last) final_outputs(i, t, F, len, 1);
        continue;
      }
      if (t.grow_blk) {
        // the larger block reserve_blocks took for this fold
        uint8_t* nb = t.grow_blk;
        const uint32_t cv1 = t.grow_cv, ce1 = t.grow_ce;
        moves.push_back({reinterpret_cast<uint64_t>(t.dg.blk), t.dg.cv, t.dg.ce, reinterpret_cast<uint64_t>(nb), cv1,
                         ce1, t.dg.V, t.dg.E, t.dg.par});
        D.old_blocks.emplace_back(t.dg.blk, t.dg_bytes);
        D.moved[i] = 1;
        t.dg.blk = nb;
        t.dg.cv = cv1;
        t.dg.ce = ce1;
        t.dg_bytes = t.grow_bytes;
        t.grow_blk = nullptr;
      }
      F.blk = t.dg.blk;
      F.cv = t.dg.cv;
      F.ce = t.dg.ce;
      F.V = t.dg.V;
      F.E = t.dg.E;
      F.par = t.dg.par;
      const bool last = si + 1 >= t.last_nonempty;
      F.flags = last ? (kFoldFinal | (t.genmsa ? kFoldMsa : 0u)) : kFoldExport;
      F.seq = t.d_static + t.seq_at[si];
      F.len = len;
      F.n_paths = t.n_paths;
      F.paths = t.d_paths;
      F.path_off = t.d_path_off;
      if (last) final_outputs(i, t, F, t.dg.V + len, t.n_paths + 1);
    }
    const size_t fin_cons = round_up(fin, 256);
    for (size_t i = 0; i < nf; ++i) D.msa_off[i] += fin_cons;
    fin = fin_cons + fin_msa;
    D.fin_bytes = fin;
    D.fin_copy = msa_back ? fin : fin_cons;
    // descriptors: DP jobs, fold jobs, fold results; then the new tasks' reads
    // and the scatter list that copies them into their blocks
    const size_t s_fold = round_up(nj * sizeof(PoaJob), 256);
    const size_t s_res = round_up(s_fold + nf * sizeof(FoldJob), 256);
    const size_t s_up = round_up(s_res + nf * sizeof(FoldResult), 256);
    const size_t s_cp = round_up(s_up + up_total, 256);
    // the final kernel's grid: the post-DP folds with kFoldFinal only (each
    // workgroup of a launch gets the launch's LDS, up to 64 KiB: a grid over
    // every fold made ~2,000 empty workgroups wait for that much LDS beside
    // the other group's DP workgroups)
    std::vector<uint32_t> fin_idx;
    for (size_t i = npre; i < nf; ++i)
      if (D.folds[i].flags & kFoldFinal) fin_idx.push_back(static_cast<uint32_t>(i - npre));
    const size_t s_fidx = round_up(s_cp + uploads.size() * sizeof(CopyDesc), 256);
    const size_t s_mv = round_up(s_fidx + fin_idx.size() * sizeof(uint32_t), 256);
    const size_t total = s_mv + moves.size() * sizeof(MoveDesc);
    D.s_fidx = s_fidx;
    D.n_fin = fin_idx.size();
    D.s_fold = s_fold;
    D.s_res = s_res;
    A.h_desc.ensure(total);
    A.d_desc.ensure(total);
    A.d_fin.ensure(fin + 64);
    A.h_fin.ensure(D.fin_copy + 64);
    A.h_feat.ensure(feat + 64);
    uint8_t* d_feat = nullptr;  // the device's view of the pinned h_feat (zero-copy writes)
    if (feat) SVS_HIP(hipHostGetDevicePointer(reinterpret_cast<void**>(&d_feat), A.h_feat.ptr, 0));
    char* dd = A.d_desc.as<char>();
    for (size_t i = 0; i < nf; ++i) {
      FoldJob& F = D.folds[i];
      F.result = reinterpret_cast<FoldResult*>(dd + s_res) + i;
      if (i >= npre) {
        F.aln = A.d_aln.as<int32_t>() + 2 * D.jobs[i - npre].aln_off;
        F.aln_status = A.d_alen.as<int32_t>() + (i - npre);
      }
      if (F.flags & kFoldFinal) {
        F.cons_out = A.d_fin.as<char>() + D.cons_off[i];
        F.msa_out = A.d_fin.as<char>() + D.msa_off[i];
        F.feat_out = (F.flags & kFoldFeat) ? d_feat + D.feat_off[i] : nullptr;
      }
    }
    char* hd = A.h_desc.as<char>();
    if (nj) std::memcpy(hd, D.jobs.data(), nj * sizeof(PoaJob));
    std::memcpy(hd + s_fold, D.folds.data(), nf * sizeof(FoldJob));
    for (size_t i = 0; i < nf; ++i) {
      FoldResult r{};
      r.status = kFoldNotRun;  // only the update kernel makes it kFoldOk
      std::memcpy(hd + s_res + i * sizeof(FoldResult), &r, sizeof(r));
    }
    if (!fin_idx.empty()) std::memcpy(hd + s_fidx, fin_idx.data(), fin_idx.size() * sizeof(uint32_t));
    for (size_t k = 0; k < moves.size(); ++k) {
      const auto& m = moves[k];
      reinterpret_cast<MoveDesc*>(hd + s_mv)[k] =
          MoveDesc{reinterpret_cast<const uint8_t*>(m[0]), reinterpret_cast<uint8_t*>(m[3]), static_cast<uint32_t>(m[1]),
                   static_cast<uint32_t>(m[2]), static_cast<uint32_t>(m[4]), static_cast<uint32_t>(m[5]),
                   static_cast<uint32_t>(m[6]), static_cast<uint32_t>(m[7]), static_cast<uint32_t>(m[8]), 0u};
    }
    CopyDesc* cps = reinterpret_cast<CopyDesc*>(hd + s_cp);
    for (size_t u = 0; u < uploads.size(); ++u)
      cps[u] = CopyDesc{dd + s_up + uploads[u].first, uploads[u].second->d_static, round_up(up_bytes[u], 64)};
    if (!uploads.empty())
      ctx->pool->parallel_for(uploads.size(), [&](size_t u) {
        write_static(*uploads[u].second, hd + s_up + uploads[u].first, round_up(up_bytes[u], 64));
      });
    host_ms += ms_since(th0);

    hipStream_t side = A.copy_stream;
    SVS_HIP(hipMemcpyAsync(dd, hd, total, hipMemcpyHostToDevice, side));
    if (!uploads.empty())
      SVS_HIP(launch_scatter_copy(reinterpret_cast<const CopyDesc*>(dd + s_cp), static_cast<int>(uploads.size()), side));
    SVS_HIP(launch_dgraph_moves(reinterpret_cast<const MoveDesc*>(dd + s_mv), static_cast<int>(moves.size()), side));
    uint32_t lds_words = 0;
    for (const FoldJob& F : D.folds) lds_words = std::max(lds_words, static_cast<uint32_t>(sort_lds_words(F.V + F.len)));
    // (the DFS stack's LDS part is in it; deeper stacks spill)
    if (lds_words > sort_lds_max)
      throw SvsError(SVS_E_INTERNAL, "sort kernel LDS over the workgroup limit despite the per-task check");
    // the final kernel's LDS per job (6 B per node, up to 64 KiB; larger
    // graphs score in global memory), 0 when a fold range has no final fold
    auto final_lds = [&](size_t i0, size_t i1) -> uint32_t {
      uint32_t w = 0;
      for (size_t i = i0; i < i1; ++i) {
        const FoldJob& F = D.folds[i];
        if (F.flags & kFoldFinal) w = std::max(w, (6 * (F.V + F.len) + 8 + 3) / 4);
      }
      return std::min(w, static_cast<uint32_t>(SVS_FINAL_LDS_CAP));
    };
    const FoldJob* dfold = reinterpret_cast<const FoldJob*>(dd + s_fold);
    SVS_HIP(hipEventRecord(A.evp, side));
    if (npre) {
      // the new tasks' first reads, and their tables, before the DP kernel
      SVS_HIP(launch_poa_fold(dfold, static_cast<int>(npre), lds_words, final_lds(0, npre), side, A.evpk));
      SVS_HIP(launch_dgraph_prep(dfold, static_cast<int>(npre), score, side));
    }
    SVS_HIP(hipEventRecord(A.evp1, side));
    if (npre && sync_check()) {
      // SVS_POA_SYNC_CHECK=1 (debugging): the chains' results before any DP
      // kernel reads their tables
      std::vector<FoldResult> rr(npre);
      SVS_HIP(hipMemcpyAsync(rr.data(), dd + s_res, npre * sizeof(FoldResult), hipMemcpyDeviceToHost, side));
      SVS_HIP(hipStreamSynchronize(side));
      for (size_t i = 0; i < npre; ++i) {
        const FoldJob& F = D.folds[i];
        if (rr[i].status != kFoldOk || rr[i].V != F.len || rr[i].E != F.len - 1 ||
            ((F.flags & kFoldExport) && rr[i].n_slots != 1))
          throw SvsError(SVS_E_INTERNAL, "sync check: chain fold " + std::to_string(i) + " status " +
                                             std::to_string(rr[i].status) + " V " + std::to_string(rr[i].V) + "/" +
                                             std::to_string(F.len) + " slots " + std::to_string(rr[i].n_slots));
      }
    }
    SVS_HIP(hipEventRecord(A.h2d, side));
    D.timed_dp = nj > 0;
    if (nj) {
      PoaLaunch pl{};
      pl.jobs = reinterpret_cast<const PoaJob*>(dd);
      pl.n_jobs = static_cast<int>(nj);
      pl.score = score;
      pl.tb = A.d_tb.as<char>();
      pl.bnd = A.d_pool.as<int32_t>();
      pl.pool = A.d_pool.as<int32_t>() + n_bnd;
      pl.aln = A.d_aln.as<int32_t>();
      pl.aln_len = A.d_alen.as<int32_t>();
      pl.lds_slots = lds_pool ? max_slots : 0;
      pl.prune = any_prune;
      pl.wide = wide;
      pl.waves_per_job = wpj;
      check_carry_base(pl.bnd);
      // the pool slots per wave the launch's LDS is sized for (its occupancy)
      g_trace.host("slots", gid(g), Clock::now(), pl.lds_slots);
      SVS_HIP(hipStreamWaitEvent(A.stream, A.h2d, 0));
      SVS_HIP(hipEventRecord(A.ev0, A.stream));
      SVS_HIP(launch_poa_strip(pl, A.stream));
      SVS_HIP(hipEventRecord(A.ev1, A.stream));
      SVS_HIP(hipStreamWaitEvent(side, A.ev1, 0));
    }
    // graph update, sort, export and table completion beside the other group's DP
    SVS_HIP(hipEventRecord(A.evf0, side));
    const uint32_t fin_lds = nj ? final_lds(npre, npre + nj) : 0u;
    D.split_final = fin_lds;
    if (nj) {
      SVS_HIP(launch_poa_fold(dfold + npre, static_cast<int>(nj), lds_words, D.split_final ? 0u : fin_lds, side, A.evk));
      if (D.split_final) {
        // a finishing task needs no tables and a continuing one no consensus:
        // the final kernel runs beside the table completion
        SVS_HIP(hipEventRecord(A.ev_sorted, side));
        SVS_HIP(hipStreamWaitEvent(A.fin_stream, A.ev_sorted, 0));
        SVS_HIP(hipEventRecord(A.ev_fin0, A.fin_stream));
        SVS_HIP(launch_poa_final(dfold + npre, reinterpret_cast<const uint32_t*>(dd + D.s_fidx),
                                 static_cast<int>(D.n_fin), fin_lds, A.fin_stream));
        SVS_HIP(hipEventRecord(A.ev_fin1, A.fin_stream));
      }
      SVS_HIP(launch_dgraph_prep(dfold + npre, static_cast<int>(nj), score, side));
    }
    SVS_HIP(hipEventRecord(A.evf1, side));
    if (D.split_final) SVS_HIP(hipStreamWaitEvent(side, A.ev_fin1, 0));
    A.h_alen.ensure(nj * 12 + 64);
    if (nj) SVS_HIP(hipMemcpyAsync(A.h_alen.ptr, A.d_alen.ptr, nj * 12, hipMemcpyDeviceToHost, side));
    SVS_HIP(hipMemcpyAsync(hd + s_res, dd + s_res, nf * sizeof(FoldResult), hipMemcpyDeviceToHost, side));
    if (D.fin_copy) SVS_HIP(hipMemcpyAsync(A.h_fin.ptr, A.d_fin.ptr, D.fin_copy, hipMemcpyDeviceToHost, side));
    if (verify) {
      A.h_aln.ensure(n_aln * 8 + 64);
      if (nj) SVS_HIP(hipMemcpyAsync(A.h_aln.ptr, A.d_aln.ptr, n_aln * 8, hipMemcpyDeviceToHost, side));
    }
    SVS_HIP(hipEventRecord(A.ev_end, side));
    SVS_HIP(hipEventRecord(A.done, side));
    if (debug_launches()) {
      uint32_t vmax = 0;
      for (const FoldJob& F : D.folds) vmax = std::max(vmax, F.V + F.len);
      std::fprintf(stderr, "[svs] dev launch g%d: %zu dp (wpj %d, slots %u, prune %d), %zu pre, %zu post folds, "
                           "max V+len %u, lds %u words, %zu moves, fin %zu\n",
                   gid(g), nj, wpj, max_slots, any_prune ? 1 : 0, npre, nf - npre, vmax, lds_words, moves.size(), fin);
      std::fflush(stderr);
    }
    st.launches += nj ? 1 : 0;
    st.alignments += nj;
    st.tb_bytes += n_tb * 2;
    st.pool_bytes += (n_bnd + n_pool) * 4;
    st.h2d_bytes += total;
    st.d2h_bytes += nj * 12 + nf * sizeof(FoldResult) + D.fin_copy;
    st.fold_jobs += nf;
    for (const FoldJob& F : D.folds) st.prep_jobs += (F.flags & kFoldExport) ? 1 : 0;
  }

  // Waits for the group's device launch and takes its results: DP statistics
  // and retries, the folded graphs' new counts, and the finished tasks.
  void finish_dev(Group& g) {
    PoaArena& A = *g.arena;
    DevLaunch& D = g.dl;
    const auto tw0 = Clock::now();
    for (;;) {
      const hipError_t q = hipEventQuery(A.done);
      if (q == hipSuccess) break;
      if (q != hipErrorNotReady) SVS_HIP(q);
      if (!reap()) break;
    }
    SVS_HIP(hipEventSynchronize(A.done));
    st.gpu_wait_ms += ms_since(tw0);
    const size_t nj = D.dp_ids.size(), nf = D.fold_ids.size();
    if (debug_launches()) {
      std::fprintf(stderr, "[svs] dev done g%d: %zu dp, %zu folds, %.1f ms wait\n", gid(g), nj, nf, ms_since(tw0));
      std::fflush(stderr);
    }
    if (D.timed_dp) {
      float ms = 0.f;
      SVS_HIP(hipEventElapsedTime(&ms, A.ev0, A.ev1));
      st.kernel_ms += ms;
      dp_busy.add(A.ev0, A.ev1, st);
      float tail = 0.f;
      SVS_HIP(hipEventElapsedTime(&tail, A.ev1, A.ev_end));
      st.dp_to_done_ms += tail;
    }
    {
      float ms = 0.f, pms = 0.f;
      SVS_HIP(hipEventElapsedTime(&ms, A.evf0, A.evf1));
      SVS_HIP(hipEventElapsedTime(&pms, A.evp, A.evp1));
      st.fold_ms += ms + pms;
      st.dgraph_peak_bytes = std::max<uint64_t>(st.dgraph_peak_bytes, darena->peak());
      st.dgraph_reserved_bytes = darena->reserved();
      // per fold kernel: update, sort, final, then the table completion
      auto phases = [&](hipEvent_t e0, const hipEvent_t* k, hipEvent_t e1) {
        float t[4] = {0.f, 0.f, 0.f, 0.f};
        SVS_HIP(hipEventElapsedTime(&t[0], e0, k[0]));
        SVS_HIP(hipEventElapsedTime(&t[1], k[0], k[1]));
        SVS_HIP(hipEventElapsedTime(&t[2], k[1], k[2]));
        SVS_HIP(hipEventElapsedTime(&t[3], k[2], e1));
        st.fold_update_ms += t[0];
        st.fold_sort_ms += t[1];
        st.fold_final_ms += t[2];
        st.fold_prep_ms += t[3];
        if (g_trace.f) {
          size_t n_final = 0;
          for (const FoldJob& F : D.folds) n_final += (F.flags & kFoldFinal) ? 1 : 0;
          std::fprintf(g_trace.f, "fph %d %.3f %.3f %.3f %.3f %zu\n", (e0 == A.evf0 ? 10 : 20) + gid(g), t[0], t[1], t[2],
                       t[3], n_final);
        }
      };
      if (nj) phases(A.evf0, A.evk, A.evf1);
      if (nj && D.split_final) {
        float t = 0.f;
        SVS_HIP(hipEventElapsedTime(&t, A.ev_fin0, A.ev_fin1));
        st.fold_final_ms += t;
      }
      if (D.n_pre) phases(A.evp, A.evpk, A.evp1);
    }
    if (g_trace.f) {
      uint64_t cells = 0;
      for (const PoaJob& J : D.jobs) cells += static_cast<uint64_t>(J.n_rows + 1) * (J.len + 1);
      g_trace.host("wait", gid(g), tw0, nf);
      uint64_t computed = 0;
      const int32_t* al = A.h_alen.as<int32_t>();
      for (size_t k = 0; k < nj; ++k) computed += 64ull * static_cast<uint32_t>(al[2 * nj + k]);
      if (D.timed_dp) g_trace.kernel(gid(g), A.ev0, A.ev1, nj, D.wpj, cells, D.prune, D.wide, computed);
      g_trace.kernel(10 + gid(g), A.evf0, A.evf1, nj, 0, 0);  // the fold chain after the DP kernel
      if (D.n_pre) g_trace.kernel(20 + gid(g), A.evp, A.evp1, D.n_pre, 0, 0);  // the chains before it
    }
    const auto th0 = Clock::now();
    const int32_t* alen = A.h_alen.as<int32_t>();
    const FoldResult* res = reinterpret_cast<const FoldResult*>(A.h_desc.as<char>() + D.s_res);
    for (size_t k = 0; k < nj; ++k) {
      PoaTask& t = tasks[D.dp_ids[k]];
      st.cells_computed += 64ull * static_cast<uint32_t>(alen[2 * nj + k]);
      t.last_rows = static_cast<uint32_t>(alen[2 * nj + k]);
      const int32_t n = alen[k];
      if (n == kPruneRetry) {
        st.prune_retries += 1;
        t.retry = true;
        t.n_retries += 1;
        t.read_retries += 1;
        continue;
      }
      if (n < 0) throw SvsError(SVS_E_INTERNAL, "GPU traceback reported an inconsistent path");
      const uint32_t len = D.jobs[k].len;
      if (!t.retry && len > 0) {
        t.rate = static_cast<double>(alen[nj + k]) / len;
        t.have_rate = true;
      }
      t.retry = false;
      t.read_retries = 0;
    }
    for (auto& b : D.old_blocks) darena->free(b.first, b.second);
    D.old_blocks.clear();
    for (size_t i = 0; i < nf; ++i) {
      PoaTask& t = tasks[D.fold_ids[i]];
      const FoldResult& r = res[i];
      const FoldJob& F = D.folds[i];
      if (r.status == kFoldSkipped) continue;  // a pruning retry: graph and tables unchanged
      if (!t.error.empty()) continue;          // the task failed at an earlier fold of this launch
      if (verify && r.status == kFoldErrStack) verify_fold(g, i, r);  // names the first table that differs
      if (r.status != kFoldOk) {
        std::string why = "device POA graph fold failed (status " + std::to_string(r.status) + "; fold of read " +
                          std::to_string(F.n_paths) + ", graph " + std::to_string(F.V) + " nodes + read of " +
                          std::to_string(F.len) + ", flags " + std::to_string(F.flags);
        if (r.status == kFoldErrStack)
          why += "; sort emitted " + std::to_string(r.pad0) + " of " + std::to_string(r.V) + " nodes, stack " +
                 (r.pad1 ? "overflowed" : "ok") + ", " + std::to_string(r.n_exam) + " examinations, " +
                 std::to_string(r.n_roots) + " roots";
        throw SvsError(SVS_E_INTERNAL, why + ")");
      }
      g_fold_times.add(r, F.flags);
      if (verify) verify_fold(g, i, r);
      if (i < D.n_pre) {
        // a chain: the counts the launch assumed for its second read
        if (r.V != F.len || r.E != F.len - 1 ||
            ((F.flags & kFoldExport) && (r.n_slots != 1 || r.max_preds != (F.len > 1 ? 1u : 0u))))
          throw SvsError(SVS_E_INTERNAL, "device POA graph: first-read chain differs from its planned tables");
      } else {
        t.dg.V = r.V;
        t.dg.E = r.E;
        t.dg.par ^= 1u;
        t.n_paths += 1;
        t.next = D.fold_seq[i] + 1;
      }
      t.dg.ncol = r.ncol;
      if (F.flags & kFoldExport) {
        t.n_slots_next = r.n_slots;
        t.max_preds_next = r.max_preds;
        // the device planner's limits (poa_prep.hip); beyond them the tables
        // are incomplete: this task fails alone
        if (r.V > planner_max_rows() || r.n_slots > kStripPrepMaxSlots || r.max_preds > kMaxInEdges) {
          fail_task(g, D.fold_ids[i],
                    "a POA graph beyond the device row-table planner's limits (" + std::to_string(r.V) + " rows, " +
                        std::to_string(r.n_slots) + " pool slots, " + std::to_string(r.max_preds) + " in-edges)");
          continue;
        }
        t.tables_ok = true;
      }
      if (F.flags & kFoldFinal) {
        const char* h = A.h_fin.as<char>();
        const uint32_t nc = r.pad0;
        t.consensus.assign(h + D.cons_off[i], nc);
        std::reverse(t.consensus.begin(), t.consensus.end());
        t.msa.clear();
        if ((F.flags & kFoldMsa) && D.fin_copy > D.msa_off[i]) {
          t.msa.reserve(t.n_paths);
          for (uint32_t s = 0; s < t.n_paths; ++s)
            t.msa.emplace_back(h + D.msa_off[i] + static_cast<size_t>(s) * F.msa_stride, r.ncol);
        }
        if (F.flags & kFoldFeat) {
          // seqdatamx, written by the final kernel straight into pinned memory
          // (counted as D2H: it crosses PCIe)
          const uint8_t* fx = A.h_feat.as<uint8_t>() + D.feat_off[i];
          t.n_feat = static_cast<int32_t>(r.pad1);
          t.feat.assign(fx, fx + static_cast<size_t>(t.n_paths - 1 + F.extra) * r.pad1);
          st.d2h_bytes += t.feat.size();
        }
        if (verify) verify_final(t);
        release_dev(t);
        g.completed.push_back(D.fold_ids[i]);
      }
    }
    if (!g.completed.empty()) {
      std::vector<uint32_t> keep;
      keep.reserve(g.active.size());
      std::vector<uint8_t> gone(tasks.size(), 0);
      for (uint32_t id : g.completed) gone[id] = 1;
      for (uint32_t id : g.active)
        if (!gone[id]) keep.push_back(id);
      g.active.swap(keep);
    }
    host_ms += ms_since(th0);
    g_trace.host("fold", gid(g), th0, nf);
  }

  // SVS_POA_VERIFY_GRAPH: replay fold i on the task's host graph and compare
  // the device's rank order and exported tables with the host's.
  void verify_fold(Group& g, size_t i, const FoldResult& r) {
    PoaArena& A = *g.arena;
    DevLaunch& D = g.dl;
    PoaTask& t = tasks[D.fold_ids[i]];
    const FoldJob& F = D.folds[i];
    const std::string& s = t.seqs[D.fold_seq[i]];
    const uint32_t V0 = t.graph.num_nodes();
    std::vector<size_t> deg0(V0), al0(V0);
    for (uint32_t v = 0; v < V0; ++v) {
      deg0[v] = t.graph.in_degree(v);
      al0[v] = t.graph.aligned_count(v);
    }
    if (F.flags & kFoldChain) {
      t.graph.add_alignment_nodes({}, s);
    } else {
      const size_t k = i - D.n_pre;
      const int32_t n = A.h_alen.as<int32_t>()[k];
      const int32_t* p = A.h_aln.as<int32_t>() + 2 * D.jobs[k].aln_off;
      std::vector<int32_t> fwd(2 * static_cast<size_t>(n));
      for (int32_t x = 0; x < n; ++x) {
        fwd[2 * x] = p[2 * (n - 1 - x)];
        fwd[2 * x + 1] = p[2 * (n - 1 - x) + 1];
      }
      t.graph.add_alignment_ranks(fwd, s);
    }
    const uint32_t V = t.graph.num_nodes(), E = t.graph.num_edges();
    // a chain whose next read was aligned and folded in the same launch: the
    // block already holds the later graph (checked with that fold)
    if (i < D.n_pre)
      for (size_t j = D.n_pre; j < D.fold_ids.size(); ++j)
        if (D.fold_ids[j] == D.fold_ids[i]) return;
    auto fail = [&](const std::string& what) {
      throw SvsError(SVS_E_INTERNAL, "device graph differs from the host graph after fold (" + what + "), read " +
                                         std::to_string(D.fold_seq[i]) + ", V " + std::to_string(V));
    };
    const DGraphLayout L = dgraph_layout(F.cv, F.ce);
    if (!(F.flags & kFoldChain) && V0) {
      // the update kernel's changed plane (the sort's reuse test)
      std::vector<uint32_t> chg((V0 + 31) / 32);
      SVS_HIP(hipMemcpy(chg.data(), F.blk + L.chg, 4 * chg.size(), hipMemcpyDeviceToHost));
      uint32_t bad = 0, first = 0, dev1 = 0, host1 = 0;
      for (uint32_t v = 0; v < V0; ++v) {
        const bool c = t.graph.in_degree(v) != deg0[v] || t.graph.aligned_count(v) != al0[v];
        const uint32_t d = (chg[v >> 5] >> (v & 31)) & 1u;
        dev1 += d;
        host1 += c ? 1u : 0u;
        if (d != (c ? 1u : 0u) && bad++ == 0) first = v;
      }
      if (bad)
        fail("changed flags: " + std::to_string(bad) + " differ, first node " + std::to_string(first) + "; device " +
             std::to_string(dev1) + " set, host " + std::to_string(host1) + "; V0 " + std::to_string(V0) +
             ", device V0 " + std::to_string(F.V) + ", par " + std::to_string(F.par) + ", cv " + std::to_string(F.cv));
    }
    if (r.V != V || r.E != E) fail("node/edge counts " + std::to_string(r.V) + "/" + std::to_string(r.E));
    std::vector<uint32_t> r2n(V);
    SVS_HIP(hipMemcpy(r2n.data(), F.blk + L.r2n, 4ull * V, hipMemcpyDeviceToHost));
    if (r2n != t.graph.rank_to_node()) fail("rank order");
    {
      // the segment starts the next sort walks (poa_fold.hip dfs_sort)
      std::vector<uint32_t> seg((V + 31) / 32);
      SVS_HIP(hipMemcpy(seg.data(), F.blk + L.seg[1 - F.par], 4 * seg.size(), hipMemcpyDeviceToHost));
      const std::vector<uint8_t>& hs = t.graph.segment_starts();
      for (uint32_t k = 0; k < V; ++k)
        if (((seg[k >> 5] >> (k & 31)) & 1u) != hs[k]) fail("segment start at rank " + std::to_string(k));
    }
    if (F.flags & kFoldExport) {
      RowTables h;
      std::vector<uint32_t> ps(V + 1), pr(E), inf(V);
      const StripLiteDst dst{ps.data(), pr.data(), inf.data()};
      t.graph.export_strip_lite(&h, &dst);
      std::vector<uint32_t> dps(V + 1), dpr(E), dinf(V);
      SVS_HIP(hipMemcpy(dps.data(), F.blk + L.pstart, 4ull * (V + 1), hipMemcpyDeviceToHost));
      if (E) SVS_HIP(hipMemcpy(dpr.data(), F.blk + L.pred, 4ull * E, hipMemcpyDeviceToHost));
      SVS_HIP(hipMemcpy(dinf.data(), F.blk + L.info, 4ull * V, hipMemcpyDeviceToHost));
      if (dps != ps) fail("pstart");
      if (dpr != pr) fail("in-edge rows");
      if (dinf != inf) fail("row words");
      if (h.n_slots != r.n_slots) fail("slot count " + std::to_string(r.n_slots) + " vs " + std::to_string(h.n_slots));
      if (h.max_preds != r.max_preds) fail("max in-degree");
      // the completed tables against the host's full export
      if (r.V <= kStripPrepMaxRows && r.n_slots <= kStripPrepMaxSlots && r.max_preds <= kMaxInEdges) {
        RowTables full;
        const int32_t gaps[4] = {score.g, score.e, score.q, score.c};
        t.graph.export_strip_rows(&full, gaps);
        std::vector<uint32_t> rec(4ull * V), psl(E);
        std::vector<int32_t> c0(3ull * V);
        SVS_HIP(hipMemcpy(rec.data(), F.blk + L.rec, rec.size() * 4, hipMemcpyDeviceToHost));
        if (E) SVS_HIP(hipMemcpy(psl.data(), F.blk + L.pslot, psl.size() * 4, hipMemcpyDeviceToHost));
        SVS_HIP(hipMemcpy(c0.data(), F.blk + L.col0, c0.size() * 4, hipMemcpyDeviceToHost));
        if (rec != full.rec) fail("row records");
        if (psl != full.pred_slot) fail("in-edge slots");
        if (c0 != full.col0) fail("column 0");
      }
    }
  }

  void verify_final(PoaTask& t) {
    const std::string cons = t.graph.consensus(cfg.min_coverage);
    if (cons != t.consensus)
      throw SvsError(SVS_E_INTERNAL, "device consensus differs from the host graph's (" +
                                         std::to_string(t.consensus.size()) + " vs " + std::to_string(cons.size()) + ")");
    if (t.genmsa && t.graph.msa() != t.msa) throw SvsError(SVS_E_INTERNAL, "device MSA differs from the host graph's");
  }

  // Prepares the group's next launch (or completes its tasks) and launches it.
  void advance(Group& g, const DoneFn& done) {
    if (dev) {
      advance_dev(g, done);
      return;
    }
    std::vector<uint8_t> needs;
    for (;;) {
      refill(g);
      if (g.active.empty()) return;
      auto th0 = Clock::now();
      needs.assign(g.active.size(), 0);
      PoaArena* stage = g.arena;
      // sequences landing on an empty graph become a fresh chain (no DP)
      ctx->pool->parallel_for(g.active.size(), [&](size_t i) {
        PoaTask& t = tasks[g.active[i]];
        const uint8_t state = t.prepped ? t.prepped : prep_task(t, cfg, stage);
        t.prepped = 0;
        needs[i] = state == 1 ? 1 : 0;
      });
      std::vector<uint32_t> ids, fin;
      for (size_t i = 0; i < g.active.size(); ++i) (needs[i] ? ids : fin).push_back(g.active[i]);
      host_ms += ms_since(th0);
      g_trace.host("prep", gid(g), th0, g.active.size());
      g.active = ids;
      if (!fin.empty()) {
        const auto td0 = Clock::now();
        done(fin);
        // graphs hold many small allocations: freeing a thousand of them takes
        // seconds, so they are released later, while the GPU runs (reap)
        for (uint32_t id : fin) graves.push_back(id);
        g_trace.host("done", gid(g), td0, fin.size());
        if (ids.empty()) continue;  // refill and try again
      }
      uint64_t total = 0, code_bytes = force_wide() ? 4 : 2;
      const KernelEnv ke;
      for (uint32_t id : ids)
        if (tasks[id].rows.max_preds > kMaxInEdgesNarrow) code_bytes = 4;
      for (uint32_t id : ids)
        total += job_bytes(tasks[id].rows, tasks[id].seqs[tasks[id].next].size(), ke, code_bytes);
      if (total <= budget) {
        order_by_cost(ids);
        g.la.ids = std::move(ids);
        g.la.arena = g.arena;
        g.la.gid = gid(g);
        const auto tp0 = Clock::now();
        pack_and_launch_strip(ctx, g.la, tasks, score, st, host_ms);
        g_trace.host("pack", gid(g), tp0, g.la.ids.size());
        g.pending = true;
        return;
      }
      // over budget: consecutive synchronous sub-launches, then prepare again
      size_t first = 0;
      while (first < ids.size()) {
        size_t last = first;
        uint64_t bytes = 0;
        while (last < ids.size()) {
          const uint64_t b =
              job_bytes(tasks[ids[last]].rows, tasks[ids[last]].seqs[tasks[ids[last]].next].size(), ke, code_bytes);
          if (last > first && bytes + b > budget) break;
          bytes += b;
          ++last;
        }
        Launch sub;
        sub.ids.assign(ids.begin() + first, ids.begin() + last);
        sub.arena = g.arena;
        sub.gid = gid(g);
        pack_and_launch_strip(ctx, sub, tasks, score, st, host_ms);
        finish(ctx, sub, tasks, st, host_ms, cfg, nullptr, &dp_busy);
        first = last;
      }
    }
  }

  int gid(const Group& g) const { return static_cast<int>(&g - groups); }

  // Longest expected job first: a launch holds more waves than the GPU keeps
  // resident, and workgroups start in job order, so the jobs that start last
  // should be short ones.  Expected cost: the strip rows the task's previous
  // alignment computed; for a retry or a task with no history, the unpruned
  // strip rows.
  void order_by_cost(std::vector<uint32_t>& ids) {
    std::vector<std::pair<uint64_t, uint32_t>> c(ids.size());
    for (size_t i = 0; i < ids.size(); ++i) {
      const PoaTask& t = tasks[ids[i]];
      const uint64_t rows = dev ? t.dg.V : t.rows.n_rows;
      const uint64_t full = rows * ((t.seqs[t.next].size() + 64) / 64);
      c[i] = {t.last_rows == 0 || t.retry ? full : t.last_rows, ids[i]};
    }
    std::stable_sort(c.begin(), c.end(), [](const auto& a, const auto& b) { return a.first > b.first; });
    for (size_t i = 0; i < ids.size(); ++i) ids[i] = c[i].second;
  }

  // Releases the storage of up to one pool-width chunk of finished tasks;
  // false when none are left.
  bool reap() {
    if (graves.empty()) return false;
    const auto t0 = Clock::now();
    const size_t n = std::min<size_t>(graves.size(), 4 * ctx->pool->size());
    const size_t base = graves.size() - n;
    ctx->pool->parallel_for(n, [&](size_t i) {
      PoaTask& t = tasks[graves[base + i]];
      t.graph = PoaGraph();
      t.rows = RowTables();
      std::vector<std::string>().swap(t.seqs);
    });
    // a long session reuses the slots of released tasks
    free_ids.insert(free_ids.end(), graves.begin() + static_cast<std::ptrdiff_t>(base), graves.end());
    graves.resize(base);
    g_trace.host("reap", -1, t0, n);
    return true;
  }

  void run(const DoneFn& done, const PollFn& poll) {
    g_trace.open(ctx->stream);
    Group* const gend = groups + n_groups;
    for (Group* gp = groups; gp != gend; ++gp) advance(*gp, done);
    for (;;) {
      bool progressed = false;
      for (Group* gp = groups; gp != gend; ++gp) {
        Group& g = *gp;
        if (!g.pending) continue;
        if (dev) finish_dev(g);
        else finish(ctx, g.la, tasks, st, host_ms, cfg, [this] { return reap(); }, &dp_busy);
        g.pending = false;
        advance(g, done);
        progressed = true;
      }
      const auto tq0 = Clock::now();
      const bool outside = poll(false);
      g_trace.host("poll", -1, tq0, 0);
      bool busy = false;
      for (Group* gp = groups; gp != gend; ++gp) {
        Group& g = *gp;
        if (!g.pending && (!queue.empty() || !g.completed.empty() || (dev && !g.active.empty()))) advance(g, done);
        busy = busy || g.pending;
      }
      if (progressed || busy) continue;
      if (outside) {
        const auto tb0 = Clock::now();
        poll(true);
        g_trace.host("block", -1, tb0, 0);
        continue;
      }
      break;
    }
    while (reap()) {
    }
    g_trace.close();
  }
};

PoaScheduler::PoaScheduler(svs_context* ctx, const svs_poa_config& cfg, svs_poa_stats& st)
    : impl_(nullptr) {
  check_poa_config(cfg);
  impl_ = new Impl(ctx, cfg, st);
}

PoaScheduler::~PoaScheduler() {
  for (auto& a : impl_->ctx->poa_arenas) {
    (void)hipStreamSynchronize(a->stream);
    (void)hipStreamSynchronize(a->copy_stream);
  }
  impl_->st.host_graph_ms += impl_->host_ms;
  delete impl_;
}

uint32_t PoaScheduler::add(PoaTask&& t) {
  t.next = 0;
  uint32_t id;
  if (!impl_->free_ids.empty()) {
    id = impl_->free_ids.back();
    impl_->free_ids.pop_back();
    impl_->tasks[id] = std::move(t);
  } else {
    id = static_cast<uint32_t>(impl_->tasks.size());
    impl_->tasks.push_back(std::move(t));
  }
  impl_->queue.push_back(id);
  impl_->queue_dirty = true;
  return id;
}

PoaTask& PoaScheduler::task(uint32_t id) { return impl_->tasks[id]; }

double PoaScheduler::host_ms() const { return impl_->host_ms; }

void PoaScheduler::run(const DoneFn& done, const PollFn& poll) { impl_->run(done, poll); }

void run_poa_tasks(svs_context* ctx, std::vector<PoaTask>& tasks, const svs_poa_config& cfg,
                   svs_poa_stats& st) {
  const auto t_wall0 = Clock::now();
  {
    PoaScheduler sched(ctx, cfg, st);
    for (auto& t : tasks) {
      t.genmsa = cfg.genmsa != 0;
      sched.add(std::move(t));
    }
    std::string first_error;
    sched.run(
        [&](const std::vector<uint32_t>& ids) {
          for (uint32_t id : ids) {
            PoaTask& t = sched.task(id);
            if (!t.error.empty() && first_error.empty())
              first_error = "POA job " + std::to_string(id) + ": " + t.error;
            tasks[id].consensus = std::move(t.consensus);
            tasks[id].msa = std::move(t.msa);
          }
        },
        [](bool) { return false; });
    // the batch API has no per-job status: a job past a limit fails the call
    // (after every other job has run)
    if (!first_error.empty()) throw SvsError(SVS_E_UNSUPPORTED, first_error);
  }
  st.wall_ms += ms_since(t_wall0);
}

}  // namespace svs
