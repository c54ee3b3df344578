// Internal declarations shared by the engine translation units.
#pragma once
#include <exception>
#include <functional>
#include <string>
#include <vector>

#include "../../include/svscope.h"
#include "features.hpp"
#include "poa_dgraph.hpp"
#include "poa_graph.hpp"

// EM results of one batch (opaque to ABI users).
struct svs_em_result {
  struct Win {
    int32_t K = 0;
    int64_t rng_used = 0;
    std::vector<int32_t> rclust;
    std::vector<double> bic, lik, gamma, pi, theta;
  };
  std::vector<Win> w;
  double kernel_ms = 0.0;
  int64_t em_reruns = 0;  // windows the K-parallel path handed to the in-order kernel
};

// Decision pipeline results (opaque to ABI users).
struct svs_decision_result {
  struct Win {
    int32_t status = 0, K = 0;
    std::vector<svs::ClusterPlan> som, germ;
    std::string error;  // SVS_DEC_FAILED: which limit
  };
  std::vector<Win> w;
  svs_decision_stats st{};
};

namespace svs {

struct PoaTask {
  std::vector<std::string> seqs;
  bool genmsa = false;  // also produce the MSA rows when the task completes
  uint32_t tag = 0;     // caller's bookkeeping (window / cluster id)
  uint32_t prio = 0;    // queue order: lower first (a session's batch number), then longest remaining
  size_t next = 0;      // index of the next sequence to align
  PoaGraph graph;
  RowTables rows;       // exported row tables of the current step (capacity reused across steps)
  // exact pruning of the strip kernel (svs_poa_engine.cpp: prune_bound)
  double rate = 0.0;      // best score / read length of the last alignment that needed no retry
  bool have_rate = false;
  bool retry = false;     // the current sequence's pruned run missed its bound: run it again (prune_bound)
  uint8_t prepped = 0;    // next step already readied after the fold: 1 export done, 2 complete
  // where the strip tables of the next step are: 1 in rows' vectors, 2 in a
  // block of the group's staging buffer (blk_off, valid while the buffer's
  // generation is still blk_gen)
  uint8_t rows_at = 0;
  uint32_t blk_gen = 0;
  uint64_t blk_off = 0;
  uint8_t n_retries = 0;     // retried alignments of this task
  uint8_t read_retries = 0;  // retries of the current sequence
  uint32_t last_rows = 0;    // strip rows (64 columns) the last alignment computed

  // device-resident graph (poa_dgraph.hpp, the default; SVS_POA_HOST_GRAPH=1
  // keeps the graph in `graph` on the host instead)
  DGraphRef dg;
  uint8_t* d_static = nullptr;    // the task's reads (padded) + path offsets + node paths
  size_t static_bytes = 0;
  size_t static_po = 0;           // path offsets' byte offset in d_static
  bool static_up = false;         // d_static reserved, its image not yet uploaded
  size_t dg_bytes = 0;            // the graph block's allocation size
  // a larger graph block reserved for this launch's fold (reserve_blocks),
  // the current one moved into it by the launch
  uint8_t* grow_blk = nullptr;
  uint32_t grow_cv = 0, grow_ce = 0;
  size_t grow_bytes = 0;
  std::vector<uint64_t> seq_at;   // byte offset of read k in d_static (its first base)
  uint32_t* d_path_off = nullptr; // non-empty reads + 1 offsets into d_paths
  uint32_t* d_paths = nullptr;
  uint32_t n_paths = 0;           // non-empty reads folded so far
  uint32_t last_nonempty = 0;     // index of the last non-empty read + 1
  uint32_t n_slots_next = 0, max_preds_next = 0;  // the exported tables of the next read
  bool tables_ok = false;         // rec / pslot / col0 / lite tables valid for seqs[next]

  std::string consensus;
  std::vector<std::string> msa;
  // decision pipeline: the window's MSAFeatureSelection on the device (device
  // graphs, FoldJob kFoldFeat) instead of the MSA rows; n_feat >= 0 on
  // completion when it ran, with seqdatamx in feat
  bool features = false;
  DeviceFeatureParams feat_params;
  int32_t n_feat = -1;
  std::vector<uint8_t> feat;
  // set when the task went past an engine limit (a per-task failure: the task
  // completes with no consensus / MSA, the others go on)
  std::string error;
};

// Continuous-batching POA driver.  Every launch aligns the next sequence of
// each active task of one task group; two groups alternate on the in-order
// POA stream so the host folds one group's alignments while the GPU runs the
// other's.  Finished tasks leave their group after every step and queued tasks
// take their place, so the GPU stays full while tasks of different lengths
// (window MSAs, cluster consensus jobs) come and go.
class PoaScheduler {
 public:
  using DoneFn = std::function<void(const std::vector<uint32_t>&)>;
  // poll(block): called between launches; may add() tasks.  Returns true while
  // outside work may still add tasks; with block=true it may wait for it.
  using PollFn = std::function<bool(bool)>;
  PoaScheduler(svs_context* ctx, const svs_poa_config& cfg, svs_poa_stats& st);
  ~PoaScheduler();
  // Queues a task; ids of finished, released tasks are reused.
  uint32_t add(PoaTask&& t);
  PoaTask& task(uint32_t id);
  double host_ms() const;  // host graph work so far (fold, export, pack)
  // Runs until no task is queued or active and poll() reports no outside work.
  // done(ids) receives each batch of completed tasks (consensus / msa filled);
  // afterwards the scheduler drops their graphs.
  void run(const DoneFn& done, const PollFn& poll);

 private:
  struct Impl;
  Impl* impl_;
};

void check_poa_config(const svs_poa_config& c);
void run_poa_tasks(svs_context* ctx, std::vector<PoaTask>& tasks, const svs_poa_config& cfg,
                   svs_poa_stats& st);

int em_validate(int32_t n_windows, const svs_em_window* wins, const uint8_t* X, std::string* err);
void run_similarity(svs_context* ctx, int32_t n, const svs_em_window* wins, const uint8_t* X, double* S_out,
                    const int64_t* s_off);
svs_em_result* run_em(svs_context* ctx, int32_t n, const svs_em_window* wins, const uint8_t* X,
                      const int32_t* labels, const svs_em_config& cfg);
class ThreadPool;
// pool == nullptr runs the host ward/maxclust step on the calling thread (used
// by the pipeline's EM worker, which must not share the driver's pool).
svs_em_result* run_em_cluster(svs_context* ctx, int32_t n, const svs_em_window* wins, const uint8_t* X,
                              const svs_em_config& cfg, ThreadPool* pool);

void run_misscore(svs_context* ctx, int32_t n_pairs, const int32_t* pair_a, const int32_t* pair_b,
                  const int64_t* seq_byte_start, const char* seq_bytes, int32_t cutoff, int32_t* out_len,
                  int32_t* out_match, int32_t* out_status, svs_misscore_stats* st);


svs_decision_result* run_decision(svs_context* ctx, int32_t n, const svs_decision_window* wins,
                                  const int64_t* seq_byte_start, const char* seq_bytes, const char* text,
                                  const uint8_t* is_tlabel, const svs_decision_config& cfg);

svs_decision_session* open_decision_session(svs_context* ctx, const svs_decision_config& cfg);
int64_t submit_decision_batch(svs_decision_session* s, int32_t n, const svs_decision_window* wins,
                              const int64_t* seq_byte_start, const char* seq_bytes, const char* text,
                              const uint8_t* is_tlabel);
svs_decision_result* wait_decision_batch(svs_decision_session* s, int64_t ticket);
void session_stats(svs_decision_session* s, svs_decision_stats* out);
std::exception_ptr close_decision_session(svs_decision_session* s);

}  // namespace svs
