/*
 * svscope.h — C ABI of libsvscope_hip.so, the MI355X (gfx950) engine behind the
 * SVScope localGraph hot path.  Plain pointers and sizes only; every entry
 * point returns 0 on success or a negative SVS_E* code, with a message from
 * svs_last_error() (thread-local).
 *
 * Seams replaced (reference = /root/reference/src):
 *   POA seam   spoa.poa(list_of_str, 1) -> (consensus, msa)   [pyspoa 0.2.1]
 *              call sites DataScanner.py:206,213 (window MSA) and
 *              DecisionMaker.py:160,171 (per-cluster consensus)
 *              -> svs_poa_batch + svs_poa_result_*
 *   EM seam    ReadsCluster.EMCluster(seqdatamx, initselection=1, max_C=9)
 *              ReadsCluster.py:221-277 (EM 190-209, E-step 132-155,
 *              M-step 162-188, loglik 104-122, BIC 211-219)
 *              -> svs_similarity_batch (pariwiseDistance, :52-59) and
 *                 svs_em_batch (everything after scipy's ward/fcluster init)
 *   MisScore   PairwiseCompare.AligmentScore / CalculateMisscore
 *              PairwiseCompare.py:19-30,54-64 (Bio.pairwise2 globalms, AlnFeature
 *              via SVscope.py:282) -> svs_aligment_score_batch
 */
#ifndef SVSCOPE_H
#define SVSCOPE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Bumped whenever a public struct's layout or a signature changes; a
 * binding checks svs_abi_version() against the value it was written for. */
#define SVS_ABI_VERSION 6

#define SVS_OK 0
#define SVS_E_INVALID (-1)     /* bad argument */
#define SVS_E_NOMEM (-2)       /* host or device allocation failed */
#define SVS_E_HIP (-3)         /* HIP runtime error (no device, launch failure) */
#define SVS_E_UNSUPPORTED (-4) /* parameters outside what the kernels implement */
#define SVS_E_INTERNAL (-5)    /* kernel reported an inconsistent traceback */

typedef struct svs_context svs_context;
typedef struct svs_poa_result svs_poa_result;

/* Scoring of pyspoa's poa(): defaults m=5 n=-4 g=-8 e=-6 q=-10 c=-4, alignment
 * type 1 (global NW), min_coverage=-1. Only type 1 with spoa's convex gap
 * subtype (g<e, g>q, e<c) is implemented on the GPU. */
typedef struct svs_poa_config {
  int32_t algorithm;
  int32_t m, n, g, e, q, c;
  int32_t min_coverage;
  int32_t genmsa;
} svs_poa_config;

typedef struct svs_poa_stats {
  uint64_t dp_cells;        /* sum over alignments of (|V|+1)*(L+1) */
  uint64_t alignments;      /* read-vs-graph DP jobs executed on the GPU */
  uint64_t launches;        /* kernel launches */
  uint64_t tb_bytes;        /* traceback-code bytes written (HBM) */
  uint64_t pool_bytes;      /* row-pool bytes written (H,F,O planes) */
  uint64_t h2d_bytes, d2h_bytes;
  double kernel_ms;         /* sum of per-launch durations (HIP events) */
  double host_graph_ms;     /* host graph update / export time */
  double wall_ms;
  double gpu_wait_ms;       /* host time blocked waiting for a launch's results */
  uint64_t cells_computed;  /* DP cells the kernel evaluated (64-column strip rows x 64;
                               below dp_cells when the exact pruning skips rows) */
  uint64_t prune_retries;   /* pruned alignments re-run (bound above the optimum) */
  double prep_ms;           /* device half of the row export (poa_strip_prep_kernel), HIP events */
  uint64_t prep_jobs;       /* alignments whose row tables the device completed */
  double fold_ms;           /* device-resident graphs: graph update + sort + export + table
                               completion (poa_fold.hip, poa_prep.hip) per launch, HIP events */
  uint64_t fold_jobs;       /* alignments (and first reads) folded into device-resident graphs */
  uint64_t wide_launches;   /* DP launches with 32-bit traceback codes (a graph node with more
                               than 31 in-edges) */
  /* fold_ms by kernel (HIP events between the kernels on the fold stream):
     poa_fold_update_kernel, poa_fold_sort_kernel, poa_fold_final_kernel,
     poa_dgraph_prep_kernel */
  double fold_update_ms, fold_sort_ms, fold_final_ms, fold_prep_ms;
  /* tasks whose graph block did not fit the arena while other tasks held it,
     run in a later launch instead (this slot held dual_launches until round
     4; it keeps the offsets of the fields below) */
  uint64_t deferred_tasks;
  /* device-resident POA graphs (the context's graph arena): the most bytes of
     task blocks live at once, and the HBM the arena holds (hipMalloc'ed chunks;
     never returned before svs_release) */
  uint64_t dgraph_peak_bytes, dgraph_reserved_bytes;
  /* device time during which at least one DP launch ran: the union of the
     launches' HIP-event intervals (kernel_ms sums them, so it counts twice the
     time two task groups' launches overlap on their DP streams) */
  double kernel_busy_ms;
  /* device time from the end of each DP launch to the end of its launch's
     fold chain and copies (what the group's next launch waits for) */
  double dp_to_done_ms;
} svs_poa_stats;

/* One context per host thread; owns a HIP stream and device arenas. */
int svs_init(int device_ordinal, svs_context** out);
void svs_release(svs_context* ctx);
const char* svs_last_error(void);
int svs_device_count(int* out);
int svs_abi_version(void); /* SVS_ABI_VERSION of the library */

/* Batched POA: job j aligns sequences [job_seq_start[j], job_seq_start[j+1])
 * in order (pyspoa semantics: empty sequences are skipped and produce no MSA
 * row).  Sequence s occupies seq_bytes[seq_byte_start[s] .. seq_byte_start[s+1]).
 * *out is library-allocated; free with svs_poa_result_free. */
int svs_poa_batch(svs_context* ctx, int32_t n_jobs, const int64_t* job_seq_start,
                  const int64_t* seq_byte_start, const char* seq_bytes,
                  const svs_poa_config* cfg, svs_poa_result** out);
int svs_poa_result_consensus(const svs_poa_result* r, int32_t job, const char** data, int64_t* len);
/* MSA rows are returned as one rows*cols char block (row-major). */
int svs_poa_result_msa(const svs_poa_result* r, int32_t job, int32_t* rows, int32_t* cols,
                       const char** data);
int svs_poa_result_stats(const svs_poa_result* r, svs_poa_stats* out);
void svs_poa_result_free(svs_poa_result* r);

/* ---------------------------------------------------------------- EM seam */
typedef struct svs_em_result svs_em_result;

/* One window's feature matrix: n_reads x n_feat symbols 0..4 (A,T,C,G,-;
 * DataScanner.SeqEncoder) at X + x_off, row-major; its fcluster labels for
 * K = 1..kmax-1 (kmax = min(max_c+1, n_reads)), (kmax-1) rows of n_reads int32
 * at labels + label_off (scipy fcluster(ward linkage(S), K, 'maxclust')). */
typedef struct svs_em_window {
  int32_t n_reads;
  int32_t n_feat;
  int64_t x_off;
  int64_t label_off;
} svs_em_window;

/* EMCluster(seqdatamx, initselection=1, max_C=9): n_step=20 (EM :190),
 * eps=1e-10 (CheckParam :70), seed=2023 (:42; re-seeded per window). */
typedef struct svs_em_config {
  int32_t max_c;
  int32_t n_step;
  int32_t seed;
  int32_t want_params; /* also return gamma/pi/theta of the chosen K */
  double eps;
} svs_em_config;

#define SVS_EM_K 0        /* int32[1]  chosen K (after the K=1 -> 2 rule) */
#define SVS_EM_RCLUST 1   /* int32[N]  argmax gamma (first max) */
#define SVS_EM_BIC 2      /* double[kmax-1] BICList */
#define SVS_EM_LIK 3      /* double[N] per-read loglik of the chosen K, last iteration */
#define SVS_EM_GAMMA 4    /* double[N*K] (want_params) */
#define SVS_EM_PI 5       /* double[K]   (want_params) */
#define SVS_EM_THETA 6    /* double[K*nf*5] (want_params) */
#define SVS_EM_RNG_USED 7 /* int64[1] exponentials consumed by dirichlet re-inits */

/* pariwiseDistance (ReadsCluster.py:52-59): S[i,j] = #equal columns / n_feat,
 * diagonal 1; window w's N*N block is written at S + s_off[w]. */
int svs_similarity_batch(svs_context* ctx, int32_t n_windows, const svs_em_window* wins, const uint8_t* X,
                         const int64_t* s_off, double* S);
int svs_em_batch(svs_context* ctx, int32_t n_windows, const svs_em_window* wins, const uint8_t* X,
                 const int32_t* labels, const svs_em_config* cfg, svs_em_result** out);
/* scipy linkage(S, 'ward') + fcluster(Z, K, 'maxclust') for K = 1..kmax-1,
 * kmax = min(max_c + 1, n_reads) (ReadsCluster.py:243 linkage, :94 fcluster;
 * third-party scipy 1.15 restated on the host, parity-tested against it).
 * S: n_reads x n_reads per window at S + s_off[w]; labels written at
 * labels + wins[w].label_off, (kmax-1) rows of n_reads.  Host-only: no context. */
int svs_ward_maxclust_batch(int32_t n_windows, const svs_em_window* wins, const double* S, const int64_t* s_off,
                            int32_t max_c, int32_t* labels);
/* Whole EMCluster (ReadsCluster.py:221-277) for a batch: similarity kernel ->
 * ward/maxclust initial labels on the host thread pool -> EM kernel.
 * wins[w].label_off is ignored (labels are internal). */
int svs_em_cluster_batch(svs_context* ctx, int32_t n_windows, const svs_em_window* wins, const uint8_t* X,
                         const svs_em_config* cfg, svs_em_result** out);
int svs_em_result_get(const svs_em_result* r, int32_t window, int32_t field, const void** data, int64_t* count);
/* The batch's EM kernel time (HIP events) and the windows the K-parallel
 * kernel handed to the in-order one (its speculation could not place them). */
int svs_em_result_stats(const svs_em_result* r, double* kernel_ms, int64_t* reruns);
void svs_em_result_free(svs_em_result* r);
/* Host-only: numpy legacy RandomState(seed).standard_exponential(n), bitwise. */
int svs_rng_exponential_table(uint32_t seed, int64_t n, double* out);

/* ---------------------------------------------------------------- Decision
 * The whole per-window decision (DecisionMaker.Decision, DecisionMaker.py:134-191)
 * for a batch of gated windows, pipelined on one device:
 *   window MSA POA (DataScanner.py:206/213) -> MSAFeatureSelection (:181-220,
 *   host) -> EMCluster (ReadsCluster.py:221-277, GPU, in batches on its own
 *   stream) -> cluster labelling (DecisionMaker.py:145-154, host) -> consensus
 *   POA per reported cluster (:155-176).
 * The POA stages share one continuous-batching scheduler, so consensus jobs of
 * early windows fill the GPU next to MSA jobs of later ones.  The caller does
 * the gate (:134) and formats the record (:178-190) from the returned read-id
 * indices and consensus strings. */
typedef struct svs_decision_window {
  int32_t n_seqs;      /* len(sequenceList): reference window sequence + reads */
  int32_t n_ids;       /* len(ReadIDs) */
  int64_t seq_start;   /* index of sequenceList[0] in seq_byte_start */
  int64_t flank5_off;  /* flank_5 = text[flank5_off : flank5_off + flank5_len] */
  int64_t flank3_off;
  int32_t flank5_len;
  int32_t flank3_len;
  int64_t tag_off;     /* is_tlabel[tag_off + i] = 1 iff ReadIDs[i]'s tag == Tlabel */
} svs_decision_window;

typedef struct svs_decision_config {
  int32_t readcutoff;  /* 3 */
  int32_t hcutoff;     /* 3 */
  double scutoff;      /* 0.05 */
  svs_poa_config poa;  /* poa(seqs, 1) defaults; genmsa ignored */
  svs_em_config em;    /* EMCluster defaults: max_c 9, n_step 20, seed 2023 */
  int32_t em_batch;    /* max windows per EM launch (0: 512); the first launch of a call takes half */
  int32_t reserved;
} svs_decision_config;

typedef struct svs_decision_stats {
  svs_poa_stats poa;   /* MSA + consensus POA together */
  double wall_ms, features_ms, labelling_ms, em_wall_ms, em_kernel_ms;
  int64_t msa_tasks, consensus_tasks, em_windows, em_launches;
  /* SURVEY.md §8(d) dense-equivalent EM FLOPs of the windows sent to EM:
   * per window sum over K of 41 x 2 N (5 nf) K (21 E-steps + 20 M-steps) */
  double em_flops;
  /* windows the K-parallel EM could not place its RNG draws for and reran with
   * K in order (em_kernels.hip em_select_kernel) */
  int64_t em_reruns;
} svs_decision_stats;

typedef struct svs_decision_result svs_decision_result;

/* Window status values */
#define SVS_DEC_NO_EM 0       /* seqdatamx has < 10 feature columns: default record */
#define SVS_DEC_EM 1          /* EM ran, no somatic + germline pair: default record */
#define SVS_DEC_EMOUTPUT 2    /* record with clusters, flag + "|EMOutput" */
#define SVS_DEC_INDEX_ERROR 3 /* a label row has no read id: the reference raises IndexError */
#define SVS_DEC_FAILED 4      /* the window went past an engine limit (svs_decision_result_window_error says
                                 which); the other windows of the batch are unaffected */

int svs_decision_batch(svs_context* ctx, int32_t n_windows, const svs_decision_window* wins,
                       const int64_t* seq_byte_start, const char* seq_bytes, const char* text,
                       const uint8_t* is_tlabel, const svs_decision_config* cfg, svs_decision_result** out);
/* Streaming form of svs_decision_batch: a session owns one worker thread and
 * one POA scheduler for every batch submitted to it, so the MSA jobs of batch
 * b+1 fill the GPU while batch b's EM and consensus jobs finish (no drain
 * between batches).  submit() queues a batch and returns a ticket at once; the
 * input arrays are read by the worker and must stay valid and unchanged until
 * wait() for that ticket has returned.  wait() blocks until the batch is
 * complete and returns its result (free with svs_decision_result_free); its
 * stats are the session's cumulative statistics at the batch's completion.
 * Batches complete in any order.  While a session is open the context must not
 * be used for other calls.  close() finishes every submitted batch, joins the
 * worker and frees the session; it returns the worker's error, if any (after
 * an error every submit/wait of the session fails with it).
 * Replaces the Pool.imap_unordered fan-out of localGraph_npz (SVscope.py:220-233)
 * over TDscope_npz / Decision. */
typedef struct svs_decision_session svs_decision_session;
int svs_decision_session_open(svs_context* ctx, const svs_decision_config* cfg, svs_decision_session** out);
int svs_decision_session_submit(svs_decision_session* s, int32_t n_windows, const svs_decision_window* wins,
                                const int64_t* seq_byte_start, const char* seq_bytes, const char* text,
                                const uint8_t* is_tlabel, int64_t* ticket);
int svs_decision_session_wait(svs_decision_session* s, int64_t ticket, svs_decision_result** out);
/* cumulative statistics of the session as of its last completed batch */
int svs_decision_session_stats(svs_decision_session* s, svs_decision_stats* out);
int svs_decision_session_close(svs_decision_session* s);

int svs_decision_result_window(const svs_decision_result* r, int32_t window, int32_t* status, int32_t* K,
                               int32_t* n_som, int32_t* n_germ);
/* the reason of an SVS_DEC_FAILED window (empty string otherwise); owned by r */
int svs_decision_result_window_error(const svs_decision_result* r, int32_t window, const char** msg);
/* cluster c of a window: somatic clusters first (c < n_som), then germline;
 * ids = ReadIDs indices of the cluster's reads, cons = its consensus ("-" when
 * every read of the cluster is empty). */
int svs_decision_result_cluster(const svs_decision_result* r, int32_t window, int32_t cluster,
                                const int32_t** ids, int32_t* n_ids, const char** cons, int64_t* cons_len);
int svs_decision_result_stats(const svs_decision_result* r, svs_decision_stats* out);
void svs_decision_result_free(svs_decision_result* r);

/* Host-only MSAFeatureSelection after the MSA (DataScanner.py:181-220) for
 * tests: msa = n_rows x width bytes; read_lens = len(sequenceList[1:]).
 * Writes seqdatamx (rows x n_feat) into feat (capacity feat_cap bytes) and the
 * returned readIDList as ReadIDs indices into id_map (capacity id_cap).
 * On SVS_E_INVALID with *rows >= 0 the capacities were too small. */
int svs_msa_features(int32_t n_rows, int32_t width, const char* msa, const char* flank5, int32_t flank5_len,
                     const char* flank3, int32_t flank3_len, int32_t n_reads, const int32_t* read_lens,
                     int32_t n_ids, int32_t hcutoff, double scutoff, int32_t* rows, int32_t* n_feat,
                     uint8_t* feat, int64_t feat_cap, int32_t* id_map, int32_t* n_map, int64_t id_cap);

/* ---------------------------------------------------------------- MisScore
 * PairwiseCompare.AligmentScore (PairwiseCompare.py:19-30) for many pairs:
 *   alignment = Bio.pairwise2.align.globalms(som, ger, 1, 0, -1, -1)[0]
 *   alig      = format_alignment(*alignment).split('\n')[1][cutoff:len-cutoff]
 *   MisScore  = len(alig) - alig.count('|')
 * Pair p aligns sequence pair_a[p] (SomConsensus) against pair_b[p]
 * (GerConsensus); sequence s is seq_bytes[seq_byte_start[s] .. seq_byte_start[s+1]).
 * Writes out_len[p] = len(alig), out_match[p] = count('|') and out_status[p]:
 * SVS_MS_OK, or SVS_MS_EMPTY when a sequence is empty (pairwise2 returns no
 * alignment and the reference's [0] raises IndexError).  cutoff 0..64.
 * Replaces the per-pair Biopython call made by CalculateMisscore
 * (PairwiseCompare.py:54-64) over the rows of MisScorePipe (:76-86). */
#define SVS_MS_OK 0
#define SVS_MS_EMPTY 4

typedef struct svs_misscore_stats {
  uint64_t pairs;       /* pairs aligned on the GPU (non-empty) */
  uint64_t dp_cells;    /* sum of len(som) * len(ger) */
  uint64_t nib_bytes;   /* 4-bit score-difference bytes written (HBM) */
  uint64_t launches;
  uint64_t tb_steps;    /* traceback DFS steps */
  double fill_ms;       /* DP kernel time (HIP events) */
  double traceback_ms;  /* traceback kernel time */
  double wall_ms;
} svs_misscore_stats;

int svs_aligment_score_batch(svs_context* ctx, int32_t n_pairs, const int32_t* pair_a, const int32_t* pair_b,
                             int32_t n_seqs, const int64_t* seq_byte_start, const char* seq_bytes, int32_t cutoff,
                             int32_t* out_len, int32_t* out_match, int32_t* out_status, svs_misscore_stats* stats);

/* Wave-primitive self test (GPU tests): per 64-lane wave, inclusive prefix max
 * and shift-right-by-one (lane 0 <- -7). */
int svs_wave_selftest(svs_context* ctx, const int32_t* in, int32_t* scan, int32_t* shift,
                      int32_t n_waves);

#ifdef __cplusplus
}
#endif
#endif /* SVSCOPE_H */
