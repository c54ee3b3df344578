// Device-resident POA graphs (host and device declarations).
//
// Every POA task (one pyspoa `poa(seqs, 1)` call of the reference: a window
// MSA at DataScanner.py:206,213 or a cluster consensus at
// DecisionMaker.py:160,171) keeps its partial-order graph in one block of HBM
// for its whole life.  After each alignment the device folds the traceback
// into the graph (spoa Graph::AddAlignment: new nodes, edges, aligned-node
// groups), re-sorts it (spoa's DFS topological sort with aligned groups kept
// contiguous), and exports the next alignment's rank-ordered row tables; when
// the task's last sequence is in, it emits the heaviest-bundle consensus and
// the MSA rows.  Only job descriptors go up and only per-job counters (and the
// finished tasks' consensus / MSA rows) come back.  Kernels: poa_fold.hip.
//
// Block layout (struct of arrays, capacities cv nodes / ce edges; every array
// 64-B aligned):
//   base     u8   [cv]       node letter
//   al       u32  [cv][4]    aligned list: [0] = count (<= 3), [1..3] members
//                            in spoa's aligned_nodes order
//   in/out   CSR by node id, two buffers (the fold writes the other one):
//            off u32[cv+1], nbr u32[ce] (tail / head), eid u32[ce]
//   ew       u32  [ce]       edge weight / 2 (spoa adds 2 per sequence: 1 + 1)
//   nin,nout u32  [cv][2]    this fold's new in / out edge of a node (eid, nbr)
//   nrec     u32  [cv][8]    the sort's node record: in-edge CSR start,
//                            in-degree | aligned count << 24, aligned list,
//                            first three in-edge tails (one scalar load)
//   r2n, n2r u32  [cv]       rank order
//   col      u32  [cv]       MSA column of a node (rank group index)
//   last     u32  [cv]       export scratch: last pool reader of a row
//   lite tables of the next alignment (PoaGraph::export_strip_lite's):
//            pstart u32[cv+1], pred u32[ce] (bit 31: last pool read), info u32[cv]
//   prep outputs (poa_prep.hip): col0 i32[3 cv], rec u32[4 cv],
//            pslot u32[ce + 4] + scratch u32[3 (cv + 4)]
//   stk      u32  [ce + 2 cv + 64]  the sort's DFS stack beyond its LDS part
//   chg      u32  [2 ceil(cv / 64)]  bit plane by node id: the fold changed the
//                            node's in-edge or aligned list (update kernel)
//   seg      u32  [2][ceil(cv / 32) + 2]  bit plane by rank: a DFS root's
//                            segment of the rank order starts here (the sort
//                            of a fold reads seg[par] and writes seg[1 - par])
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

namespace svs {

struct DGraphLayout {
  size_t base, al, in_off[2], in_nbr[2], in_eid[2], out_off[2], out_nbr[2], out_eid[2], ew, nin, nout;
  size_t nrec, r2n, n2r, col, last, pstart, pred, info, col0, rec, pslot, stk, chg, seg[2], bytes;
};

__host__ __device__ inline DGraphLayout dgraph_layout(uint32_t cv, uint32_t ce) {
  DGraphLayout L{};
  size_t o = 0;
  auto take = [&](size_t bytes) {
    const size_t at = o;
    o = (o + bytes + 63) / 64 * 64;
    return at;
  };
  const size_t V = cv, E = ce;
  L.base = take(V);
  L.al = take(16 * V);
  for (int b = 0; b < 2; ++b) {
    L.in_off[b] = take(4 * (V + 1));
    L.in_nbr[b] = take(4 * E);
    L.in_eid[b] = take(4 * E);
    L.out_off[b] = take(4 * (V + 1));
    L.out_nbr[b] = take(4 * E);
    L.out_eid[b] = take(4 * E);
  }
  L.ew = take(4 * E);
  L.nin = take(8 * V);
  L.nout = take(8 * V);
  L.nrec = take(32 * V);
  L.r2n = take(4 * V);
  L.n2r = take(4 * V);
  L.col = take(4 * V);
  L.last = take(4 * V);
  L.pstart = take(4 * (V + 1));
  L.pred = take(4 * E);
  L.info = take(4 * V);
  L.col0 = take(12 * V);
  L.rec = take(16 * V);
  L.pslot = take(4 * (E + 4) + 12 * (V + 4));
  L.stk = take(4 * (E + 2 * V + 64));
  L.chg = take(8 * ((V + 63) / 64));
  for (int b = 0; b < 2; ++b) L.seg[b] = take(4 * ((V + 31) / 32 + 2));
  L.bytes = o;
  return L;
}

// One task's graph on the device: its block and the counts the host tracks.
struct DGraphRef {
  uint8_t* blk = nullptr;
  uint32_t cv = 0, ce = 0;  // capacities of the block
  uint32_t V = 0, E = 0;    // nodes / edges after the last fold
  uint32_t par = 0;         // CSR buffer holding the current graph
  uint32_t ncol = 0;        // MSA columns after the last sort
};

// Status values of a fold (FoldResult::status).
constexpr int32_t kFoldOk = 0;
constexpr int32_t kFoldSkipped = 1;       // the alignment was a pruning retry: graph unchanged
constexpr int32_t kFoldErrCapacity = -1;  // block too small (host sized it: internal error)
constexpr int32_t kFoldErrPath = -2;      // a node twice on one sequence's path / no sequence consumed
constexpr int32_t kFoldErrAligned = -3;   // an aligned group of more than 4 nodes (letters outside ACGT)
constexpr int32_t kFoldErrAln = -4;       // the DP traceback reported an inconsistent path
constexpr int32_t kFoldErrStack = -5;     // DFS stack beyond its spill area
constexpr int32_t kFoldNotRun = -100;     // the host's initial value: no fold kernel wrote the result

// What the host reads back per fold job.
struct FoldResult {
  int32_t status;
  uint32_t V, E, n_slots, max_preds, ncol, pad0, pad1;
  // phase times in 10 ns ticks (s_memrealtime): update kernel, sort, export,
  // consensus + MSA rows (SVS_POA_FOLD_TIMES prints their totals)
  uint32_t t_upd, t_sort, t_exp, t_fin;
  uint32_t n_exam, n_roots;  // DFS examinations and DFS starts of the sort
  uint32_t prof[4];          // SVS_FOLD_PROF builds: DFS phase clocks / 1024
};

// One fold job: fold the job's alignment (or, with kFoldChain, the whole
// sequence as a fresh chain) into the task's graph, sort it, and export the
// next step's lite tables (kFoldExport) and/or emit consensus + MSA rows
// (kFoldFinal).
constexpr uint32_t kFoldChain = 1;   // the sequence lands on an empty graph (no alignment)
constexpr uint32_t kFoldExport = 2;  // a next sequence follows: export its lite tables
constexpr uint32_t kFoldFinal = 4;   // the task is complete: consensus (+ MSA rows with kFoldMsa)
constexpr uint32_t kFoldMsa = 8;
// With kFoldFinal | kFoldMsa: the window's MSAFeatureSelection on the device
// (poa_fold_final_kernel, DataScanner.py:146-179,195-219): seqdatamx goes to
// feat_out, the MSA rows stay in device scratch
constexpr uint32_t kFoldFeat = 16;
// FoldJob::f5_take / f3_take beyond a column count: every row-0 column of its
// end (the flank did not match), or the empty-flank rule of CallMargin
constexpr int32_t kTakeAll = -1, kTakeEmptyFlank = -2;

struct FoldJob {
  uint8_t* blk;
  uint32_t cv, ce;
  uint32_t V, E;            // graph before this fold
  uint32_t par;             // CSR buffer of the graph before this fold (the fold writes 1 - par)
  uint32_t flags;
  const uint8_t* seq;       // the sequence being added (zero pad byte at seq[-1])
  uint32_t len;
  uint32_t n_paths;         // sequences already in the graph (paths[0 .. n_paths-1])
  uint32_t* paths;          // per non-empty sequence of the task: its node path (offsets below)
  const uint32_t* path_off; // path_off[k]: start of sequence k's path in paths
  const int32_t* aln;       // traceback pairs (reversed), from the DP launch
  const int32_t* aln_status;  // the DP job's aln_len entry (pair count / kPruneRetry / < 0)
  FoldResult* result;
  // kFoldFinal outputs (device buffers the host copies back)
  char* cons_out;           // consensus, <= V + len bytes
  char* msa_out;            // n_paths + 1 rows of msa_stride bytes
  uint32_t msa_stride;
  uint32_t pad;
  // kFoldFeat: seqdatamx, (n_paths + extra) rows x n_feat symbols 0..4, into
  // host-mapped pinned memory (FoldResult::pad1 = n_feat)
  uint8_t* feat_out;
  int32_t f5_take, f3_take;  // CallMargin: row-0 columns kept from the start / the end (>= 0), or kTake*
  uint32_t extra;            // all-gap rows after the MSA rows (the full-DEL read quirk, DataScanner.py:204)
  uint32_t cut;              // FindNonSameSite: keep a column whose second-largest count is >= cut
};

}  // namespace svs
