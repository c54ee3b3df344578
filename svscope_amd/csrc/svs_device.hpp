// Device-side job descriptors shared by the host engine and the HIP kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace svs {

struct PoaScore {
  int32_t m, n, g, e, q, c;
};

// One read-vs-graph NW alignment (one workgroup of the strip kernel).  The
// row tables are device pointers: into the launch's staging copy (host-built
// graphs) or into the task's graph block (device-resident graphs,
// poa_dgraph.hpp); the outputs are element offsets into the launch buffers.
struct PoaJob {
  const uint32_t* rec;    // row records, kRecWords per row (export_strip_rows)
  const uint32_t* pstart; // n_rows + 1 CSR offsets of the in-edge rows, rank order
  const uint32_t* pred;   // 1-based in-edge rows (bit 31: export_strip_lite's last-read flag)
  const uint32_t* pslot;  // pool slots of the in-edges
  const int32_t* col0;    // H, F, O of DP column 0 per row
  const uint8_t* seq;     // the read; seq[-1] is a zero pad byte, region ls + 64 bytes
  const uint32_t* info;   // prep jobs: per-row words (export_strip_lite)
  uint64_t tb_off;        // uint16 traceback codes, rows 1..n_rows, stride ls
  uint64_t bnd_off;       // int32 strip-boundary carries
  uint64_t pool_off;      // int32 global row pool (pools that do not fit LDS)
  uint64_t aln_off;       // output pairs (2 x int32), capacity n_rows + len + 1
  uint32_t n_rows;        // graph nodes
  uint32_t len;           // read length
  uint32_t ls;            // row stride (>= len + 1, multiple of 64)
  uint32_t n_slots;       // pool slots (slot 0 = virtual row 0)
  int32_t lb;             // pruning bound (kNoPrune = off), see poa_strip.hip
  uint32_t prep;          // bit 0: rec, pslot and col0 come from poa_strip_prep_kernel;
                          // bits 1..: the first pool slot
};

// PoaJob::lb value that turns the strip kernel's exact pruning off.
constexpr int32_t kNoPrune = INT32_MIN;
// The same for a job in a launch of the pruning variant: a bound below every
// real score (and above the VNEG of a skipped input), so no cell is pruned.
constexpr int32_t kPruneAll = INT32_MIN / 4;
// aln_len[job] for a pruned job whose best sink score fell below its bound
// (the bound was not a lower bound of the optimum: run it again unpruned).
constexpr int32_t kPruneRetry = -2;

struct PoaLaunch {
  const PoaJob* jobs;
  int n_jobs;
  PoaScore score;
  void* tb;              // traceback codes: uint16 (wide: uint32) per cell
  int32_t* bnd;          // strip-boundary carries
  int32_t* pool;         // global row pools
  int32_t* aln;
  int32_t* aln_len;      // per job: path length; also [n_jobs + job] best sink score
                         // and [2 n_jobs + job] strip rows computed
  int waves_per_job;     // strip-pipeline waves per job: 1, 2, 4, 8 (16 with the pool in LDS)
  uint32_t lds_slots;    // pool slots per wave held in LDS (max n_slots of the launch)
  bool prune;            // some job has a pruning bound: the pruning kernel variant
  bool wide;             // some row has more than 31 in-edges: 32-bit codes (TbFmt, poa_wave.hpp)
};

// One block copy of launch_scatter_copy (bytes a multiple of 64, both ends
// 64-byte aligned).
struct CopyDesc {
  const char* src;
  uint8_t* dst;
  uint64_t bytes;
};
hipError_t launch_scatter_copy(const CopyDesc* d, int n, hipStream_t stream);

// In-edges per graph node the traceback codes can name: 31 with 16-bit codes,
// 4094 with 32-bit ones (launches with such a node; TbFmt, poa_wave.hpp).
constexpr uint32_t kMaxInEdgesNarrow = 31, kMaxInEdges = 4094;

// Row stride of a strip job: len + 1 rounded up to whole 64-column strips.
inline uint32_t strip_ls(uint32_t len) { return (len + 1 + 63) / 64 * 64; }

// Strip-major kernel: LDS bytes per pool slot (65 int32 H incl. the boundary
// column + 64 packed uint16 F/O distances), and the largest pool kept in LDS.
constexpr uint32_t kStripSlotBytes = 65 * 4 + 64 * 2;
constexpr uint32_t kStripMaxLdsSlots = 80;
// LDS a strip workgroup's pools may take (160 KiB per CU on gfx950, less the
// kernel's own few static words)
constexpr uint64_t kStripLdsBytes = 160 * 1024 - 256;
// Strip carries (16 B per row) are published to the next strip's wave in
// whole lines of this many rows (poa_strip.hip wait_vm_stores); a job's carry
// region starts at a multiple of kCarryAlignInts int32 (256 B).
constexpr uint32_t kCarryLineRows = 8;
constexpr uint64_t kCarryAlignInts = 64;

hipError_t launch_poa_strip(const PoaLaunch& a, hipStream_t stream);
// Device half of the strip row export (poa_prep.hip) for the jobs with
// PoaJob::prep bit 0.
// rows of a prep job (its path lengths for the pruning bound are kept in 16
// bits, clamped: exact for reads shorter than 65535 bases, the engine prunes
// no longer read)
constexpr uint32_t kStripPrepMaxRows = 1u << 24;
constexpr uint32_t kPruneMaxReadLen = 65534;
constexpr uint32_t kStripPrepMaxSlots = 1024;  // pool slots of a prep job (free list: a VGPR, then LDS)
size_t strip_prep_scratch_words(uint32_t n_rows);  // after the job's in-edge slots (rounded to 4)
hipError_t launch_poa_strip_prep(const PoaJob* jobs, int n_jobs, const PoaScore& score, uint32_t max_rows,
                                 hipStream_t stream);
// Device-resident graphs (poa_fold.hip, poa_prep.hip; poa_dgraph.hpp).
struct FoldJob;
// update + sort (+ the final kernel when final_lds_words > 0: some job of the
// launch has kFoldFinal); marks (optional, 3 events) are recorded after the
// update, the sort and the final kernel
hipError_t launch_poa_fold(const FoldJob* jobs, int n_jobs, uint32_t lds_words, uint32_t final_lds_words,
                           hipStream_t stream, const hipEvent_t* marks = nullptr);
// the final kernel alone (after the sort, on a stream of its own), one
// workgroup per final fold: jobs[idx[k]], k < n_final
hipError_t launch_poa_final(const FoldJob* jobs, const uint32_t* idx, int n_final, uint32_t final_lds_words,
                            hipStream_t stream);
hipError_t launch_dgraph_prep(const FoldJob* jobs, int n_jobs, const PoaScore& score, hipStream_t stream);
// A task's graph moved into a larger block (capacities cv1 >= cv0, ce1 >= ce0);
// every move of a launch in one kernel
struct MoveDesc {
  const uint8_t* src;
  uint8_t* dst;
  uint32_t cv0, ce0, cv1, ce1, V, E, par, pad;
};
hipError_t launch_dgraph_moves(const MoveDesc* d, int n, hipStream_t stream);
hipError_t launch_wave_selftest(const int32_t* in, int32_t* scan, int32_t* shift, int n_waves,
                                hipStream_t stream);

}  // namespace svs
