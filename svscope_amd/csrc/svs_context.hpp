// Host-side runtime of libsvscope_hip: context, device arenas, pinned staging,
// a small fork-join thread pool for per-window graph work.
#pragma once
#include <hip/hip_runtime.h>

#include "threadpool.hpp"

#include <algorithm>
#include <atomic>
#include <cstring>
#include <memory>

#include <cstdint>
#include <stdexcept>
#include <string>
#include <vector>

namespace svs {

struct SvsError : std::runtime_error {
  int code;
  SvsError(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

#define SVS_HIP(x)                                                                    \
  do {                                                                                \
    hipError_t _e = (x);                                                              \
    if (_e != hipSuccess)                                                             \
      throw ::svs::SvsError(-3, std::string(#x) + ": " + hipGetErrorString(_e));      \
  } while (0)

// Growable device buffer (never shrinks; contents not preserved on growth).
// Growth is geometric (at least doubling), and `hint` (e.g. the launch budget)
// is tried first.  hipFree waits for the whole device, so a buffer that
// regrows during a run would stall the pipeline (a 4-s stall in a traced bench
// run, profiles/r02_v11; host pack phases of 20-60 ms behind the other group's
// DP kernel in round 4, profiles/r04_g8): the old buffer is retired instead
// and freed with the buffer (release), when the device is idle anyway.
// Retired buffers of geometric growth add at most the final size again; a
// buffer of 1 GiB or more (the traceback and carry buffers, sized once from
// the budget) is freed at once instead, so that its rare regrow cannot hold
// twice its size.
struct DeviceBuf {
  void* ptr = nullptr;
  size_t cap = 0;
  std::vector<void*> retired;
  void ensure(size_t bytes, size_t hint = 0) {
    if (bytes <= cap) return;
    if (ptr) {
      if (cap >= (size_t(1) << 30)) SVS_HIP(hipFree(ptr));
      else retired.push_back(ptr);
    }
    ptr = nullptr;
    const size_t grown = std::max(bytes + bytes / 4 + 4096, 2 * cap);
    cap = 0;
    size_t want = std::max(grown, hint);
    if (want != grown && hipMalloc(&ptr, want) != hipSuccess) {
      (void)hipGetLastError();
      ptr = nullptr;
      want = grown;
    }
    if (!ptr && hipMalloc(&ptr, want) != hipSuccess) {
      (void)hipGetLastError();
      want = bytes;
      if (hipMalloc(&ptr, want) != hipSuccess) {
        (void)hipGetLastError();
        ptr = nullptr;
        throw SvsError(-2, "hipMalloc failed for " + std::to_string(bytes) + " bytes");
      }
    }
    cap = want;
  }
  template <class T> T* as() const { return static_cast<T*>(ptr); }
  void release() {
    if (ptr) (void)hipFree(ptr);
    for (void* r : retired) (void)hipFree(r);
    retired.clear();
    ptr = nullptr;
    cap = 0;
  }
};

// Growable pinned host buffer; a regrow retires the old buffer like DeviceBuf
// (hipHostFree synchronises too).
struct PinnedBuf {
  void* ptr = nullptr;
  size_t cap = 0;
  unsigned flags = hipHostMallocDefault;  // hipHostMallocMapped: kernels write it (hipHostGetDevicePointer)
  std::vector<void*> retired;
  void ensure(size_t bytes) {
    if (bytes <= cap) return;
    if (ptr) {
      if (cap >= (size_t(256) << 20)) SVS_HIP(hipHostFree(ptr));
      else retired.push_back(ptr);
    }
    ptr = nullptr;
    const size_t want = std::max(bytes + bytes / 4 + 4096, 2 * cap);  // geometric: few regrows
    cap = 0;
    SVS_HIP(hipHostMalloc(&ptr, want, flags));
    cap = want;
  }
  // grows to at least `bytes`, keeping the first `keep` bytes
  void grow_keep(size_t bytes, size_t keep) {
    if (bytes <= cap) return;
    void* old = ptr;
    const size_t want = std::max(bytes + bytes / 4 + 4096, 2 * cap);
    void* p = nullptr;
    SVS_HIP(hipHostMalloc(&p, want, hipHostMallocDefault));
    if (old && keep) std::memcpy(p, old, std::min(keep, cap));
    // as in ensure(): a buffer of 256 MiB or more is freed at once (hipHostFree
    // waits for the device), so that regrows never hold twice the peak
    if (old) {
      if (cap >= (size_t(256) << 20)) SVS_HIP(hipHostFree(old));
      else retired.push_back(old);
    }
    ptr = p;
    cap = want;
  }
  template <class T> T* as() const { return static_cast<T*>(ptr); }
  void release() {
    if (ptr) (void)hipHostFree(ptr);
    for (void* r : retired) (void)hipHostFree(r);
    retired.clear();
    ptr = nullptr;
    cap = 0;
  }
};

// Device + pinned buffers for one in-flight POA launch of a task group.
// Kernels go to the shared in-order POA stream (groups alternate on the GPU);
// the group's own copy stream carries its H2D tables and D2H alignments, so
// they overlap the other group's kernel.
struct PoaArena {
  DeviceBuf d_in, d_tb, d_pool, d_aln, d_alen;
  PinnedBuf h_in, h_aln, h_alen;
  // device-resident graphs: the launch's job / fold descriptors and fold
  // results, and the finished tasks' consensus + MSA rows
  DeviceBuf d_desc, d_fin;
  PinnedBuf h_desc, h_fin;
  PinnedBuf h_feat;  // window seqdatamx written by the final fold kernel (zero-copy)
  hipStream_t stream = nullptr;       // kernel stream (shared by both groups)
  hipStream_t copy_stream = nullptr;  // this group's copies
  hipEvent_t ev0 = nullptr, ev1 = nullptr, done = nullptr, h2d = nullptr;
  hipEvent_t ev_end = nullptr;  // timed twin of done (device-resident graphs)
  hipEvent_t evp = nullptr, evp1 = nullptr;  // around the launch's poa_strip_prep_kernel
  hipEvent_t evf0 = nullptr, evf1 = nullptr;  // around the launch's fold kernels (device-resident graphs)
  // after the update, sort and final fold kernels: of the folds after the DP
  // kernel (evk) and of the new tasks' chains before it (evpk)
  hipEvent_t evk[3] = {nullptr, nullptr, nullptr}, evpk[3] = {nullptr, nullptr, nullptr};
  // the final kernel on a stream of its own beside the table completion,
  // forked after the sort, joined before the copies
  hipStream_t fin_stream = nullptr;
  hipEvent_t ev_sorted = nullptr, ev_fin0 = nullptr, ev_fin1 = nullptr;
  // Staging of the next launch's strip tables in h_in: the fold exports each
  // job's tables straight into a block claimed with an atomic bump (st_cur), so
  // packing the launch copies nothing.  A new generation (st_gen) starts when
  // the group's previous launch is done; st_peak = largest staging used so far.
  std::atomic<size_t> st_cur{0};
  uint32_t st_gen = 1;
  size_t st_peak = 0;
  // Kernels of both groups alternate on the shared stream s; the group's
  // copies and (device-resident graphs) its fold kernels go to its copy
  // stream, at the highest stream priority, so that as the other group's DP
  // workgroups finish, the fold's workgroups are dispatched first and the
  // group's next launch is ready when the DP stream gets to it.
  PoaArena(int device, hipStream_t s) : stream(s) {
    SVS_HIP(hipSetDevice(device));
    h_feat.flags = hipHostMallocMapped;
    int least = 0, greatest = 0;
    SVS_HIP(hipDeviceGetStreamPriorityRange(&least, &greatest));
    SVS_HIP(hipStreamCreateWithPriority(&copy_stream, hipStreamNonBlocking, greatest));
    SVS_HIP(hipStreamCreateWithPriority(&fin_stream, hipStreamNonBlocking, greatest));
    SVS_HIP(hipEventCreateWithFlags(&ev_sorted, hipEventDisableTiming));
    SVS_HIP(hipEventCreate(&ev_fin0));
    SVS_HIP(hipEventCreate(&ev_fin1));
    SVS_HIP(hipEventCreate(&ev0));
    SVS_HIP(hipEventCreate(&ev1));
    SVS_HIP(hipEventCreate(&evp));
    SVS_HIP(hipEventCreate(&evp1));
    SVS_HIP(hipEventCreate(&evf0));
    SVS_HIP(hipEventCreate(&evf1));
    for (int k = 0; k < 3; ++k) {
      SVS_HIP(hipEventCreate(&evk[k]));
      SVS_HIP(hipEventCreate(&evpk[k]));
    }
    SVS_HIP(hipEventCreateWithFlags(&done, hipEventDisableTiming));
    SVS_HIP(hipEventCreate(&ev_end));
    SVS_HIP(hipEventCreateWithFlags(&h2d, hipEventDisableTiming));
  }
  ~PoaArena() {
    if (stream) (void)hipStreamSynchronize(stream);
    if (copy_stream) (void)hipStreamSynchronize(copy_stream);
    if (fin_stream) (void)hipStreamSynchronize(fin_stream);
    for (DeviceBuf* b : {&d_in, &d_tb, &d_pool, &d_aln, &d_alen, &d_desc, &d_fin}) b->release();
    for (PinnedBuf* b : {&h_in, &h_aln, &h_alen, &h_desc, &h_fin, &h_feat}) b->release();
    if (ev0) (void)hipEventDestroy(ev0);
    if (ev1) (void)hipEventDestroy(ev1);
    if (evp) (void)hipEventDestroy(evp);
    if (evp1) (void)hipEventDestroy(evp1);
    if (evf0) (void)hipEventDestroy(evf0);
    if (evf1) (void)hipEventDestroy(evf1);
    for (int k = 0; k < 3; ++k) {
      if (evk[k]) (void)hipEventDestroy(evk[k]);
      if (evpk[k]) (void)hipEventDestroy(evpk[k]);
    }
    if (done) (void)hipEventDestroy(done);
    if (ev_end) (void)hipEventDestroy(ev_end);
    if (h2d) (void)hipEventDestroy(h2d);
    if (ev_sorted) (void)hipEventDestroy(ev_sorted);
    if (ev_fin0) (void)hipEventDestroy(ev_fin0);
    if (ev_fin1) (void)hipEventDestroy(ev_fin1);
    if (fin_stream) (void)hipStreamDestroy(fin_stream);
    if (copy_stream) (void)hipStreamDestroy(copy_stream);
  }
  PoaArena(const PoaArena&) = delete;
  PoaArena& operator=(const PoaArena&) = delete;
};

class DevArena;

}  // namespace svs

struct svs_context {
  int device = 0;
  hipStream_t stream = nullptr;     // POA launches (task groups alternate on it)
  hipStream_t em_stream = nullptr;  // similarity + EM kernels, concurrent with POA
  hipEvent_t ev_start = nullptr, ev_stop = nullptr;
  // EM K-parallel path: after its kernel, and before the in-order rerun (the
  // host check between them is not kernel time)
  hipEvent_t ev_mid = nullptr, ev_rerun = nullptr;
  svs::ThreadPool* pool = nullptr;
  size_t device_budget = 0;  // bytes usable for traceback + row pool per launch
  size_t dgraph_budget = 0;  // limit of dgraph_arena (the device-resident POA graphs)
  // POA arenas, one per concurrently in-flight task group
  std::vector<std::unique_ptr<svs::PoaArena>> poa_arenas;
  // blocks of the device-resident POA graphs (svs_devarena.hpp)
  std::unique_ptr<svs::DevArena> dgraph_arena;
  // EM arenas
  svs::DeviceBuf d_em_in, d_em_ws, d_em_out, d_rng;
  svs::PinnedBuf h_em_in, h_em_out;
  // MisScore arenas (svs_misscore_engine.cpp)
  svs::DeviceBuf d_ms_pairs, d_ms_seq, d_ms_nib, d_ms_carry, d_ms_stack, d_ms_out;
  size_t rng_len = 0;
  uint32_t rng_seed = 0;
};
