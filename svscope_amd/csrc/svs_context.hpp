// Host-side runtime of libsvscope_hip: context, device arenas, pinned staging,
// a small fork-join thread pool for per-window graph work.
#pragma once
#include <hip/hip_runtime.h>

#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <functional>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
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
struct DeviceBuf {
  void* ptr = nullptr;
  size_t cap = 0;
  void ensure(size_t bytes) {
    if (bytes <= cap) return;
    if (ptr) SVS_HIP(hipFree(ptr));
    ptr = nullptr;
    cap = 0;
    size_t want = bytes + bytes / 4 + 4096;
    if (hipMalloc(&ptr, want) != hipSuccess) {
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
    ptr = nullptr;
    cap = 0;
  }
};

// Growable pinned host buffer.
struct PinnedBuf {
  void* ptr = nullptr;
  size_t cap = 0;
  void ensure(size_t bytes) {
    if (bytes <= cap) return;
    if (ptr) SVS_HIP(hipHostFree(ptr));
    ptr = nullptr;
    cap = 0;
    const size_t want = bytes + bytes / 4 + 4096;
    SVS_HIP(hipHostMalloc(&ptr, want, hipHostMallocDefault));
    cap = want;
  }
  template <class T> T* as() const { return static_cast<T*>(ptr); }
  void release() {
    if (ptr) (void)hipHostFree(ptr);
    ptr = nullptr;
    cap = 0;
  }
};

// Fork-join pool: parallel_for(n, fn) runs fn(i) for i in [0, n).
class ThreadPool {
 public:
  explicit ThreadPool(unsigned n);
  ~ThreadPool();
  unsigned size() const { return static_cast<unsigned>(workers_.size()) + 1; }
  void parallel_for(size_t n, const std::function<void(size_t)>& fn);

 private:
  void worker_loop();
  std::vector<std::thread> workers_;
  std::mutex mu_;
  std::condition_variable cv_, done_cv_;
  const std::function<void(size_t)>* fn_ = nullptr;
  size_t n_ = 0;
  std::atomic<size_t> next_{0};
  unsigned active_ = 0;
  uint64_t generation_ = 0;
  bool stop_ = false;
  std::exception_ptr err_;
};

}  // namespace svs

struct svs_context {
  int device = 0;
  hipStream_t stream = nullptr;
  hipEvent_t ev_start = nullptr, ev_stop = nullptr;
  svs::ThreadPool* pool = nullptr;
  size_t device_budget = 0;  // bytes usable for traceback + row pool per launch
  // POA arenas
  svs::DeviceBuf d_jobs, d_row_info, d_row_slot, d_row_pstart, d_pred_row, d_pred_slot, d_seqs;
  svs::DeviceBuf d_tb, d_pool, d_aln, d_aln_len;
  svs::PinnedBuf h_stage, h_aln, h_aln_len;
  // EM arenas
  svs::DeviceBuf d_em_in, d_em_ws, d_em_out, d_rng;
  svs::PinnedBuf h_em_in, h_em_out;
  size_t rng_len = 0;
};
