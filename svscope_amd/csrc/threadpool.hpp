// Fork-join thread pool for per-window host graph work (no HIP dependency).
#pragma once
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <exception>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace svs {

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
  size_t pending_ = 0;  // workers that have not yet finished the current generation
  uint64_t generation_ = 0;
  bool stop_ = false;
  std::exception_ptr err_;
};

}  // namespace svs
