// Fork-join thread pool (see threadpool.hpp).
#include "threadpool.hpp"

namespace svs {

ThreadPool::ThreadPool(unsigned n) {
  for (unsigned i = 1; i < n; ++i) workers_.emplace_back([this] { worker_loop(); });
}

ThreadPool::~ThreadPool() {
  {
    std::lock_guard<std::mutex> lk(mu_);
    stop_ = true;
  }
  cv_.notify_all();
  for (auto& t : workers_) t.join();
}

void ThreadPool::worker_loop() {
  uint64_t seen = 0;
  while (true) {
    const std::function<void(size_t)>* fn;
    size_t n;
    {
      std::unique_lock<std::mutex> lk(mu_);
      cv_.wait(lk, [&] { return stop_ || generation_ != seen; });
      if (stop_) return;
      seen = generation_;
      fn = fn_;
      n = n_;
    }
    for (size_t i = next_.fetch_add(1); i < n; i = next_.fetch_add(1)) {
      try {
        (*fn)(i);
      } catch (...) {
        std::lock_guard<std::mutex> lk(mu_);
        if (!err_) err_ = std::current_exception();
      }
    }
    {
      std::lock_guard<std::mutex> lk(mu_);
      if (--pending_ == 0) done_cv_.notify_all();
    }
  }
}

// Every worker takes part in every generation exactly once (pending_ counts
// them down), so no worker can still hold a previous generation's fn/n when
// the next parallel_for resets the work counter.
void ThreadPool::parallel_for(size_t n, const std::function<void(size_t)>& fn) {
  if (n == 0) return;
  if (workers_.empty() || n == 1) {
    for (size_t i = 0; i < n; ++i) fn(i);
    return;
  }
  {
    std::lock_guard<std::mutex> lk(mu_);
    fn_ = &fn;
    n_ = n;
    next_.store(0);
    err_ = nullptr;
    pending_ = workers_.size();
    ++generation_;
  }
  cv_.notify_all();
  for (size_t i = next_.fetch_add(1); i < n; i = next_.fetch_add(1)) {
    try {
      fn(i);
    } catch (...) {
      std::lock_guard<std::mutex> lk(mu_);
      if (!err_) err_ = std::current_exception();
    }
  }
  std::unique_lock<std::mutex> lk(mu_);
  done_cv_.wait(lk, [&] { return pending_ == 0; });
  fn_ = nullptr;
  if (err_) {
    auto e = err_;
    err_ = nullptr;
    std::rethrow_exception(e);
  }
}

}  // namespace svs
