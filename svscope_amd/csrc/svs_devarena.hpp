// Device memory for the device-resident POA graphs (poa_dgraph.hpp): one
// block per task, sized to the task, freed when the task completes.  Blocks
// come from large hipMalloc'ed chunks in power-of-two size classes (>= 64 KiB)
// with a free list per class, so the thousands of task starts and ends of a
// session never call hipMalloc / hipFree (both can stall the whole device).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <map>
#include <vector>

#include "svs_context.hpp"

namespace svs {

class DevArena {
 public:
  explicit DevArena(size_t chunk_bytes = size_t(4) << 30) : chunk_(chunk_bytes) {}
  ~DevArena() {
    for (void* c : chunks_) (void)hipFree(c);
  }
  DevArena(const DevArena&) = delete;
  DevArena& operator=(const DevArena&) = delete;

  static size_t size_class(size_t bytes) {
    size_t c = size_t(64) << 10;
    while (c < bytes) c <<= 1;
    return c;
  }
  // A block of at least `bytes` (its class size is what free() takes back).
  void* alloc(size_t bytes) {
    const size_t c = size_class(bytes);
    auto it = free_.find(c);
    if (it != free_.end() && !it->second.empty()) {
      void* p = it->second.back();
      it->second.pop_back();
      in_use_ += c;
      return p;
    }
    if (c > chunk_) {  // larger than a chunk: a chunk of its own
      void* p = nullptr;
      SVS_HIP(hipMalloc(&p, c));
      chunks_.push_back(p);
      in_use_ += c;
      return p;
    }
    if (!cur_ || used_ + c > chunk_) {
      void* p = nullptr;
      SVS_HIP(hipMalloc(&p, chunk_));
      chunks_.push_back(p);
      cur_ = static_cast<char*>(p);
      used_ = 0;
    }
    void* p = cur_ + used_;
    used_ += c;
    in_use_ += c;
    peak_ = std::max(peak_, in_use_);
    return p;
  }
  void free(void* p, size_t bytes) {
    if (!p) return;
    const size_t c = size_class(bytes);
    free_[c].push_back(p);
    in_use_ -= c;
  }
  size_t in_use() const { return in_use_; }
  size_t peak() const { return peak_; }

 private:
  size_t chunk_;
  std::vector<void*> chunks_;
  char* cur_ = nullptr;
  size_t used_ = 0, in_use_ = 0, peak_ = 0;
  std::map<size_t, std::vector<void*>> free_;
};

}  // namespace svs
