// Device memory for the device-resident POA graphs (poa_dgraph.hpp): one
// block per task, sized to the task, freed when the task completes.  Blocks
// come from large hipMalloc'ed chunks in power-of-two size classes (>= 64 KiB)
// with a free list per class, so the thousands of task starts and ends of a
// session never call hipMalloc / hipFree (both can stall the whole device).
// The arena has a byte limit (svs_context::dgraph_budget: the HBM left after
// the per-launch budget, svs_abi.cpp); a block that would take the chunks past
// it fails loudly (SvsError -2) instead of running the device out of memory,
// and chunks are sized from the limit.  Blocks go back to their class's free
// list, never to HIP: reserved() only grows, peak() is the largest in_use().
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <map>
#include <string>
#include <vector>

#include "svs_context.hpp"

namespace svs {

class DevArena {
 public:
  explicit DevArena(size_t limit) : limit_(limit) {
    // a sixteenth of the limit, 256 MiB .. 4 GiB, in whole 64-KiB classes
    chunk_ = std::min<size_t>(size_t(4) << 30, std::max<size_t>(size_t(256) << 20, limit / 16)) & ~((size_t(64) << 10) - 1);
  }
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
      return take(p, c);
    }
    if (c > chunk_) return take(new_chunk(c), c);  // larger than a chunk: a chunk of its own
    if (!cur_ || used_ + c > chunk_) {
      cur_ = static_cast<char*>(new_chunk(chunk_));
      used_ = 0;
    }
    void* p = cur_ + used_;
    used_ += c;
    return take(p, c);
  }
  void free(void* p, size_t bytes) {
    if (!p) return;
    const size_t c = size_class(bytes);
    free_[c].push_back(p);
    in_use_ -= c;
  }
  size_t in_use() const { return in_use_; }
  size_t peak() const { return peak_; }
  size_t reserved() const { return reserved_; }
  size_t limit() const { return limit_; }

 private:
  void* take(void* p, size_t c) {
    in_use_ += c;
    peak_ = std::max(peak_, in_use_);
    return p;
  }
  void* new_chunk(size_t bytes) {
    if (reserved_ + bytes > limit_)
      throw SvsError(-2, "device graph arena: " + std::to_string(reserved_ + bytes) + " bytes would pass its limit of " +
                             std::to_string(limit_) + " (SVS_DEVICE_BUDGET_GB, fewer tasks in flight)");
    void* p = nullptr;
    SVS_HIP(hipMalloc(&p, bytes));
    chunks_.push_back(p);
    reserved_ += bytes;
    return p;
  }
  size_t limit_, chunk_;
  std::vector<void*> chunks_;
  char* cur_ = nullptr;
  size_t used_ = 0, in_use_ = 0, peak_ = 0, reserved_ = 0;
  std::map<size_t, std::vector<void*>> free_;
};

}  // namespace svs
