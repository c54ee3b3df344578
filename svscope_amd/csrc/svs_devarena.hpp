// Device memory for the device-resident POA graphs (poa_dgraph.hpp): one
// block per task, sized to the task, freed when the task completes.  Blocks
// come from large hipMalloc'ed chunks in power-of-two size classes (>= 64 KiB)
// with a free list per class, so the thousands of task starts and ends of a
// session never call hipMalloc / hipFree (both can stall the whole device).
// The arena has a byte limit (svs_context::dgraph_budget: the HBM left after
// the per-launch budget, svs_abi.cpp); chunks are sized from it.  Before a new
// chunk is cut, a free block of a larger class is split in halves down to the
// class asked for; when neither fits, try_alloc returns null (the engine fails
// that task alone, svs_poa_engine.cpp reserve_blocks) and alloc throws
// (SvsError -2) instead of running the device out of memory.  Blocks go back
// to their class's free list, never to HIP: reserved() only grows, peak() is
// the largest in_use().
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
  // A block of at least `bytes` (its class size is what free() takes back),
  // or null when it would take the arena past its limit.
  void* try_alloc(size_t bytes) {
    const size_t c = size_class(bytes);
    auto it = free_.find(c);
    if (it != free_.end() && !it->second.empty()) {
      void* p = it->second.back();
      it->second.pop_back();
      return take(p, c);
    }
    if (c > chunk_) {  // larger than a chunk: a chunk of its own
      void* p = new_chunk(c);
      return p ? take(p, c) : split_larger(c);
    }
    if (!cur_ || used_ + c > chunk_) {
      // the rest of the current chunk goes to the free lists, largest first
      if (cur_) {
        size_t left = chunk_ - used_;
        for (size_t k = chunk_; k >= (size_t(64) << 10); k >>= 1)
          while (left >= k) {
            free_[k].push_back(cur_ + used_);
            used_ += k;
            left -= k;
          }
      }
      void* n = new_chunk(chunk_);
      if (!n) {
        cur_ = nullptr;
        used_ = 0;
        return split_larger(c);
      }
      cur_ = static_cast<char*>(n);
      used_ = 0;
    }
    void* p = cur_ + used_;
    used_ += c;
    return take(p, c);
  }
  void* alloc(size_t bytes) {
    void* p = try_alloc(bytes);
    if (!p)
      throw SvsError(-2, "device graph arena: a block of " + std::to_string(bytes) + " bytes would pass its limit of " +
                             std::to_string(limit_) + " (SVS_DEVICE_BUDGET_GB, fewer tasks in flight)");
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
  size_t reserved() const { return reserved_; }
  size_t limit() const { return limit_; }

 private:
  void* take(void* p, size_t c) {
    in_use_ += c;
    peak_ = std::max(peak_, in_use_);
    return p;
  }
  // a free block of the smallest larger class, halved down to class c (the
  // upper halves go to their free lists); null when there is none
  void* split_larger(size_t c) {
    for (auto it = free_.upper_bound(c); it != free_.end(); ++it) {
      if (it->second.empty()) continue;
      char* p = static_cast<char*>(it->second.back());
      it->second.pop_back();
      for (size_t k = it->first; k > c; k >>= 1) free_[k >> 1].push_back(p + (k >> 1));
      return take(p, c);
    }
    return nullptr;
  }
  void* new_chunk(size_t bytes) {
    if (reserved_ + bytes > limit_) return nullptr;
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
