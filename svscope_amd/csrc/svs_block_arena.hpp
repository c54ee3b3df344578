// Power-of-two block arena over large chunks, independent of where the chunks
// come from (svs_devarena.hpp gives it hipMalloc; tests/cpp/block_arena_emu.cpp
// gives it a fake allocator and checks that live blocks never overlap).
//
// Size classes are powers of two, at least 64 KiB, and so is the chunk size
// (a sixteenth of the limit, 256 MiB .. 4 GiB, rounded down to a power of
// two, and no more than the limit).  A chunk is cut front to back in request order.  What keeps live
// blocks disjoint is that every free-list key is a power of two and every
// block filed under key k spans exactly k bytes: a chunk's unused tail is
// filed as a descending run of powers of two, and split_larger halves a
// block of class k into k/2 + k/2 down to the class asked for (a
// chunk size that was not a power of two filed tails under keys like 3 * 2^n,
// and halving those could hand out overlapping blocks).  try_alloc returns
// null when the limit leaves no room (the engine then defers or fails that
// task, svs_poa_engine.cpp reserve_blocks); blocks go back to their class's
// free list, never to the allocator.
#pragma once
#include <algorithm>
#include <cassert>
#include <cstddef>
#include <cstdint>
#include <map>
#include <vector>

namespace svs {

class BlockArena {
 public:
  using ChunkAlloc = void* (*)(size_t bytes, void* user);  // null when it cannot
  using ChunkFree = void (*)(void* p, void* user);

  static constexpr size_t kMinClass = size_t(64) << 10;

  BlockArena(size_t limit, ChunkAlloc a, ChunkFree f, void* user) : limit_(limit), alloc_(a), free_chunk_(f), user_(user) {
    chunk_ = floor_pow2(std::min<size_t>(size_t(4) << 30, std::max<size_t>(size_t(256) << 20, limit / 16)));
    chunk_ = std::max(kMinClass, std::min(chunk_, floor_pow2(std::max<size_t>(limit, 1))));  // one chunk fits the limit
  }
  ~BlockArena() {
    for (void* c : chunks_) free_chunk_(c, user_);
  }
  BlockArena(const BlockArena&) = delete;
  BlockArena& operator=(const BlockArena&) = delete;

  static size_t size_class(size_t bytes) {
    size_t c = kMinClass;
    while (c < bytes) c <<= 1;
    return c;
  }
  static bool is_pow2(size_t x) { return x && !(x & (x - 1)); }
  static size_t floor_pow2(size_t x) {
    size_t p = 1;
    while (p <= x / 2) p <<= 1;
    return p;
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
      // the rest of the current chunk goes to the free lists as a descending
      // run of powers of two (each block exactly its key's size)
      if (cur_) {
        size_t left = chunk_ - used_;
        for (size_t k = floor_pow2(std::max<size_t>(left, 1)); k >= kMinClass && left >= kMinClass; k >>= 1)
          if (left >= k) {
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
  size_t chunk_bytes() const { return chunk_; }

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
      assert(is_pow2(it->first) && "block arena: a free-list key that is not a power of two");
      char* p = static_cast<char*>(it->second.back());
      it->second.pop_back();
      for (size_t k = it->first; k > c; k >>= 1) free_[k >> 1].push_back(p + (k >> 1));
      return take(p, c);
    }
    return nullptr;
  }
  void* new_chunk(size_t bytes) {
    if (reserved_ + bytes > limit_) return nullptr;
    void* p = alloc_(bytes, user_);
    if (!p) return nullptr;
    chunks_.push_back(p);
    reserved_ += bytes;
    return p;
  }
  size_t limit_, chunk_ = 0;
  ChunkAlloc alloc_;
  ChunkFree free_chunk_;
  void* user_;
  std::vector<void*> chunks_;
  char* cur_ = nullptr;
  size_t used_ = 0, in_use_ = 0, peak_ = 0, reserved_ = 0;
  std::map<size_t, std::vector<void*>> free_;
};

}  // namespace svs
