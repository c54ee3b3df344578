// CPU check of the device graph arena's block logic (svscope_amd/csrc/
// svs_block_arena.hpp): a fake chunk allocator hands out address
// ranges, a seeded workload of task-sized allocations and frees runs the
// arena past its limit (so that chunk tails, split_larger and null returns
// all happen), and every returned block is checked against every live block
// for overlap and against its chunk for bounds.  Built by
// tests/test_bench_host.py with g++.
#include <cstdint>
#include <cstdio>
#include <map>
#include <random>
#include <vector>

#include "../../svscope_amd/csrc/svs_block_arena.hpp"

namespace {

struct FakeHeap {
  uintptr_t next = uintptr_t(1) << 40;
  std::map<uintptr_t, size_t> chunks;  // base -> bytes
};

void* fake_alloc(size_t bytes, void* user) {
  FakeHeap* h = static_cast<FakeHeap*>(user);
  const uintptr_t p = h->next;
  h->chunks[p] = bytes;
  h->next += bytes + (uintptr_t(1) << 30);  // a gap, so a block past its chunk is caught
  return reinterpret_cast<void*>(p);
}
void fake_free(void*, void*) {}

}  // namespace

extern "C" {

// Runs `steps` random operations against an arena of `limit` bytes; returns
// the number of violations (overlaps, blocks outside their chunk, a block
// handed out twice, a non-power-of-two chunk) and writes how often
// try_alloc returned null and how many blocks were checked.
int emu_block_arena(uint64_t limit, uint64_t seed, int steps, int* n_null, int* n_checked) {
  FakeHeap heap;
  int bad = 0, nulls = 0, checked = 0;
  {
    svs::BlockArena A(static_cast<size_t>(limit), &fake_alloc, &fake_free, &heap);
    if (!svs::BlockArena::is_pow2(A.chunk_bytes())) ++bad;
    std::mt19937_64 rng(seed);
    std::map<uintptr_t, size_t> live;  // base -> class bytes
    std::vector<std::pair<void*, size_t>> held;
    // task-like sizes: mostly 0.1 .. 40 MB, some tiny, a few above a chunk
    auto draw = [&]() -> size_t {
      const uint64_t r = rng() % 100;
      if (r < 10) return 1 + rng() % (64 << 10);
      if (r < 95) return (size_t(100) << 10) + rng() % (size_t(40) << 20);
      return A.chunk_bytes() + 1 + rng() % (A.chunk_bytes() * 2);
    };
    for (int s = 0; s < steps; ++s) {
      const bool do_free = !held.empty() && (rng() % 100) < 45;
      if (do_free) {
        const size_t k = rng() % held.size();
        const uintptr_t p = reinterpret_cast<uintptr_t>(held[k].first);
        A.free(held[k].first, held[k].second);
        live.erase(p);
        held[k] = held.back();
        held.pop_back();
        continue;
      }
      const size_t want = draw();
      void* v = A.try_alloc(want);
      if (!v) {
        ++nulls;
        continue;
      }
      ++checked;
      const uintptr_t p = reinterpret_cast<uintptr_t>(v);
      const size_t c = svs::BlockArena::size_class(want);
      // inside one chunk
      auto ch = heap.chunks.upper_bound(p);
      if (ch == heap.chunks.begin()) {
        ++bad;
      } else {
        --ch;
        if (p + c > ch->first + ch->second) ++bad;
      }
      // disjoint from every live block
      auto nx = live.lower_bound(p);
      if (nx != live.end() && nx->first < p + c) ++bad;
      if (nx != live.begin()) {
        auto pv = std::prev(nx);
        if (pv->first + pv->second > p) ++bad;
      }
      if (live.count(p)) ++bad;
      live[p] = c;
      held.emplace_back(v, want);
      if (A.reserved() > A.limit()) ++bad;
    }
  }
  *n_null = nulls;
  *n_checked = checked;
  return bad;
}

}  // extern "C"
