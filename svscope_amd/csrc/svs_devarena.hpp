// Device memory for the device-resident POA graphs (poa_dgraph.hpp): one
// block per task, sized to the task, freed when the task completes.  Blocks
// come from large hipMalloc'ed chunks in power-of-two size classes (>= 64 KiB)
// with a free list per class (svs_block_arena.hpp), so the thousands of task
// starts and ends of a session never call hipMalloc / hipFree (both can stall
// the whole device).  The arena has a byte limit (svs_context::dgraph_budget:
// the HBM left after the per-launch budget, svs_abi.cpp); chunks are sized
// from it.  When no block fits, try_alloc returns null (the engine defers or
// fails that task, svs_poa_engine.cpp reserve_blocks) and alloc throws
// (SvsError -2) instead of running the device out of memory.
#pragma once
#include <hip/hip_runtime.h>

#include <string>

#include "svs_block_arena.hpp"
#include "svs_context.hpp"

namespace svs {

class DevArena : public BlockArena {
 public:
  explicit DevArena(size_t limit) : BlockArena(limit, &hip_chunk, &hip_free, nullptr) {}

  void* alloc(size_t bytes) {
    void* p = try_alloc(bytes);
    if (!p)
      throw SvsError(-2, "device graph arena: a block of " + std::to_string(bytes) + " bytes would pass its limit of " +
                             std::to_string(limit()) + " (SVS_DEVICE_BUDGET_GB, fewer tasks in flight)");
    return p;
  }

 private:
  static void* hip_chunk(size_t bytes, void*) {
    void* p = nullptr;
    SVS_HIP(hipMalloc(&p, bytes));
    return p;
  }
  static void hip_free(void* p, void*) { (void)hipFree(p); }
};

}  // namespace svs
