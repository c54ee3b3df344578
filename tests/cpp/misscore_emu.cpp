// TEST INFRASTRUCTURE: CPU emulation of the MisScore HIP path
// (svscope_amd/csrc/misscore_kernels.hip).  The fill is a plain scalar loop
// producing the kernel's 4-bit (dh, dv) cells; the traceback is the product's
// own shared code (misscore_tb.hpp).  Lets the CPU suite check the 4-bit
// derivation of pairwise2's trace bits and the DFS against the oracle without
// a GPU.  Not part of the product library.
#include <algorithm>
#include <cstdint>
#include <vector>

#define SVS_MS_FN inline
#include "../../svscope_amd/csrc/misscore_tb.hpp"

namespace {
struct EmuEnv {
  const char* A;
  const char* B;
  int32_t la, lb;
  std::vector<uint8_t> nibs;  // (r-1) * lb + (c-1)
  std::vector<svs::MsState> stack;
  size_t cap;
  int32_t max_depth = 0;
  uint32_t nib(int32_t r, int32_t c) const { return nibs[static_cast<size_t>(r - 1) * lb + (c - 1)]; }
  uint8_t a(int32_t i) const { return static_cast<uint8_t>(A[i]); }
  uint8_t b(int32_t j) const { return static_cast<uint8_t>(B[j]); }
  bool push(const svs::MsState& s) {
    if (stack.size() >= cap) return false;
    stack.push_back(s);
    return true;
  }
  void pop(svs::MsState& s) {
    s = stack.back();
    stack.pop_back();
  }
};
}  // namespace

extern "C" int emu_aligment_counts(const char* a, int la, const char* b, int lb, int cutoff, int stack_cap,
                                   int* out /* status, cols, matches, trim_len, trim_match, max_depth */,
                                   long long* steps) {
  EmuEnv env{a, b, la, lb, {}, {}, static_cast<size_t>(stack_cap)};
  if (la > 0 && lb > 0) {
    env.nibs.resize(static_cast<size_t>(la) * lb);
    std::vector<int32_t> prev(lb + 1), cur(lb + 1);
    for (int c = 0; c <= lb; ++c) prev[c] = -c;
    for (int r = 1; r <= la; ++r) {
      cur[0] = -r;
      for (int c = 1; c <= lb; ++c) {
        const int32_t s = a[r - 1] == b[c - 1] ? 1 : 0;
        const int32_t h = std::max(prev[c - 1] + s, std::max(prev[c], cur[c - 1]) - 1);
        const int32_t dh = h - cur[c - 1], dv = h - prev[c];
        env.nibs[static_cast<size_t>(r - 1) * lb + (c - 1)] = static_cast<uint8_t>((dh + 1) | ((dv + 1) << 2));
        cur[c] = h;
      }
      std::swap(prev, cur);
    }
  }
  const svs::MsResult r = svs::ms_first_alignment(env, la, lb, cutoff, 8ll * (la + lb) + 4096);
  out[0] = r.status;
  out[1] = r.cols;
  out[2] = r.matches;
  out[3] = r.trim_len;
  out[4] = r.trim_match;
  out[5] = r.max_depth;
  *steps = r.steps;
  return 0;
}
