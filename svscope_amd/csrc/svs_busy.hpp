// Union of time intervals, kept as disjoint merged [start, end) pairs: the DP
// busy time of bench.py's roofline.dp_busy (svs_poa_engine.cpp DpBusyClock).
// Host-only, no HIP: tests/cpp/busy_union_emu.cpp checks it against a brute
// force on the CPU.
#pragma once
#include <algorithm>
#include <iterator>
#include <map>

namespace svs {

// Adds [lo, hi] to the union iv (start -> end, disjoint) and returns by how
// much the union's total length grew.
inline double busy_union_add(std::map<double, double>& iv, double lo, double hi) {
  hi = std::max(lo, hi);
  double gone = 0.0;
  // fold every interval that touches [lo, hi] into it
  auto it = iv.upper_bound(lo);
  if (it != iv.begin() && std::prev(it)->second >= lo) --it;
  while (it != iv.end() && it->first <= hi) {
    lo = std::min(lo, it->first);
    hi = std::max(hi, it->second);
    gone += it->second - it->first;
    it = iv.erase(it);
  }
  iv.emplace(lo, hi);
  return (hi - lo) - gone;
}

}  // namespace svs
