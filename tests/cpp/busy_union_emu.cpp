// CPU harness for svscope_amd/csrc/svs_busy.hpp (tests/test_bench_host.py):
// adds n intervals in the given order and returns the union length after
// each, as the POA engine accumulates kernel_busy_ms.
#include "../../svscope_amd/csrc/svs_busy.hpp"

extern "C" void emu_busy_union(const double* lo, const double* hi, int n, double* total_after) {
  std::map<double, double> iv;
  double t = 0.0;
  for (int i = 0; i < n; ++i) {
    t += svs::busy_union_add(iv, lo[i], hi[i]);
    total_after[i] = t;
  }
}
