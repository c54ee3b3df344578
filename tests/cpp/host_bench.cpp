// Host graph-engine microbenchmark (development tool, not a test): replays
// recorded read-vs-graph alignments (kernel_emu.cpp, EMU_RECORD) through the
// product's PoaGraph and times each host phase of one POA step: strip-row
// export, column-0 fill, alignment fold (incl. topological sort).
//   g++ -O3 -std=c++17 -I svscope_amd/csrc tests/cpp/host_bench.cpp svscope_amd/csrc/poa_graph.cpp
//   ./a.out rec.bin first_seq.txt reps
#include <algorithm>
#include <chrono>
#include <ctime>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <string>
#include <vector>

#include "poa_graph.hpp"

int main(int argc, char** argv) {
  if (argc < 4) return 2;
  std::ifstream fs(argv[2]);
  std::string first;
  std::getline(fs, first);
  std::vector<std::string> seqs;
  std::vector<std::vector<int32_t>> alns;
  FILE* f = std::fopen(argv[1], "rb");
  if (!f) return 3;
  for (;;) {
    uint32_t ls, la;
    if (std::fread(&ls, 4, 1, f) != 1) break;
    std::string s(ls, '\0');
    if (std::fread(&s[0], 1, ls, f) != ls) return 4;
    if (std::fread(&la, 4, 1, f) != 1) return 4;
    std::vector<int32_t> a(la);
    if (std::fread(a.data(), 4, la, f) != la) return 4;
    seqs.push_back(std::move(s));
    alns.push_back(std::move(a));
  }
  std::fclose(f);
  const int reps = std::atoi(argv[3]);
  // thread CPU time, minimum of three runs of each repeatable phase (the
  // development container is shared: wall time is noisy)
  auto now = [] {
    timespec ts;
    clock_gettime(CLOCK_THREAD_CPUTIME_ID, &ts);
    return ts.tv_sec * 1e6 + ts.tv_nsec * 1e-3;
  };
  double t_exp = 0, t_col = 0, t_fold = 0;
  uint64_t rows = 0;
  for (int rep = 0; rep < reps; ++rep) {
    svs::PoaGraph g;
    svs::RowTables T;
    g.add_alignment_nodes({}, first);
    for (size_t i = 0; i < seqs.size(); ++i) {
      double be = 1e30, bc = 1e30;
      for (int x = 0; x < 3; ++x) {
        const double t0 = now();
        const int32_t gaps[4] = {-8, -6, -10, -4};
        g.export_strip_rows(&T, gaps);
        const double t1 = now();
        const double t2 = now();
        be = std::min(be, t1 - t0);
        bc = std::min(bc, t2 - t1);
      }
      const double t2 = now();
      g.add_alignment_ranks(alns[i], seqs[i]);
      const double t3 = now();
      t_exp += be;
      t_col += bc;
      t_fold += t3 - t2;
      rows += T.pstart.size() - 1;
    }
  }
  const double n = static_cast<double>(reps) * seqs.size();
  std::printf("steps %.0f  mean rows %.0f  per step (us): export %.1f  col0 %.1f  fold %.1f  total %.1f\n", n,
              rows / n, t_exp / n, t_col / n, t_fold / n, (t_exp + t_col + t_fold) / n);
  return 0;
}
