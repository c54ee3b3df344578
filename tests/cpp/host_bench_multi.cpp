// Host graph-engine microbenchmark with production-like caches (development
// tool, not a test): G copies of one recorded window (kernel_emu.cpp,
// EMU_RECORD) are folded round-robin, one alignment per graph per step, on T
// threads, so each graph comes back to a thread cold, as in the engine's fold
// (1024 jobs per launch over 16 threads).  Times fold + strip-row export.
//   g++ -O3 -std=c++17 -pthread -I svscope_amd/csrc tests/cpp/host_bench_multi.cpp svscope_amd/csrc/poa_graph.cpp
//   ./a.out rec.bin first_seq.txt G T
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <string>
#include <thread>
#include <vector>

#include "poa_graph.hpp"

int main(int argc, char** argv) {
  if (argc < 5) return 2;
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
  const int G = std::atoi(argv[3]), T = std::atoi(argv[4]);
  std::vector<svs::PoaGraph> g(G);
  std::vector<svs::RowTables> tabs(G);
  for (auto& x : g) x.add_alignment_nodes({}, first);
  const int32_t gaps[4] = {-8, -6, -10, -4};
  double total = 0;
  for (size_t i = 0; i < seqs.size(); ++i) {
    const auto t0 = std::chrono::steady_clock::now();
    std::atomic<int> next{0};
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t)
      th.emplace_back([&] {
        for (int k; (k = next.fetch_add(1)) < G;) {
          g[k].export_strip_rows(&tabs[k], gaps);
          g[k].add_alignment_ranks(alns[i], seqs[i]);
        }
      });
    for (auto& x : th) x.join();
    total += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  }
  std::printf("graphs %d threads %d: %.1f us per alignment per thread (export + fold), %.2f ms per step\n", G, T,
              total * 1e3 * T / (static_cast<double>(G) * seqs.size()), total / seqs.size());
  return 0;
}
