// Internal declarations shared by the engine translation units.
#pragma once
#include <string>
#include <vector>

#include "../../include/svscope.h"
#include "poa_graph.hpp"

namespace svs {

struct PoaTask {
  std::vector<std::string> seqs;
  PoaGraph graph;
  RowTables rows;  // exported row tables of the current step (capacity reused across steps)
  std::string consensus;
  std::vector<std::string> msa;
};

void check_poa_config(const svs_poa_config& c);
void run_poa_tasks(svs_context* ctx, std::vector<PoaTask>& tasks, const svs_poa_config& cfg,
                   svs_poa_stats& st);

int em_validate(int32_t n_windows, const svs_em_window* wins, const uint8_t* X, std::string* err);
void run_similarity(svs_context* ctx, int32_t n, const svs_em_window* wins, const uint8_t* X, double* S_out,
                    const int64_t* s_off);
svs_em_result* run_em(svs_context* ctx, int32_t n, const svs_em_window* wins, const uint8_t* X,
                      const int32_t* labels, const svs_em_config& cfg);
svs_em_result* run_em_cluster(svs_context* ctx, int32_t n, const svs_em_window* wins, const uint8_t* X,
                              const svs_em_config& cfg);

}  // namespace svs
