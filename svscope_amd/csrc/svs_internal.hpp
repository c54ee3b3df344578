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
  std::string consensus;
  std::vector<std::string> msa;
};

void check_poa_config(const svs_poa_config& c);
void run_poa_tasks(svs_context* ctx, std::vector<PoaTask>& tasks, const svs_poa_config& cfg,
                   svs_poa_stats& st);

}  // namespace svs
