// Host restatement of the per-window feature selection and cluster labelling
// that sit between the window MSA and the EM / consensus stages:
//   DataScanner.SeqEncoder / CallMargin / FindNonSameSite / MSAFeatureSelection
//     (/root/reference/src/DataScanner.py:124-220, incl. the DEL-read id quirk :204)
//   DecisionMaker.Decision cluster labelling + consensus inputs (DecisionMaker.py:137-176)
// Integer/byte work on at most ~65 x 10k symbols per window; it runs on the
// engine's thread pool while the GPU aligns other windows.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace svs {

struct WindowFeatures {
  int32_t rows = 0;               // rows of seqdatamx (encoded rows - 1)
  int32_t n_feat = 0;             // columns of seqdatamx
  std::vector<uint8_t> feat;      // rows x n_feat, symbols 0..4
  std::vector<int32_t> id_map;    // returned readIDList[k] = ReadIDs[id_map[k]]
  // SeqDecoder(seqencode[r + 1]) of every seqdatamx row r: the ungapped,
  // upper-case read a cluster's consensus POA takes (DecisionMaker.py:157-171)
  std::vector<std::string> row_reads;
};

// msa: the window MSA rows (all of one width); read_lens: len() of
// sequenceList[1:]; n_ids: len(ReadIDs).  Throws SvsError(SVS_E_INVALID) on a
// symbol outside ATCGatcg- (the reference's SeqEncoder raises KeyError).
void msa_feature_select(const std::vector<std::string>& msa, const std::string& flank_5, const std::string& flank_3,
                        const std::vector<int32_t>& read_lens, int32_t n_ids, int32_t hcutoff, double scutoff,
                        WindowFeatures* out);

// The device's form of the same selection (poa_fold.hip msa_features): the
// host works out from the window's reads and flanks what does not need the
// MSA, the device selects the columns.
struct DeviceFeatureParams {
  int32_t f5_take = 0, f3_take = 0;  // CallMargin's stops (FoldJob::f5_take / f3_take)
  uint32_t extra = 0;                // all-gap rows after the MSA rows (full-DEL reads)
  uint32_t cut = 0;                  // FindNonSameSite: second-largest count >= cut
  int32_t msa_rows = 0;              // MSA rows (non-empty sequences)
  bool ok = true;                    // false: a read holds '-' (the MSA's gaps and its letters mix): host path
};
// seqs: the window's sequenceList (MSA row k = the k-th non-empty one).
// Throws SvsError(SVS_E_INVALID) on a letter SeqEncoder would reject.
DeviceFeatureParams device_feature_params(const std::vector<std::string>& seqs, const std::string& flank_5,
                                          const std::string& flank_3, const std::vector<int32_t>& read_lens,
                                          int32_t n_ids, int32_t hcutoff, double scutoff);
// WindowFeatures from the device's seqdatamx (rows x n_feat).
void device_features(const std::vector<std::string>& seqs, const std::vector<int32_t>& read_lens, int32_t n_ids,
                     const DeviceFeatureParams& p, int32_t n_feat, std::vector<uint8_t>&& feat, WindowFeatures* out);

struct ClusterPlan {
  bool som = false;
  std::vector<int32_t> rows;      // seqdatamx row indices of the cluster (ascending)
  std::vector<int32_t> ids;       // ReadIDs indices of those rows (via id_map)
  std::vector<std::string> reads; // ungapped, upper-case reads for the consensus POA
  std::string consensus = "-";
};

// Labels in ascending order -> somatic / germline clusters (DecisionMaker.py:145-154).
// is_tlabel[i]: ReadIDs[i]'s tag equals Tlabel.  Returns false when a label
// row has no read id (the reference raises IndexError there).
bool plan_clusters(const WindowFeatures& f, const int32_t* rclust, const uint8_t* is_tlabel, int32_t readcutoff,
                   std::vector<ClusterPlan>* som, std::vector<ClusterPlan>* germ);

}  // namespace svs
