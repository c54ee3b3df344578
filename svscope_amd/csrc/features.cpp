// Feature selection + cluster labelling on the host (see features.hpp).
#include "features.hpp"

#include <algorithm>

#include "../../include/svscope.h"
#include "svs_context.hpp"

namespace svs {

namespace {

// SeqEncoder alphabet (DataScanner.py:124-129): A0 T1 C2 G3 -4, case-folded.
struct Codes {
  uint8_t enc[256];
  Codes() {
    std::fill(enc, enc + 256, 255);
    const char* s = "ATCG-";
    for (int i = 0; i < 5; ++i) {
      enc[static_cast<unsigned char>(s[i])] = static_cast<uint8_t>(i);
      if (i < 4) enc[static_cast<unsigned char>(s[i] + 32)] = static_cast<uint8_t>(i);
    }
  }
};
const Codes kCodes;
const char kDecode[4] = {'A', 'T', 'C', 'G'};

// CallMargin (DataScanner.py:146-165): columns of MSA row 0 spent on the
// flanks.  The forward walk stops once the ungapped prefix equals flank_5
// (otherwise it keeps every ungapped column); the backward walk over columns
// len-1 .. 1 likewise for flank_3.  Returns a per-column "in pool" mask.
std::vector<uint8_t> call_margin(const std::string& ex, const std::string& f5, const std::string& f3) {
  const int64_t W = static_cast<int64_t>(ex.size());
  std::vector<uint8_t> pool(W, 0);
  {
    size_t got = 0;  // ungapped chars taken so far
    bool match = true;  // taken chars equal f5's prefix
    for (int64_t i = 0; i < W; ++i) {
      if (ex[i] != '-') {
        pool[i] = 1;
        if (got < f5.size()) match = match && ex[i] == f5[got];
        else match = false;
        ++got;
      }
      if (match && got == f5.size()) break;
    }
  }
  {
    size_t got = 0;
    bool match = true;
    for (int64_t i = W - 1; i >= 1; --i) {
      if (ex[i] != '-') {
        pool[i] = 1;
        if (got < f3.size()) match = match && ex[i] == f3[f3.size() - 1 - got];
        else match = false;
        ++got;
      }
      if (match && got == f3.size()) break;
    }
  }
  return pool;
}

}  // namespace

void msa_feature_select(const std::vector<std::string>& msa, const std::string& flank_5, const std::string& flank_3,
                        const std::vector<int32_t>& read_lens, int32_t n_ids, int32_t hcutoff, double scutoff,
                        WindowFeatures* out) {
  WindowFeatures& F = *out;
  const int32_t R0 = static_cast<int32_t>(msa.size());
  const int32_t W = R0 ? static_cast<int32_t>(msa[0].size()) : 0;
  // full-DEL reads (DataScanner.py:195-208): ids become UnDEL + UnDEL (the
  // reference's quirk), encoded gains one all-gap row per UnDEL id
  std::vector<int32_t> undel;
  bool has_del = false;
  for (int32_t len : read_lens) has_del = has_del || len == 0;
  F.id_map.clear();
  int32_t extra = 0;
  if (has_del) {
    std::vector<uint8_t> is_del(std::max<int32_t>(n_ids, 0), 0);
    for (size_t i = 0; i < read_lens.size(); ++i)
      if (read_lens[i] == 0 && static_cast<int32_t>(i) < n_ids) is_del[i] = 1;
    for (int32_t i = 0; i < n_ids; ++i)
      if (!is_del[i]) undel.push_back(i);
    F.id_map = undel;
    F.id_map.insert(F.id_map.end(), undel.begin(), undel.end());
    extra = static_cast<int32_t>(undel.size());
  } else {
    F.id_map.resize(std::max<int32_t>(n_ids, 0));
    for (int32_t i = 0; i < n_ids; ++i) F.id_map[i] = i;
  }
  const int32_t R = R0 + extra;
  F.width = W;
  F.rows = R > 0 ? R - 1 : 0;
  F.encoded.assign(static_cast<size_t>(R) * W, 4);
  for (int32_t r = 0; r < R0; ++r) {
    const std::string& row = msa[r];
    if (static_cast<int32_t>(row.size()) != W) throw SvsError(SVS_E_INTERNAL, "MSA rows of unequal width");
    uint8_t* e = F.encoded.data() + static_cast<size_t>(r) * W;
    for (int32_t c = 0; c < W; ++c) {
      const uint8_t v = kCodes.enc[static_cast<unsigned char>(row[c])];
      if (v == 255)
        throw SvsError(SVS_E_INVALID, std::string("SeqEncoder: symbol '") + row[c] +
                                          "' is not in {A,T,C,G,-} (the reference raises KeyError)");
      e[c] = v;
    }
  }
  // columns outside the flank margins, then FindNonSameSite (:167-179) over rows 1..R-1
  std::vector<int32_t> cols;
  if (R0 > 0) {
    const std::vector<uint8_t> pool = call_margin(msa[0], flank_5, flank_3);
    for (int32_t c = 0; c < W; ++c)
      if (!pool[c]) cols.push_back(c);
  } else {
    for (int32_t c = 0; c < W; ++c) cols.push_back(c);
  }
  const double cutoff = std::max(static_cast<double>(hcutoff), static_cast<double>(R) * scutoff);
  std::vector<int32_t> keep;
  std::vector<int32_t> cnt(5 * cols.size(), 0);
  for (int32_t r = 1; r < R; ++r) {
    const uint8_t* e = F.encoded.data() + static_cast<size_t>(r) * W;
    for (size_t k = 0; k < cols.size(); ++k) ++cnt[5 * k + e[cols[k]]];
  }
  for (size_t k = 0; k < cols.size(); ++k) {
    int32_t a[5];
    std::copy(cnt.begin() + 5 * k, cnt.begin() + 5 * k + 5, a);
    std::sort(a, a + 5);
    if (static_cast<double>(a[3]) >= cutoff) keep.push_back(cols[k]);
  }
  F.n_feat = static_cast<int32_t>(keep.size());
  F.feat.resize(static_cast<size_t>(F.rows) * F.n_feat);
  for (int32_t r = 0; r < F.rows; ++r) {
    const uint8_t* e = F.encoded.data() + static_cast<size_t>(r + 1) * W;
    uint8_t* o = F.feat.data() + static_cast<size_t>(r) * F.n_feat;
    for (int32_t k = 0; k < F.n_feat; ++k) o[k] = e[keep[k]];
  }
}

bool plan_clusters(const WindowFeatures& f, const int32_t* rclust, const uint8_t* is_tlabel, int32_t readcutoff,
                   std::vector<ClusterPlan>* som, std::vector<ClusterPlan>* germ) {
  som->clear();
  germ->clear();
  std::vector<int32_t> labels(rclust, rclust + f.rows);
  std::sort(labels.begin(), labels.end());
  labels.erase(std::unique(labels.begin(), labels.end()), labels.end());
  const int32_t n_ids = static_cast<int32_t>(f.id_map.size());
  for (int32_t L : labels) {
    ClusterPlan p;
    bool all_t = true;
    for (int32_t r = 0; r < f.rows; ++r) {
      if (rclust[r] != L) continue;
      if (r >= n_ids) return false;  // np.array(ReadIDs)[idx] -> IndexError
      p.rows.push_back(r);
      p.ids.push_back(f.id_map[r]);
      all_t = all_t && is_tlabel[f.id_map[r]];
    }
    const bool big = static_cast<int32_t>(p.rows.size()) >= readcutoff;
    if (!big) continue;
    p.som = all_t;
    // SeqDecoder(seqencode_New[idx + 1]): ungapped, upper-case
    size_t longest = 0;
    for (int32_t r : p.rows) {
      const uint8_t* e = f.encoded.data() + static_cast<size_t>(r + 1) * f.width;
      std::string s;
      for (int32_t c = 0; c < f.width; ++c)
        if (e[c] != 4) s.push_back(kDecode[e[c]]);
      longest = std::max(longest, s.size());
      p.reads.push_back(std::move(s));
    }
    if (longest == 0) p.reads.clear();  // consensus stays "-"
    (p.som ? som : germ)->push_back(std::move(p));
  }
  return true;
}

}  // namespace svs
