// Feature selection + cluster labelling on the host (see features.hpp).
#include "features.hpp"

#include <algorithm>
#include <cmath>

#include "../../include/svscope.h"
#include "poa_dgraph.hpp"
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

// The full-DEL read quirk (DataScanner.py:195-208): with a zero-length read
// the returned ids become UnDEL + UnDEL and the encoding gains one all-gap row
// per UnDEL id.  Fills id_map; returns the number of all-gap rows.
int32_t feature_id_map(const std::vector<int32_t>& read_lens, int32_t n_ids, std::vector<int32_t>* id_map) {
  bool has_del = false;
  for (int32_t len : read_lens) has_del = has_del || len == 0;
  id_map->clear();
  if (!has_del) {
    id_map->resize(std::max<int32_t>(n_ids, 0));
    for (int32_t i = 0; i < n_ids; ++i) (*id_map)[i] = i;
    return 0;
  }
  std::vector<uint8_t> is_del(std::max<int32_t>(n_ids, 0), 0);
  for (size_t i = 0; i < read_lens.size(); ++i)
    if (read_lens[i] == 0 && static_cast<int32_t>(i) < n_ids) is_del[i] = 1;
  std::vector<int32_t> undel;
  for (int32_t i = 0; i < n_ids; ++i)
    if (!is_del[i]) undel.push_back(i);
  *id_map = undel;
  id_map->insert(id_map->end(), undel.begin(), undel.end());
  return static_cast<int32_t>(undel.size());
}

std::string upper_acgt(const std::string& s) {
  std::string u(s);
  for (char& c : u) c = kDecode[kCodes.enc[static_cast<unsigned char>(c)]];
  return u;
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
  const int32_t extra = feature_id_map(read_lens, n_ids, &F.id_map);
  const int32_t R = R0 + extra;
  F.rows = R > 0 ? R - 1 : 0;
  std::vector<uint8_t> encoded(static_cast<size_t>(R) * W, 4);
  for (int32_t r = 0; r < R0; ++r) {
    const std::string& row = msa[r];
    if (static_cast<int32_t>(row.size()) != W) throw SvsError(SVS_E_INTERNAL, "MSA rows of unequal width");
    uint8_t* e = encoded.data() + static_cast<size_t>(r) * W;
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
    const uint8_t* e = encoded.data() + static_cast<size_t>(r) * W;
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
  F.row_reads.assign(F.rows, std::string());
  for (int32_t r = 0; r < F.rows; ++r) {
    const uint8_t* e = encoded.data() + static_cast<size_t>(r + 1) * W;
    uint8_t* o = F.feat.data() + static_cast<size_t>(r) * F.n_feat;
    for (int32_t k = 0; k < F.n_feat; ++k) o[k] = e[keep[k]];
    // SeqDecoder: ungapped, upper case
    std::string& s = F.row_reads[r];
    for (int32_t c = 0; c < W; ++c)
      if (e[c] != 4) s.push_back(kDecode[e[c]]);
  }
}

DeviceFeatureParams device_feature_params(const std::vector<std::string>& seqs, const std::string& flank_5,
                                          const std::string& flank_3, const std::vector<int32_t>& read_lens,
                                          int32_t n_ids, int32_t hcutoff, double scutoff) {
  DeviceFeatureParams p;
  const std::string* row0 = nullptr;
  for (const std::string& s : seqs) {
    for (const char c : s) {
      if (kCodes.enc[static_cast<unsigned char>(c)] == 255)
        throw SvsError(SVS_E_INVALID, std::string("SeqEncoder: symbol '") + c +
                                          "' is not in {A,T,C,G,-} (the reference raises KeyError)");
      if (c == '-') p.ok = false;
    }
    if (!s.empty()) {
      if (!row0) row0 = &s;
      ++p.msa_rows;
    }
  }
  // CallMargin (:146-165) on MSA row 0, whose letters are the first non-empty
  // sequence: the forward walk stops after |f5| letters when they spell f5
  // (else it keeps every row-0 column); the backward walk, over columns >= 1,
  // likewise for f3 when |f3| <= len - 1 (a longer f3 keeps every row-0
  // column >= 1 either way); an empty flank keeps every row-0 column unless
  // the walk's first column is a gap (decided on the device)
  const size_t L0 = row0 ? row0->size() : 0;
  const size_t k5 = flank_5.size(), k3 = flank_3.size();
  if (k5 == 0) p.f5_take = kTakeEmptyFlank;
  else if (k5 <= L0 && row0->compare(0, k5, flank_5) == 0) p.f5_take = static_cast<int32_t>(k5);
  else p.f5_take = kTakeAll;
  if (k3 == 0) p.f3_take = kTakeEmptyFlank;
  else if (k3 + 1 <= L0 && row0->compare(L0 - k3, k3, flank_3) == 0) p.f3_take = static_cast<int32_t>(k3);
  else p.f3_take = kTakeAll;
  std::vector<int32_t> id_map;
  p.extra = static_cast<uint32_t>(feature_id_map(read_lens, n_ids, &id_map));
  // FindNonSameSite (:167-179): second-largest count >= max(h, R s), R the
  // encoded rows; counts are integers, so >= the ceiling
  const double cutoff = std::max(static_cast<double>(hcutoff), static_cast<double>(p.msa_rows + p.extra) * scutoff);
  p.cut = cutoff <= 0.0 ? 0u : static_cast<uint32_t>(std::ceil(cutoff));
  return p;
}

void device_features(const std::vector<std::string>& seqs, const std::vector<int32_t>& read_lens, int32_t n_ids,
                     const DeviceFeatureParams& p, int32_t n_feat, std::vector<uint8_t>&& feat, WindowFeatures* out) {
  WindowFeatures& F = *out;
  feature_id_map(read_lens, n_ids, &F.id_map);
  const int32_t R = p.msa_rows + static_cast<int32_t>(p.extra);
  F.rows = R > 0 ? R - 1 : 0;
  F.n_feat = n_feat;
  if (feat.size() != static_cast<size_t>(F.rows) * n_feat)
    throw SvsError(SVS_E_INTERNAL, "device seqdatamx size differs from rows x features");
  F.feat = std::move(feat);
  // MSA row k's letters are the k-th non-empty sequence; the all-gap rows decode to ""
  F.row_reads.assign(F.rows, std::string());
  int32_t k = 0;
  for (const std::string& s : seqs) {
    if (s.empty()) continue;
    if (k >= 1 && k - 1 < F.rows) F.row_reads[k - 1] = upper_acgt(s);
    ++k;
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
      longest = std::max(longest, f.row_reads[r].size());
      p.reads.push_back(f.row_reads[r]);
    }
    if (longest == 0) p.reads.clear();  // consensus stays "-"
    (p.som ? som : germ)->push_back(std::move(p));
  }
  return true;
}

}  // namespace svs
