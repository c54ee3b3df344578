// Host restatement of the two third-party calls the reference makes between
// the similarity matrix and the EM initialisation (ReadsCluster.py:243 and :94):
//   Z = scipy.cluster.hierarchy.linkage(S, 'ward')        (S rows = observations)
//   T = scipy.cluster.hierarchy.fcluster(Z, K, 'maxclust') for K = 1..kmax-1
// scipy 1.15 is the pinned dependency; parity is checked bit-exact against the
// installed scipy in tests/test_ward_host.py (random, tied and degenerate inputs).
#pragma once
#include <cstdint>
#include <vector>

namespace svs {

// Linkage matrix rows (a, b, dist, size) after scipy's stable sort by dist and
// union-find relabelling, exactly as linkage(..., 'ward') returns them.
struct WardMerge {
  int32_t a, b;
  double dist;
  int32_t size;
};

// pdist(S, 'euclidean') + nn-chain ward + mergesort-by-distance + relabel.
// S is n x n row-major (n observations of n features).  out: n-1 merges.
void ward_linkage(const double* S, int n, std::vector<WardMerge>* out);

// fcluster(Z, K, 'maxclust') for K = 1..kmax-1; labels[(K-1)*n + i] in 1..K.
void maxclust_labels(const std::vector<WardMerge>& Z, int n, int kmax, int32_t* labels);

}  // namespace svs
