// Ward linkage + maxclust flat clusters on the host (see ward.hpp).
//
// Why host code: per window this is ~0.1 M flops of strictly sequential,
// data-dependent work (the nearest-neighbour chain), 64 observations at most
// in the reference's windows; it runs on the engine's thread pool while the
// GPU works on the other task group.  The numerics follow scipy's operation
// order so that labels (and thus the EM initialisation) are bit-identical:
//  * pdist euclidean: sequential sum of squared differences, then sqrt;
//  * ward Lance-Williams update
//      d(xy,i) = sqrt((ni+nx)/T d_xi^2 + (ni+ny)/T d_yi^2 - ni/T d_xy^2)
//    evaluated as ((ni+nx)*t)*d_xi*d_xi + ... with t = 1/(nx+ny+ni);
//  * nn-chain tie rules: strict '<', the previous chain element preferred;
//  * stable sort of merges by distance, union-find relabelling (n, n+1, ...);
//  * maxclust: the smallest cut threshold (a node's subtree-max distance, or
//    "below everything") giving at most K clusters; labels numbered in the
//    depth-first order scipy's cluster_monocrit walks the tree.
#include "ward.hpp"

#include <algorithm>
#include <cmath>
#include <limits>
#include <numeric>

#pragma STDC FP_CONTRACT OFF

namespace svs {

namespace {

inline int64_t cond_index(int n, int i, int j) {
  if (i > j) std::swap(i, j);
  return static_cast<int64_t>(n) * i - (static_cast<int64_t>(i) * (i + 1)) / 2 + (j - i - 1);
}

inline double ward_update(double d_xi, double d_yi, double d_xy, int nx, int ny, int ni) {
  const double t = 1.0 / static_cast<double>(nx + ny + ni);
  const double a = static_cast<double>(ni + nx) * t * d_xi * d_xi;
  const double b = static_cast<double>(ni + ny) * t * d_yi * d_yi;
  const double c = static_cast<double>(ni) * t * d_xy * d_xy;
  return std::sqrt(a + b - c);
}

}  // namespace

void ward_linkage(const double* S, int n, std::vector<WardMerge>* out) {
  out->clear();
  if (n < 2) return;
  std::vector<double> D(static_cast<size_t>(n) * (n - 1) / 2);
  for (int i = 0; i < n; ++i) {
    const double* xi = S + static_cast<size_t>(i) * n;
    for (int j = i + 1; j < n; ++j) {
      const double* xj = S + static_cast<size_t>(j) * n;
      double acc = 0.0;
      for (int k = 0; k < n; ++k) {
        const double d = std::fabs(xi[k] - xj[k]);
        acc = acc + d * d;
      }
      D[cond_index(n, i, j)] = std::sqrt(acc);
    }
  }
  std::vector<int> size(n, 1), chain(n);
  std::vector<WardMerge> Z(n - 1);
  int chain_len = 0;
  for (int k = 0; k < n - 1; ++k) {
    if (chain_len == 0) {
      for (int i = 0; i < n; ++i)
        if (size[i] > 0) {
          chain[0] = i;
          break;
        }
      chain_len = 1;
    }
    int x = 0, y = 0;
    double cur = 0.0;
    for (;;) {
      x = chain[chain_len - 1];
      if (chain_len > 1) {
        y = chain[chain_len - 2];
        cur = D[cond_index(n, x, y)];
      } else {
        cur = std::numeric_limits<double>::infinity();
      }
      for (int i = 0; i < n; ++i) {
        if (size[i] == 0 || i == x) continue;
        const double d = D[cond_index(n, x, i)];
        if (d < cur) {
          cur = d;
          y = i;
        }
      }
      if (chain_len > 1 && y == chain[chain_len - 2]) break;
      chain[chain_len++] = y;
    }
    chain_len -= 2;
    if (x > y) std::swap(x, y);
    const int nx = size[x], ny = size[y];
    Z[k] = WardMerge{x, y, cur, nx + ny};
    size[x] = 0;
    size[y] = nx + ny;
    for (int i = 0; i < n; ++i) {
      const int ni = size[i];
      if (ni == 0 || i == y) continue;
      D[cond_index(n, i, y)] = ward_update(D[cond_index(n, i, x)], D[cond_index(n, i, y)], cur, nx, ny, ni);
    }
  }
  std::stable_sort(Z.begin(), Z.end(), [](const WardMerge& p, const WardMerge& q) { return p.dist < q.dist; });
  // union-find relabelling: a merged cluster gets id n, n+1, ... in row order
  std::vector<int> parent(2 * n - 1);
  std::iota(parent.begin(), parent.end(), 0);
  std::vector<int> csize(2 * n - 1, 1);
  auto find = [&](int v) {
    int r = v;
    while (parent[r] != r) r = parent[r];
    while (parent[v] != r) {
      const int p = parent[v];
      parent[v] = r;
      v = p;
    }
    return r;
  };
  int next = n;
  for (int k = 0; k < n - 1; ++k) {
    int rx = find(Z[k].a), ry = find(Z[k].b);
    if (rx > ry) std::swap(rx, ry);
    Z[k].a = rx;
    Z[k].b = ry;
    parent[rx] = next;
    parent[ry] = next;
    csize[next] = csize[rx] + csize[ry];
    Z[k].size = csize[next];
    ++next;
  }
  *out = std::move(Z);
}

namespace {

// Number of flat clusters when every node whose subtree-max distance is <= t
// becomes a cluster (t = -inf: all singletons).
int count_clusters(const std::vector<WardMerge>& Z, const std::vector<double>& mc, int n, double t) {
  int nc = 0;
  std::vector<int> stack;
  stack.push_back(2 * n - 2);
  while (!stack.empty()) {
    const int node = stack.back();
    stack.pop_back();
    if (node < n) {
      ++nc;
      continue;
    }
    const int r = node - n;
    if (mc[r] <= t) {
      ++nc;
      continue;
    }
    stack.push_back(Z[r].a);
    stack.push_back(Z[r].b);
  }
  return nc;
}

// scipy cluster_monocrit walk: non-leaf children are descended left first;
// a node's leaf children are labelled when the node is left.
void label_monocrit(const std::vector<WardMerge>& Z, const std::vector<double>& mc, int n, double t,
                    int32_t* T) {
  std::vector<int> cur(n);
  std::vector<uint8_t> visited(2 * n - 1, 0);
  int k = 0, n_cluster = 0, leader = -1;
  cur[0] = 2 * n - 2;
  while (k >= 0) {
    const int root = cur[k] - n;
    const int lc = Z[root].a, rc = Z[root].b;
    if (leader == -1 && mc[root] <= t) {
      leader = root;
      ++n_cluster;
    }
    if (lc >= n && !visited[lc]) {
      visited[lc] = 1;
      cur[++k] = lc;
      continue;
    }
    if (rc >= n && !visited[rc]) {
      visited[rc] = 1;
      cur[++k] = rc;
      continue;
    }
    if (lc < n) {
      if (leader == -1) ++n_cluster;
      T[lc] = n_cluster;
    }
    if (rc < n) {
      if (leader == -1) ++n_cluster;
      T[rc] = n_cluster;
    }
    if (leader == root) leader = -1;
    --k;
  }
}

}  // namespace

void maxclust_labels(const std::vector<WardMerge>& Z, int n, int kmax, int32_t* labels) {
  if (kmax <= 1) return;
  if (n == 1) {
    for (int K = 1; K < kmax; ++K) labels[K - 1] = 1;
    return;
  }
  // subtree-max merge distance per node (children rows precede parents)
  std::vector<double> mc(n - 1);
  for (int r = 0; r < n - 1; ++r) {
    double m = Z[r].dist;
    if (Z[r].a >= n) m = std::max(m, mc[Z[r].a - n]);
    if (Z[r].b >= n) m = std::max(m, mc[Z[r].b - n]);
    mc[r] = m;
  }
  // candidate thresholds in ascending order: "below everything" (all
  // singletons) then each distinct subtree-max value
  std::vector<double> cand(mc);
  std::sort(cand.begin(), cand.end());
  cand.erase(std::unique(cand.begin(), cand.end()), cand.end());
  cand.insert(cand.begin(), -std::numeric_limits<double>::infinity());
  std::vector<int> nc(cand.size());
  nc[0] = n;
  for (size_t i = 1; i < cand.size(); ++i) nc[i] = count_clusters(Z, mc, n, cand[i]);
  for (int K = 1; K < kmax; ++K) {
    size_t pick = cand.size() - 1;
    for (size_t i = 0; i < cand.size(); ++i)
      if (nc[i] <= K) {
        pick = i;
        break;
      }
    label_monocrit(Z, mc, n, cand[pick], labels + static_cast<size_t>(K - 1) * n);
  }
}

}  // namespace svs
