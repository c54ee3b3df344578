// MI355X (gfx950) device half of the POA graph (poa_dgraph.hpp): the
// per-alignment graph update, topological sort and row export, and the
// heaviest-bundle consensus + MSA rows of a finished task.
//
// Replaces, for the device-resident graphs, what PoaGraph (poa_graph.cpp)
// does on the host after every alignment: spoa 4.x Graph::AddAlignment,
// Graph::TopologicalSort, the row export of the strip kernel's tables, and at
// the end Graph::GenerateMultipleSequenceAlignment / GenerateConsensus, all
// reached by the reference through `poa(seqs, 1)` (DataScanner.py:206,213,
// DecisionMaker.py:160,171).  Results are identical to the host graph's, which
// the engine can check table for table (SVS_POA_VERIFY_GRAPH=1).
//
// One wave per task and launch.  The work is latency-bound and mostly
// sequential (a DFS, a heaviest-path scan), so the kernels are built to share
// the CUs with the other task group's DP kernel, which they run beside on a
// stream of their own: one wave per workgroup, no LDS in the update, a few KB
// in the sort (two bit planes of node flags and the top of the DFS stack).
//   poa_fold_update_kernel  AddAlignment: the alignment's nodes (matches,
//       aligned-group members, new nodes; node ids in spoa's creation order),
//       edges (existing ones gain weight), then both CSR adjacency lists
//       rebuilt with each node's new edge appended (spoa's push_back order)
//   poa_fold_sort_kernel    DFS topological sort (spoa's order), then either
//       the next alignment's lite tables (export_strip_lite) or, for a finished
//       task, the consensus and the MSA rows
#include <hip/hip_runtime.h>
#include <cstdint>

#include "poa_dgraph.hpp"
#include "svs_device.hpp"

namespace svs {

namespace {

constexpr uint32_t kNone = 0xFFFFFFFFu;

// Pointers into a task block are global memory: say so, or every access is a
// flat one (generic address, counted in both vmcnt and lgkmcnt, never scalar).
#define GLB __attribute__((address_space(1)))
typedef GLB uint32_t gu32;
typedef GLB int32_t gi32;
typedef GLB uint8_t gu8;
typedef GLB char gch;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
template <class T> __device__ __forceinline__ GLB T* glb(T* p) { return (GLB T*)(p); }
template <class T> __device__ __forceinline__ const GLB T* glb(const T* p) { return (const GLB T*)(p); }

__device__ __forceinline__ uint32_t uni(uint32_t x) { return __builtin_amdgcn_readfirstlane(x); }
__device__ __forceinline__ uint32_t lanei() { return threadIdx.x & 63u; }
__device__ __forceinline__ uint64_t below() { return (1ull << lanei()) - 1ull; }
__device__ __forceinline__ uint32_t popc64(uint64_t m) { return static_cast<uint32_t>(__builtin_popcountll(m)); }
__device__ __forceinline__ uint64_t ballot(bool p) { return __builtin_amdgcn_ballot_w64(p); }
__device__ __forceinline__ uint32_t lane_val(uint32_t v, uint32_t l) {
  return static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int32_t>(v), static_cast<int32_t>(l)));
}

// Loads past the vector L1 (agent scope): for words this wave stored earlier
// in the same kernel (the L1 may still hold the line from before the store).
__device__ __forceinline__ uint32_t ldc(const gu32* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int32_t ldci(const gi32* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t ldc_u8(const gu8* base, uint32_t i) {
  const uint32_t w = ldc(reinterpret_cast<const gu32*>(base) + (i >> 2));
  return (w >> (8 * (i & 3u))) & 0xFFu;
}
// This wave's stores done, and its L1 invalidated, so that plain loads after
// it see them.
__device__ __forceinline__ void wave_sync_mem() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
  __builtin_amdgcn_s_waitcnt(0);
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
}

__device__ __forceinline__ uint32_t wave_add(uint32_t x) {
  for (int o = 32; o >= 1; o >>= 1) x += __shfl_xor(x, o, 64);
  return x;
}
__device__ __forceinline__ uint32_t wave_max(uint32_t x) {
  for (int o = 32; o >= 1; o >>= 1) x = max(x, static_cast<uint32_t>(__shfl_xor(x, o, 64)));
  return x;
}
__device__ __forceinline__ uint32_t wave_min(uint32_t x) {
  for (int o = 32; o >= 1; o >>= 1) x = min(x, static_cast<uint32_t>(__shfl_xor(x, o, 64)));
  return x;
}
__device__ __forceinline__ int32_t wave_min_i(int32_t x) {
  for (int o = 32; o >= 1; o >>= 1) x = min(x, __shfl_xor(x, o, 64));
  return x;
}
__device__ __forceinline__ int32_t wave_max_i(int32_t x) {
  for (int o = 32; o >= 1; o >>= 1) x = max(x, __shfl_xor(x, o, 64));
  return x;
}
// exclusive prefix sum over the wave; *total = the sum of all lanes
__device__ __forceinline__ uint32_t wave_excl(uint32_t x, uint32_t* total) {
  uint32_t s = x;
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(s, o, 64);
    if (static_cast<int>(lanei()) >= o) s += y;
  }
  *total = uni(__shfl(s, 63, 64));
  return s - x;
}

// The block's arrays (poa_dgraph.hpp layout); b = CSR buffer.
struct GPtr {
  gu8* base;
  gu32* al;
  gu32 *in_off, *in_nbr, *in_eid, *out_off, *out_nbr, *out_eid;
  gu32* ew;
  gu32 *nin, *nout, *nrec, *r2n, *n2r, *col, *last, *pstart, *pred, *info, *stk;
  gu32* chg;
  gu32 *seg, *seg_other;  // segment-start plane of buffer b, of 1 - b
};

__device__ __forceinline__ GPtr gptr(uint8_t* blk, uint32_t cv, uint32_t ce, uint32_t b) {
  const DGraphLayout L = dgraph_layout(cv, ce);
  GPtr g;
  gu8* gb = glb(blk);
  auto u = [&](size_t off) { return reinterpret_cast<gu32*>(gb + off); };
  g.base = gb + L.base;
  g.al = u(L.al);
  // (selects, not a dynamic index: the layout stays in registers)
  g.in_off = u(b ? L.in_off[1] : L.in_off[0]);
  g.in_nbr = u(b ? L.in_nbr[1] : L.in_nbr[0]);
  g.in_eid = u(b ? L.in_eid[1] : L.in_eid[0]);
  g.out_off = u(b ? L.out_off[1] : L.out_off[0]);
  g.out_nbr = u(b ? L.out_nbr[1] : L.out_nbr[0]);
  g.out_eid = u(b ? L.out_eid[1] : L.out_eid[0]);
  g.ew = u(L.ew);
  g.nin = u(L.nin);
  g.nout = u(L.nout);
  g.nrec = u(L.nrec);
  g.r2n = u(L.r2n);
  g.n2r = u(L.n2r);
  g.col = u(L.col);
  g.last = u(L.last);
  g.pstart = u(L.pstart);
  g.pred = u(L.pred);
  g.info = u(L.info);
  g.stk = u(L.stk);
  g.chg = u(L.chg);
  g.seg = u(b ? L.seg[1] : L.seg[0]);
  g.seg_other = u(b ? L.seg[0] : L.seg[1]);
  return g;
}

// One CSR list (in or out) rebuilt into buffer b1 from b0 for nodes
// 0 .. V1-1, each node's new entry (nw[2v] = eid, nw[2v+1] = neighbour, eid
// kNone = none) appended; the new-entry slots are reset.  For the in-list
// (nrec given) also every node's sort record (poa_dgraph.hpp) and the changed
// plane chg: a node of the old graph whose in-edge list gained an entry or
// whose aligned list grew (the record's aligned count differs), and every new
// node.  Returns the number of new entries found.
//
// Per 64-node chunk the old entries are moved edge-parallel, 64 per store:
// an old entry x of node v moves by the chunk's running offset plus one for
// every node u < v of the chunk that gains an entry (u's new entry goes at the
// end of u's list), i.e. every such u whose old list ends at or before x (a
// per-node loop over each node's entries had the lanes wait on one
// dependent load after another: 68 % of the update kernel's clocks).
__device__ uint32_t rebuild_csr(uint32_t V0, uint32_t V1, const gu32* __restrict__ off0,
                                const gu32* __restrict__ nbr0, const gu32* __restrict__ eid0, gu32* __restrict__ off1,
                                gu32* __restrict__ nbr1, gu32* __restrict__ eid1, gu32* __restrict__ nw,
                                gu32* __restrict__ nrec, const gu32* __restrict__ al, gu32* __restrict__ chg) {
  const uint32_t lane = lanei();
  uint32_t run = 0, found = 0;
  for (uint32_t v0 = 0; v0 < V1; v0 += 64) {
    const uint32_t v = v0 + lane;
    uint32_t a = 0, d = 0, ne = kNone, nb = 0;
    if (v < V1) {
      if (v < V0) {
        a = off0[v];
        d = off0[v + 1] - a;
      }
      ne = nw[2 * v];
      nb = nw[2 * v + 1];
    }
    const uint32_t has = ne != kNone ? 1u : 0u;
    uint32_t tot;
    const uint32_t o = run + wave_excl(d + has, &tot);
    if (v0 < V0) {
      // the chunk's old entries [xa, xb), contiguous in both buffers but for
      // the new entries that land between them
      const uint32_t nold = min(64u, V0 - v0);
      const uint32_t xa = lane_val(a, 0), xb = lane_val(a + d, nold - 1u);
      const uint64_t hm = ballot(has != 0u && v < V0);
      const uint32_t end = a + d;  // node v's old list ends here
      for (uint32_t x0 = xa; x0 < xb; x0 += 64u) {
        const uint32_t x = x0 + lane;
        uint32_t s = run - xa;
        for (uint64_t m = hm; m; m &= m - 1u) s += x >= lane_val(end, static_cast<uint32_t>(__builtin_ctzll(m))) ? 1u : 0u;
        if (x < xb) {
          nbr1[x + s] = nbr0[x];
          eid1[x + s] = eid0[x];
        }
      }
    }
    bool changed = true;
    if (v < V1) {
      off1[v] = o;
      if (has) {
        nbr1[o + d] = nb;
        eid1[o + d] = ne;
        nw[2 * v] = kNone;
      }
      if (nrec) {
        auto tail = [&](uint32_t k) -> uint32_t { return k < d ? nbr0[a + k] : (k == d && has ? nb : 0u); };
        const u32x4 alw = *reinterpret_cast<const GLB u32x4*>(al + 4 * v);
        GLB u32x4* nr = reinterpret_cast<GLB u32x4*>(nrec + 8 * v);
        if (v < V0) changed = has || (nrec[8 * v + 1] >> 24) != alw.x;
        nr[0] = u32x4{o, (d + has) | (alw.x << 24), alw.y, alw.z};
        nr[1] = u32x4{alw.w, tail(0), tail(1), tail(2)};
      }
    }
    if (nrec) {
      const uint64_t cm = ballot(v < V1 && changed);
      if (lane < 2u) chg[(v0 >> 5) + lane] = static_cast<uint32_t>(lane ? cm >> 32 : cm);
    }
    found += wave_add(has);
    run += tot;
  }
  if (lane == 0) off1[V1] = run;
  return uni(found);
}

}  // namespace

// The fold kernels run one wave per job beside the DP kernel's waves on the
// same SIMDs and sit on the chain DP -> fold -> next DP of their group: they
// issue ahead of the DP waves (s_setprio), which only wait on them.
#ifndef SVS_FOLD_PRIO_LEVEL
#define SVS_FOLD_PRIO_LEVEL 3
#endif
#define SVS_FOLD_PRIO() __builtin_amdgcn_s_setprio(SVS_FOLD_PRIO_LEVEL)

// ---------------------------------------------------------------- update
// spoa Graph::AddAlignment (poa_graph.cpp add_alignment_nodes): nodes of the
// prefix chain, then the suffix chain, then the middle's new nodes in path
// order; a middle position takes its aligned node when the letters match, else
// a member of that node's aligned group with its letter, else a new node that
// joins the group (spoa's aligned_nodes order: the anchor's list, then the
// anchor; every member appends the newcomer).  Then one edge per consecutive
// path pair, existing ones gaining weight.
__global__ __launch_bounds__(64) void poa_fold_update_kernel(const FoldJob* __restrict__ jobs) {
  SVS_FOLD_PRIO();
  const uint64_t T0 = __builtin_amdgcn_s_memrealtime();
  const FoldJob J = jobs[blockIdx.x];
  const uint32_t lane = lanei();
  GLB FoldResult* res = glb(J.result);
  int32_t n = 0;
  if (!(J.flags & kFoldChain)) {
    n = *glb(J.aln_status);
    if (n == kPruneRetry) {
      if (lane == 0) res->status = kFoldSkipped;
      return;
    }
    if (n < 0) {
      if (lane == 0) res->status = kFoldErrAln;
      return;
    }
  }
  const uint32_t V0 = J.V, E0 = J.E, len = J.len;
  const uint32_t b0 = J.par, b1 = 1u - J.par;
  const GPtr g = gptr(J.blk, J.cv, J.ce, b0);
  const GPtr h = gptr(J.blk, J.cv, J.ce, b1);
#ifdef SVS_FOLD_PROF_UPD
  // development builds: clocks of the update's phases into prof[0..3] (middle,
  // edges, in-list rebuild, out-list rebuild)
  uint64_t pu = __builtin_readcyclecounter();
  uint32_t pud[4] = {0, 0, 0, 0};
  auto pmark = [&](int k) {
    const uint64_t t = __builtin_readcyclecounter();
    pud[k] = static_cast<uint32_t>((t - pu) >> 10);
    pu = t;
  };
#else
  auto pmark = [](int) {};
#endif
  gu32* __restrict__ path = glb(J.paths) + glb(J.path_off)[J.n_paths];
  const gu8* __restrict__ seq = glb(J.seq);
  const gi32* __restrict__ aln = glb(J.aln);
  auto fail = [&](int32_t st) {
    if (lane == 0) res->status = st;
  };
  if (V0 + len > J.cv || E0 + len + 1 > J.ce) return fail(kFoldErrCapacity);

  // first / last aligned read position (positions increase along the path)
  int32_t first = static_cast<int32_t>(len), last = static_cast<int32_t>(len) - 1;
  if (n > 0) {
    int32_t mn = INT32_MAX, mx = -1;
    for (int32_t c0 = 0; c0 < n; c0 += 64) {
      const int32_t i = c0 + static_cast<int32_t>(lane);
      if (i < n) {
        const int32_t pos = aln[2 * (n - 1 - i) + 1];
        if (pos >= 0) {
          mn = min(mn, pos);
          mx = max(mx, pos);
        }
      }
    }
    mn = wave_min_i(mn);
    mx = wave_max_i(mx);
    if (mx < 0 || mx >= static_cast<int32_t>(len)) return fail(kFoldErrPath);
    first = mn;
    last = mx;
  }
  const uint32_t nsuf = len - 1u - static_cast<uint32_t>(last);
  // prefix and suffix chains: fresh nodes V0 .. V0 + first - 1, then the suffix's
  auto fresh = [&](uint32_t id, uint32_t p) {
    g.base[id] = seq[p];
    g.al[4 * id] = 0;
    g.nin[2 * id] = kNone;
    g.nout[2 * id] = kNone;
    path[p] = id;
  };
  for (uint32_t p = lane; p < static_cast<uint32_t>(first); p += 64) fresh(V0 + p, p);
  for (uint32_t p = static_cast<uint32_t>(last) + 1 + lane; p < len; p += 64)
    fresh(V0 + static_cast<uint32_t>(first) + (p - static_cast<uint32_t>(last) - 1), p);
  uint32_t next = V0 + static_cast<uint32_t>(first) + nsuf;

  // the middle, 64 forward pairs at a time
  for (int32_t c0 = 0; c0 < n; c0 += 64) {
    const int32_t i = c0 + static_cast<int32_t>(lane);
    int32_t row = -1, pos = -1;
    if (i < n) {
      row = aln[2 * (n - 1 - i)];
      pos = aln[2 * (n - 1 - i) + 1];
    }
    const bool act = pos >= 0;
    const uint32_t letter = act ? seq[pos] : 0u;
    uint32_t nn = kNone, cur = kNone;
    // kinds: matched (cur known), insertion (a new node), mismatch (resolved in order below)
    bool ins = false, mis = false, bad = false;
    if (act) {
      if (row < 0) {
        ins = true;
      } else if (static_cast<uint32_t>(row) >= V0) {
        bad = true;
      } else {
        nn = g.r2n[row];
        if (g.base[nn] == letter) cur = nn;  // an old node's letter: never written by this kernel
        else mis = true;
      }
    }
    if (ballot(bad)) return fail(kFoldErrAln);
    const uint64_t ins_m = ballot(ins);
    uint64_t mis_m = ballot(mis), creat_m = 0;
    uint32_t created = 0;
    // mismatches in path order: the aligned group as updated so far (coherent loads)
    while (mis_m) {
      const uint32_t j = static_cast<uint32_t>(__builtin_ctzll(mis_m));
      mis_m &= mis_m - 1;
      const uint32_t nj = lane_val(nn, j), lt = lane_val(letter, j);
      __builtin_amdgcn_s_waitcnt(0);  // this wave's earlier group updates have landed
      const uint32_t cnt = uni(ldc(g.al + 4 * nj));
      if (cnt > 3) return fail(kFoldErrAligned);
      uint32_t mem[3] = {0, 0, 0};
      uint32_t found = kNone;
      for (uint32_t k = 0; k < cnt; ++k) {
        mem[k] = uni(ldc(g.al + 4 * nj + 1 + k));
        if (found == kNone && uni(ldc_u8(g.base, mem[k])) == lt) found = mem[k];
      }
      uint32_t cj = found;
      if (found == kNone) {
        if (cnt >= 3) return fail(kFoldErrAligned);  // a fifth letter in one column
        const uint64_t bj = (1ull << j) - 1ull;
        cj = next + popc64(ins_m & bj) + created;
        ++created;
        creat_m |= 1ull << j;
        if (lane == 0) {
          g.base[cj] = static_cast<uint8_t>(lt);
          g.nin[2 * cj] = kNone;
          g.nout[2 * cj] = kNone;
          // newcomer's list: the anchor's list, then the anchor
          g.al[4 * cj] = cnt + 1;
          for (uint32_t k = 0; k < cnt; ++k) g.al[4 * cj + 1 + k] = mem[k];
          g.al[4 * cj + 1 + cnt] = nj;
        }
        // every member, then the anchor, appends the newcomer
        for (uint32_t k = 0; k <= cnt; ++k) {
          const uint32_t a = k < cnt ? mem[k] : nj;
          const uint32_t ca = uni(ldc(g.al + 4 * a));
          if (ca >= 3) return fail(kFoldErrAligned);
          if (lane == 0) {
            g.al[4 * a + 1 + ca] = cj;
            g.al[4 * a] = ca + 1;
          }
          __builtin_amdgcn_s_waitcnt(0);
        }
      }
      if (lane == j) cur = cj;
    }
    if (ins) {
      cur = next + popc64(ins_m & below()) + popc64(creat_m & below());
      g.base[cur] = static_cast<uint8_t>(letter);
      g.al[4 * cur] = 0;
      g.nin[2 * cur] = kNone;
      g.nout[2 * cur] = kNone;
    }
    next += popc64(ins_m) + created;
    if (act) path[pos] = cur;
  }
  if (next > J.cv || next - V0 > len) return fail(kFoldErrCapacity);
  wave_sync_mem();
  pmark(0);

  // edges along the path: existing ones gain weight, new ones are recorded at
  // their head (nin) and tail (nout) for the CSR rebuild
  uint32_t E1 = E0;
  for (uint32_t c0 = 0; c0 + 1 < len; c0 += 64) {
    const uint32_t p = c0 + lane;
    const bool inb = p + 1 < len;
    uint32_t prev = 0, cur = 0, eid = kNone;
    if (inb) {
      prev = path[p];
      cur = path[p + 1];
      if (prev < V0 && cur < V0) {
        const uint32_t a = g.out_off[prev], b = g.out_off[prev + 1];
        for (uint32_t x = a; x < b; ++x)
          if (g.out_nbr[x] == cur) {
            eid = g.out_eid[x];
            break;
          }
      }
    }
    const bool isnew = inb && eid == kNone;
    const uint64_t nm = ballot(isnew);
    if (isnew) {
      eid = E1 + popc64(nm & below());
      g.ew[eid] = 1;
      g.nin[2 * cur] = eid;
      g.nin[2 * cur + 1] = prev;
      g.nout[2 * prev] = eid;
      g.nout[2 * prev + 1] = cur;
    } else if (inb) {
      g.ew[eid] += 1;
    }
    E1 += popc64(nm);
  }
  wave_sync_mem();
  pmark(1);
  const uint32_t V1 = next;
  // both adjacency lists into the other buffer, the new edge of each node last
  const uint32_t fin =
      rebuild_csr(V0, V1, g.in_off, g.in_nbr, g.in_eid, h.in_off, h.in_nbr, h.in_eid, g.nin, g.nrec, g.al, g.chg);
  pmark(2);
  const uint32_t fout =
      rebuild_csr(V0, V1, g.out_off, g.out_nbr, g.out_eid, h.out_off, h.out_nbr, h.out_eid, g.nout, nullptr, nullptr,
                  nullptr);
  pmark(3);
  // a node twice on the path would have lost one of its new edges
  if (fin != E1 - E0 || fout != E1 - E0) return fail(kFoldErrPath);
  if (lane == 0) {
#ifdef SVS_FOLD_PROF_UPD
    for (int k = 0; k < 4; ++k) res->prof[k] = pud[k];
#endif
    res->status = kFoldOk;
    res->V = V1;
    res->E = E1;
    res->t_upd = static_cast<uint32_t>(__builtin_amdgcn_s_memrealtime() - T0);
  }
}

// ---------------------------------------------------------------- sort
// spoa Graph::TopologicalSort (poa_graph.cpp sort_ranks): roots in node-id
// order; a node on top of the stack pushes its unfinished in-edge tails (in
// in-edge order) and, unless it was itself pushed as an aligned node, its
// unfinished aligned nodes (flagging them); once nothing was pushed it is done
// and, unless flagged, emitted together with its aligned list, which also
// makes one MSA column.
//
// Node flags live in LDS (two bit planes), the stack's top in LDS (the rest
// spills to the block's stk array in blocks of half the LDS stack).
//
// Reuse of the previous sort.  Everything emitted between one root's start
// and the next root's is that root's segment of the rank order, and the
// segments tile it.  A root's DFS reads only the records of the nodes it
// emits, and flags that, at a root's start, only ever grow from one fold to
// the next (the done set is then the ancestor-and-aligned closure of every
// smaller id, and a fold only adds edges and aligned members).  So, walking
// the previous order segment by segment: a segment none of whose nodes the
// fold changed (chg) and none of whose nodes is done yet is emitted again
// unchanged; any other segment's root (its smallest id) runs the DFS unless
// it is done; and the new ids follow as roots in id order.  The result is
// spoa's order exactly; on the config-3 windows 91 % of the examinations are
// skipped (a host replay of spoa's sort with this walk, profiles/r05_s1).
namespace {

struct SortState {
  uint32_t* done;  // LDS bit plane
  uint32_t* ign;   // LDS bit plane
  const uint32_t* chg;  // LDS copy of the fold's changed plane (by node id)
  uint32_t* nseg;  // LDS bit plane by rank: the new segment starts
  uint32_t* st;    // LDS stack
  uint32_t cap;    // LDS stack entries (even)
  gu32* spill;     // global spill area
  uint32_t spilled;  // entries in the spill area (below the LDS part)
  uint32_t sp;       // entries in the LDS part
  uint32_t spill_cap;  // entries the spill area holds
  bool err;            // the stack outgrew its spill area
  uint32_t n_exam, n_roots;  // statistics
  uint32_t n_emit;           // nodes emitted (V unless the sort failed)
  uint64_t prof[4];          // SVS_FOLD_PROF: fast roots, DFS runs, window loads, rest (clocks)
};
#include "poa_fold_prof.hpp"  // development profile builds only; no-ops otherwise

// lane L of x replaced by the uniform s (one v_writelane_b32)
template <int L> __device__ __forceinline__ uint32_t write_lane_c(uint32_t x, uint32_t s) {
  asm("v_writelane_b32 %0, %1, %2" : "+v"(x) : "s"(s), "n"(L));
  return x;
}
#define write_lane(x, s, L) write_lane_c<L>((x), (s))

}  // namespace

// The sort, export and finalize helpers take the arrays as restrict
// parameters so the compiler can read the read-only ones through the scalar
// cache.
// V0: the node count before this fold (nodes >= V0 are the fold's new ones);
// r2n_old: the previous sort's rank order of nodes < V0 (a copy: r2n is
// overwritten as nodes are emitted); seg_old: the previous sort's segment
// starts (nullptr: no reuse, every root runs).
__device__ int32_t dfs_sort(uint32_t V, uint32_t V0, const gu32* __restrict__ nrec, const gu32* __restrict__ in_nbr,
                            gu32* __restrict__ r2n, gu32* __restrict__ n2r, const gu32* __restrict__ r2n_old,
                            gu32* __restrict__ col, const gu32* __restrict__ seg_old, SortState& S,
                            uint32_t* ncol_out) {
  const uint32_t lane = lanei();
  const uint32_t W = (V + 31u) >> 5;
  for (uint32_t w = lane; w < W; w += 64) {
    S.done[w] = 0;
    S.ign[w] = 0;
    S.nseg[w] = 0;
  }
  uint32_t cnt = 0, ncol = 0;
  // Uniform control throughout.  LDS operations of one wave complete in
  // order, so a bit set or a push is seen by the next read without a wait;
  // only the spill area (global memory) needs its stores drained.
  uint32_t top = 0;  // the entry last pushed
  // spill the lower half of the LDS part (S.sp >= half); false: no room
  auto spill_half = [&]() -> bool {
    const uint32_t half = S.cap / 2;
    if (S.spilled + half > S.spill_cap) {
      S.err = true;
      return false;
    }
    // (loops with uniform trip counts and predicated lanes: a loop whose
    // lanes leave at different trips makes the whole DFS loop divergent)
    for (uint32_t k0 = 0; k0 < half; k0 += 64) {
      const uint32_t k = k0 + lane;
      if (k < half) S.spill[S.spilled + k] = S.st[k];
    }
    for (uint32_t k0 = 0; k0 < half; k0 += 64) {
      const uint32_t k = k0 + lane;
      const uint32_t x = k < half ? S.st[k + half] : 0u;
      __builtin_amdgcn_wave_barrier();
      if (k < half) S.st[k] = x;
    }
    S.spilled += half;
    S.sp -= half;
    return true;
  };
  auto push = [&](uint32_t v) {
    if (S.sp == S.cap && !spill_half()) return;
    S.st[S.sp] = v;  // (every lane the same word: no divergent branch)
    ++S.sp;
    top = v;
  };
  // The lanes of pm push their val, in lane order (one store for all); the
  // highest one ends on top.
  auto push_lanes = [&](uint64_t pm, uint32_t val) {
    const uint32_t np = popc64(pm);
    if (np == 0) return;
    if (S.sp + np > S.cap && !spill_half()) return;  // (np <= 6, S.cap >= 64)
    if ((pm >> lane) & 1u) S.st[S.sp + popc64(pm & below())] = val;
    S.sp += np;
    top = lane_val(val, 63u - static_cast<uint32_t>(__builtin_clzll(pm)));
  };
  auto refill = [&]() {
    // the LDS part is empty: bring back up to half of it from the spill area
    const uint32_t half = S.cap / 2;
    const uint32_t k0 = S.spilled > half ? S.spilled - half : 0u, m = S.spilled - k0;
    __builtin_amdgcn_s_waitcnt(0);
    for (uint32_t j0 = 0; j0 < m; j0 += 64) {
      const uint32_t k = j0 + lane;
      if (k < m) S.st[k] = ldc(S.spill + k0 + k);
    }
    S.spilled = k0;
    S.sp = m;
  };
  // A flag set is an LDS atomic OR by every lane (no returned value to wait
  // for; a lane-0 branch would make the DFS loop divergent: values in vector
  // registers, control through exec masks).
  auto set_bit = [&](uint32_t* plane, uint32_t v) {
    __hip_atomic_fetch_or(plane + (v >> 5), 1u << (v & 31u), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  };
  // Emitted nodes collect in two registers (lane k: the k-th buffered node and
  // its column) and go out 64 at a time, one store per table per 64 nodes
  // (nothing reads an emitted node's entries during the sort).
  uint32_t eb_node = 0, eb_col = 0, eb_n = 0;
  // the buffered emissions out (positions cnt - eb_n ..): before any store
  // that advances cnt otherwise (the bulk path) and at the end
  auto flush_emit = [&]() {
    if (lane < eb_n) {
      const uint32_t rk = cnt - eb_n + lane;
      r2n[rk] = eb_node;
      n2r[eb_node] = rk;
      col[eb_node] = eb_col;
    }
    eb_n = 0;
  };
  auto emit = [&](uint32_t node) {
    const bool mine = lane == eb_n;  // (selects: lane eb_n takes the entry)
    eb_node = mine ? node : eb_node;
    eb_col = mine ? ncol : eb_col;
    ++cnt;
    if (++eb_n == 64u) {
      const uint32_t rk = cnt - 64u + lane;
      r2n[rk] = eb_node;
      n2r[eb_node] = rk;
      col[eb_node] = eb_col;
      eb_n = 0;
    }
  };
  // every examination pops or pushes: a bound on them stops a corrupt graph
  uint32_t steps = 0;
  const uint32_t max_steps = 64u * (V + S.spill_cap) + 4096u;
  auto done_of = [&](uint32_t v) -> uint32_t { return (S.done[v >> 5] >> (v & 31u)) & 1u; };
  // Node records come from two 64-node windows held in registers (lane l one
  // node's record): O holds 64 consecutive old nodes in the previous sort's
  // rank order, which the DFS follows closely (a node and the deep nodes it
  // reaches sit together there), found by comparing ids across the lanes; N
  // holds 64 consecutive new nodes by id (the fold's read adds them in path
  // order).  A miss loads a whole window with coalesced loads; a hit costs
  // lane reads only.
  uint32_t oid = kNone;  // lane: node id of the O window entry (kNone: empty)
  uint32_t bN = 0x80000000u;  // N window base (empty: no id < 2^31 is within 64 of it)
  uint32_t o0 = 0, o1 = 0, o2 = 0, o3 = 0, o4 = 0, o5 = 0, o6 = 0, o7 = 0;
  uint32_t d0w = 0, d1w = 0, d2w = 0, d3w = 0, d4w = 0, d5w = 0, d6w = 0, d7w = 0;
  auto load_rec = [&](uint32_t v, bool ok, uint32_t& w0, uint32_t& w1, uint32_t& w2, uint32_t& w3, uint32_t& w4,
                      uint32_t& w5, uint32_t& w6, uint32_t& w7) {
    const uint32_t u = ok ? v : 0u;
    const u32x4 x = *reinterpret_cast<const GLB u32x4*>(nrec + 8 * u);
    const u32x4 y = *reinterpret_cast<const GLB u32x4*>(nrec + 8 * u + 4);
    w0 = x.x; w1 = x.y; w2 = x.z; w3 = x.w;
    w4 = y.x; w5 = y.y; w6 = y.z; w7 = y.w;
  };
  // record of node v: off, in-degree | aligned count << 24, aligned list, first three tails
  auto record = [&](uint32_t v, uint32_t& off, uint32_t& w1, uint32_t& m0, uint32_t& m1, uint32_t& m2, uint32_t& t0,
                    uint32_t& t1, uint32_t& t2) {
    if (v >= V0) {
      if (v - bN >= 64u) {
        bN = v >= V0 + 32u ? v - 32u : V0;
        const uint32_t u = bN + lane;
        load_rec(u, u < V, d0w, d1w, d2w, d3w, d4w, d5w, d6w, d7w);
        SVS_PF_COUNT(2);
      }
      const uint32_t l = v - bN;
      off = lane_val(d0w, l); w1 = lane_val(d1w, l); m0 = lane_val(d2w, l); m1 = lane_val(d3w, l);
      m2 = lane_val(d4w, l); t0 = lane_val(d5w, l); t1 = lane_val(d6w, l); t2 = lane_val(d7w, l);
      return;
    }
    uint64_t hit = ballot(oid == v);
    if (!hit) {
      // the old rank of v (n2r still holds it: v is not emitted yet), a few
      // ranks of look-behind
      const uint32_t rk = uni(n2r[v]);
      const uint32_t b = rk > 8u ? rk - 8u : 0u;
      const uint32_t k = b + lane;
      oid = k < V0 ? r2n_old[k] : kNone;
      load_rec(oid, oid != kNone, o0, o1, o2, o3, o4, o5, o6, o7);
      SVS_PF_COUNT(3);
      hit = ballot(oid == v);
    }
    const uint32_t l = static_cast<uint32_t>(__builtin_ctzll(hit));
    off = lane_val(o0, l); w1 = lane_val(o1, l); m0 = lane_val(o2, l); m1 = lane_val(o3, l);
    m2 = lane_val(o4, l); t0 = lane_val(o5, l); t1 = lane_val(o6, l); t2 = lane_val(o7, l);
  };
  // The previous order's segment starts at ranks p .. p + 63 (bit l: rank
  // p + l); the end of the old order counts as a start.
  auto seg_window = [&](uint32_t p) -> uint64_t {
    const uint32_t a = p >> 5, s = p & 31u;
    const uint64_t lo = uni(seg_old[a]) | (static_cast<uint64_t>(uni(seg_old[a + 1])) << 32);
    const uint64_t hi = uni(seg_old[a + 2]);
    uint64_t m = s ? (lo >> s) | (hi << (64u - s)) : lo;
    const uint32_t left = V0 - p;
    if (left < 64u) m = (m & ((1ull << left) - 1ull)) | (1ull << left);
    return m;
  };
  auto next_start = [&](uint32_t q) -> uint32_t {  // the first segment start >= q
    while (q < V0) {
      const uint32_t w = uni(seg_old[q >> 5]) >> (q & 31u);
      if (w) return min(q + static_cast<uint32_t>(__builtin_ctz(w)), V0);
      q = (q | 31u) + 1u;
    }
    return V0;
  };
  // the fold changed node v, or it is emitted already
  auto bad_of = [&](uint32_t v) -> uint32_t { return ((S.chg[v >> 5] | S.done[v >> 5]) >> (v & 31u)) & 1u; };
  // a chunk of the previous order (lane: node nd, old column co; lanes < k)
  // emitted again at cnt + lane, columns shifted by ncol - c0; st: the
  // chunk's segment starts.  Returns the chunk's last old column.
  auto copy_ranks = [&](uint32_t nd, uint32_t co, uint32_t k, uint32_t c0, uint64_t st) -> uint32_t {
    if (lane < k) {
      r2n[cnt + lane] = nd;
      n2r[nd] = cnt + lane;
      col[nd] = ncol + co - c0;
      set_bit(S.done, nd);
      if ((st >> lane) & 1u) set_bit(S.nseg, cnt + lane);
    }
    return lane_val(co, k - 1u);
  };
  // Every node with an id below the current root is done (each root's DFS
  // finishes all it pushed), so flags are only read for larger ids and a root
  // whose tails and aligned nodes all have smaller ids is emitted at once,
  // with no stack and no flag access (its own done bit is then never read).
  // The root scan keeps its done word in a register while no DFS writes.
  uint32_t p = 0;                          // the walk's next segment start
  uint32_t scan = seg_old ? V0 : 0u;       // the root scan's next id
  uint32_t dwi = kNone, dwv = 0;
  while (!S.err) {
    uint32_t root;
    if (seg_old && p < V0) {
      // the previous order, 64 ranks at a time: every whole segment before
      // the first changed or done node is emitted again in one pass
      const uint32_t q = p + lane;
      const bool in = q < V0;
      const uint32_t nd = in ? r2n_old[q] : 0u;
      const uint64_t sm = seg_window(p);
      const uint64_t bad = ballot(in && bad_of(nd) != 0u);
      const uint64_t upto = bad ? (2ull << __builtin_ctzll(bad)) - 1ull : ~0ull;
      const uint64_t ends = sm & upto & ~1ull;
      if (ends) {
        const uint32_t k = 63u - static_cast<uint32_t>(__builtin_clzll(ends));
        flush_emit();
        const uint32_t co = col[nd];
        const uint32_t c0 = lane_val(co, 0);
        const uint32_t cl = copy_ranks(nd, co, k, c0, sm);
        cnt += k;
        ncol += cl + 1u - c0;
        p += k;
        continue;
      }
      // the segment at p is longer than the window or holds a bad node:
      // its end, its root, and whether it can still be copied
      const uint64_t rest = sm & ~1ull;
      const uint32_t e = rest ? p + static_cast<uint32_t>(__builtin_ctzll(rest)) : next_start(p + 64u);
      const uint32_t n0 = min(e - p, 64u);
      uint32_t r = uni(wave_min(lane < n0 ? nd : kNone));
      bool clean = (bad & (n0 < 64u ? (1ull << n0) - 1ull : ~0ull)) == 0;
      for (uint32_t c = p + 64u; c < e; c += 64u) {
        const uint32_t cq = c + lane;
        const uint32_t cn = cq < e ? r2n_old[cq] : kNone;
        clean = clean && ballot(cq < e && bad_of(cn) != 0u) == 0;
        r = min(r, uni(wave_min(cn)));
      }
      if (clean) {
        flush_emit();
        const uint32_t c0 = lane_val(col[nd], 0);
        uint32_t cl = c0;
        for (uint32_t c = p; c < e; c += 64u) {
          const uint32_t cq = c + lane;
          const uint32_t cn = cq < e ? r2n_old[cq] : 0u;
          cl = copy_ranks(cn, col[cn], min(e - c, 64u), c0, c == p ? 1ull : 0ull);
          cnt += min(e - c, 64u);
        }
        ncol += cl + 1u - c0;
        p = e;
        continue;
      }
      p = e;
      if (done_of(r)) continue;  // emitted by an earlier root's DFS
      root = r;
    } else {
      // the new ids (or, with no previous order, every id) in id order
      if (scan >= V) break;
      if ((scan >> 5) != dwi) {
        dwi = scan >> 5;
        dwv = uni(S.done[dwi]);
      }
      const uint32_t fw = ~dwv >> (scan & 31u);
      if (fw == 0) {
        scan = (scan | 31u) + 1u;
        continue;
      }
      scan += static_cast<uint32_t>(__builtin_ctz(fw));
      if (scan >= V) break;
      root = scan++;
    }
    ++S.n_roots;
    set_bit(S.nseg, cnt);  // root's segment starts here
    const uint64_t pf0 = SVS_PF_CLK();
    {
      uint32_t off, w1, m0, m1, m2, t0, t1, t2;
      record(root, off, w1, m0, m1, m2, t0, t1, t2);
      const uint32_t deg = w1 & 0xFFFFFFu, alc = w1 >> 24;
      if (deg <= 3u) {
        const bool fast = (deg < 1u || t0 < root) && (deg < 2u || t1 < root) && (deg < 3u || t2 < root) &&
                          (alc < 1u || m0 < root) && (alc < 2u || m1 < root) && (alc < 3u || m2 < root);
        if (fast) {
          ++steps;
          emit(root);
          if (alc > 0u) emit(m0);
          if (alc > 1u) emit(m1);
          if (alc > 2u) emit(m2);
          ++ncol;
          SVS_PF_ADD(0, pf0);
          continue;
        }
      }
    }
    dwi = kNone;  // the DFS below sets done bits
    push(root);
    uint32_t cur = root;
    while (!S.err) {
      if (++steps > max_steps) {
        S.err = true;
        break;
      }
      // the node record (register windows); then every flag the examination
      // needs in one batch of LDS reads
      uint32_t off, w1, m0, m1, m2, t0, t1, t2;
      [[maybe_unused]] const uint64_t px0 = SVS_PF_CLK();
      record(cur, off, w1, m0, m1, m2, t0, t1, t2);
      SVS_PF_EXAM(0, px0);
      [[maybe_unused]] const uint64_t px1 = SVS_PF_CLK();
      const uint32_t deg = w1 & 0xFFFFFFu, alc = w1 >> 24;
      // The eight flags in one vector read and one ballot: lane k < 3 tail k,
      // lanes 3..5 aligned node k - 3 (unused slots read cur's word and count
      // as done; ids below the root are done), lane 6 cur's done bit, lane 7
      // cur's ignore bit (was eight scalar address computations and reads).
      uint32_t fid = cur;
      fid = write_lane(fid, t0, 0);
      fid = write_lane(fid, t1, 1);
      fid = write_lane(fid, t2, 2);
      fid = write_lane(fid, m0, 3);
      fid = write_lane(fid, m1, 4);
      fid = write_lane(fid, m2, 5);
      const bool fused = lane < 3u ? lane < deg : (lane < 6u ? lane - 3u < alc : false);
      const uint32_t fv = fused ? fid : cur;
      const uint32_t* fplane = lane == 7u ? S.ign : S.done;
      const uint32_t fbit = (fplane[fv >> 5] >> (fv & 31u)) & 1u;
      const uint64_t fm = ballot(fbit != 0u || (lane < 6u && !(fused && fv >= root)));
      const uint32_t fl = static_cast<uint32_t>(fm);
      const uint32_t dc = (fl >> 6) & 1u, ig = (fl >> 7) & 1u;
      bool pop = dc != 0;
      SVS_PF_EXAM(1, px1);
      [[maybe_unused]] const uint64_t px2 = SVS_PF_CLK();
      if (!pop) {
        // unfinished tails in in-edge order (the first three from the flag
        // lanes, one store; more from memory), then, unless cur was itself
        // pushed as an aligned node, its unfinished aligned nodes (flagged)
        const uint64_t tpm = ~fm & ballot(lane < 3u && lane < deg);
        push_lanes(tpm, fid);
        bool valid = tpm == 0;
        for (uint32_t x = 3; x < deg; ++x) {
          const uint32_t t = uni(in_nbr[off + x]);
          const uint32_t dt = t < root ? 1u : uni(done_of(t));
          if (!dt) {
            push(t);
            valid = false;
          }
        }
        if (!ig) {
          const uint64_t apm = ~fm & ballot(lane >= 3u && lane < 6u && lane - 3u < alc);
          push_lanes(apm, fid);
          if ((apm >> lane) & 1u) set_bit(S.ign, fid);
          valid = valid && apm == 0;
        }
        if (valid) {
          set_bit(S.done, cur);
          if (!ig) {
            emit(cur);
            for (uint32_t k = 0; k < alc; ++k) emit(k == 0 ? m0 : (k == 1 ? m1 : m2));
            ++ncol;
          }
          pop = true;  // the entry popped is cur's (pushes only happen when !valid)
        }
      }
      SVS_PF_EXAM(2, px2);
      [[maybe_unused]] const uint64_t px3 = SVS_PF_CLK();
      if (pop) {
        if (S.sp == 0) refill();
        --S.sp;
        if (S.sp + S.spilled == 0) {
          SVS_PF_EXAM(3, px3);
          break;
        }
        if (S.sp == 0) refill();
        cur = uni(S.st[S.sp - 1]);
      } else {
        cur = top;  // something was pushed: the last push is on top
      }
      SVS_PF_EXAM(3, px3);
    }
    SVS_PF_ADD(1, pf0);
  }
  flush_emit();
  *ncol_out = ncol;
  S.n_exam = static_cast<uint32_t>(steps);
  S.n_emit = cnt;
  return (cnt == V && !S.err) ? kFoldOk : kFoldErrStack;
}

// Lite export of the next alignment's row tables (PoaGraph::export_strip_lite):
// per rank row its in-edge rows (CSR, in-edge order; bit 31: this in-edge is
// its tail row's last pool read), base | sink << 8 | store << 9 | in-degree
// << 10; the planner's slot count and the largest in-degree.
__device__ void export_lite(uint32_t V, const gu8* __restrict__ base, const gu32* __restrict__ in_off,
                            const gu32* __restrict__ in_nbr, const gu32* __restrict__ out_off,
                            const gu32* __restrict__ r2n, const gu32* __restrict__ n2r, gu32* __restrict__ last,
                            gu32* __restrict__ pstart, gu32* __restrict__ pred, gu32* __restrict__ info,
                            uint32_t* n_slots, uint32_t* max_preds) {
  const uint32_t lane = lanei();
  // pass 1: pstart, in-edge rows, per row words without the store bit; last
  // pool reader of every row (an in-edge from the row just above is served
  // from registers and does not count)
  for (uint32_t r = lane; r < V; r += 64) last[r] = 0;
  wave_sync_mem();
  uint32_t run = 0, mp = 0;
  for (uint32_t r0 = 0; r0 < V; r0 += 64) {
    const uint32_t r = r0 + lane;
    uint32_t node = 0, a = 0, d = 0;
    if (r < V) {
      node = r2n[r];
      a = in_off[node];
      d = in_off[node + 1] - a;
    }
    uint32_t tot;
    const uint32_t o = run + wave_excl(d, &tot);
    if (r < V) {
      pstart[r] = o;
      const bool sink = out_off[node + 1] == out_off[node];
      info[r] = static_cast<uint32_t>(base[node]) | (sink ? 0x100u : 0u) | (min(d, 63u) << 10);  // 63: >= 63
      for (uint32_t k = 0; k < d; ++k) {
        const uint32_t pr = n2r[in_nbr[a + k]];
        pred[o + k] = pr + 1;
        if (pr + 1 != r) __hip_atomic_fetch_max(last + pr, r + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    mp = max(mp, d);
    run += tot;
  }
  if (lane == 0) pstart[V] = run;
  wave_sync_mem();
  // pass 2: store bits, last-read flags, and the slot count of the planner
  // (slots in use after row r's own: stores so far - frees before r)
  int32_t live_max = 0, carry = 0;  // carry: stores - frees before the chunk
  for (uint32_t r0 = 0; r0 < V; r0 += 64) {
    const uint32_t r = r0 + lane;
    uint32_t st = 0, fr = 0;
    if (r < V) {
      st = last[r] != 0 ? 1u : 0u;
      if (st) info[r] |= 0x200u;
      const uint32_t a = pstart[r], b = (r + 1 < V) ? pstart[r + 1] : run;
      for (uint32_t x = a; x < b; ++x) {
        const uint32_t pr = pred[x] - 1;
        if (pr + 1 != r && last[pr] == r + 1) {
          pred[x] = (pr + 1) | 0x80000000u;
          ++fr;
        }
      }
    }
    uint32_t tst, tfr;
    const uint32_t est = wave_excl(st, &tst), efr = wave_excl(fr, &tfr);
    const int32_t live = carry + static_cast<int32_t>(est + st) - static_cast<int32_t>(efr);
    live_max = max(live_max, wave_max_i(r < V ? live : 0));
    carry += static_cast<int32_t>(tst) - static_cast<int32_t>(tfr);
  }
  *n_slots = 1u + static_cast<uint32_t>(max(0, live_max));
  *max_preds = uni(wave_max(mp));
}

// Heaviest-bundle consensus (PoaGraph::consensus, spoa GenerateConsensus with
// min_coverage <= 0).  Edge weights are kept halved (spoa adds 2 per
// sequence); with score' = (score - 1) / 2 every comparison is the same.
// Written into out reversed; returns its length.
__device__ uint32_t consensus_rev(uint32_t V, const gu8* __restrict__ base, const gu32* __restrict__ in_off,
                                  const gu32* __restrict__ in_nbr, const gu32* __restrict__ in_eid,
                                  const gu32* __restrict__ out_off, const gu32* __restrict__ out_nbr,
                                  const gu32* __restrict__ ew, const gu32* __restrict__ r2n,
                                  const gu32* __restrict__ n2r, gi32* __restrict__ score, gi32* __restrict__ predn,
                                  gch* __restrict__ out) {
  const uint32_t lane = lanei();
  auto sc = [&](int32_t v) -> int32_t { return ldci(score + v); };
  for (uint32_t v = lane; v < V; v += 64) {
    score[v] = -1;
    predn[v] = -1;
  }
  wave_sync_mem();
  int32_t best = -1, best_sc = 0;
  for (uint32_t r = 0; r < V; ++r) {
    const uint32_t node = r2n[r];
    int32_t s = -1, p = -1, sp = 0;
    for (uint32_t x = in_off[node]; x < in_off[node + 1]; ++x) {
      const int32_t t = static_cast<int32_t>(in_nbr[x]);
      const int32_t w = static_cast<int32_t>(ew[in_eid[x]]);
      const int32_t st = sc(t);
      if (s < w || (s == w && sp <= st)) {
        s = w;
        p = t;
        sp = st;
      }
    }
    if (p != -1) s += sp;
    if (lane == 0) {
      score[node] = s;
      predn[node] = p;
    }
    __builtin_amdgcn_s_waitcnt(0);
    if (best == -1 || best_sc < s) {
      best = static_cast<int32_t>(node);
      best_sc = s;
    }
  }
  // branch completion while the best node has successors
  while (out_off[best + 1] != out_off[best]) {
    const uint32_t start = static_cast<uint32_t>(best), rank = n2r[start];
    for (uint32_t e = out_off[start]; e < out_off[start + 1]; ++e) {
      const uint32_t hd = out_nbr[e];
      for (uint32_t f = in_off[hd]; f < in_off[hd + 1]; ++f)
        if (in_nbr[f] != start && lane == 0) score[in_nbr[f]] = -1;
    }
    __builtin_amdgcn_s_waitcnt(0);
    best = -1;
    best_sc = 0;
    for (uint32_t r = rank + 1; r < V; ++r) {
      const uint32_t node = r2n[r];
      int32_t s = -1, p = -1, sp = 0;
      for (uint32_t x = in_off[node]; x < in_off[node + 1]; ++x) {
        const int32_t t = static_cast<int32_t>(in_nbr[x]);
        const int32_t st = sc(t);
        if (st == -1) continue;
        const int32_t w = static_cast<int32_t>(ew[in_eid[x]]);
        if (s < w || (s == w && sp <= st)) {
          s = w;
          p = t;
          sp = st;
        }
      }
      if (p != -1) s += sp;
      if (lane == 0) {
        score[node] = s;
        predn[node] = p;
      }
      __builtin_amdgcn_s_waitcnt(0);
      if (best == -1 || best_sc < s) {
        best = static_cast<int32_t>(node);
        best_sc = s;
      }
    }
  }
  uint32_t n = 0;
  for (int32_t x = best; x != -1; x = ldci(predn + x)) {
    if (lane == 0) out[n] = static_cast<char>(base[x]);
    ++n;
  }
  return n;
}

// consensus_rev with the scores and predecessors in LDS (sc: V int32, pn: V
// uint16, 0xFFFF = none; V < 65535) and each 64-row chunk's nodes and first
// four in-edges (tail, weight) loaded into lanes with coalesced loads before
// the chunk's rows are scored one by one, so a row costs LDS reads instead of
// a chain of dependent global loads.  Same comparisons, same order.
__device__ uint32_t consensus_rev_lds(uint32_t V, const gu8* __restrict__ base, const gu32* __restrict__ in_off,
                                      const gu32* __restrict__ in_nbr, const gu32* __restrict__ in_eid,
                                      const gu32* __restrict__ out_off, const gu32* __restrict__ out_nbr,
                                      const gu32* __restrict__ ew, const gu32* __restrict__ r2n,
                                      const gu32* __restrict__ n2r, int32_t* sc, uint16_t* pn, gch* __restrict__ out) {
  const uint32_t lane = lanei();
  constexpr uint16_t kNoPred = 0xFFFFu;
  for (uint32_t v = lane; v < V; v += 64) {
    sc[v] = -1;
    pn[v] = kNoPred;
  }
  int32_t best = -1, best_sc = 0;
  // rows rbeg .. V-1 in rank order; rescan: in-edges from an unscored (-1) tail are skipped
  auto pass = [&](uint32_t rbeg, bool rescan) {
    best = -1;
    best_sc = 0;
    for (uint32_t c0 = rbeg; c0 < V; c0 += 64) {
      const uint32_t r = c0 + lane;
      uint32_t node = 0, a = 0, deg = 0, ta = 0, tb = 0, tc = 0, td = 0, wa = 0, wb = 0, wc = 0, wd = 0;
      if (r < V) {
        node = r2n[r];
        a = in_off[node];
        deg = in_off[node + 1] - a;
        if (deg > 0) { ta = in_nbr[a]; wa = ew[in_eid[a]]; }
        if (deg > 1) { tb = in_nbr[a + 1]; wb = ew[in_eid[a + 1]]; }
        if (deg > 2) { tc = in_nbr[a + 2]; wc = ew[in_eid[a + 2]]; }
        if (deg > 3) { td = in_nbr[a + 3]; wd = ew[in_eid[a + 3]]; }
      }
      const uint32_t nh = min(64u, V - c0);
      for (uint32_t i = 0; i < nh; ++i) {
        const uint32_t nd = lane_val(node, i), dg = lane_val(deg, i);
        int32_t s = -1, p = -1, sp = 0;
        auto edge = [&](uint32_t t, uint32_t wu) {
          const int32_t st = static_cast<int32_t>(uni(static_cast<uint32_t>(sc[t])));
          if (rescan && st == -1) return;
          const int32_t w = static_cast<int32_t>(wu);
          if (s < w || (s == w && sp <= st)) {
            s = w;
            p = static_cast<int32_t>(t);
            sp = st;
          }
        };
        if (dg > 0) edge(lane_val(ta, i), lane_val(wa, i));
        if (dg > 1) edge(lane_val(tb, i), lane_val(wb, i));
        if (dg > 2) edge(lane_val(tc, i), lane_val(wc, i));
        if (dg > 3) edge(lane_val(td, i), lane_val(wd, i));
        if (dg > 4) {
          const uint32_t ai = lane_val(a, i);
          for (uint32_t x = 4; x < dg; ++x) edge(uni(in_nbr[ai + x]), uni(ew[in_eid[ai + x]]));
        }
        if (p != -1) s += sp;
        if (lane == 0) {
          sc[nd] = s;
          pn[nd] = p == -1 ? kNoPred : static_cast<uint16_t>(p);
        }
        if (best == -1 || best_sc < s) {
          best = static_cast<int32_t>(nd);
          best_sc = s;
        }
      }
    }
  };
  pass(0, false);
  if (best < 0) return 0;
  // branch completion while the best node has successors
  while (out_off[best + 1] != out_off[best]) {
    const uint32_t start = static_cast<uint32_t>(best), rank = n2r[start];
    for (uint32_t e = out_off[start]; e < out_off[start + 1]; ++e) {
      const uint32_t hd = out_nbr[e];
      for (uint32_t f = in_off[hd]; f < in_off[hd + 1]; ++f)
        if (in_nbr[f] != start && lane == 0) sc[in_nbr[f]] = -1;
    }
    pass(rank + 1, true);
  }
  // the path back from best, node ids first into sc (scores are done), then
  // its letters gathered by all lanes
  uint32_t n = 0;
  for (uint32_t x = static_cast<uint32_t>(best); x != kNoPred && n < V; x = uni(pn[x])) {
    if (lane == 0) sc[n] = static_cast<int32_t>(x);
    ++n;
  }
  for (uint32_t k = lane; k < n; k += 64) out[k] = static_cast<char>(base[sc[k]]);
  return n;
}

// DataScanner.SeqEncoder: A0 T1 C2 G3 -4, case-folded (the host checks the
// window's reads for other letters before it asks for features).
__device__ __forceinline__ uint32_t seq_code(uint32_t ch) {
  const uint32_t u = ch & 0xDFu;  // upper case ('-' becomes 0x0D)
  return u == 'A' ? 0u : (u == 'T' ? 1u : (u == 'C' ? 2u : (u == 'G' ? 3u : 4u)));
}

// MSAFeatureSelection (DataScanner.py:195-219) over the MSA rows this wave
// has just written: CallMargin on row 0 (:146-165; the walks' stops are
// worked out on the host from the flanks, only which columns row 0 occupies
// is known here), then FindNonSameSite (:167-179) over rows 1 .. R-1 (R0
// MSA rows and `extra` all-gap rows), then the kept columns of rows 1 .. R-1
// as seqdatamx.  The kept column indices go through `keep` (task block
// scratch).  Returns n_feat.
//
// The counts: a lane takes four adjacent columns (one 32-bit word per row;
// rows are 64-B aligned) and counts A, T, C, G in packed byte counters, eight
// rows' words loaded before any is counted so that the loads overlap (one wave
// per window: a load per row and column chunk in turn was a chain of ~7,000
// dependent L2 round trips per window).  Everything else is a gap for
// FindNonSameSite (SeqEncoder's 4), so n4 = extra + (R0 - 1) - (nA+nT+nC+nG).
__device__ __forceinline__ uint32_t zero_bytes_hi(uint32_t t) {
  // bit 7 of each byte set iff that byte of t is zero (exact, no borrow between bytes)
  return ~(((t & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | t | 0x7F7F7F7Fu);
}
__device__ uint32_t msa_features(const FoldJob& J, const gu32* __restrict__ col, uint32_t ncol,
                                 const gch* __restrict__ msa, gu32* __restrict__ keep) {
  const uint32_t lane = lanei();
  const uint32_t R0 = J.n_paths + 1, stride = J.msa_stride;
  const gu32* paths = glb(J.paths);
  const gu32* poff = glb(J.path_off);
  // row 0's columns in order are col[] of path 0's nodes
  const uint32_t a0 = uni(poff[0]), L0 = uni(poff[1]) - a0;
  const uint32_t c_first = L0 ? uni(col[uni(paths[a0])]) : kNone;
  const uint32_t c_last = L0 ? uni(col[uni(paths[a0 + L0 - 1])]) : kNone;
  // forward walk: the first m5 row-0 columns
  uint32_t m5;
  if (J.f5_take >= 0) m5 = min(L0, static_cast<uint32_t>(J.f5_take));
  else if (J.f5_take == kTakeAll) m5 = L0;
  else m5 = (L0 && c_first == 0u) ? L0 : 0u;  // empty f5: stops at once on a leading gap
  // backward walk over columns ncol-1 .. 1: the last m3 row-0 columns >= 1
  const uint32_t n3 = L0 - ((L0 && c_first == 0u) ? 1u : 0u);
  uint32_t m3;
  if (J.f3_take >= 0) m3 = min(n3, static_cast<uint32_t>(J.f3_take));
  else if (J.f3_take == kTakeAll) m3 = n3;
  else m3 = (n3 && ncol >= 2u && c_last == ncol - 1u) ? n3 : 0u;
  // row-0 columns <= lo or >= hi are in the flank pool
  const int64_t lo = m5 ? static_cast<int64_t>(uni(col[uni(paths[a0 + m5 - 1])])) : -1;
  const int64_t hi = m3 ? static_cast<int64_t>(uni(col[uni(paths[a0 + L0 - m3])])) : static_cast<int64_t>(ncol);
  const gu32* __restrict__ m32 = reinterpret_cast<const gu32*>(msa);
  const uint32_t sw = stride >> 2;  // words per row
  uint32_t n_feat = 0;
  for (uint32_t c0 = 0; c0 < ncol; c0 += 256) {
    const uint32_t cw = (c0 >> 2) + lane;  // this lane's word: columns 4 cw .. 4 cw + 3
    const bool live = 4u * cw < ncol;
    uint32_t nA = 0, nT = 0, nC = 0, nG = 0;  // packed byte counters (<= 255 rows between flushes)
    uint32_t tA = 0, tT = 0, tC = 0, tG = 0;  // the same, 16-bit fields: bytes 0, 2
    uint32_t uA = 0, uT = 0, uC = 0, uG = 0;  // bytes 1, 3
    auto count = [&](uint32_t x) {
      const uint32_t u = x & 0xDFDFDFDFu;  // upper case
      nA += zero_bytes_hi(u ^ 0x41414141u) >> 7;
      nT += zero_bytes_hi(u ^ 0x54545454u) >> 7;
      nC += zero_bytes_hi(u ^ 0x43434343u) >> 7;
      nG += zero_bytes_hi(u ^ 0x47474747u) >> 7;
    };
    auto flush = [&]() {
      tA += nA & 0x00FF00FFu; uA += (nA >> 8) & 0x00FF00FFu; nA = 0;
      tT += nT & 0x00FF00FFu; uT += (nT >> 8) & 0x00FF00FFu; nT = 0;
      tC += nC & 0x00FF00FFu; uC += (nC >> 8) & 0x00FF00FFu; nC = 0;
      tG += nG & 0x00FF00FFu; uG += (nG >> 8) & 0x00FF00FFu; nG = 0;
    };
    uint32_t x0 = 0;
    if (live) {
      x0 = m32[cw];
      uint32_t r = 1, blk = 0;
      for (; r + 8 <= R0; r += 8) {
        uint32_t x[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) x[i] = m32[static_cast<uint64_t>(r + i) * sw + cw];
#pragma unroll
        for (int i = 0; i < 8; ++i) count(x[i]);
        if ((blk += 8) >= 248u) {
          flush();
          blk = 0;
        }
      }
      for (; r < R0; ++r) count(m32[static_cast<uint64_t>(r) * sw + cw]);
      flush();
    }
    // 16-bit fields: rows < 65536 (the host keeps windows far below that)
    uint32_t kbits = 0;
#pragma unroll
    for (uint32_t b = 0; b < 4; ++b) {
      const uint32_t c = 4u * cw + b;
      if (c >= ncol) continue;
      const bool in_pool = ((x0 >> (8 * b)) & 0xFFu) != '-' &&
                           (static_cast<int64_t>(c) <= lo || static_cast<int64_t>(c) >= hi);
      if (in_pool) continue;
      const uint32_t sh = 16 * (b >> 1);
      auto field = [&](uint32_t even, uint32_t odd) { return (((b & 1u) ? odd : even) >> sh) & 0xFFFFu; };
      const uint32_t n0 = field(tA, uA), n1 = field(tT, uT), n2 = field(tC, uC), n3c = field(tG, uG);
      const uint32_t n4 = J.extra + (R0 - 1) - (n0 + n1 + n2 + n3c);
      // second-largest count (sorted(counts)[3])
      uint32_t m1 = 0, m2 = 0;
      for (const uint32_t v : {n0, n1, n2, n3c, n4}) {
        m2 = v > m1 ? m1 : max(m2, v);
        m1 = max(m1, v);
      }
      if (m2 >= J.cut) kbits |= 1u << b;
    }
    // kept columns in column order: lane-major, then within the lane's word
    const uint32_t kc = __builtin_popcount(kbits);
    uint32_t off = 0, tot = 0;
#pragma unroll
    for (uint32_t bit = 0; bit < 3; ++bit) {
      const uint64_t m = ballot((kc >> bit) & 1u);
      off += popc64(m & below()) << bit;
      tot += popc64(m) << bit;
    }
    uint32_t o = n_feat + off;
#pragma unroll
    for (uint32_t b = 0; b < 4; ++b)
      if ((kbits >> b) & 1u) keep[o++] = 4u * cw + b;
    n_feat += tot;
  }
  wave_sync_mem();
  // seqdatamx: rows 1 .. R0-1 of the MSA, then `extra` all-gap rows; eight
  // rows' gathers in flight at a time
  gu8* out = glb(J.feat_out);
  const uint32_t rows = R0 - 1 + J.extra;
  for (uint32_t k0 = 0; k0 < n_feat; k0 += 64) {
    const uint32_t k = k0 + lane;
    if (k < n_feat) {
      const uint32_t c = keep[k];
      uint32_t r = 1;
      for (; r + 8 <= R0; r += 8) {
        uint32_t x[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) x[i] = static_cast<uint8_t>(msa[static_cast<uint64_t>(r + i) * stride + c]);
#pragma unroll
        for (int i = 0; i < 8; ++i) out[static_cast<uint64_t>(r + i - 1) * n_feat + k] = static_cast<uint8_t>(seq_code(x[i]));
      }
      for (; r < R0; ++r)
        out[static_cast<uint64_t>(r - 1) * n_feat + k] =
            static_cast<uint8_t>(seq_code(static_cast<uint8_t>(msa[static_cast<uint64_t>(r) * stride + c])));
      for (r = R0 - 1; r < rows; ++r) out[static_cast<uint64_t>(r) * n_feat + k] = 4u;
    }
  }
  return n_feat;
}

// MSA rows: every sequence's path nodes at their columns, '-' elsewhere.  The
// rows (stride and start 64-B aligned, stride >= ncol rounded up to 16) are
// filled with 16-B stores, then each path's nodes are placed eight 64-node
// chunks at a time (their node, column and letter loads all in flight before
// the stores).
__device__ void msa_rows(uint32_t n_paths, const gu32* __restrict__ paths, const gu32* __restrict__ path_off,
                         const gu32* __restrict__ colv, const gu8* __restrict__ base, uint32_t ncol,
                         gch* __restrict__ out, uint32_t stride) {
  const uint32_t lane = lanei();
  const uint32_t w16 = (ncol + 15u) >> 4;
  const u32x4 dash = {0x2D2D2D2Du, 0x2D2D2D2Du, 0x2D2D2D2Du, 0x2D2D2D2Du};
  for (uint32_t s = 0; s < n_paths; ++s) {
    GLB u32x4* row = reinterpret_cast<GLB u32x4*>(out + static_cast<uint64_t>(s) * stride);
    for (uint32_t c = lane; c < w16; c += 64) row[c] = dash;
  }
  wave_sync_mem();
  constexpr uint32_t kU = 8;
  for (uint32_t s = 0; s < n_paths; ++s) {
    gch* row = out + static_cast<uint64_t>(s) * stride;
    const uint32_t a = path_off[s], b = path_off[s + 1];
    for (uint32_t k = a + lane; k < b; k += 64 * kU) {
      uint32_t nd[kU], cc[kU], bb[kU];
#pragma unroll
      for (uint32_t i = 0; i < kU; ++i) nd[i] = k + 64 * i < b ? paths[k + 64 * i] : 0u;
#pragma unroll
      for (uint32_t i = 0; i < kU; ++i) {
        cc[i] = colv[nd[i]];
        bb[i] = base[nd[i]];
      }
#pragma unroll
      for (uint32_t i = 0; i < kU; ++i)
        if (k + 64 * i < b) row[cc[i]] = static_cast<char>(bb[i]);
    }
  }
}

__global__ __launch_bounds__(64) void poa_fold_sort_kernel(const FoldJob* __restrict__ jobs, uint32_t lds_words) {
  SVS_FOLD_PRIO();
  extern __shared__ uint32_t lds[];
  const uint64_t T0 = __builtin_amdgcn_s_memrealtime();
  const FoldJob J = jobs[blockIdx.x];
  GLB FoldResult* res = glb(J.result);
  if (uni(static_cast<uint32_t>(res->status)) != static_cast<uint32_t>(kFoldOk)) return;
  const uint32_t V = uni(res->V);
  const uint32_t b1 = 1u - J.par;
  const GPtr g = gptr(J.blk, J.cv, J.ce, b1);
  const uint32_t W = (V + 31u) >> 5;
  SortState S;
  S.done = lds;
  S.ign = lds + W;
  S.chg = lds + 2 * W;
  S.nseg = lds + 3 * W;
  S.st = lds + 4 * W;
  S.cap = ((lds_words - 4 * W) / 2) * 2;
  S.spill = g.stk;
  S.spilled = 0;
  S.sp = 0;
  S.spill_cap = J.ce + 2 * J.cv + 64;
  S.err = false;
  S.n_exam = 0;
  S.n_roots = 0;
  S.n_emit = 0;
  S.prof[0] = S.prof[1] = S.prof[2] = S.prof[3] = 0;
  uint32_t ncol = 0;
  if (S.cap < 64) {
    if (lanei() == 0) res->status = kFoldErrStack;
    return;
  }
  int32_t st = kFoldOk;
  if (J.flags & kFoldChain) {
    // a fresh chain (node i's only in-edge from i - 1): the DFS order is the
    // identity, one column per node
    for (uint32_t v = lanei(); v < V; v += 64) {
      g.r2n[v] = v;
      g.n2r[v] = v;
      g.col[v] = v;
    }
    for (uint32_t w = lanei(); w < W; w += 64) g.seg[w] = ~0u;  // every node its own root
    ncol = V;
  } else {
    // the previous rank order, kept for the DFS's record windows (export
    // reuses `last` after the sort), and the fold's changed plane
    const uint32_t V0 = min(J.V, V);
    for (uint32_t r = lanei(); r < V0; r += 64) g.last[r] = g.r2n[r];
    for (uint32_t w = lanei(); w < W; w += 64) lds[2 * W + w] = g.chg[w];
    wave_sync_mem();
    st = dfs_sort(V, V0, g.nrec, g.in_nbr, g.r2n, g.n2r, g.last, g.col, V0 ? g.seg_other : nullptr, S, &ncol);
    if (st == kFoldOk)
      for (uint32_t w = lanei(); w < W; w += 64) g.seg[w] = S.nseg[w];
  }
  if (st != kFoldOk) {
    if (lanei() == 0) {
      // for the host's message: nodes emitted, whether the stack overflowed
      res->pad0 = S.n_emit;
      res->pad1 = S.err ? 1u : 0u;
      res->n_exam = S.n_exam;
      res->n_roots = S.n_roots;
      res->status = st;
    }
    return;
  }
  wave_sync_mem();
  const uint64_t T1 = __builtin_amdgcn_s_memrealtime();
  uint32_t n_slots = 0, max_preds = 0;
  if (J.flags & kFoldExport)
    export_lite(V, g.base, g.in_off, g.in_nbr, g.out_off, g.r2n, g.n2r, g.last, g.pstart, g.pred, g.info, &n_slots,
                &max_preds);
  const uint64_t T2 = __builtin_amdgcn_s_memrealtime();
  if (lanei() == 0) {
    res->n_slots = n_slots;
    res->max_preds = max_preds;
    res->ncol = ncol;
    res->t_sort = static_cast<uint32_t>(T1 - T0);
    res->t_exp = static_cast<uint32_t>(T2 - T1);
    res->n_exam = S.n_exam;
    res->n_roots = S.n_roots;
#ifndef SVS_FOLD_PROF_UPD
    for (int k = 0; k < 4; ++k) res->prof[k] = static_cast<uint32_t>(S.prof[k] >> SVS_PF_SHIFT(k));
#endif
  }
}

// The last read's fold (kFoldFinal): consensus and MSA rows, after the sort.
// lds_words: the LDS the launch gives each job (6 B per node for the scores
// and predecessors; larger graphs score in global memory).
// idx (optional): the final folds' indices into jobs, one per workgroup.
__global__ __launch_bounds__(64) void poa_fold_final_kernel(const FoldJob* __restrict__ jobs, uint32_t lds_words,
                                                            const uint32_t* __restrict__ idx) {
  SVS_FOLD_PRIO();
  extern __shared__ uint32_t lds[];
  const uint64_t T0 = __builtin_amdgcn_s_memrealtime();
  const FoldJob J = jobs[idx ? idx[blockIdx.x] : blockIdx.x];
  if (!(J.flags & kFoldFinal)) return;
  GLB FoldResult* res = glb(J.result);
  if (uni(static_cast<uint32_t>(res->status)) != static_cast<uint32_t>(kFoldOk)) return;
  const uint32_t V = uni(res->V), ncol = uni(res->ncol);
  const GPtr g = gptr(J.blk, J.cv, J.ce, 1u - J.par);
  uint32_t nc;
  if (V < 65535u && 6ull * V + 8 <= 4ull * lds_words) {
    int32_t* sc = reinterpret_cast<int32_t*>(lds);
    uint16_t* pn = reinterpret_cast<uint16_t*>(lds + V);
    nc = consensus_rev_lds(V, g.base, g.in_off, g.in_nbr, g.in_eid, g.out_off, g.out_nbr, g.ew, g.r2n, g.n2r, sc, pn,
                           glb(J.cons_out));
  } else {
    nc = consensus_rev(V, g.base, g.in_off, g.in_nbr, g.in_eid, g.out_off, g.out_nbr, g.ew, g.r2n, g.n2r,
                       reinterpret_cast<gi32*>(g.last), reinterpret_cast<gi32*>(g.pstart), glb(J.cons_out));
  }
  if (J.flags & kFoldMsa)
    msa_rows(J.n_paths + 1, glb(J.paths), glb(J.path_off), g.col, g.base, ncol, glb(J.msa_out), J.msa_stride);
  uint32_t n_feat = 0;
  if (J.flags & kFoldFeat) {
    wave_sync_mem();  // the MSA rows this wave has just stored
    n_feat = msa_features(J, g.col, ncol, glb(static_cast<const char*>(J.msa_out)), g.last);
  }
  if (lanei() == 0) {
    res->pad1 = n_feat;
    res->pad0 = nc;
    res->t_fin = static_cast<uint32_t>(__builtin_amdgcn_s_memrealtime() - T0);
  }
}

// Block growth: the graph of a task moved into a larger block (capacities
// cv1 >= cv0, ce1 >= ce0), both CSR buffers' current one only; one row of
// workgroups per move (blockIdx.y), every move of a launch in one kernel
// (one kernel per move had ~36 small kernels per launch queue up on the copy
// stream ahead of the DP kernel).
__global__ __launch_bounds__(256) void poa_dgraph_move_kernel(const MoveDesc* __restrict__ moves) {
  const MoveDesc M = moves[blockIdx.y];
  const uint8_t* __restrict__ src = M.src;
  uint8_t* __restrict__ dst = M.dst;
  const uint32_t V = M.V, E = M.E, par = M.par;
  const DGraphLayout A = dgraph_layout(M.cv0, M.ce0), B = dgraph_layout(M.cv1, M.ce1);
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x, nt = gridDim.x * blockDim.x;
  auto cp = [&](size_t a, size_t b, size_t bytes) {
    const uint32_t* s = reinterpret_cast<const uint32_t*>(src + a);
    uint32_t* d = reinterpret_cast<uint32_t*>(dst + b);
    for (size_t k = t; k < (bytes + 3) / 4; k += nt) d[k] = s[k];
  };
  cp(A.base, B.base, V);
  cp(A.al, B.al, 16ull * V);
  auto pick = [&](const size_t* x) { return par ? x[1] : x[0]; };
  cp(pick(A.in_off), pick(B.in_off), 4ull * (V + 1));
  cp(pick(A.in_nbr), pick(B.in_nbr), 4ull * E);
  cp(pick(A.in_eid), pick(B.in_eid), 4ull * E);
  cp(pick(A.out_off), pick(B.out_off), 4ull * (V + 1));
  cp(pick(A.out_nbr), pick(B.out_nbr), 4ull * E);
  cp(pick(A.out_eid), pick(B.out_eid), 4ull * E);
  cp(A.ew, B.ew, 4ull * E);
  cp(A.nin, B.nin, 8ull * V);
  cp(A.nout, B.nout, 8ull * V);
  cp(A.r2n, B.r2n, 4ull * V);
  cp(A.n2r, B.n2r, 4ull * V);
  cp(A.col, B.col, 4ull * V);
  cp(A.pstart, B.pstart, 4ull * (V + 1));
  cp(A.pred, B.pred, 4ull * E);
  cp(A.info, B.info, 4ull * V);
  // the next alignment's completed tables (a pruning retry reuses them)
  cp(A.col0, B.col0, 12ull * V);
  cp(A.rec, B.rec, 16ull * V);
  cp(A.pslot, B.pslot, 4ull * E);
  // the last sort's segment starts (the next sort walks them), and the node
  // records (the next update tells a changed aligned list by their counts)
  cp(pick(A.seg), pick(B.seg), 4ull * ((V + 31) / 32 + 2));
  cp(A.nrec, B.nrec, 32ull * V);
}

hipError_t launch_poa_fold(const FoldJob* jobs, int n_jobs, uint32_t lds_words, uint32_t final_lds_words,
                           hipStream_t stream, const hipEvent_t* marks) {
  if (n_jobs <= 0) return hipSuccess;
  hipLaunchKernelGGL(poa_fold_update_kernel, dim3(n_jobs), dim3(64), 0, stream, jobs);
  if (marks) (void)hipEventRecord(marks[0], stream);
  hipLaunchKernelGGL(poa_fold_sort_kernel, dim3(n_jobs), dim3(64), lds_words * 4, stream, jobs, lds_words);
  if (marks) (void)hipEventRecord(marks[1], stream);
  if (final_lds_words)
    hipLaunchKernelGGL(poa_fold_final_kernel, dim3(n_jobs), dim3(64), final_lds_words * 4, stream, jobs,
                       final_lds_words, static_cast<const uint32_t*>(nullptr));
  if (marks) (void)hipEventRecord(marks[2], stream);
  return hipGetLastError();
}

hipError_t launch_poa_final(const FoldJob* jobs, const uint32_t* idx, int n_final, uint32_t final_lds_words,
                            hipStream_t stream) {
  if (n_final <= 0 || final_lds_words == 0) return hipSuccess;
  hipLaunchKernelGGL(poa_fold_final_kernel, dim3(n_final), dim3(64), final_lds_words * 4, stream, jobs, final_lds_words,
                     idx);
  return hipGetLastError();
}

// The new tasks' read blocks from the launch's staging into their own blocks:
// one workgroup per copy, 16-byte words.
__global__ __launch_bounds__(256) void scatter_copy_kernel(const CopyDesc* __restrict__ d) {
  const CopyDesc c = d[blockIdx.x];
  const u32x4* __restrict__ s = reinterpret_cast<const u32x4*>(c.src);
  u32x4* __restrict__ t = reinterpret_cast<u32x4*>(c.dst);
  for (uint64_t k = threadIdx.x; k < c.bytes / 16; k += blockDim.x) t[k] = s[k];
}

hipError_t launch_scatter_copy(const CopyDesc* d, int n, hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(scatter_copy_kernel, dim3(n), dim3(256), 0, stream, d);
  return hipGetLastError();
}

hipError_t launch_dgraph_moves(const MoveDesc* d, int n, hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(poa_dgraph_move_kernel, dim3(16, static_cast<uint32_t>(n)), dim3(256), 0, stream, d);
  return hipGetLastError();
}

}  // namespace svs
