// Host driver of the MisScore seam: PairwiseCompare.AligmentScore for many
// (somatic, germline) consensus pairs at once
// (/root/reference/src/PairwiseCompare.py:19-30, called per pair by
// CalculateMisscore :54-64 inside MisScorePipe :76-86).
//
// Pairs are sorted by DP size (largest first) and packed into launches that
// fit the context's device budget.  A launch uploads the sequences its pairs
// use once, runs the fill (misscore_fill2_kernel: two neighbouring pairs per
// wave in packed int16; misscore_fill_kernel: one pair per wave in int32 for
// pairs over kMsPackedMaxLen), writing 4-bit score differences to HBM, then
// misscore_traceback_kernel (one lane per pair, pairwise2's DFS), and
// downloads one MsResult per pair.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/svscope.h"
#include "misscore_device.hpp"
#include "svs_context.hpp"
#include "svs_internal.hpp"

namespace svs {

namespace {
constexpr int32_t kMsMaxLen = 1 << 20;

size_t align256(size_t x) { return (x + 255) / 256 * 256; }

struct PairCost {
  uint64_t nib_bytes, carry_bytes, stack_bytes;
  uint64_t total() const { return nib_bytes + carry_bytes + stack_bytes; }
};

PairCost pair_cost(int32_t la, int32_t lb) {
  return PairCost{ms_nib_words(la, lb) * 4, align256(static_cast<uint64_t>(la) * 4),
                  static_cast<uint64_t>(ms_stack_cap(la, lb)) * sizeof(MsState)};
}
}  // namespace

void run_misscore(svs_context* ctx, int32_t n_pairs, const int32_t* pair_a, const int32_t* pair_b,
                  const int64_t* seq_byte_start, const char* seq_bytes, int32_t cutoff, int32_t* out_len,
                  int32_t* out_match, int32_t* out_status, svs_misscore_stats* st) {
  const auto t_wall = std::chrono::steady_clock::now();
  svs_misscore_stats stats{};
  auto seq_len = [&](int32_t s) { return seq_byte_start[s + 1] - seq_byte_start[s]; };
  std::vector<int32_t> order;
  order.reserve(n_pairs);
  for (int32_t p = 0; p < n_pairs; ++p) {
    const int64_t la = seq_len(pair_a[p]), lb = seq_len(pair_b[p]);
    if (la > kMsMaxLen || lb > kMsMaxLen)
      throw SvsError(SVS_E_UNSUPPORTED, "pair " + std::to_string(p) + ": sequence longer than 2^20");
    out_len[p] = 0;
    out_match[p] = 0;
    if (la == 0 || lb == 0) {  // pairwise2 returns [] and the reference's [0] raises IndexError
      out_status[p] = kMsEmpty;
      continue;
    }
    out_status[p] = kMsOk;
    order.push_back(p);
  }
  std::stable_sort(order.begin(), order.end(), [&](int32_t x, int32_t y) {
    return seq_len(pair_a[x]) * seq_len(pair_b[x]) > seq_len(pair_a[y]) * seq_len(pair_b[y]);
  });

  hipEvent_t ev[3] = {nullptr, nullptr, nullptr};
  for (auto& e : ev) SVS_HIP(hipEventCreate(&e));
  struct EvGuard {
    hipEvent_t* e;
    ~EvGuard() {
      for (int i = 0; i < 3; ++i)
        if (e[i]) (void)hipEventDestroy(e[i]);
    }
  } guard{ev};

  // a launch's buffers: at most half the context's budget, and at most 3/4 of
  // the HBM free now (the POA traceback and carry buffers, sized
  // from the same budget, never shrink, so a MisScore call after a POA run
  // must size itself from what they left)
  size_t free_now = 0, total_now = 0;
  SVS_HIP(hipMemGetInfo(&free_now, &total_now));
  const uint64_t budget = std::max<uint64_t>(std::min<uint64_t>(ctx->device_budget / 2, free_now / 4 * 3), 256ull << 20);
  size_t i = 0;
  while (i < order.size()) {
    // one launch: the largest remaining pairs that fit the budget (at least one)
    size_t j = i;
    uint64_t bytes = 0, seq_total = 0;
    std::unordered_map<int32_t, uint32_t> seq_at;
    while (j < order.size()) {
      const int32_t p = order[j];
      const PairCost pc = pair_cost(static_cast<int32_t>(seq_len(pair_a[p])), static_cast<int32_t>(seq_len(pair_b[p])));
      uint64_t add_seq = 0;
      for (int32_t s : {pair_a[p], pair_b[p]})
        if (!seq_at.count(s)) add_seq += static_cast<uint64_t>(seq_len(s)) + 64;
      if (j > i && (bytes + pc.total() + seq_total + add_seq > budget || seq_total + add_seq > 0xF0000000ull)) break;
      for (int32_t s : {pair_a[p], pair_b[p]})
        if (!seq_at.count(s)) {
          seq_at.emplace(s, static_cast<uint32_t>(seq_total));
          seq_total += static_cast<uint64_t>(seq_len(s)) + 64;
        }
      bytes += pc.total();
      ++j;
    }
    const int32_t n = static_cast<int32_t>(j - i);
    std::vector<MsPair> pairs(n);
    std::vector<MsDuo> duos;
    std::vector<int32_t> solo;
    std::vector<uint8_t> seqbuf(seq_total, 0);
    for (const auto& kv : seq_at) std::memcpy(seqbuf.data() + kv.second, seq_bytes + seq_byte_start[kv.first], seq_len(kv.first));
    uint64_t nib_w = 0, carry_w = 0, stack_e = 0;
    auto carry_entries = [](int32_t la) { return (static_cast<uint64_t>(la) + 63) / 64 * 64; };
    for (int32_t k = 0; k < n; ++k) {
      const int32_t p = order[i + k];
      MsPair& P = pairs[k];
      P.la = static_cast<int32_t>(seq_len(pair_a[p]));
      P.lb = static_cast<int32_t>(seq_len(pair_b[p]));
      P.a_off = seq_at[pair_a[p]];
      P.b_off = seq_at[pair_b[p]];
      P.nib_off = nib_w;
      P.carry_off = static_cast<uint32_t>(carry_w);
      P.stack_off = stack_e;
      P.stack_cap = ms_stack_cap(P.la, P.lb);
      P.out_idx = k;
      P.pad = 0;
      nib_w += ms_nib_words(P.la, P.lb);
      stack_e += P.stack_cap;
      stats.dp_cells += static_cast<uint64_t>(P.la) * P.lb;
    }
    // Fill work: neighbours in the size order share a wave of the packed
    // int16 kernel; pairs longer than it takes (or SVS_MS_FILL=32) get the
    // int32 kernel.
    const char* fe = std::getenv("SVS_MS_FILL");
    const bool packed = !(fe && std::atoi(fe) == 32);
    int32_t pend = -1;  // a packable pair waiting for a partner
    for (int32_t k = 0; k < n; ++k) {
      const MsPair& P = pairs[k];
      if (!packed || P.la > kMsPackedMaxLen || P.lb > kMsPackedMaxLen) {
        pairs[k].carry_off = static_cast<uint32_t>(carry_w);
        carry_w += carry_entries(P.la);
        solo.push_back(k);
      } else if (pend < 0) {
        pend = k;
      } else {
        duos.push_back(MsDuo{pend, k, static_cast<uint32_t>(carry_w), 0});
        carry_w += carry_entries(std::max(pairs[pend].la, P.la));
        pend = -1;
      }
    }
    if (pend >= 0) {
      duos.push_back(MsDuo{pend, -1, static_cast<uint32_t>(carry_w), 0});
      carry_w += carry_entries(pairs[pend].la);
    }
    if (carry_w > 0xFFFFFFFFull) throw SvsError(SVS_E_UNSUPPORTED, "carry buffer over 2^32 entries");
    const size_t off_duo = align256(n * sizeof(MsPair)), off_solo = off_duo + align256(duos.size() * sizeof(MsDuo));
    std::vector<uint8_t> desc(off_solo + solo.size() * sizeof(int32_t) + 4);
    std::memcpy(desc.data(), pairs.data(), n * sizeof(MsPair));
    if (!duos.empty()) std::memcpy(desc.data() + off_duo, duos.data(), duos.size() * sizeof(MsDuo));
    if (!solo.empty()) std::memcpy(desc.data() + off_solo, solo.data(), solo.size() * sizeof(int32_t));
    ctx->d_ms_pairs.ensure(desc.size());
    ctx->d_ms_seq.ensure(std::max<uint64_t>(seq_total, 64));
    ctx->d_ms_nib.ensure(nib_w * 4);
    ctx->d_ms_carry.ensure(carry_w * 4);
    ctx->d_ms_stack.ensure(stack_e * sizeof(MsState));
    ctx->d_ms_out.ensure(n * sizeof(MsResult));
    SVS_HIP(hipMemcpyAsync(ctx->d_ms_pairs.ptr, desc.data(), desc.size(), hipMemcpyHostToDevice, ctx->stream));
    SVS_HIP(hipMemcpyAsync(ctx->d_ms_seq.ptr, seqbuf.data(), seq_total, hipMemcpyHostToDevice, ctx->stream));
    uint8_t* dd = ctx->d_ms_pairs.as<uint8_t>();
    SVS_HIP(launch_misscore(ctx->d_ms_pairs.as<MsPair>(), n, reinterpret_cast<const MsDuo*>(dd + off_duo),
                            static_cast<int>(duos.size()), reinterpret_cast<const int32_t*>(dd + off_solo),
                            static_cast<int>(solo.size()), ctx->d_ms_seq.as<uint8_t>(), ctx->d_ms_nib.as<uint32_t>(),
                            ctx->d_ms_carry.as<int32_t>(), ctx->d_ms_stack.as<MsState>(), cutoff,
                            ctx->d_ms_out.as<MsResult>(), ctx->stream, ev[0], ev[1]));
    SVS_HIP(hipEventRecord(ev[2], ctx->stream));
    std::vector<MsResult> res(n);
    SVS_HIP(hipMemcpyAsync(res.data(), ctx->d_ms_out.ptr, n * sizeof(MsResult), hipMemcpyDeviceToHost, ctx->stream));
    SVS_HIP(hipStreamSynchronize(ctx->stream));
    float f_ms = 0.f, t_ms = 0.f;
    SVS_HIP(hipEventElapsedTime(&f_ms, ev[0], ev[1]));
    SVS_HIP(hipEventElapsedTime(&t_ms, ev[1], ev[2]));
    stats.fill_ms += f_ms;
    stats.traceback_ms += t_ms;
    stats.launches += 1;
    stats.nib_bytes += nib_w * 4;
    for (int32_t k = 0; k < n; ++k) {
      const int32_t p = order[i + k];
      const MsResult& r = res[k];
      if (r.status != kMsOk) {
        static const char* why[] = {"ok", "traceback step budget exceeded", "DFS stack full", "no alignment recovered",
                                    "empty sequence"};
        throw SvsError(SVS_E_INTERNAL, "pair " + std::to_string(p) + ": " +
                                           (r.status >= 0 && r.status <= 4 ? why[r.status] : "bad status"));
      }
      out_len[p] = r.trim_len;
      out_match[p] = r.trim_match;
      stats.tb_steps += static_cast<uint64_t>(r.steps);
    }
    stats.pairs += static_cast<uint64_t>(n);
    i = j;
  }
  stats.wall_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_wall).count();
  if (st) *st = stats;
}

}  // namespace svs
