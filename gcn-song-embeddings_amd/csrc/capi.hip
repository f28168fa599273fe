// C-ABI entry points (see include/pinsage_hip.h) other than the engine's.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "aggw.h"
#include "../../include/pinsage_hip.h"
#include "common.h"
#include "gemm.h"
#include "wgrad.h"
#include "mt19937.h"

namespace ps {

static thread_local std::string g_err;
void set_error(const std::string& msg) { g_err = msg; }
const char* last_error() { return g_err.c_str(); }

int launch_mt_expand(const MTChunk*, int64_t, int64_t, int64_t, uint32_t*, hipStream_t);
int launch_walk(const int64_t*, const int32_t*, const int64_t*, int64_t, int64_t, float,
                const uint32_t*, uint64_t, uint32_t, int64_t, int32_t*, int*, hipStream_t);
int launch_visit_topk(const int32_t*, const int64_t*, int64_t, int64_t, int64_t, int64_t, void*,
                      double*, int64_t*, float*, int32_t*, int64_t, hipStream_t);
int launch_visit_dense(const int32_t*, const int64_t*, int64_t, int64_t, int64_t, double*,
                       hipStream_t);
int64_t fly_workspace_bytes(int64_t, int64_t, int64_t, int64_t, int64_t);
int fly_init_workspace(void*, int64_t, int64_t, int64_t, int64_t, int64_t, hipStream_t);
int fly_publish_err(const int*, void*, int64_t, int64_t, const int64_t*, int64_t, hipStream_t);
int fly_gate_adam(int*, float*, hipStream_t);
int fly_sample(const int64_t*, const int32_t*, int64_t, const int64_t*, int64_t, int64_t, int64_t, int64_t, int64_t,
               float, const uint64_t*, void*, int64_t, int32_t* const*, float* const*, int32_t**, int64_t, int64_t*,
               int*, int64_t*, int64_t, const float*, int64_t, int64_t, float*, int64_t, int*, hipStream_t);
int launch_walk_runs(const int64_t*, const int32_t*, const int64_t*, int64_t, int, float,
                     const uint32_t*, uint64_t, uint32_t, int64_t, uint2*, int*, int*, hipStream_t);
int launch_heap_topk(const uint2*, const int*, int64_t, int, int, double*, int64_t*, float*, int32_t*,
                     int, hipStream_t, const int* n_src_dev = nullptr);
int64_t bitset_words(int64_t universe);
int64_t bitset_blocks(int64_t universe);
int launch_mark_i64(unsigned long long*, const int64_t*, int64_t, int64_t, int*, hipStream_t);
int launch_mark_table_i64(unsigned long long*, const int64_t*, int64_t, const int32_t*, int64_t,
                          int, int64_t, int*, hipStream_t);
int64_t triplet_loss_scratch_bytes(int64_t B, int64_t d);
int launch_triplet_loss(const float* Z, int B, int d, float margin, float* G, void* scratch, float* scal,
                        hipStream_t st);
int launch_set_finalize(unsigned long long*, const unsigned long long*, const unsigned long long*,
                        int64_t, uint32_t*, uint32_t*, int32_t*, int*, hipStream_t);
int launch_agg(const float*, int, const int32_t*, const float*, int, const int*, int64_t, float*,
               hipStream_t);
int launch_gather_rows(const float*, int64_t, int64_t, int, const int64_t*, int64_t, float*, int64_t,
                       hipStream_t);
int launch_l2norm_rows(float* y, int64_t n, int out, float* norms, hipStream_t st);
int launch_set_rank_table(const int64_t*, int64_t, const int32_t*, int64_t, int, const unsigned long long*,
                          const uint32_t*, int32_t*, hipStream_t);
int launch_norm_lrelu_bwd(const float*, const float*, const float*, int, const int*, int64_t, float*, float*,
                          int, const int*, int*, int64_t, hipStream_t);
int64_t knn_scratch_bytes(int64_t, int64_t);
int launch_knn_cosine(const float*, int64_t, int64_t, int64_t, const int64_t*, int64_t, int64_t,
                      float, void*, int64_t, float*, int64_t*, int*, hipStream_t);

// Fisher-Yates prefix of torch.randperm(n): first k entries, all n-1 draws consumed.
// Only the <= 2k positions the first k swaps touch are stored (open addressing).
static void randperm_prefix(MTState& g, int64_t n, int64_t k, int64_t* out) {
  k = std::min(k, n);
  const int64_t steps = std::min(k, n - 1);
  int lg = 4;
  while ((int64_t(1) << lg) < 4 * steps + 16) ++lg;
  const size_t mask = (size_t(1) << lg) - 1;
  std::vector<int64_t> keys(mask + 1, -1), vals(mask + 1);
  auto slot = [&](int64_t i) {
    size_t h = (size_t)(((uint64_t)i * 0x9E3779B97F4A7C15ull) >> (64 - lg));
    while (keys[h] != -1 && keys[h] != i) h = (h + 1) & mask;
    return h;
  };
  auto get = [&](int64_t i) {
    const size_t h = slot(i);
    return keys[h] == i ? vals[h] : i;
  };
  auto put = [&](int64_t i, int64_t v) {
    const size_t h = slot(i);
    keys[h] = i;
    vals[h] = v;
  };
  for (int64_t i = 0; i < steps; ++i) {
    const int64_t z = (int64_t)(g.draw() % (uint64_t)(n - i));
    const int64_t a = get(i), b = get(i + z);
    put(i, b);
    put(i + z, a);
  }
  for (int64_t i = 0; i < k; ++i) out[i] = get(i);
  if (n - 1 > steps) g.skip(n - 1 - steps);
}

// sample_batch with easy negatives (pinsage_training.py:53-77, 89-97); shared
// with the batch sampler runtime (loader.hip)
int sample_batch_easy(MTState& g, const int64_t* positives, int64_t P, int64_t n_items,
                      int64_t batch_size, int64_t* batch_out, int64_t* nodeset_out,
                      int64_t* n_nodeset) {
  const int64_t B = std::min(batch_size, P);
  std::vector<int64_t> sel((size_t)B);
  randperm_prefix(g, P, B, sel.data());
  std::vector<int64_t> mem;
  mem.reserve((size_t)(2 * B));
  for (int64_t b = 0; b < B; ++b) {
    const int64_t a = positives[2 * sel[(size_t)b]], p = positives[2 * sel[(size_t)b] + 1];
    if (a < 0 || a >= n_items || p < 0 || p >= n_items) {
      set_error("sample_batch: positive pair id out of range");
      return kErrIndex;
    }
    batch_out[3 * b] = a;
    batch_out[3 * b + 1] = p;
    mem.push_back(a);
    mem.push_back(p);
  }
  std::sort(mem.begin(), mem.end());
  mem.erase(std::unique(mem.begin(), mem.end()), mem.end());
  const int64_t m = n_items - (int64_t)mem.size();
  std::vector<int64_t> r((size_t)B);
  randperm_prefix(g, m, B, r.data());
  const int64_t nneg = std::min(B, m);
  for (int64_t b = 0; b < B; ++b) {
    if (b >= nneg) {
      // the reference's torch.cat fails when fewer negatives than pairs exist
      set_error("sample_batch: fewer candidate negatives than pairs");
      return kErrArg;
    }
    // r[b]-th smallest id not in mem
    const int64_t want = r[(size_t)b];
    int64_t v = want, c = 0;
    for (;;) {
      const int64_t c2 = std::upper_bound(mem.begin(), mem.end(), v) - mem.begin();
      if (c2 == c) break;
      c = c2;
      v = want + c;
    }
    batch_out[3 * b + 2] = v;
  }
  if (nodeset_out) {  // batch.flatten().unique(): sorted union of mem and the negatives
    std::vector<int64_t> neg((size_t)B);
    for (int64_t b = 0; b < B; ++b) neg[(size_t)b] = batch_out[3 * b + 2];
    std::sort(neg.begin(), neg.end());
    neg.erase(std::unique(neg.begin(), neg.end()), neg.end());
    int64_t* e = std::set_union(mem.begin(), mem.end(), neg.begin(), neg.end(), nodeset_out);
    if (n_nodeset) *n_nodeset = (int64_t)(e - nodeset_out);
  }
  return kOk;
}

}  // namespace ps

using namespace ps;

extern "C" {

int pinsage_version(void) { return 100; }
const char* pinsage_last_error(void) { return ps::last_error(); }
int pinsage_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

// ------------------------------------------------------------------ RNG
int pinsage_mt_state_bytes(void) { return (int)sizeof(MTState); }
int pinsage_mt_from_torch(void* mt, const uint8_t* st, int64_t nbytes) {
  if (!reinterpret_cast<MTState*>(mt)->from_torch(st, nbytes)) {
    set_error("mt_from_torch: not a valid torch CPU generator state");
    return kErrArg;
  }
  return kOk;
}
int pinsage_mt_to_torch(const void* mt, uint8_t* st, int64_t nbytes) {
  if (nbytes < MTState::kTorchBytes) {
    set_error("mt_to_torch: buffer smaller than torch.get_rng_state()");
    return kErrArg;
  }
  reinterpret_cast<const MTState*>(mt)->to_torch(st);
  return kOk;
}
int pinsage_mt_seed(void* mt, uint64_t seed) {
  reinterpret_cast<MTState*>(mt)->seed_with(seed);
  return kOk;
}
int pinsage_mt_skip(void* mt, int64_t n) {
  reinterpret_cast<MTState*>(mt)->skip(n);
  return kOk;
}
int pinsage_mt_draws(void* mt, uint32_t* out, int64_t n) {
  MTState* g = reinterpret_cast<MTState*>(mt);
  for (int64_t i = 0; i < n; ++i) out[i] = g->draw();
  return kOk;
}
int pinsage_mt_randperm_prefix(void* mt, int64_t n, int64_t k, int64_t* out) {
  if (n < 0 || k < 0) {
    set_error("randperm_prefix: negative size");
    return kErrArg;
  }
  randperm_prefix(*reinterpret_cast<MTState*>(mt), n, k, out);
  return kOk;
}

int pinsage_sample_batch_easy(void* mt, const int64_t* positives, int64_t P, int64_t n_items,
                              int64_t batch_size, int64_t* batch_out, int64_t* nodeset_out,
                              int64_t* n_nodeset) {
  return sample_batch_easy(*reinterpret_cast<MTState*>(mt), positives, P, n_items, batch_size,
                           batch_out, nodeset_out, n_nodeset);
}

// ------------------------------------------------------------------ walks
int64_t pinsage_walk_mt_workspace(int64_t n_src, int64_t n_hops) {
  const int64_t chunks = 1024;
  return align_up(chunks * (int64_t)sizeof(MTChunk), 256) + 256 +
         align_up(std::max<int64_t>(n_src, 1) * 3 * n_hops * 4, 256);
}

int pinsage_walk_mt(const int64_t* indptr, const int32_t* indices, int64_t n_all,
                    const int64_t* sources, int64_t n_src, int64_t n_hops, float alpha, void* mt,
                    void* ws, int64_t ws_bytes, int32_t* trace, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  PS_REQUIRE(n_src >= 0 && n_hops > 0 && n_all > 0, kErrArg, "walk_mt: bad sizes");
  if (n_src == 0) return kOk;
  MTState& g = *reinterpret_cast<MTState*>(mt);
  const int64_t kChunks = 1024;
  const int64_t desc_bytes = align_up(kChunks * (int64_t)sizeof(MTChunk), 256);
  char* base = static_cast<char*>(ws);
  MTChunk* desc_dev = reinterpret_cast<MTChunk*>(base);
  int* err_dev = reinterpret_cast<int*>(base + desc_bytes);
  uint32_t* raw = reinterpret_cast<uint32_t*>(base + desc_bytes + 256);
  const int64_t per_src = 3 * n_hops;
  const int64_t room = (ws_bytes - desc_bytes - 256) / (per_src * 4);
  PS_REQUIRE(room >= 1, kErrWorkspace, "walk_mt: workspace too small for one source");
  std::vector<MTChunk> desc((size_t)kChunks);
  PS_CHECK_HIP(hipMemsetAsync(err_dev, 0x7f, 4, st));
  for (int64_t r0 = 0; r0 < n_src; r0 += room) {
    const int64_t nr = std::min(room, n_src - r0);
    const int64_t spc = (nr + kChunks - 1) / kChunks;  // sources per chunk
    const int64_t n_chunks = (nr + spc - 1) / spc;
    const int64_t wpc = spc * per_src;
    for (int64_t c = 0; c < n_chunks; ++c) {
      MTChunk& d = desc[(size_t)c];
      std::memcpy(d.s, g.s, sizeof(d.s));
      d.next = g.next;
      d.avail = (uint32_t)g.avail();
      const int64_t words = std::min(wpc, (nr - c * spc) * per_src);
      g.skip(words);
    }
    PS_CHECK_HIP(hipMemcpyAsync(desc_dev, desc.data(), (size_t)n_chunks * sizeof(MTChunk),
                                hipMemcpyHostToDevice, st));
    PS_TRY(launch_mt_expand(desc_dev, n_chunks, wpc, nr * per_src, raw, st));
    PS_TRY(launch_walk(indptr, indices, sources + r0, nr, n_hops, alpha, raw, 0, 0, 0,
                       trace + r0 * n_hops, err_dev, st));
    PS_CHECK_HIP(hipStreamSynchronize(st));  // desc host buffer is reused next round
  }
  int err = 0;
  PS_CHECK_HIP(hipMemcpy(&err, err_dev, 4, hipMemcpyDeviceToHost));
  if (err != 0x7f7f7f7f) {
    set_error("walk: zero-degree node met (the reference's torch.randint(0) raises here)");
    return kErrGraph;
  }
  return kOk;
}

int pinsage_walk_philox(const int64_t* indptr, const int32_t* indices, int64_t n_all,
                        const int64_t* sources, int64_t n_src, int64_t n_hops, float alpha,
                        uint64_t seed, uint32_t offset, int64_t src_base, int32_t* trace,
                        void* stream) {
  hipStream_t st = (hipStream_t)stream;
  PS_REQUIRE(n_src >= 0 && n_hops > 0 && n_all > 0, kErrArg, "walk_philox: bad sizes");
  if (n_src == 0) return kOk;
  int* err_dev = nullptr;
  PS_CHECK_HIP(hipMallocAsync((void**)&err_dev, 4, st));
  PS_CHECK_HIP(hipMemsetAsync(err_dev, 0x7f, 4, st));
  int rc = launch_walk(indptr, indices, sources, n_src, n_hops, alpha, nullptr, seed, offset,
                       src_base, trace, err_dev, st);
  int err = 0x7f7f7f7f;
  if (rc == kOk) {
    PS_CHECK_HIP(hipMemcpyAsync(&err, err_dev, 4, hipMemcpyDeviceToHost, st));
    PS_CHECK_HIP(hipStreamSynchronize(st));
  }
  PS_CHECK_HIP(hipFreeAsync(err_dev, st));
  if (rc != kOk) return rc;
  if (err != 0x7f7f7f7f) {
    set_error("walk: zero-degree node met (the reference's torch.randint(0) raises here)");
    return kErrGraph;
  }
  return kOk;
}

// ------------------------------------------------------------------ fused walk + top-k
// Workspace: [MT chunk states | err | n_runs[R] | runs[R][n_hops] | MT raw words[R][3 n_hops]]
// for R sources per round (R = all of them with pinsage_ppr_topk_workspace's size).
static int64_t ppr_round_bytes(int64_t n_hops, bool mt) {
  return 4 + n_hops * 8 + (mt ? 3 * n_hops * 4 : 0);
}
static constexpr int64_t kPprChunks = 1024;
static int64_t ppr_fixed_bytes() {
  return align_up(kPprChunks * (int64_t)sizeof(MTChunk), 256) + 256;
}

int64_t pinsage_ppr_topk_workspace(int64_t n_src, int64_t n_hops, int rng_mt) {
  return ppr_fixed_bytes() + 3 * 256 + std::max<int64_t>(n_src, 1) * ppr_round_bytes(n_hops, rng_mt != 0);
}

int pinsage_ppr_topk(const int64_t* indptr, const int32_t* indices, int64_t n_all,
                     const int64_t* sources, int64_t n_src, int64_t n_hops, float alpha, int64_t k,
                     void* mt, uint64_t seed, uint32_t offset, int64_t src_base, void* ws,
                     int64_t ws_bytes, double* w_out, int64_t* nb_out, float* wn_out,
                     int32_t* nb32_out, int64_t t_norm, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  PS_REQUIRE(n_src >= 0 && n_hops > 0 && n_all > 0, kErrArg, "ppr_topk: bad sizes");
  PS_REQUIRE(k >= 1 && k <= n_all, kErrArg, "ppr_topk: k out of range (torch: selected index k out of range)");
  PS_REQUIRE(k * 64 <= n_all, kErrArg,
             "ppr_topk: the nth_element regime (k * 64 > n_all) needs pinsage_visit_topk");
  PS_REQUIRE(n_hops < 65536 && k + n_hops < 65536, kErrArg, "ppr_topk: n_hops / k too large");
  PS_REQUIRE(n_hops <= 8192, kErrArg, "ppr_topk: n_hops too large for the LDS sort");
  PS_REQUIRE(n_all < (int64_t)0xFFFFFFFF, kErrArg, "ppr_topk: n_all must fit 32 bits");
  PS_REQUIRE(!wn_out || (t_norm >= 1 && t_norm <= k), kErrArg, "ppr_topk: t_norm must be in [1, k]");
  if (n_src == 0) return kOk;
  const bool use_mt = mt != nullptr;
  char* base = static_cast<char*>(ws);
  MTChunk* desc_dev = reinterpret_cast<MTChunk*>(base);
  const int64_t fixed = ppr_fixed_bytes();
  int* err_dev = reinterpret_cast<int*>(base + fixed - 256);
  const int64_t room = (ws_bytes - fixed - 3 * 256) / ppr_round_bytes(n_hops, use_mt);
  PS_REQUIRE(room >= 1, kErrWorkspace, "ppr_topk: workspace too small for one source");
  const int64_t R = std::min(room, n_src);
  int* nr_dev = reinterpret_cast<int*>(base + fixed);
  uint2* runs_dev = reinterpret_cast<uint2*>(base + fixed + align_up(R * 4, 256));
  uint32_t* raw = reinterpret_cast<uint32_t*>(base + fixed + align_up(R * 4, 256) +
                                              align_up(R * n_hops * 8, 256));
  PS_CHECK_HIP(hipMemsetAsync(err_dev, 0x7f, 4, st));
  std::vector<MTChunk> desc(use_mt ? (size_t)kPprChunks : 0);
  const int64_t per_src = 3 * n_hops;
  for (int64_t r0 = 0; r0 < n_src; r0 += R) {
    const int64_t nr = std::min(R, n_src - r0);
    if (use_mt) {
      MTState& g = *reinterpret_cast<MTState*>(mt);
      const int64_t spc = (nr + kPprChunks - 1) / kPprChunks;
      const int64_t n_chunks = (nr + spc - 1) / spc;
      const int64_t wpc = spc * per_src;
      for (int64_t c = 0; c < n_chunks; ++c) {
        MTChunk& d = desc[(size_t)c];
        std::memcpy(d.s, g.s, sizeof(d.s));
        d.next = g.next;
        d.avail = (uint32_t)g.avail();
        g.skip(std::min(wpc, (nr - c * spc) * per_src));
      }
      PS_CHECK_HIP(hipMemcpyAsync(desc_dev, desc.data(), (size_t)n_chunks * sizeof(MTChunk),
                                  hipMemcpyHostToDevice, st));
      PS_TRY(launch_mt_expand(desc_dev, n_chunks, wpc, nr * per_src, raw, st));
    }
    PS_TRY(launch_walk_runs(indptr, indices, sources + r0, nr, (int)n_hops, alpha,
                            use_mt ? raw : nullptr, seed, offset, src_base + r0, runs_dev, nr_dev,
                            err_dev, st));
    PS_TRY(launch_heap_topk(runs_dev, nr_dev, nr, (int)n_hops, (int)k, w_out ? w_out + r0 * k : nullptr,
                            nb_out ? nb_out + r0 * k : nullptr, wn_out ? wn_out + r0 * t_norm : nullptr,
                            nb32_out ? nb32_out + r0 * t_norm : nullptr, (int)t_norm, st));
    if (use_mt && r0 + nr < n_src) PS_CHECK_HIP(hipStreamSynchronize(st));  // desc is reused
  }
  int err = 0;
  PS_CHECK_HIP(hipMemcpyAsync(&err, err_dev, 4, hipMemcpyDeviceToHost, st));
  PS_CHECK_HIP(hipStreamSynchronize(st));
  if (err != 0x7f7f7f7f) {
    set_error("walk: zero-degree node met (the reference's torch.randint(0) raises here)");
    return kErrGraph;
  }
  return kOk;
}

int pinsage_ppr_topk_segments(const int64_t* indptr, const int32_t* indices, int64_t n_all,
                              const int64_t* sources, int64_t n_seg, const int64_t* seg_start,
                              const uint64_t* seg_seed, const int64_t* seg_base, int64_t n_hops,
                              float alpha, int64_t k, uint32_t offset, void* ws, int64_t ws_bytes,
                              double* w_out, int64_t* nb_out, float* wn_out, int32_t* nb32_out,
                              int64_t t_norm, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  PS_REQUIRE(n_seg >= 1 && seg_start && seg_seed && seg_base && seg_start[0] == 0, kErrArg,
             "ppr_topk_segments: bad segment table");
  for (int64_t i = 0; i < n_seg; ++i)
    PS_REQUIRE(seg_start[i + 1] >= seg_start[i], kErrArg, "ppr_topk_segments: segments out of order");
  const int64_t n_src = seg_start[n_seg];
  PS_REQUIRE(n_hops > 0 && n_all > 0, kErrArg, "ppr_topk: bad sizes");
  PS_REQUIRE(k >= 1 && k <= n_all, kErrArg, "ppr_topk: k out of range (torch: selected index k out of range)");
  PS_REQUIRE(k * 64 <= n_all, kErrArg,
             "ppr_topk: the nth_element regime (k * 64 > n_all) needs pinsage_visit_topk");
  PS_REQUIRE(n_hops < 65536 && k + n_hops < 65536, kErrArg, "ppr_topk: n_hops / k too large");
  PS_REQUIRE(n_hops <= 8192, kErrArg, "ppr_topk: n_hops too large for the LDS sort");
  PS_REQUIRE(n_all < (int64_t)0xFFFFFFFF, kErrArg, "ppr_topk: n_all must fit 32 bits");
  PS_REQUIRE(!wn_out || (t_norm >= 1 && t_norm <= k), kErrArg, "ppr_topk: t_norm must be in [1, k]");
  if (n_src == 0) return kOk;
  char* base = static_cast<char*>(ws);
  const int64_t fixed = ppr_fixed_bytes();
  int* err_dev = reinterpret_cast<int*>(base + fixed - 256);
  const int64_t room = (ws_bytes - fixed - 3 * 256) / ppr_round_bytes(n_hops, false);
  PS_REQUIRE(room >= n_src, kErrWorkspace,
             "ppr_topk_segments: workspace below pinsage_ppr_topk_workspace(n_src, n_hops, 0)");
  int* nr_dev = reinterpret_cast<int*>(base + fixed);
  uint2* runs_dev = reinterpret_cast<uint2*>(base + fixed + align_up(n_src * 4, 256));
  PS_CHECK_HIP(hipMemsetAsync(err_dev, 0x7f, 4, st));
  // one walk launch per segment (its own key and source numbering), one top-k
  // pass over every segment's runs, one zero-degree check
  for (int64_t i = 0; i < n_seg; ++i) {
    const int64_t s0 = seg_start[i], ns = seg_start[i + 1] - s0;
    PS_TRY(launch_walk_runs(indptr, indices, sources + s0, ns, (int)n_hops, alpha, nullptr, seg_seed[i],
                            offset, seg_base[i], runs_dev + s0 * n_hops, nr_dev + s0, err_dev, st));
  }
  PS_TRY(launch_heap_topk(runs_dev, nr_dev, n_src, (int)n_hops, (int)k, w_out, nb_out, wn_out, nb32_out,
                          (int)t_norm, st));
  int err = 0;
  PS_CHECK_HIP(hipMemcpyAsync(&err, err_dev, 4, hipMemcpyDeviceToHost, st));
  PS_CHECK_HIP(hipStreamSynchronize(st));
  if (err != 0x7f7f7f7f) {
    set_error("walk: zero-degree node met (the reference's torch.randint(0) raises here)");
    return kErrGraph;
  }
  return kOk;
}

// ------------------------------------------------------------------ visits / top-k
int64_t pinsage_visit_topk_scratch(int64_t n_src, int64_t n_all, int64_t k) {
  return (k * 64 <= n_all) ? 0 : n_src * n_all * 8;
}

int pinsage_visit_topk(const int32_t* trace, const int64_t* sources, int64_t n_src,
                       int64_t n_hops, int64_t n_all, int64_t k, void* dense_scratch,
                       double* w_out, int64_t* nb_out, float* wn_out, int32_t* nb32_out,
                       int64_t t_norm, void* stream) {
  PS_REQUIRE(k >= 1 && k <= n_all, kErrArg, "visit_topk: k out of range (torch: selected index k out of range)");
  PS_REQUIRE(!wn_out || (t_norm >= 1 && t_norm <= k), kErrArg, "visit_topk: t_norm must be in [1, k]");
  PS_REQUIRE(k * 64 <= n_all || dense_scratch, kErrWorkspace,
             "visit_topk: nth_element regime needs dense scratch");
  PS_REQUIRE(n_all < (int64_t)0xFFFFFFFF, kErrArg, "visit_topk: n_all must fit 32 bits");
  return launch_visit_topk(trace, sources, n_src, n_hops, n_all, k, dense_scratch, w_out, nb_out,
                           wn_out, nb32_out, t_norm, (hipStream_t)stream);
}

int pinsage_visit_dense(const int32_t* trace, const int64_t* sources, int64_t n_src,
                        int64_t n_hops, int64_t n_all, double* dense, void* stream) {
  return launch_visit_dense(trace, sources, n_src, n_hops, n_all, dense, (hipStream_t)stream);
}

// ------------------------------------------------------------------ frontier step
int64_t pinsage_frontier_workspace(int64_t n_items) {
  const int64_t nw = bitset_words(n_items);
  return align_up(nw * 8, 256) + align_up(nw * 4, 256) +
         align_up(std::max<int64_t>(bitset_blocks(n_items), 1) * 4, 256) + 256;
}

int pinsage_frontier_step(const int64_t* nodeset, int64_t n, const int32_t* nb_table, int64_t ld,
                          int64_t T, int64_t n_items, void* ws, int32_t* nodes_out,
                          int32_t* count_out, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  const int64_t nw = bitset_words(n_items);
  char* b = static_cast<char*>(ws);
  auto* bits = reinterpret_cast<unsigned long long*>(b);
  auto* prefix = reinterpret_cast<uint32_t*>(b + align_up(nw * 8, 256));
  auto* bsum = reinterpret_cast<uint32_t*>(b + align_up(nw * 8, 256) + align_up(nw * 4, 256));
  int* err = reinterpret_cast<int*>(b + align_up(nw * 8, 256) + align_up(nw * 4, 256) +
                                    align_up(std::max<int64_t>(bitset_blocks(n_items), 1) * 4, 256));
  PS_CHECK_HIP(hipMemsetAsync(bits, 0, (size_t)nw * 8, st));
  PS_CHECK_HIP(hipMemsetAsync(err, 0, 4, st));
  PS_TRY(launch_mark_i64(bits, nodeset, n, n_items, err, st));
  PS_TRY(launch_mark_table_i64(bits, nodeset, n, nb_table, ld, (int)T, n_items, err, st));
  PS_TRY(launch_set_finalize(bits, bits, nullptr, n_items, bsum, prefix, nodes_out, count_out, st));
  int herr = 0;
  PS_CHECK_HIP(hipMemcpyAsync(&herr, err, 4, hipMemcpyDeviceToHost, st));
  PS_CHECK_HIP(hipStreamSynchronize(st));
  if (herr) {
    set_error("frontier: node id out of range of the feature table (reference: IndexError)");
    return kErrIndex;
  }
  return kOk;
}

int pinsage_frontier_local_idx(const int64_t* nodeset, int64_t n, const int32_t* nb_table, int64_t ld, int64_t T,
                               int64_t n_items, const void* ws, int32_t* local_idx, void* stream) {
  if (n < 0 || T <= 0 || ld < T || n_items <= 0 || !ws) {
    set_error("frontier_local_idx: bad sizes");
    return kErrArg;
  }
  const int64_t nw = bitset_words(n_items);
  const char* b = static_cast<const char*>(ws);
  const auto* bits = reinterpret_cast<const unsigned long long*>(b);
  const auto* prefix = reinterpret_cast<const uint32_t*>(b + align_up(nw * 8, 256));
  return launch_set_rank_table(nodeset, n, nb_table, ld, (int)T, bits, prefix, local_idx, (hipStream_t)stream);
}

// ------------------------------------------------------------------ single kernels
int pinsage_linear(const float* A, int64_t lda, const int32_t* a_idx, int64_t M, int64_t K,
                   const float* W, const float* bias, int64_t N, int act, float* C, int64_t ldc,
                   void* stream) {
  GemmParams p;
  p.M = (int)M;
  p.N = (int)N;
  p.K = (int)K;
  p.a = A;
  p.lda = lda;
  p.a_idx = a_idx;
  p.b = W;
  p.ldb = K;
  p.c = C;
  p.ldc = ldc;
  p.bias = bias;
  p.act = act != 0;
  return launch_gemm(p, (hipStream_t)stream);
}

int64_t pinsage_wgrad_scratch_bytes(int64_t M, int64_t N) {
  if (M <= 0 || N <= 0) return 0;
  return align_up(wgrad_kw_tickets((int)M, (int)N) * 4, 256) + wgrad_kw_slab_floats((int)M, (int)N) * 4 +
         wgrad_kw_bslab_floats((int)M) * 4;
}

int pinsage_wgrad(int64_t M, int64_t N, const int* K_dev, int64_t K_max, const float* A, int64_t lda,
                  const float* B, int64_t ldb, const int32_t* b_idx, int64_t N1, const float* B2, int64_t ldb2,
                  float* dst, int64_t ld_dst, float* dst_b, int splits, void* scratch, float* adam_p,
                  float* adam_m, float* adam_v, float* adam_pb, float* adam_mb, float* adam_vb,
                  const float* coef, double beta1, double beta2, float eps, void* stream) {
  PS_REQUIRE(M > 0 && N > 0 && M <= INT32_MAX && N <= INT32_MAX && K_max >= 0 && K_max <= INT32_MAX &&
                 splits >= 0 && scratch,
             kErrArg, "wgrad: bad argument");
  KwParams p;
  p.A = A;
  p.lda = lda;
  p.M = (int)M;
  p.B = B;
  p.ldb = ldb;
  p.b_idx = b_idx;
  p.N1 = B2 ? (int)N1 : -1;
  p.B2 = B2;
  p.ldb2 = ldb2;
  p.N = (int)N;
  p.K_dev = K_dev;
  p.K_max = (int)K_max;
  p.dst = dst;
  p.ld_dst = ld_dst;
  p.dst_b = dst_b;
  if (adam_p) {
    p.ad.p = adam_p;
    p.ad.m = adam_m;
    p.ad.v = adam_v;
    p.ad.pb = adam_pb;
    p.ad.mb = adam_mb;
    p.ad.vb = adam_vb;
    p.ad.coef = coef;
    p.ad.beta1 = beta1;
    p.ad.beta2 = beta2;
    p.ad.eps = eps;
  }
  char* sc = static_cast<char*>(scratch);
  p.cnt = reinterpret_cast<int*>(sc);
  sc += align_up(wgrad_kw_tickets((int)M, (int)N) * 4, 256);
  p.slab = reinterpret_cast<float*>(sc);
  sc += wgrad_kw_slab_floats((int)M, (int)N) * 4;
  p.bslab = reinterpret_cast<float*>(sc);
  p.S = splits;
  return launch_wgrad_kw(p, (hipStream_t)stream);
}

int pinsage_wgrad_probe(int64_t M, int64_t N, const int* K_dev, int64_t K_max, const float* A, const float* B,
                        const int32_t* b_idx, float* dst, float* dst_b, int splits, void* scratch, int probe,
                        void* stream) {
  PS_REQUIRE(M > 0 && N > 0 && M <= INT32_MAX && N <= INT32_MAX && K_max >= 0 && K_max <= INT32_MAX &&
                 splits >= 0 && scratch && probe >= 1 && probe <= 4,
             kErrArg, "wgrad_probe: bad argument (probe 1-4)");
  KwParams p;
  p.A = A;
  p.lda = M;
  p.M = (int)M;
  p.B = B;
  p.ldb = N;
  p.b_idx = b_idx;
  p.N = (int)N;
  p.K_dev = K_dev;
  p.K_max = (int)K_max;
  p.dst = dst;
  p.ld_dst = N;
  p.dst_b = dst_b;
  char* sc = static_cast<char*>(scratch);
  p.cnt = reinterpret_cast<int*>(sc);
  sc += align_up(wgrad_kw_tickets((int)M, (int)N) * 4, 256);
  p.slab = reinterpret_cast<float*>(sc);
  sc += wgrad_kw_slab_floats((int)M, (int)N) * 4;
  p.bslab = reinterpret_cast<float*>(sc);
  p.S = splits;
  return launch_wgrad_kw_probe(p, probe, (hipStream_t)stream);
}

int pinsage_wgrad_planes(int64_t M, int64_t N, const int* K_dev, int64_t K_max, const uint16_t* A3, int64_t a3_ps,
                         int64_t lda, const uint16_t* B3, int64_t b3_ps, int64_t ldb, const int32_t* b_idx,
                         float* dst, int64_t ld_dst, float* dst_b, int splits, void* scratch, void* stream) {
  PS_REQUIRE(M > 0 && N > 0 && M <= INT32_MAX && N <= INT32_MAX && K_max >= 0 && K_max <= INT32_MAX &&
                 splits >= 0 && scratch && A3 && B3 && a3_ps >= 0 && b3_ps >= 0,
             kErrArg, "wgrad_planes: bad argument");
  KwParams p;
  p.A3 = A3;
  p.a3_ps = a3_ps;
  p.lda = lda;
  p.M = (int)M;
  p.B3 = B3;
  p.b3_ps = b3_ps;
  p.ldb = ldb;
  p.b_idx = b_idx;
  p.N = (int)N;
  p.K_dev = K_dev;
  p.K_max = (int)K_max;
  p.dst = dst;
  p.ld_dst = ld_dst;
  p.dst_b = dst_b;
  char* sc = static_cast<char*>(scratch);
  p.cnt = reinterpret_cast<int*>(sc);
  sc += align_up(wgrad_kw_tickets((int)M, (int)N) * 4, 256);
  p.slab = reinterpret_cast<float*>(sc);
  sc += wgrad_kw_slab_floats((int)M, (int)N) * 4;
  p.bslab = reinterpret_cast<float*>(sc);
  p.S = splits;
  return launch_wgrad_kw(p, (hipStream_t)stream);
}

int pinsage_gemm_ex(int64_t M, int64_t N, int64_t K, int a_kmajor, int b_kmajor, const float* A,
                    int64_t lda, const int32_t* a_idx, const float* B, int64_t ldb,
                    const int32_t* b_idx, float* C, int64_t ldc, const float* bias, int act,
                    int epi, int splits, int cfg, int stream_k, void* stream) {
  if (M < 0 || N <= 0 || K < 0 || M > INT32_MAX || N > INT32_MAX || K > INT32_MAX ||
      (epi != kEpiStore && epi != kEpiAccum && epi != kEpiPartial) || splits < 1 || cfg < -1 ||
      cfg > 5) {
    set_error("gemm_ex: bad argument");
    return kErrArg;
  }
  GemmParams p;
  p.M = (int)M;
  p.N = (int)N;
  p.K = (int)K;
  p.a_kmajor = a_kmajor != 0;
  p.b_kmajor = b_kmajor != 0;
  p.a = A;
  p.lda = lda;
  p.a_idx = a_idx;
  p.b = B;
  p.ldb = ldb;
  p.b_idx = b_idx;
  p.c = C;
  p.ldc = ldc;
  p.bias = bias;
  p.act = act != 0;
  p.epi = epi;
  p.splits = splits;
  p.cfg = cfg;
  p.stream_k = stream_k;
  if (cfg == 5 && (!gemm_ws_supported(p) || stream_k == 1 || gemm_default_prec() != 1)) {
    set_error("gemm_ex: cfg 5 needs split-bf16 products, K-major A and B, a store epilogue, K % 32 == 0, "
              "N % 128 == 0 and no stream-K");
    return kErrArg;
  }
  if (stream_k != 0) {  // library-owned stream-K scratch (tests and microbenchmarks)
    static float* slab = nullptr;
    static int* cnt = nullptr;
    constexpr int64_t kCnt = 1 << 20;
    if (!slab) {
      if (hipMalloc(&slab, (size_t)gemm_sk_slab_floats() * sizeof(float)) != hipSuccess ||
          hipMalloc(&cnt, (size_t)kCnt * sizeof(int)) != hipSuccess ||
          hipMemset(cnt, 0, (size_t)kCnt * sizeof(int)) != hipSuccess) {
        set_error("gemm_ex: stream-K scratch allocation failed");
        return kErrHip;
      }
    }
    p.sk_slab = slab;
    p.sk_cnt = cnt;
    p.sk_cnt_len = kCnt;
  }
  return launch_gemm(p, (hipStream_t)stream);
}

int pinsage_gemm_set_prec(int prec) {
  if (prec < 0 || prec > 1) {
    set_error("gemm_set_prec: 0 (fp32 MFMA) or 1 (split bf16)");
    return kErrArg;
  }
  gemm_set_default_prec(prec);
  return kOk;
}

int pinsage_gemm_get_prec(void) { return gemm_default_prec(); }

int pinsage_split_planes(const float* W, int64_t rows, int64_t cols, int64_t ldw, uint16_t* out,
                         void* stream) {
  return launch_split_planes(W, rows, cols, ldw, out, (hipStream_t)stream);
}

int64_t pinsage_triplet_loss_scratch_bytes(int64_t B, int64_t d) {
  return B <= 0 || d <= 0 ? -1 : triplet_loss_scratch_bytes(B, d);
}

int pinsage_triplet_loss(const float* Z, int64_t B, int64_t d, float margin, float* G, void* scratch, float* scal,
                         void* stream) {
  if (!Z || !G || !scratch || !scal || B <= 0 || B > (INT32_MAX / 9) || d <= 0 || d > 256) {
    set_error("triplet_loss: bad argument");
    return kErrArg;
  }
  return launch_triplet_loss(Z, (int)B, (int)d, margin, G, scratch, scal, (hipStream_t)stream);
}

int pinsage_split_ilv(const float* src, int64_t ld, int64_t rows, int64_t K, uint16_t* out, int64_t ldo,
                      void* stream) {
  if (K <= 0 || K > INT32_MAX) {
    set_error("split_ilv: bad argument");
    return kErrArg;
  }
  return launch_split_ilv(src, ld, rows, (int)K, out, ldo, (hipStream_t)stream);
}

int pinsage_linear_ilv(const uint16_t* A_ilv, int64_t lda_ilv, const int32_t* a_idx, int64_t M, const int* M_dev,
                       int64_t M_max, int64_t K, const float* W, const uint16_t* W_ilv, int64_t ldw_ilv,
                       const float* bias, int64_t N, int act, float* C, int64_t ldc, void* stream) {
  if (M < 0 || N <= 0 || K <= 0 || M > INT32_MAX || N > INT32_MAX || K > INT32_MAX || M_max < 0 ||
      M_max > INT32_MAX || (M_dev && M_max == 0)) {
    set_error("linear_ilv: bad argument");
    return kErrArg;
  }
  GemmParams p;
  p.M = (int)M;
  p.M_dev = M_dev;
  p.M_max = (int)M_max;
  p.N = (int)N;
  p.K = (int)K;
  p.a_ilv = A_ilv;
  p.lda_ilv = lda_ilv;
  p.a_idx = a_idx;
  p.b = W;
  p.ldb = K;
  p.b_ilv = W_ilv;
  p.ldb_ilv = W_ilv ? ldw_ilv : 0;
  p.c = C;
  p.ldc = ldc;
  p.bias = bias;
  p.act = act != 0;
  p.prec = 1;
  return launch_gemm(p, (hipStream_t)stream);
}

int pinsage_linear_split_b(const float* A, int64_t lda, const int32_t* a_idx, int64_t M, int64_t K,
                           const float* W, const uint16_t* W_planes, int64_t ldws,
                           const float* bias, int64_t N, int act, float* C, int64_t ldc, int cfg,
                           void* stream) {
  if (M < 0 || N <= 0 || K < 0 || M > INT32_MAX || N > INT32_MAX || K > INT32_MAX || cfg < -1 ||
      cfg > 5) {
    set_error("linear_split_b: bad argument");
    return kErrArg;
  }
  if (ldws != K) {  // pinsage_split_planes writes planes of row stride cols = K, plane stride N*K
    set_error("linear_split_b: W_planes must come from pinsage_split_planes(W, N, K, ...): ldws == K");
    return kErrArg;
  }
  GemmParams p;
  p.M = (int)M;
  p.N = (int)N;
  p.K = (int)K;
  p.a = A;
  p.lda = lda;
  p.a_idx = a_idx;
  p.b = W;
  p.ldb = K;
  p.b_split = W_planes;
  p.ldb_split = ldws;
  p.c = C;
  p.ldc = ldc;
  p.bias = bias;
  p.act = act != 0;
  p.cfg = cfg;
  p.stream_k = 0;
  p.prec = 1;
  return launch_gemm(p, (hipStream_t)stream);
}

int64_t pinsage_knn_scratch_bytes(int64_t n, int64_t batch_rows) {
  return knn_scratch_bytes(n, batch_rows < 1 ? 1 : batch_rows);
}

int pinsage_knn_cosine(const float* emb, int64_t n, int64_t d, int64_t ld, const int64_t* queries,
                       int64_t nq, int64_t k, float eps, void* scratch, int64_t scratch_bytes,
                       float* out_w, int64_t* out_n, void* stream) {
  return launch_knn_cosine(emb, n, d, ld, queries, nq, k, eps, scratch, scratch_bytes, out_w, out_n,
                           nullptr, (hipStream_t)stream);
}

int pinsage_weighted_agg(const float* q, int64_t hid, const int32_t* loc, const float* w,
                         int64_t n_rows, int64_t T, float* agg, void* stream) {
  return launch_agg(q, (int)hid, loc, w, (int)T, nullptr, n_rows, agg, (hipStream_t)stream);
}

int64_t pinsage_fly_workspace_bytes(int64_t n, int64_t B, int64_t n_layers, int64_t T, int64_t n_hops) {
  if (n <= 0 || B <= 0 || n_layers < 1 || n_layers > 8 || T < 1 || n_hops < 1) return -1;
  return fly_workspace_bytes(n, B, n_layers, T, n_hops);
}

int pinsage_fly_init_workspace(void* ws, int64_t n, int64_t B, int64_t n_layers, int64_t T, int64_t n_hops,
                               void* stream) {
  PS_REQUIRE(ws && n > 0 && B > 0 && n_layers >= 1 && n_layers <= 8 && T >= 1 && n_hops >= 1, kErrArg,
             "fly_init_workspace: bad argument");
  return fly_init_workspace(ws, n, B, n_layers, T, n_hops, (hipStream_t)stream);
}

int pinsage_fly_sample(const int64_t* indptr, const int32_t* indices, int64_t n_all, const int64_t* batch,
                       int64_t B, int64_t n, int64_t n_layers, int64_t T, int64_t n_hops, float alpha,
                       const uint64_t* seeds, void* ws, int64_t ws_bytes, int32_t* const* nbt, float* const* wnt,
                       int32_t** tab_ptrs, int64_t rows_cap, int64_t* pos_ids, int* n_x, int64_t* ids_xo,
                       int64_t x_cap, const float* feats, int64_t ld_f, int64_t d, float* fx, int64_t ld_x,
                       int* err, void* stream) {
  PS_REQUIRE(indptr && indices && batch && seeds && ws && nbt && wnt && tab_ptrs && pos_ids && n_x && ids_xo && err,
             kErrArg, "fly_sample: null argument");
  for (int64_t l = 0; l < n_layers; ++l) PS_REQUIRE(nbt[l] && wnt[l], kErrArg, "fly_sample: null table");
  PS_REQUIRE(!fx || (feats && d > 0 && ld_f >= d && ld_x >= d), kErrArg, "fly_sample: feature rows");
  return fly_sample(indptr, indices, n_all, batch, B, n, n_layers, T, n_hops, alpha, seeds, ws, ws_bytes, nbt, wnt,
                    tab_ptrs, rows_cap, pos_ids, n_x, ids_xo, x_cap, feats, ld_f, d, fx, ld_x, err,
                    (hipStream_t)stream);
}

int pinsage_fly_publish_err(const int* err, void* ring, int64_t slot_bytes, int64_t R, const int64_t* ctr,
                            int64_t err_off, void* stream) {
  return fly_publish_err(err, ring, slot_bytes, R, ctr, err_off, (hipStream_t)stream);
}

int pinsage_fly_gate_adam(int* err, float* coef, void* stream) {
  return fly_gate_adam(err, coef, (hipStream_t)stream);
}

int pinsage_conv_agg_project(const float* h, int64_t ldh, int64_t d, const int32_t* self_src,
                             const float* q, int64_t hid, int64_t q_rows, const int32_t* loc,
                             const float* w, int64_t n_rows, int64_t T, const float* W,
                             const float* bias, int64_t out, uint16_t* W_planes, float* y,
                             float* norms, float* agg, void* stream) {
  if (!agg_w_supported(d, hid, out, T) || n_rows < 0 || q_rows <= 0 || n_rows > INT32_MAX || ldh < d ||
      ldh % 4 != 0) {
    set_error("conv_agg_project: out_dim must be 128, 1 <= T <= 64, d + hid a multiple of 64 and d, hid "
              "multiples of 4");
    return kErrArg;
  }
  if (n_rows == 0) return kOk;
  // the engine's kernel (aggw.hip): the form by row count, rows from n_rows
  // (W_planes: scratch of 3 x 128 x (d + hid) bf16 that lets the 32-row form
  // run pipelined, W split into it first; null runs the unpipelined forms)
  return launch_agg_w(h, ldh, (int)d, self_src, q, (int)hid, loc, w, (int)T, nullptr, n_rows, n_rows, W, bias, y,
                      norms, agg, (hipStream_t)stream, nullptr, nullptr, W_planes, 0);
}

int pinsage_gather_rows(const float* h, int64_t ldh, int64_t n_h, int64_t d, const int64_t* idx, int64_t n,
                        float* out, int64_t ldo, void* stream) {
  if (d < 0 || d > INT32_MAX || n < 0 || n_h < 0 || ldh < d || ldo < d) {
    set_error("gather_rows: bad sizes");
    return kErrArg;
  }
  return launch_gather_rows(h, ldh, n_h, (int)d, idx, n, out, ldo, (hipStream_t)stream);
}

int pinsage_concat_linear_l2norm(const float* h, int64_t ldh, const int32_t* self_idx, int64_t n, int64_t d,
                                 const float* agg, int64_t ld_agg, int64_t hid, const float* W,
                                 const float* bias, int64_t out, float* y, float* norms, void* stream) {
  if (n < 0 || n > INT32_MAX || d <= 0 || hid <= 0 || d + hid > INT32_MAX || out <= 0 || out > INT32_MAX ||
      ldh < d || ld_agg < hid || d % 4 != 0) {
    set_error("concat_linear_l2norm: bad sizes");
    return kErrArg;
  }
  if (n == 0) return kOk;
  if (out > 128) {
    // wider than the fused L2-norm epilogue: the GEMM with bias + LeakyReLU,
    // then the row normalisation in place
    GemmParams p;
    p.M = (int)n;
    p.N = (int)out;
    p.K = (int)(d + hid);
    p.a = h;
    p.lda = ldh;
    p.a_idx = self_idx;
    p.K1 = (int)d;
    p.a2 = agg;
    p.lda2 = ld_agg;
    p.b = W;
    p.ldb = d + hid;
    p.c = y;
    p.ldc = out;
    p.bias = bias;
    p.act = true;
    p.stream_k = 0;
    PS_TRY(launch_gemm(p, (hipStream_t)stream));
    return launch_l2norm_rows(y, n, (int)out, norms, (hipStream_t)stream);
  }
  GemmParams p;
  p.M = (int)n;
  p.N = (int)out;
  p.K = (int)(d + hid);
  p.a = h;
  p.lda = ldh;
  p.a_idx = self_idx;
  p.K1 = (int)d;
  p.a2 = agg;
  p.lda2 = ld_agg;
  p.b = W;
  p.ldb = d + hid;
  p.c = y;
  p.ldc = out;
  p.bias = bias;
  p.epi = kEpiL2Norm;
  p.norms = norms;
  p.stream_k = 0;
  return launch_gemm(p, (hipStream_t)stream);
}

int pinsage_norm_lrelu_backward(const float* y, const float* norms, const float* dy, int64_t n, int64_t out,
                                float* dp, void* stream) {
  if (n < 0 || out <= 0 || out > INT32_MAX) {
    set_error("norm_lrelu_backward: bad sizes");
    return kErrArg;
  }
  if (n == 0) return kOk;
  return launch_norm_lrelu_bwd(y, norms, dy, (int)out, nullptr, n, dp, nullptr, 0, nullptr, nullptr, 0,
                               (hipStream_t)stream);
}

}  // extern "C"
