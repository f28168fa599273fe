// On-the-fly sampling of a train step's model calls on the device, with no
// host synchronisation (so the whole on-the-fly step is one captured graph):
// relevant_nodes_per_layer (pinsage_model.py:142-154) for the C = 3 calls of
// pinsage_training.py:183-185, laid out as pinsage_model._fly_tables_merged
// lays them out for the engine (Philox mode; bitwise the same tables):
//
//   * call c's node v is c * n + v everywhere (table rows and neighbour ids);
//   * top layer: the calls' nodesets as given (call-major, repeats included)
//     are walked; a repeated id's LAST occurrence in its call owns the id's
//     row (put_embeddings' last write wins, :29), every earlier occurrence is
//     a virtual node x0 + j (x0 = C n, j in call-major position order) whose
//     top-layer row holds its own draws and whose rows below are its real
//     node's;
//   * layer below: unique(cat(nb.flatten(), cur)) over every row drawn (:152),
//     walked per call (each call's segment keyed by its own seed, sources
//     numbered from 0 within the call), rows written at the nodes' ids.
//
// Every size lives on the device: the walks and top-k run over capacity grids
// and read their counts; the sets are bitmaps over [0, C n) (frontier.hip).
// A walk meeting a zero-degree node sets err[0] (as pinsage_ppr_topk), a drawn
// neighbour id >= n sets err[1] (the reference's h[nb] raises there).
#include <algorithm>

#include "common.h"

namespace ps {

int64_t bitset_words(int64_t universe);
int launch_set_finalize(unsigned long long*, const unsigned long long*, const unsigned long long*, int64_t,
                        uint32_t*, uint32_t*, int32_t*, int*, hipStream_t);
int ppr_walk_lds_bytes(int n_hops, int* P_out);
int launch_walk_runs_seg(const int64_t* indptr, const int32_t* indices, const int64_t* sources64,
                         const int32_t* sources32, int64_t n_src_cap, const int* seg, int C, const uint64_t* seeds,
                         int key_stride, int64_t id_unit, int n_hops, float alpha, uint32_t offset, uint2* runs,
                         int* n_runs, int* err, hipStream_t st);
int launch_heap_topk(const uint2*, const int*, int64_t, int, int, double*, int64_t*, float*, int32_t*, int,
                     hipStream_t, const int* n_src_dev);

constexpr int kFlyC = 3;  // calls per step (q, pos, neg)

// source capacity of every fly layer (0 = top): C B, then min(C n, cap (T + 1))
static void fly_caps(int64_t n, int64_t B, int64_t L, int64_t T, int64_t* caps) {
  int64_t c = kFlyC * B;
  for (int64_t l = 0; l < L; ++l) {
    caps[l] = c;
    c = std::min<int64_t>(kFlyC * n, c * (T + 1));
  }
}

struct FlyWs {
  uint2* runs;
  int* n_runs;
  float* wn;
  int32_t* nb32;
  int64_t* src_top;
  int32_t* cur[2];
  unsigned long long* bits;
  uint32_t* prefix;
  uint32_t* bsum;
  int* cnt;       // [2] member counts (ping-pong)
  int* seg;       // [L][C + 1]
  int* last;      // [C n], -1 between steps
  int* vj;        // [C B] virtual index of a top position, or -1
  int64_t total;
};

static FlyWs fly_carve(void* ws, int64_t n, int64_t B, int64_t L, int64_t T, int64_t n_hops) {
  int64_t caps[64];
  fly_caps(n, B, L, T, caps);
  int64_t cmax = 0;
  for (int64_t l = 0; l < L; ++l) cmax = std::max(cmax, caps[l]);
  const int64_t U = kFlyC * n;
  char* base = static_cast<char*>(ws);
  int64_t off = 0;
  auto take = [&](int64_t bytes) {
    char* p = base ? base + off : nullptr;
    off += align_up(std::max<int64_t>(bytes, 1), 256);
    return p;
  };
  FlyWs w;
  w.runs = reinterpret_cast<uint2*>(take(cmax * n_hops * 8));
  w.n_runs = reinterpret_cast<int*>(take(cmax * 4));
  w.wn = reinterpret_cast<float*>(take(cmax * T * 4));
  w.nb32 = reinterpret_cast<int32_t*>(take(cmax * T * 4));
  w.src_top = reinterpret_cast<int64_t*>(take(kFlyC * B * 8));
  w.cur[0] = reinterpret_cast<int32_t*>(take(cmax * 4));
  w.cur[1] = reinterpret_cast<int32_t*>(take(cmax * 4));
  w.bits = reinterpret_cast<unsigned long long*>(take(bitset_words(U) * 8));
  w.prefix = reinterpret_cast<uint32_t*>(take(bitset_words(U) * 4));
  w.bsum = reinterpret_cast<uint32_t*>(take((bitset_words(U) / 1024 + 2) * 4));
  w.cnt = reinterpret_cast<int*>(take(2 * 4));
  w.seg = reinterpret_cast<int*>(take(L * (kFlyC + 1) * 4));
  w.last = reinterpret_cast<int*>(take(U * 4));
  w.vj = reinterpret_cast<int*>(take(kFlyC * B * 4));
  w.total = off;
  return w;
}

// ---------------------------------------------------------------- kernels
__global__ void fly_fill_kernel(int* __restrict__ p, int64_t n, int v) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    p[i] = v;
}

// top layer's sources (call-major: m = c B + i), the engine's positions
// (3 i + c, the loss's triple layout), each id's last position, the segment
// table, the error flags
__global__ void fly_top_kernel(const int64_t* __restrict__ batch, int B, int64_t n, int64_t* __restrict__ src,
                               int64_t* __restrict__ pos_ids, int* __restrict__ last, int* __restrict__ seg,
                               int* __restrict__ err) {
  const int64_t m = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (m == 0) {
    err[0] = 0x7f7f7f7f;
    err[1] = 0;
    for (int c = 0; c <= kFlyC; ++c) seg[c] = c * B;
  }
  if (m >= (int64_t)kFlyC * B) return;
  const int c = (int)(m / B), i = (int)(m - (int64_t)c * B);
  const int64_t id = batch[(int64_t)i * kFlyC + c] + (int64_t)c * n;
  src[m] = id;
  pos_ids[(int64_t)i * kFlyC + c] = id;
  atomicMax(last + id, (int)m);
}

// one block: positions that are not their id's last occurrence, compacted in
// position order -> virtual nodes j (vj[m] = j, else -1), their real ids, count
__global__ __launch_bounds__(1024) void fly_virtual_kernel(const int64_t* __restrict__ src, int64_t M,
                                                           const int* __restrict__ last, int* __restrict__ vj,
                                                           int64_t* __restrict__ ids_xo, int* __restrict__ n_x) {
  __shared__ int wsum[16];
  __shared__ int carry;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  if (tid == 0) carry = 0;
  __syncthreads();
  for (int64_t m0 = 0; m0 < M; m0 += 1024) {
    const int64_t m = m0 + tid;
    const bool x = m < M && last[src[m]] != (int)m;
    const unsigned long long bal = __ballot(x);
    if (lane == 0) wsum[wv] = __popcll(bal);
    __syncthreads();
    int pre = carry;
    for (int w = 0; w < wv; ++w) pre += wsum[w];
    const int j = pre + __popcll(bal & ((1ull << lane) - 1ull));
    if (m < M) vj[m] = x ? j : -1;
    if (x) ids_xo[j] = src[m];
    __syncthreads();
    if (tid == 0) {
      int t = 0;
      for (int w = 0; w < 16; ++w) t += wsum[w];
      carry += t;
    }
    __syncthreads();
  }
  if (tid == 0) *n_x = carry;
}

// table rows of the top layer: id's row from its last position, virtual rows
// x0 + j from theirs; neighbour ids moved into the source's call range
__global__ void fly_top_tables_kernel(const int64_t* __restrict__ src, int B, int T, int64_t n,
                                      const int* __restrict__ last, const int* __restrict__ vj, int64_t x0,
                                      const int32_t* __restrict__ nb32, const float* __restrict__ wn,
                                      int32_t* __restrict__ nbt, float* __restrict__ wnt, int* __restrict__ err) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (int64_t)kFlyC * B * T) return;
  const int64_t m = e / T;
  const int t = (int)(e - m * T);
  const int c = (int)(m / B);
  const int64_t id = src[m];
  const int64_t row = vj[m] >= 0 ? x0 + vj[m] : id;
  const int32_t v = nb32[e];
  // a drawn id outside [0, n) flags err[1] and is stored as the source itself
  // with weight 0, so no table entry ever names a node outside the universe
  // (the engine's frontier marks table ids unchecked, before the error is read)
  const bool bad = v < 0 || v >= n;
  if (bad) atomicOr(err + 1, 1);
  nbt[row * T + t] = bad ? (int32_t)id : v + (int32_t)(c * n);
  wnt[row * T + t] = bad ? 0.f : wn[e];
  (void)last;
}

// table rows of a lower layer: every source (sorted ids) at its own id
__global__ void fly_tables_kernel(const int32_t* __restrict__ cur, const int* __restrict__ seg, int T, int64_t n,
                                  const int32_t* __restrict__ nb32, const float* __restrict__ wn,
                                  int32_t* __restrict__ nbt, float* __restrict__ wnt, int* __restrict__ err) {
  const int64_t N = (int64_t)seg[kFlyC] * T;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < N; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t s = e / T;
    const int t = (int)(e - s * T);
    int c = 0;
    while (c + 1 < kFlyC && s >= seg[c + 1]) ++c;
    const int32_t v = nb32[e];
    const bool bad = v < 0 || v >= n;  // (as fly_top_tables_kernel: the source itself, weight 0)
    if (bad) atomicOr(err + 1, 1);
    const int64_t row = cur[s];
    nbt[row * T + t] = bad ? (int32_t)row : v + (int32_t)(c * n);
    wnt[row * T + t] = bad ? 0.f : wn[e];
  }
}

// mark the next layer's set: every drawn neighbour (moved into its call's
// range) and every current source; sources are int64 (top) or int32 with the
// count in seg[C]
template <typename Src>
__global__ void fly_mark_kernel(unsigned long long* __restrict__ bits, const Src* __restrict__ cur, int64_t n_fixed,
                                const int* __restrict__ seg, int T, int64_t n, int B,
                                const int32_t* __restrict__ nb32) {
  const int64_t ns = seg ? (int64_t)seg[kFlyC] : n_fixed;
  const int64_t N = ns * (T + 1);
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < N; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t s = e / (T + 1);
    const int t = (int)(e - s * (T + 1));
    int c = 0;
    if (seg) {
      while (c + 1 < kFlyC && s >= seg[c + 1]) ++c;
    } else {
      c = (int)(s / B);
    }
    if (t < T && (nb32[s * T + t] < 0 || nb32[s * T + t] >= n)) continue;  // (err[1]: the table kernels)
    const int64_t v = t < T ? (int64_t)nb32[s * T + t] + (int64_t)c * n : (int64_t)cur[s];
    if (v < 0 || v >= kFlyC * n) continue;
    const unsigned long long bit = 1ull << (v & 63);
    if (!(__hip_atomic_load(bits + (v >> 6), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & bit))
      atomicOr(bits + (v >> 6), bit);
  }
}

__global__ void fly_zero_kernel(unsigned long long* __restrict__ p, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    p[i] = 0ull;
}

// segment starts of a finalised set: seg[c] = rank of c n, seg[C] = count
__global__ void fly_segments_kernel(const unsigned long long* __restrict__ bits, const uint32_t* __restrict__ prefix,
                                    const int* __restrict__ count, int64_t n, int* __restrict__ seg) {
  const int c = threadIdx.x;
  if (c > kFlyC) return;
  if (c == 0) {
    seg[0] = 0;
  } else if (c == kFlyC) {
    seg[kFlyC] = *count;
  } else {
    const int64_t v = (int64_t)c * n;
    seg[c] = (int)(prefix[v >> 6] + (uint32_t)__popcll(bits[v >> 6] & ((1ull << (v & 63)) - 1ull)));
  }
}

// the virtual nodes' rows below the top are their real nodes' (every lower
// nodeset contains the one above it), and their feature rows; then each top
// id's last position goes back to -1 (the next step starts clean)
__global__ void fly_finish_kernel(const int* __restrict__ n_x, const int64_t* __restrict__ ids_xo, int64_t x0,
                                  int32_t* const* __restrict__ nbt, float* const* __restrict__ wnt, int n_low, int T,
                                  const float* __restrict__ feats, int64_t ld_f, int d, float* __restrict__ fx,
                                  int64_t ld_x, int64_t n, const int64_t* __restrict__ src, int64_t M,
                                  int* __restrict__ last) {
  const int64_t nx = *n_x;
  const int64_t gt = (int64_t)blockIdx.x * blockDim.x + threadIdx.x, gs = (int64_t)gridDim.x * blockDim.x;
  for (int64_t e = gt; e < nx * n_low * T; e += gs) {
    const int64_t j = e / ((int64_t)n_low * T);
    const int64_t r = e - j * n_low * T;
    const int l = (int)(r / T), t = (int)(r - (int64_t)l * T);
    const int64_t id = ids_xo[j];
    nbt[l][(x0 + j) * T + t] = nbt[l][id * T + t];
    wnt[l][(x0 + j) * T + t] = wnt[l][id * T + t];
  }
  if (fx) {
    for (int64_t e = gt; e < nx * d; e += gs) {
      const int64_t j = e / d;
      const int k = (int)(e - j * d);
      fx[(x0 + j) * ld_x + k] = feats[(ids_xo[j] % n) * ld_f + k];
    }
  }
  for (int64_t m = gt; m < M; m += gs) last[src[m]] = -1;
}

// the step's error flags into the host ring slot the device counter picks
// (read by the host when it next waits for that slot)
__global__ void fly_publish_err_kernel(const int* __restrict__ err, char* __restrict__ ring, int64_t slot_bytes,
                                       int64_t R, const int64_t* __restrict__ ctr, int64_t err_off) {
  if (threadIdx.x < 2) {
    int* dst = reinterpret_cast<int*>(ring + (*ctr % R) * slot_bytes + err_off);
    dst[threadIdx.x] = err[threadIdx.x];
  }
}

// Refuse the step's optimizer update when its sampling failed: err[2] is a
// sticky halt word (set here, cleared only by the host once it has raised the
// error), and a halted step's Adam coefficient bc2 = 0 makes every Adam kernel
// of the step leave parameters and moments untouched (conv.hip adam_kernel,
// reduce_slabs_2d_kernel).  The reference raises before optimizer.step().
__global__ void fly_gate_adam_kernel(int* __restrict__ err, float* __restrict__ coef) {
  if (threadIdx.x == 0) {
    if (err[0] != 0x7f7f7f7f || err[1] != 0) err[2] = 1;
    if (err[2]) coef[1] = 0.f;
  }
}

// ---------------------------------------------------------------- host side
int fly_gate_adam(int* err, float* coef, hipStream_t st) {
  PS_REQUIRE(err && coef, kErrArg, "fly_gate_adam: null argument");
  hipLaunchKernelGGL(fly_gate_adam_kernel, dim3(1), dim3(64), 0, st, err, coef);
  PS_CHECK_LAUNCH();
  return kOk;
}

int fly_publish_err(const int* err, void* ring, int64_t slot_bytes, int64_t R, const int64_t* ctr, int64_t err_off,
                    hipStream_t st) {
  PS_REQUIRE(err && ring && ctr && R > 0 && err_off >= 0 && err_off % 4 == 0 && err_off + 8 <= slot_bytes, kErrArg,
             "fly_publish_err: bad argument");
  hipLaunchKernelGGL(fly_publish_err_kernel, dim3(1), dim3(64), 0, st, err, static_cast<char*>(ring), slot_bytes, R,
                     ctr, err_off);
  PS_CHECK_LAUNCH();
  return kOk;
}

int64_t fly_workspace_bytes(int64_t n, int64_t B, int64_t L, int64_t T, int64_t n_hops) {
  return fly_carve(nullptr, n, B, L, T, n_hops).total;
}

int fly_init_workspace(void* ws, int64_t n, int64_t B, int64_t L, int64_t T, int64_t n_hops, hipStream_t st) {
  FlyWs w = fly_carve(ws, n, B, L, T, n_hops);
  hipLaunchKernelGGL(fly_fill_kernel, dim3(grid_for(kFlyC * n, 256)), dim3(256), 0, st, w.last, kFlyC * n, -1);
  PS_CHECK_LAUNCH();
  return kOk;
}

int fly_sample(const int64_t* indptr, const int32_t* indices, int64_t n_all, const int64_t* batch, int64_t B,
               int64_t n, int64_t L, int64_t T, int64_t n_hops, float alpha, const uint64_t* seeds, void* ws,
               int64_t ws_bytes, int32_t* const* nbt_host, float* const* wnt_host, int32_t** tab_ptrs_dev,
               int64_t rows_cap, int64_t* pos_ids, int* n_x, int64_t* ids_xo, int64_t x_cap, const float* feats,
               int64_t ld_f, int64_t d, float* fx, int64_t ld_x, int* err, hipStream_t st) {
  PS_REQUIRE(L >= 1 && L <= 8 && T >= 1 && n_hops >= 1 && B >= 1 && n >= 1 && n_all >= n, kErrArg,
             "fly_sample: bad sizes");
  PS_REQUIRE(T * 64 <= n_all && n_hops <= 8192 && n_hops + T < 65536, kErrArg,
             "fly_sample: the fused sampler's regime (T * 64 <= n_all, n_hops <= 8192)");
  PS_REQUIRE(kFlyC * n + x_cap <= rows_cap && x_cap >= kFlyC * B && kFlyC * n + x_cap < INT32_MAX, kErrArg,
             "fly_sample: table rows below C n + x_cap, or x_cap below C B");
  FlyWs w = fly_carve(ws, n, B, L, T, n_hops);
  PS_REQUIRE(ws_bytes >= w.total, kErrWorkspace, "fly_sample: workspace below pinsage_fly_workspace_bytes");
  int64_t caps[64];
  fly_caps(n, B, L, T, caps);
  const int64_t U = kFlyC * n, x0 = U, M = kFlyC * B;
  const int64_t nw = bitset_words(U);
  // fly layer k (0 = top) is the engine's layer L - 1 - k
  auto nbt = [&](int64_t k) { return nbt_host[L - 1 - k]; };
  auto wnt = [&](int64_t k) { return wnt_host[L - 1 - k]; };
  hipLaunchKernelGGL(fly_top_kernel, dim3(ceil_div(M, 256)), dim3(256), 0, st, batch, (int)B, n, w.src_top, pos_ids,
                     w.last, w.seg, err);
  PS_CHECK_LAUNCH();
  for (int64_t k = 0; k < L; ++k) {
    int* seg = w.seg + k * (kFlyC + 1);
    const int32_t* cur = k == 0 ? nullptr : w.cur[(k - 1) & 1];
    PS_TRY(launch_walk_runs_seg(indptr, indices, k == 0 ? w.src_top : nullptr, cur, caps[k], seg, kFlyC,
                                seeds + k, (int)L, n, (int)n_hops, alpha, 0u, w.runs, w.n_runs, err, st));
    PS_TRY(launch_heap_topk(w.runs, w.n_runs, caps[k], (int)n_hops, (int)T, nullptr, nullptr, w.wn, w.nb32, (int)T,
                            st, seg + kFlyC));
    if (k == 0) {
      hipLaunchKernelGGL(fly_virtual_kernel, dim3(1), dim3(1024), 0, st, w.src_top, M, w.last, w.vj, ids_xo, n_x);
      PS_CHECK_LAUNCH();
      hipLaunchKernelGGL(fly_top_tables_kernel, dim3(ceil_div(M * T, 256)), dim3(256), 0, st, w.src_top, (int)B,
                         (int)T, n, w.last, w.vj, x0, w.nb32, w.wn, nbt(0), wnt(0), err);
    } else {
      hipLaunchKernelGGL(fly_tables_kernel, dim3(grid_for(caps[k] * T, 256)), dim3(256), 0, st, cur, seg, (int)T, n,
                         w.nb32, w.wn, nbt(k), wnt(k), err);
    }
    PS_CHECK_LAUNCH();
    if (k + 1 == L) break;
    // the next layer's nodeset: unique(cat(nb.flatten(), cur))
    hipLaunchKernelGGL(fly_zero_kernel, dim3(grid_for(nw, 256)), dim3(256), 0, st, w.bits, nw);
    PS_CHECK_LAUNCH();
    if (k == 0)
      hipLaunchKernelGGL(fly_mark_kernel<int64_t>, dim3(grid_for(M * (T + 1), 256)), dim3(256), 0, st, w.bits,
                         w.src_top, M, (const int*)nullptr, (int)T, n, (int)B, w.nb32);
    else
      hipLaunchKernelGGL(fly_mark_kernel<int32_t>, dim3(grid_for(caps[k] * (T + 1), 256)), dim3(256), 0, st, w.bits,
                         cur, (int64_t)0, seg, (int)T, n, (int)B, w.nb32);
    PS_CHECK_LAUNCH();
    int32_t* nxt = w.cur[k & 1];
    PS_TRY(launch_set_finalize(w.bits, w.bits, nullptr, U, w.bsum, w.prefix, nxt, w.cnt + (k & 1), st));
    hipLaunchKernelGGL(fly_segments_kernel, dim3(1), dim3(64), 0, st, w.bits, w.prefix, w.cnt + (k & 1), n,
                       w.seg + (k + 1) * (kFlyC + 1));
    PS_CHECK_LAUNCH();
  }
  hipLaunchKernelGGL(fly_finish_kernel, dim3(grid_for(std::max<int64_t>(x_cap * (L - 1) * T, M), 256)), dim3(256), 0,
                     st, n_x, ids_xo, x0, tab_ptrs_dev, reinterpret_cast<float* const*>(tab_ptrs_dev + L), (int)(L - 1),
                     (int)T, feats, ld_f, (int)d, fx, ld_x, n, w.src_top, M, w.last);
  PS_CHECK_LAUNCH();
  return kOk;
}

}  // namespace ps
