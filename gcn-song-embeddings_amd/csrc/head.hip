// The PinSage head as two fused row-block kernels (pinsage_model.py:223-224,
// G2(leaky_relu(G1 y)); and its backward down to the top conv layer's
// normalisation).  Each workgroup owns 32 rows of the top frontier and keeps
// the whole 128-wide row chain on chip: both 128 x 128 weights are staged in
// LDS once, the intermediate rows never leave the CU, and one launch replaces
// two GEMM launches forward and two GEMMs plus the top layer's
// normalisation backward in reverse.  The rows are few (one per distinct top
// node), so the kernels are latency-bound; what they save is launches and
// round trips, not FLOPs.
//
// MFMA convention as in gemm.hip (v_mfma_f32_32x32x2_f32): in the r-th MFMA of
// k-octet s, lane (l32, h) supplies k = 8s + 4h + r; accumulator element r of
// lane (l32, h) is row (r & 3) + 8 (r >> 2) + 4h, column l32 of the 32 x 32 tile.
#include "common.h"

#include <algorithm>

namespace ps {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kHeadRows = 32;   // rows per workgroup
constexpr int kHeadDim = 128;   // out_dim capacity (4 waves x 32 columns)
constexpr int kHeadLd = 132;    // padded LDS row (floats): b128 fragment reads spread banks

// acc = A[32][K] * B, A rows in sA (ld kHeadLd).  B(k, n) = sW[n][k] (kNK:
// an nn.Linear weight [out][in] used as x W^T; b128 fragment reads) or
// sW[k][n] (!kNK: the weight used as dY W; four b32 reads, consecutive lanes
// on consecutive n).  Fragments of octet s+1 are read while octet s's MFMAs
// run (sched_barrier pins that order).
template <bool kNK>
__device__ __forceinline__ float4 head_bfrag(const float* sW, int n, int k4) {
  if constexpr (kNK) {
    return *reinterpret_cast<const float4*>(sW + n * kHeadLd + k4);
  } else {
    return make_float4(sW[(k4 + 0) * kHeadLd + n], sW[(k4 + 1) * kHeadLd + n],
                       sW[(k4 + 2) * kHeadLd + n], sW[(k4 + 3) * kHeadLd + n]);
  }
}
template <bool kNK>
__device__ __forceinline__ f32x16 head_mm(const float* sA, const float* sW, int n0, int l32,
                                          int h) {
  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  const float* arow = sA + l32 * kHeadLd + 4 * h;
  float4 a = *reinterpret_cast<const float4*>(arow);
  float4 b = head_bfrag<kNK>(sW, n0 + l32, 4 * h);
#pragma unroll
  for (int s = 0; s < kHeadDim / 8; ++s) {
    float4 an = a, bn = b;
    if (s + 1 < kHeadDim / 8) {
      an = *reinterpret_cast<const float4*>(arow + 8 * (s + 1));
      bn = head_bfrag<kNK>(sW, n0 + l32, 8 * (s + 1) + 4 * h);
    }
    __builtin_amdgcn_sched_barrier(0);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.x, b.x, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.y, b.y, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.z, b.z, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.w, b.w, acc, 0, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
    a = an;
    b = bn;
  }
  return acc;
}

// rows [r0, r0+32) of src[R][o] -> sA (zero outside), all threads
// (every global load of a staging pass is issued before the first LDS write:
// one memory round trip per pass, not one per float4)
__device__ __forceinline__ void head_fetch_rows(float4 (&v)[kHeadRows * (kHeadDim / 4) / 256],
                                                const float* __restrict__ src, int64_t r0, int64_t R, int o,
                                                int tid) {
  constexpr int NI = kHeadRows * (kHeadDim / 4) / 256;
#pragma unroll
  for (int j = 0; j < NI; ++j) {
    const int i = tid + 256 * j, row = i / (kHeadDim / 4), c = 4 * (i % (kHeadDim / 4));
    const float4 x = *reinterpret_cast<const float4*>(src + std::min<int64_t>(r0 + row, R - 1) * o + std::min(c, o - 4));
    v[j] = r0 + row < R && c < o ? x : make_float4(0.f, 0.f, 0.f, 0.f);
  }
}
__device__ __forceinline__ void head_put_rows(float* sA, const float4 (&v)[kHeadRows * (kHeadDim / 4) / 256],
                                              int tid) {
  constexpr int NI = kHeadRows * (kHeadDim / 4) / 256;
#pragma unroll
  for (int j = 0; j < NI; ++j) {
    const int i = tid + 256 * j, row = i / (kHeadDim / 4), c = 4 * (i % (kHeadDim / 4));
    *reinterpret_cast<float4*>(sA + row * kHeadLd + c) = v[j];
  }
}
// W[o][o] row-major -> sW (same layout, zero padded to 128 x 128), in two
// halves: the loads into registers (head_fetch_weight), then the LDS writes
// (head_put_weight) -- a kernel issues all of its global loads before its
// first store or LDS write, so its staging costs one memory round trip
constexpr int kHeadWNI = kHeadDim * (kHeadDim / 4) / 256;
__device__ __forceinline__ void head_fetch_weight(float4 (&v)[kHeadWNI], const float* __restrict__ W, int o,
                                                  int tid) {
#pragma unroll
  for (int j = 0; j < kHeadWNI; ++j) {
    const int i = tid + 256 * j, row = i / (kHeadDim / 4), c = 4 * (i % (kHeadDim / 4));
    const float4 x = *reinterpret_cast<const float4*>(W + (int64_t)std::min(row, o - 1) * o + std::min(c, o - 4));
    v[j] = row < o && c < o ? x : make_float4(0.f, 0.f, 0.f, 0.f);
  }
}
__device__ __forceinline__ void head_put_weight(float* sW, const float4 (&v)[kHeadWNI], int tid) {
#pragma unroll
  for (int j = 0; j < kHeadWNI; ++j) {
    const int i = tid + 256 * j, row = i / (kHeadDim / 4), c = 4 * (i % (kHeadDim / 4));
    *reinterpret_cast<float4*>(sW + row * kHeadLd + c) = v[j];
  }
}

__device__ __forceinline__ int head_row(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

// H1 = lrelu(y G1^T + b1), Z = H1 G2^T over the *nrows rows of y
__global__ __launch_bounds__(256) void head_fwd_kernel(const float* __restrict__ y, int o,
                                                       const int* __restrict__ nrows,
                                                       const float* __restrict__ G1w,
                                                       const float* __restrict__ G1b,
                                                       const float* __restrict__ G2w,
                                                       float* __restrict__ H1,
                                                       float* __restrict__ Z) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  float* sA = lds;
  float* sW1 = sA + kHeadRows * kHeadLd;
  float* sW2 = sW1 + kHeadDim * kHeadLd;
  const int64_t R = *nrows;
  const int64_t r0 = (int64_t)blockIdx.x * kHeadRows;
  if (r0 >= R) return;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, l32 = lane & 31, h = lane >> 5;
  const int n0 = 32 * w, col = n0 + l32;
  // every global load first (rows, both weights, the bias), then the LDS writes
  float4 yr[kHeadRows * (kHeadDim / 4) / 256], w1[kHeadWNI], w2[kHeadWNI];
  head_fetch_rows(yr, y, r0, R, o, tid);
  head_fetch_weight(w1, G1w, o, tid);
  head_fetch_weight(w2, G2w, o, tid);
  const float b = col < o ? G1b[col] : 0.f;
  head_put_rows(sA, yr, tid);
  head_put_weight(sW1, w1, tid);
  head_put_weight(sW2, w2, tid);
  __syncthreads();
  f32x16 acc = head_mm<true>(sA, sW1, n0, l32, h);
  __syncthreads();  // every wave is done reading y from sA
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int row = head_row(r, h);
    const float v = col < o ? lrelu(acc[r] + b) : 0.f;
    sA[row * kHeadLd + col] = v;
    if (r0 + row < R && col < o) H1[(r0 + row) * o + col] = v;
  }
  __syncthreads();
  acc = head_mm<true>(sA, sW2, n0, l32, h);
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int row = head_row(r, h);
    if (r0 + row < R && col < o) Z[(r0 + row) * o + col] = acc[r];
  }
}

// dZ rows r0 .. r0+31 formed from the loss's accumulators, dZ[r] = sum_c K[c][r]
// G[c][r] (c = query / positive / negative call, pinsage_training.py:186-189
// with put_embeddings' repeated-id semantics, conv.hip loss), staged in sA and
// written out (the dG2 weight gradient reads them).  Every K and G value of the
// block is loaded in one round; the block then zeroes what it read (the next
// step's loss accumulates into zeros).  K[c][r] = 0 means G[c][r] is +0, so the
// terms it adds change nothing (bitwise the old dZ = sum over k != 0).
constexpr int kHeadRNI = kHeadRows * (kHeadDim / 4) / 256;
__device__ __forceinline__ float4 add4(float4 a, float4 b) {
  return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
}
// Gp (optional): the loss left a repeated rank's rows in Gp (det_put, conv.hip)
// and no rep_sum pass ran; head_sum_reps sums its group rows, from zero in
// position order (pos_sorted, groups p % 3) -- the additions rep_sum_kernel
// makes, so the rows come out bitwise the same.  head_fetch_dz also loads each
// row's position range (o0, o1).
__device__ __forceinline__ void head_fetch_dz(float4 (&g)[3][kHeadRNI], int (&k)[3][kHeadRNI],
                                              int (&o0)[kHeadRNI], int (&o1)[kHeadRNI],
                                              const float* __restrict__ G, const int* __restrict__ Kc,
                                              int64_t S_max, int64_t r0, int64_t R, int o, int tid,
                                              const int* __restrict__ rank_off, bool reps) {
  constexpr int NI = kHeadRNI;
#pragma unroll
  for (int j = 0; j < NI; ++j) {
    const int i = tid + 256 * j, row = i / (kHeadDim / 4), c = 4 * (i % (kHeadDim / 4));
    const bool ok = r0 + row < R && c < o;
    const int64_t rr = std::min<int64_t>(r0 + row, R - 1);
    const int cc = std::min(c, o - 4);
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      const int kv = Kc[q * S_max + rr];
      const float4 gv = *reinterpret_cast<const float4*>(G + ((int64_t)q * S_max + rr) * o + cc);
      k[q][j] = ok ? kv : 0;
      g[q][j] = ok ? gv : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    const int a0 = rank_off[reps ? rr : 0], a1 = rank_off[reps ? rr + 1 : 0];
    o0[j] = reps && ok ? a0 : 0;
    o1[j] = reps && ok ? a1 : 0;
  }
}
constexpr int kHeadRepBatch = 8;  // positions whose rows are in flight together
constexpr int kHeadRepFirst = 4;  // the first positions of every item, all items together
__device__ __forceinline__ void head_rep_add(float4 (&a)[3], int p, const float4& v) {
  const int grp = p % 3;
#pragma unroll
  for (int q = 0; q < 3; ++q)
    if (q == grp) a[q] = add4(a[q], v);
}
__device__ __forceinline__ void head_sum_reps(float4 (&g)[3][kHeadRNI], const int (&o0)[kHeadRNI],
                                              const int (&o1)[kHeadRNI], int o, int tid,
                                              const int32_t* __restrict__ pos_sorted,
                                              const float* __restrict__ Gp) {
  // the first kHeadRepFirst positions of every repeated item: their position
  // ids, then their rows, each as one round of loads over all items (item by
  // item, every item cost two round trips of its own)
  int pp[kHeadRNI][kHeadRepFirst];
  float4 v[kHeadRNI][kHeadRepFirst];
#pragma unroll
  for (int j = 0; j < kHeadRNI; ++j)
#pragma unroll
    for (int t = 0; t < kHeadRepFirst; ++t) {
      const int pv = pos_sorted[std::max(std::min(o0[j] + t, o1[j] - 1), 0)];
      pp[j][t] = o1[j] - o0[j] >= 2 && o0[j] + t < o1[j] ? pv : -1;
    }
#pragma unroll
  for (int j = 0; j < kHeadRNI; ++j) {
    const int c = 4 * ((tid + 256 * j) % (kHeadDim / 4));
#pragma unroll
    for (int t = 0; t < kHeadRepFirst; ++t) {
      const float4 x = *reinterpret_cast<const float4*>(Gp + (int64_t)std::max(pp[j][t], 0) * o + c);
      v[j][t] = pp[j][t] >= 0 ? x : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
#pragma unroll
  for (int j = 0; j < kHeadRNI; ++j) {
    if (o1[j] - o0[j] < 2) continue;
    const int c = 4 * ((tid + 256 * j) % (kHeadDim / 4));
    float4 a[3];
#pragma unroll
    for (int q = 0; q < 3; ++q) a[q] = make_float4(0.f, 0.f, 0.f, 0.f);
    // from zero in position order (rep_sum_kernel's additions)
#pragma unroll
    for (int t = 0; t < kHeadRepFirst; ++t)
      if (pp[j][t] >= 0) head_rep_add(a, pp[j][t], v[j][t]);
    for (int u0 = o0[j] + kHeadRepFirst; u0 < o1[j]; u0 += kHeadRepBatch) {
      int pb[kHeadRepBatch];
      float4 w[kHeadRepBatch];
#pragma unroll
      for (int t = 0; t < kHeadRepBatch; ++t) {
        const int pv = pos_sorted[std::min(u0 + t, o1[j] - 1)];
        pb[t] = u0 + t < o1[j] ? pv : -1;
      }
#pragma unroll
      for (int t = 0; t < kHeadRepBatch; ++t) {
        const float4 x = *reinterpret_cast<const float4*>(Gp + (int64_t)std::max(pb[t], 0) * o + c);
        w[t] = pb[t] >= 0 ? x : make_float4(0.f, 0.f, 0.f, 0.f);
      }
#pragma unroll
      for (int t = 0; t < kHeadRepBatch; ++t)
        if (pb[t] >= 0) head_rep_add(a, pb[t], w[t]);
    }
#pragma unroll
    for (int q = 0; q < 3; ++q) g[q][j] = a[q];
  }
}
__device__ __forceinline__ void head_put_dz(float* sA, float* __restrict__ G, const float4 (&g)[3][kHeadRNI],
                                            const int (&k)[3][kHeadRNI], int64_t S_max, float* __restrict__ dZ,
                                            int64_t r0, int64_t R, int o, int tid) {
  constexpr int NI = kHeadRNI;
#pragma unroll
  for (int j = 0; j < NI; ++j) {
    const int i = tid + 256 * j, row = i / (kHeadDim / 4), c = 4 * (i % (kHeadDim / 4));
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      if (k[q][j]) {
        const float kf = (float)k[q][j];
        v.x += kf * g[q][j].x;
        v.y += kf * g[q][j].y;
        v.z += kf * g[q][j].z;
        v.w += kf * g[q][j].w;
        *reinterpret_cast<float4*>(G + ((int64_t)q * S_max + r0 + row) * o + c) =
            make_float4(0.f, 0.f, 0.f, 0.f);
      }
    }
    *reinterpret_cast<float4*>(sA + row * kHeadLd + c) = v;
    if (r0 + row < R && c < o) *reinterpret_cast<float4*>(dZ + (r0 + row) * o + c) = v;
  }
}

// From the loss's accumulators: dZ (above); dP1 = (dZ G2) * lrelu'(H1); dY =
// dP1 G1; then the top conv layer's normalisation backward (y = u / ||u||,
// u = lrelu(pre)):  dp = lrelu'(y) * (dY - y (y . dY)) / ||u||.  The block
// zeroes the multiplicity counters of its rows once every thread has read them.
__global__ __launch_bounds__(256) void head_bwd_kernel(
    float* __restrict__ G, int* __restrict__ Kc, int64_t S_max, float* __restrict__ dZ, int o,
    const int* __restrict__ nrows, const float* __restrict__ H1, const float* __restrict__ G1w,
    const float* __restrict__ G2w, const float* __restrict__ y, const float* __restrict__ nrm,
    float* __restrict__ dP1, float* __restrict__ dp, const int* __restrict__ rank_off,
    const int32_t* __restrict__ pos_sorted, const float* __restrict__ Gp) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  float* sA = lds;
  float* sW2 = sA + kHeadRows * kHeadLd;
  float* sW1 = sW2 + kHeadDim * kHeadLd;
  float* red = sW1 + kHeadDim * kHeadLd;  // [4 waves][32 rows] partial dots
  const int tid = threadIdx.x;
  const int64_t R = *nrows;
  const int64_t r0 = (int64_t)blockIdx.x * kHeadRows;
  if (r0 >= R) return;
  const int lane = tid & 63, w = tid >> 6, l32 = lane & 31, h = lane >> 5;
  const int n0 = 32 * w, col = n0 + l32;
#ifdef PS_HEAD_PROBE  // (diagnostic build only) wall-clock phases of block 0
  uint64_t pt[10] = {__builtin_amdgcn_s_memrealtime(), 0, 0, 0, 0, 0, 0, 0, 0, 0};
  int pti = 1;
#define PS_HPROBE() do { if (pti < 10) pt[pti++] = __builtin_amdgcn_s_memrealtime(); } while (0)
#else
#define PS_HPROBE() do { } while (0)
#endif
  // this lane's H1 (mask) and y values, fetched beside the staging loads
  // (every load of the staging is unconditional, from a clamped address, and
  // masked after: a load under a branch made the compiler wait for it inside
  // the branch -- 16 serial round trips for these rows alone)
  float hv[16], yv[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int row = head_row(r, h);
    const bool ok = r0 + row < R && col < o;
    const int64_t at = std::min<int64_t>(r0 + row, R - 1) * o + std::min(col, o - 1);
    const float hx = H1[at], yx = y[at];
    hv[r] = ok ? hx : 0.f;
    yv[r] = ok ? yx : 0.f;
  }
  // every global load first (the loss accumulators, both weights, the norms),
  // then the stores and LDS writes: a load issued behind a store waits for it
  // (vmcnt counts both), which made this staging ~10 us of the kernel's ~21
  float4 g[3][kHeadRNI], w1[kHeadWNI], w2[kHeadWNI];
  int k[3][kHeadRNI];
  // repeated ranks summed here (Gp set, rank_off[0] >= 0; rank_off[0] < 0:
  // the loss used atomics into G)
  const bool reps = Gp && rank_off[0] >= 0;
  int o0[kHeadRNI], o1[kHeadRNI];
  head_fetch_dz(g, k, o0, o1, G, Kc, S_max, r0, R, o, tid, rank_off, reps);
  head_fetch_weight(w2, G2w, o, tid);
  head_fetch_weight(w1, G1w, o, tid);
  float inv[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int row = head_row(r, h);
    const float nx = nrm[std::min<int64_t>(r0 + row, R - 1)];
    inv[r] = r0 + row < R ? nx : 1.f;
  }
  PS_HPROBE();
  if (reps) head_sum_reps(g, o0, o1, o, tid, pos_sorted, Gp);
  PS_HPROBE();
  head_put_dz(sA, G, g, k, S_max, dZ, r0, R, o, tid);
  PS_HPROBE();
  head_put_weight(sW2, w2, tid);
  head_put_weight(sW1, w1, tid);
  PS_HPROBE();
#pragma unroll
  for (int r = 0; r < 16; ++r) inv[r] = 1.f / inv[r];
  __syncthreads();
  PS_HPROBE();
  if (tid < 3 * kHeadRows) {  // every K of the block's rows has been read
    const int q = tid / kHeadRows, row = tid % kHeadRows;
    if (r0 + row < R) Kc[q * S_max + r0 + row] = 0;
  }
  f32x16 acc = head_mm<false>(sA, sW2, n0, l32, h);
  __syncthreads();  // every wave is done reading dZ from sA
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int row = head_row(r, h);
    float v = 0.f;
    if (r0 + row < R && col < o) {
      v = acc[r] * lrelu_grad(hv[r]);
      dP1[(r0 + row) * o + col] = v;
    }
    sA[row * kHeadLd + col] = v;
  }
  __syncthreads();
  PS_HPROBE();
  acc = head_mm<false>(sA, sW1, n0, l32, h);  // dY
  PS_HPROBE();
  // row dots y . dY: lane-partial over this wave's 32 columns, then 4 waves.
  // The 16 rows' butterflies advance together, one level at a time: each level
  // issues 16 independent cross-lane reads and waits once (row by row, every
  // read waited for the one before it: 80 serial LDS-unit round trips, ~4 us)
  float d[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) d[r] = yv[r] * acc[r];
#pragma unroll
  for (int m = 1; m < 32; m <<= 1) {
    float x[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) x[r] = __shfl_xor(d[r], m, 64);
#pragma unroll
    for (int r = 0; r < 16; ++r) d[r] += x[r];
  }
#pragma unroll
  for (int r = 0; r < 16; ++r)
    if (l32 == 0) red[w * kHeadRows + head_row(r, h)] = d[r];
  __syncthreads();
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int row = head_row(r, h);
    if (r0 + row < R && col < o) {
      const float dot = (red[row] + red[kHeadRows + row]) + (red[2 * kHeadRows + row] + red[3 * kHeadRows + row]);
      dp[(r0 + row) * o + col] = lrelu_grad(yv[r]) * (acc[r] - yv[r] * dot) * inv[r];
    }
  }
#ifdef PS_HEAD_PROBE
  __syncthreads();
  PS_HPROBE();
  if (blockIdx.x == 0 && tid == 0)
    printf("head_bwd probe [10ns]: issue %d reps %d put_dz %d put_w %d sync %d mm1+dP1 %d mm2 %d tail %d\n",
           (int)(pt[1] - pt[0]), (int)(pt[2] - pt[1]), (int)(pt[3] - pt[2]), (int)(pt[4] - pt[3]),
           (int)(pt[5] - pt[4]), (int)(pt[6] - pt[5]), (int)(pt[7] - pt[6]), (int)(pt[8] - pt[7]));
#endif
}

constexpr size_t kHeadFwdLds = (size_t)(kHeadRows + 2 * kHeadDim) * kHeadLd * 4;
constexpr size_t kHeadBwdLds = kHeadFwdLds + 4 * kHeadRows * 4;

static int head_prepare() {
  static int rc = [] {
    if (hipFuncSetAttribute((const void*)head_fwd_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)kHeadFwdLds) != hipSuccess ||
        hipFuncSetAttribute((const void*)head_bwd_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)kHeadBwdLds) != hipSuccess)
      return (int)kErrHip;
    return (int)kOk;
  }();
  if (rc != kOk) set_error("head: cannot raise the dynamic LDS limit");
  return rc;
}

int head_supported(int64_t o) { return o > 0 && o <= kHeadDim && o % 4 == 0; }

int launch_head_fwd(const float* y, int o, const int* nrows, int64_t max_rows, const float* G1w,
                    const float* G1b, const float* G2w, float* H1, float* Z, hipStream_t st) {
  PS_REQUIRE(head_supported(o), kErrArg, "head: out_dim must be a multiple of 4, <= 128");
  PS_TRY(head_prepare());
  if (max_rows <= 0) return kOk;
  hipLaunchKernelGGL(head_fwd_kernel, dim3((unsigned)ceil_div(max_rows, kHeadRows)), dim3(256),
                     kHeadFwdLds, st, y, o, nrows, G1w, G1b, G2w, H1, Z);
  PS_CHECK_LAUNCH();
  return kOk;
}

int launch_head_bwd(float* G, int* Kc, int64_t S_max, float* dZ, int o, const int* nrows,
                    int64_t max_rows, const float* H1, const float* G1w, const float* G2w,
                    const float* y, const float* nrm, float* dP1, float* dp, const int* rank_off,
                    const int32_t* pos_sorted, const float* Gp, hipStream_t st) {
  PS_REQUIRE(head_supported(o), kErrArg, "head: out_dim must be a multiple of 4, <= 128");
  PS_REQUIRE(!Gp || (rank_off && pos_sorted), kErrArg, "head: repeated-rank rows need rank_off and pos_sorted");
  PS_TRY(head_prepare());
  if (max_rows <= 0) return kOk;
  // head_fetch_dz reads rank_off[0] whether or not the repeated ranks are
  // summed: without Gp any valid int works (the loss's Kc counters)
  const int* ro = rank_off ? rank_off : Kc;
  hipLaunchKernelGGL(head_bwd_kernel, dim3((unsigned)ceil_div(max_rows, kHeadRows)), dim3(256),
                     kHeadBwdLds, st, G, Kc, S_max, dZ, o, nrows, H1, G1w, G2w, y, nrm, dP1, dp, ro,
                     pos_sorted, Gp);
  PS_CHECK_LAUNCH();
  return kOk;
}

}  // namespace ps
