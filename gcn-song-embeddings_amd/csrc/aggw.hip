// The convolution's aggregation and W projection in one kernel
// (pinsage_model.py:201-211):
//
//   agg[f]  = sum_t w[f,t] * q[loc[f,t]]                 (:201-205, weights
//             pre-normalised by their f64 row sum = sum(w*q)/sum(w))
//   y[f]    = normalize(lrelu([h[self f] || agg[f]] W^T + b))   (:208-211)
//
// A workgroup owns a contiguous range of rows (~F / #blocks), in tiles.  Per
// tile it stages [h_self || agg] in LDS -- the self rows gathered from h, the
// aggregate formed right there from the T gathered q rows (fma in slot order
// t = 0, 1, ..., the same arithmetic as agg_kernel) and also written out for
// the backward's weight gradient -- so agg is never read back from memory.
// The projection runs on split-bf16 MFMA (each fp32 operand split exactly into
// bf16 hi / mid / lo in registers, six products, fp32 accumulation:
// bf16split.h), then bias, LeakyReLU and the row L2 norm through an LDS image.
// Two shapes: 16 rows per 512-thread workgroup, two workgroups per CU
// (v_mfma_f32_16x16x32_bf16, each wave 16 output columns over all of K), and
// 32 rows per 1024-thread workgroup, one per CU (v_mfma_f32_32x32x16_bf16, K
// split four ways over the waves; W read once per 32 rows).
#include <algorithm>
#include <cstdlib>

#include "bf16split.h"
#include "common.h"
#include "lds_dma.h"

namespace ps {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kAwRows = 16;     // rows per workgroup
constexpr int kAwOut = 128;     // out_dim (8 column groups of 16)
constexpr int kAwThreads = 512;
constexpr int kAwTMax = 64;     // fanout held in LDS per row

// LDS: A tile [16][K + 4] floats (row stride = 4 mod 64 banks: the b128
// fragment reads of 16 rows x 4 k-quads hit distinct banks), then the tile's
// slot lists.
__device__ __forceinline__ int aw_lda(int K) { return K + 4; }

__global__ __launch_bounds__(kAwThreads, 2) void agg_w_kernel(
    const float* __restrict__ h, int64_t ldh, int d, const int32_t* __restrict__ self_src,
    const float* __restrict__ q, int hid, const int32_t* __restrict__ loc,
    const float* __restrict__ wloc, int T, const int* __restrict__ nS,
    const float* __restrict__ W, const float* __restrict__ bias, float* __restrict__ y,
    float* __restrict__ nrm_out, float* __restrict__ agg) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int K = d + hid, lda = aw_lda(K);
  float* sA = lds;                                          // [16][lda]
  int* sLoc = reinterpret_cast<int*>(lds + kAwRows * lda);  // [16][T]
  float* sW = reinterpret_cast<float*>(sLoc + kAwRows * kAwTMax);  // [16][T]
  int* sSelf = reinterpret_cast<int*>(sW + kAwRows * kAwTMax);     // [16]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // rows dealt in contiguous ranges: block b of G owns [F b / G, F (b+1) / G)
  // in near-equal tiles of <= 16 rows (two blocks per CU: G ~ F / 12 fills them)
  const int64_t F = *nS;
  const int64_t G = gridDim.x, b = blockIdx.x;
  const int64_t rb = F * b / G, len = F * (b + 1) / G - rb;
  const int ntile = (int)((len + kAwRows - 1) / kAwRows);
  for (int tile = 0; tile < ntile; ++tile) {
    const int64_t r0 = rb + len * tile / ntile;
    const int nrows = (int)(rb + len * (tile + 1) / ntile - r0);
    // ---- slot lists and self-row indices of the tile
    for (int i = tid; i < kAwRows * T; i += kAwThreads) {
      const int row = i / T, t = i - row * T;
      const bool ok = row < nrows;
      sLoc[row * kAwTMax + t] = ok ? loc[(r0 + row) * T + t] : 0;
      sW[row * kAwTMax + t] = ok ? wloc[(r0 + row) * T + t] : 0.f;
    }
    if (tid < kAwRows) sSelf[tid] = tid < nrows ? self_src[r0 + tid] : 0;
    __syncthreads();
    // ---- self rows -> A[:, 0:d)
    {
      const int d4 = d >> 2;
      for (int i = tid; i < kAwRows * d4; i += kAwThreads) {
        const int row = i / d4, c4 = i - row * d4;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (row < nrows) v = *reinterpret_cast<const float4*>(h + (int64_t)sSelf[row] * ldh + 4 * c4);
        *reinterpret_cast<float4*>(sA + row * lda + 4 * c4) = v;
      }
    }
    // ---- aggregate -> A[:, d:K) and agg (thread: row tid / 32, float4 columns
    //      (tid % 32) + 32 j); four slots' rows in flight per round
    {
      const int row = tid >> 5, c0 = tid & 31, h4 = hid >> 2;
      const int nj = (h4 + 31) / 32;
      for (int j0 = 0; j0 < nj; j0 += 4) {
        float4 a[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) a[j] = make_float4(0.f, 0.f, 0.f, 0.f);
        if (row < nrows) {
          int t = 0;
          for (; t + 4 <= T; t += 4) {
            float4 x[4][4];
            float w[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
              const float4* qr = reinterpret_cast<const float4*>(q + (int64_t)sLoc[row * kAwTMax + t + u] * hid);
              w[u] = sW[row * kAwTMax + t + u];
#pragma unroll
              for (int j = 0; j < 4; ++j) {
                const int c = min(c0 + 32 * (j0 + j), h4 - 1);
                x[u][j] = qr[c];
              }
            }
#pragma unroll
            for (int u = 0; u < 4; ++u)
#pragma unroll
              for (int j = 0; j < 4; ++j) {
                a[j].x = fmaf(w[u], x[u][j].x, a[j].x);
                a[j].y = fmaf(w[u], x[u][j].y, a[j].y);
                a[j].z = fmaf(w[u], x[u][j].z, a[j].z);
                a[j].w = fmaf(w[u], x[u][j].w, a[j].w);
              }
          }
          for (; t < T; ++t) {
            const float4* qr = reinterpret_cast<const float4*>(q + (int64_t)sLoc[row * kAwTMax + t] * hid);
            const float w = sW[row * kAwTMax + t];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const int c = min(c0 + 32 * (j0 + j), h4 - 1);
              const float4 x = qr[c];
              a[j].x = fmaf(w, x.x, a[j].x);
              a[j].y = fmaf(w, x.y, a[j].y);
              a[j].z = fmaf(w, x.z, a[j].z);
              a[j].w = fmaf(w, x.w, a[j].w);
            }
          }
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int c = c0 + 32 * (j0 + j);
          if (c < h4) {
            *reinterpret_cast<float4*>(sA + row * lda + d + 4 * c) = a[j];
            if (row < nrows) *reinterpret_cast<float4*>(agg + (r0 + row) * hid + 4 * c) = a[j];
          }
        }
      }
    }
    __syncthreads();
    // ---- projection: wave w, columns 16 w .. 16 w + 15, all of K, on split-bf16
    // products (v_mfma_f32_16x16x32_bf16, six per 32-k step; A and W split into
    // bf16 hi / mid / lo in registers, bf16split.h).  Lane l supplies
    // A[row l & 15][k0 + 8 (l >> 4) ..] and W[col l & 15][same k]; W fragments
    // of step s+1 load from L2 while step s runs.
    const int l16 = lane & 15, g = lane >> 4;
    const float* wrow = W + (int64_t)(wave * 16 + l16) * K + 8 * g;
    const float* arow = sA + l16 * lda + 8 * g;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    const int nst = K / 32;
    float4 b0 = *reinterpret_cast<const float4*>(wrow), b1 = *reinterpret_cast<const float4*>(wrow + 4);
    for (int s = 0; s < nst; ++s) {
      const int kn = s + 1 < nst ? 32 * (s + 1) : 32 * s;  // (the last step reloads itself)
      const float4 n0 = *reinterpret_cast<const float4*>(wrow + kn);
      const float4 n1 = *reinterpret_cast<const float4*>(wrow + kn + 4);
      const float* ap = arow + 32 * s;
      bf16x8 aH, aM, aL, bH, bM, bL;
      split3(*reinterpret_cast<const float4*>(ap), *reinterpret_cast<const float4*>(ap + 4), aH, aM, aL);
      split3(b0, b1, bH, bM, bL);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(aL, bH, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(aH, bL, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(aM, bM, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(aM, bH, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(aH, bM, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(aH, bH, acc, 0, 0, 0);
      b0 = n0;
      b1 = n1;
    }
    __syncthreads();  // every wave is done reading the A tile
    // ---- the [16][128] output tile -> LDS, then bias, lrelu, row L2 norm
    float* red = sA;
#pragma unroll
    for (int r = 0; r < 4; ++r) red[(4 * g + r) * kAwOut + wave * 16 + l16] = acc[r];
    __syncthreads();
    {
      const int row = tid >> 5, c4 = tid & 31;  // 4 columns 4 c4 .. 4 c4 + 3
      float v[4];
      float s2 = 0.f;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int col = 4 * c4 + e;
        const float x = lrelu(red[row * kAwOut + col] + bias[col]);
        v[e] = x;
        s2 += x * x;
      }
#pragma unroll
      for (int o = 1; o < 32; o <<= 1) s2 += __shfl_xor(s2, o, 64);
      const float nrm = sqrtf(s2);
      if (row < nrows) {
        *reinterpret_cast<float4*>(y + (r0 + row) * kAwOut + 4 * c4) =
            make_float4(v[0] / nrm, v[1] / nrm, v[2] / nrm, v[3] / nrm);
        if (c4 == 0 && nrm_out) nrm_out[r0 + row] = nrm;
      }
    }
    __syncthreads();  // LDS is reused by the next tile
  }
}

typedef float aw_f32x16 __attribute__((ext_vector_type(16)));

// The 32-row variant (one 1024-thread workgroup per CU, K split four ways
// over the waves, v_mfma_f32_32x32x2_f32): reads W once per 32 rows instead
// of per 16, which wins at K = d + hid = 1024 (C2/C3 layer 0: 41.6 vs 54.9 us
// at C2); the 16-row kernel above wins at K = 640 (C2 layer 1: 22.5 vs 29.9 us).
constexpr int kAw32Rows = 32;     // rows per workgroup
constexpr int kAw32Out = 128;     // out_dim (4 column groups of 32)
constexpr int kAw32Threads = 1024;
constexpr int kAw32TMax = 64;     // fanout held in LDS per row

// LDS: A tile [32][K + 4] floats (row stride = 4 mod 64 banks: b128 fragment
// reads of 16 consecutive rows hit distinct banks), then the tile's slot lists.
__device__ __forceinline__ int aw32_lda(int K) { return K + 4; }

__global__ __launch_bounds__(kAw32Threads) void agg_w32_kernel(
    const float* __restrict__ h, int64_t ldh, int d, const int32_t* __restrict__ self_src,
    const float* __restrict__ q, int hid, const int32_t* __restrict__ loc,
    const float* __restrict__ wloc, int T, const int* __restrict__ nS,
    const float* __restrict__ W, const float* __restrict__ bias, float* __restrict__ y,
    float* __restrict__ nrm_out, float* __restrict__ agg) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int K = d + hid, lda = aw32_lda(K);
  float* sA = lds;                                          // [32][lda]
  int* sLoc = reinterpret_cast<int*>(lds + kAw32Rows * lda);  // [32][T]
  float* sW = reinterpret_cast<float*>(sLoc + kAw32Rows * kAw32TMax);  // [32][T]
  int* sSelf = reinterpret_cast<int*>(sW + kAw32Rows * kAw32TMax);     // [32]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // rows dealt in contiguous ranges: block b of G owns [F b / G, F (b+1) / G)
  // in near-equal tiles of <= 32 rows, so G ~ F / 24 blocks fill the CUs
  const int64_t F = *nS;
  const int64_t G = gridDim.x, b = blockIdx.x;
  const int64_t rb = F * b / G, len = F * (b + 1) / G - rb;
  const int ntile = (int)((len + kAw32Rows - 1) / kAw32Rows);
  for (int tile = 0; tile < ntile; ++tile) {
    const int64_t r0 = rb + len * tile / ntile;
    const int nrows = (int)(rb + len * (tile + 1) / ntile - r0);
    // ---- slot lists and self-row indices of the tile
    for (int i = tid; i < kAw32Rows * T; i += kAw32Threads) {
      const int row = i / T, t = i - row * T;
      const bool ok = row < nrows;
      sLoc[row * kAw32TMax + t] = ok ? loc[(r0 + row) * T + t] : 0;
      sW[row * kAw32TMax + t] = ok ? wloc[(r0 + row) * T + t] : 0.f;
    }
    if (tid < kAw32Rows) sSelf[tid] = tid < nrows ? self_src[r0 + tid] : 0;
    __syncthreads();
    // ---- self rows -> A[:, 0:d)
    {
      const int d4 = d >> 2;
      for (int i = tid; i < kAw32Rows * d4; i += kAw32Threads) {
        const int row = i / d4, c4 = i - row * d4;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (row < nrows) v = *reinterpret_cast<const float4*>(h + (int64_t)sSelf[row] * ldh + 4 * c4);
        *reinterpret_cast<float4*>(sA + row * lda + 4 * c4) = v;
      }
    }
    // ---- aggregate -> A[:, d:K) and agg (thread: row tid / 32, float4 columns
    //      (tid % 32) + 32 j); four slots' rows in flight per round
    {
      const int row = tid >> 5, c0 = tid & 31, h4 = hid >> 2;
      const int nj = (h4 + 31) / 32;
      for (int j0 = 0; j0 < nj; j0 += 4) {
        float4 a[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) a[j] = make_float4(0.f, 0.f, 0.f, 0.f);
        if (row < nrows) {
          int t = 0;
          for (; t + 4 <= T; t += 4) {
            float4 x[4][4];
            float w[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
              const float4* qr = reinterpret_cast<const float4*>(q + (int64_t)sLoc[row * kAw32TMax + t + u] * hid);
              w[u] = sW[row * kAw32TMax + t + u];
#pragma unroll
              for (int j = 0; j < 4; ++j) {
                const int c = min(c0 + 32 * (j0 + j), h4 - 1);
                x[u][j] = qr[c];
              }
            }
#pragma unroll
            for (int u = 0; u < 4; ++u)
#pragma unroll
              for (int j = 0; j < 4; ++j) {
                a[j].x = fmaf(w[u], x[u][j].x, a[j].x);
                a[j].y = fmaf(w[u], x[u][j].y, a[j].y);
                a[j].z = fmaf(w[u], x[u][j].z, a[j].z);
                a[j].w = fmaf(w[u], x[u][j].w, a[j].w);
              }
          }
          for (; t < T; ++t) {
            const float4* qr = reinterpret_cast<const float4*>(q + (int64_t)sLoc[row * kAw32TMax + t] * hid);
            const float w = sW[row * kAw32TMax + t];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const int c = min(c0 + 32 * (j0 + j), h4 - 1);
              const float4 x = qr[c];
              a[j].x = fmaf(w, x.x, a[j].x);
              a[j].y = fmaf(w, x.y, a[j].y);
              a[j].z = fmaf(w, x.z, a[j].z);
              a[j].w = fmaf(w, x.w, a[j].w);
            }
          }
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int c = c0 + 32 * (j0 + j);
          if (c < h4) {
            *reinterpret_cast<float4*>(sA + row * lda + d + 4 * c) = a[j];
            if (row < nrows) *reinterpret_cast<float4*>(agg + (r0 + row) * hid + 4 * c) = a[j];
          }
        }
      }
    }
    __syncthreads();
    // ---- projection: wave (kq, cg), k quarter kq, columns 32 cg ..; split-bf16
    // products (v_mfma_f32_32x32x16_bf16, six per 16-k step: A and W split into
    // bf16 hi / mid / lo in registers, bf16split.h), 2.67x the fp32 MFMA rate:
    // at fp32 MFMA the projection of a 32-row tile (8.4 MFLOP) held a CU ~14 us
    const int cg = wave & 3, kq = wave >> 2;
    const int l32 = lane & 31, hh = lane >> 5;
    const int kspan = K >> 2, kb = kq * kspan;
    const float* wrow = W + (int64_t)(cg * 32 + l32) * K + kb + 8 * hh;
    const float* arow = sA + l32 * lda + kb + 8 * hh;
    aw_f32x16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
    // chunks of two 16-k steps (32 k); W fragments of chunk c+1 load while c runs
    const int nch = kspan / 32;
    float4 bcur[4], bnxt[4];
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      bcur[2 * s2] = *reinterpret_cast<const float4*>(wrow + 16 * s2);
      bcur[2 * s2 + 1] = *reinterpret_cast<const float4*>(wrow + 16 * s2 + 4);
    }
    for (int ch = 0; ch < nch; ++ch) {
      const int k0 = 32 * ch;
      const int kn = ch + 1 < nch ? k0 + 32 : k0;  // (the last chunk reloads itself: no branch)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        bnxt[2 * s2] = *reinterpret_cast<const float4*>(wrow + kn + 16 * s2);
        bnxt[2 * s2 + 1] = *reinterpret_cast<const float4*>(wrow + kn + 16 * s2 + 4);
      }
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const float* ap = arow + k0 + 16 * s2;
        bf16x8 aH, aM, aL, bH, bM, bL;
        split3(*reinterpret_cast<const float4*>(ap), *reinterpret_cast<const float4*>(ap + 4), aH, aM, aL);
        split3(bcur[2 * s2], bcur[2 * s2 + 1], bH, bM, bL);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(aL, bH, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(aH, bL, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(aM, bM, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(aM, bH, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(aH, bM, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(aH, bH, acc, 0, 0, 0);
      }
#pragma unroll
      for (int s2 = 0; s2 < 4; ++s2) bcur[s2] = bnxt[s2];
    }
    __syncthreads();  // every wave is done reading the A tile
    // ---- partial tiles -> LDS red[kq][row][col], fixed-order sum, epilogue
    float* red = sA;  // [4][32][128]
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = (r & 3) + 8 * (r >> 2) + 4 * hh;
      red[(kq * kAw32Rows + row) * kAw32Out + cg * 32 + l32] = acc[r];
    }
    __syncthreads();
    {
      const int row = tid >> 5, c4 = tid & 31;  // 4 columns 4 c4 .. 4 c4 + 3
      float v[4];
      float s2 = 0.f;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int col = 4 * c4 + e;
        float x = red[(0 * kAw32Rows + row) * kAw32Out + col];
        x += red[(1 * kAw32Rows + row) * kAw32Out + col];
        x += red[(2 * kAw32Rows + row) * kAw32Out + col];
        x += red[(3 * kAw32Rows + row) * kAw32Out + col];
        x = lrelu(x + bias[col]);
        v[e] = x;
        s2 += x * x;
      }
#pragma unroll
      for (int o = 1; o < 32; o <<= 1) s2 += __shfl_xor(s2, o, 64);
      const float nrm = sqrtf(s2);
      if (row < nrows) {
        *reinterpret_cast<float4*>(y + (r0 + row) * kAw32Out + 4 * c4) =
            make_float4(v[0] / nrm, v[1] / nrm, v[2] / nrm, v[3] / nrm);
        if (c4 == 0 && nrm_out) nrm_out[r0 + row] = nrm;
      }
    }
    __syncthreads();  // LDS is reused by the next tile
  }
}

// ---------------------------------------------------------------------------
// Round-3 form: the aggregation and the projection pipelined inside every wave,
// the projection on split-bf16 MFMA (v_mfma_f32_32x32x16_bf16, six products per
// 16-k step) with W pre-split into hi / mid / lo planes stored in MFMA fragment
// order, K split over the eight waves of a 512-thread workgroup (one per CU).
//
// A tile is <= 32 rows.  K is cut into 32-float chunks (one 128-B line of a
// row); wave w owns chunks w, w + 8, ... of the aggregate part (k in
// [d, d + hid)) and of the self part (k in [0, d)).  For a chunk, the wave
// streams the tile's slot rows of q in units of one slot (32 rows x 128 B:
// four loads per lane, each instruction 8 full rows = 8 whole lines -- the
// MFMA-fragment-shaped loads of the first form touched 32 lines per
// instruction and were bound by the load path), RD units in flight, and sums
// them in slot order t = 0, 1, ... (the fma chain of agg_kernel).  At the
// chunk's last slot the aggregate goes to agg (the W weight gradient reads it)
// and through a wave-private LDS image into the MFMA A layout; each of its two
// 16-k steps runs 4 column blocks x 6 products against B fragments that are
// one contiguous 1-KB load per (step, column block, plane).  LDS also holds the
// tile's slot offsets / weights and, at the end, the eight waves' partial
// [32][128] tiles (aliasing the A images), summed in wave order with bias,
// LeakyReLU and the row L2 norm (pinsage_model.py:208-211).
//
// Rows are dealt in contiguous ranges: block b of G owns [F b / G, F (b+1) / G)
// in near-equal tiles of <= 32 rows, so G ~ F / 24 blocks fill the CUs (C2
// layer 0: 238 blocks of 24 rows); padded MFMA rows issue no loads.
constexpr int kA3Rows = 32;
constexpr int kA3Waves = 8;
constexpr int kA3Out = 128;
constexpr int kA3TMax = 64;
constexpr int kA3TS = kA3TMax + 1;  // slot-table row stride (words)
constexpr int kA3RD = 3;            // slot units in flight per wave
constexpr int kA3AS = 36;           // A image row stride (floats): conflict-free b128 reads

typedef __attribute__((ext_vector_type(16))) float a3_f32x16;
typedef int a3_v4i __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float4 a3_ld(__amdgpu_buffer_rsrc_t r, unsigned voff, unsigned soff) {
  return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 0));
}
__device__ __forceinline__ bf16x8 a3_ldb(__amdgpu_buffer_rsrc_t r, unsigned voff, unsigned soff) {
  return __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 0));
}
__device__ __forceinline__ void a3_fma4(float w, const float4& a, float4& x) {
  x.x = fmaf(w, a.x, x.x);
  x.y = fmaf(w, a.y, x.y);
  x.z = fmaf(w, a.z, x.z);
  x.w = fmaf(w, a.w, x.w);
}
constexpr unsigned kA3Off = 0x80000000u;  // past the buffer: the load returns 0, no request

// W [128][K] fp32 -> three bf16 planes in MFMA fragment order:
// Wf[ks][cb][p][lane][8] = plane p of W[32 cb + lane % 32][16 ks + 8 (lane / 32) + j]
// (the split is bf16split.h's, so the products are those of the GEMM's split)
__global__ __launch_bounds__(256) void split_w_frag_kernel(const float* __restrict__ W, int K,
                                                           uint16_t* __restrict__ out) {
  const int i = blockIdx.x * 256 + threadIdx.x;  // (ks, cb, lane)
  const int nks = K >> 4;
  if (i >= nks * 4 * 64) return;
  const int lane = i & 63, cb = (i >> 6) & 3, ks = i >> 8;
  const float* src = W + (int64_t)(32 * cb + (lane & 31)) * K + 16 * ks + 8 * (lane >> 5);
  bf16x8 H, M, L;
  split3(*reinterpret_cast<const float4*>(src), *reinterpret_cast<const float4*>(src + 4), H, M, L);
  bf16x8* dst = reinterpret_cast<bf16x8*>(out) + ((int64_t)(ks * 4 + cb) * 3) * 64 + lane;
  dst[0] = H;
  dst[64] = M;
  dst[128] = L;
}

// q: [rows][hid] with rows * hid * 4 < 2^31 (launch_agg_w3 checks)
__global__ __launch_bounds__(kA3Waves * 64, 2) void agg_w3_kernel(
    const float* __restrict__ h, int64_t ldh, int d, const int32_t* __restrict__ self_src,
    const float* __restrict__ q, int hid, const int32_t* __restrict__ loc,
    const float* __restrict__ wloc, int T, const int* __restrict__ nS, int64_t n_static,
    const uint16_t* __restrict__ Wf, const float* __restrict__ bias, float* __restrict__ y,
    float* __restrict__ nrm_out, float* __restrict__ agg, int dbg) {
  __shared__ __attribute__((aligned(16))) float red[kA3Waves * kA3Rows * kA3Out];  // 128 KiB
  __shared__ unsigned sOff[kA3Rows * kA3TS];  // byte offsets of the tile's slot rows in q
  __shared__ float sW[kA3Rows * kA3TS];
  __shared__ int sSelf[kA3Rows];
  static_assert(kA3Waves * kA3Rows * kA3AS <= kA3Waves * kA3Rows * kA3Out, "A images alias red");
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // uniform: SGPR offsets
  // load layout: lane (rs, kq) holds rows rs + 8 j (j < 4), floats 4 kq .. 4 kq + 3 of a chunk
  const int rs = lane >> 3, kq = lane & 7;
  // MFMA layout: lane (row, half) supplies A[row][8 half .. 8 half + 7] of a 16-k step
  const int row = lane & 31, half = lane >> 5;
  float* Aimg = red + wave * kA3Rows * kA3AS;  // this wave's [32][36] A image
  const __amdgpu_buffer_rsrc_t qr = __builtin_amdgcn_make_buffer_rsrc((void*)q, 0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc((void*)Wf, 0, 0x7fffffff, 0x00020000);
  const int64_t F = nS ? (int64_t)*nS : n_static;
  const int64_t G = gridDim.x, b = blockIdx.x;
  const int64_t rb = F * b / G, re = F * (b + 1) / G;
  const int64_t len = re - rb;
  const int ntile = (int)((len + kA3Rows - 1) / kA3Rows);
  // this wave's chunks: aggregate part first (T slot units each), then the self part (one unit)
  const int nca = hid >> 5, ncs = d >> 5;
  const int na = nca > wave ? (nca - wave + kA3Waves - 1) / kA3Waves : 0;
  const int ns = ncs > wave ? (ncs - wave + kA3Waves - 1) / kA3Waves : 0;
  const int nunits = na * T + ns;

  for (int tile = 0; tile < ntile; ++tile) {
    const int64_t r0 = rb + len * tile / ntile;
    const int nrows = (int)(rb + len * (tile + 1) / ntile - r0);
    for (int i = tid; i < kA3Rows * T; i += kA3Waves * 64) {
      const int r = i / T, t = i - r * T;
      const bool ok = r < nrows;
      sOff[r * kA3TS + t] = ok && !(dbg & 1) ? (unsigned)loc[(r0 + r) * T + t] * (unsigned)hid * 4u : kA3Off;
      sW[r * kA3TS + t] = ok ? wloc[(r0 + r) * T + t] : 0.f;
    }
    if (tid < kA3Rows) sSelf[tid] = tid < nrows ? self_src[r0 + tid] : -1;
    __syncthreads();

    a3_f32x16 acc[4];
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[c][r] = 0.f;

    // unit s: aggregate chunk s / T, slot s % T; or self chunk s - na T
    float4 buf[kA3RD][4];
    auto issue = [&](int s, int u) __attribute__((always_inline)) {
      if (s < na * T) {
        const int ci = s / T, t = s - ci * T;
        const unsigned kb = 128u * (unsigned)(wave + kA3Waves * ci) + 16u * kq;  // bytes into the q row
#pragma unroll
        for (int j = 0; j < 4; ++j) buf[u][j] = a3_ld(qr, sOff[(rs + 8 * j) * kA3TS + t] + kb, 0);
      } else {
        const int k0 = 32 * (wave + kA3Waves * (s - na * T)) + 4 * kq;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int sr = sSelf[rs + 8 * j];
          buf[u][j] = sr >= 0 ? *reinterpret_cast<const float4*>(h + (int64_t)sr * ldh + k0)
                              : make_float4(0.f, 0.f, 0.f, 0.f);
        }
      }
    };
#pragma unroll
    for (int u = 0; u < kA3RD; ++u)
      if (u < nunits) issue(u, u);

    float4 x[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) x[j] = make_float4(0.f, 0.f, 0.f, 0.f);
    int ci = 0, t = 0;  // chunk (in this wave's list) and slot of the unit being consumed
    for (int s0 = 0; s0 < nunits; s0 += kA3RD) {
#pragma unroll
      for (int u = 0; u < kA3RD; ++u) {
        const int s = s0 + u;
        if (s >= nunits) break;
        const bool is_agg = ci < na;
        if (is_agg) {
#pragma unroll
          for (int j = 0; j < 4; ++j) a3_fma4(sW[(rs + 8 * j) * kA3TS + t], buf[u][j], x[j]);
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j) x[j] = buf[u][j];
        }
        if (s + kA3RD < nunits) issue(s + kA3RD, u);
        if (is_agg && ++t < T) continue;
        // ---- the chunk is complete: agg out, A image, two 16-k steps of MFMAs
        const int kc = is_agg ? d + 32 * (wave + kA3Waves * ci) : 32 * (wave + kA3Waves * (ci - na));
        if (is_agg) {
#pragma unroll
          for (int j = 0; j < 4; ++j)
            if (rs + 8 * j < nrows)
              *reinterpret_cast<float4*>(agg + (r0 + rs + 8 * j) * hid + (kc - d) + 4 * kq) = x[j];
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) *reinterpret_cast<float4*>(Aimg + (rs + 8 * j) * kA3AS + 4 * kq) = x[j];
#pragma unroll
        for (int j = 0; j < 4; ++j) x[j] = make_float4(0.f, 0.f, 0.f, 0.f);
        ++ci;
        t = 0;
#pragma unroll
        for (int st = 0; st < 2; ++st) {
          const int ks = (kc >> 4) + st;
          bf16x8 bw[3][4];
#pragma unroll
          for (int p = 0; p < 3; ++p)
#pragma unroll
            for (int c = 0; c < 4; ++c)
              bw[p][c] = a3_ldb(wr, (dbg & 2) ? kA3Off : (unsigned)lane * 16u, (unsigned)(((ks * 4 + c) * 3 + p) * 1024));
          if (dbg & 4) continue;
          const float* ar = Aimg + row * kA3AS + 16 * st + 8 * half;
          bf16x8 aH, aM, aL;
          split3(*reinterpret_cast<const float4*>(ar), *reinterpret_cast<const float4*>(ar + 4), aH, aM, aL);
#define PS_A3_ALL(X, P)                                                                         \
  _Pragma("unroll") for (int c = 0; c < 4; ++c) acc[c] =                                      \
      __builtin_amdgcn_mfma_f32_32x32x16_bf16(X, bw[P][c], acc[c], 0, 0, 0);
          PS_A3_ALL(aL, 0)
          PS_A3_ALL(aH, 2)
          PS_A3_ALL(aM, 1)
          PS_A3_ALL(aM, 0)
          PS_A3_ALL(aH, 1)
          PS_A3_ALL(aH, 0)
#undef PS_A3_ALL
        }
      }
    }
    __syncthreads();  // every wave is done with its A image (red aliases them)
    // partial tiles -> red[wave][row][col]; acc[c][r] is row (r & 3) + 8 (r >> 2) + 4 half, col 32 c + row
    {
      float* mine = red + wave * kA3Rows * kA3Out;
#pragma unroll
      for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int r = 0; r < 16; ++r) mine[((r & 3) + 8 * (r >> 2) + 4 * half) * kA3Out + 32 * c + row] = acc[c][r];
    }
    __syncthreads();
    {
      const int er = tid >> 4, c8 = (tid & 15) * 8;  // 16 threads per row, 8 columns each
      float v[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = 0.f;
#pragma unroll
      for (int w = 0; w < kA3Waves; ++w) {
        const float* src = red + (w * kA3Rows + er) * kA3Out + c8;
        const float4 a = *reinterpret_cast<const float4*>(src);
        const float4 bq = *reinterpret_cast<const float4*>(src + 4);
        v[0] += a.x;
        v[1] += a.y;
        v[2] += a.z;
        v[3] += a.w;
        v[4] += bq.x;
        v[5] += bq.y;
        v[6] += bq.z;
        v[7] += bq.w;
      }
      float s2 = 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        v[e] = lrelu(v[e] + bias[c8 + e]);
        s2 += v[e] * v[e];
      }
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) s2 += __shfl_xor(s2, o, 64);
      const float nrm = sqrtf(s2);
      if (er < nrows) {
        float* dst = y + (r0 + er) * kA3Out + c8;
        *reinterpret_cast<float4*>(dst) = make_float4(v[0] / nrm, v[1] / nrm, v[2] / nrm, v[3] / nrm);
        *reinterpret_cast<float4*>(dst + 4) = make_float4(v[4] / nrm, v[5] / nrm, v[6] / nrm, v[7] / nrm);
        if ((tid & 15) == 0 && nrm_out) nrm_out[r0 + er] = nrm;
      }
    }
    __syncthreads();  // red, the A images and the slot tables are reused by the next tile
  }
}

// ---------------------------------------------------------------------------
// Round-3 form, warp-specialised (the default): in a 512-thread workgroup per
// CU, waves 0-3 only GATHER and waves 4-7 only MULTIPLY, so the slot-row
// stream never pauses for the projection.
//
// Producer wave j streams, for round b, the slot rows of aggregate chunk
// c = 4 b + j (32 floats of q = one 128-B line per row; one unit = one slot =
// 32 rows x 128 B = four loads per lane, each instruction 8 whole lines) with
// RD units in flight (RD | T, so the stream runs on into its next chunk
// without a bubble), sums them in slot order t = 0, 1, ... (agg_kernel's fma
// chain), writes agg, splits the sum into bf16 hi / mid / lo and stores the
// three planes into its ring slot; the self rows of self chunk 4 b + j
// (k in [0, d)) go to a second slot (loaded a round ahead).  Consumer wave j
// owns output columns 32 j .. 32 j + 31 for the whole K: per round it runs the
// round's chunks' 16-k steps (v_mfma_f32_32x32x16_bf16, six products) with B
// fragments read as contiguous 1-KB lines of the fragment-ordered fp32 W
// (prefetched a round ahead, split in registers), so no cross-wave reduction
// is needed.  Rounds are double-buffered halves of an LDS ring (one barrier per
// round).  The epilogue sums nothing: bias, LeakyReLU and the row L2 norm over
// the four consumers' [32][32] blocks.
constexpr int kA4Rows = 32;
constexpr int kA4RowB = 80;    // ring plane row stride (bytes): conflict-free b64 writes / b128 reads
constexpr int kA4Plane = kA4Rows * kA4RowB;   // 2560 B
constexpr int kA4Img = 3 * kA4Plane;          // 7680 B: one chunk image (hi, mid, lo)
constexpr int kA4Half = 4 * 2 * kA4Img;       // 4 producers x (aggregate, self) images
constexpr int kA4BMax = 16;                   // 16-k steps per round per consumer (8 chunks x 2)

// fp32 W [128][K] -> MFMA fragment order Wr[ks][cb][qh][lane][4] =
// W[32 cb + lane % 32][16 ks + 8 (lane / 32) + 4 qh + e]: one 16-k step of one
// column block is two contiguous 1-KB loads
__global__ __launch_bounds__(256) void reorder_w_frag_kernel(const float* __restrict__ W, int K,
                                                             float* __restrict__ out) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= (K >> 4) * 512) return;
  const int lane = i & 63, qh = (i >> 6) & 1, cb = (i >> 7) & 3, ks = i >> 9;
  const float* src = W + (int64_t)(32 * cb + (lane & 31)) * K + 16 * ks + 8 * (lane >> 5) + 4 * qh;
  reinterpret_cast<float4*>(out)[i] = *reinterpret_cast<const float4*>(src);
}

constexpr int kA4TS = kA3TMax + 4;  // slot-table row stride (words): room for T padded to RD

template <int RD>
__global__ __launch_bounds__(512, 2) void agg_w4_kernel(
    const float* __restrict__ h, int64_t ldh, int d, const int32_t* __restrict__ self_src,
    const float* __restrict__ q, int hid, const int32_t* __restrict__ loc,
    const float* __restrict__ wloc, int T, const int* __restrict__ nS, int64_t n_static,
    const float* __restrict__ Wr, const float* __restrict__ bias, float* __restrict__ y,
    float* __restrict__ nrm_out, float* __restrict__ agg) {
  __shared__ __attribute__((aligned(16))) unsigned char ring[2 * kA4Half];  // 120 KiB
  __shared__ unsigned sOff[kA3Rows * kA4TS];
  __shared__ float sW[kA3Rows * kA4TS];
  __shared__ int sSelf[kA3Rows];
  float* red = reinterpret_cast<float*>(ring);  // [32][128] in the epilogue
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const bool producer = wave < 4;
  const int pj = wave & 3;
  const int rs = lane >> 3, kq = lane & 7;      // producer: rows rs + 8 j, floats 4 kq ..
  const int row = lane & 31, half = lane >> 5;  // consumer: MFMA lane
  const __amdgpu_buffer_rsrc_t qr = __builtin_amdgcn_make_buffer_rsrc((void*)q, 0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc((void*)Wr, 0, 0x7fffffff, 0x00020000);
  const int64_t F = nS ? (int64_t)*nS : n_static;
  const int64_t G = gridDim.x, b = blockIdx.x;
  const int64_t rb = F * b / G, re = F * (b + 1) / G;
  const int64_t len = re - rb;
  const int ntile = (int)((len + kA4Rows - 1) / kA4Rows);
  const int nca = hid >> 5, ncs = d >> 5;
  const int nr = max((nca + 3) >> 2, (ncs + 3) >> 2);  // rounds
  const int pa = nca > pj ? (nca - pj + 3) >> 2 : 0;   // this producer's aggregate chunks
  const int Tp = (T + RD - 1) / RD * RD;

  for (int tile = 0; tile < ntile; ++tile) {
    const int64_t r0 = rb + len * tile / ntile;
    const int nrows = (int)(rb + len * (tile + 1) / ntile - r0);
    // slots T .. Tp - 1 (T padded to a multiple of RD) read nothing with weight 0
    for (int i = tid; i < kA3Rows * Tp; i += 512) {
      const int r = i / Tp, t = i - r * Tp;
      const bool ok = r < nrows && t < T;
      sOff[r * kA4TS + t] = ok ? (unsigned)loc[(r0 + r) * T + t] * (unsigned)hid * 4u : kA3Off;
      sW[r * kA4TS + t] = ok ? wloc[(r0 + r) * T + t] : 0.f;
    }
    if (tid < kA3Rows) sSelf[tid] = tid < nrows ? self_src[r0 + tid] : -1;
    __syncthreads();

    if (producer) {
      float4 buf[RD][4], sb[4], x[4];
      // unit (ci, t): slot t of this producer's aggregate chunk ci into buf[t % RD]
      auto issue = [&](int ci, int t, int u) __attribute__((always_inline)) {
        const unsigned cbase = 128u * (unsigned)(4 * ci + pj);
#pragma unroll
        for (int j = 0; j < 4; ++j) buf[u][j] = a3_ld(qr, sOff[(rs + 8 * j) * kA4TS + t] + 16u * kq, cbase);
      };
      // self rows of self chunk 4 rr + pj into sb
      auto issue_self = [&](int rr) __attribute__((always_inline)) {
        const int c = 4 * rr + pj;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int sr = sSelf[rs + 8 * j];
          sb[j] = (c < ncs && sr >= 0) ? *reinterpret_cast<const float4*>(h + (int64_t)sr * ldh + 32 * c + 4 * kq)
                                       : make_float4(0.f, 0.f, 0.f, 0.f);
        }
      };
      // split 4 rows x 4 floats into the three planes of an image
      auto put = [&](unsigned char* img) __attribute__((always_inline)) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          unsigned H0, M0, L0, H1, M1, L1;
          split_pair(f32x2{x[j].x, x[j].y}, H0, M0, L0);
          split_pair(f32x2{x[j].z, x[j].w}, H1, M1, L1);
          unsigned char* r = img + (rs + 8 * j) * kA4RowB + 8 * kq;
          *reinterpret_cast<uint2*>(r) = make_uint2(H0, H1);
          *reinterpret_cast<uint2*>(r + kA4Plane) = make_uint2(M0, M1);
          *reinterpret_cast<uint2*>(r + 2 * kA4Plane) = make_uint2(L0, L1);
        }
      };
      if (pa > 0) {
#pragma unroll
        for (int u = 0; u < RD; ++u) issue(0, u, u);
      }
      issue_self(0);
      for (int bb = 0; bb <= nr; ++bb) {
        if (bb < nr) {
          unsigned char* slot = ring + (bb & 1) * kA4Half + pj * 2 * kA4Img;
          if (bb < pa) {
#pragma unroll
            for (int j = 0; j < 4; ++j) x[j] = make_float4(0.f, 0.f, 0.f, 0.f);
            for (int t0 = 0; t0 < Tp; t0 += RD) {
#pragma unroll
              for (int u = 0; u < RD; ++u) {
                const int t = t0 + u;
#pragma unroll
                for (int j = 0; j < 4; ++j) a3_fma4(sW[(rs + 8 * j) * kA4TS + t], buf[u][j], x[j]);
                __builtin_amdgcn_sched_barrier(0);
                if (t + RD < Tp) issue(bb, t + RD, u);
                else if (bb + 1 < pa) issue(bb + 1, t + RD - Tp, u);
                __builtin_amdgcn_sched_barrier(0);
              }
            }
            const int c = 4 * bb + pj;
#pragma unroll
            for (int j = 0; j < 4; ++j)
              if (rs + 8 * j < nrows)
                *reinterpret_cast<float4*>(agg + (r0 + rs + 8 * j) * hid + 32 * c + 4 * kq) = x[j];
            put(slot);
          }
          if (4 * bb + pj < ncs) {
#pragma unroll
            for (int j = 0; j < 4; ++j) x[j] = sb[j];
            issue_self(bb + 1);
            put(slot + kA4Img);
          }
        }
        __syncthreads();
      }
    } else {
      // consumer: column block pj for all of K
      a3_f32x16 acc;
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[r] = 0.f;
      // B fragments of 16-k steps, a ring of kA4BP steps ahead (static indices:
      // the 16 steps of a round are unrolled, 16 % kA4BP == 0, so the ring runs
      // on into the next round)
      constexpr int kA4BP = 4;
      float4 bq[kA4BP][2];
      // the 16-k steps of round rr, in order: aggregate chunks 4 rr .. 4 rr + 3 (two steps
      // each), then self chunks 4 rr .. 4 rr + 3; step i of the round -> global 16-k step
      auto ks_of = [&](int rr, int i) -> int {
        const int c = 4 * rr + (i >> 1) % 4;
        return i < 8 ? ((d >> 4) + 2 * c + (i & 1)) : (2 * c + (i & 1));
      };
      auto valid_step = [&](int rr, int i) -> bool {
        const int c = 4 * rr + (i >> 1) % 4;
        return rr < nr && (i < 8 ? c < nca : c < ncs);
      };
      auto load_b = [&](int rr, int i, int u) __attribute__((always_inline)) {
        if (valid_step(rr, i)) {
          const unsigned so = (unsigned)((ks_of(rr, i) * 4 + pj) * 2) * 1024u;
          bq[u][0] = a3_ld(wr, (unsigned)lane * 16u, so);
          bq[u][1] = a3_ld(wr, (unsigned)lane * 16u, so + 1024u);
        }
      };
#pragma unroll
      for (int i = 0; i < kA4BP; ++i) load_b(0, i, i);
      for (int bb = 0; bb <= nr; ++bb) {
        if (bb >= 1) {
          const int rr = bb - 1;
          const unsigned char* hbase = ring + (rr & 1) * kA4Half;
#pragma unroll
          for (int i = 0; i < kA4BMax; ++i) {
            __builtin_amdgcn_sched_barrier(0);
            if (valid_step(rr, i)) {
              const int src = (i >> 1) % 4, kind = i < 8 ? 0 : 1;
              const unsigned char* ap =
                  hbase + (src * 2 + kind) * kA4Img + row * kA4RowB + (16 * (i & 1) + 8 * half) * 2;
              const bf16x8 aH = *reinterpret_cast<const bf16x8*>(ap);
              const bf16x8 aM = *reinterpret_cast<const bf16x8*>(ap + kA4Plane);
              const bf16x8 aL = *reinterpret_cast<const bf16x8*>(ap + 2 * kA4Plane);
              bf16x8 bH, bM, bL;
              split3(bq[i % kA4BP][0], bq[i % kA4BP][1], bH, bM, bL);
              acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(aL, bH, acc, 0, 0, 0);
              acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(aH, bL, acc, 0, 0, 0);
              acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(aM, bM, acc, 0, 0, 0);
              acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(aM, bH, acc, 0, 0, 0);
              acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(aH, bM, acc, 0, 0, 0);
              acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(aH, bH, acc, 0, 0, 0);
            }
            // the step kA4BP ahead (into the next round for the last ones)
            if (i + kA4BP < kA4BMax) load_b(rr, i + kA4BP, i % kA4BP);
            else load_b(rr + 1, i + kA4BP - kA4BMax, i % kA4BP);
          }
        }
        __syncthreads();
      }
      // the [32][32] block of columns 32 pj .. -> red (the ring is idle now)
#pragma unroll
      for (int r = 0; r < 16; ++r) red[((r & 3) + 8 * (r >> 2) + 4 * half) * kA3Out + 32 * pj + row] = acc[r];
    }
    __syncthreads();
    {
      const int er = tid >> 4, c8 = (tid & 15) * 8;
      float v[8];
      float s2 = 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        v[e] = lrelu(red[er * kA3Out + c8 + e] + bias[c8 + e]);
        s2 += v[e] * v[e];
      }
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) s2 += __shfl_xor(s2, o, 64);
      const float nrm = sqrtf(s2);
      if (er < nrows) {
        float* dst = y + (r0 + er) * kA3Out + c8;
        *reinterpret_cast<float4*>(dst) = make_float4(v[0] / nrm, v[1] / nrm, v[2] / nrm, v[3] / nrm);
        *reinterpret_cast<float4*>(dst + 4) = make_float4(v[4] / nrm, v[5] / nrm, v[6] / nrm, v[7] / nrm);
        if ((tid & 15) == 0 && nrm_out) nrm_out[r0 + er] = nrm;
      }
    }
    __syncthreads();  // red (the ring) and the slot tables are reused by the next tile
  }
}

// ---------------------------------------------------------------------------
// Form 5: warp-specialised, the gather on LDS-DMA.  One 512-thread workgroup
// per CU owns a contiguous row range, in tiles of <= 32 rows.  Waves 0-3
// (producers) stream slot rows of q HBM -> LDS with global_load_lds_dwordx4
// (a unit = one 128-B chunk of 32 rows = four wave-instructions of 8 rows x
// 128 B, k5RD units in flight per producer ~ 64 KiB per CU) and retire them with
// counted s_waitcnt vmcnt: the compiler's waitcnt pass never sees these loads,
// so it cannot drain the queue at control-flow joins (the register-load forms
// 3 and 4 compiled to vmcnt(0) / vmcnt(1) waits between nearly every unit).
// Producer j sums chunk c = 4 r + j of the aggregate over the slots in order
// t = 0, 1, ... (agg_kernel's fma chain), writes it to agg (the W gradient
// reads it) and into the round's fp32 A image; the self rows' chunk 4 r + j
// (k in [0, d)) goes through the same ring.  Waves 4-7 (consumers) own 32
// output columns each over all of K: per round, 16 k-steps of
// v_mfma_f32_32x32x16_bf16 x 6 (A and W split into bf16 hi / mid / lo in
// registers; W fragments from L2 prefetched 8 steps ahead).  A images are
// double-buffered per round, one s_barrier per round.  Epilogue: bias,
// LeakyReLU and the row L2 norm (pinsage_model.py:208-211).
int agg_w3_supported(int64_t d, int64_t hid, int64_t out, int64_t T);

constexpr int k5Rows = 32;
constexpr int k5RD = 4;                 // units in flight per producer
constexpr int k5Unit = k5Rows * 128;    // bytes per unit
constexpr int k5AS = 36;                // A image row stride (floats): conflict-free b128 reads
constexpr int k5ImgF = k5Rows * k5AS;   // floats per A image
constexpr int k5TS = kA3TMax + 4;       // slot-table row stride (words)
constexpr int k5WP = 8;                 // W fragment prefetch distance (16-k steps)

__device__ __forceinline__ void k5_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
}

__global__ __launch_bounds__(512, 1) void agg_w5_kernel(
    const float* __restrict__ h, int64_t ldh, int d, const int32_t* __restrict__ self_src,
    const float* __restrict__ q, int hid, const int32_t* __restrict__ loc,
    const float* __restrict__ wloc, int T, const int* __restrict__ nS, int64_t n_static,
    const float* __restrict__ W, const float* __restrict__ bias, float* __restrict__ y,
    float* __restrict__ nrm_out, float* __restrict__ agg) {
  __shared__ __attribute__((aligned(16))) unsigned char ring[4 * k5RD * k5Unit];  // 64 KiB
  __shared__ __attribute__((aligned(16))) float aimg[2 * 8 * k5ImgF];            // 72 KiB
  __shared__ int sLoc[k5Rows * k5TS];
  __shared__ float sW[k5Rows * k5TS];
  __shared__ int sSelf[k5Rows];
  float* red = reinterpret_cast<float*>(ring);  // [32][128] in the epilogue
  const unsigned ring_lds = (unsigned)(size_t)((__attribute__((address_space(3))) unsigned char*)ring);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const bool producer = wave < 4;
  const int pj = wave & 3;
  const int rs = lane >> 3, kq = lane & 7;      // producer lane: rows rs + 8 j, floats 4 kq ..
  const int row = lane & 31, half = lane >> 5;  // consumer lane: MFMA row / k half
  const int K = d + hid;
  const int64_t F = nS ? (int64_t)*nS : n_static;
  const int64_t G = gridDim.x, b = blockIdx.x;
  const int64_t rb = F * b / G, re = F * (b + 1) / G;
  const int64_t len = re - rb;
  const int ntile = (int)((len + k5Rows - 1) / k5Rows);
  const int nca = hid >> 5, ncs = d >> 5;
  const int nr = max((nca + 3) >> 2, (ncs + 3) >> 2);  // rounds

  for (int tile = 0; tile < ntile; ++tile) {
    const int64_t r0 = rb + len * tile / ntile;
    const int nrows = (int)(rb + len * (tile + 1) / ntile - r0);
    // padded rows read the tile's first row (a cache hit) with weight 0
    for (int i = tid; i < k5Rows * T; i += 512) {
      const int r = i / T, t = i - r * T;
      const int rr = r < nrows ? r : 0;
      sLoc[r * k5TS + t] = loc[(r0 + rr) * T + t];
      sW[r * k5TS + t] = r < nrows ? wloc[(r0 + rr) * T + t] : 0.f;
    }
    if (tid < k5Rows) sSelf[tid] = self_src[r0 + (tid < nrows ? tid : 0)];
    __syncthreads();

    if (producer) {
      // this producer's units, round by round: T aggregate slots of chunk
      // 4 r + pj (if < nca), then the self chunk 4 r + pj (if < ncs)
      auto n_in = [&](int r) { return (4 * r + pj < nca ? T : 0) + (4 * r + pj < ncs ? 1 : 0); };
      int total = 0;
      for (int r = 0; r < nr; ++r) total += n_in(r);
      int ir = 0, ik = 0;  // issue cursor (round, position in round)
      auto issue_next = [&](int slot) __attribute__((always_inline)) {
        while (ik >= n_in(ir)) {
          ++ir;
          ik = 0;
        }
        const int c = 4 * ir + pj;
        const bool is_agg = 4 * ir + pj < nca && ik < T;
        const unsigned dst = ring_lds + (unsigned)(pj * k5RD + slot) * k5Unit;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int rw = rs + 8 * j;
          const float* src = is_agg ? q + (int64_t)sLoc[rw * k5TS + ik] * hid + 32 * c + 4 * kq
                                    : h + (int64_t)sSelf[rw] * ldh + 32 * c + 4 * kq;
          glds16(src, dst + j * 1024);
        }
        ++ik;
      };
      for (int u = 0; u < k5RD && u < total; ++u) issue_next(u);
      float4 x[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) x[j] = make_float4(0.f, 0.f, 0.f, 0.f);
      int s = 0;
      for (int r = 0; r < nr; ++r) {
        float* img = aimg + ((r & 1) * 8) * k5ImgF;
        const int na = 4 * r + pj < nca ? T : 0, nin = n_in(r);
        for (int k = 0; k < nin; ++k, ++s) {
          wait_stage<4, k5RD - 1>(min(k5RD - 1, total - 1 - s));
          const unsigned char* src = ring + (pj * k5RD + s % k5RD) * k5Unit + lane * 16;
          float4 v[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) v[j] = *reinterpret_cast<const float4*>(src + j * 1024);
          if (k < na) {
#pragma unroll
            for (int j = 0; j < 4; ++j) a3_fma4(sW[(rs + 8 * j) * k5TS + k], v[j], x[j]);
          }
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the slot is read: refill it
          if (s + k5RD < total) issue_next(s % k5RD);
          if (k == na - 1) {  // aggregate chunk complete: agg out, A image
            const int c = 4 * r + pj;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              if (rs + 8 * j < nrows)
                *reinterpret_cast<float4*>(agg + (r0 + rs + 8 * j) * hid + 32 * c + 4 * kq) = x[j];
              *reinterpret_cast<float4*>(img + pj * k5ImgF + (rs + 8 * j) * k5AS + 4 * kq) = x[j];
              x[j] = make_float4(0.f, 0.f, 0.f, 0.f);
            }
          } else if (k >= na) {  // self chunk
#pragma unroll
            for (int j = 0; j < 4; ++j)
              *reinterpret_cast<float4*>(img + (4 + pj) * k5ImgF + (rs + 8 * j) * k5AS + 4 * kq) = v[j];
          }
        }
        k5_barrier();  // round r's images are complete
      }
    } else {
      // consumer pj: output columns 32 pj .. 32 pj + 31 over all of K.  Step i of
      // round r: aggregate chunk 4 r + (i >> 1) % 4 (i < 8) or self chunk (i >= 8),
      // 16-k half i & 1
      a3_f32x16 acc;
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[e] = 0.f;
      auto kk_of = [&](int r, int i) -> int {  // global 16-k step, clamped into range
        const int c = 4 * r + ((i >> 1) & 3);
        const int kk = i < 8 ? (d >> 4) + 2 * c + (i & 1) : 2 * c + (i & 1);
        return min(kk, (K >> 4) - 1);
      };
      const float* wrow = W + (int64_t)(32 * pj + row) * K + 8 * half;
      float4 bq[k5WP][2];
#pragma unroll
      for (int i = 0; i < k5WP; ++i) {
        const float* p = wrow + 16 * kk_of(0, i);
        bq[i][0] = *reinterpret_cast<const float4*>(p);
        bq[i][1] = *reinterpret_cast<const float4*>(p + 4);
      }
      for (int r = 0; r < nr; ++r) {
        k5_barrier();  // round r's images are complete
        const float* img = aimg + ((r & 1) * 8) * k5ImgF;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int c = 4 * r + ((i >> 1) & 3);
          const bool valid = i < 8 ? c < nca : c < ncs;
          const float4 b0 = bq[i % k5WP][0], b1 = bq[i % k5WP][1];
          {  // refill the slot with the step k5WP ahead (into the next round for the last ones)
            const int rn = i + k5WP < 16 ? r : r + 1, in = (i + k5WP) & 15;
            const float* p = wrow + 16 * kk_of(rn < nr ? rn : r, in);
            bq[i % k5WP][0] = *reinterpret_cast<const float4*>(p);
            bq[i % k5WP][1] = *reinterpret_cast<const float4*>(p + 4);
          }
          if (valid) {
            const float* ar = img + (i < 8 ? ((i >> 1) & 3) : 4 + ((i >> 1) & 3)) * k5ImgF + row * k5AS +
                              16 * (i & 1) + 8 * half;
            bf16x8 aH, aM, aL, bH, bM, bL;
            split3(*reinterpret_cast<const float4*>(ar), *reinterpret_cast<const float4*>(ar + 4), aH, aM, aL);
            split3(b0, b1, bH, bM, bL);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(aL, bH, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(aH, bL, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(aM, bM, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(aM, bH, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(aH, bM, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(aH, bH, acc, 0, 0, 0);
          }
        }
      }
      // every producer passed its last round's barrier: the ring is idle
#pragma unroll
      for (int e = 0; e < 16; ++e) red[((e & 3) + 8 * (e >> 2) + 4 * half) * kA3Out + 32 * pj + row] = acc[e];
    }
    __syncthreads();
    {
      const int er = tid >> 4, c8 = (tid & 15) * 8;
      float v[8];
      float s2 = 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        v[e] = lrelu(red[er * kA3Out + c8 + e] + bias[c8 + e]);
        s2 += v[e] * v[e];
      }
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) s2 += __shfl_xor(s2, o, 64);
      const float nrm = sqrtf(s2);
      if (er < nrows) {
        float* dst = y + (r0 + er) * kA3Out + c8;
        *reinterpret_cast<float4*>(dst) = make_float4(v[0] / nrm, v[1] / nrm, v[2] / nrm, v[3] / nrm);
        *reinterpret_cast<float4*>(dst + 4) = make_float4(v[4] / nrm, v[5] / nrm, v[6] / nrm, v[7] / nrm);
        if ((tid & 15) == 0 && nrm_out) nrm_out[r0 + er] = nrm;
      }
    }
    __syncthreads();  // red (the ring) and the slot tables are reused by the next tile
  }
}

int launch_agg_w5(const float* h, int64_t ldh, int d, const int32_t* self_src, const float* q, int hid,
                  const int32_t* loc, const float* wloc, int T, const int* nS, int64_t n_static, int64_t S_est,
                  const float* W, const float* bias, float* y, float* nrm, float* agg, hipStream_t st) {
  PS_REQUIRE(agg_w3_supported(d, hid, kA3Out, T), kErrArg, "agg_w5: unsupported shape");
  PS_REQUIRE(ldh % 4 == 0 && (uintptr_t)h % 16 == 0 && (uintptr_t)q % 16 == 0 && (uintptr_t)agg % 16 == 0 &&
                 (uintptr_t)y % 16 == 0 && (uintptr_t)W % 16 == 0,
             kErrArg, "agg_w5: 16-B aligned rows required");
  if (S_est <= 0) return kOk;
  static int rows_per_block = -1;
  if (rows_per_block < 0) {
    const char* e = getenv("PINSAGE_AGGW_ROWS");
    rows_per_block = e ? std::max(1, atoi(e)) : 16;
  }
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
    cus = 256;
  const int64_t g = std::min<int64_t>(cus, std::max<int64_t>(1, (S_est + rows_per_block - 1) / rows_per_block));
  hipLaunchKernelGGL(agg_w5_kernel, dim3((unsigned)g), dim3(512), 0, st, h, ldh, d, self_src, q, hid, loc, wloc,
                     T, nS, n_static, W, bias, y, nrm, agg);
  PS_CHECK_LAUNCH();
  return kOk;
}

int launch_reorder_w_frag(const float* W, int64_t K, float* Wr, hipStream_t st) {
  PS_REQUIRE(K % 16 == 0 && K > 0 && (uintptr_t)W % 16 == 0 && (uintptr_t)Wr % 16 == 0, kErrArg,
             "reorder_w_frag: K % 16 == 0, 16-B aligned");
  const int n = (int)(K / 16) * 512;
  hipLaunchKernelGGL(reorder_w_frag_kernel, dim3((n + 255) / 256), dim3(256), 0, st, W, (int)K, Wr);
  PS_CHECK_LAUNCH();
  return kOk;
}

int agg_w3_supported(int64_t d, int64_t hid, int64_t out, int64_t T) {
  return out == kA3Out && d % 32 == 0 && hid % 32 == 0 && d > 0 && hid > 0 && T >= 1 && T <= kA3TMax;
}

// the fragment-ordered planes of W [128][K] (3 * 128 * K uint16 at Wf)
int launch_split_w_frag(const float* W, int64_t K, uint16_t* Wf, hipStream_t st) {
  PS_REQUIRE(K % 16 == 0 && K > 0 && (uintptr_t)W % 16 == 0 && (uintptr_t)Wf % 16 == 0, kErrArg,
             "split_w_frag: K % 16 == 0, 16-B aligned");
  const int n = (int)(K / 16) * 4 * 64;
  hipLaunchKernelGGL(split_w_frag_kernel, dim3((n + 255) / 256), dim3(256), 0, st, W, (int)K, Wf);
  PS_CHECK_LAUNCH();
  return kOk;
}

int launch_agg_w4(const float* h, int64_t ldh, int d, const int32_t* self_src, const float* q, int hid,
                  int64_t q_rows_cap, const int32_t* loc, const float* wloc, int T, const int* nS,
                  int64_t n_static, int64_t S_est, const float* Wr, const float* bias, float* y, float* nrm,
                  float* agg, hipStream_t st) {
  PS_REQUIRE(agg_w3_supported(d, hid, kA3Out, T), kErrArg, "agg_w4: unsupported shape");
  PS_REQUIRE(q_rows_cap * hid * 4 < (1LL << 31) && (int64_t)kA3Out * (d + hid) * 4 < (1LL << 31), kErrArg,
             "agg_w4: q or W too large for 32-bit buffer offsets");
  PS_REQUIRE(ldh % 4 == 0 && (uintptr_t)h % 16 == 0 && (uintptr_t)q % 16 == 0 && (uintptr_t)agg % 16 == 0 &&
                 (uintptr_t)y % 16 == 0 && (uintptr_t)Wr % 16 == 0,
             kErrArg, "agg_w4: 16-B aligned rows required");
  if (S_est <= 0) return kOk;
  const char* e = getenv("PINSAGE_AGGW_ROWS");
  const int rows = e ? std::max(1, atoi(e)) : 24;
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
    cus = 256;
  const int64_t g = std::min<int64_t>(cus, std::max<int64_t>(1, (S_est + rows - 1) / rows));
  const dim3 gr((unsigned)g), bl(512);
#define PS_A4(R) \
  hipLaunchKernelGGL(agg_w4_kernel<R>, gr, bl, 0, st, h, ldh, d, self_src, q, hid, loc, wloc, T, nS, n_static, Wr, \
                     bias, y, nrm, agg)
  PS_A4(4);
#undef PS_A4
  PS_CHECK_LAUNCH();
  return kOk;
}

static int g_aggw3_rows = -1;  // target rows per workgroup (PINSAGE_AGGW_ROWS)

int launch_agg_w3(const float* h, int64_t ldh, int d, const int32_t* self_src, const float* q, int hid,
                  int64_t q_rows_cap, const int32_t* loc, const float* wloc, int T, const int* nS,
                  int64_t n_static, int64_t S_est, const uint16_t* Wf, const float* bias, float* y, float* nrm,
                  float* agg, hipStream_t st) {
  PS_REQUIRE(agg_w3_supported(d, hid, kA3Out, T), kErrArg, "agg_w3: unsupported shape");
  PS_REQUIRE(q_rows_cap * hid * 4 < (1LL << 31) && (int64_t)kA3Out * (d + hid) * 2 * 3 < (1LL << 31), kErrArg,
             "agg_w3: q or W planes too large for 32-bit buffer offsets");
  PS_REQUIRE(ldh % 4 == 0 && (uintptr_t)h % 16 == 0 && (uintptr_t)q % 16 == 0 && (uintptr_t)agg % 16 == 0 &&
                 (uintptr_t)y % 16 == 0 && (uintptr_t)Wf % 16 == 0,
             kErrArg, "agg_w3: 16-B aligned rows required");
  if (S_est <= 0) return kOk;
  if (g_aggw3_rows < 0) {
    const char* e = getenv("PINSAGE_AGGW_ROWS");
    g_aggw3_rows = e ? std::max(1, atoi(e)) : 24;
  }
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
    cus = 256;
  const int64_t g = std::min<int64_t>(cus, std::max<int64_t>(1, (S_est + g_aggw3_rows - 1) / g_aggw3_rows));
  static const int dbg = getenv("PINSAGE_AGGW_DBG") ? atoi(getenv("PINSAGE_AGGW_DBG")) : 0;  // A/B only
  hipLaunchKernelGGL(agg_w3_kernel, dim3((unsigned)g), dim3(kA3Waves * 64), 0, st, h, ldh, d, self_src, q,
                     hid, loc, wloc, T, nS, n_static, Wf, bias, y, nrm, agg, dbg);
  PS_CHECK_LAUNCH();
  return kOk;
}

static int agg_w32_supported(int64_t d, int64_t hid, int64_t T) {
  const int64_t K = d + hid;
  const int64_t lds = (int64_t)kAw32Rows * (K + 4) * 4 + 2 * kAw32Rows * kAw32TMax * 4 + kAw32Rows * 4;
  return K % 128 == 0 && K + 4 >= 4 * kAw32Out && T <= kAw32TMax && lds <= 160 * 1024;
}

int agg_w_supported(int64_t d, int64_t hid, int64_t out, int64_t T) {
  const int64_t K = d + hid;
  const int64_t lds = (int64_t)kAwRows * (K + 4) * 4 + 2 * kAwRows * kAwTMax * 4 + kAwRows * 4;
  // the A tile's LDS is reused for the [16][128] output tile (K + 4 >= 128);
  // two workgroups per CU; the aggregation pass covers hid in passes of 512
  return out == kAwOut && K % 64 == 0 && K + 4 >= kAwOut && hid % 4 == 0 && d % 4 == 0 &&
         T >= 1 && T <= kAwTMax && 2 * lds <= 160 * 1024;
}

// S_max: the expected row count (the frontier size hint; the kernels read the
// actual count from nS and deal it over their blocks)
int launch_agg_w(const float* h, int64_t ldh, int d, const int32_t* self_src, const float* q, int hid,
                 const int32_t* loc, const float* wloc, int T, const int* nS, int64_t S_max,
                 const float* W, const float* bias, float* y, float* nrm, float* agg, hipStream_t st) {
  PS_REQUIRE(agg_w_supported(d, hid, kAwOut, T), kErrArg, "agg_w: unsupported shape");
  const int K = d + hid;
  const int lds = kAwRows * (K + 4) * 4 + 2 * kAwRows * kAwTMax * 4 + kAwRows * 4;
  static int prepared = 0;
  if (prepared < lds) {
    PS_CHECK_HIP(hipFuncSetAttribute((const void*)agg_w_kernel,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    prepared = 160 * 1024;
  }
  if (S_max <= 0) return kOk;
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
    cus = 256;
  // ~12 rows per block (a 16-row tile with headroom), two blocks per CU
  const int grid = (int)std::max<int64_t>(1, std::min<int64_t>(2 * (int64_t)cus, (S_max + 11) / 12));
  // The 32-row form (one block per CU, W read once per 32 rows) when the rows
  // fill ~16 per CU; below that the 16-row form (two blocks per CU, one's gather
  // beside the other's products) hides more latency.  Measured (bench.py):
  // C2 layer 0 (5.7k rows, K 1024) 36.5 vs 55.3 us, C4 layer 0 (8.6k, K 640)
  // 50.2 vs 73.4 us; the layers 1 (1.5-2k rows, K 640) 21.5-21.8 vs 24.7-25.3 us.
  // PINSAGE_AGGW32_MIN_ROWS overrides the switch point (A/B).
  const int64_t min_rows32 =
      getenv("PINSAGE_AGGW32_MIN_ROWS") ? atoll(getenv("PINSAGE_AGGW32_MIN_ROWS")) : 16 * (int64_t)cus;
  if (S_max >= min_rows32 && agg_w32_supported(d, hid, T)) {
    const int lds32 = kAw32Rows * (K + 4) * 4 + 2 * kAw32Rows * kAw32TMax * 4 + kAw32Rows * 4;
    static bool prepared32 = false;
    if (!prepared32) {
      PS_CHECK_HIP(hipFuncSetAttribute((const void*)agg_w32_kernel,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
      prepared32 = true;
    }
    // ~24 rows per block (a 32-row tile with headroom) over every CU
    const int64_t g32 = std::max<int64_t>(1, std::min<int64_t>(cus, (S_max + 23) / 24));
    hipLaunchKernelGGL(agg_w32_kernel, dim3((int)g32), dim3(kAw32Threads), lds32,
                       st, h, ldh, d, self_src, q, hid, loc, wloc, T, nS, W, bias, y, nrm, agg);
  } else {
    hipLaunchKernelGGL(agg_w_kernel, dim3(grid), dim3(kAwThreads), lds, st, h, ldh, d, self_src, q, hid,
                       loc, wloc, T, nS, W, bias, y, nrm, agg);
  }
  PS_CHECK_LAUNCH();
  return kOk;
}

}  // namespace ps
