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

#include "aggw.h"
#include "bf16split.h"
#include "common.h"

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

// HEAD: the model head's forward may be fused (hd.G1w set); without it the
// kernel fits 128 VGPRs, so two 512-thread blocks share a CU (agg_w_nh_kernel)
template <bool HEAD>
__device__ __forceinline__ void agg_w_body(
    const float* __restrict__ h, int64_t ldh, int d, const int32_t* __restrict__ self_src,
    const float* __restrict__ q, int hid, const int32_t* __restrict__ loc,
    const float* __restrict__ wloc, int T, const int* __restrict__ nS, int64_t n_static,
    const float* __restrict__ W, const float* __restrict__ bias, float* __restrict__ y,
    float* __restrict__ nrm_out, float* __restrict__ agg, AggHead hd) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int K = d + hid, lda = aw_lda(K);
  float* sA = lds;                                          // [16][lda]
  int* sLoc = reinterpret_cast<int*>(lds + kAwRows * lda);  // [16][T]
  float* sW = reinterpret_cast<float*>(sLoc + kAwRows * kAwTMax);  // [16][T]
  int* sSelf = reinterpret_cast<int*>(sW + kAwRows * kAwTMax);     // [16]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // rows dealt in contiguous ranges: block b of G owns [F b / G, F (b+1) / G)
  // in near-equal tiles of <= 16 rows (two blocks per CU: G ~ F / 12 fills them)
  const int64_t F = nS ? (int64_t)*nS : n_static;
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
    // the head's weight rows (column 16 wave + l16, k = 32 g .. 32 g + 31 of G1
    // and G2), fetched under the epilogue
    float4 hw1[8], hw2[8];
    float hb1 = 0.f;
    if (HEAD && hd.G1w) {
      const int hc = wave * 16 + l16;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        hw1[i] = *reinterpret_cast<const float4*>(hd.G1w + hc * kAwOut + 32 * g + 4 * i);
        hw2[i] = *reinterpret_cast<const float4*>(hd.G2w + hc * kAwOut + 32 * g + 4 * i);
      }
      hb1 = hd.G1b[hc];
    }
    __syncthreads();  // every wave is done reading the A tile
    // ---- the [16][128] output tile -> LDS, then bias, lrelu, row L2 norm
    float* red = sA;
    float* sY = sA + kAwRows * kAwOut;         // [16][kAwHd] the head's y, then H1 rows
    constexpr int kAwHd = kAwOut + 4;
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
      const float4 yv = row < nrows ? make_float4(v[0] / nrm, v[1] / nrm, v[2] / nrm, v[3] / nrm)
                                    : make_float4(0.f, 0.f, 0.f, 0.f);
      if (HEAD && hd.G1w) *reinterpret_cast<float4*>(sY + row * kAwHd + 4 * c4) = yv;
      if (row < nrows) {
        *reinterpret_cast<float4*>(y + (r0 + row) * kAwOut + 4 * c4) = yv;
        if (c4 == 0 && nrm_out) nrm_out[r0 + row] = nrm;
      }
    }
    __syncthreads();  // LDS is reused by the next tile (or the head below)
    if (HEAD && hd.G1w) {
      // ---- head: wave w, columns 16 w .. 16 w + 15 of H1 and Z; lane l
      // supplies row l16 and k = 32 g + s at step s (v_mfma_f32_16x16x4_f32)
      const int hc = wave * 16 + l16;
      f32x4 a1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float4 av = *reinterpret_cast<const float4*>(sY + l16 * kAwHd + 32 * g + 4 * i);
        a1 = __builtin_amdgcn_mfma_f32_16x16x4f32(av.x, hw1[i].x, a1, 0, 0, 0);
        a1 = __builtin_amdgcn_mfma_f32_16x16x4f32(av.y, hw1[i].y, a1, 0, 0, 0);
        a1 = __builtin_amdgcn_mfma_f32_16x16x4f32(av.z, hw1[i].z, a1, 0, 0, 0);
        a1 = __builtin_amdgcn_mfma_f32_16x16x4f32(av.w, hw1[i].w, a1, 0, 0, 0);
      }
      __syncthreads();  // every wave is done reading y
      float hv[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        hv[r] = lrelu(a1[r] + hb1);
        sY[(4 * g + r) * kAwHd + hc] = hv[r];
      }
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (4 * g + r < nrows) hd.H1[(r0 + 4 * g + r) * kAwOut + hc] = hv[r];
      __syncthreads();
      f32x4 a2 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float4 av = *reinterpret_cast<const float4*>(sY + l16 * kAwHd + 32 * g + 4 * i);
        a2 = __builtin_amdgcn_mfma_f32_16x16x4f32(av.x, hw2[i].x, a2, 0, 0, 0);
        a2 = __builtin_amdgcn_mfma_f32_16x16x4f32(av.y, hw2[i].y, a2, 0, 0, 0);
        a2 = __builtin_amdgcn_mfma_f32_16x16x4f32(av.z, hw2[i].z, a2, 0, 0, 0);
        a2 = __builtin_amdgcn_mfma_f32_16x16x4f32(av.w, hw2[i].w, a2, 0, 0, 0);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (4 * g + r < nrows) hd.Z[(r0 + 4 * g + r) * kAwOut + hc] = a2[r];
      __syncthreads();  // every wave is done reading H1 from LDS
    }
  }
}

#define PS_AW_ARGS                                                                                        \
  const float *__restrict__ h, int64_t ldh, int d, const int32_t *__restrict__ self_src,                  \
      const float *__restrict__ q, int hid, const int32_t *__restrict__ loc, const float *__restrict__ wloc, \
      int T, const int *__restrict__ nS, int64_t n_static, const float *__restrict__ W,                    \
      const float *__restrict__ bias, float *__restrict__ y, float *__restrict__ nrm_out,                  \
      float *__restrict__ agg, AggHead hd
__global__ __launch_bounds__(kAwThreads, 2) void agg_w_kernel(PS_AW_ARGS) {
  agg_w_body<true>(h, ldh, d, self_src, q, hid, loc, wloc, T, nS, n_static, W, bias, y, nrm_out, agg, hd);
}
// no head: held to 128 VGPRs, so two blocks share a CU (one's gather beside
// the other's products: PINSAGE_AGGW_NH, the 16-row form's launches without
// the head)
__global__ __launch_bounds__(kAwThreads) __attribute__((amdgpu_waves_per_eu(4, 4))) void agg_w_nh_kernel(
    PS_AW_ARGS) {
  agg_w_body<false>(h, ldh, d, self_src, q, hid, loc, wloc, T, nS, n_static, W, bias, y, nrm_out, agg, hd);
}
#undef PS_AW_ARGS

typedef float aw_f32x16 __attribute__((ext_vector_type(16)));

// The 32-row form: one 1024-thread workgroup per CU, W read once per 32 rows
// (wins at K = d + hid = 1024: C2/C3 layer 0; the 16-row kernel above wins at
// K = 640, C2 layer 1).
constexpr int kAw32Rows = 32;     // rows per workgroup
constexpr int kAw32Out = 128;     // out_dim (4 column groups of 32)
constexpr int kAw32Threads = 1024;
constexpr int kAw32TMax = 64;     // fanout held in LDS per row
constexpr int kAw32Lq = kAw32Out + 4;  // LDS row of the y tile the next-layer Q projection reads
__device__ __forceinline__ int aw32_lda(int K) { return K + 4; }

// ---------------------------------------------------------------- 32-row form, A split once per two column groups
// The gather: every thread's loads in flight at once (thread: row tid / 32,
// float4 columns (tid % 32) + 32 j, four slots' rows per round; agg bitwise
// agg_kernel's).  The projection: wave w owns k eighth w / 2 and column groups
// 2 (w % 2), +1, so each A fragment read from LDS is split into bf16 hi / mid /
// lo once for 12 MFMAs (round 4's form: once per 6, every fragment split by
// four waves, W split in every workgroup: C2 layer 0 36.3 -> 32.5 us), and W
// comes pre-split from its fragment-order planes (split_wplanes_kernel, one
// coalesced 1 KiB load per plane and fragment; the next 16-k step's fragments
// load while the current step's products run).  Without planes (PL false) W is
// split in registers.  The eight k-eighth partial tiles meet in LDS in order.
constexpr int kWpOut = 128;   // out_dim
constexpr int kWpCG = 4;      // 32-column groups of the output
#ifndef PS_AGGWS_PROBE  // timing-only builds (results wrong by construction): bit 0 no products, bit 1 no aggregate gather
#define PS_AGGWS_PROBE 0
#endif

// W [128][K] (row stride ldw) -> fragment-order planes: chunk c = (s, cg, lane)
// of 8 bf16 at planes[((c >> 6) * 3 + p) * 512 + (c & 63) * 8] holds plane p of
// W[32 cg + lane % 32][16 s + 8 (lane / 32) + i], i < 8 -- the B fragment lane
// `lane` supplies to v_mfma_f32_32x32x16_bf16 in 16-k step s for column group
// cg.  The split is split3's (bf16split.h), so the products equal the
// in-register split's.
__global__ __launch_bounds__(256) void split_wplanes_kernel(const float* __restrict__ W, int64_t ldw, int K,
                                                            uint16_t* __restrict__ planes) {
  const int64_t n = (int64_t)K * kWpOut / 8;  // chunks
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= n) return;
  const int lane = (int)(c & 63);
  const int64_t rest = c >> 6;
  const int cg = (int)(rest % kWpCG), s = (int)(rest / kWpCG);
  const float* src = W + (int64_t)(32 * cg + (lane & 31)) * ldw + 16 * s + 8 * (lane >> 5);
  bf16x8 H, M, L;
  split3(*reinterpret_cast<const float4*>(src), *reinterpret_cast<const float4*>(src + 4), H, M, L);
  uint16_t* o = planes + (rest * 3) * 512 + lane * 8;
  *reinterpret_cast<bf16x8*>(o) = H;
  *reinterpret_cast<bf16x8*>(o + 512) = M;
  *reinterpret_cast<bf16x8*>(o + 1024) = L;
}

// LDS: max(A tile [32][K + 4], the partial tiles [8][32][128]), then the slot lists
static int64_t ws_lds_bytes(int64_t K) {
  const int64_t tile = std::max<int64_t>((int64_t)kAw32Rows * (K + 4), (int64_t)8 * kAw32Rows * kWpOut);
  return (tile + 2 * kAw32Rows * kAw32TMax + kAw32Rows) * 4;
}

template <bool PL>
__global__ __launch_bounds__(kAw32Threads) void agg_w32s_kernel(
    const float* __restrict__ h, int64_t ldh, int d, const int32_t* __restrict__ self_src,
    const float* __restrict__ q, int hid, const int32_t* __restrict__ loc,
    const float* __restrict__ wloc, int T, const int* __restrict__ nS, int64_t n_static,
    const float* __restrict__ W, const uint16_t* __restrict__ planes, const float* __restrict__ bias,
    float* __restrict__ y, float* __restrict__ nrm_out, float* __restrict__ agg, AggNextQ nx) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int K = d + hid, lda = aw32_lda(K);
  const int64_t tile_f = std::max<int64_t>((int64_t)kAw32Rows * lda, (int64_t)8 * kAw32Rows * kWpOut);
  float* sA = lds;                                            // [32][lda]; the partial tiles after the products
  int* sLoc = reinterpret_cast<int*>(lds + tile_f);           // [32][T]
  float* sW = reinterpret_cast<float*>(sLoc + kAw32Rows * kAw32TMax);  // [32][T]
  int* sSelf = reinterpret_cast<int*>(sW + kAw32Rows * kAw32TMax);     // [32]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t F = nS ? (int64_t)*nS : n_static;
  const int64_t G = gridDim.x, b = blockIdx.x;
  const int64_t rb = F * b / G, len = F * (b + 1) / G - rb;
  const int ntile = (int)((len + kAw32Rows - 1) / kAw32Rows);
  typedef float f32x16 __attribute__((ext_vector_type(16)));
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
      for (int j0 = 0; j0 < nj && !(PS_AGGWS_PROBE & 2); j0 += 4) {
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
    // ---- projection: wave (kq8 = w / 2, column groups 2 cp, 2 cp + 1)
    const int kq8 = wave >> 1, cp = wave & 1;
    const int l32 = lane & 31, hh = lane >> 5;
    const int ksp = K >> 3, nst = ksp >> 4;
    const float* arow = sA + l32 * lda + kq8 * ksp + 8 * hh;
    f32x16 acc[2];
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[c][r] = 0.f;
    if constexpr (PL) {
      const int sg0 = (kq8 * ksp) >> 4;
      auto ldb = [&](int s, bf16x8 (&bb)[2][3]) __attribute__((always_inline)) {
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          const bf16x8* p =
              reinterpret_cast<const bf16x8*>(planes + ((int64_t)((sg0 + s) * kWpCG + 2 * cp + c) * 3 * 64 + lane) * 8);
          bb[c][0] = p[0];
          bb[c][1] = p[64];
          bb[c][2] = p[128];
        }
      };
      bf16x8 bc[2][3], bn[2][3];
      ldb(0, bc);
      for (int s = 0; s < nst && !(PS_AGGWS_PROBE & 1); ++s) {
        ldb(s + 1 < nst ? s + 1 : s, bn);  // (the last step reloads itself: no branch)
        bf16x8 aH, aM, aL;
        split3(*reinterpret_cast<const float4*>(arow + 16 * s), *reinterpret_cast<const float4*>(arow + 16 * s + 4),
               aH, aM, aL);
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          acc[c] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(aL, bc[c][0], acc[c], 0, 0, 0);
          acc[c] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(aH, bc[c][2], acc[c], 0, 0, 0);
          acc[c] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(aM, bc[c][1], acc[c], 0, 0, 0);
          acc[c] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(aM, bc[c][0], acc[c], 0, 0, 0);
          acc[c] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(aH, bc[c][1], acc[c], 0, 0, 0);
          acc[c] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(aH, bc[c][0], acc[c], 0, 0, 0);
        }
#pragma unroll
        for (int c = 0; c < 2; ++c)
#pragma unroll
          for (int e = 0; e < 3; ++e) bc[c][e] = bn[c][e];
      }
    } else {
      const float* wrow = W + (int64_t)(2 * cp * 32 + l32) * K + kq8 * ksp + 8 * hh;  // column group 2 cp; +32 rows: 2 cp + 1
      float4 bc[2][2], bn[2][2];
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        bc[c][0] = *reinterpret_cast<const float4*>(wrow + (int64_t)c * 32 * K);
        bc[c][1] = *reinterpret_cast<const float4*>(wrow + (int64_t)c * 32 * K + 4);
      }
      for (int s = 0; s < nst; ++s) {
        const int kn = 16 * (s + 1 < nst ? s + 1 : s);
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          bn[c][0] = *reinterpret_cast<const float4*>(wrow + (int64_t)c * 32 * K + kn);
          bn[c][1] = *reinterpret_cast<const float4*>(wrow + (int64_t)c * 32 * K + kn + 4);
        }
        bf16x8 aH, aM, aL;
        split3(*reinterpret_cast<const float4*>(arow + 16 * s), *reinterpret_cast<const float4*>(arow + 16 * s + 4),
               aH, aM, aL);
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          bf16x8 bH, bM, bL;
          split3(bc[c][0], bc[c][1], bH, bM, bL);
          acc[c] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(aL, bH, acc[c], 0, 0, 0);
          acc[c] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(aH, bL, acc[c], 0, 0, 0);
          acc[c] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(aM, bM, acc[c], 0, 0, 0);
          acc[c] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(aM, bH, acc[c], 0, 0, 0);
          acc[c] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(aH, bM, acc[c], 0, 0, 0);
          acc[c] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(aH, bH, acc[c], 0, 0, 0);
        }
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          bc[c][0] = bn[c][0];
          bc[c][1] = bn[c][1];
        }
      }
    }
    __syncthreads();  // every wave is done reading the A tile
    // ---- partial tiles -> LDS red[kq8][row][col], fixed-order sum, epilogue
    float* red = sA;  // [8][32][128]
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = (r & 3) + 8 * (r >> 2) + 4 * hh;
        red[(kq8 * kAw32Rows + row) * kWpOut + (2 * cp + c) * 32 + l32] = acc[c][r];
      }
    __syncthreads();
    {
      const int row = tid >> 5, c4 = tid & 31;  // 4 columns 4 c4 .. 4 c4 + 3
      float4 sm = *reinterpret_cast<const float4*>(red + row * kWpOut + 4 * c4);
#pragma unroll
      for (int j = 1; j < 8; ++j) {
        const float4 p = *reinterpret_cast<const float4*>(red + (j * kAw32Rows + row) * kWpOut + 4 * c4);
        sm.x += p.x;
        sm.y += p.y;
        sm.z += p.z;
        sm.w += p.w;
      }
      const float4 bv = *reinterpret_cast<const float4*>(bias + 4 * c4);
      const float v[4] = {lrelu(sm.x + bv.x), lrelu(sm.y + bv.y), lrelu(sm.z + bv.z), lrelu(sm.w + bv.w)};
      float s2 = v[0] * v[0] + v[1] * v[1] + v[2] * v[2] + v[3] * v[3];
#pragma unroll
      for (int o = 1; o < 32; o <<= 1) s2 += __shfl_xor(s2, o, 64);
      const float nrm = sqrtf(s2);
      const float4 yv = make_float4(v[0] / nrm, v[1] / nrm, v[2] / nrm, v[3] / nrm);
      if (row < nrows) {
        *reinterpret_cast<float4*>(y + (r0 + row) * kWpOut + 4 * c4) = yv;
        if (c4 == 0 && nrm_out) nrm_out[r0 + row] = nrm;
      }
      if (nx.q) {
        // ---- the next layer's Q projection of these rows (AggNextQ), as in
        //      agg_w32_kernel: the y tile to LDS (over red, once every thread
        //      has read it) with each row's next-layer q row (-1: none)
        float* sY = sA;  // [32][kAw32Lq]
        int* sU = sLoc;  // [32]
        __syncthreads();
        *reinterpret_cast<float4*>(sY + row * kAw32Lq + 4 * c4) = yv;
        if (c4 == 0) {
          int u = -1;
          if (row < nrows) {
            const int64_t id = nx.S_mem[r0 + row];
            if ((nx.bits[id >> 6] >> (id & 63)) & 1ull)
              u = (int)(nx.pref[id >> 6] + __popcll(nx.bits[id >> 6] & ((1ull << (id & 63)) - 1ull)));
          }
          sU[row] = u;
        }
      }
    }
    if (nx.q) {
      __syncthreads();
      for (int cq = wave; cq < nx.hid / 32; cq += kAw32Threads / 64) {
        const float* qrow = nx.Qw + (int64_t)(cq * 32 + l32) * kWpOut + 8 * hh;
        f32x16 qa;
#pragma unroll
        for (int r = 0; r < 16; ++r) qa[r] = 0.f;
        const float* ap = sA + l32 * kAw32Lq + 8 * hh;
#pragma unroll 2
        for (int s = 0; s < 8; ++s) {
          bf16x8 aH, aM, aL, bH, bM, bL;
          split3(*reinterpret_cast<const float4*>(ap + 16 * s), *reinterpret_cast<const float4*>(ap + 16 * s + 4),
                 aH, aM, aL);
          split3(*reinterpret_cast<const float4*>(qrow + 16 * s), *reinterpret_cast<const float4*>(qrow + 16 * s + 4),
                 bH, bM, bL);
          qa = __builtin_amdgcn_mfma_f32_32x32x16_bf16(aL, bH, qa, 0, 0, 0);
          qa = __builtin_amdgcn_mfma_f32_32x32x16_bf16(aH, bL, qa, 0, 0, 0);
          qa = __builtin_amdgcn_mfma_f32_32x32x16_bf16(aM, bM, qa, 0, 0, 0);
          qa = __builtin_amdgcn_mfma_f32_32x32x16_bf16(aM, bH, qa, 0, 0, 0);
          qa = __builtin_amdgcn_mfma_f32_32x32x16_bf16(aH, bM, qa, 0, 0, 0);
          qa = __builtin_amdgcn_mfma_f32_32x32x16_bf16(aH, bH, qa, 0, 0, 0);
        }
        const int col = cq * 32 + l32;
        const float bq = nx.Qb[col];
        float qv[16];
        int us[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          us[r] = sLoc[(r & 3) + 8 * (r >> 2) + 4 * hh];
          qv[r] = lrelu(qa[r] + bq);
          asm volatile("" : "+v"(qv[r]), "+v"(us[r]));
        }
#pragma unroll
        for (int r = 0; r < 16; ++r)
          if (us[r] >= 0) nx.q[(int64_t)us[r] * nx.hid + col] = qv[r];
      }
    }
    __syncthreads();  // LDS is reused by the next tile
  }
}

int64_t agg_w_planes_bytes(int64_t d, int64_t hid) { return 3 * kWpOut * (d + hid) * 2; }

int launch_split_wplanes(const float* W, int64_t ldw, int K, uint16_t* planes, hipStream_t st) {
  PS_REQUIRE(K % 16 == 0 && ldw >= K && ldw % 4 == 0, kErrArg, "split_wplanes: K % 16 == 0, ldw >= K, ldw % 4 == 0");
  const int64_t n = (int64_t)K * kWpOut / 8;
  hipLaunchKernelGGL(split_wplanes_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, W, ldw, K, planes);
  PS_CHECK_LAUNCH();
  return kOk;
}

static int agg_w32_supported(int64_t d, int64_t hid, int64_t T) {
  const int64_t K = d + hid;
  const int64_t lds = (int64_t)kAw32Rows * (K + 4) * 4 + 2 * kAw32Rows * kAw32TMax * 4 + kAw32Rows * 4;
  return K % 128 == 0 && K + 4 >= 4 * kAw32Out && T <= kAw32TMax && lds <= 160 * 1024;
}

// the 32-row form (agg_w32s_kernel) also needs its LDS (the 8 partial tiles)
static int agg_w32s_supported(int64_t d, int64_t hid, int64_t T) {
  return agg_w32_supported(d, hid, T) && T >= 1 && ws_lds_bytes(d + hid) <= 160 * 1024;
}

int agg_w_supported(int64_t d, int64_t hid, int64_t out, int64_t T) {
  const int64_t K = d + hid;
  const int64_t lds = (int64_t)kAwRows * (K + 4) * 4 + 2 * kAwRows * kAwTMax * 4 + kAwRows * 4;
  // the A tile's LDS is reused for the [16][128] output tile (K + 4 >= 128);
  // two workgroups per CU; the aggregation pass covers hid in passes of 512
  return out == kAwOut && K % 64 == 0 && K + 4 >= kAwOut && hid % 4 == 0 && d % 4 == 0 &&
         T >= 1 && T <= kAwTMax && 2 * lds <= 160 * 1024;
}

static int64_t aggw_min_rows32(int cus) {
  return getenv("PINSAGE_AGGW32_MIN_ROWS") ? atoll(getenv("PINSAGE_AGGW32_MIN_ROWS")) : 16 * (int64_t)cus;
}

static int device_cus() {
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
    cus = 256;
  return cus;
}

int agg_w_uses_planes(int64_t d, int64_t hid, int64_t out, int64_t T, int64_t S_est) {
  return out == kWpOut && S_est > 0 && S_est >= aggw_min_rows32(device_cus()) && agg_w32s_supported(d, hid, T);
}

int agg_w_next_q_pays(int64_t d, int64_t hid, int64_t T, int64_t S_est) {
  const int cus = device_cus();
  return S_est > 0 && S_est >= aggw_min_rows32(cus) && agg_w32s_supported(d, hid, T) &&
         (S_est + kAw32Rows - 1) / kAw32Rows <= cus;
}

// S_max: the expected row count (the frontier size hint; the kernels read the
// actual count from nS, or take n_static when nS is null, and deal it over
// their blocks)
int launch_agg_w(const float* h, int64_t ldh, int d, const int32_t* self_src, const float* q, int hid,
                 const int32_t* loc, const float* wloc, int T, const int* nS, int64_t n_static, int64_t S_max,
                 const float* W, const float* bias, float* y, float* nrm, float* agg, hipStream_t st,
                 const AggNextQ* next, int* next_done, uint16_t* planes, int planes_ready,
                 const AggHead* head, int* head_done) {
  if (next_done) *next_done = 0;
  if (head_done) *head_done = 0;
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
  const int cus = device_cus();
  // ~12 rows per block (a 16-row tile with headroom), two blocks per CU
  const int grid = (int)std::max<int64_t>(1, std::min<int64_t>(2 * (int64_t)cus, (S_max + 11) / 12));
  // The 32-row form (one block per CU, W read once per 32 rows) when the rows
  // fill ~16 per CU; below that the 16-row form (two blocks per CU, one's gather
  // beside the other's products) hides more latency.  Measured (bench.py):
  // C2 layer 0 (5.7k rows, K 1024) 36.5 vs 55.3 us, C4 layer 0 (8.6k, K 640)
  // 50.2 vs 73.4 us; the layers 1 (1.5-2k rows, K 640) 21.5-21.8 vs 24.7-25.3 us.
  // PINSAGE_AGGW32_MIN_ROWS overrides the switch point (A/B).
  const int64_t min_rows32 = aggw_min_rows32(cus);
  if (S_max >= min_rows32 && agg_w32s_supported(d, hid, T)) {
    // ~24 rows per block (a 32-row tile with headroom) over every CU
    const int64_t g32 = std::max<int64_t>(1, std::min<int64_t>(cus, (S_max + 23) / 24));
    AggNextQ nx;
    if (next && next->q) {
      PS_REQUIRE(next->hid > 0 && next->hid % 32 == 0 && next->S_mem && next->bits && next->pref &&
                     next->Qw && next->Qb,
                 kErrArg, "agg_w: next-layer Q projection needs hid % 32 == 0 and every pointer");
      nx = *next;
      if (next_done) *next_done = 1;
    }
    const int lds_s = (int)ws_lds_bytes(K);
    static bool prepared_s = false;
    if (!prepared_s) {
      PS_CHECK_HIP(hipFuncSetAttribute((const void*)agg_w32s_kernel<true>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
      PS_CHECK_HIP(hipFuncSetAttribute((const void*)agg_w32s_kernel<false>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
      prepared_s = true;
    }
    if (planes) {
      if (!planes_ready) PS_TRY(launch_split_wplanes(W, K, K, planes, st));
      hipLaunchKernelGGL(agg_w32s_kernel<true>, dim3((int)g32), dim3(kAw32Threads), lds_s, st, h, ldh, d, self_src,
                         q, hid, loc, wloc, T, nS, n_static, W, (const uint16_t*)planes, bias, y, nrm, agg, nx);
    } else {
      hipLaunchKernelGGL(agg_w32s_kernel<false>, dim3((int)g32), dim3(kAw32Threads), lds_s, st, h, ldh, d,
                         self_src, q, hid, loc, wloc, T, nS, n_static, W, (const uint16_t*)nullptr, bias, y, nrm,
                         agg, nx);
    }
  } else {
    AggHead hd;
    if (head && head->G1w && K >= 2 * kAwOut) {  // (y and H1 beside the output tile in the A tile's LDS)
      PS_REQUIRE(head->G1b && head->G2w && head->H1 && head->Z, kErrArg, "agg_w: the fused head needs every pointer");
      hd = *head;
      if (head_done) *head_done = 1;
    }
    // PINSAGE_AGGW_NH (default 1): a launch without the head runs the
    // 128-VGPR form (two blocks per CU; the with-head form compiles to more)
    static const int nh = getenv("PINSAGE_AGGW_NH") ? atoi(getenv("PINSAGE_AGGW_NH")) : 1;
    static bool prepared_nh = false;
    if (!prepared_nh) {
      PS_CHECK_HIP(hipFuncSetAttribute((const void*)agg_w_nh_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       160 * 1024));
      prepared_nh = true;
    }
    if (nh && !hd.G1w)
      hipLaunchKernelGGL(agg_w_nh_kernel, dim3(grid), dim3(kAwThreads), lds, st, h, ldh, d, self_src, q, hid,
                         loc, wloc, T, nS, n_static, W, bias, y, nrm, agg, hd);
    else
      hipLaunchKernelGGL(agg_w_kernel, dim3(grid), dim3(kAwThreads), lds, st, h, ldh, d, self_src, q, hid,
                         loc, wloc, T, nS, n_static, W, bias, y, nrm, agg, hd);
  }
  PS_CHECK_LAUNCH();
  return kOk;
}

}  // namespace ps
