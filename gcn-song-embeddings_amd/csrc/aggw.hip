// The convolution's aggregation and W projection in one kernel
// (pinsage_model.py:201-211):
//
//   agg[f]  = sum_t w[f,t] * q[loc[f,t]]                 (:201-205, weights
//             pre-normalised by their f64 row sum = sum(w*q)/sum(w))
//   y[f]    = normalize(lrelu([h[self f] || agg[f]] W^T + b))   (:208-211)
//
// One workgroup (16 waves) per 32 rows.  It stages the 32 rows' A operand
// [h_self || agg] in LDS -- the self rows gathered from h, the aggregate formed
// right there from the T gathered q rows (fma in slot order t = 0, 1, ..., the
// same arithmetic as agg_kernel) and also written out for the backward's
// weight gradient -- so agg is never read back from memory and the launch
// between the two disappears.  The projection then runs on fp32 MFMA
// (v_mfma_f32_32x32x2_f32) with the K dimension split four ways across the
// waves: wave (kq, cg) owns output columns 32 cg .. 32 cg + 31 over the k
// quarter kq, so a 32-row tile's dependent MFMA chain is K / 8 long instead of
// K / 2 (the unfused 32 x 128 tile ran one chain per SIMD over all of K and was
// latency-bound).  B fragments (W rows, K-major) stream from global / L2 with a
// one-chunk register double buffer.  The four quarters' partial tiles are
// summed in LDS in a fixed order, then bias, LeakyReLU and the row L2 norm.
#include <algorithm>

#include "common.h"

namespace ps {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kAwRows = 32;     // rows per workgroup
constexpr int kAwOut = 128;     // out_dim (4 column groups of 32)
constexpr int kAwThreads = 1024;
constexpr int kAwTMax = 64;     // fanout held in LDS per row

// LDS: A tile [32][K + 4] floats (row stride = 4 mod 64 banks: b128 fragment
// reads of 16 consecutive rows hit distinct banks), then the tile's slot lists.
__device__ __forceinline__ int aw_lda(int K) { return K + 4; }

__global__ __launch_bounds__(kAwThreads) void agg_w_kernel(
    const float* __restrict__ h, int64_t ldh, int d, const int32_t* __restrict__ self_src,
    const float* __restrict__ q, int hid, const int32_t* __restrict__ loc,
    const float* __restrict__ wloc, int T, const int* __restrict__ nS,
    const float* __restrict__ W, const float* __restrict__ bias, float* __restrict__ y,
    float* __restrict__ nrm_out, float* __restrict__ agg) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int K = d + hid, lda = aw_lda(K);
  float* sA = lds;                                          // [32][lda]
  int* sLoc = reinterpret_cast<int*>(lds + kAwRows * lda);  // [32][T]
  float* sW = reinterpret_cast<float*>(sLoc + kAwRows * kAwTMax);  // [32][T]
  int* sSelf = reinterpret_cast<int*>(sW + kAwRows * kAwTMax);     // [32]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t F = *nS;
  const int64_t tiles = (F + kAwRows - 1) / kAwRows;
  for (int64_t tile = blockIdx.x; tile < tiles; tile += gridDim.x) {
    const int64_t r0 = tile * kAwRows;
    const int nrows = (int)min((int64_t)kAwRows, F - r0);
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
    // ---- projection: wave (kq, cg), k quarter kq, columns 32 cg ..
    const int cg = wave & 3, kq = wave >> 2;
    const int l32 = lane & 31, hh = lane >> 5;
    const int kspan = K >> 2, kb = kq * kspan;
    const float* wrow = W + (int64_t)(cg * 32 + l32) * K;
    const float* arow = sA + l32 * lda;
    f32x16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
    // chunks of 4 k-octets (32 k); B fragments of chunk c+1 load while c runs
    const int nch = kspan / 32;
    float4 bcur[4], bnxt[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) bcur[s] = *reinterpret_cast<const float4*>(wrow + kb + 8 * s + 4 * hh);
    for (int ch = 0; ch < nch; ++ch) {
      const int k0 = kb + 32 * ch;
      if (ch + 1 < nch) {
#pragma unroll
        for (int s = 0; s < 4; ++s)
          bnxt[s] = *reinterpret_cast<const float4*>(wrow + k0 + 32 + 8 * s + 4 * hh);
      }
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const float4 av = *reinterpret_cast<const float4*>(arow + k0 + 8 * s + 4 * hh);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av.x, bcur[s].x, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av.y, bcur[s].y, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av.z, bcur[s].z, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av.w, bcur[s].w, acc, 0, 0, 0);
      }
#pragma unroll
      for (int s = 0; s < 4; ++s) bcur[s] = bnxt[s];
    }
    __syncthreads();  // every wave is done reading the A tile
    // ---- partial tiles -> LDS red[kq][row][col], fixed-order sum, epilogue
    float* red = sA;  // [4][32][128]
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = (r & 3) + 8 * (r >> 2) + 4 * hh;
      red[(kq * kAwRows + row) * kAwOut + cg * 32 + l32] = acc[r];
    }
    __syncthreads();
    {
      const int row = tid >> 5, c4 = tid & 31;  // 4 columns 4 c4 .. 4 c4 + 3
      float v[4];
      float s2 = 0.f;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int col = 4 * c4 + e;
        float x = red[(0 * kAwRows + row) * kAwOut + col];
        x += red[(1 * kAwRows + row) * kAwOut + col];
        x += red[(2 * kAwRows + row) * kAwOut + col];
        x += red[(3 * kAwRows + row) * kAwOut + col];
        x = lrelu(x + bias[col]);
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

int agg_w_supported(int64_t d, int64_t hid, int64_t out, int64_t T) {
  const int64_t K = d + hid;
  const int64_t lds = (int64_t)kAwRows * (K + 4) * 4 + 2 * kAwRows * kAwTMax * 4 + kAwRows * 4;
  // the A tile's LDS is reused for the four partial 32 x 128 tiles: K + 4 >= 512
  return out == kAwOut && K % 128 == 0 && K + 4 >= 4 * kAwOut && hid % 4 == 0 && d % 4 == 0 &&
         T >= 1 && T <= kAwTMax && lds <= 160 * 1024;
}

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
  const int64_t tiles = (S_max + kAwRows - 1) / kAwRows;
  const int grid = (int)std::min<int64_t>(tiles, cus);
  hipLaunchKernelGGL(agg_w_kernel, dim3(grid), dim3(kAwThreads), lds, st, h, ldh, d, self_src, q, hid,
                     loc, wloc, T, nS, W, bias, y, nrm, agg);
  PS_CHECK_LAUNCH();
  return kOk;
}

}  // namespace ps
