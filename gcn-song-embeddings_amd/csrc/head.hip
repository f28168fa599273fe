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
// MFMA conventions as in gemm.hip: exact fp32 (v_mfma_f32_32x32x2_f32: in the
// r-th MFMA of k-octet s, lane (l32, h) supplies k = 8s + 4h + r) or split bf16
// (head_mm_bf); accumulator element r of lane (l32, h) is row (r & 3) + 8 (r >>
// 2) + 4h, column l32 of the 32 x 32 tile.
#include "bf16split.h"
#include "common.h"

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
__device__ __forceinline__ f32x16 head_mm_f32(const float* sA, const float* sW, int n0, int l32,
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

// The same product with split-bf16 MFMAs (the GEMMs' arithmetic, gemm.hip):
// each fp32 operand = hi + mid + lo bf16, six v_mfma_f32_32x32x16_bf16 per
// 16-k step, smallest products first; lane (l32, h) supplies k = 16 s + 8 h
// + [0, 8).  48 MFMAs of 32 cycles per wave against 64 f32 MFMAs of 64:
// the head's two row-block products were a third of its kernels' time at C2.
template <bool kNK>
__device__ __forceinline__ f32x16 head_mm_bf(const float* sA, const float* sW, int n0, int l32, int h) {
  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  const float* arow = sA + l32 * kHeadLd + 8 * h;
  const int n = n0 + l32;
#pragma unroll 2
  for (int s = 0; s < kHeadDim / 16; ++s) {
    const float4 a0 = *reinterpret_cast<const float4*>(arow + 16 * s);
    const float4 a1 = *reinterpret_cast<const float4*>(arow + 16 * s + 4);
    float4 b0, b1;
    if constexpr (kNK) {
      b0 = *reinterpret_cast<const float4*>(sW + n * kHeadLd + 16 * s + 8 * h);
      b1 = *reinterpret_cast<const float4*>(sW + n * kHeadLd + 16 * s + 8 * h + 4);
    } else {
      const float* c = sW + (16 * s + 8 * h) * kHeadLd + n;
      b0 = make_float4(c[0], c[kHeadLd], c[2 * kHeadLd], c[3 * kHeadLd]);
      b1 = make_float4(c[4 * kHeadLd], c[5 * kHeadLd], c[6 * kHeadLd], c[7 * kHeadLd]);
    }
    bf16x8 aH, aM, aL, bH, bM, bL;
    split3(a0, a1, aH, aM, aL);
    split3(b0, b1, bH, bM, bL);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(aL, bH, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(aH, bL, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(aM, bM, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(aM, bH, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(aH, bM, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(aH, bH, acc, 0, 0, 0);
  }
  return acc;
}
// products in the GEMMs' default arithmetic (gemm_default_prec: 1 split bf16,
// 0 exact fp32 MFMA), a kernel template parameter chosen per launch
template <bool kNK, bool BF>
__device__ __forceinline__ f32x16 head_mm(const float* sA, const float* sW, int n0, int l32, int h) {
  if constexpr (BF) return head_mm_bf<kNK>(sA, sW, n0, l32, h);
  else return head_mm_f32<kNK>(sA, sW, n0, l32, h);
}

// rows [r0, r0+32) of src[R][o] -> sA (zero outside), all threads
// (every global load of a staging pass is issued before the first LDS write:
// one memory round trip per pass, not one per float4)
__device__ __forceinline__ void head_load_rows(float* sA, const float* __restrict__ src, int64_t r0,
                                               int64_t R, int o, int tid) {
  constexpr int NI = kHeadRows * (kHeadDim / 4) / 256;
  float4 v[NI];
#pragma unroll
  for (int j = 0; j < NI; ++j) {
    const int i = tid + 256 * j, row = i / (kHeadDim / 4), c = 4 * (i % (kHeadDim / 4));
    v[j] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (r0 + row < R && c < o) v[j] = *reinterpret_cast<const float4*>(src + (r0 + row) * o + c);
  }
#pragma unroll
  for (int j = 0; j < NI; ++j) {
    const int i = tid + 256 * j, row = i / (kHeadDim / 4), c = 4 * (i % (kHeadDim / 4));
    *reinterpret_cast<float4*>(sA + row * kHeadLd + c) = v[j];
  }
}
// W[o][o] row-major -> sW (same layout, zero padded to 128 x 128)
__device__ __forceinline__ void head_load_weight(float* sW, const float* __restrict__ W, int o,
                                                 int tid) {
  constexpr int NI = kHeadDim * (kHeadDim / 4) / 256;
  float4 v[NI];
#pragma unroll
  for (int j = 0; j < NI; ++j) {
    const int i = tid + 256 * j, row = i / (kHeadDim / 4), c = 4 * (i % (kHeadDim / 4));
    v[j] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (row < o && c < o) v[j] = *reinterpret_cast<const float4*>(W + (int64_t)row * o + c);
  }
#pragma unroll
  for (int j = 0; j < NI; ++j) {
    const int i = tid + 256 * j, row = i / (kHeadDim / 4), c = 4 * (i % (kHeadDim / 4));
    *reinterpret_cast<float4*>(sW + row * kHeadLd + c) = v[j];
  }
}

__device__ __forceinline__ int head_row(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

// H1 = lrelu(y G1^T + b1), Z = H1 G2^T over the *nrows rows of y
template <bool BF>
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
  head_load_rows(sA, y, r0, R, o, tid);
  head_load_weight(sW1, G1w, o, tid);
  head_load_weight(sW2, G2w, o, tid);
  __syncthreads();
  f32x16 acc = head_mm<true, BF>(sA, sW1, n0, l32, h);
  const float b = col < o ? G1b[col] : 0.f;
  __syncthreads();  // every wave is done reading y from sA
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int row = head_row(r, h);
    const float v = col < o ? lrelu(acc[r] + b) : 0.f;
    sA[row * kHeadLd + col] = v;
    if (r0 + row < R && col < o) H1[(r0 + row) * o + col] = v;
  }
  __syncthreads();
  acc = head_mm<true, BF>(sA, sW2, n0, l32, h);
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
__device__ __forceinline__ void head_load_dz(float* sA, float* __restrict__ G, int* __restrict__ Kc,
                                             int64_t S_max, float* __restrict__ dZ, int64_t r0, int64_t R,
                                             int o, int tid) {
  constexpr int NI = kHeadRows * (kHeadDim / 4) / 256;
  float4 g[3][NI];
  int k[3][NI];
#pragma unroll
  for (int j = 0; j < NI; ++j) {
    const int i = tid + 256 * j, row = i / (kHeadDim / 4), c = 4 * (i % (kHeadDim / 4));
    const bool ok = r0 + row < R && c < o;
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      k[q][j] = ok ? Kc[q * S_max + r0 + row] : 0;
      g[q][j] = ok ? *reinterpret_cast<const float4*>(G + ((int64_t)q * S_max + r0 + row) * o + c)
                   : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
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
template <bool BF>
__global__ __launch_bounds__(256) void head_bwd_kernel(
    float* __restrict__ G, int* __restrict__ Kc, int64_t S_max, float* __restrict__ dZ, int o,
    const int* __restrict__ nrows, const float* __restrict__ H1, const float* __restrict__ G1w,
    const float* __restrict__ G2w, const float* __restrict__ y, const float* __restrict__ nrm,
    float* __restrict__ dP1, float* __restrict__ dp) {
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
  // this lane's H1 (mask) and y values, fetched beside the staging loads
  float hv[16], yv[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int row = head_row(r, h);
    const bool ok = r0 + row < R && col < o;
    hv[r] = ok ? H1[(r0 + row) * o + col] : 0.f;
    yv[r] = ok ? y[(r0 + row) * o + col] : 0.f;
  }
  head_load_dz(sA, G, Kc, S_max, dZ, r0, R, o, tid);
  head_load_weight(sW2, G2w, o, tid);
  head_load_weight(sW1, G1w, o, tid);
  __syncthreads();
  if (tid < 3 * kHeadRows) {  // every K of the block's rows has been read
    const int q = tid / kHeadRows, row = tid % kHeadRows;
    if (r0 + row < R) Kc[q * S_max + r0 + row] = 0;
  }
  f32x16 acc = head_mm<false, BF>(sA, sW2, n0, l32, h);
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
  acc = head_mm<false, BF>(sA, sW1, n0, l32, h);  // dY
  // row dots y . dY: lane-partial over this wave's 32 columns, then 4 waves
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int row = head_row(r, h);
    float d = yv[r] * acc[r];
#pragma unroll
    for (int m = 1; m < 32; m <<= 1) d += __shfl_xor(d, m, 64);
    if (l32 == 0) red[w * kHeadRows + row] = d;
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int row = head_row(r, h);
    if (r0 + row < R && col < o) {
      const float dot = (red[row] + red[kHeadRows + row]) + (red[2 * kHeadRows + row] + red[3 * kHeadRows + row]);
      const float inv = 1.f / nrm[r0 + row];
      dp[(r0 + row) * o + col] = lrelu_grad(yv[r]) * (acc[r] - yv[r] * dot) * inv;
    }
  }
}

constexpr size_t kHeadFwdLds = (size_t)(kHeadRows + 2 * kHeadDim) * kHeadLd * 4;
constexpr size_t kHeadBwdLds = kHeadFwdLds + 4 * kHeadRows * 4;

int gemm_default_prec();

static int head_prepare() {
  static int rc = [] {
    auto lds = [](const void* f, size_t b) {
      return hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)b) == hipSuccess;
    };
    if (!lds((const void*)head_fwd_kernel<true>, kHeadFwdLds) || !lds((const void*)head_fwd_kernel<false>, kHeadFwdLds) ||
        !lds((const void*)head_bwd_kernel<true>, kHeadBwdLds) || !lds((const void*)head_bwd_kernel<false>, kHeadBwdLds))
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
  if (gemm_default_prec() == 1)
    hipLaunchKernelGGL(head_fwd_kernel<true>, dim3((unsigned)ceil_div(max_rows, kHeadRows)), dim3(256),
                       kHeadFwdLds, st, y, o, nrows, G1w, G1b, G2w, H1, Z);
  else
    hipLaunchKernelGGL(head_fwd_kernel<false>, dim3((unsigned)ceil_div(max_rows, kHeadRows)), dim3(256),
                       kHeadFwdLds, st, y, o, nrows, G1w, G1b, G2w, H1, Z);
  PS_CHECK_LAUNCH();
  return kOk;
}

int launch_head_bwd(float* G, int* Kc, int64_t S_max, float* dZ, int o, const int* nrows,
                    int64_t max_rows, const float* H1, const float* G1w, const float* G2w,
                    const float* y, const float* nrm, float* dP1, float* dp, hipStream_t st) {
  PS_REQUIRE(head_supported(o), kErrArg, "head: out_dim must be a multiple of 4, <= 128");
  PS_TRY(head_prepare());
  if (max_rows <= 0) return kOk;
  if (gemm_default_prec() == 1)
    hipLaunchKernelGGL(head_bwd_kernel<true>, dim3((unsigned)ceil_div(max_rows, kHeadRows)), dim3(256),
                       kHeadBwdLds, st, G, Kc, S_max, dZ, o, nrows, H1, G1w, G2w, y, nrm, dP1, dp);
  else
    hipLaunchKernelGGL(head_bwd_kernel<false>, dim3((unsigned)ceil_div(max_rows, kHeadRows)), dim3(256),
                       kHeadBwdLds, st, G, Kc, S_max, dZ, o, nrows, H1, G1w, G2w, y, nrm, dP1, dp);
  PS_CHECK_LAUNCH();
  return kOk;
}

}  // namespace ps
