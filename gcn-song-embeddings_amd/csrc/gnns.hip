// Segmented weighted mean: the MEAN aggregator of lib/gnns
// (GNNs_unsupervised.py:537-588, GNN_model.aggregate with agg_func 'MEAN').
// The reference builds a dense [F, U] mask (ones at each sampled neighbour,
// times sqrt(edge count), L1-normalised by F.normalize(p=1)) and multiplies it
// with the [U, d] embedding matrix; the mask has a handful of non-zeros per
// row, so here it is a CSR (seg_ptr, cols, w) and the product is a per-row
// gather-and-accumulate: HBM-bound, one wave per row, float4 column chunks per
// lane, four neighbour rows' loads in flight per step.  The backward of the
// product (dH = mask^T dOut) is the same kernel over the transposed CSR with
// the normalisation already folded into its weights (normalize = 0), so no
// atomics and a fixed summation order.
#include "../../include/pinsage_hip.h"
#include "common.h"

namespace ps {

// out[i, :] = sum_j w_j * h[cols_j, :] / den_i,  den_i = max(sum_j |w_j|, 1e-12)
// (normalize) or 1.  Rows whose neighbours are out of [0, n_h) skip them.
template <bool VEC>
__global__ __launch_bounds__(256) void segment_wmean_kernel(
    const float* __restrict__ h, int64_t ldh, int64_t n_h, int d, const int64_t* __restrict__ seg_ptr,
    const int32_t* __restrict__ cols, const float* __restrict__ w, int64_t n_seg, int normalize,
    float* __restrict__ out, int64_t ldo) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= n_seg) return;
  const int64_t b = seg_ptr[row], e = seg_ptr[row + 1];
  float inv = 1.f;
  if (normalize) {
    float s = 0.f;
    for (int64_t j = b + lane; j < e; j += 64) s += fabsf(w[j]);
    s = wave_sum(s);
    inv = 1.f / fmaxf(s, 1e-12f);
  }
  float* o = out + row * ldo;
  if constexpr (VEC) {
    for (int c = 4 * lane; c < d; c += 256) {
      float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
      int64_t j = b;
      for (; j + 4 <= e; j += 4) {
        float4 x[4];
        float wj[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int64_t r = cols[j + u];
          const bool ok = (uint64_t)r < (uint64_t)n_h;
          wj[u] = ok ? w[j + u] * inv : 0.f;
          x[u] = *reinterpret_cast<const float4*>(h + (ok ? r : 0) * ldh + c);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          acc.x = fmaf(wj[u], x[u].x, acc.x);
          acc.y = fmaf(wj[u], x[u].y, acc.y);
          acc.z = fmaf(wj[u], x[u].z, acc.z);
          acc.w = fmaf(wj[u], x[u].w, acc.w);
        }
      }
      for (; j < e; ++j) {
        const int64_t r = cols[j];
        if ((uint64_t)r >= (uint64_t)n_h) continue;
        const float wj = w[j] * inv;
        const float4 x = *reinterpret_cast<const float4*>(h + r * ldh + c);
        acc.x = fmaf(wj, x.x, acc.x);
        acc.y = fmaf(wj, x.y, acc.y);
        acc.z = fmaf(wj, x.z, acc.z);
        acc.w = fmaf(wj, x.w, acc.w);
      }
      *reinterpret_cast<float4*>(o + c) = acc;
    }
  } else {
    for (int c = lane; c < d; c += 64) {
      float acc = 0.f;
      for (int64_t j = b; j < e; ++j) {
        const int64_t r = cols[j];
        if ((uint64_t)r >= (uint64_t)n_h) continue;
        acc = fmaf(w[j] * inv, h[r * ldh + c], acc);
      }
      o[c] = acc;
    }
  }
}

}  // namespace ps

using namespace ps;

extern "C" {

int pinsage_segment_wmean(const float* h, int64_t ldh, int64_t n_h, int64_t d, const int64_t* seg_ptr,
                          const int32_t* cols, const float* w, int64_t n_seg, int normalize, float* out,
                          int64_t ldo, void* stream) {
  if (n_seg < 0 || d <= 0 || d > (1 << 24) || n_h < 0 || ldh < d || ldo < d || !seg_ptr ||
      (n_seg > 0 && !out) || (n_h > 0 && !h)) {
    set_error("segment_wmean: bad argument");
    return kErrArg;
  }
  if (n_seg == 0) return kOk;
  const bool vec = n_h > 0 && d % 4 == 0 && ldh % 4 == 0 && ldo % 4 == 0 && ((uintptr_t)h & 15) == 0 &&
                   ((uintptr_t)out & 15) == 0;
  const dim3 grid((unsigned)ceil_div(n_seg, 4)), block(256);
  if (vec)
    hipLaunchKernelGGL(segment_wmean_kernel<true>, grid, block, 0, (hipStream_t)stream, h, ldh, n_h, (int)d,
                       seg_ptr, cols, w, n_seg, normalize, out, ldo);
  else
    hipLaunchKernelGGL(segment_wmean_kernel<false>, grid, block, 0, (hipStream_t)stream, h, ldh, n_h, (int)d,
                       seg_ptr, cols, w, n_seg, normalize, out, ldo);
  PS_CHECK_LAUNCH();
  return kOk;
}

}  // extern "C"
