// Weight gradients of the nn.Linear layers (pinsage_model.py:196-201, 208-210;
// the AddmmBackward of every Q / W projection and of the head): over the
// device-side row count K,
//   dW[M][N] = A^T [B || B2]     A [K][M] row-major (M-major), B rows gathered
//   db[M]    = column sums of A
// optionally followed by torch.optim.Adam on the slice (the step's last
// gradient, Q0's, applies its own update).
//
// Long-K form.  The split-K GEMM (gemm.hip, kEpiPartial) cuts K into up to 64
// short slices so that its 128 x 128 tiles fill the chip, writes one fp32 slab
// per slice and leaves the sum to reduce_slabs_2d (C2 layer 0: 32 slabs of
// 1 MB, a second launch on the chain).  Here a 512-thread workgroup owns one
// 64 x 64 output tile and a LONG run of K:
//   * its 8 waves take the run's 16-row stages round-robin, each wave with a
//     private double-buffered LDS ring fed by LDS-DMA (no block barrier in the
//     k loop: a wave waits only for its own DMAs, with a counted vmcnt), and
//     accumulates the whole 64 x 64 tile (2 x 2 fragments, so each split
//     operand fragment feeds six MFMAs twice: half the hi / mid / lo
//     conversions per product of a 32 x 32 wave tile);
//   * the 8 wave partials are added in LDS in wave order;
//   * K is cut into S <= 16 splits only as far as the grid needs (~one
//     workgroup per CU); the splits of a tile are combined IN the launch by
//     the last to arrive (write-through sc1 slab stores, one agent-scope
//     ticket per workgroup, sc1 loads in split order -- the stream-K hand-off
//     of gemm.hip), which also writes the bias, and applies Adam.
// Every sum has a fixed order (k within a wave's stages, waves, splits), so the
// result does not depend on timing.  Products: the split-bf16 arithmetic of
// gemm.hip (x = hi + mid + lo bf16 exactly to 2^-26, the six products >=
// 2^-18 hi*hi as v_mfma_f32_32x32x16_bf16, fp32 accumulation).
#include "wgrad.h"

#include <algorithm>

#include "bf16split.h"
#include "lds_dma.h"

namespace ps {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kKwWaves = 8;
constexpr int kKwBK = 16;                     // k-rows per stage
constexpr int kKwT = 64;                      // tile edge (M and N)
constexpr int kKwImg = kKwBK * kKwT;          // floats per operand image
constexpr int kKwStage = 2 * kKwImg;          // A + B
constexpr int kKwRing = kKwWaves * 2 * kKwStage;  // two stages per wave: 32768 floats (128 KiB)
constexpr int kKwWin = 6144;                  // gathered row numbers staged per pass (24 KiB)
constexpr int kKwMaxSplits = 16;
static_assert(kKwRing >= kKwWaves * kKwT * kKwT, "the wave partials reuse the ring");

// lane l of a 1-KiB DMA covers row 4 j + l / 16 of a stage, columns 4 (l % 16) ..
__device__ __forceinline__ float4 kw_frag(const float* img, int col, int k4) {
  return make_float4(img[(k4 + 0) * kKwT + col], img[(k4 + 1) * kKwT + col], img[(k4 + 2) * kKwT + col],
                     img[(k4 + 3) * kKwT + col]);
}

__global__ __launch_bounds__(512, 1) void wgrad_kw_kernel(KwParams p) {
  __shared__ __attribute__((aligned(16))) float smem[kKwRing + kKwWin];
  int* const sidx = reinterpret_cast<int*>(smem + kKwRing);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int h = lane >> 5, l32 = lane & 31;
  const int K = p.K_dev ? *p.K_dev : p.K_max;
  const int tm = p.M / kKwT, tn = p.N / kKwT, S = p.S;
  const int G = tm * tn * S;
  // blocks b and b + 8 share an XCD: with G % 8 == 0 each XCD takes a
  // contiguous run of n-blocks, so the workgroups reading one B column slice
  // (the gathered rows) share its L2
  const int b = blockIdx.x;
  const int L = (G % 8 == 0) ? (b % 8) * (G / 8) + b / 8 : b;
  const int nb = L / (tm * S), rem = L - nb * tm * S;
  const int mb = rem / S, s = rem - (rem / S) * S;
  const int m0 = mb * kKwT, n0 = nb * kKwT;
  const int tile = nb * tm + mb;
  // this split's rows, on the 16-row stage grid
  const int kc = ((K + S - 1) / S + kKwBK - 1) / kKwBK * kKwBK;
  const int kb = min(K, s * kc), ke = min(K, kb + kc);
  // the B segment of this column block (launch_wgrad_kw: N1 % 64 == 0)
  const bool seg2 = p.B2 && n0 >= p.N1;
  const float* Bp = seg2 ? p.B2 : p.B;
  const int64_t ldb = seg2 ? p.ldb2 : p.ldb;
  const int32_t* bidx = seg2 ? p.b2_idx : p.b_idx;
  const int bc0 = seg2 ? n0 - p.N1 : n0;
  const bool do_bias = p.dst_b && nb == 0;
  const unsigned smem_lds = (unsigned)(size_t)((__attribute__((address_space(3))) float*)smem);
  const unsigned ring_w = smem_lds + (unsigned)(wave * 2 * kKwStage) * 4u;  // this wave's two stages
  // this lane's DMA column chunk and row within each 1-KiB group
  const int dc = 4 * (lane & 15), dr = lane >> 4;

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  float bsum = 0.f;

  for (int pb = kb; pb < ke; pb += kKwWin) {
    const int pe = min(ke, pb + kKwWin);
    if (bidx) {
      for (int i = tid; i < pe - pb; i += 512) sidx[i] = bidx[pb + i];
      __syncthreads();
    }
    const int ns = (pe - pb + kKwBK - 1) / kKwBK;  // stages of this pass
    const int nw = ns > wave ? (ns - wave + kKwWaves - 1) / kKwWaves : 0;  // this wave's
    // stage it of this wave: rows pb + 16 (wave + 8 it) ..
    auto issue = [&](int it) __attribute__((always_inline)) {
      const int k0 = pb + kKwBK * (wave + kKwWaves * it);
      const unsigned img = ring_w + (unsigned)((it & 1) * kKwStage) * 4u;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int k = min(k0 + 4 * j + dr, pe - 1);
        glds16(p.A + (int64_t)k * p.lda + m0 + dc, img + (unsigned)j * 1024u);
        const int64_t row = bidx ? sidx[k - pb] : k;
        glds16(Bp + row * ldb + bc0 + dc, img + (unsigned)(kKwImg * 4 + j * 1024));
      }
    };
    if (nw > 0) issue(0);
    for (int it = 0; it < nw; ++it) {
      // stage it has landed (nothing younger is in flight yet); then stage it+1
      // goes out into the other slot (read by this wave one iteration ago)
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (it + 1 < nw) issue(it + 1);
      float* const As = smem + wave * 2 * kKwStage + (it & 1) * kKwStage;
      const float* const Bs = As + kKwImg;
      const int k0 = pb + kKwBK * (wave + kKwWaves * it);
      if (k0 + kKwBK > pe) {  // k-tail: A rows past the pass end contribute nothing
        for (int r = pe - k0; r < kKwBK; ++r) As[r * kKwT + lane] = 0.f;
      }
      if (do_bias) {
#pragma unroll
        for (int r = 0; r < kKwBK; ++r) bsum += As[r * kKwT + lane];
      }
      // 16 k: lane (col l32, half h) holds k = 8 h .. 8 h + 7 of each fragment
      bf16x8 aH[2], aM[2], aL[2], bH[2], bM[2], bL[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        split3(kw_frag(As, i * 32 + l32, 8 * h), kw_frag(As, i * 32 + l32, 8 * h + 4), aH[i], aM[i], aL[i]);
        split3(kw_frag(Bs, i * 32 + l32, 8 * h), kw_frag(Bs, i * 32 + l32, 8 * h + 4), bH[i], bM[i], bL[i]);
      }
#define PS_KW_ALL(X, Y)                                                                            \
  _Pragma("unroll") for (int i = 0; i < 2; ++i) _Pragma("unroll") for (int j = 0; j < 2; ++j) \
      acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(X[i], Y[j], acc[i][j], 0, 0, 0);
      PS_KW_ALL(aL, bH)
      PS_KW_ALL(aH, bL)
      PS_KW_ALL(aM, bM)
      PS_KW_ALL(aM, bH)
      PS_KW_ALL(aH, bM)
      PS_KW_ALL(aH, bH)
#undef PS_KW_ALL
    }
    __syncthreads();  // (the next pass rewrites sidx; the epilogue reuses the ring)
  }

  // ---- the 8 wave partials, added in wave order
  float* const part = smem;  // [wave][64 x 64] row-major (the ring is free)
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h, n = j * 32 + l32;
        part[wave * kKwT * kKwT + m * kKwT + n] = acc[i][j][r];
      }
  float* const bpart = smem + kKwRing;  // [wave][64] (sidx is free)
  if (do_bias) bpart[wave * kKwT + lane] = bsum;
  __syncthreads();
  const int e = tid * 8;  // this thread's 8 consecutive elements of the tile
  float v[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) v[q] = 0.f;
#pragma unroll
  for (int w = 0; w < kKwWaves; ++w) {
    const float4 x0 = *reinterpret_cast<const float4*>(part + w * kKwT * kKwT + e);
    const float4 x1 = *reinterpret_cast<const float4*>(part + w * kKwT * kKwT + e + 4);
    v[0] += x0.x; v[1] += x0.y; v[2] += x0.z; v[3] += x0.w;
    v[4] += x1.x; v[5] += x1.y; v[6] += x1.z; v[7] += x1.w;
  }
  float bv = 0.f;
  if (do_bias && tid < kKwT)
#pragma unroll
    for (int w = 0; w < kKwWaves; ++w) bv += bpart[w * kKwT + tid];

  // ---- the splits of this tile, combined by the last to arrive (in split order)
  if (S > 1) {
    typedef int v4i __attribute__((ext_vector_type(4)));
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(p.slab, 0, 0x7fffffff, 0x00020000);
    const unsigned so = (unsigned)(((int64_t)tile * S + s) * kKwT * kKwT + e) * 4u;
    const v4i w0{__float_as_int(v[0]), __float_as_int(v[1]), __float_as_int(v[2]), __float_as_int(v[3])};
    const v4i w1{__float_as_int(v[4]), __float_as_int(v[5]), __float_as_int(v[6]), __float_as_int(v[7])};
    __builtin_amdgcn_raw_buffer_store_b128(w0, rs, so, 0, 16);
    __builtin_amdgcn_raw_buffer_store_b128(w1, rs, so + 16u, 0, 16);
    if (do_bias && tid < kKwT)
      __hip_atomic_store(p.bslab + ((int64_t)mb * S + s) * kKwT + tid, bv, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    int* const flag = reinterpret_cast<int*>(smem);
    if (tid == 0) flag[0] = __hip_atomic_fetch_add(p.cnt + tile, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    const bool last = flag[0] == S - 1;
    if (!last) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (int q = 0; q < 8; ++q) v[q] = 0.f;
    bv = 0.f;
    for (int t = 0; t < S; ++t) {
      const unsigned o = (unsigned)(((int64_t)tile * S + t) * kKwT * kKwT + e) * 4u;
      const v4i y0 = __builtin_amdgcn_raw_buffer_load_b128(rs, o, 0, 16);
      const v4i y1 = __builtin_amdgcn_raw_buffer_load_b128(rs, o + 16u, 0, 16);
      v[0] += __int_as_float(y0.x); v[1] += __int_as_float(y0.y);
      v[2] += __int_as_float(y0.z); v[3] += __int_as_float(y0.w);
      v[4] += __int_as_float(y1.x); v[5] += __int_as_float(y1.y);
      v[6] += __int_as_float(y1.z); v[7] += __int_as_float(y1.w);
      if (do_bias && tid < kKwT)
        bv += __hip_atomic_load(p.bslab + ((int64_t)mb * S + t) * kKwT + tid, __ATOMIC_RELAXED,
                                __HIP_MEMORY_SCOPE_AGENT);
    }
    if (tid == 0) __hip_atomic_store(p.cnt + tile, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }

  // ---- store (and Adam)
  const int m = m0 + e / kKwT, n = n0 + (e % kKwT);
  const int64_t o = (int64_t)m * p.ld_dst + n;
  const float4 g0 = make_float4(v[0], v[1], v[2], v[3]), g1 = make_float4(v[4], v[5], v[6], v[7]);
  *reinterpret_cast<float4*>(p.dst + o) = g0;
  *reinterpret_cast<float4*>(p.dst + o + 4) = g1;
  if (do_bias && tid < kKwT) p.dst_b[m0 + tid] = bv;
  if (p.ad.p) {
    const float ss = p.ad.coef[0], bc2 = p.ad.coef[1];
    if (!(bc2 > 0.f)) return;  // a refused step (pinsage_fly_gate_adam)
    const float omb1 = (float)(1.0 - p.ad.beta1), omb2 = (float)(1.0 - p.ad.beta2);
    const float b2 = (float)p.ad.beta2, eps = p.ad.eps;
    auto adam1 = [&](float& pp, float g, float& mm, float& vv) {
      mm = mm + omb1 * (g - mm);
      vv = vv * b2 + omb2 * g * g;
      const float denom = sqrtf(vv) / bc2 + eps;
      pp = pp - ss * (mm / denom);
    };
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      float4 pp = *reinterpret_cast<const float4*>(p.ad.p + o + 4 * q);
      float4 mm = *reinterpret_cast<const float4*>(p.ad.m + o + 4 * q);
      float4 vv = *reinterpret_cast<const float4*>(p.ad.v + o + 4 * q);
      const float4 g = q ? g1 : g0;
      adam1(pp.x, g.x, mm.x, vv.x);
      adam1(pp.y, g.y, mm.y, vv.y);
      adam1(pp.z, g.z, mm.z, vv.z);
      adam1(pp.w, g.w, mm.w, vv.w);
      *reinterpret_cast<float4*>(p.ad.p + o + 4 * q) = pp;
      *reinterpret_cast<float4*>(p.ad.m + o + 4 * q) = mm;
      *reinterpret_cast<float4*>(p.ad.v + o + 4 * q) = vv;
    }
    if (do_bias && tid < kKwT && p.ad.pb) adam1(p.ad.pb[m0 + tid], bv, p.ad.mb[m0 + tid], p.ad.vb[m0 + tid]);
  }
}

// ---------------------------------------------------------------- host side
bool wgrad_kw_supported(int M, int N, int N1, bool has_b2) {
  return M > 0 && N > 0 && M % kKwT == 0 && N % kKwT == 0 && (!has_b2 || (N1 >= 0 && N1 % kKwT == 0));
}

int wgrad_kw_splits(int M, int N, int64_t K_est) {
  const int tiles = (M / kKwT) * (N / kKwT);
  int S = std::max(1, (256 + tiles - 1) / tiles);
  S = std::min<int64_t>(S, std::max<int64_t>(1, K_est / 256));  // >= 256 rows (16 stages) per split
  S = std::min(S, kKwMaxSplits);
  while (S > 1 && (tiles * S) % 8 != 0 && tiles * S > 8) --S;  // (XCD-aware placement)
  return S;
}

int64_t wgrad_kw_slab_floats(int M, int N) { return (int64_t)kKwMaxSplits * M * N; }
int64_t wgrad_kw_bslab_floats(int M) { return (int64_t)kKwMaxSplits * M; }
int64_t wgrad_kw_tickets(int M, int N) { return (int64_t)(M / kKwT) * (N / kKwT); }

int launch_wgrad_kw(const KwParams& p_in, hipStream_t st) {
  KwParams p = p_in;
  PS_REQUIRE(wgrad_kw_supported(p.M, p.N, p.N1, p.B2 != nullptr), kErrArg,
             "wgrad: M, N (and N1) must be multiples of 64");
  PS_REQUIRE(p.A && p.B && p.dst && p.lda % 4 == 0 && p.ldb % 4 == 0 && (!p.B2 || p.ldb2 % 4 == 0) &&
                 p.ld_dst % 4 == 0 && p.K_max >= 0,
             kErrArg, "wgrad: operands and 16-B aligned row strides");
  PS_REQUIRE(!p.ad.p || (p.ad.m && p.ad.v && p.ad.coef && (!p.dst_b || (p.ad.pb && p.ad.mb && p.ad.vb))),
             kErrArg, "wgrad: incomplete Adam slice");
  if (p.S <= 0) p.S = wgrad_kw_splits(p.M, p.N, p.K_max);
  p.S = std::min(p.S, kKwMaxSplits);
  PS_REQUIRE(p.S == 1 || (p.slab && p.cnt && (!p.dst_b || p.bslab)), kErrArg, "wgrad: split scratch not set");
  const int grid = (p.M / kKwT) * (p.N / kKwT) * p.S;
  hipLaunchKernelGGL(wgrad_kw_kernel, dim3(grid), dim3(512), 0, st, p);
  PS_CHECK_LAUNCH();
  return kOk;
}

}  // namespace ps
