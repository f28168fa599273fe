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
#include <cstdlib>

#include "bf16split.h"
#include "lds_dma.h"

namespace ps {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kKwBK = 16;                     // k-rows per stage
constexpr int kKwT = 64;                      // tile edge (M and N)
constexpr int kKwImg = kKwBK * kKwT;          // floats per operand image
constexpr int kKwStage = 2 * kKwImg;          // A + B (8 KiB)
constexpr int kKwWin = 6144;                  // gathered row numbers staged per pass (24 KiB)
constexpr int kKwMaxSplits = 16;

// four k-rows of one column of a [16][64] stage image
__device__ __forceinline__ float4 kw_frag(const float* img, int col, int k4) {
  return make_float4(img[(k4 + 0) * kKwT + col], img[(k4 + 1) * kKwT + col], img[(k4 + 2) * kKwT + col],
                     img[(k4 + 3) * kKwT + col]);
}

// The end of a long-K launch (both k-loop forms): the NW wave partials added
// in wave order, the K splits of the tile combined by the last to arrive (in
// split order), the bias and the fused Adam step.  smem: the ring (>= NW 64 x
// 64 floats) followed by >= NW x 64 floats (the bias partials).
template <int NW>
__device__ __forceinline__ void kw_finish(const KwParams& p, f32x16 (&acc)[2][2], float bsum, float* smem,
                                          int ring_floats, int tile, int mb, int s, int m0, int n0,
                                          bool do_bias) {
  constexpr int NT = NW * 64;
  constexpr int E4 = kKwT * kKwT / 4 / NT;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int h = lane >> 5, l32 = lane & 31;
  const int S = p.S;
  // ---- the NW wave partials, added in wave order
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
  float* const bpart = smem + ring_floats;  // [wave][64] (sidx is free)
  if (do_bias) bpart[wave * kKwT + lane] = bsum;
  __syncthreads();
  // this thread's float4s of the tile: e4 = q NT + tid (coalesced rows)
  float4 v[E4];
#pragma unroll
  for (int q = 0; q < E4; ++q) {
    v[q] = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int w = 0; w < NW; ++w) {
      const float4 x = *reinterpret_cast<const float4*>(part + w * kKwT * kKwT + 4 * (q * NT + tid));
      v[q].x += x.x;
      v[q].y += x.y;
      v[q].z += x.z;
      v[q].w += x.w;
    }
  }
  float bv = 0.f;
  if (do_bias && tid < kKwT)
#pragma unroll
    for (int w = 0; w < NW; ++w) bv += bpart[w * kKwT + tid];

  // ---- the splits of this tile, combined by the last to arrive (in split order)
  if (S > 1) {
    typedef int v4i __attribute__((ext_vector_type(4)));
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(p.slab, 0, 0x7fffffff, 0x00020000);
    const unsigned so = (unsigned)(((int64_t)tile * S + s) * kKwT * kKwT) * 4u;
#pragma unroll
    for (int q = 0; q < E4; ++q) {
      const v4i w{__float_as_int(v[q].x), __float_as_int(v[q].y), __float_as_int(v[q].z), __float_as_int(v[q].w)};
      __builtin_amdgcn_raw_buffer_store_b128(w, rs, so + (unsigned)(q * NT + tid) * 16u, 0, 16);
    }
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
    for (int q = 0; q < E4; ++q) v[q] = make_float4(0.f, 0.f, 0.f, 0.f);
    bv = 0.f;
    for (int t = 0; t < S; ++t) {
      const unsigned o = (unsigned)(((int64_t)tile * S + t) * kKwT * kKwT) * 4u;
#pragma unroll
      for (int q = 0; q < E4; ++q) {
        const v4i y = __builtin_amdgcn_raw_buffer_load_b128(rs, o + (unsigned)(q * NT + tid) * 16u, 0, 16);
        v[q].x += __int_as_float(y.x);
        v[q].y += __int_as_float(y.y);
        v[q].z += __int_as_float(y.z);
        v[q].w += __int_as_float(y.w);
      }
      if (do_bias && tid < kKwT)
        bv += __hip_atomic_load(p.bslab + ((int64_t)mb * S + t) * kKwT + tid, __ATOMIC_RELAXED,
                                __HIP_MEMORY_SCOPE_AGENT);
    }
    if (tid == 0) __hip_atomic_store(p.cnt + tile, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }

  // ---- store (and Adam)
  if (do_bias && tid < kKwT) p.dst_b[m0 + tid] = bv;
  const bool adam = p.ad.p && p.ad.coef[1] > 0.f;  // (bc2 = 0: a refused step, pinsage_fly_gate_adam)
  const float ss = adam ? p.ad.coef[0] : 0.f, bc2 = adam ? p.ad.coef[1] : 1.f;
  const float omb1 = (float)(1.0 - p.ad.beta1), omb2 = (float)(1.0 - p.ad.beta2);
  const float b2 = (float)p.ad.beta2, eps = p.ad.eps;
  auto adam1 = [&](float& pp, float g, float& mm, float& vv) {
    mm = mm + omb1 * (g - mm);
    vv = vv * b2 + omb2 * g * g;
    const float denom = sqrtf(vv) / bc2 + eps;
    pp = pp - ss * (mm / denom);
  };
#pragma unroll
  for (int q = 0; q < E4; ++q) {
    const int e = 4 * (q * NT + tid);
    const int64_t o = (int64_t)(m0 + e / kKwT) * p.ld_dst + n0 + (e % kKwT);
    *reinterpret_cast<float4*>(p.dst + o) = v[q];
    if (adam) {
      float4 pp = *reinterpret_cast<const float4*>(p.ad.p + o);
      float4 mm = *reinterpret_cast<const float4*>(p.ad.m + o);
      float4 vv = *reinterpret_cast<const float4*>(p.ad.v + o);
      adam1(pp.x, v[q].x, mm.x, vv.x);
      adam1(pp.y, v[q].y, mm.y, vv.y);
      adam1(pp.z, v[q].z, mm.z, vv.z);
      adam1(pp.w, v[q].w, mm.w, vv.w);
      *reinterpret_cast<float4*>(p.ad.p + o) = pp;
      *reinterpret_cast<float4*>(p.ad.m + o) = mm;
      *reinterpret_cast<float4*>(p.ad.v + o) = vv;
    }
  }
  if (adam && do_bias && tid < kKwT && p.ad.pb) adam1(p.ad.pb[m0 + tid], bv, p.ad.mb[m0 + tid], p.ad.vb[m0 + tid]);
}

// NW waves, each with an NS-stage private ring (NW * NS * 8 KiB):
// (8, 2) two waves per SIMD, one stage in flight per wave (128 KiB); (4, 4) one
// wave per SIMD, three stages in flight (128 KiB); (4, 2) one wave per SIMD, one
// stage in flight (64 KiB: the side stream's form, which leaves a CU room for the
// chain's kernels beside it -- a 152-KiB workgroup holds its CU alone).  GATHER: B rows come through the staged row
// numbers (the identity for an ungathered segment), so no DMA branches.
// PROBE (timing diagnostics only, tools/wgrad_bench.py; results are wrong):
// 1 = the DMAs without the products, 2 = the products without the DMAs,
// 3 = 2 without the split (the LDS reads and MFMAs only), 4 = the whole k loop
// without the split
// REG: the k loop without the LDS ring -- every load is one 256-B row of A
// or B (row base in SGPRs: the gathered row numbers are wave-uniform, read by
// scalar loads; lane l takes column l), held in a three-stage register ring
// (two stages in flight while one is multiplied: twice the LDS ring's bytes
// in flight per CU), and one v_permlane32_swap per pair of rows turns the
// row layout into the MFMA operand layout (lanes 0-31: k 0..7, lanes 32-63:
// k 8..15 of the same 32 columns).
template <int NW, int NS, bool GATHER, int PROBE = 0, bool REG = false>
__global__ __launch_bounds__(NW * 64, 8 / NW) void wgrad_kw_kernel(KwParams p) {
  constexpr int kKwRing = NW * NS * kKwStage;  // ring floats
  static_assert(kKwRing >= NW * kKwT * kKwT, "the wave partials reuse the ring");
  constexpr int NT = NW * 64;
  constexpr int E4 = kKwT * kKwT / 4 / NT;  // float4s of the tile per thread
  __shared__ __attribute__((aligned(16))) float smem[kKwRing + kKwWin];
  int* const sidx = reinterpret_cast<int*>(smem + kKwRing);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int h = lane >> 5, l32 = lane & 31;
  const int K = p.K_dev ? *p.K_dev : p.K_max;
  const int tm = p.M / kKwT, tn = p.N / kKwT, S = p.S;
  const int G = tm * tn * S;
  // blocks b and b + 8 share an XCD: with G % 8 == 0 each XCD takes a
  // contiguous run of L, and L runs over the tiles of one split before the
  // next split, so an XCD's workgroups work on ONE split's rows of A and B
  // (or, for S < 8, on 8 / S of its tiles): every A / B row of a split is
  // fetched into one or two XCDs' L2 and re-read there by the tiles that share
  // it.  (Ordered n-block first, the eight m-blocks of a column slice shared an
  // XCD but every XCD read all of A: 4.2x the algorithmic bytes at C2 dQ0,
  // profiles/r06/pmc_c2_q_wgrad.json.)
  const int b = blockIdx.x;
  const int L = (G % 8 == 0) ? (b % 8) * (G / 8) + b / 8 : b;
  const int s = L / (tm * tn), t_ = L - s * tm * tn;
  const int nb = t_ / tm, mb = t_ - nb * tm;
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
  const unsigned ring_w = smem_lds + (unsigned)(wave * NS * kKwStage) * 4u;  // this wave's stages
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

  if constexpr (REG) {
    const int wv = __builtin_amdgcn_readfirstlane(wave);
    const int ns = (ke - kb + kKwBK - 1) / kKwBK;
    const int nw = ns > wv ? (ns - wv + NW - 1) / NW : 0;
    float ra[3][16], rb[3][16];
    // Every stage loads and multiplies unconditionally (the row numbers clamp
    // to the split's last row and rows past it are zeroed in A), so the
    // loop has no branches for the wait-count pass to merge: a stage waits
    // for its own 32 loads only, with the next two stages still in flight.
    const int nw3 = (nw + 2) / 3 * 3;
    const int32_t* bix = GATHER ? bidx : nullptr;
    auto load = [&](int it, float (&xa)[16], float (&xb)[16]) __attribute__((always_inline)) {
      const int k0 = kb + kKwBK * (wv + NW * it);
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const int k = min(k0 + j, ke - 1);
        const float* ar = p.A + (int64_t)k * p.lda + m0;
        xa[j] = ar[lane];
      }
      if (bix) {
#pragma unroll
        for (int j = 0; j < 16; ++j) {
          const int k = min(k0 + j, ke - 1);
          xb[j] = (Bp + (int64_t)bix[k] * ldb + bc0)[lane];
        }
      } else {
#pragma unroll
        for (int j = 0; j < 16; ++j) {
          const int k = min(k0 + j, ke - 1);
          xb[j] = (Bp + (int64_t)k * ldb + bc0)[lane];
        }
      }
    };
    auto compute = [&](int it, float (&xa)[16], float (&xb)[16]) __attribute__((always_inline)) {
      const int k0 = kb + kKwBK * (wv + NW * it);
#pragma unroll
      for (int j = 0; j < 16; ++j) xa[j] = k0 + j < ke ? xa[j] : 0.f;  // rows past the split's end
      if (do_bias) {
#pragma unroll
        for (int j = 0; j < 16; ++j) bsum += xa[j];
      }
      float fa[2][8], fb[2][8];
#pragma unroll
      for (int jj = 0; jj < 8; ++jj) {
        const auto ya = __builtin_amdgcn_permlane32_swap(__float_as_int(xa[jj]), __float_as_int(xa[8 + jj]), false,
                                                         false);
        fa[0][jj] = __int_as_float(ya[0]);
        fa[1][jj] = __int_as_float(ya[1]);
        const auto yb = __builtin_amdgcn_permlane32_swap(__float_as_int(xb[jj]), __float_as_int(xb[8 + jj]), false,
                                                         false);
        fb[0][jj] = __int_as_float(yb[0]);
        fb[1][jj] = __int_as_float(yb[1]);
      }
      bf16x8 aH[2], aM[2], aL[2], bH[2], bM[2], bL[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        split3(make_float4(fa[i][0], fa[i][1], fa[i][2], fa[i][3]), make_float4(fa[i][4], fa[i][5], fa[i][6], fa[i][7]),
               aH[i], aM[i], aL[i]);
        split3(make_float4(fb[i][0], fb[i][1], fb[i][2], fb[i][3]), make_float4(fb[i][4], fb[i][5], fb[i][6], fb[i][7]),
               bH[i], bM[i], bL[i]);
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
    };
    if (nw > 0) {
      load(0, ra[0], rb[0]);
      load(1, ra[1], rb[1]);
      for (int it = 0; it < nw3; it += 3) {
#pragma unroll
        for (int q = 0; q < 3; ++q) {
          load(it + q + 2, ra[(q + 2) % 3], rb[(q + 2) % 3]);
          compute(it + q, ra[q], rb[q]);
        }
      }
    }
    __syncthreads();  // (the epilogue's LDS)
  } else
  for (int pb = kb; pb < ke; pb += kKwWin) {
    const int pe = min(ke, pb + kKwWin);
    if constexpr (GATHER) {
      for (int i = tid; i < pe - pb; i += NT) sidx[i] = bidx ? bidx[pb + i] : pb + i;
      __syncthreads();
    }
    const int ns = (pe - pb + kKwBK - 1) / kKwBK;  // stages of this pass
    const int nw = ns > wave ? (ns - wave + NW - 1) / NW : 0;  // this wave's
    // stage it of this wave: rows pb + 16 (wave + NW it) ..; the gathered row
    // numbers of the next stage to issue are read from LDS one iteration early
    // (into `nxt`), so issuing a stage waits on no LDS round trip
    int nxt[4];
    auto fetch_rows = [&](int it) __attribute__((always_inline)) {
      const int k0 = pb + kKwBK * (wave + NW * it);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int k = min(k0 + 4 * j + dr, pe - 1);
        nxt[j] = GATHER ? sidx[k - pb] : k;
      }
    };
    auto issue = [&](int it) __attribute__((always_inline)) {
      if constexpr (PROBE == 2 || PROBE == 3) return;
      const int k0 = pb + kKwBK * (wave + NW * it);
      const unsigned img = ring_w + (unsigned)((it % NS) * kKwStage) * 4u;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int k = min(k0 + 4 * j + dr, pe - 1);
        glds16(p.A + (int64_t)k * p.lda + m0 + dc, img + (unsigned)j * 1024u);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j)
        glds16(Bp + (int64_t)nxt[j] * ldb + bc0 + dc, img + (unsigned)(kKwImg * 4 + j * 1024));
    };
    for (int st = 0; st < NS - 1 && st < nw; ++st) {
      fetch_rows(st);
      issue(st);
    }
    if (NS - 1 < nw) fetch_rows(NS - 1);
    for (int it = 0; it < nw; ++it) {
      // stage it has landed (the younger ones stay in flight); stage it+NS-1
      // goes out into the slot this wave read one iteration ago
      wait_stage<8, NS - 2 >= 1 ? NS - 2 : 1>(min(NS - 2, nw - 1 - it));
      if (it + NS - 1 < nw) {
        issue(it + NS - 1);
        if (it + NS < nw) fetch_rows(it + NS);
      }
      float* const As = smem + wave * NS * kKwStage + (it % NS) * kKwStage;
      const float* const Bs = As + kKwImg;
      const int k0 = pb + kKwBK * (wave + NW * it);
      if (k0 + kKwBK > pe) {  // k-tail: A rows past the pass end contribute nothing
        for (int r = pe - k0; r < kKwBK; ++r) As[r * kKwT + lane] = 0.f;
      }
      if (do_bias) {
#pragma unroll
        for (int r = 0; r < kKwBK; ++r) bsum += As[r * kKwT + lane];
      }
      if constexpr (PROBE == 1) continue;
      // 16 k: lane (col l32, half h) holds k = 8 h .. 8 h + 7 of each fragment
      bf16x8 aH[2], aM[2], aL[2], bH[2], bM[2], bL[2];
      if constexpr (PROBE >= 3) {  // the operands' bits as bf16, unsplit (timing only)
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const float4 a0 = kw_frag(As, i * 32 + l32, 8 * h), a1 = kw_frag(As, i * 32 + l32, 8 * h + 4);
          const float4 b0 = kw_frag(Bs, i * 32 + l32, 8 * h), b1 = kw_frag(Bs, i * 32 + l32, 8 * h + 4);
          aH[i] = aM[i] = aL[i] = __builtin_bit_cast(bf16x8, make_float4(a0.x + a1.x, a0.y + a1.y, a0.z + a1.z, a0.w + a1.w));
          bH[i] = bM[i] = bL[i] = __builtin_bit_cast(bf16x8, make_float4(b0.x + b1.x, b0.y + b1.y, b0.z + b1.z, b0.w + b1.w));
        }
      } else
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
      // the next issue's row numbers are in registers by now (read at the top
      // of this iteration): pinning them here keeps the compiler from sinking
      // the LDS reads down to the DMAs that use them
#pragma unroll
      for (int j = 0; j < 4; ++j) asm volatile("" : "+v"(nxt[j]));
    }
    __syncthreads();  // (the next pass rewrites sidx; the epilogue reuses the ring)
  }

  kw_finish<NW>(p, acc, bsum, smem, kKwRing, tile, mb, s, m0, n0, do_bias);
}

// ---------------------------------------------------------------- pre-split operands
// The same long-K weight gradient with both operands already split into hi /
// mid / lo bf16 planes (the layer-0 Q weight gradient: dpq planes written by
// the transposed aggregation, the feature table's planes made once): the k
// loop does no conversions (the split was 16 of the fp32 form's 54 us at C2,
// tools/wgrad_bench.py PROBE 4).  A stage is 16 k-rows x 64 columns of each of
// the six planes (12 KiB); 4 waves x 3-stage rings (two stages in flight per
// wave, as the fp32 form's two waves per SIMD with one each).  The DMA is
// lane-linear (1 KiB = 8 rows of 128 B per instruction), so a row's 16-B
// chunks are stored XOR-swizzled (chunk c of row R at c ^ 4 ((R >> 1) & 1)),
// which makes the ds_read_b64_tr_b16 operand reads bank-conflict free: a
// 32-lane half reads rows R..R+3, chunks 0..3 -> banks 32 R + 4 c' without
// repeats.  Each tr read gives a lane 4 k-rows of its column; two give the
// 8-k half of a 32 x 32 x 16 operand fragment, in the k order the fp32 form
// splits, so the products -- and with the same wave count the sums -- equal
// the fp32 form's (4, NS) launch bit for bit.  The bias sums (H + M) + L, the
// planes' value (within 2^-24 of the fp32 row).
typedef short kw_s4 __attribute__((ext_vector_type(4)));
constexpr int kPlImg = kKwBK * kKwT * 2;  // bytes per plane image (2 KiB)
constexpr int kPlStage = 6 * kPlImg;      // A and B, three planes each (12 KiB)
constexpr int kPlWin = 2048;              // gathered row numbers staged per pass (8 KiB)

__device__ __forceinline__ bf16x8 kw_tr_frag(unsigned lds_lo, unsigned lds_hi) {
  const kw_s4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) kw_s4*)(size_t)lds_lo);
  const kw_s4 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) kw_s4*)(size_t)lds_hi);
  typedef short s8 __attribute__((ext_vector_type(8)));
  const s8 v{a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
  return __builtin_bit_cast(bf16x8, v);
}

template <int NW, int NS, bool GATHER>
__global__ __launch_bounds__(NW * 64, 1) void wgrad_pl_kernel(KwParams p) {
  constexpr int kRing = NW * NS * kPlStage / 4;  // ring floats
  static_assert(kRing >= NW * kKwT * kKwT, "the wave partials reuse the ring");
  constexpr int NT = NW * 64;
  __shared__ __attribute__((aligned(16))) float smem[kRing + kPlWin];
  int* const sidx = reinterpret_cast<int*>(smem + kRing);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int K = p.K_dev ? *p.K_dev : p.K_max;
  const int tm = p.M / kKwT, tn = p.N / kKwT, S = p.S;
  const int G = tm * tn * S;
  const int b = blockIdx.x;  // (the split-major XCD placement of wgrad_kw_kernel)
  const int L = (G % 8 == 0) ? (b % 8) * (G / 8) + b / 8 : b;
  const int s = L / (tm * tn), t_ = L - s * tm * tn;
  const int nb = t_ / tm, mb = t_ - nb * tm;
  const int m0 = mb * kKwT, n0 = nb * kKwT;
  const int tile = nb * tm + mb;
  const int kc = ((K + S - 1) / S + kKwBK - 1) / kKwBK * kKwBK;
  const int kb = min(K, s * kc), ke = min(K, kb + kc);
  const bool do_bias = p.dst_b && nb == 0;
  const unsigned smem_lds = (unsigned)(size_t)((__attribute__((address_space(3))) float*)smem);
  const unsigned ring_w = smem_lds + (unsigned)(wave * NS * kPlStage);
  char* const ring_g = reinterpret_cast<char*>(smem) + wave * NS * kPlStage;
  // DMA: lane -> row 8 j + dR of the stage, physical chunk lane & 7 (logical dcol / 8)
  const int dR = lane >> 3;
  const int dcol = 8 * ((lane & 7) ^ (4 * ((dR >> 1) & 1)));
  // tr reads: lane (group g, row q, quad pp) addresses row kq + 4 t + q, columns
  // 32 i + mq + 4 pp; the byte offsets within a plane image for t, i
  unsigned toff[2][2];
  {
    const int g = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3;
    const int kq = 8 * (g >> 1), mq = 16 * (g & 1) + 4 * pp;
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int R = kq + 4 * t + q, col = 32 * i + mq;
        toff[t][i] = (unsigned)(R * 128 + (((col >> 3) ^ (4 * ((R >> 1) & 1))) << 4) + ((col & 7) << 1));
      }
  }
  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  float bs2[2] = {0.f, 0.f};  // bias partials of columns 32 i + (lane & 31), k half lane >> 5

  for (int pb = kb; pb < ke; pb += kPlWin) {
    const int pe = min(ke, pb + kPlWin);
    if constexpr (GATHER) {
      for (int i = tid; i < pe - pb; i += NT) sidx[i] = p.b_idx[pb + i];
      __syncthreads();
    }
    const int ns = (pe - pb + kKwBK - 1) / kKwBK;
    const int nw = ns > wave ? (ns - wave + NW - 1) / NW : 0;
    int nxt[2];
    auto fetch_rows = [&](int it) __attribute__((always_inline)) {
      const int k0 = pb + kKwBK * (wave + NW * it);
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int k = min(k0 + 8 * j + dR, pe - 1);
        nxt[j] = GATHER ? sidx[k - pb] : k;
      }
    };
    auto issue = [&](int it) __attribute__((always_inline)) {
      const int k0 = pb + kKwBK * (wave + NW * it);
      const unsigned img = ring_w + (unsigned)((it % NS) * kPlStage);
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int k = min(k0 + 8 * j + dR, pe - 1);
#pragma unroll
        for (int P = 0; P < 3; ++P)
          glds16(reinterpret_cast<const float*>(p.A3 + P * p.a3_ps + (int64_t)k * p.lda + m0 + dcol),
                 img + (unsigned)(P * kPlImg + j * 1024));
      }
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int P = 0; P < 3; ++P)
          glds16(reinterpret_cast<const float*>(p.B3 + P * p.b3_ps + (int64_t)nxt[j] * p.ldb + n0 + dcol),
                 img + (unsigned)((3 + P) * kPlImg + j * 1024));
    };
    for (int st = 0; st < NS - 1 && st < nw; ++st) {
      fetch_rows(st);
      issue(st);
    }
    if (NS - 1 < nw) fetch_rows(NS - 1);
    for (int it = 0; it < nw; ++it) {
      wait_stage<12, NS - 2 >= 1 ? NS - 2 : 1>(min(NS - 2, nw - 1 - it));
      if (it + NS - 1 < nw) {
        issue(it + NS - 1);
        if (it + NS < nw) fetch_rows(it + NS);
      }
      const unsigned stg = ring_w + (unsigned)((it % NS) * kPlStage);
      const int k0 = pb + kKwBK * (wave + NW * it);
      if (k0 + kKwBK > pe) {  // k-tail: A rows past the pass end contribute nothing
        char* const sg = ring_g + (it % NS) * kPlStage;
        for (int r = pe - k0; r < kKwBK; ++r)
#pragma unroll
          for (int P = 0; P < 3; ++P) reinterpret_cast<uint16_t*>(sg + P * kPlImg + r * 128)[lane] = 0;
      }
      bf16x8 aX[3][2], bX[3][2];
#pragma unroll
      for (int P = 0; P < 3; ++P)
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          aX[P][i] = kw_tr_frag(stg + P * kPlImg + toff[0][i], stg + P * kPlImg + toff[1][i]);
          bX[P][i] = kw_tr_frag(stg + (3 + P) * kPlImg + toff[0][i], stg + (3 + P) * kPlImg + toff[1][i]);
        }
      if (do_bias) {
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int e = 0; e < 8; ++e)
            bs2[i] += ((float)aX[0][i][e] + (float)aX[1][i][e]) + (float)aX[2][i][e];
      }
#define PS_PL_ALL(X, Y)                                                                            \
  _Pragma("unroll") for (int i = 0; i < 2; ++i) _Pragma("unroll") for (int j = 0; j < 2; ++j) \
      acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(aX[X][i], bX[Y][j], acc[i][j], 0, 0, 0);
      PS_PL_ALL(2, 0)  // (the fp32 form's order: lo hi, hi lo, mid mid, mid hi, hi mid, hi hi)
      PS_PL_ALL(0, 2)
      PS_PL_ALL(1, 1)
      PS_PL_ALL(1, 0)
      PS_PL_ALL(0, 1)
      PS_PL_ALL(0, 0)
#undef PS_PL_ALL
#pragma unroll
      for (int j = 0; j < 2; ++j) asm volatile("" : "+v"(nxt[j]));
    }
    __syncthreads();
  }
  // bias partials to the fp32 form's layout: lane l holds column l
  const float v0 = bs2[0] + __shfl_xor(bs2[0], 32, 64), v1 = bs2[1] + __shfl_xor(bs2[1], 32, 64);
  const float bsum = lane < 32 ? v0 : v1;
  kw_finish<NW>(p, acc, bsum, smem, kRing, tile, mb, s, m0, n0, do_bias);
}

// ---------------------------------------------------------------- host side
bool wgrad_kw_supported(int M, int N, int N1, bool has_b2) {
  return M > 0 && N > 0 && M % kKwT == 0 && N % kKwT == 0 && (!has_b2 || (N1 >= 0 && N1 % kKwT == 0));
}

int wgrad_kw_splits(int M, int N, int64_t K_est, int target) {
  const int tiles = (M / kKwT) * (N / kKwT);
  int S = std::max(1, (std::max(1, target) + tiles - 1) / tiles);
  S = std::min<int64_t>(S, std::max<int64_t>(1, K_est / 256));  // >= 256 rows (16 stages) per split
  S = std::min(S, kKwMaxSplits);
  while (S > 1 && (tiles * S) % 8 != 0 && tiles * S > 8) --S;  // (XCD-aware placement)
  return S;
}

int64_t wgrad_kw_slab_floats(int M, int N) { return (int64_t)kKwMaxSplits * M * N; }
int64_t wgrad_kw_bslab_floats(int M) { return (int64_t)kKwMaxSplits * M; }
int64_t wgrad_kw_tickets(int M, int N) { return (int64_t)(M / kKwT) * (N / kKwT); }

// probe: 0, or a timing-only build of the k loop (1-4, PROBE above: the
// results are WRONG; only pinsage_wgrad_probe, a measurement entry, passes one)
int launch_wgrad_kw_probe(const KwParams& p_in, int probe, hipStream_t st);
int launch_wgrad_kw(const KwParams& p_in, hipStream_t st) { return launch_wgrad_kw_probe(p_in, 0, st); }

int launch_wgrad_kw_probe(const KwParams& p_in, int probe, hipStream_t st) {
  KwParams p = p_in;
  PS_REQUIRE(wgrad_kw_supported(p.M, p.N, p.N1, p.B2 != nullptr), kErrArg,
             "wgrad: M, N (and N1) must be multiples of 64");
  PS_REQUIRE((p.A || p.A3) && (p.B || p.B3) && p.dst && p.lda % 4 == 0 && p.ldb % 4 == 0 && (!p.B2 || p.ldb2 % 4 == 0) &&
                 p.ld_dst % 4 == 0 && p.K_max >= 0,
             kErrArg, "wgrad: operands and 16-B aligned row strides");
  PS_REQUIRE(!p.ad.p || (p.ad.m && p.ad.v && p.ad.coef && (!p.dst_b || (p.ad.pb && p.ad.mb && p.ad.vb))),
             kErrArg, "wgrad: incomplete Adam slice");
  if (p.S <= 0) p.S = wgrad_kw_splits(p.M, p.N, p.K_max, 256);
  p.S = std::min(p.S, kKwMaxSplits);
  PS_REQUIRE(p.S == 1 || (p.slab && p.cnt && (!p.dst_b || p.bslab)), kErrArg, "wgrad: split scratch not set");
  const int grid = (p.M / kKwT) * (p.N / kKwT) * p.S;
  // PINSAGE_KW_WAVES: 8 (default: 8 waves x 2-stage rings) or 4 (4 x 4)
  const int waves = getenv("PINSAGE_KW_WAVES") ? atoi(getenv("PINSAGE_KW_WAVES")) : 8;  // (per call: A/B)
  const bool gather = p.b_idx || p.b2_idx;
  if (p.A3 || p.B3) {  // pre-split operands
    PS_REQUIRE(p.A3 && p.B3 && !p.B2 && p.lda % 8 == 0 && p.ldb % 8 == 0, kErrArg,
               "wgrad: pre-split A and B planes (no B2 segment), row strides multiples of 8");
    if (p.b_idx) hipLaunchKernelGGL((wgrad_pl_kernel<4, 3, true>), dim3(grid), dim3(256), 0, st, p);
    else hipLaunchKernelGGL((wgrad_pl_kernel<4, 3, false>), dim3(grid), dim3(256), 0, st, p);
    PS_CHECK_LAUNCH();
    return kOk;
  }
  // PINSAGE_KW_FORM (tests / microbenchmarks through the C-ABI): the form of a
  // launch whose caller did not choose one
  if (p.form == 0 && getenv("PINSAGE_KW_FORM")) p.form = atoi(getenv("PINSAGE_KW_FORM"));
  if (waves == 1) {  // PINSAGE_KW_WAVES=1: the register-ring k loop (REG), 8 waves
    if (gather) hipLaunchKernelGGL((wgrad_kw_kernel<8, 2, true, 0, true>), dim3(grid), dim3(512), 0, st, p);
    else hipLaunchKernelGGL((wgrad_kw_kernel<8, 2, false, 0, true>), dim3(grid), dim3(512), 0, st, p);
  } else if (probe >= 1 && probe <= 4) {  // timing diagnostics (pinsage_wgrad_probe): wrong results
    if (probe == 1) hipLaunchKernelGGL((wgrad_kw_kernel<8, 2, true, 1>), dim3(grid), dim3(512), 0, st, p);
    else if (probe == 2) hipLaunchKernelGGL((wgrad_kw_kernel<8, 2, true, 2>), dim3(grid), dim3(512), 0, st, p);
    else if (probe == 3) hipLaunchKernelGGL((wgrad_kw_kernel<8, 2, true, 3>), dim3(grid), dim3(512), 0, st, p);
    else hipLaunchKernelGGL((wgrad_kw_kernel<8, 2, true, 4>), dim3(grid), dim3(512), 0, st, p);
  } else if (p.form == 1) {  // 4 waves x 2 stages: 64-KiB ring
    if (gather) hipLaunchKernelGGL((wgrad_kw_kernel<4, 2, true>), dim3(grid), dim3(256), 0, st, p);
    else hipLaunchKernelGGL((wgrad_kw_kernel<4, 2, false>), dim3(grid), dim3(256), 0, st, p);
  } else if (waves == 4) {
    if (gather) hipLaunchKernelGGL((wgrad_kw_kernel<4, 4, true>), dim3(grid), dim3(256), 0, st, p);
    else hipLaunchKernelGGL((wgrad_kw_kernel<4, 4, false>), dim3(grid), dim3(256), 0, st, p);
  } else {
    if (gather) hipLaunchKernelGGL((wgrad_kw_kernel<8, 2, true>), dim3(grid), dim3(512), 0, st, p);
    else hipLaunchKernelGGL((wgrad_kw_kernel<8, 2, false>), dim3(grid), dim3(512), 0, st, p);
  }
  PS_CHECK_LAUNCH();
  return kOk;
}

}  // namespace ps
