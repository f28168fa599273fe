// fp32 MFMA GEMM (v_mfma_f32_32x32x2_f32: exact fp32 FMA chain, 64 FLOP/clk/SIMD
// on gfx950; there is no xf32 path, and the reference computes in fp32).
//
// Block tile 128x128x16, 256 threads = 4 waves in 2x2, each wave 64x64 =
// 2x2 MFMA tiles of 32x32 (64 accumulator registers).  Operand tiles are staged
// global -> registers -> LDS (double-buffered, one barrier per k-tile) in a
// k-major [BK][128+4] image whatever the global layout, so every MFMA operand
// fragment is one conflict-free ds_read_b32 (lanes 0-31: 32 consecutive rows of
// one k; lanes 32-63: the next k).  Persistent grid: tiles are dealt so that
// the column tiles of one row panel (or the tiles of one split-K slice) share
// an XCD's L2 (blocks b and b+8 land on one XCD).
#include "gemm.h"

#include <algorithm>

namespace ps {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int PADF = 4;  // LDS row padding (floats): conflict-free b32 fragment reads, 16-B aligned rows

// Rows of a K-major operand ([row][k] in memory) handled by this thread.
template <int NV>
struct KRows {
  const float* p[NV];
  const float* p2[NV];
};

template <int R, int BK>
struct Shape {
  static constexpr int KV = BK / 4;               // float4 per row per stage (K-major)
  static constexpr int TOT_K = R * KV;            // float4 per stage, K-major
  static constexpr int MV = R / 4;                // float4 per k-row (MN-major)
  static constexpr int TOT_MN = BK * MV;          // float4 per stage, MN-major
  static constexpr int NV = (TOT_K + 255) / 256;  // float4 per thread (same count both layouts)
  static constexpr int W = R + PADF;              // MN-major image: [BK][R + 4]
  static constexpr int WK = BK + 4;               // K-major image:  [R][BK + 4]
  static constexpr int SZ = (R * WK > BK * W) ? R * WK : BK * W;  // floats per stage
};

template <int R, int BK>
__device__ __forceinline__ void kmajor_rows(KRows<(Shape<R, BK>::NV)>& Rw, int tid, int r0, int rmax,
                                            const float* a, int64_t lda, const int32_t* idx,
                                            const float* a2, int64_t lda2, const int32_t* idx2) {
  using S = Shape<R, BK>;
#pragma unroll
  for (int i = 0; i < S::NV; ++i) {
    const int lin = tid + 256 * i;
    const int row = r0 + lin / S::KV;
    Rw.p[i] = nullptr;
    Rw.p2[i] = nullptr;
    if (lin < S::TOT_K && row < rmax) {
      const int64_t r = idx ? idx[row] : row;
      Rw.p[i] = a + r * lda;
      if (a2) {
        const int64_t r2 = idx2 ? idx2[row] : row;
        Rw.p2[i] = a2 + r2 * lda2;
      }
    }
  }
}

// K-major operand stage -> registers.  Each float4 chunk picks its K segment
// on its own (torch.cat along K without a concat buffer), so K1 % 4 == 0 suffices.
template <int R, int BK>
__device__ __forceinline__ void kmajor_load(float4 (&v)[(Shape<R, BK>::NV)],
                                            const KRows<(Shape<R, BK>::NV)>& Rw, int tid, int k0,
                                            int kend, int K1) {
  using S = Shape<R, BK>;
#pragma unroll
  for (int i = 0; i < S::NV; ++i) {
    const int lin = tid + 256 * i;
    const int k = k0 + (lin % S::KV) * 4;
    const bool seg2 = K1 >= 0 && k >= K1;
    const float* base = seg2 ? Rw.p2[i] : Rw.p[i];
    if (Rw.p[i] && k < kend) v[i] = *reinterpret_cast<const float4*>(base + (seg2 ? k - K1 : k));
    else v[i] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
}
// K-major stage image is row-major [R][BK+4]: one ds_write_b128 per float4, and
// the fragment reader takes 4 consecutive k of a row with one ds_read_b128.
template <int R, int BK>
__device__ __forceinline__ void kmajor_store(float* Sm, const float4 (&v)[(Shape<R, BK>::NV)],
                                             int tid) {
  using S = Shape<R, BK>;
#pragma unroll
  for (int i = 0; i < S::NV; ++i) {
    const int lin = tid + 256 * i;
    if (lin >= S::TOT_K) continue;
    const int row = lin / S::KV, kc = (lin % S::KV) * 4;
    *reinterpret_cast<float4*>(Sm + row * S::WK + kc) = v[i];
  }
}

// MN-major operand ([k][col] in memory, k rows optionally gathered); columns
// >= c1 (if c1 >= 0) come from a second matrix a2 (torch.cat along columns)
template <int R, int BK>
__device__ __forceinline__ void mnmajor_load(float4 (&v)[(Shape<R, BK>::NV)], int tid, const float* a,
                                             int64_t lda, const int32_t* idx, int c0, int cmax,
                                             int k0, int kend, int c1 = -1,
                                             const float* a2 = nullptr, int64_t lda2 = 0,
                                             const int32_t* idx2 = nullptr) {
  using S = Shape<R, BK>;
#pragma unroll
  for (int i = 0; i < S::NV; ++i) {
    const int lin = tid + 256 * i;
    const int kr = lin / S::MV, cc = lin % S::MV;
    const int k = k0 + kr;
    const int c = c0 + cc * 4;
    if (lin < S::TOT_MN && k < kend && c < cmax) {
      if (a2 && c >= c1) {
        const int64_t r = idx2 ? idx2[k] : k;
        v[i] = *reinterpret_cast<const float4*>(a2 + r * lda2 + (c - c1));
      } else {
        const int64_t r = idx ? idx[k] : k;
        v[i] = *reinterpret_cast<const float4*>(a + r * lda + c);
      }
    } else {
      v[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
}
template <int R, int BK>
__device__ __forceinline__ void mnmajor_store(float* Sm, const float4 (&v)[(Shape<R, BK>::NV)],
                                              int tid) {
  using S = Shape<R, BK>;
#pragma unroll
  for (int i = 0; i < S::NV; ++i) {
    const int lin = tid + 256 * i;
    if (lin >= S::TOT_MN) continue;
    const int kr = lin / S::MV, cc = lin % S::MV;
    *reinterpret_cast<float4*>(Sm + kr * S::W + cc * 4) = v[i];
  }
}

// 4 consecutive k (8s + 4h .. +3) of row `row` from a staged image
template <bool KM, int R, int BK>
__device__ __forceinline__ float4 frag4(const float* Sm, int row, int k4) {
  using S = Shape<R, BK>;
  if (KM) return *reinterpret_cast<const float4*>(Sm + row * S::WK + k4);
  return make_float4(Sm[(k4 + 0) * S::W + row], Sm[(k4 + 1) * S::W + row],
                     Sm[(k4 + 2) * S::W + row], Sm[(k4 + 3) * S::W + row]);
}

// WM x WN waves, each TM x TN MFMA tiles of 32x32; stage depth BK.
template <bool AK, bool BKM, int WM, int WN, int TM, int TN, int BK>
__global__ __launch_bounds__(256, 2) void gemm_f32_kernel(GemmParams p) {
  constexpr int BM = WM * TM * 32, BN = WN * TN * 32;
  using SA = Shape<BM, BK>;
  using SB = Shape<BN, BK>;
  __shared__ __attribute__((aligned(16))) float As[2][SA::SZ];
  __shared__ __attribute__((aligned(16))) float Bs[2][SB::SZ];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int M = p.M_dev ? *p.M_dev : p.M;
  const int K = p.K_dev ? *p.K_dev : p.K;
  const int N = p.N;
  const int tiles_m = (M + BM - 1) / BM, tiles_n = (N + BN - 1) / BN;
  const int splits = p.epi == kEpiPartial ? p.splits : 1;
  const int kchunk = (((K + splits - 1) / splits) + BK - 1) / BK * BK;
  int G, W;
  if (splits > 1) {
    G = splits;
    W = tiles_m * tiles_n;
  } else {
    G = tiles_m;
    W = tiles_n;
  }
  // tiles of one row panel (or one split) are dealt to blocks b, b+8, ...:
  // one XCD under round-robin placement, so they share its L2 (speed only)
  const int iters = 8 * ((G + 7) / 8) * W;
  for (int t = blockIdx.x; t < iters; t += gridDim.x) {
    const int xcd = t & 7, s = t >> 3;
    const int g = (s / W) * 8 + xcd, w = s % W;
    if (g >= G) continue;
    int split, tm, tn;
    if (splits > 1) {
      split = g;
      tm = w / tiles_n;
      tn = w % tiles_n;
    } else {
      split = 0;
      tm = g;
      tn = w;
    }
    const int m0 = tm * BM, n0 = tn * BN;
    const int kb = split * kchunk;
    const int ke = min(K, kb + kchunk);
    const int nk = ke > kb ? (ke - kb + BK - 1) / BK : 0;

    KRows<SA::NV> RA;
    KRows<SB::NV> RB;
    if (AK) kmajor_rows<BM, BK>(RA, tid, m0, M, p.a, p.lda, p.a_idx, p.a2, p.lda2, p.a2_idx);
    if (BKM) kmajor_rows<BN, BK>(RB, tid, n0, N, p.b, p.ldb, nullptr, nullptr, 0, nullptr);

    f32x16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    // Two register stages: the global loads of tile t+2 are issued before the
    // MFMAs of tile t and written to LDS after those of tile t+1, so two k-tiles
    // of MFMA work cover the HBM latency of the (row-gathered) operand loads.
    float4 va0[SA::NV], vb0[SB::NV], va1[SA::NV], vb1[SB::NV];
    auto load = [&](float4 (&va)[SA::NV], float4 (&vb)[SB::NV], int k0) {
      if (AK) kmajor_load<BM, BK>(va, RA, tid, k0, ke, p.K1);
      else mnmajor_load<BM, BK>(va, tid, p.a, p.lda, p.a_idx, m0, M, k0, ke);
      if (BKM) kmajor_load<BN, BK>(vb, RB, tid, k0, ke, -1);
      else mnmajor_load<BN, BK>(vb, tid, p.b, p.ldb, p.b_idx, n0, N, k0, ke, p.N1, p.b2, p.ldb2,
                                p.b2_idx);
    };
    auto store = [&](const float4 (&va)[SA::NV], const float4 (&vb)[SB::NV], int buf) {
      if (AK) kmajor_store<BM, BK>(As[buf], va, tid);
      else mnmajor_store<BM, BK>(As[buf], va, tid);
      if (BKM) kmajor_store<BN, BK>(Bs[buf], vb, tid);
      else mnmajor_store<BN, BK>(Bs[buf], vb, tid);
    };
    const int h = lane >> 5, l32 = lane & 31;
    const bool do_bias = !AK && p.bias_part && tn == 0 && tid < BM;
    float bsum = 0.f;
    // MFMA k-assignment: in the r-th MFMA of octet s, lane half h supplies
    // k = 8s + 4h + r for both operands (any bijection onto the 8 k works).
    auto compute = [&](int cur) {
      if (do_bias) {  // column sums of A^T over this tile's k rows (zero-padded)
#pragma unroll
        for (int k = 0; k < BK; ++k) bsum += As[cur][k * SA::W + tid];
      }
#pragma unroll
      for (int s8 = 0; s8 < BK / 8; ++s8) {
        const int k4 = 8 * s8 + 4 * h;
        float4 a[TM], b[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i) a[i] = frag4<AK, BM, BK>(As[cur], (wm * TM + i) * 32 + l32, k4);
#pragma unroll
        for (int j = 0; j < TN; ++j) b[j] = frag4<BKM, BN, BK>(Bs[cur], (wn * TN + j) * 32 + l32, k4);
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i].x, b[j].x, acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i].y, b[j].y, acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i].z, b[j].z, acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i].w, b[j].w, acc[i][j], 0, 0, 0);
          }
      }
    };
    if (nk > 0) {
      load(va0, vb0, kb);
      store(va0, vb0, 0);
    }
    if (nk > 1) load(va1, vb1, kb + BK);
    __syncthreads();
    for (int it = 0; it < nk; it += 2) {
      if (it + 2 < nk) load(va0, vb0, kb + (it + 2) * BK);
      compute(0);
      if (it + 1 < nk) store(va1, vb1, 1);
      __syncthreads();
      if (it + 1 >= nk) break;
      if (it + 3 < nk) load(va1, vb1, kb + (it + 3) * BK);
      compute(1);
      if (it + 2 < nk) store(va0, vb0, 0);
      __syncthreads();
    }

    // ------------------------------------------------------------ epilogue
    // acc[i][j][r] -> row m0 + (wm*TM+i)*32 + (r&3) + 8*(r>>2) + 4*h, col n0 + (wn*TN+j)*32 + l32
    if (p.epi == kEpiPartial) {
      if (do_bias && m0 + tid < M) p.bias_part[(int64_t)split * M + m0 + tid] = bsum;
      float* C = p.c + (int64_t)split * M * p.ldc;
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = m0 + (wm * TM + i) * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
          if (row >= M) continue;
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            const int col = n0 + (wn * TN + j) * 32 + l32;
            if (col < N) C[(int64_t)row * p.ldc + col] = acc[i][j][r];
          }
        }
    } else if (p.epi == kEpiL2Norm) {
      float* red = &As[0][0];  // [WN][BM] row partial sums (LDS free after the k loop)
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          float s2 = 0.f;
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            const int col = n0 + (wn * TN + j) * 32 + l32;
            float v = acc[i][j][r] + (p.bias && col < N ? p.bias[col] : 0.f);
            v = lrelu(v);
            if (col >= N) v = 0.f;
            acc[i][j][r] = v;
            s2 += v * v;
          }
#pragma unroll
          for (int o = 1; o < 32; o <<= 1) s2 += __shfl_xor(s2, o, 64);
          if (l32 == 0) red[wn * BM + (wm * TM + i) * 32 + (r & 3) + 8 * (r >> 2) + 4 * h] = s2;
        }
      __syncthreads();
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int lrow = (wm * TM + i) * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
          const int row = m0 + lrow;
          if (row >= M) continue;
          float tot = 0.f;
#pragma unroll
          for (int q = 0; q < WN; ++q) tot += red[q * BM + lrow];
          const float nrm = sqrtf(tot);
          const int64_t dst = p.c_idx ? p.c_idx[row] : row;
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            const int col = n0 + (wn * TN + j) * 32 + l32;
            if (col < N) p.c[dst * p.ldc + col] = acc[i][j][r] / nrm;
          }
          if (p.norms && wn == 0 && l32 == 0) p.norms[row] = nrm;
        }
    } else {
      const bool accum = p.epi == kEpiAccum;
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = m0 + (wm * TM + i) * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
          if (row >= M) continue;
          const int64_t dst = p.c_idx ? p.c_idx[row] : row;
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            const int col = n0 + (wn * TN + j) * 32 + l32;
            if (col >= N) continue;
            float v = acc[i][j][r];
            if (p.bias) v += p.bias[col];
            if (p.act) v = lrelu(v);
            if (p.mask) v *= lrelu_grad(p.mask[(int64_t)row * p.ldm + col]);
            if (p.c2 && col >= p.N1) {
              p.c2[(int64_t)row * p.ldc2 + (col - p.N1)] = v;
            } else {
              float* o = p.c + dst * p.ldc + col;
              *o = accum ? *o + v : v;
            }
          }
        }
    }
    __syncthreads();
  }
}

constexpr int kCfgBM[3] = {128, 64, 32};

// Cost model: tiles are dealt round-robin over 256 CUs, so a launch takes
// ~ceil(tiles / 256) tile-times and a tile-time is ~ BM (fixed BN, same K).
// Pick the cheapest; ties go to the larger tile (fewer operand re-reads).
int gemm_pick_config(int M, int N, int splits) {
  if (splits > 1) return 0;
  const int64_t tn = (N + 127) / 128;
  int best = 0;
  int64_t best_cost = -1;
  for (int c = 0; c < 3; ++c) {
    const int64_t tiles = ((M + kCfgBM[c] - 1) / kCfgBM[c]) * tn;
    const int64_t cost = ((tiles + 255) / 256) * kCfgBM[c];
    if (best_cost < 0 || cost < best_cost) {
      best = c;
      best_cost = cost;
    }
  }
  return best;
}

template <bool AK, bool BKM>
static void launch_cfg(int cfg, dim3 g, hipStream_t st, const GemmParams& p) {
  if (cfg == 0)
    hipLaunchKernelGGL((gemm_f32_kernel<AK, BKM, 2, 2, 2, 2, 16>), g, dim3(256), 0, st, p);
  else if (cfg == 1)
    hipLaunchKernelGGL((gemm_f32_kernel<AK, BKM, 2, 2, 1, 2, 32>), g, dim3(256), 0, st, p);
  else
    hipLaunchKernelGGL((gemm_f32_kernel<AK, BKM, 1, 4, 1, 1, 32>), g, dim3(256), 0, st, p);
}

int launch_gemm(const GemmParams& p, hipStream_t st) {
  const int Mmax = p.M_dev ? p.M_max : p.M;
  const int Kmax = p.K_dev ? p.K_max : p.K;
  PS_REQUIRE(p.N > 0 && Mmax >= 0 && Kmax >= 0, kErrArg, "gemm: bad sizes");
  if (Mmax == 0) return kOk;
  PS_REQUIRE(p.K % 4 == 0 || p.K_dev, kErrArg, "gemm: K must be a multiple of 4");
  PS_REQUIRE(p.K1 < 0 || (p.K1 % 4 == 0 && p.a_kmajor && p.a2), kErrArg,
             "gemm: second K segment must start on a multiple of 4");
  PS_REQUIRE(p.a_kmajor || (p.M % 4 == 0 && !p.M_dev), kErrArg,
             "gemm: M-major A needs a static M that is a multiple of 4");
  PS_REQUIRE(p.b_kmajor || p.N % 4 == 0, kErrArg, "gemm: N-major B needs N % 4 == 0");
  PS_REQUIRE(!p.b2 || (!p.b_kmajor && p.N1 >= 0 && p.N1 % 4 == 0), kErrArg,
             "gemm: a second B segment needs N-major B and N1 % 4 == 0");
  PS_REQUIRE(!p.c2 || (p.N1 >= 0 && p.epi != kEpiL2Norm && p.epi != kEpiPartial), kErrArg,
             "gemm: split output needs N1 and a store/accumulate epilogue");
  PS_REQUIRE(p.epi != kEpiL2Norm || p.N <= 128, kErrArg, "gemm: L2-norm epilogue needs N <= 128");
  PS_REQUIRE(p.epi != kEpiPartial || (!p.M_dev && !p.c_idx), kErrArg,
             "gemm: split-K partials need a static M");
  const int splits = p.epi == kEpiPartial ? p.splits : 1;
  const int Mest = p.M_dev ? (p.M_hint > 0 ? std::min(p.M_hint, Mmax) : Mmax) : p.M;
  const int cfg = p.cfg >= 0 ? p.cfg : gemm_pick_config(Mest, p.N, splits);
  const int BMc = kCfgBM[cfg];
  const int tiles_m = (Mmax + BMc - 1) / BMc, tiles_n = (p.N + 127) / 128;
  int G = splits > 1 ? splits : tiles_m, W = splits > 1 ? tiles_m * tiles_n : tiles_n;
  int64_t iters = 8LL * ((G + 7) / 8) * W;
  int grid = (int)(iters < 1024 ? iters : 1024);
  grid = (grid + 7) / 8 * 8;
  dim3 g(grid);
  if (p.a_kmajor && p.b_kmajor) launch_cfg<true, true>(cfg, g, st, p);
  else if (p.a_kmajor && !p.b_kmajor) launch_cfg<true, false>(cfg, g, st, p);
  else if (!p.a_kmajor && p.b_kmajor) launch_cfg<false, true>(cfg, g, st, p);
  else launch_cfg<false, false>(cfg, g, st, p);
  PS_CHECK_LAUNCH();
  return kOk;
}

}  // namespace ps
