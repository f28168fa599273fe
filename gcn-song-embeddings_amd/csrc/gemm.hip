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

namespace ps {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int BM = 128, BN = 128, BK = 16, PADF = 4;
constexpr int LDS_W = 128 + PADF;  // floats per k-row of a staged tile

// Rows of a K-major operand ([row][k] in memory) for this thread: 2 float4 per tile.
// p2 is the row base in the second K segment (k >= K1), if any.
struct KRows {
  const float* p[2];
  const float* p2[2];
};

__device__ __forceinline__ void kmajor_rows(KRows& R, int tid, int r0, int rmax, const float* a,
                                            int64_t lda, const int32_t* idx, const float* a2,
                                            int64_t lda2, const int32_t* idx2) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int lin = tid + 256 * i;
    const int row = r0 + (lin >> 2);
    if (row < rmax) {
      const int64_t r = idx ? idx[row] : row;
      R.p[i] = a + r * lda;
      if (a2) {
        const int64_t r2 = idx2 ? idx2[row] : row;
        R.p2[i] = a2 + r2 * lda2;
      } else {
        R.p2[i] = nullptr;
      }
    } else {
      R.p[i] = nullptr;
      R.p2[i] = nullptr;
    }
  }
}

// K-major operand tile -> registers (k0 = absolute k of the tile).  Each float4
// chunk picks its segment on its own, so K1 only has to be a multiple of 4.
__device__ __forceinline__ void kmajor_load(float4 (&v)[2], const KRows& R, int tid, int k0,
                                            int kend, int K1) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int kc = (tid + 256 * i) & 3;
    const int k = k0 + kc * 4;
    const bool seg2 = K1 >= 0 && k >= K1;
    const float* base = seg2 ? R.p2[i] : R.p[i];
    if (R.p[i] && k < kend) v[i] = *reinterpret_cast<const float4*>(base + (seg2 ? k - K1 : k));
    else v[i] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
}
__device__ __forceinline__ void kmajor_store(float (*S)[LDS_W], const float4 (&v)[2], int tid) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int lin = tid + 256 * i;
    const int row = lin >> 2, kc = lin & 3;
    S[kc * 4 + 0][row] = v[i].x;
    S[kc * 4 + 1][row] = v[i].y;
    S[kc * 4 + 2][row] = v[i].z;
    S[kc * 4 + 3][row] = v[i].w;
  }
}

// MN-major operand ([k][col] in memory, k rows optionally gathered)
__device__ __forceinline__ void mnmajor_load(float4 (&v)[2], int tid, const float* a, int64_t lda,
                                             const int32_t* idx, int c0, int cmax, int k0,
                                             int kend) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int lin = tid + 256 * i;
    const int kr = lin >> 5, cc = lin & 31;
    const int k = k0 + kr;
    const int c = c0 + cc * 4;
    if (k < kend && c < cmax) {
      const int64_t r = idx ? idx[k] : k;
      v[i] = *reinterpret_cast<const float4*>(a + r * lda + c);
    } else {
      v[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
}
__device__ __forceinline__ void mnmajor_store(float (*S)[LDS_W], const float4 (&v)[2], int tid) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int lin = tid + 256 * i;
    const int kr = lin >> 5, cc = lin & 31;
    *reinterpret_cast<float4*>(&S[kr][cc * 4]) = v[i];
  }
}

template <bool AK, bool BKM>
__global__ __launch_bounds__(256, 2) void gemm_f32_kernel(GemmParams p) {
  __shared__ __attribute__((aligned(16))) float As[2][BK][LDS_W];
  __shared__ __attribute__((aligned(16))) float Bs[2][BK][LDS_W];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
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

    KRows RA, RB;
    if (AK) kmajor_rows(RA, tid, m0, M, p.a, p.lda, p.a_idx, p.a2, p.lda2, p.a2_idx);
    if (BKM) kmajor_rows(RB, tid, n0, N, p.b, p.ldb, nullptr, nullptr, 0, nullptr);

    f32x16 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    float4 va[2], vb[2];
    auto load = [&](int k0) {
      if (AK) kmajor_load(va, RA, tid, k0, ke, p.K1);
      else mnmajor_load(va, tid, p.a, p.lda, p.a_idx, m0, M, k0, ke);
      if (BKM) kmajor_load(vb, RB, tid, k0, ke, -1);
      else mnmajor_load(vb, tid, p.b, p.ldb, p.b_idx, n0, N, k0, ke);
    };
    auto store = [&](int buf) {
      if (AK) kmajor_store(As[buf], va, tid);
      else mnmajor_store(As[buf], va, tid);
      if (BKM) kmajor_store(Bs[buf], vb, tid);
      else mnmajor_store(Bs[buf], vb, tid);
    };
    if (nk > 0) {
      load(kb);
      store(0);
    }
    __syncthreads();
    const int h = lane >> 5, l32 = lane & 31;
    for (int it = 0; it < nk; ++it) {
      const int cur = it & 1;
      if (it + 1 < nk) load(kb + (it + 1) * BK);
#pragma unroll
      for (int kk = 0; kk < BK / 2; ++kk) {
        const int k = 2 * kk + h;
        const float a0 = As[cur][k][wm * 64 + l32];
        const float a1 = As[cur][k][wm * 64 + 32 + l32];
        const float b0 = Bs[cur][k][wn * 64 + l32];
        const float b1 = Bs[cur][k][wn * 64 + 32 + l32];
        acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b0, acc[0][0], 0, 0, 0);
        acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b1, acc[0][1], 0, 0, 0);
        acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b0, acc[1][0], 0, 0, 0);
        acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b1, acc[1][1], 0, 0, 0);
      }
      if (it + 1 < nk) store(cur ^ 1);
      __syncthreads();
    }

    // ------------------------------------------------------------ epilogue
    // acc[i][j][r] -> row m0 + wm*64 + i*32 + (r&3) + 8*(r>>2) + 4*h, col n0 + wn*64 + j*32 + l32
    if (p.epi == kEpiPartial) {
      float* C = p.c + (int64_t)split * M * p.ldc;
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = m0 + wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
          if (row >= M) continue;
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            const int col = n0 + wn * 64 + j * 32 + l32;
            if (col < N) C[(int64_t)row * p.ldc + col] = acc[i][j][r];
          }
        }
    } else if (p.epi == kEpiL2Norm) {
      float* red = &As[0][0][0];  // [2][128] row partial sums (LDS free after the k loop)
      float ss[2][16];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          float s2 = 0.f;
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            const int col = n0 + wn * 64 + j * 32 + l32;
            float v = acc[i][j][r] + (p.bias && col < N ? p.bias[col] : 0.f);
            v = lrelu(v);
            if (col >= N) v = 0.f;
            acc[i][j][r] = v;
            s2 += v * v;
          }
#pragma unroll
          for (int o = 1; o < 32; o <<= 1) s2 += __shfl_xor(s2, o, 64);
          ss[i][r] = s2;
        }
      if (l32 == 0) {
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int r = 0; r < 16; ++r)
            red[wn * 128 + wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h] = ss[i][r];
      }
      __syncthreads();
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int lrow = wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
          const int row = m0 + lrow;
          if (row >= M) continue;
          const float nrm = sqrtf(red[lrow] + red[128 + lrow]);
          const int64_t dst = p.c_idx ? p.c_idx[row] : row;
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            const int col = n0 + wn * 64 + j * 32 + l32;
            if (col < N) p.c[dst * p.ldc + col] = acc[i][j][r] / nrm;
          }
          if (p.norms && wn == 0 && l32 == 0) p.norms[row] = nrm;
        }
    } else {
      const bool accum = p.epi == kEpiAccum;
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = m0 + wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
          if (row >= M) continue;
          const int64_t dst = p.c_idx ? p.c_idx[row] : row;
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            const int col = n0 + wn * 64 + j * 32 + l32;
            if (col >= N) continue;
            float v = acc[i][j][r];
            if (p.bias) v += p.bias[col];
            if (p.act) v = lrelu(v);
            if (p.mask) v *= lrelu_grad(p.mask[(int64_t)row * p.ldm + col]);
            float* o = p.c + dst * p.ldc + col;
            *o = accum ? *o + v : v;
          }
        }
    }
    __syncthreads();
  }
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
  PS_REQUIRE(p.epi != kEpiL2Norm || p.N <= BN, kErrArg, "gemm: L2-norm epilogue needs N <= 128");
  PS_REQUIRE(p.epi != kEpiPartial || (!p.M_dev && !p.c_idx), kErrArg,
             "gemm: split-K partials need a static M");
  const int tiles_m = (Mmax + BM - 1) / BM, tiles_n = (p.N + BN - 1) / BN;
  const int splits = p.epi == kEpiPartial ? p.splits : 1;
  int G = splits > 1 ? splits : tiles_m, W = splits > 1 ? tiles_m * tiles_n : tiles_n;
  int64_t iters = 8LL * ((G + 7) / 8) * W;
  int grid = (int)(iters < 1024 ? iters : 1024);
  grid = (grid + 7) / 8 * 8;
  dim3 g(grid), b(256);
  if (p.a_kmajor && p.b_kmajor)
    hipLaunchKernelGGL((gemm_f32_kernel<true, true>), g, b, 0, st, p);
  else if (p.a_kmajor && !p.b_kmajor)
    hipLaunchKernelGGL((gemm_f32_kernel<true, false>), g, b, 0, st, p);
  else if (!p.a_kmajor && p.b_kmajor)
    hipLaunchKernelGGL((gemm_f32_kernel<false, true>), g, b, 0, st, p);
  else
    hipLaunchKernelGGL((gemm_f32_kernel<false, false>), g, b, 0, st, p);
  PS_CHECK_LAUNCH();
  return kOk;
}

}  // namespace ps
