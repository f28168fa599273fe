// fp32 MFMA GEMM (v_mfma_f32_32x32x2_f32: exact fp32 FMA chain, 64 FLOP/clk/SIMD
// on gfx950; there is no xf32 path, and the reference computes in fp32).
//
// Block tiles of BM x 128 (BM = 128 / 64 / 32), 256 threads = 4 waves, each
// wave TM x TN MFMA tiles of 32x32.  Operands are staged HBM -> LDS with
// global_load_lds (LDS-DMA, 16 B per lane, no staging registers) into a ring of
// three stage buffers: stage t is computed while t+1 and t+2 are in flight,
// retired by a counted s_waitcnt vmcnt and a raw s_barrier (a __syncthreads
// would drain the DMA queue).  K-major images are [R][BK] with 16-B chunks
// XOR-swizzled by row (conflict-free ds_read_b128 fragments; the swizzle is
// applied on the per-lane SOURCE address, the DMA writes lane-linearly);
// MN-major images are linear [BK][R] read with ds_read_b32.  Out-of-range rows,
// k and columns read clamped in-range addresses; the k-tail is zeroed in LDS
// after it lands, other garbage only reaches discarded outputs.  Gathered
// k-row numbers (MN-major operands) are staged in LDS per 1024-row window so
// that no ordinary VGPR load sits between DMA issue and use.  Persistent grid:
// the tiles of one row panel (or of one split-K slice) are dealt to blocks
// b, b+8, ... so they share an XCD's L2.
#include "gemm.h"

#include <algorithm>

#include "bf16split.h"
#include "lds_dma.h"
#include <type_traits>

namespace ps {

typedef float f32x16 __attribute__((ext_vector_type(16)));
// the exact hi / mid / lo split of the split-bf16 products: bf16split.h

constexpr int kLdsBudget = 81920;  // bytes per workgroup: two workgroups per CU
constexpr int kLdsBudget3 = 54272;  // three workgroups per CU (cfg 3)
constexpr int kLdsBudget4 = 40960;  // four workgroups per CU (cfg 4)
constexpr int kIdxWin = 1024;  // gathered k-rows staged in LDS at a time

__device__ __forceinline__ void zero16(float* l) {
  *reinterpret_cast<float4*>(l) = make_float4(0.f, 0.f, 0.f, 0.f);
}

// K-major operand: global [row][k] (rows optionally gathered), LDS image
// [R][BK] with chunk c of row r stored at chunk c ^ swz(r).  Chunk q = j*256 +
// tid of a stage is this thread's j-th DMA; all of one wave's 64 chunks of an
// instruction are contiguous in LDS (lane-linear), as the DMA requires.
template <int R, int BK>
struct KOp {
  static constexpr int CPR = BK / 4;
  static constexpr int NI = R * CPR / 256;
  static constexpr int SZ = R * BK;  // floats per stage image
  static_assert(R * CPR % 256 == 0, "whole DMAs per thread");
  static constexpr int SH = BK == 32 ? 1 : 2;
  __device__ static __forceinline__ int swz(int row) { return (row >> SH) & (CPR - 1); }
  __device__ static __forceinline__ float4 frag(const float* img, int row, int k4) {
    return *reinterpret_cast<const float4*>(img + row * BK + 4 * ((k4 >> 2) ^ swz(row)));
  }
  const float* rp[NI];
  const float* rp2[NI];
  int lc[NI];
  __device__ __forceinline__ void init(int tid, int r0, int rmax, const float* a, int64_t lda,
                                       const int32_t* idx, const float* a2, int64_t lda2,
                                       const int32_t* idx2) {
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const int q = j * 256 + tid, row = q / CPR;
      lc[j] = 4 * ((q % CPR) ^ swz(row));
      const int g = r0 + row, rc = g < rmax ? g : rmax - 1;
      rp[j] = a + (int64_t)(idx ? idx[rc] : rc) * lda;
      rp2[j] = a2 ? a2 + (int64_t)(idx2 ? idx2[rc] : rc) * lda2 : rp[j];
    }
  }
  __device__ __forceinline__ void issue(unsigned img, int wave, int k0, int kend, int K1) const {
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const int k = min(k0 + lc[j], kend - 4);
      const float* src = (K1 >= 0 && k >= K1) ? rp2[j] + (k - K1) : rp[j] + k;
      glds16(src, img + (unsigned)(j * 256 + wave * 64) * 16u);
    }
  }
  __device__ __forceinline__ void zero_tail(float* img, int tid, int k0, int kend) const {
#pragma unroll
    for (int j = 0; j < NI; ++j)
      if (k0 + lc[j] >= kend) zero16(img + (j * 256 + tid) * 4);
  }
};

// K-major operand stored pre-split (GemmParams::b_split): three bf16 planes
// [R][ldb] each, the stage image of each plane a KOp image of BK/2 floats per
// row (8 bf16 per 16-B chunk, so a lane's 8 k of one 16-k step are one
// swizzled ds_read_b128 per plane).  k coordinates are in elements; the plane
// images are addressed in floats (k / 2).
template <int R, int BK>
struct KSplitOp {
  using P = KOp<R, BK / 2>;
  static constexpr int NI = 3 * P::NI;
  static constexpr int SZ = 3 * P::SZ;
  __device__ static __forceinline__ float4 frag(const float* img, int row, int k4) {
    return P::frag(img, row, k4);  // (only the split-bf16 path reads this operand)
  }
  P op;
  int64_t pstride;  // floats between planes
  __device__ __forceinline__ void init(int tid, int r0, int rmax, const uint16_t* b, int64_t ldb,
                                       int64_t rows) {
    op.init(tid, r0, rmax, reinterpret_cast<const float*>(b), ldb / 2, nullptr, nullptr, 0, nullptr);
    pstride = rows * ldb / 2;
  }
  __device__ __forceinline__ void issue(unsigned img, int wave, int k0, int kend, int) const {
#pragma unroll
    for (int q = 0; q < 3; ++q)
#pragma unroll
      for (int j = 0; j < P::NI; ++j) {
        const int k = min(k0 / 2 + op.lc[j], kend / 2 - 4);
        glds16(op.rp[j] + q * pstride + k,
               img + (unsigned)(q * P::SZ) * 4u + (unsigned)(j * 256 + wave * 64) * 16u);
      }
  }
  __device__ __forceinline__ void zero_tail(float* img, int tid, int k0, int kend) const {
#pragma unroll
    for (int q = 0; q < 3; ++q) op.zero_tail(img + q * P::SZ, tid, k0 / 2, kend / 2);
  }
};

// Interleaved-plane operand (GemmParams::a_ilv / b_ilv, launch_split_ilv):
// each row of the table is K/16 stages of 96 B -- the hi / mid / lo bf16 of
// its 16 k as six 16-B chunks, chunk w = plane * 2 + half -- so one row's
// stage is a single contiguous piece however the rows are gathered.  LDS
// image: row r's six chunks at slots r*6 .., chunk w at slot (w + ((r >> 3) & 1))
// % 6 (the rotation makes every ds_read_b128 lane group of a fragment
// conflict-free at the 96-B row pitch).
template <int R>
struct IlvOp {
  static constexpr int SZ = R * 24;          // floats per stage image
  static constexpr int NI = R * 6 / 256;     // 16-B DMAs per thread per stage
  static_assert(R * 6 % 256 == 0, "whole DMAs per thread");
  __device__ static __forceinline__ float4 frag(const float* img, int row, int w) {
    int sl = w + ((row >> 3) & 1);
    sl = sl >= 6 ? sl - 6 : sl;
    return *reinterpret_cast<const float4*>(img + (row * 6 + sl) * 4);
  }
  const char* rp[NI];
  __device__ __forceinline__ void init(int tid, int r0, int rmax, const uint16_t* t, int64_t ld,
                                       const int32_t* idx) {
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const int i = j * 256 + tid, row = i / 6, sl = i - row * 6;
      int w = sl - ((row >> 3) & 1);
      w = w < 0 ? w + 6 : w;
      const int g = r0 + row, rc = g < rmax ? g : rmax - 1;
      rp[j] = reinterpret_cast<const char*>(t + (int64_t)(idx ? idx[rc] : rc) * ld) + w * 16;
    }
  }
  __device__ __forceinline__ void issue(unsigned img, int wave, int k0, int, int) const {
#pragma unroll
    for (int j = 0; j < NI; ++j)
      glds16(reinterpret_cast<const float*>(rp[j] + (k0 / 16) * 96), img + (unsigned)(j * 256 + wave * 64) * 16u);
  }
  __device__ __forceinline__ void zero_tail(float*, int, int, int) const {}  // (K % 16 == 0)
};

// MN-major operand: global [k][col] (k rows optionally gathered; columns >= c1
// from a second matrix), LDS image linear [BK][R].
template <int R, int BK>
struct MNOp {
  static constexpr int CPR = R / 4;
  static constexpr int NI = BK * CPR / 256;
  static constexpr int SZ = BK * R;
  static constexpr int KSTEP = 256 / CPR;  // k-rows between a thread's DMAs
  static_assert(BK * CPR % 256 == 0 && 256 % CPR == 0, "whole DMAs per thread");
  __device__ static __forceinline__ float4 frag(const float* img, int col, int k4) {
    return make_float4(img[(k4 + 0) * R + col], img[(k4 + 1) * R + col], img[(k4 + 2) * R + col],
                       img[(k4 + 3) * R + col]);
  }
  const float* base;
  int64_t ld;
  bool gathered;
  int kr0;
  __device__ __forceinline__ void init(int tid, int c0, int cmax, const float* a, int64_t lda,
                                       const int32_t* idx, int c1, const float* a2, int64_t lda2,
                                       const int32_t* idx2) {
    kr0 = tid / CPR;
    const int cc = c0 + 4 * (tid % CPR), cl = cc < cmax ? cc : cmax - 4;
    if (a2 && cl >= c1) {
      base = a2 + (cl - c1);
      ld = lda2;
      gathered = idx2 != nullptr;
    } else {
      base = a + cl;
      ld = lda;
      gathered = idx != nullptr;
    }
  }
  // sidx: LDS window of gathered row numbers starting at k-row wb
  __device__ __forceinline__ void issue(unsigned img, int wave, int k0, int kend, const int* sidx,
                                        int wb) const {
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const int k = min(k0 + kr0 + KSTEP * j, kend - 1);
      const int64_t r = gathered ? sidx[k - wb] : k;
      glds16(base + r * ld, img + (unsigned)(j * 256 + wave * 64) * 16u);
    }
  }
  __device__ __forceinline__ void zero_tail(float* img, int tid, int k0, int kend) const {
#pragma unroll
    for (int j = 0; j < NI; ++j)
      if (k0 + kr0 + KSTEP * j >= kend) zero16(img + (j * 256 + tid) * 4);
  }
};

// Stream-K arrival ticket and slab addressing (work units = (tile, k-step)).
// Block b of the Ga active blocks owns units [b*U/Ga, (b+1)*U/Ga); a tile cut
// by a block boundary is finished by the last of its blocks to arrive.  Every
// block keeps at most two partial tiles (its first and its last), in slab
// slots 2b and 2b+1.
struct SkPlan {
  int64_t U;
  int I, Ga;
  __device__ __forceinline__ int64_t start(int b) const { return (int64_t)b * U / Ga; }
  __device__ __forceinline__ int block_of(int64_t u) const {  // the block owning unit u
    return (int)(((u + 1) * Ga - 1) / U);
  }
};

// 4 x 4 transposes inside lane quads, by two DPP butterflies: v[4g + k] of
// lane (quad q, i = lane & 3) holds row k of column 4q + i of row group g
// (the 32x32 f32 accumulator layout: register r is row (r & 3) + 8 (r >> 2) of
// column l32); afterwards it holds row i, column 4q + k -- four consecutive
// columns of one row, one 16-B store instead of four 4-B ones.
__device__ __forceinline__ float dpp_xor1(float x) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), 0xB1, 0xF, 0xF, false));  // quad_perm 1,0,3,2
}
__device__ __forceinline__ float dpp_xor2(float x) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), 0x4E, 0xF, 0xF, false));  // quad_perm 2,3,0,1
}
__device__ __forceinline__ void quad_transpose16(float (&v)[16], int lane) {
  const int i = lane & 3;
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    float t[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) t[k] = dpp_xor1(v[4 * g + (k ^ 1)]);
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if ((i & 1) != (k & 1)) v[4 * g + k] = t[k];
#pragma unroll
    for (int k = 0; k < 4; ++k) t[k] = dpp_xor2(v[4 * g + (k ^ 2)]);
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if ((i & 2) != (k & 2)) v[4 * g + k] = t[k];
  }
}

// WM x WN waves, each TM x TN MFMA tiles of 32x32; stage depth BK; at most
// NSMAX stage buffers in the ring.  SK: the kernel carries the stream-K
// schedule (cfg 1 and 2, the tiles launch_gemm runs it on); without it the
// tile loop is inlined once and the code is ~40 % smaller, which a launch
// pays for in instruction fetch before its first MFMA.
template <bool AK, bool BKM, int WM, int WN, int TM, int TN, int BK, int NSMAX = 4, int WPC = 2,
          bool BF = false, bool PB = false, bool SK = true, int IL = 0>
__global__ __launch_bounds__(256, WPC) void gemm_f32_kernel(GemmParams p) {
  static_assert(!BF || BK % 16 == 0, "split-bf16 products: 16-k steps");
  static_assert(!PB || (BF && BKM), "pre-split B: split-bf16 products, K-major B");
  // IL 1: A and B from interleaved tables; 2: A from one, B fp32 split in registers
  static_assert(!IL || (BF && AK && BKM && !PB && !SK && BK == 16), "interleaved planes: split bf16, K-major A and B");
  constexpr int BM = WM * TM * 32, BN = WN * TN * 32;
  using OpA = typename std::conditional<
      IL != 0, IlvOp<BM>, typename std::conditional<AK, KOp<BM, BK>, MNOp<BM, BK>>::type>::type;
  using OpBp = typename std::conditional<
      PB, KSplitOp<BN, BK>, typename std::conditional<BKM, KOp<BN, BK>, MNOp<BN, BK>>::type>::type;
  using OpB = typename std::conditional<IL == 1, IlvOp<BN>, OpBp>::type;
  constexpr int SZA = OpA::SZ, SZB = OpB::SZ, SZS = SZA + SZB;
  constexpr int NG = OpA::NI + OpB::NI;  // DMAs per wave per stage
  constexpr bool GA = !AK, GB = !BKM;    // operands that may need gathered k-rows
  // ring depth: as many stage buffers as fit two workgroups per CU (3 or 4);
  // the k-row windows exist only for MN-major (possibly gathered) operands
  constexpr int IDXF = (GA ? kIdxWin : 0) + (GB ? kIdxWin : 0);
  constexpr int NSA = ((WPC == 2 ? kLdsBudget : WPC == 3 ? kLdsBudget3 : kLdsBudget4) / 4 - IDXF) / SZS;
  constexpr int NS = NSA > NSMAX ? NSMAX : NSA;
  static_assert(NS >= 3, "stage buffers do not fit");
  __shared__ __attribute__((aligned(16))) float smem[NS * SZS + IDXF];
  int* const sidxA = reinterpret_cast<int*>(smem + NS * SZS);
  int* const sidxB = sidxA + (GA ? kIdxWin : 0);

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
#ifdef PS_GEMM_PROBE  // (diagnostic build only) wall-clock phases of block 0's first tile
  uint64_t pt[6] = {__builtin_amdgcn_s_memrealtime(), 0, 0, 0, 0, 0};
  int pti = 1;
#define PS_PROBE() do { if (pti < 6) pt[pti++] = __builtin_amdgcn_s_memrealtime(); } while (0)
#else
#define PS_PROBE() do { } while (0)
#endif
  const int M = p.M_dev ? *p.M_dev : p.M;
  const int K = p.K_dev ? *p.K_dev : p.K;
  const int N = p.N;
  const int tiles_m = (M + BM - 1) / BM, tiles_n = (N + BN - 1) / BN;
  const int splits = p.epi == kEpiPartial ? p.splits : 1;
  // split-K chunks on a 32-k grid whatever the stage depth (BK 16 or 32): the
  // cut points -- and with them every slab's summation order -- are the same
  // for every tile config, so the tuner's choice cannot change the gradient
  static_assert(32 % BK == 0, "split-K chunks are whole stages");
  const int kchunk = (((K + splits - 1) / splits) + 31) / 32 * 32;
  const int32_t* idxA = GA ? p.a_idx : nullptr;
  const int32_t* idxB = GB ? p.b_idx : nullptr;
  const int32_t* idxB2 = GB ? p.b2_idx : nullptr;
  const int32_t* idxBw = idxB ? idxB : idxB2;  // one gathered B segment (launch_gemm checks)
  const bool needA = GA && idxA;
  const bool needB = GB && (idxB || idxB2);
  const int h = lane >> 5, l32 = lane & 31;
  // LDS byte address of the ring (a constant: the cast of the __shared__
  // array itself, not of a computed generic pointer)
  const unsigned smem_lds = (unsigned)(size_t)((__attribute__((address_space(3))) float*)smem);

  // one tile (tm, tn) over k in [kb, ke): k loop, then the epilogue.  sk_t >= 0:
  // a stream-K segment of tile sk_t that does not cover all of k (publish the
  // partial sum; the last segment to arrive adds them up and runs the epilogue)
  auto run_item = [&](int tm, int tn, int split, int kb, int ke, int sk_t, int sk_slot,
                      const SkPlan& sk) __attribute__((always_inline)) {
    const int m0 = tm * BM, n0 = tn * BN;
    const int nk = ke > kb ? (ke - kb + BK - 1) / BK : 0;
    const bool tail = ((ke - kb) % BK) != 0;

    OpA opa;
    OpB opb;
    if constexpr (IL) {
      opa.init(tid, m0, M, p.a_ilv, p.lda_ilv, p.a_idx);
      if constexpr (IL == 1) opb.init(tid, n0, N, p.b_ilv, p.ldb_ilv, nullptr);
    } else if constexpr (AK) opa.init(tid, m0, M, p.a, p.lda, p.a_idx, p.a2, p.lda2, p.a2_idx);
    else opa.init(tid, m0, M, p.a, p.lda, idxA, -1, nullptr, 0, nullptr);
    if constexpr (IL == 1) {
    } else if constexpr (PB) opb.init(tid, n0, N, p.b_split, p.ldb_split, N);
    else if constexpr (BKM) opb.init(tid, n0, N, p.b, p.ldb, nullptr, nullptr, 0, nullptr);
    else opb.init(tid, n0, N, p.b, p.ldb, idxB, p.N1, p.b2, p.ldb2, idxB2);

    // gathered k-row numbers of the first window (no DMA is in flight here)
    int wb = kb;
    auto fill_idx = [&](int w0) __attribute__((always_inline)) {
      for (int i = tid; i < kIdxWin; i += 256) {
        const int k = min(w0 + i, ke - 1);
        if (needA) sidxA[i] = idxA[k];
        if (needB) sidxB[i] = idxBw[k];
      }
    };
    if ((needA || needB) && nk > 0) {
      fill_idx(wb);
      __syncthreads();
    }

    f32x16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    auto issue = [&](int st) __attribute__((always_inline)) {
      const int k0 = kb + st * BK;
      const unsigned base = smem_lds + (unsigned)((st % NS) * SZS) * 4u;
      if constexpr (AK) opa.issue(base, wave, k0, ke, p.K1);
      else opa.issue(base, wave, k0, ke, sidxA, wb);
      if constexpr (BKM) opb.issue(base + SZA * 4u, wave, k0, ke, -1);
      else opb.issue(base + SZA * 4u, wave, k0, ke, sidxB, wb);
    };
    const bool do_bias = !AK && p.bias_part && tn == 0 && tid < BM;
    float bsum = 0.f;
    // the store / accumulate epilogue's bias, fetched under the k loop (a load
    // issued in the epilogue put one more memory round trip on every tile)
    float bj[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int col = n0 + (wn * TN + j) * 32 + l32;
      bj[j] = (p.bias && col < N && p.epi != kEpiL2Norm && p.epi != kEpiPartial) ? p.bias[col] : 0.f;
    }
    // MFMA k-assignment: in the r-th MFMA of octet s, lane half h supplies
    // k = 8s + 4h + r for both operands (any bijection onto the 8 k works).
    // Fragments of octet s+1 are read from LDS while octet s's MFMAs run.
    auto compute = [&](const float* As, const float* Bs) __attribute__((always_inline)) {
      if (do_bias) {  // column sums of A^T over this tile's k rows (tail zeroed)
#pragma unroll
        for (int k = 0; k < BK; ++k) bsum += As[k * BM + tid];
      }
      auto rd = [&](float4 (&fa)[TM], float4 (&fb)[TN], int s8) __attribute__((always_inline)) {
        const int k4 = 8 * s8 + 4 * h;
#pragma unroll
        for (int i = 0; i < TM; ++i) fa[i] = OpA::frag(As, (wm * TM + i) * 32 + l32, k4);
#pragma unroll
        for (int j = 0; j < TN; ++j) fb[j] = OpB::frag(Bs, (wn * TN + j) * 32 + l32, k4);
      };
      auto mm = [&](const float4 (&fa)[TM], const float4 (&fb)[TN]) __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[i].x, fb[j].x, acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[i].y, fb[j].y, acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[i].z, fb[j].z, acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[i].w, fb[j].w, acc[i][j], 0, 0, 0);
          }
      };
      if constexpr (BF) {
        // 16-k steps: lane (row l32, half h) holds k = 16 t + 8 h + j, j = 0..7
        // (two float4 fragments of the K-major or M-/N-major image), split into hi / mid / lo;
        // the products whose magnitude is >= 2^-18 of hi*hi, smallest first
#pragma unroll
        for (int t = 0; t < BK / 16; ++t) {
          bf16x8 aH[TM], aM[TM], aL[TM], bH[TN], bM[TN], bL[TN];
#pragma unroll
          for (int i = 0; i < TM; ++i) {
            const int r = (wm * TM + i) * 32 + l32;
            if constexpr (IL) {  // interleaved planes: chunk plane * 2 + h of row r
              aH[i] = __builtin_bit_cast(bf16x8, OpA::frag(As, r, h));
              aM[i] = __builtin_bit_cast(bf16x8, OpA::frag(As, r, 2 + h));
              aL[i] = __builtin_bit_cast(bf16x8, OpA::frag(As, r, 4 + h));
            } else {
              split3(OpA::frag(As, r, 16 * t + 8 * h), OpA::frag(As, r, 16 * t + 8 * h + 4), aH[i], aM[i],
                     aL[i]);
            }
          }
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            const int c = (wn * TN + j) * 32 + l32;
            if constexpr (IL == 1) {
              bH[j] = __builtin_bit_cast(bf16x8, OpB::frag(Bs, c, h));
              bM[j] = __builtin_bit_cast(bf16x8, OpB::frag(Bs, c, 2 + h));
              bL[j] = __builtin_bit_cast(bf16x8, OpB::frag(Bs, c, 4 + h));
            } else if constexpr (PB) {  // the planes' 8 k of this lane: one chunk each
              using P = typename OpB::P;
              bH[j] = __builtin_bit_cast(bf16x8, P::frag(Bs, c, 8 * t + 4 * h));
              bM[j] = __builtin_bit_cast(bf16x8, P::frag(Bs + P::SZ, c, 8 * t + 4 * h));
              bL[j] = __builtin_bit_cast(bf16x8, P::frag(Bs + 2 * P::SZ, c, 8 * t + 4 * h));
            } else {
              split3(OpB::frag(Bs, c, 16 * t + 8 * h), OpB::frag(Bs, c, 16 * t + 8 * h + 4), bH[j],
                     bM[j], bL[j]);
            }
          }
          // product by product over the blocks: consecutive MFMAs write
          // different accumulators (1-3 % over block by block)
#define PS_BF_ALL(X, Y)                                                                       \
  _Pragma("unroll") for (int i = 0; i < TM; ++i) _Pragma("unroll") for (int j = 0; j < TN; ++j) \
      acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(X[i], Y[j], acc[i][j], 0, 0, 0);
          PS_BF_ALL(aL, bH)
          PS_BF_ALL(aH, bL)
          PS_BF_ALL(aM, bM)
          PS_BF_ALL(aM, bH)
          PS_BF_ALL(aH, bM)
          PS_BF_ALL(aH, bH)
#undef PS_BF_ALL
        }
        return;
      }
      static_assert((BK / 8) % 2 == 0, "octets are processed in pairs");
      // sched_barrier pins the prefetch distance (the scheduler otherwise
      // sinks each read next to its MFMAs and exposes the LDS latency)
      float4 fa0[TM], fb0[TN], fa1[TM], fb1[TN];
      rd(fa0, fb0, 0);
#pragma unroll
      for (int s8 = 0; s8 < BK / 8; s8 += 2) {
        rd(fa1, fb1, s8 + 1);
        __builtin_amdgcn_sched_barrier(0);
        mm(fa0, fb0);
        __builtin_amdgcn_sched_barrier(0);
        if (s8 + 2 < BK / 8) rd(fa0, fb0, s8 + 2);
        __builtin_amdgcn_sched_barrier(0);
        mm(fa1, fb1);
        __builtin_amdgcn_sched_barrier(0);
      }
    };

    // ring: stage t is computed from slot t % NS while stages t+1 .. t+NS-2 are
    // in flight; stage t+NS-1 is issued into the slot stage t-1 used
    auto slot = [&](int st) __attribute__((always_inline)) { return smem + (st % NS) * SZS; };
    PS_PROBE();
    for (int st = 0; st < NS - 1 && st < nk; ++st) issue(st);
    for (int it = 0; it < nk; ++it) {
      // retire this wave's DMAs of stage it; the younger stages stay in flight
      const int younger = min(NS - 2, nk - 1 - it);
      wait_stage<NG, NS - 2>(younger);
      if (it == 0) PS_PROBE();
      float* cur = slot(it);
      if (tail && it == nk - 1) {  // zero the k-tail this thread's DMAs brought in
        const int k0 = kb + it * BK;
        opa.zero_tail(cur, tid, k0, ke);
        opb.zero_tail(cur + SZA, tid, k0, ke);
      }
      // publish stage it; every wave is done reading stage it-1's slot
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      const int nx = it + NS - 1;
      if (nx < nk) {
        const int k2 = kb + nx * BK;
        if ((needA || needB) && k2 >= wb + kIdxWin) {  // next window of row numbers
          wb += kIdxWin;
          fill_idx(wb);
          asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
          __builtin_amdgcn_s_barrier();
        }
        issue(nx);
      }
      compute(cur, cur + SZA);
    }
    __syncthreads();  // stage buffers are reused by the epilogue / next tile
    PS_PROBE();

    // ------------------------------------------------------------ stream-K
    // Publish (write-through sc1 slab stores, every wave drains, one ticket
    // add per block); the block drawing the last ticket reads every segment's
    // slab with sc1 loads in block order (a fixed summation order: the result
    // does not depend on which block arrives last) and runs the epilogue.
    if constexpr (SK) if (sk_t >= 0) {
      typedef int v4i __attribute__((ext_vector_type(4)));
      const __amdgpu_buffer_rsrc_t rs =
          __builtin_amdgcn_make_buffer_rsrc(p.sk_slab, 0, 0x7fffffff, 0x00020000);
      constexpr int SLAB = BM * BN * 4;  // bytes per slot
      const unsigned lo = (unsigned)tid * 16u;
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const float4 v = make_float4(acc[i][j][4 * q], acc[i][j][4 * q + 1], acc[i][j][4 * q + 2],
                                         acc[i][j][4 * q + 3]);
            __builtin_amdgcn_raw_buffer_store_b128(*reinterpret_cast<const v4i*>(&v), rs,
                                                   lo + (unsigned)(((i * TN + j) * 4 + q) * 4096),
                                                   sk_slot * SLAB, 16);
          }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      int* const flag = reinterpret_cast<int*>(smem);
      const int tile = sk_t;
      const int bf = sk.block_of((int64_t)tile * sk.I), bl = sk.block_of((int64_t)(tile + 1) * sk.I - 1);
      if (tid == 0)
        flag[0] = __hip_atomic_fetch_add(p.sk_cnt + tile, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __syncthreads();
      const bool last = flag[0] == bl - bf;
      __syncthreads();
      if (!last) return;
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
      for (int bb = bf; bb <= bl; ++bb) {
        const int sl = 2 * bb + ((int)(sk.start(bb) / sk.I) == tile ? 0 : 1);
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              const v4i x = __builtin_amdgcn_raw_buffer_load_b128(
                  rs, lo + (unsigned)(((i * TN + j) * 4 + q) * 4096), sl * SLAB, 16);
              const float4 v = *reinterpret_cast<const float4*>(&x);
              acc[i][j][4 * q] += v.x;
              acc[i][j][4 * q + 1] += v.y;
              acc[i][j][4 * q + 2] += v.z;
              acc[i][j][4 * q + 3] += v.w;
            }
      }
      if (tid == 0) __hip_atomic_store(p.sk_cnt + tile, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }

    // ------------------------------------------------------------ epilogue
    // acc[i][j][r] -> row m0 + (wm*TM+i)*32 + (r&3) + 8*(r>>2) + 4*h, col n0 + (wn*TN+j)*32 + l32
    if (p.epi == kEpiPartial) {
      if (do_bias && m0 + tid < M) p.bias_part[(int64_t)split * M + m0 + tid] = bsum;
      float* C = p.c + (int64_t)split * M * p.ldc;
      // (dword stores: the store epilogue's 16-B form, quad_transpose16,
      // measured slower on these split-K slabs -- C2 dQ0 68 -> 77 us)
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
      float* red = smem;  // [WN][BM] row partial sums (LDS free after the k loop)
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
      for (int i = 0; i < TM; ++i) {
        int64_t dsts[16];  // scatter rows loaded before the stores (see below)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = m0 + (wm * TM + i) * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
          dsts[r] = row < M ? (p.c_idx ? (int64_t)p.c_idx[row] : (int64_t)row) : -1;
        }
        // (all scatter rows in registers before the first store: see the store
        // epilogue below)
#pragma unroll
        for (int r = 0; r < 16; ++r) asm volatile("" : "+v"(dsts[r]));
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int lrow = (wm * TM + i) * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
          const int row = m0 + lrow;
          if (row >= M) continue;
          float tot = 0.f;
#pragma unroll
          for (int q = 0; q < WN; ++q) tot += red[q * BM + lrow];
          const float nrm = sqrtf(tot);
          const int64_t dst = dsts[r];
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            const int col = n0 + (wn * TN + j) * 32 + l32;
            if (col < N) p.c[dst * p.ldc + col] = acc[i][j][r] / nrm;
          }
          if (p.norms && wn == 0 && l32 == 0) p.norms[row] = nrm;
        }
      }
    } else {
      // (the bias bj came in under the k loop: an epilogue load interleaved with
      // stores that may alias it was re-issued and waited on per element)
      const bool accum = p.epi == kEpiAccum;
      // 16-B rows (quad_transpose16): bias and activation per column first,
      // then per lane four consecutive columns of one row -- its mask /
      // accumulated values one 16-B load, its output one 16-B store (the store
      // tail was bound by store-instruction issue: four times fewer).  Needs
      // 16-B aligned rows of every operand the epilogue touches.
      const bool wide = N % 4 == 0 && p.ldc % 4 == 0 && (reinterpret_cast<uintptr_t>(p.c) & 15) == 0 &&
                        (!p.c2 || (p.ldc2 % 4 == 0 && p.N1 % 4 == 0 && (reinterpret_cast<uintptr_t>(p.c2) & 15) == 0)) &&
                        (!p.mask || (p.ldm % 4 == 0 && (reinterpret_cast<uintptr_t>(p.mask) & 15) == 0));
      if (wide) {
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            float v[16];
#pragma unroll
            for (int r = 0; r < 16; ++r) {
              float x = acc[i][j][r] + bj[j];
              if (p.act) x = lrelu(x);
              v[r] = x;
            }
            quad_transpose16(v, lane);
            const int col = n0 + (wn * TN + j) * 32 + 4 * (l32 >> 2);
            const bool second = p.c2 && col >= p.N1;
            int rows[4];
            int64_t dst[4];
#pragma unroll
            for (int g = 0; g < 4; ++g) {
              rows[g] = m0 + (wm * TM + i) * 32 + (l32 & 3) + 8 * g + 4 * h;
              dst[g] = rows[g] < M && col < N ? (p.c_idx ? (int64_t)p.c_idx[rows[g]] : (int64_t)rows[g]) : -1;
            }
            float4 pre[4];
#pragma unroll
            for (int g = 0; g < 4; ++g) {
              pre[g] = make_float4(0.f, 0.f, 0.f, 0.f);
              if (dst[g] >= 0) {
                if (p.mask) pre[g] = *reinterpret_cast<const float4*>(p.mask + (int64_t)rows[g] * p.ldm + col);
                else if (accum && !second) pre[g] = *reinterpret_cast<const float4*>(p.c + dst[g] * p.ldc + col);
              }
            }
            float4 val[4];
#pragma unroll
            for (int g = 0; g < 4; ++g) {
              float4 x = make_float4(v[4 * g], v[4 * g + 1], v[4 * g + 2], v[4 * g + 3]);
              if (p.mask) {
                x.x *= lrelu_grad(pre[g].x);
                x.y *= lrelu_grad(pre[g].y);
                x.z *= lrelu_grad(pre[g].z);
                x.w *= lrelu_grad(pre[g].w);
              } else if (accum && !second) {
                x.x = pre[g].x + x.x;
                x.y = pre[g].y + x.y;
                x.z = pre[g].z + x.z;
                x.w = pre[g].w + x.w;
              }
              val[g] = x;
              asm volatile("" : "+v"(val[g].x), "+v"(val[g].y), "+v"(val[g].z), "+v"(val[g].w));
            }
#pragma unroll
            for (int g = 0; g < 4; ++g)
              if (dst[g] >= 0)
                *reinterpret_cast<float4*>(second ? p.c2 + (int64_t)rows[g] * p.ldc2 + (col - p.N1)
                                                  : p.c + dst[g] * p.ldc + col) = val[g];
          }
      } else {
      // (the scalar form, any alignment)
      // Per 8 rows of a 32-row block: every load (scatter rows, lrelu' masks, the
      // values an accumulate adds to) is issued before those rows' first store --
      // loads interleaved with stores that may alias them were waited on one
      // element at a time (vmcnt counts the stores too): the C2 layer-1
      // scatter-adds of dh / dcat took ~30 us per launch
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int r0 = 0; r0 < 16; r0 += 8) {
          int dsts[8];
#pragma unroll
          for (int r = 0; r < 8; ++r) {
            const int row = m0 + (wm * TM + i) * 32 + ((r0 + r) & 3) + 8 * ((r0 + r) >> 2) + 4 * h;
            dsts[r] = row < M ? (p.c_idx ? p.c_idx[row] : row) : -1;
          }
          // pre: lrelu'(mask) with a mask, else the values an accumulate adds to
          // (launch_gemm refuses a mask with an accumulate)
          float pre[8][TN];
#pragma unroll
          for (int r = 0; r < 8; ++r) {
            const int row = m0 + (wm * TM + i) * 32 + ((r0 + r) & 3) + 8 * ((r0 + r) >> 2) + 4 * h;
#pragma unroll
            for (int j = 0; j < TN; ++j) {
              const int col = n0 + (wn * TN + j) * 32 + l32;
              const bool ok = dsts[r] >= 0 && col < N;
              float x = 0.f;
              if (p.mask) x = ok ? lrelu_grad(p.mask[(int64_t)row * p.ldm + col]) : 0.f;
              else if (accum && !(p.c2 && col >= p.N1)) x = ok ? p.c[(int64_t)dsts[r] * p.ldc + col] : 0.f;
              pre[r][j] = x;
            }
          }
          // every value and row address is formed (and pinned in registers)
          // before the first store: a use of a loaded value among the stores
          // made the compiler wait for all earlier stores before each one
          // (vmcnt counts stores too) -- ~8 us per 64 x 128 tile, more than the
          // k loop of a K = 128 launch
          float val[8][TN];
          float* rowp[8];
#pragma unroll
          for (int r = 0; r < 8; ++r) {
            rowp[r] = p.c + (int64_t)(dsts[r] < 0 ? 0 : dsts[r]) * p.ldc;
            asm volatile("" : "+v"(rowp[r]));
#pragma unroll
            for (int j = 0; j < TN; ++j) {
              const int col = n0 + (wn * TN + j) * 32 + l32;
              float v = acc[i][j][r0 + r] + bj[j];
              if (p.act) v = lrelu(v);
              if (p.mask) v *= pre[r][j];
              else if (accum && !(p.c2 && col >= p.N1)) v = pre[r][j] + v;
              val[r][j] = v;
              asm volatile("" : "+v"(val[r][j]));
            }
          }
#pragma unroll
          for (int r = 0; r < 8; ++r) {
            const int row = m0 + (wm * TM + i) * 32 + ((r0 + r) & 3) + 8 * ((r0 + r) >> 2) + 4 * h;
            if (row >= M) continue;
#pragma unroll
            for (int j = 0; j < TN; ++j) {
              const int col = n0 + (wn * TN + j) * 32 + l32;
              if (col >= N) continue;
              float* o = p.c2 && col >= p.N1 ? p.c2 + (int64_t)row * p.ldc2 + (col - p.N1) : rowp[r] + col;
              *o = val[r][j];
            }
          }
        }
      }
    }
    // the next tile's stage buffers / the L2-norm partials reuse LDS: wait for
    // this tile's LDS traffic only -- its global stores drain under the next
    // tile's k loop (a __syncthreads would wait for every store to complete)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    PS_PROBE();
#ifdef PS_GEMM_PROBE
    if (blockIdx.x == 0 && tid == 0)
      printf("gemm probe [10ns]: init %d wait0 %d kloop %d epi %d\n", (int)(pt[1] - pt[0]), (int)(pt[2] - pt[1]),
             (int)(pt[3] - pt[2]), (int)(pt[4] - pt[3]));
#endif
  };

  if constexpr (SK) if (p.sk_cnt) {
    // stream-K: the tiles' k-steps laid end to end and cut into equal runs,
    // at least sk_min_units k-steps each (launch_gemm: K-major or ungathered
    // operands, K > 0, no split-K partials)
    SkPlan sk;
    sk.I = (K + BK - 1) / BK;
    sk.U = (int64_t)tiles_m * tiles_n * sk.I;
    if (sk.U == 0) return;
    const int64_t ga = sk.U / p.sk_min_units;
    sk.Ga = (int)(ga < 1 ? 1 : (ga < (int64_t)gridDim.x ? ga : (int64_t)gridDim.x));
    if (sk.Ga >= 8) sk.Ga &= ~7;
    // runs are numbered so that consecutive runs go to blocks b, b+8, ...
    // (one XCD under round-robin placement: a tile's pieces and neighbouring
    // tiles' shared A rows stay in one L2; speed only)
    const int per = sk.Ga >= 8 ? sk.Ga / 8 : sk.Ga;
    const int b = sk.Ga >= 8 ? (int)(blockIdx.x % 8) * per + (int)(blockIdx.x / 8) : (int)blockIdx.x;
    if ((int)blockIdx.x >= sk.Ga) return;
    const int64_t u0 = sk.start(b), u1 = sk.start(b + 1);
    const int t_first = (int)(u0 / sk.I);
    for (int64_t u = u0; u < u1;) {
      const int t = (int)(u / sk.I), i0 = (int)(u - (int64_t)t * sk.I);
      const int i1 = (int)min((int64_t)sk.I, i0 + (u1 - u));
      const bool part = !(i0 == 0 && i1 == sk.I);
      run_item(t / tiles_n, t % tiles_n, 0, i0 * BK, min(K, i1 * BK), part ? t : -1,
               2 * b + (t == t_first ? 0 : 1), sk);
      u += i1 - i0;
    }
    return;
  }

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
  const SkPlan none{};
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
    const int kb = split * kchunk;
    run_item(tm, tn, split, kb, min(K, kb + kchunk), -1, 0, none);
  }
}

// ---------------------------------------------------------------- warp-specialised split-bf16 GEMM
// C = act(A B^T + bias) with A [M][K] (rows gathered by a_idx) and B [N][K]
// both K-major -- the Q projections (pinsage_model.py:196-201).  One
// 512-thread workgroup per CU, persistent over 64 x 128 tiles.  Waves 4-7
// (producers) load fp32 k-blocks of A and B from global memory (coalesced
// rows, two k-blocks ahead in registers), split every element ONCE into its
// bf16 hi / mid / lo pieces (split3's arithmetic: bitwise the in-register
// split of gemm_f32_kernel) and write them to a 3-slot LDS ring of bf16
// planes.  Waves 0-3 (consumers, one per SIMD beside one producer) read
// fragments of the three planes and run only the six products per 16-k step
// (v_mfma_f32_32x32x16_bf16, two 32x32 accumulators per wave): the
// conversions leave the MFMA waves, each element is converted once per tile
// instead of once per wave that reads it, and the VALU work of the producers
// runs beside the MFMAs of the consumers on every SIMD.  Same k order and
// product order as gemm_f32_kernel's split-bf16 path: bitwise its results.
constexpr int kWsBM = 64, kWsBN = 128;
constexpr int kWsRows = kWsBM + kWsBN;  // 192 rows of a k-block

template <int BK>
struct WsGeom {
  static constexpr int RowB = BK * 2 + 16;            // bytes per plane row of a slot (+16: b128 reads spread banks)
  static constexpr int PlaneA = kWsBM * RowB, PlaneB = kWsBN * RowB;
  static constexpr int Slot = 3 * (PlaneA + PlaneB);
  static constexpr int Per = kWsRows * (BK / 4) / 256;  // float4 per producer lane per k-block
};
constexpr int kWsSlots = 3;

__device__ __forceinline__ void ws_split4(const float4& v, uint2& H, uint2& M, uint2& L) {
  unsigned h0, m0, l0, h1, m1, l1;
  split_pair(f32x2{v.x, v.y}, h0, m0, l0);
  split_pair(f32x2{v.z, v.w}, h1, m1, l1);
  H = make_uint2(h0, h1);
  M = make_uint2(m0, m1);
  L = make_uint2(l0, l1);
}

// BK: k per slot; AHEAD: k-blocks a producer lane holds loaded ahead of the
// one it writes (global latency cover); WPC: workgroups per CU
template <int BK, int AHEAD, int WPC>
__global__ __launch_bounds__(512, 2 * WPC) void gemm_ws_kernel(GemmParams p) {
  using Gm = WsGeom<BK>;
  constexpr int PER = Gm::Per;
  extern __shared__ __attribute__((aligned(16))) unsigned char ws_lds[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int M = p.M_dev ? *p.M_dev : p.M;
  const int N = p.N, K = p.K;
  const int tiles_m = (M + kWsBM - 1) / kWsBM, tiles_n = N / kWsBN;
  const int nkb = K / BK;
  const bool producer = wave >= 4;
  // tiles of one row panel go to blocks b, b + 8, ... (one XCD: they share
  // the panel's A rows in its L2; speed only)
  const int G = tiles_m, W = tiles_n;
  const int iters = 8 * ((G + 7) / 8) * W;
  for (int t = blockIdx.x; t < iters; t += gridDim.x) {
    const int xcd = t & 7, s = t >> 3;
    const int tm = (s / W) * 8 + xcd, tn = s % W;
    if (tm >= G) continue;
    const int m0 = tm * kWsBM, n0 = tn * kWsBN;
    if (producer) {
      // lane pl (0..255) owns float4 q = pl + 256 j of the 192 x (BK / 4) grid
      const int pl = tid - 256;
      const float* src[PER];
      int dst[PER];  // byte offset inside a slot, plane 0
#pragma unroll
      for (int j = 0; j < PER; ++j) {
        const int q = pl + 256 * j, r = q / (BK / 4), c4 = q % (BK / 4);
        if (r < kWsBM) {
          const int g = min(m0 + r, M - 1);
          src[j] = p.a + (int64_t)(p.a_idx ? p.a_idx[g] : g) * p.lda + 4 * c4;
          dst[j] = r * Gm::RowB + c4 * 8;
        } else {
          const int rb = r - kWsBM;
          src[j] = p.b + (int64_t)(n0 + rb) * p.ldb + 4 * c4;
          dst[j] = 3 * Gm::PlaneA + rb * Gm::RowB + c4 * 8;
        }
      }
      auto load = [&](int kb, float4 (&v)[PER]) __attribute__((always_inline)) {
#pragma unroll
        for (int j = 0; j < PER; ++j) v[j] = *reinterpret_cast<const float4*>(src[j] + kb * BK);
      };
      auto put = [&](int kb, const float4 (&v)[PER]) __attribute__((always_inline)) {
        unsigned char* slot = ws_lds + (kb % kWsSlots) * Gm::Slot;
#pragma unroll
        for (int j = 0; j < PER; ++j) {
          uint2 H, Mi, L;
          ws_split4(v[j], H, Mi, L);
          const int plane = dst[j] < 3 * Gm::PlaneA ? Gm::PlaneA : Gm::PlaneB;
          *reinterpret_cast<uint2*>(slot + dst[j]) = H;
          *reinterpret_cast<uint2*>(slot + dst[j] + plane) = Mi;
          *reinterpret_cast<uint2*>(slot + dst[j] + 2 * plane) = L;
        }
      };
      // prologue: k-blocks 0 and 1 into slots 0 and 1; v[r] <- k-block 2 + r
      float4 v[AHEAD][PER];
      {
        float4 a0[PER], a1[PER];
        load(0, a0);
        if (nkb > 1) load(1, a1);
#pragma unroll
        for (int r = 0; r < AHEAD; ++r)
          if (2 + r < nkb) load(2 + r, v[r]);
        put(0, a0);
        if (nkb > 1) put(1, a1);
      }
      __syncthreads();
      // iteration kb (consumers on slot kb % 3): k-block kb + 2 (in v[kb %
      // AHEAD]) goes to slot (kb + 2) % 3, which iteration kb - 1 read; then
      // that register set loads k-block kb + 2 + AHEAD
      for (int kb0 = 0; kb0 < nkb; kb0 += AHEAD) {
#pragma unroll
        for (int r = 0; r < AHEAD; ++r) {
          const int kb = kb0 + r;
          if (kb < nkb) {
            if (kb + 2 < nkb) {
              put(kb + 2, v[r]);
              if (kb + 2 + AHEAD < nkb) load(kb + 2 + AHEAD, v[r]);
            }
            __syncthreads();
          }
        }
      }
      __syncthreads();  // (the consumers' epilogue barrier)
    } else {
      const int wm = wave >> 1, wn = wave & 1;
      const int l32 = lane & 31, kh = lane >> 5;
      f32x16 acc[2];
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;
      const int arow = (wm * 32 + l32) * Gm::RowB + 16 * kh;
      const int brow0 = 3 * Gm::PlaneA + (wn * 64 + l32) * Gm::RowB + 16 * kh;
      const int brow1 = brow0 + 32 * Gm::RowB;
      __syncthreads();  // the prologue's slots
      for (int kb = 0; kb < nkb; ++kb) {
        const unsigned char* slot = ws_lds + (kb % kWsSlots) * Gm::Slot;
#pragma unroll
        for (int st = 0; st < BK / 16; ++st) {
          const int ko = 32 * st;  // bytes: 16 k of bf16
          const bf16x8 aH = *reinterpret_cast<const bf16x8*>(slot + arow + ko);
          const bf16x8 aM = *reinterpret_cast<const bf16x8*>(slot + arow + ko + Gm::PlaneA);
          const bf16x8 aL = *reinterpret_cast<const bf16x8*>(slot + arow + ko + 2 * Gm::PlaneA);
          bf16x8 bH[2], bM[2], bL[2];
          bH[0] = *reinterpret_cast<const bf16x8*>(slot + brow0 + ko);
          bM[0] = *reinterpret_cast<const bf16x8*>(slot + brow0 + ko + Gm::PlaneB);
          bL[0] = *reinterpret_cast<const bf16x8*>(slot + brow0 + ko + 2 * Gm::PlaneB);
          bH[1] = *reinterpret_cast<const bf16x8*>(slot + brow1 + ko);
          bM[1] = *reinterpret_cast<const bf16x8*>(slot + brow1 + ko + Gm::PlaneB);
          bL[1] = *reinterpret_cast<const bf16x8*>(slot + brow1 + ko + 2 * Gm::PlaneB);
#define PS_WS2(X, Y)                                                                   \
  acc[0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(X, Y[0], acc[0], 0, 0, 0);          \
  acc[1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(X, Y[1], acc[1], 0, 0, 0);
          PS_WS2(aL, bH)
          PS_WS2(aH, bL)
          PS_WS2(aM, bM)
          PS_WS2(aM, bH)
          PS_WS2(aH, bM)
          PS_WS2(aH, bH)
#undef PS_WS2
        }
        __syncthreads();  // slot kb % 3 is free for k-block kb + 3
      }
      // epilogue: bias (+ LeakyReLU) and the stores, straight from registers
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int col = n0 + wn * 64 + 32 * j + l32;
        const float bj = p.bias ? p.bias[col] : 0.f;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = m0 + wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * kh;
          if (row < M) {
            float v = acc[j][r] + bj;
            if (p.act) v = lrelu(v);
            p.c[(int64_t)row * p.ldc + col] = v;
          }
        }
      }
      __syncthreads();
    }
  }
}

bool gemm_ws_supported(const GemmParams& p) {
  return p.a_kmajor && p.b_kmajor && p.K1 < 0 && !p.a2 && !p.c_idx && !p.c2 && !p.mask && !p.b_split &&
         p.epi == kEpiStore && !p.K_dev && p.K > 0 && p.K % 32 == 0 && p.N % kWsBN == 0 && p.lda % 4 == 0 &&
         p.ldb % 4 == 0;
}

// gemm_ws_kernel's launch: 32-k slots, 3 k-blocks ahead, one workgroup per CU
// (A/B'd against 16-k slots two ahead at two per CU and 32-k slots one ahead:
// slower, removed)
static int launch_gemm_ws(const GemmParams& p, int Mmax, hipStream_t st) {
  constexpr int BK = 32, AHEAD = 3, WPC = 1;
  static bool prepared = false;
  const int lds = kWsSlots * WsGeom<BK>::Slot;
  if (!prepared) {
    PS_CHECK_HIP(hipFuncSetAttribute((const void*)gemm_ws_kernel<BK, AHEAD, WPC>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, lds));
    prepared = true;
  }
  const int tm = (Mmax + kWsBM - 1) / kWsBM;
  const int tiles = tm * (p.N / kWsBN);
  const int iters = 8 * ((tm + 7) / 8) * (p.N / kWsBN);
  int grid = std::min(std::max(tiles, 1), WPC * gemm_slots() / 2);
  grid = std::min(grid, iters);
  hipLaunchKernelGGL((gemm_ws_kernel<BK, AHEAD, WPC>), dim3(grid), dim3(512), lds, st, p);
  PS_CHECK_LAUNCH();
  return kOk;
}

// rows per tile of each cfg (5: gemm_ws_kernel's 64-row tiles)
constexpr int kCfgBM[6] = {128, 64, 32, 64, 64, 64};

// the product arithmetic of GEMMs that do not choose (GemmParams::prec < 0):
// PINSAGE_GEMM_PREC at load, then pinsage_gemm_set_prec
static int g_prec = -1;
int gemm_default_prec() {
  if (g_prec < 0) g_prec = getenv("PINSAGE_GEMM_PREC") ? atoi(getenv("PINSAGE_GEMM_PREC")) : 1;
  return g_prec;
}
void gemm_set_default_prec(int prec) { g_prec = prec; }

int gemm_slots() {
  static const int slots = [] {
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        cus <= 0)
      cus = 256;
    return 2 * cus;
  }();
  return slots;
}

int64_t gemm_sk_slab_floats() { return (int64_t)gemm_slots() * 2 * 64 * 128; }

// Cost model: tiles are dealt round-robin over 256 CUs, so a launch takes
// ~ceil(tiles / 256) tile-times and a tile-time is ~ BM (fixed BN, same K).
// Pick the cheapest; ties go to the larger tile (fewer operand re-reads).
// Exception: 64-row tiles that overflow two resident workgroups per CU but fit
// three go to cfg 3 (64 x 128 x 16, three per CU): one round instead of a full
// round plus a tail of lone workgroups (tools/gemm_bench.py: 10541x512x512
// 73 -> 69 us, 5716x1024x128 32 -> 28 us; at 1024 tiles cfg 3 is slower), and
// so do short-K launches (K <= 256) of more than two 64-row tiles per CU, where
// the per-tile fill and epilogue dominate and a third resident workgroup hides
// them (K = 128, bias + LeakyReLU: 24369 x 512 69 -> 48 us, 49152 x 512
// 100 -> 92 us against the 128 x 128 tiles this model picked before).
int gemm_pick_config(int M, int N, int K, int splits) {
  if (splits > 1) return 0;
  const int64_t tn = (N + 127) / 128;
  const int64_t cus = gemm_slots() / 2;
  const int64_t t64 = ((M + 63) / 64) * tn;
  if (t64 > 2 * cus && (t64 <= 3 * cus || K <= 256)) return 3;
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

// 8 elements per thread: the same split_pair as the GEMM's in-register split,
// so a pre-split operand gives bitwise the same products
__global__ __launch_bounds__(256) void split_planes_kernel(const float* __restrict__ w, int64_t rows,
                                                           int64_t cols, int64_t ldw,
                                                           uint16_t* __restrict__ out) {
  const int64_t per_row = cols / 8, n = rows * per_row;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t r = i / per_row, c = (i - r * per_row) * 8;
  const float4 a = *reinterpret_cast<const float4*>(w + r * ldw + c);
  const float4 b = *reinterpret_cast<const float4*>(w + r * ldw + c + 4);
  bf16x8 H, M, L;
  split3(a, b, H, M, L);
  const int64_t o = r * cols + c, ps = rows * cols;
  *reinterpret_cast<bf16x8*>(out + o) = H;
  *reinterpret_cast<bf16x8*>(out + ps + o) = M;
  *reinterpret_cast<bf16x8*>(out + 2 * ps + o) = L;
}

int launch_split_planes(const float* w, int64_t rows, int64_t cols, int64_t ldw, uint16_t* out,
                        hipStream_t st) {
  PS_REQUIRE(rows >= 0 && cols % 8 == 0 && ldw % 4 == 0 && ldw >= cols &&
                 (uintptr_t)w % 16 == 0 && (uintptr_t)out % 16 == 0,
             kErrArg, "split_planes: cols and ldw must be multiples of 8 and 4, pointers 16-B aligned");
  const int64_t n = rows * (cols / 8);
  if (n == 0) return kOk;
  hipLaunchKernelGGL(split_planes_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, w, rows,
                     cols, ldw, out);
  PS_CHECK_LAUNCH();
  return kOk;
}

// one thread per (row, 8 k): the interleaved table row (IlvOp): stage
// k / 16, chunks plane * 2 + (k % 16) / 8
__global__ __launch_bounds__(256) void split_ilv_kernel(const float* __restrict__ src, int64_t ld, int64_t rows,
                                                        int K, uint16_t* __restrict__ out, int64_t ldo) {
  const int k8 = K / 8;
  const int64_t n = rows * k8;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / k8;
    const int kc = (int)(i - r * k8);
    const float4 a = *reinterpret_cast<const float4*>(src + r * ld + 8 * kc);
    const float4 b = *reinterpret_cast<const float4*>(src + r * ld + 8 * kc + 4);
    bf16x8 H, Md, L;
    split3(a, b, H, Md, L);
    uint16_t* o = out + r * ldo + (kc >> 1) * 48 + (kc & 1) * 8;
    *reinterpret_cast<bf16x8*>(o) = H;
    *reinterpret_cast<bf16x8*>(o + 16) = Md;
    *reinterpret_cast<bf16x8*>(o + 32) = L;
  }
}

int launch_split_ilv(const float* src, int64_t ld, int64_t rows, int K, uint16_t* out, int64_t ldo, hipStream_t st) {
  PS_REQUIRE(K > 0 && K % 16 == 0 && ld % 4 == 0 && ld >= K && ldo % 8 == 0 && ldo >= 3LL * K &&
                 (uintptr_t)src % 16 == 0 && (uintptr_t)out % 16 == 0 && rows >= 0,
             kErrArg, "split_ilv: K a multiple of 16, ld of 4, ldo of 8 and >= 3K, 16-B aligned pointers");
  const int64_t n = rows * (K / 8);
  if (n == 0) return kOk;
  hipLaunchKernelGGL(split_ilv_kernel, dim3((unsigned)std::min<int64_t>((n + 255) / 256, 16384)), dim3(256), 0, st,
                     src, ld, rows, K, out, ldo);
  PS_CHECK_LAUNCH();
  return kOk;
}

template <bool AK, bool BKM>
static void launch_cfg(int cfg, dim3 g, hipStream_t st, const GemmParams& p) {
  if constexpr (BKM) {
    if (p.prec == 1 && p.b_split && (cfg == 0 || cfg == 3)) {  // pre-split B planes
      if (cfg == 0)
        hipLaunchKernelGGL((gemm_f32_kernel<AK, BKM, 2, 2, 2, 2, 16, 4, 2, true, true, false>), g, dim3(256),
                           0, st, p);
      else
        hipLaunchKernelGGL((gemm_f32_kernel<AK, BKM, 2, 2, 1, 2, 16, 4, 3, true, true, false>), g, dim3(256),
                           0, st, p);
      return;
    }
  }
  if (p.prec == 1) {  // split-bf16 products (same tiles, same LDS images)
    if (cfg == 0)
      hipLaunchKernelGGL((gemm_f32_kernel<AK, BKM, 2, 2, 2, 2, 16, 4, 2, true, false, false>), g, dim3(256), 0,
                         st, p);
    else if (cfg == 1)
      hipLaunchKernelGGL((gemm_f32_kernel<AK, BKM, 2, 2, 1, 2, 32, 4, 2, true>), g, dim3(256), 0, st, p);
    else if (cfg == 2)
      hipLaunchKernelGGL((gemm_f32_kernel<AK, BKM, 1, 4, 1, 1, 32, 4, 2, true>), g, dim3(256), 0, st, p);
    else if (cfg == 3)
      hipLaunchKernelGGL((gemm_f32_kernel<AK, BKM, 2, 2, 1, 2, 16, 4, 3, true, false, false>), g, dim3(256), 0,
                         st, p);
    else if constexpr (AK && BKM)
      hipLaunchKernelGGL((gemm_f32_kernel<AK, BKM, 2, 2, 1, 2, 16, 3, 4, true, false, false>), g, dim3(256), 0,
                         st, p);
    else
      hipLaunchKernelGGL((gemm_f32_kernel<AK, BKM, 2, 2, 1, 2, 16, 4, 3, true, false, false>), g, dim3(256), 0,
                         st, p);
    return;
  }
  if (cfg == 0)
    hipLaunchKernelGGL((gemm_f32_kernel<AK, BKM, 2, 2, 2, 2, 16, 4, 2, false, false, false>), g, dim3(256), 0, st,
                       p);
  else if (cfg == 1)
    hipLaunchKernelGGL((gemm_f32_kernel<AK, BKM, 2, 2, 1, 2, 32>), g, dim3(256), 0, st, p);
  else if (cfg == 2)
    hipLaunchKernelGGL((gemm_f32_kernel<AK, BKM, 1, 4, 1, 1, 32>), g, dim3(256), 0, st, p);
  else if (cfg == 3)
    hipLaunchKernelGGL((gemm_f32_kernel<AK, BKM, 2, 2, 1, 2, 16, 4, 3, false, false, false>), g, dim3(256), 0, st,
                       p);
  else if constexpr (AK && BKM)  // four per CU: K-major operands only (no k-row windows)
    hipLaunchKernelGGL((gemm_f32_kernel<AK, BKM, 2, 2, 1, 2, 16, 3, 4, false, false, false>), g, dim3(256), 0, st,
                       p);
  else
    hipLaunchKernelGGL((gemm_f32_kernel<AK, BKM, 2, 2, 1, 2, 16, 4, 3, false, false, false>), g, dim3(256), 0, st,
                       p);
}

// whether the calling thread's last launch_gemm ran stream-K (its k ranges cut
// over blocks: a different fp32 summation order than a whole-K tile)
static thread_local int g_last_sk = 0;
int gemm_last_stream_k() { return g_last_sk; }

int launch_gemm(const GemmParams& p_in, hipStream_t st) {
  GemmParams p = p_in;
  g_last_sk = 0;
  const int Mmax = p.M_dev ? p.M_max : p.M;
  const int Kmax = p.K_dev ? p.K_max : p.K;
  PS_REQUIRE(p.N > 0 && Mmax >= 0 && Kmax >= 0, kErrArg, "gemm: bad sizes");
  if (Mmax == 0) return kOk;
  PS_REQUIRE(p.K % 4 == 0 || p.K_dev, kErrArg, "gemm: K must be a multiple of 4");
  PS_REQUIRE(!p.K_dev || (!p.a_kmajor && !p.b_kmajor), kErrArg,
             "gemm: a device-side K needs M-major A and N-major B");
  PS_REQUIRE(!(p.b_idx && p.b2_idx) || p.b_idx == p.b2_idx, kErrArg,
             "gemm: at most one gathered B segment");
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
  PS_REQUIRE(!(p.mask && p.epi == kEpiAccum), kErrArg, "gemm: a mask with an accumulate epilogue");
  PS_REQUIRE(p.epi != kEpiPartial || (!p.M_dev && !p.c_idx), kErrArg,
             "gemm: split-K partials need a static M");
  PS_REQUIRE(p.sk_min_units >= 1, kErrArg, "gemm: sk_min_units must be positive");
  PS_REQUIRE(p.cfg != 4 || (p.a_kmajor && p.b_kmajor), kErrArg,
             "gemm: cfg 4 (four workgroups per CU) needs K-major A and B");
  if (p.a_ilv || p.b_ilv) {  // interleaved plane tables: cfg 0's 128 x 128 tiles, gathered A rows
    PS_REQUIRE(p.a_ilv && p.a_kmajor && p.b_kmajor && !p.K_dev && p.K % 16 == 0 && p.K1 < 0 &&
                   (p.epi == kEpiStore || p.epi == kEpiAccum) && !p.c2 && p.lda_ilv % 8 == 0 &&
                   p.lda_ilv >= 3LL * p.K && (uintptr_t)p.a_ilv % 16 == 0 &&
                   (p.b_ilv ? p.ldb_ilv % 8 == 0 && p.ldb_ilv >= 3LL * p.K && (uintptr_t)p.b_ilv % 16 == 0
                            : p.b != nullptr),
               kErrArg, "gemm: interleaved planes need A's table, static K % 16 == 0 and a store epilogue");
    g_last_sk = 0;
    const int tiles_m = (Mmax + 127) / 128, tiles_n = (p.N + 127) / 128;
    const int64_t iters = 8LL * ((tiles_m + 7) / 8) * tiles_n;
    const int grid = (int)((std::min<int64_t>(iters, 1024) + 7) / 8 * 8);
    if (p.b_ilv)
      hipLaunchKernelGGL((gemm_f32_kernel<true, true, 2, 2, 2, 2, 16, 4, 2, true, false, false, 1>), dim3(grid),
                         dim3(256), 0, st, p);
    else
      hipLaunchKernelGGL((gemm_f32_kernel<true, true, 2, 2, 2, 2, 16, 4, 2, true, false, false, 2>), dim3(grid),
                         dim3(256), 0, st, p);
    PS_CHECK_LAUNCH();
    return kOk;
  }
  if (p.cfg == 5) {  // the warp-specialised split-bf16 kernel (K-major A and B, store epilogue)
    if (gemm_ws_supported(p) && (p.prec == 1 || (p.prec < 0 && gemm_default_prec() == 1))) {
      g_last_sk = 0;
      return launch_gemm_ws(p, Mmax, st);
    }
    p.cfg = 3;  // a launch it cannot run: the same products and k order on cfg 3's tiles
    p.stream_k = 0;
  }
  PS_REQUIRE(!p.b_split || (p.b_kmajor && p.ldb_split % 8 == 0 && p.ldb_split >= Kmax &&
                            (p.K_dev || p.K % 8 == 0) && (uintptr_t)p.b_split % 16 == 0),
             kErrArg, "gemm: pre-split B needs K-major B, K and ldb_split multiples of 8, 16-B aligned planes");
  if (p.prec < 0) p.prec = gemm_default_prec();
  const int splits = p.epi == kEpiPartial ? p.splits : 1;
  const int Mest = p.M_dev ? (p.M_hint > 0 ? std::min(p.M_hint, Mmax) : Mmax) : p.M;
  int cfg = p.cfg >= 0 ? p.cfg : gemm_pick_config(Mest, p.N, Kmax, splits);
  const int tiles_n = (p.N + 127) / 128;
  const int slots = gemm_slots();

  // stream-K: allowed for whole-tile epilogues with no per-window gathered
  // k-rows; chosen when the tiles do not fill the resident slots evenly
  const bool sk_allowed =
      p.sk_slab && p.sk_cnt && p.stream_k != 0 && p.epi != kEpiPartial && !p.K_dev && p.K > 0 &&
      (p.a_kmajor || !p.a_idx) && (p.b_kmajor || (!p.b_idx && !p.b2_idx));
  bool sk = false;
  if (sk_allowed) {
    // by measurement (tools/gemm_bench.py): stream-K pays for long-K launches
    // whose 32-row tiles leave most slots idle (a lone workgroup per CU runs
    // ~1 us per k-step); the per-piece fill / publish / combine (~8 us) eats
    // the gain on short K and on launches that already fill the chip
    // (the kernels of cfg 1 and 2 carry the schedule: gemm_f32_kernel's SK)
    const int skc = p.stream_k == 1 ? (p.cfg >= 0 ? p.cfg : 1) : 2;
    const int64_t tiles_max = (int64_t)((Mmax + kCfgBM[skc] - 1) / kCfgBM[skc]) * tiles_n;
    if ((skc == 1 || skc == 2) && tiles_max <= p.sk_cnt_len) {
      if (p.stream_k == 1) {
        sk = true;
      } else if (p.cfg < 0) {
        const int64_t tiles = (int64_t)((Mest + kCfgBM[skc] - 1) / kCfgBM[skc]) * tiles_n;
        sk = p.K >= 512 && tiles <= slots / 2;
      }
      if (sk) cfg = skc;
    }
  }
  if (!sk) {
    p.sk_cnt = nullptr;
    p.sk_slab = nullptr;
  }
  g_last_sk = sk ? 1 : 0;
  const int BMc = kCfgBM[cfg];
  const int tiles_m = (Mmax + BMc - 1) / BMc;
  int grid;
  if (sk) {
    grid = slots;
  } else {
    const int G = splits > 1 ? splits : tiles_m, W = splits > 1 ? tiles_m * tiles_n : tiles_n;
    const int64_t iters = 8LL * ((G + 7) / 8) * W;
    grid = (int)(iters < 1024 ? iters : 1024);
    grid = (grid + 7) / 8 * 8;
  }
  dim3 g(grid);
  if (p.a_kmajor && p.b_kmajor) launch_cfg<true, true>(cfg, g, st, p);
  else if (p.a_kmajor && !p.b_kmajor) launch_cfg<true, false>(cfg, g, st, p);
  else if (!p.a_kmajor && p.b_kmajor) launch_cfg<false, true>(cfg, g, st, p);
  else launch_cfg<false, false>(cfg, g, st, p);
  PS_CHECK_LAUNCH();
  return kOk;
}

}  // namespace ps
