// fp32 MFMA GEMM for the PinSage projections (Q, W, G1, G2 and their
// backward products).  C[M,N] = op(A)[M,K] * op(B)[K,N] with:
//   A K-major  ("N"): A(m,k) = a[row(m)*lda + k], row(m) = a_idx ? a_idx[m] : m
//   A M-major  ("T"): A(m,k) = a[row(k)*lda + m], row(k) = a_idx ? a_idx[k] : k
//   B K-major  ("T", nn.Linear weight [N][K]): B(k,n) = b[n*ldb + k]
//   B N-major  ("N"): B(k,n) = b[row(k)*ldb + n], row(k) = b_idx ? b_idx[k] : k
// An optional second K segment (K-major A only) implements torch.cat along K
// without a concat buffer (pinsage_model.py:208).  M and K may be device-side
// counts (data-dependent frontier sizes): the kernel is persistent and reads
// them at run time, so no host sync is needed between frontier and GEMM.
#pragma once
#include "common.h"

namespace ps {

enum GemmEpi : int {
  kEpiStore = 0,    // C = acc (+bias) (lrelu) (*lrelu'(mask))   [C row via c_idx]
  kEpiAccum = 1,    // C += acc (same options)
  kEpiL2Norm = 2,   // y = normalize(lrelu(acc + bias)) per row; norms[m] = ||.||  (N <= 128)
  kEpiPartial = 3,  // split-K slab: C[split][M][N] = acc
};

struct GemmParams {
  int M = 0, N = 0, K = 0;
  const int* M_dev = nullptr;  // if set, M = *M_dev (<= M_max for the grid)
  const int* K_dev = nullptr;  // if set, K = *K_dev
  int M_max = 0, K_max = 0;
  bool a_kmajor = true, b_kmajor = true;
  const float* a = nullptr;
  int64_t lda = 0;
  const int32_t* a_idx = nullptr;
  // second K segment of A (K-major only): used for k >= K1
  int K1 = -1;
  const float* a2 = nullptr;
  int64_t lda2 = 0;
  const int32_t* a2_idx = nullptr;
  const float* b = nullptr;
  int64_t ldb = 0;
  const int32_t* b_idx = nullptr;
  // second N segment of an N-major B (torch.cat along N): columns n >= N1
  int N1 = -1;
  const float* b2 = nullptr;
  int64_t ldb2 = 0;
  const int32_t* b2_idx = nullptr;
  float* c = nullptr;
  int64_t ldc = 0;
  const int32_t* c_idx = nullptr;  // output row scatter
  // split output (kEpiStore/kEpiAccum): columns n >= N1 are stored plainly to
  // c2[m][n - N1] instead of C (so one launch can scatter-add one block of
  // columns and write the rest)
  float* c2 = nullptr;
  int64_t ldc2 = 0;
  // kEpiPartial: column sums of A over this split's K rows -> bias_part[split][M]
  // (the bias gradient of a weight gradient dW = A^T B, A M-major)
  float* bias_part = nullptr;
  int epi = kEpiStore;
  const float* bias = nullptr;
  bool act = false;               // leaky_relu
  const float* mask = nullptr;    // multiply by lrelu'(mask[m*ldm + n])
  int64_t ldm = 0;
  float* norms = nullptr;         // kEpiL2Norm: per-row L2 norms
  int splits = 1;                 // kEpiPartial: split-K count
  int M_hint = 0;                 // expected M (device-side M): picks the block tile
  int cfg = -1;                   // force a tile config 0..5 (tests, tuner); -1 = choose by size
  // stream-K (kEpiStore / kEpiAccum / kEpiL2Norm, static K > 0, K-major or
  // ungathered MN-major operands): the launch's k-steps are cut into equal runs
  // over a full grid, and tiles cut between blocks are combined in-launch.
  // Scratch: gemm_sk_slab_floats() floats and sk_cnt_len zeroed ints (the
  // tickets reset themselves), one set per stream.
  float* sk_slab = nullptr;
  int* sk_cnt = nullptr;
  int64_t sk_cnt_len = 0;
  int stream_k = -1;              // -1 choose by size, 0 off, 1 on (when allowed)
  int sk_min_units = 4;           // k-steps per block at least
  // product arithmetic: 0 = v_mfma_f32_32x32x2_f32 (exact fp32 FMA chains);
  // 1 = split bf16 (each fp32 operand = hi + mid + lo bf16 exactly to 2^-26,
  // six v_mfma_f32_32x32x16_bf16 products per 16-k step, fp32 accumulation:
  // fp32-level error at 2.67x the f32 MFMA rate); K-major A and B only;
  // -1 = the library default (PINSAGE_GEMM_PREC, else 1 where allowed)
  int prec = -1;
  // split-bf16 only, K-major B: B already split into its hi / mid / lo bf16
  // planes (launch_split_planes: three [N][ldb_split] planes, bitwise the
  // kernel's own in-register split), read instead of b.  The kernel then
  // converts A only.  Used by cfg 0 and 3 (the other tiles' rings do not fit
  // the 1.5x larger B image); ignored elsewhere.  K and ldb_split % 8 == 0.
  const uint16_t* b_split = nullptr;
  int64_t ldb_split = 0;
  // split-bf16, K-major A and B read from interleaved plane tables
  // (launch_split_ilv; row strides lda_ilv / ldb_ilv in bf16 elements, >= 3K),
  // A's rows gathered by a_idx; replace a and b.  Static K % 16 == 0, store
  // epilogue; runs cfg 0's 128 x 128 tiles.
  const uint16_t* a_ilv = nullptr;
  const uint16_t* b_ilv = nullptr;
  int64_t lda_ilv = 0, ldb_ilv = 0;
};

// Interleaved plane table of src[rows][K] (GemmParams::a_ilv / b_ilv): row r
// at out + r * ldo (ldo >= 3K bf16 elements, % 8 == 0), K/16 stages of the
// six 16-B chunks hi0 hi1 mid0 mid1 lo0 lo1 (8 k each).  K % 16 == 0.
int launch_split_ilv(const float* src, int64_t ld, int64_t rows, int K, uint16_t* out, int64_t ldo, hipStream_t st);

// hi / mid / lo bf16 planes of a row-major fp32 matrix w[rows][cols] (row
// stride ldw floats): out[p][r][c], plane stride rows*cols (cols % 8 == 0)
int launch_split_planes(const float* w, int64_t rows, int64_t cols, int64_t ldw, uint16_t* out,
                        hipStream_t st);

// default product arithmetic (GemmParams::prec = -1): 0 fp32 MFMA, 1 split bf16
int gemm_default_prec();
void gemm_set_default_prec(int prec);

// slab floats a stream-K launch may use (two partial tiles per resident block)
int64_t gemm_sk_slab_floats();
// resident workgroups of one GEMM launch (two per CU)
int gemm_slots();

// Block-tile configurations (4 waves each): rows x cols, k-depth per stage.
//   0: 128 x 128 x 16  (2x2 waves of 64x64)      large M
//   1:  64 x 128 x 32  (2x2 waves of 32x64)      medium M
//   2:  32 x 128 x 32  (1x4 waves of 32x32)      small M, N = 128 (W projection)
//   3:  64 x 128 x 16  (2x2 waves of 32x64), three workgroups per CU
//   5:  64 x 128 x 32 warp-specialised split bf16 (K-major A and B, store
//       epilogue; other launches run cfg 3), one 512-thread workgroup per CU
int gemm_pick_config(int M, int N, int K, int splits);

int launch_gemm(const GemmParams& p, hipStream_t st);
// 1 if the calling thread's last launch_gemm ran stream-K, else 0
int gemm_last_stream_k();
// whether cfg 5 (gemm_ws_kernel) can run this launch
bool gemm_ws_supported(const GemmParams& p);

}  // namespace ps
