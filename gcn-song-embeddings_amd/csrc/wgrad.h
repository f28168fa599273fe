// Long-K weight gradients with in-launch split combine and fused Adam
// (wgrad.hip): dW[M][N] = A^T [B || B2], db[M] = column sums of A.
#pragma once
#include "common.h"

namespace ps {

struct KwParams {
  const float* A = nullptr;  // [K][M] row-major
  int64_t lda = 0;
  int M = 0;
  const float* B = nullptr;  // columns < N1: B[b_idx ? b_idx[k] : k][n]
  int64_t ldb = 0;
  const int32_t* b_idx = nullptr;
  int N1 = -1;               // columns >= N1 from B2 (torch.cat along N); N1 % 64 == 0
  const float* B2 = nullptr;
  int64_t ldb2 = 0;
  const int32_t* b2_idx = nullptr;
  int N = 0;
  const int* K_dev = nullptr;  // device row count (else K_max rows)
  int K_max = 0;
  float* dst = nullptr;       // [M][ld_dst]
  int64_t ld_dst = 0;
  float* dst_b = nullptr;     // [M] or null
  AdamSlice ad;               // ad.p set: Adam on the slice (dst's layout)
  // split scratch: slab wgrad_kw_slab_floats, bslab wgrad_kw_bslab_floats,
  // cnt wgrad_kw_tickets ints zeroed once (the tickets reset themselves)
  float* slab = nullptr;
  float* bslab = nullptr;
  int* cnt = nullptr;
  // pre-split operands (wgrad_pl_kernel): A and B as hi / mid / lo bf16
  // planes [3][rows][ld] (plane strides a3_ps / b3_ps elements; row strides lda
  // / ldb elements; B rows gathered by b_idx), the exact split the fp32 form
  // does in registers, so the products are the same; no B2 segment
  const uint16_t* A3 = nullptr;
  int64_t a3_ps = 0;
  const uint16_t* B3 = nullptr;
  int64_t b3_ps = 0;
  int S = 0;                  // K splits (0: wgrad_kw_splits)
  int form = 0;               // 0: 8 waves, 128-KiB ring; 1: 4 waves, 64-KiB ring
};

bool wgrad_kw_supported(int M, int N, int N1, bool has_b2);
int wgrad_kw_splits(int M, int N, int64_t K_est, int target = 256);  // ~target workgroups
int64_t wgrad_kw_slab_floats(int M, int N);
int64_t wgrad_kw_bslab_floats(int M);
int64_t wgrad_kw_tickets(int M, int N);
int launch_wgrad_kw(const KwParams& p, hipStream_t st);
// timing-only k loops (probe 1-4: DMAs only, products only, without the split;
// results are wrong) for tools/wgrad_bench.py through pinsage_wgrad_probe
int launch_wgrad_kw_probe(const KwParams& p, int probe, hipStream_t st);

}  // namespace ps
