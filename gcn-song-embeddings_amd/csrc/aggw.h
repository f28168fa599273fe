// Aggregation + W projection launcher (aggw.hip), shared by the engine and the C-ABI.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace ps {

// The next layer's Q projection fused into this layer's output tile
// (engine layer 0 -> 1): for every output row f whose node is in the next
// layer's neighbour set N (bit of S_mem[f] in bits), q[rank] = lrelu(y[f]
// Qw^T + Qb), rank = its row in N (prefix count) -- the rows the next layer's
// Q GEMM would compute from y.  Qw is [hid][out] (out = the tile's 128).
struct AggNextQ {
  const int32_t* S_mem = nullptr;           // node id of each output row
  const unsigned long long* bits = nullptr;  // next layer's N bitmap
  const uint32_t* pref = nullptr;            // its per-word prefix counts
  const float* Qw = nullptr;
  const float* Qb = nullptr;
  float* q = nullptr;  // [|N|][hid]
  int hid = 0;
};

// The model head fused into the top layer's 16-row tile (engine: the last
// layer): H1 = lrelu(y G1^T + b1), Z = H1 G2^T on exact fp32 MFMAs, both
// [rows][128] -- what head_fwd_kernel (head.hip) computes from y.
struct AggHead {
  const float* G1w = nullptr;  // [128][128]
  const float* G1b = nullptr;
  const float* G2w = nullptr;  // [128][128]
  float* H1 = nullptr;
  float* Z = nullptr;
};

int agg_w_supported(int64_t d, int64_t hid, int64_t out, int64_t T);
// bytes of W's fragment-order bf16 planes (3 x 128 x (d + hid) x 2)
int64_t agg_w_planes_bytes(int64_t d, int64_t hid);
// whether launch_agg_w runs the pipelined 32-row form (which reads W from its
// bf16 planes) at an expected row count S_est
int agg_w_uses_planes(int64_t d, int64_t hid, int64_t out, int64_t T, int64_t S_est);
// whether fusing the next layer's Q projection (AggNextQ) is expected to pay
// at S_est rows: the 32-row form runs and its tiles fit one pass over the CUs
// (the fused products lengthen every tile; a second pass of tiles doubles that)
int agg_w_next_q_pays(int64_t d, int64_t hid, int64_t T, int64_t S_est);
// W [128][K] -> the pipelined form's fragment-order bf16 planes
int launch_split_wplanes(const float* W, int64_t ldw, int K, uint16_t* planes, hipStream_t st);
// next (optional): fuse the next layer's Q projection; *next_done is set to 1
// when the chosen kernel form did it (the 32-row forms), else 0.
// planes (optional, agg_w_planes_bytes): lets the 32-row form run pipelined
// (agg_w_uses_planes); planes_ready 0: split W into them first, 1: they
// already hold W (launch_split_wplanes)
// head (optional): fuse the model head (AggHead); *head_done is set to 1 when
// the chosen kernel form did it (the 16-row form), else 0.
int launch_agg_w(const float* h, int64_t ldh, int d, const int32_t* self_src, const float* q, int hid,
                 const int32_t* loc, const float* wloc, int T, const int* nS, int64_t n_static, int64_t S_max,
                 const float* W, const float* bias, float* y, float* nrm, float* agg, hipStream_t st,
                 const AggNextQ* next = nullptr, int* next_done = nullptr, uint16_t* planes = nullptr,
                 int planes_ready = 0, const AggHead* head = nullptr, int* head_done = nullptr);

}  // namespace ps
