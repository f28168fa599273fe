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

int agg_w_supported(int64_t d, int64_t hid, int64_t out, int64_t T);
// next (optional): fuse the next layer's Q projection; *next_done is set to 1
// when the chosen kernel form did it (the 32-row form), else 0
int launch_agg_w(const float* h, int64_t ldh, int d, const int32_t* self_src, const float* q, int hid,
                 const int32_t* loc, const float* wloc, int T, const int* nS, int64_t n_static, int64_t S_max,
                 const float* W, const float* bias, float* y, float* nrm, float* agg, hipStream_t st,
                 const AggNextQ* next = nullptr, int* next_done = nullptr);

}  // namespace ps
