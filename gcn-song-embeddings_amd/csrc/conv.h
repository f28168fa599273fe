// Index-table preparation of the frontier's layers (conv.hip layer_prep_kernel).
#pragma once
#include "common.h"

namespace ps {

// For f < *nS (rows of the layer's node set S_l, sorted ids):
//   self_src[f]   = row of h_l holding node f (rank in S_{l-1} via P_bits, or the id at l = 0)
//   loc[f*T+t]    = rank of nb[id][t] in N_l (row of the Q output)
//   wloc[f*T+t]   = normalised importance weight
// for u < *nN (rows of N_l): q_src[u] = row of h_l holding that node; for the
// top layer pos_rank[i] = rank of ids[i] in S_l; z (nullable) = the layer
// below's dY rows (*z_rows x z_n), zeroed.
struct LayerPrep {
  const int32_t* S_mem;
  const int* nS;
  const int32_t* N_mem;
  const int* nN;
  const unsigned long long* N_bits;
  const uint32_t* N_pref;
  const unsigned long long* P_bits;
  const uint32_t* P_pref;
  const int32_t* nb;
  const float* wn;
  int64_t ldT;
  int32_t* self_src;
  int32_t* q_src;
  int32_t* loc;
  float* wloc;
  const unsigned long long* S_bits;
  const uint32_t* S_pref;
  const int64_t* ids;
  int64_t n_ids;
  int32_t* pos_rank;
  float* z;
  int z_n;
  const int* z_rows;
};
constexpr int kMaxPrepLayers = 4;
struct LayerPreps {
  LayerPrep L[kMaxPrepLayers];
  int n, T;
};

// every layer's tables in one launch (S_max / N_max: the sets' capacities)
int launch_layer_preps(const LayerPrep* p, const int64_t* S_max, const int64_t* N_max, int n, int T, hipStream_t st);

}  // namespace ps
