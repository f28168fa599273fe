// Fused importance sampler: random walk + visit counting + libstdc++-exact
// top-k, without the [n_src][n_hops] trace ever reaching HBM.
//
//   sample_neighborhood_topt  pinsage_model.py:88-107 (walk :32-53, visit_prob
//   :96-99, visit_prob.topk(T, 1)) and precompute_neighborhoods_topt :109-132;
//   baselines.py:114-151 PersPageRank.knn (1000 hops).
//
// walk_runs_kernel: one wave per source.  The 64 lanes take 64 consecutive
// hops at a time.  Every hop's three random words are known up front (MT19937
// words expanded per source, or Philox keyed by hop and source), so the restart
// test of hop j-1 tells hop j whether it starts at the source (alpha = 0.85: 85 %
// of hops); the rest start at hop j-1's item and are resolved in a few rounds
// of lane shuffles.  The hops' items land in LDS, are bitonic-sorted, and run-
// length encoded (ballot + popcount) into (id, count) runs in id order; the
// source's own run is dropped (visit_prob[:, self] = 0, :99).  Only the runs
// (<= n_hops x 8 B, typically far fewer) are written, coalesced.
//
// heap_topk_kernel: one LANE per source.  Tensor.topk on CPU runs libstdc++
// partial_sort when k * 64 <= n_all: heap of the first k dense entries, then
// __heap_select over the rest, then __sort_heap.  Only dense entries 0..k-1 and
// nonzero entries (strict '>' against a root >= 0) can enter the heap, so the
// replay runs over the sparse runs alone, step for step (same sift order, so
// equal counts come out in the reference's order).  Each lane keeps its heap
// in LDS as 32-bit entries (count << 16 | ref, ref = id < k or k + run index),
// at an odd stride so the 64 lanes' heaps sit in distinct banks.  The outputs
// are written cooperatively (one source at a time, coalesced).
#include "common.h"

namespace ps {

__device__ __forceinline__ uint4 philox10_(uint64_t key, uint4 c) {
  uint32_t k0 = (uint32_t)key, k1 = (uint32_t)(key >> 32);
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    uint64_t p0 = (uint64_t)0xD2511F53u * c.x;
    uint64_t p1 = (uint64_t)0xCD9E8D57u * c.z;
    uint32_t n0 = (uint32_t)(p1 >> 32) ^ c.y ^ k0;
    uint32_t n2 = (uint32_t)(p0 >> 32) ^ c.w ^ k1;
    c = make_uint4(n0, (uint32_t)p1, n2, (uint32_t)p0);
    if (r < 9) {
      k0 += 0x9E3779B9u;
      k1 += 0xBB67AE85u;
    }
  }
  return c;
}

// One source's walk (one wave, LDS keys[2P]): source index s (its runs' slot),
// graph node src, Philox key seed and stream position pos (kMT: raw words).
template <bool kMT>
__device__ __forceinline__ void walk_runs_body(
    const int64_t* __restrict__ indptr, const int32_t* __restrict__ indices, int64_t s, int64_t src,
    int n_hops, float alpha, const uint32_t* __restrict__ raw, uint64_t seed, uint32_t offset, uint64_t pos,
    int P, uint2* __restrict__ runs, int* __restrict__ n_runs, int* __restrict__ err, uint32_t* keys) {
  const int lane = threadIdx.x;
  const int64_t sb = indptr[src];
  const int64_t sd = indptr[src + 1] - sb;
  const uint32_t* rw = kMT ? raw + s * 3 * (int64_t)n_hops : nullptr;
  int64_t carry_item = src;  // item of the previous round's last hop
  bool carry_rst = true;     // hop -1 "restarted": hop 0 starts at the source
  bool bad = false;
  for (int base = 0; base < n_hops; base += 64) {
    const int j = base + lane;
    const bool active = j < n_hops;
    uint32_t r0 = 0, r1 = 0, r2 = 0;
    if (active) {
      if (kMT) {
        r0 = rw[3 * j];
        r1 = rw[3 * j + 1];
        r2 = rw[3 * j + 2];
      } else {
        const uint4 r = philox10_(seed, make_uint4((uint32_t)j, (uint32_t)pos, (uint32_t)(pos >> 32), offset));
        r0 = r.x;
        r1 = r.y;
        r2 = r.z;
      }
    }
    const bool rst = active && ((float)(r2 & 0xFFFFFFu) * 0x1p-24f < alpha);
    const int up_rst = __shfl_up((int)rst, 1, 64);  // every lane executes the shuffle
    const bool prev_rst = lane == 0 ? carry_rst : up_rst != 0;
    bool known = lane == 0 || prev_rst;
    int64_t start = (lane == 0 && !carry_rst) ? carry_item : src;
    bool done = !active;
    int64_t item = src;
    for (;;) {
      if (known && !done) {
        int64_t b = sb, d = sd;
        if (start != src) {
          b = indptr[start];
          d = indptr[start + 1] - b;
        }
        if (d > 0) {
          const int64_t col = indices[b + (int64_t)(r0 % (uint64_t)d)];
          const int64_t cb = indptr[col];
          const int64_t cd = indptr[col + 1] - cb;
          if (cd > 0) item = indices[cb + (int64_t)(r1 % (uint64_t)cd)];
          else bad = true;
        } else {
          bad = true;
        }
        done = true;
      }
      if (__ballot(!done) == 0) break;
      const int64_t prev_item = __shfl_up(item, 1, 64);
      const bool prev_done = __shfl_up((int)done, 1, 64) != 0;
      if (!known && lane > 0 && prev_done) {
        known = true;
        start = prev_item;
      }
    }
    if (active) keys[j] = (uint32_t)item;
    const int last = min(63, n_hops - 1 - base);
    carry_item = __shfl(item, last, 64);
    carry_rst = __shfl((int)rst, last, 64) != 0;
  }
  if (__ballot(bad)) {
    if (lane == 0) atomicMin(err, (int)(s < 0x7fffffff ? s : 0x7fffffff));
    if (lane == 0) n_runs[s] = 0;
    return;
  }
  for (int i = n_hops + lane; i < P; i += 64) keys[i] = 0xFFFFFFFFu;
  __syncthreads();
  // bitonic sort of the P keys (one wave: __syncthreads is a wave barrier here)
  for (int kk = 2; kk <= P; kk <<= 1) {
    for (int jj = kk >> 1; jj > 0; jj >>= 1) {
      for (int i = lane; i < P; i += 64) {
        const int ixj = i ^ jj;
        if (ixj > i) {
          const uint32_t a = keys[i], b = keys[ixj];
          const bool up = (i & kk) == 0;
          if ((a > b) == up) {
            keys[i] = b;
            keys[ixj] = a;
          }
        }
      }
      __syncthreads();
    }
  }
  // runs: a run starts where the key changes (ballot + popcount compaction of
  // the start positions); its count is the distance to the next start.  The
  // source's own run is dropped.
  uint32_t* run_pos = keys + P;  // [P]
  int nstart = 0;
  for (int base = 0; base < n_hops; base += 64) {
    const int i = base + lane;
    const bool start = i < n_hops && (i == 0 || keys[i] != keys[i - 1]);
    const unsigned long long m = __ballot(start);
    if (start) run_pos[nstart + __popcll(m & ((1ull << lane) - 1))] = (uint32_t)i;
    nstart += __popcll(m);
  }
  __syncthreads();
  const uint32_t self = (uint32_t)src;
  uint2* out = runs + s * (int64_t)n_hops;
  int nr = 0;
  for (int base = 0; base < nstart; base += 64) {
    const int r = base + lane;
    uint32_t id = 0, cnt = 0;
    if (r < nstart) {
      const uint32_t p0 = run_pos[r];
      id = keys[p0];
      cnt = (r + 1 < nstart ? run_pos[r + 1] : (uint32_t)n_hops) - p0;
    }
    const bool keep = r < nstart && id != self;
    const unsigned long long m = __ballot(keep);
    if (keep) out[nr + __popcll(m & ((1ull << lane) - 1))] = make_uint2(id, cnt);
    nr += __popcll(m);
  }
  if (lane == 0) n_runs[s] = nr;
}

template <bool kMT>
__global__ __launch_bounds__(64) void walk_runs_kernel(
    const int64_t* __restrict__ indptr, const int32_t* __restrict__ indices,
    const int64_t* __restrict__ sources, int64_t n_src, int n_hops, float alpha,
    const uint32_t* __restrict__ raw, uint64_t seed, uint32_t offset, int64_t src_base, int P,
    uint2* __restrict__ runs, int* __restrict__ n_runs, int* __restrict__ err) {
  extern __shared__ __attribute__((aligned(16))) uint32_t keys[];  // [P] keys, [P] run starts
  const int64_t s = blockIdx.x;
  if (s >= n_src) return;
  walk_runs_body<kMT>(indptr, indices, s, sources[s], n_hops, alpha, raw, seed, offset, (uint64_t)(src_base + s),
                      P, runs, n_runs, err, keys);
}

// The on-the-fly sampler's walks (fly.hip): sources are C calls' nodes at
// c * id_unit + id, sorted by call, the calls' segment starts and Philox keys
// on the device (seg[0..C], seeds[c * key_stride]); source s of segment c is
// the (s - seg[c])-th of its call (the per-call path's numbering).  The grid
// covers a capacity; sources past *n_src_dev (or seg[C]) return.
template <typename Src>
__global__ __launch_bounds__(64) void walk_runs_seg_kernel(
    const int64_t* __restrict__ indptr, const int32_t* __restrict__ indices, const Src* __restrict__ sources,
    const int* __restrict__ seg, int C, const uint64_t* __restrict__ seeds, int key_stride, int64_t id_unit,
    int n_hops, float alpha, uint32_t offset, int P, uint2* __restrict__ runs, int* __restrict__ n_runs,
    int* __restrict__ err) {
  extern __shared__ __attribute__((aligned(16))) uint32_t keys[];
  const int64_t s = blockIdx.x;
  if (s >= (int64_t)seg[C]) return;
  int c = 0;
  while (c + 1 < C && s >= (int64_t)seg[c + 1]) ++c;
  const int64_t src = (int64_t)sources[s] - (int64_t)c * id_unit;
  walk_runs_body<false>(indptr, indices, s, src, n_hops, alpha, nullptr, seeds[(int64_t)c * key_stride], offset,
                        (uint64_t)(s - seg[c]), P, runs, n_runs, err, keys);
}

// ---------------------------------------------------------------- lane-per-source heap replay
// libstdc++ __adjust_heap / __push_heap / __make_heap / __pop_heap /
// __heap_select / __sort_heap over 32-bit entries ordered by count (bits 16..31).
__device__ __forceinline__ bool hgt(uint32_t a, uint32_t b) { return (a >> 16) > (b >> 16); }

__device__ __forceinline__ void h_push(uint32_t* f, int hole, int top, uint32_t v) {
  int parent = (hole - 1) / 2;
  while (hole > top && hgt(f[parent], v)) {
    f[hole] = f[parent];
    hole = parent;
    parent = (hole - 1) / 2;
  }
  f[hole] = v;
}
__device__ __forceinline__ void h_adjust(uint32_t* f, int hole, int len, uint32_t v) {
  const int top = hole;
  int child = hole;
  while (child < (len - 1) / 2) {
    child = 2 * (child + 1);
    if (hgt(f[child], f[child - 1])) child--;
    f[hole] = f[child];
    hole = child;
  }
  if ((len & 1) == 0 && child == (len - 2) / 2) {
    child = 2 * (child + 1);
    f[hole] = f[child - 1];
    hole = child - 1;
  }
  h_push(f, hole, top, v);
}

__global__ __launch_bounds__(64) void heap_topk_kernel(
    const uint2* __restrict__ runs, const int* __restrict__ n_runs, int64_t n_src, int n_hops, int k,
    int kp, int G, double* __restrict__ out_w, int64_t* __restrict__ out_nb, float* __restrict__ out_wn,
    int32_t* __restrict__ out_nb32, int T_norm, const int* __restrict__ n_src_dev) {
  extern __shared__ __attribute__((aligned(16))) uint32_t heaps[];  // [G][kp]
  __shared__ double rowsum[64];
  const int lane = threadIdx.x;
  if (n_src_dev) n_src = min(n_src, (int64_t)*n_src_dev);  // (a capacity grid: the count on the device)
  const int64_t s0 = (int64_t)blockIdx.x * G;
  const int64_t s = s0 + lane;
  uint32_t* f = heaps + lane * kp;
  if (lane < G && s < n_src) {
    const uint2* rs = runs + s * (int64_t)n_hops;
    const int nr = n_runs[s];
    for (int j = 0; j < k; ++j) f[j] = (uint32_t)j;  // dense entries 0..k-1, count 0
    int r = 0;
    for (; r < nr; ++r) {  // runs are in id order: ids < k set their dense entry
      const uint2 e = rs[r];
      if ((int64_t)e.x >= k) break;
      f[e.x] = (e.y << 16) | e.x;
    }
    // __make_heap
    if (k >= 2) {
      for (int parent = (k - 2) / 2;; --parent) {
        h_adjust(f, parent, k, f[parent]);
        if (parent == 0) break;
      }
    }
    // __heap_select over the sparse tail: pop_heap(first, middle, i) when *i > *first.
    // The runs are read 8 at a time ahead of their comparisons (one load per
    // run inside the loop left every iteration waiting on its own global
    // load: with few sources per launch, as on the fly, that latency was the
    // kernel) and the root stays in a register between adjustments.
    uint32_t root = f[0];
    for (; r < nr; r += 8) {
      uint2 b[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) b[i] = rs[min(r + i, nr - 1)];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const uint32_t v = (b[i].y << 16) | (uint32_t)(k + r + i);
        if (r + i < nr && hgt(v, root)) {
          h_adjust(f, 0, k, v);
          root = f[0];
        }
      }
    }
    // __sort_heap
    for (int len = k; len > 1;) {
      --len;
      const uint32_t v = f[len];
      f[len] = f[0];
      h_adjust(f, 0, len, v);
    }
    double sum = 0.0;
    for (int j = 0; j < T_norm; ++j) sum += (double)(f[j] >> 16) / (double)n_hops;
    rowsum[lane] = sum;
  }
  __syncthreads();
  // outputs, one source at a time (coalesced rows)
  const int64_t nb_blk = min((int64_t)G, n_src - s0);
  for (int q = 0; q < nb_blk; ++q) {
    const int64_t sq = s0 + q;
    const uint32_t* fq = heaps + q * kp;
    const uint2* rq = runs + sq * (int64_t)n_hops;
    for (int j = lane; j < k; j += 64) {
      const uint32_t e = fq[j];
      const uint32_t ref = e & 0xFFFFu;
      const int64_t id = ref < (uint32_t)k ? (int64_t)ref : (int64_t)rq[ref - k].x;
      const double w = (double)(e >> 16) / (double)n_hops;
      if (out_w) {
        out_w[sq * k + j] = w;
        out_nb[sq * k + j] = id;
      }
      if (out_wn && j < T_norm) {
        out_wn[sq * T_norm + j] = (float)(w / rowsum[q]);
        out_nb32[sq * T_norm + j] = (int32_t)id;
      }
    }
  }
}

int ppr_walk_lds_bytes(int n_hops, int* P_out) {
  int P = 64;
  while (P < n_hops) P <<= 1;
  if (P_out) *P_out = P;
  return 2 * P * 4;  // keys + run starts
}

int launch_walk_runs(const int64_t* indptr, const int32_t* indices, const int64_t* sources,
                     int64_t n_src, int n_hops, float alpha, const uint32_t* raw, uint64_t seed,
                     uint32_t offset, int64_t src_base, uint2* runs, int* n_runs, int* err,
                     hipStream_t st) {
  if (n_src <= 0) return kOk;
  int P;
  const int lds = ppr_walk_lds_bytes(n_hops, &P);
  PS_REQUIRE(lds <= 64 * 1024, kErrArg, "ppr_topk: n_hops too large");
  if (raw)
    hipLaunchKernelGGL(walk_runs_kernel<true>, dim3((unsigned)n_src), dim3(64), lds, st, indptr,
                       indices, sources, n_src, n_hops, alpha, raw, seed, offset, src_base, P, runs,
                       n_runs, err);
  else
    hipLaunchKernelGGL(walk_runs_kernel<false>, dim3((unsigned)n_src), dim3(64), lds, st, indptr,
                       indices, sources, n_src, n_hops, alpha, raw, seed, offset, src_base, P, runs,
                       n_runs, err);
  PS_CHECK_LAUNCH();
  return kOk;
}

int launch_heap_topk(const uint2* runs, const int* n_runs, int64_t n_src, int n_hops, int k,
                     double* out_w, int64_t* out_nb, float* out_wn, int32_t* out_nb32, int T_norm,
                     hipStream_t st, const int* n_src_dev) {
  if (n_src <= 0) return kOk;
  const int kp = k | 1;
  // sources per block: 64 (one per lane) while the heaps fit 64 KB of LDS,
  // fewer for large k (PersPageRank's k up to 1000)
  int G = 64;
  while (G > 1 && G * kp * 4 > 64 * 1024) G >>= 1;
  // few sources (the on-the-fly sampler's nodesets): fewer lanes per block, so
  // more CUs share the sources and a wave's divergent heap adjustments are the
  // union over fewer lanes (each lane's replay is serial either way)
  while (G > 1 && ceil_div(n_src, G) < 1024) G >>= 1;
  const int lds = G * kp * 4;
  PS_REQUIRE(lds <= 64 * 1024, kErrArg, "ppr_topk: k too large for the LDS heaps");
  hipLaunchKernelGGL(heap_topk_kernel, dim3((unsigned)ceil_div(n_src, G)), dim3(64), lds, st, runs,
                     n_runs, n_src, n_hops, k, kp, G, out_w, out_nb, out_wn, out_nb32, T_norm, n_src_dev);
  PS_CHECK_LAUNCH();
  return kOk;
}

// n_src_cap sources at most, the count in seg[C] (sources int64 or int32)
template <typename Src>
static int launch_walk_runs_seg_t(const int64_t* indptr, const int32_t* indices, const Src* sources,
                                  int64_t n_src_cap, const int* seg, int C, const uint64_t* seeds, int key_stride,
                                  int64_t id_unit, int n_hops, float alpha, uint32_t offset, uint2* runs,
                                  int* n_runs, int* err, hipStream_t st) {
  if (n_src_cap <= 0) return kOk;
  int P;
  const int lds = ppr_walk_lds_bytes(n_hops, &P);
  PS_REQUIRE(lds <= 64 * 1024, kErrArg, "ppr_topk: n_hops too large");
  hipLaunchKernelGGL(walk_runs_seg_kernel<Src>, dim3((unsigned)n_src_cap), dim3(64), lds, st, indptr, indices,
                     sources, seg, C, seeds, key_stride, id_unit, n_hops, alpha, offset, P, runs, n_runs, err);
  PS_CHECK_LAUNCH();
  return kOk;
}
int launch_walk_runs_seg(const int64_t* indptr, const int32_t* indices, const int64_t* sources64,
                         const int32_t* sources32, int64_t n_src_cap, const int* seg, int C, const uint64_t* seeds,
                         int key_stride, int64_t id_unit, int n_hops, float alpha, uint32_t offset, uint2* runs,
                         int* n_runs, int* err, hipStream_t st) {
  if (sources64)
    return launch_walk_runs_seg_t(indptr, indices, sources64, n_src_cap, seg, C, seeds, key_stride, id_unit, n_hops,
                                  alpha, offset, runs, n_runs, err, st);
  return launch_walk_runs_seg_t(indptr, indices, sources32, n_src_cap, seg, C, seeds, key_stride, id_unit, n_hops,
                                alpha, offset, runs, n_runs, err, st);
}

}  // namespace ps
