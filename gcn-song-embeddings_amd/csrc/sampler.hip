// Importance sampler kernels for gfx950: random walk with restart over the
// track-collection CSR, visit counting, libstdc++-exact top-k.
//
//   do_random_walks              pinsage_model.py:32-53   -> walk_kernel
//   sample_neighborhood (dense)  pinsage_model.py:88-101  -> visit_dense_*
//   topk(T, 1) on visit_prob     pinsage_model.py:103-107 -> visit_topk_kernel
//
// RNG modes: "mt19937" consumes torch's CPU MT19937 stream exactly as the
// reference does (3 draws per hop: collection, item, restart test).  The
// stream is expanded on the GPU: the host snapshots the generator at the start
// of every chunk of sources, one workgroup per chunk re-twists and tempers its
// words into HBM.  "philox" is a counter-based Philox4x32-10 keyed by
// (seed; hop, source position, offset) with a bit-exact CPU twin in oracle/.
#include "common.h"
#include "mt19937.h"

namespace ps {

// ---------------------------------------------------------------- MT expand
__device__ __forceinline__ uint32_t mt_tw(uint32_t u, uint32_t v) {
  uint32_t y = (u & 0x80000000u) | (v & 0x7fffffffu);
  return (y >> 1) ^ ((v & 1u) ? 0x9908b0dfu : 0u);
}
__device__ __forceinline__ uint32_t mt_temper(uint32_t y) {
  y ^= (y >> 11);
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  y ^= (y >> 18);
  return y;
}

// In-LDS twist of the 624-word state by a 256-thread block in three dependent
// phases (i < 227 reads only old words; 227..453 reads words 0..226 of the new
// state; 454..623 reads 227..396 of the new state, 623 also new word 0).
__device__ __forceinline__ void mt_twist_block(uint32_t* s) {
  const int t = threadIdx.x;
  uint32_t r = 0;
  if (t < 227) r = s[t + 397] ^ mt_tw(s[t], s[t + 1]);
  __syncthreads();
  if (t < 227) s[t] = r;
  __syncthreads();
  if (t < 227) r = s[t] ^ mt_tw(s[t + 227], s[t + 228]);
  __syncthreads();
  if (t < 227) s[t + 227] = r;
  __syncthreads();
  if (t < 170) {
    const int i = t + 454;
    r = s[i - 227] ^ mt_tw(s[i], i == 623 ? s[0] : s[i + 1]);
  }
  __syncthreads();
  if (t < 170) s[t + 454] = r;
  __syncthreads();
}

__global__ __launch_bounds__(256) void mt_expand_kernel(const MTChunk* __restrict__ chunks,
                                                        int64_t words_per_chunk, int64_t total,
                                                        uint32_t* __restrict__ out) {
  __shared__ uint32_t s[MTState::N];
  const MTChunk* c = chunks + blockIdx.x;
  for (int i = threadIdx.x; i < MTState::N; i += blockDim.x) s[i] = c->s[i];
  int64_t next = c->next, avail = c->avail;
  const int64_t base = (int64_t)blockIdx.x * words_per_chunk;
  int64_t n = total - base;
  if (n > words_per_chunk) n = words_per_chunk;
  __syncthreads();
  int64_t done = 0;
  while (done < n) {
    if (avail == 0) {
      mt_twist_block(s);
      next = 0;
      avail = MTState::N;
    }
    int64_t take = avail < n - done ? avail : n - done;
    for (int64_t t = threadIdx.x; t < take; t += blockDim.x)
      out[base + done + t] = mt_temper(s[next + t]);
    done += take;
    next += take;
    avail -= take;
    __syncthreads();
  }
}

// ---------------------------------------------------------------- Philox4x32-10
__device__ __forceinline__ uint4 philox10(uint64_t key, uint4 c) {
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

// ---------------------------------------------------------------- walk
// One lane per source.  The source's own CSR row is cached in registers: with
// alpha = 0.85 most hops restart there.  trace is int32 [n_src][n_hops].
template <bool kMT>
__global__ __launch_bounds__(256) void walk_kernel(
    const int64_t* __restrict__ indptr, const int32_t* __restrict__ indices,
    const int64_t* __restrict__ sources, int64_t n_src, int64_t n_hops, float alpha,
    const uint32_t* __restrict__ raw, uint64_t seed, uint32_t offset, int64_t src_base,
    int32_t* __restrict__ trace, int* __restrict__ err) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_src) return;
  const int64_t src = sources[i];
  const int64_t sb = indptr[src];
  const int64_t sd = indptr[src + 1] - sb;
  int64_t item = src;
  const uint32_t* rw = kMT ? raw + i * 3 * n_hops : nullptr;
  int32_t* tr = trace + i * n_hops;
  const uint64_t pos = (uint64_t)(src_base + i);
  for (int64_t j = 0; j < n_hops; ++j) {
    uint32_t r0, r1, r2;
    if (kMT) {
      r0 = rw[3 * j];
      r1 = rw[3 * j + 1];
      r2 = rw[3 * j + 2];
    } else {
      uint4 r = philox10(seed, make_uint4((uint32_t)j, (uint32_t)pos, (uint32_t)(pos >> 32), offset));
      r0 = r.x;
      r1 = r.y;
      r2 = r.z;
    }
    int64_t b = sb, d = sd;
    if (item != src) {
      b = indptr[item];
      d = indptr[item + 1] - b;
    }
    if (d <= 0) {
      atomicMin(err, (int)(i < 0x7fffffff ? i : 0x7fffffff));
      return;
    }
    const int64_t col = indices[b + (int64_t)(r0 % (uint64_t)d)];
    const int64_t cb = indptr[col];
    const int64_t cd = indptr[col + 1] - cb;
    if (cd <= 0) {
      atomicMin(err, (int)(i < 0x7fffffff ? i : 0x7fffffff));
      return;
    }
    item = indices[cb + (int64_t)(r1 % (uint64_t)cd)];
    tr[j] = (int32_t)item;
    const float u = (float)(r2 & 0xFFFFFFu) * 0x1p-24f;
    if (u < alpha) item = src;
  }
}

// ---------------------------------------------------------------- libstdc++ heap / introselect
// Elements are (visit count, node id); ordering is by count only, as the
// reference's comparator orders by value = count / n_hops (strictly monotone,
// exact ties preserved).  These replay libstdc++'s __adjust_heap, __make_heap,
// __pop_heap, __heap_select, __sort_heap, __introselect, std::sort step by
// step, so equal counts come out in the reference's order.
struct CE {
  uint32_t c, i;
};
__device__ __forceinline__ bool gt(const CE& a, const CE& b) { return a.c > b.c; }

__device__ void push_heap_(CE* f, int64_t hole, int64_t top, CE v) {
  int64_t parent = (hole - 1) / 2;
  while (hole > top && gt(f[parent], v)) {
    f[hole] = f[parent];
    hole = parent;
    parent = (hole - 1) / 2;
  }
  f[hole] = v;
}
__device__ void adjust_heap_(CE* f, int64_t hole, int64_t len, CE v) {
  const int64_t top = hole;
  int64_t child = hole;
  while (child < (len - 1) / 2) {
    child = 2 * (child + 1);
    if (gt(f[child], f[child - 1])) child--;
    f[hole] = f[child];
    hole = child;
  }
  if ((len & 1) == 0 && child == (len - 2) / 2) {
    child = 2 * (child + 1);
    f[hole] = f[child - 1];
    hole = child - 1;
  }
  push_heap_(f, hole, top, v);
}
__device__ void make_heap_(CE* f, int64_t len) {
  if (len < 2) return;
  for (int64_t parent = (len - 2) / 2;; --parent) {
    CE v = f[parent];
    adjust_heap_(f, parent, len, v);
    if (parent == 0) return;
  }
}
__device__ __forceinline__ void pop_heap_(CE* f, int64_t len, CE* result) {
  CE v = *result;
  *result = f[0];
  adjust_heap_(f, 0, len, v);
}
__device__ void heap_select_(CE* f, int64_t mid, int64_t last) {
  make_heap_(f, mid);
  for (int64_t i = mid; i < last; ++i)
    if (gt(f[i], f[0])) pop_heap_(f, mid, &f[i]);
}
__device__ void sort_heap_(CE* f, int64_t len) {
  while (len > 1) {
    --len;
    pop_heap_(f, len, &f[len]);
  }
}
__device__ __forceinline__ void swp(CE* a, CE* b) {
  CE t = *a;
  *a = *b;
  *b = t;
}
__device__ void median_to_first_(CE* r, CE* a, CE* b, CE* c) {
  if (gt(*a, *b)) {
    if (gt(*b, *c)) swp(r, b);
    else if (gt(*a, *c)) swp(r, c);
    else swp(r, a);
  } else if (gt(*a, *c)) swp(r, a);
  else if (gt(*b, *c)) swp(r, c);
  else swp(r, b);
}
__device__ CE* unguarded_partition_(CE* first, CE* last, CE* pivot) {
  for (;;) {
    while (gt(*first, *pivot)) ++first;
    --last;
    while (gt(*pivot, *last)) --last;
    if (!(first < last)) return first;
    swp(first, last);
    ++first;
  }
}
__device__ CE* partition_pivot_(CE* first, CE* last) {
  CE* mid = first + (last - first) / 2;
  median_to_first_(first, first + 1, mid, last - 1);
  return unguarded_partition_(first + 1, last, first);
}
__device__ void linear_insert_(CE* last) {
  CE v = *last;
  CE* nx = last - 1;
  while (gt(v, *nx)) {
    *last = *nx;
    last = nx;
    --nx;
  }
  *last = v;
}
__device__ void insertion_sort_(CE* first, CE* last) {
  if (first == last) return;
  for (CE* i = first + 1; i != last; ++i) {
    if (gt(*i, *first)) {
      CE v = *i;
      for (CE* p = i; p != first; --p) *p = *(p - 1);
      *first = v;
    } else {
      linear_insert_(i);
    }
  }
}
__device__ __forceinline__ int lg2_(int64_t n) { return 63 - __clzll((unsigned long long)n); }
__device__ void introselect_(CE* first, CE* nth, CE* last, int depth) {
  while (last - first > 3) {
    if (depth == 0) {
      heap_select_(first, (nth + 1) - first, last - first);
      swp(first, nth);
      return;
    }
    --depth;
    CE* cut = partition_pivot_(first, last);
    if (cut <= nth) first = cut;
    else last = cut;
  }
  insertion_sort_(first, last);
}
// std::sort = introsort loop (recursion unrolled with an explicit stack) +
// final insertion sort; the recursion order does not affect the result.
__device__ void std_sort_(CE* first, CE* last) {
  if (last - first < 2) return;
  struct Fr {
    CE* f;
    CE* l;
    int d;
  } stk[64];
  int sp = 0;
  stk[sp++] = {first, last, lg2_(last - first) * 2};
  while (sp > 0) {
    Fr fr = stk[--sp];
    CE* f = fr.f;
    CE* l = fr.l;
    int depth = fr.d;
    while (l - f > 16) {
      if (depth == 0) {
        heap_select_(f, l - f, l - f);
        sort_heap_(f, l - f);
        break;
      }
      --depth;
      CE* cut = partition_pivot_(f, l);
      stk[sp++] = {cut, l, depth};
      l = cut;
    }
  }
  if (last - first > 16) {
    insertion_sort_(first, first + 16);
    for (CE* i = first + 16; i != last; ++i) linear_insert_(i);
  } else {
    insertion_sort_(first, last);
  }
}

// ---------------------------------------------------------------- visit counting + top-k
// One wave per source.  The source's n_hops visits are bitonic-sorted in LDS,
// run-length encoded into (id, count) runs in id order, the source's own id is
// zeroed (pinsage_model.py:99), then the top-k is selected with the exact
// libstdc++ algorithm the reference's Tensor.topk runs:
//   k*64 <= n_all: partial_sort. Only the dense entries 0..k-1 and NONZERO
//     entries >= k can enter the heap (strict '>' against a root >= 0), so the
//     heap is replayed over the sparse runs alone.
//   otherwise: nth_element + sort of the first k-1 over the dense row, which is
//     materialised in `dense_scratch` (only for graphs with n_all < 64k).
__global__ __launch_bounds__(64) void visit_topk_kernel(
    const int32_t* __restrict__ trace, const int64_t* __restrict__ sources, int64_t n_src,
    int64_t n_hops, int P, int64_t n_all, int64_t k, CE* __restrict__ dense_scratch,
    double* __restrict__ out_w, int64_t* __restrict__ out_nb, float* __restrict__ out_wn,
    int32_t* __restrict__ out_nb32, int64_t T_norm) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  uint32_t* keys = lds;                  // [P]
  uint32_t* run_pos = lds + P;           // [P] start index of each run
  CE* heap = (CE*)(lds + 2 * P);         // [k]
  const int lane = threadIdx.x;
  const int64_t s = blockIdx.x;
  if (s >= n_src) return;
  const int32_t* tr = trace + s * n_hops;
  for (int i = lane; i < P; i += 64) keys[i] = i < n_hops ? (uint32_t)tr[i] : 0xFFFFFFFFu;
  __syncthreads();
  for (int kk = 2; kk <= P; kk <<= 1) {
    for (int j = kk >> 1; j > 0; j >>= 1) {
      for (int i = lane; i < P; i += 64) {
        const int ixj = i ^ j;
        if (ixj > i) {
          uint32_t a = keys[i], b = keys[ixj];
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
  // run starts via ballot + popcount compaction
  int n_runs = 0;
  for (int base = 0; base < P; base += 64) {
    const int i = base + lane;
    const bool start = i < n_hops && (i == 0 || keys[i] != keys[i - 1]);
    const unsigned long long m = __ballot(start);
    if (start) run_pos[n_runs + __popcll(m & ((1ull << lane) - 1))] = (uint32_t)i;
    n_runs += __popcll(m);
  }
  __syncthreads();
  const uint32_t self = (uint32_t)sources[s];
  const double inv_hops_d = (double)n_hops;
  if (k * 64 <= n_all) {
    if (lane == 0) {
      for (int64_t j = 0; j < k; ++j) heap[j] = CE{0u, (uint32_t)j};
      int r = 0;
      for (; r < n_runs; ++r) {
        const uint32_t id = keys[run_pos[r]];
        if ((int64_t)id >= k) break;
        const uint32_t end = r + 1 < n_runs ? run_pos[r + 1] : (uint32_t)n_hops;
        heap[id].c = id == self ? 0u : end - run_pos[r];
      }
      make_heap_(heap, k);
      for (; r < n_runs; ++r) {
        const uint32_t id = keys[run_pos[r]];
        if (id == self) continue;
        const uint32_t end = r + 1 < n_runs ? run_pos[r + 1] : (uint32_t)n_hops;
        CE v{end - run_pos[r], id};
        if (gt(v, heap[0])) {
          CE tmp = v;
          pop_heap_(heap, k, &tmp);
        }
      }
      sort_heap_(heap, k);
    }
  } else {
    CE* D = dense_scratch + s * n_all;
    for (int64_t j = lane; j < n_all; j += 64) D[j] = CE{0u, (uint32_t)j};
    __threadfence_block();
    __syncthreads();
    for (int r = lane; r < n_runs; r += 64) {
      const uint32_t id = keys[run_pos[r]];
      const uint32_t end = r + 1 < n_runs ? run_pos[r + 1] : (uint32_t)n_hops;
      if (id != self && id < n_all) D[id].c = end - run_pos[r];
    }
    __threadfence_block();
    __syncthreads();
    if (lane == 0) {
      introselect_(D, D + k - 1, D + n_all, lg2_(n_all) * 2);
      std_sort_(D, D + k - 1);
      for (int64_t j = 0; j < k; ++j) heap[j] = D[j];
    }
  }
  __syncthreads();
  // outputs: reference dtype (f64 weights, i64 ids) and/or the device table
  // (first T_norm columns, weights normalised by their row sum, f32 / i32).
  double rowsum = 0.0;
  if (out_wn) {
    for (int64_t j = 0; j < T_norm; ++j) rowsum += (double)heap[j].c / inv_hops_d;
  }
  for (int64_t j = lane; j < k; j += 64) {
    const CE e = heap[j];
    const double w = (double)e.c / inv_hops_d;
    if (out_w) {
      out_w[s * k + j] = w;
      out_nb[s * k + j] = (int64_t)e.i;
    }
    if (out_wn && j < T_norm) {
      out_wn[s * T_norm + j] = (float)(w / rowsum);
      out_nb32[s * T_norm + j] = (int32_t)e.i;
    }
  }
}

// Dense visit_prob (pinsage_model.py:96-99): counts by f64 atomics (exact for
// integers), then / n_hops and the self column zeroed.
__global__ void visit_dense_count_kernel(const int32_t* __restrict__ trace, int64_t n_src,
                                         int64_t n_hops, int64_t n_all, double* __restrict__ dense) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n_src * n_hops) return;
  const int64_t s = e / n_hops;
  atomicAdd(dense + s * n_all + trace[e], 1.0);
}
__global__ void visit_dense_norm_kernel(const int64_t* __restrict__ sources, int64_t n_src,
                                        int64_t n_hops, int64_t n_all, double* __restrict__ dense) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n_src * n_all) return;
  const int64_t s = e / n_all, j = e - s * n_all;
  dense[e] = (j == sources[s]) ? 0.0 : dense[e] / (double)n_hops;
}

// ---------------------------------------------------------------- host launchers
int launch_mt_expand(const MTChunk* chunks_dev, int64_t n_chunks, int64_t words_per_chunk,
                     int64_t total, uint32_t* out, hipStream_t st) {
  if (n_chunks <= 0) return kOk;
  hipLaunchKernelGGL(mt_expand_kernel, dim3((unsigned)n_chunks), dim3(256), 0, st, chunks_dev,
                     words_per_chunk, total, out);
  PS_CHECK_LAUNCH();
  return kOk;
}

int launch_walk(const int64_t* indptr, const int32_t* indices, const int64_t* sources,
                int64_t n_src, int64_t n_hops, float alpha, const uint32_t* raw, uint64_t seed,
                uint32_t offset, int64_t src_base, int32_t* trace, int* err, hipStream_t st) {
  if (n_src <= 0) return kOk;
  dim3 grid((unsigned)ceil_div(n_src, 256)), block(256);
  if (raw)
    hipLaunchKernelGGL(walk_kernel<true>, grid, block, 0, st, indptr, indices, sources, n_src,
                       n_hops, alpha, raw, seed, offset, src_base, trace, err);
  else
    hipLaunchKernelGGL(walk_kernel<false>, grid, block, 0, st, indptr, indices, sources, n_src,
                       n_hops, alpha, raw, seed, offset, src_base, trace, err);
  PS_CHECK_LAUNCH();
  return kOk;
}

int visit_topk_lds_bytes(int64_t n_hops, int64_t k, int* P_out) {
  int P = 64;
  while (P < n_hops) P <<= 1;
  if (P_out) *P_out = P;
  return (int)(2 * P * 4 + align_up(k * 8, 16));
}

int launch_visit_topk(const int32_t* trace, const int64_t* sources, int64_t n_src, int64_t n_hops,
                      int64_t n_all, int64_t k, void* dense_scratch, double* out_w,
                      int64_t* out_nb, float* out_wn, int32_t* out_nb32, int64_t T_norm,
                      hipStream_t st) {
  if (n_src <= 0) return kOk;
  int P;
  const int lds = visit_topk_lds_bytes(n_hops, k, &P);
  PS_REQUIRE(lds <= 160 * 1024, kErrArg, "visit_topk: n_hops/k too large for LDS");
  if (lds > 64 * 1024)
    PS_CHECK_HIP(hipFuncSetAttribute((const void*)visit_topk_kernel,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, lds));
  hipLaunchKernelGGL(visit_topk_kernel, dim3((unsigned)n_src), dim3(64), lds, st, trace, sources,
                     n_src, n_hops, P, n_all, k, (CE*)dense_scratch, out_w, out_nb, out_wn,
                     out_nb32, T_norm);
  PS_CHECK_LAUNCH();
  return kOk;
}

int launch_visit_dense(const int32_t* trace, const int64_t* sources, int64_t n_src,
                       int64_t n_hops, int64_t n_all, double* dense, hipStream_t st) {
  if (n_src <= 0) return kOk;
  PS_CHECK_HIP(hipMemsetAsync(dense, 0, (size_t)(n_src * n_all) * sizeof(double), st));
  hipLaunchKernelGGL(visit_dense_count_kernel, dim3((unsigned)ceil_div(n_src * n_hops, 256)),
                     dim3(256), 0, st, trace, n_src, n_hops, n_all, dense);
  PS_CHECK_LAUNCH();
  hipLaunchKernelGGL(visit_dense_norm_kernel, dim3((unsigned)ceil_div(n_src * n_all, 256)),
                     dim3(256), 0, st, sources, n_src, n_hops, n_all, dense);
  PS_CHECK_LAUNCH();
  return kOk;
}

}  // namespace ps
