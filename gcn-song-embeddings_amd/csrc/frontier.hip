// Frontier construction on gfx950 (relevant_nodes_per_layer_precomp,
// pinsage_model.py:156-168): the reference builds each lower layer as
// unique(cat(nb.flatten(), nodeset)) with a sort.  Here a node set over the
// track universe [0, n) is a bitmap: marking is one atomicOr per id, the
// sorted unique list and every id's rank come from a per-word popcount prefix,
// so no sort runs and ranks are O(1) lookups (bitmap + prefix stay in L2).
#include "common.h"

#include <algorithm>

namespace ps {

int64_t bitset_words(int64_t universe);

constexpr int kScanBlock = 256;
constexpr int kWordsPerThread = 4;
constexpr int kWordsPerBlock = kScanBlock * kWordsPerThread;  // 1024 words = 64k ids

// test before set: popular ids are marked by thousands of lanes; a plain load
// of an already-set bit avoids serialising them on one atomic word
__device__ __forceinline__ void mark(unsigned long long* bits, int64_t v) {
  const unsigned long long bit = 1ull << (v & 63);
  if (!(__hip_atomic_load(bits + (v >> 6), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & bit))
    atomicOr(bits + (v >> 6), bit);
}

__device__ __forceinline__ int32_t rank_of(const unsigned long long* bits, const uint32_t* prefix,
                                           int64_t v) {
  const unsigned long long w = bits[v >> 6];
  return (int32_t)(prefix[v >> 6] + __popcll(w & ((1ull << (v & 63)) - 1ull)));
}

// mark a list of int64 ids (host-known count)
__global__ void bits_mark_i64_kernel(unsigned long long* __restrict__ bits,
                                     const int64_t* __restrict__ ids, int64_t n, int64_t limit,
                                     int* __restrict__ err) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t v = ids[i];
    if (v < 0 || v >= limit) {
      if (err) atomicExch(err, 1);
      continue;
    }
    mark(bits, v);
  }
}

// Single-block finalisation for bitmaps of <= kSmallWords words (<= 1M ids):
// OR, popcount, block scan, prefixes, compaction and count in one launch.
constexpr int kSmallWords = 16384;
// kCoherent: read the bitmap with device-coherent loads (it was written by
// atomics of this same kernel, which bypass the CU's L1)
template <bool kCoherent>
__device__ __forceinline__ void finalize_block(unsigned long long* __restrict__ dst,
                                               const unsigned long long* a,
                                               const unsigned long long* __restrict__ b,
                                               int64_t nwords, uint32_t* __restrict__ prefix,
                                               int32_t* __restrict__ members,
                                               int* __restrict__ count_out) {
  __shared__ uint32_t wsum[16];
  const int per = (int)((nwords + 1023) / 1024);
  const int64_t w0 = (int64_t)threadIdx.x * per;
  unsigned long long xs[16];
  uint32_t c = 0;
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    xs[q] = 0ull;
    const int64_t w = w0 + q;
    if (q < per && w < nwords) {
      unsigned long long x =
          kCoherent ? __hip_atomic_load(a + w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : a[w];
      if (b) x |= b[w];
      if (dst != a || b) dst[w] = x;
      xs[q] = x;
      c += __popcll(x);
    }
  }
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint32_t inc = c;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    uint32_t y = __shfl_up(inc, o, 64);
    if (lane >= o) inc += y;
  }
  if (lane == 63) wsum[wv] = inc;
  __syncthreads();
  uint32_t p = inc - c;
  for (int i = 0; i < wv; ++i) p += wsum[i];
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int64_t w = w0 + q;
    if (q < per && w < nwords) {
      prefix[w] = p;
      unsigned long long m = xs[q];
      uint32_t j = p;
      while (m) {
        const int bit = __ffsll((long long)m) - 1;
        members[j++] = (int32_t)(w * 64 + bit);
        m &= m - 1;
      }
      p += __popcll(xs[q]);
    }
  }
  if (threadIdx.x == 1023) *count_out = (int)p;
}

// The finalisations a mark launch runs itself (its last block to finish, so
// no separate single-block launch follows it): the marked set N (prefix,
// members, count) and optionally S_lo = N | S_l.  ticket: a zeroed int (the
// frontier's bitmap region, which the step's first kernel zeroes; the last
// block also resets it).
struct MarkFinalize {
  int* ticket = nullptr;
  uint32_t* prefN = nullptr;
  int32_t* memN = nullptr;
  int* cntN = nullptr;
  unsigned long long* dstS = nullptr;  // null: N only
  const unsigned long long* bS = nullptr;
  uint32_t* prefS = nullptr;
  int32_t* memS = nullptr;
  int* cntS = nullptr;
};

// mark nb_table[members[f]][t] for f < *count, t < T (table row stride ld).
// lds_words > 0: each block marks its contiguous slice into an LDS copy of the
// bitmap and ORs the touched words into HBM once (popular ids repeat thousands
// of times; global atomics on their words would serialise).  range_words > 0
// (bitmaps larger than LDS): the bitmap is cut into windows of range_words and
// the work into (window, slice) items, about two per workgroup; a block marks
// the ids of its slice that fall in its window into LDS (the slice's table rows
// are re-read once per window, from L2 / the Infinity Cache after the first).
__global__ __launch_bounds__(1024) void bits_mark_table_kernel(unsigned long long* bits,
                                                               const int32_t* __restrict__ members,
                                                               const int* __restrict__ count,
                                                               const int32_t* __restrict__ nb,
                                                               int64_t ld, int T, int lds_words,
                                                               int64_t nwords, int range_words, MarkFinalize fz) {
  extern __shared__ unsigned long long lbits[];
  const int64_t n = (int64_t)(*count) * T;
  if (range_words > 0) {
    const int64_t R = (nwords + range_words - 1) / range_words;
    const int64_t S = max((int64_t)1, (int64_t)(2 * gridDim.x + R - 1) / R);
    const int64_t slice = (n + S - 1) / S;
    for (int64_t it = blockIdx.x; it < R * S; it += gridDim.x) {
      const int64_t r = it % R, w0 = r * range_words;
      const int nwr = (int)min((int64_t)range_words, nwords - w0);
      const int64_t v0 = w0 * 64, vn = (int64_t)nwr * 64;
      const int64_t e0 = (it / R) * slice, e1 = min(n, e0 + slice);
      for (int w = threadIdx.x; w < nwr; w += blockDim.x) lbits[w] = 0ull;
      __syncthreads();
      for (int64_t e = e0 + threadIdx.x; e < e1; e += blockDim.x) {
        const int64_t f = e / T, t = e - f * T;
        const int64_t v = (int64_t)nb[(int64_t)members[f] * ld + t] - v0;
        if (v >= 0 && v < vn) atomicOr(lbits + (v >> 6), 1ull << (v & 63));
      }
      __syncthreads();
      for (int w = threadIdx.x; w < nwr; w += blockDim.x)
        if (lbits[w]) atomicOr(bits + w0 + w, lbits[w]);
      __syncthreads();  // the next item zeroes lbits
    }
  } else if (lds_words > 0) {
    for (int w = threadIdx.x; w < lds_words; w += blockDim.x) lbits[w] = 0ull;
    __syncthreads();
    const int64_t per = (n + gridDim.x - 1) / gridDim.x;
    const int64_t e0 = (int64_t)blockIdx.x * per, e1 = min(n, e0 + per);
    for (int64_t e = e0 + threadIdx.x; e < e1; e += blockDim.x) {
      const int64_t f = e / T, t = e - f * T;
      const int64_t v = nb[(int64_t)members[f] * ld + t];
      if (v >= 0 && v < (int64_t)lds_words * 64) atomicOr(lbits + (v >> 6), 1ull << (v & 63));
    }
    __syncthreads();
    for (int w = threadIdx.x; w < lds_words; w += blockDim.x)
      if (lbits[w]) atomicOr(bits + w, lbits[w]);
  } else {
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n;
         e += (int64_t)gridDim.x * blockDim.x) {
      const int64_t f = e / T, t = e - f * T;
      const int64_t v = nb[(int64_t)members[f] * ld + t];
      if (v >= 0 && v < nwords * 64) mark(bits, v);
    }
  }
  if (!fz.ticket) return;
  // The last block to finish finalises (the split-K counter hand-off of the
  // HIP guide): every wave drains its atomics, then ONE lane per block runs an
  // agent-scope release before its ticket add, and the block drawing the last
  // ticket runs ONE agent-scope acquire before it reads the bitmap back (with
  // device-coherent loads, finalize_block<true>).  One fence per block, not
  // per thread: a __threadfence in every thread made this launch slower than
  // the two it replaces.
  __shared__ int last;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (keep: the fence's own wait can be dropped)
    const bool l = __hip_atomic_fetch_add(fz.ticket, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
                   (int)gridDim.x - 1;
    if (l) {
      __hip_atomic_store(fz.ticket, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    last = l;
  }
  __syncthreads();
  if (!last) return;
  finalize_block<true>(bits, bits, nullptr, nwords, fz.prefN, fz.memN, fz.cntN);
  if (fz.dstS) {
    __syncthreads();  // (finalize_block's scan scratch is reused)
    finalize_block<true>(fz.dstS, bits, fz.bS, nwords, fz.prefS, fz.memS, fz.cntS);
  }
}

// mark nb_table[ids[i]][t] for an int64 id list (API frontier step)
__global__ void bits_mark_table_i64_kernel(unsigned long long* __restrict__ bits,
                                           const int64_t* __restrict__ ids, int64_t n,
                                           const int32_t* __restrict__ nb, int64_t ld, int T,
                                           int64_t limit, int* __restrict__ err) {
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n * T;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t f = e / T, t = e - f * T;
    const int64_t v = nb[ids[f] * ld + t];
    if (v < 0 || v >= limit) {
      atomicExch(err, 1);
      continue;
    }
    mark(bits, v);
  }
}

// dst = a | b (b may be null); per-block popcount totals
__global__ __launch_bounds__(kScanBlock) void bits_or_count_kernel(
    unsigned long long* __restrict__ dst, const unsigned long long* __restrict__ a,
    const unsigned long long* __restrict__ b, int64_t nwords, uint32_t* __restrict__ block_sums) {
  __shared__ int red[kScanBlock / 64];
  const int64_t w0 = (int64_t)blockIdx.x * kWordsPerBlock + threadIdx.x * kWordsPerThread;
  int c = 0;
#pragma unroll
  for (int q = 0; q < kWordsPerThread; ++q) {
    const int64_t w = w0 + q;
    if (w < nwords) {
      unsigned long long x = a[w];
      if (b) x |= b[w];
      if (dst != a || b) dst[w] = x;
      c += __popcll(x);
    }
  }
  c = wave_sum_i(c);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    int t = 0;
    for (int i = 0; i < kScanBlock / 64; ++i) t += red[i];
    block_sums[blockIdx.x] = (uint32_t)t;
  }
}

// per-word exclusive prefix + sorted member list + total count
__global__ __launch_bounds__(kScanBlock) void bits_scan_compact_kernel(
    const unsigned long long* __restrict__ bits, int64_t nwords,
    const uint32_t* __restrict__ block_sums, uint32_t* __restrict__ prefix,
    int32_t* __restrict__ members, int* __restrict__ count_out) {
  __shared__ uint32_t wsum[kScanBlock / 64];
  __shared__ uint32_t base_sh;
  // offset of this block = sum of the preceding blocks' totals
  uint32_t off = 0;
  for (int i = threadIdx.x; i < (int)blockIdx.x; i += kScanBlock) off += block_sums[i];
  off = (uint32_t)wave_sum_i((int)off);
  if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = off;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t t = 0;
    for (int i = 0; i < kScanBlock / 64; ++i) t += wsum[i];
    base_sh = t;
  }
  __syncthreads();
  const uint32_t base = base_sh;
  __syncthreads();
  const int64_t w0 = (int64_t)blockIdx.x * kWordsPerBlock + threadIdx.x * kWordsPerThread;
  unsigned long long x[kWordsPerThread];
  uint32_t c = 0;
#pragma unroll
  for (int q = 0; q < kWordsPerThread; ++q) {
    x[q] = (w0 + q < nwords) ? bits[w0 + q] : 0ull;
    c += __popcll(x[q]);
  }
  // inclusive wave scan of c
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint32_t inc = c;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    uint32_t y = __shfl_up(inc, o, 64);
    if (lane >= o) inc += y;
  }
  if (lane == 63) wsum[wv] = inc;
  __syncthreads();
  uint32_t wo = 0;
  for (int i = 0; i < wv; ++i) wo += wsum[i];
  uint32_t p = base + wo + inc - c;
#pragma unroll
  for (int q = 0; q < kWordsPerThread; ++q) {
    const int64_t w = w0 + q;
    if (w < nwords) {
      prefix[w] = p;
      unsigned long long m = x[q];
      uint32_t j = p;
      while (m) {
        const int bit = __ffsll((long long)m) - 1;
        members[j++] = (int32_t)(w * 64 + bit);
        m &= m - 1;
      }
      p += __popcll(x[q]);
    }
  }
  if (blockIdx.x == gridDim.x - 1 && threadIdx.x == kScanBlock - 1) *count_out = (int)p;
}

__global__ __launch_bounds__(1024) void bits_finalize_small_kernel(
    unsigned long long* __restrict__ dst, const unsigned long long* a,
    const unsigned long long* __restrict__ b, int64_t nwords, uint32_t* __restrict__ prefix,
    int32_t* __restrict__ members, int* __restrict__ count_out) {
  finalize_block<false>(dst, a, b, nwords, prefix, members, count_out);
}

// The first kernel of a train step: zero every frontier bitmap of the step
// (zero_words u64 words from zero), mark the batch ids into the top set and
// finalise it -- one block, replacing a memset, a mark and a finalise launch.
// Ids outside [0, limit) are skipped (callers validate them).
// x_n (nullable): the ids x0 .. x0 + *x_n - 1 join the set too (the on-the-fly
// step's virtual nodes, fly.hip).
__global__ __launch_bounds__(1024) void bits_top_set_kernel(
    unsigned long long* __restrict__ zero, int64_t zero_words, unsigned long long* bits,
    const int64_t* __restrict__ ids, int64_t n, int64_t limit, int64_t nwords,
    uint32_t* __restrict__ prefix, int32_t* __restrict__ members, int* __restrict__ count_out, int64_t x0,
    const int* __restrict__ x_n) {
  // (one block: the zeroing stores are agent-scope atomic stores, like the
  // ORs that follow them on the same words, so the block's own completion
  // (vmcnt) and barrier order them; the bitmap is read back with
  // device-coherent loads)
  for (int64_t w = threadIdx.x; w < zero_words; w += 1024)
    __hip_atomic_store(zero + w, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int64_t i = threadIdx.x; i < n; i += 1024) {
    const int64_t v = ids[i];
    if (v >= 0 && v < limit) atomicOr(bits + (v >> 6), 1ull << (v & 63));
  }
  if (x_n) {
    const int64_t nx = *x_n;
    for (int64_t v = x0 + threadIdx.x; v < x0 + nx; v += 1024)
      if (v >= 0 && v < limit) atomicOr(bits + (v >> 6), 1ull << (v & 63));
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  finalize_block<true>(bits, bits, nullptr, nwords, prefix, members, count_out);
}

// mark the id range x0 .. x0 + *x_n - 1
__global__ void bits_mark_range_kernel(unsigned long long* __restrict__ bits, int64_t x0,
                                       const int* __restrict__ x_n, int64_t limit) {
  const int64_t nx = *x_n;
  for (int64_t v = x0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < x0 + nx;
       v += (int64_t)gridDim.x * blockDim.x)
    if (v >= 0 && v < limit) atomicOr(bits + (v >> 6), 1ull << (v & 63));
}

// zero n u64 words (a kernel, not a memset: keeps captured step graphs
// kernel-only)
__global__ void zero_words_kernel(unsigned long long* __restrict__ p, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    p[i] = 0ull;
}

// ---------------------------------------------------------------- host side
int64_t bitset_words(int64_t universe) { return (universe + 63) / 64; }
int64_t bitset_blocks(int64_t universe) { return ceil_div(bitset_words(universe), kWordsPerBlock); }

int launch_mark_i64(unsigned long long* bits, const int64_t* ids, int64_t n, int64_t limit,
                    int* err, hipStream_t st) {
  if (n <= 0) return kOk;
  hipLaunchKernelGGL(bits_mark_i64_kernel, dim3(grid_for(n, 256)), dim3(256), 0, st, bits, ids, n,
                     limit, err);
  PS_CHECK_LAUNCH();
  return kOk;
}

static int launch_mark_table_fz(unsigned long long* bits, const int32_t* members, const int* count,
                                int64_t max_count, const int32_t* nb, int64_t ld, int T, int64_t universe,
                                hipStream_t st, const MarkFinalize* fz) {
  const int64_t nw = bitset_words(universe);
  if (fz && (nw > kSmallWords || max_count <= 0)) return kErrArg;  // (callers check mark_finalize_fits)
  if (max_count <= 0) return kOk;
  const MarkFinalize f = fz ? *fz : MarkFinalize{};
  // windows of a full CU's LDS less the finalisation's scan scratch (the limit
  // is raised once, on the first call, before any graph capture); beyond 64
  // windows, global atomics
  constexpr int kWinWords = 20448;  // 159.75 KiB
  static const int win_ok = hipFuncSetAttribute((const void*)bits_mark_table_kernel,
                                                hipFuncAttributeMaxDynamicSharedMemorySize,
                                                kWinWords * 8) == hipSuccess;
  constexpr int max_win = 64;
  if (nw * 8 <= 64 * 1024) {
    const int gb = std::max(1, std::min(64, ceil_div(max_count * T, 4096)));
    hipLaunchKernelGGL(bits_mark_table_kernel, dim3(gb), dim3(1024), (size_t)nw * 8, st, bits,
                       members, count, nb, ld, T, (int)nw, nw, 0, f);
  } else if (win_ok && ceil_div(nw, kWinWords) <= max_win) {
    hipLaunchKernelGGL(bits_mark_table_kernel, dim3(256), dim3(1024), (size_t)kWinWords * 8, st,
                       bits, members, count, nb, ld, T, 0, nw, kWinWords, f);
  } else {
    hipLaunchKernelGGL(bits_mark_table_kernel, dim3(grid_for(max_count * T, 1024)), dim3(1024), 0,
                       st, bits, members, count, nb, ld, T, 0, nw, 0, f);
  }
  PS_CHECK_LAUNCH();
  return kOk;
}

int launch_mark_table(unsigned long long* bits, const int32_t* members, const int* count,
                      int64_t max_count, const int32_t* nb, int64_t ld, int T, int64_t universe,
                      hipStream_t st) {
  return launch_mark_table_fz(bits, members, count, max_count, nb, ld, T, universe, st, nullptr);
}

// whether launch_mark_table can finalise its set itself (single-block finalisation)
bool mark_finalize_fits(int64_t universe) { return bitset_words(universe) <= kSmallWords; }

// mark N from the table rows of S and finalise N (and S_lo = N | S_l when
// dstS is set) in the same launch
int launch_mark_finalize(unsigned long long* bitsN, const int32_t* membersS, const int* countS, int64_t max_count,
                         const int32_t* nb, int64_t ld, int T, int64_t universe, int* ticket, uint32_t* prefN,
                         int32_t* memN, int* cntN, unsigned long long* dstS, const unsigned long long* bS,
                         uint32_t* prefS, int32_t* memS, int* cntS, hipStream_t st) {
  MarkFinalize f;
  f.ticket = ticket;
  f.prefN = prefN;
  f.memN = memN;
  f.cntN = cntN;
  f.dstS = dstS;
  f.bS = bS;
  f.prefS = prefS;
  f.memS = memS;
  f.cntS = cntS;
  return launch_mark_table_fz(bitsN, membersS, countS, max_count, nb, ld, T, universe, st, &f);
}

int launch_mark_table_i64(unsigned long long* bits, const int64_t* ids, int64_t n,
                          const int32_t* nb, int64_t ld, int T, int64_t limit, int* err,
                          hipStream_t st) {
  if (n <= 0) return kOk;
  hipLaunchKernelGGL(bits_mark_table_i64_kernel, dim3(grid_for(n * T, 256)), dim3(256), 0, st, bits,
                     ids, n, nb, ld, T, limit, err);
  PS_CHECK_LAUNCH();
  return kOk;
}

// local_idx[f][t] = rank of nb[nodeset[f]][t] in a finalised set (its
// position in the sorted members: the word's prefix + popcount below the bit)
// -- the index tables of relevant_nodes_per_layer_precomp's unique
// (pinsage_model.py:164-166) as the convolution reads them
__global__ __launch_bounds__(256) void set_rank_table_kernel(const int64_t* __restrict__ nodeset, int64_t n,
                                                             const int32_t* __restrict__ nb, int64_t ld, int T,
                                                             const unsigned long long* __restrict__ bits,
                                                             const uint32_t* __restrict__ prefix,
                                                             int32_t* __restrict__ out) {
  const int64_t total = n * T;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t f = i / T, t = i - f * T;
    const int64_t id = nb[nodeset[f] * ld + t];
    const unsigned long long wd = bits[id >> 6];
    out[i] = (int32_t)(prefix[id >> 6] + (uint32_t)__popcll(wd & ((1ull << (id & 63)) - 1ull)));
  }
}

int launch_set_rank_table(const int64_t* nodeset, int64_t n, const int32_t* nb, int64_t ld, int T,
                          const unsigned long long* bits, const uint32_t* prefix, int32_t* out, hipStream_t st) {
  if (n <= 0) return kOk;
  hipLaunchKernelGGL(set_rank_table_kernel, dim3(grid_for(n * T, 256)), dim3(256), 0, st, nodeset, n, nb, ld, T,
                     bits, prefix, out);
  PS_CHECK_LAUNCH();
  return kOk;
}

// Finalise a set: dst = a | b, prefix, sorted members, device count.
int launch_set_finalize(unsigned long long* dst, const unsigned long long* a,
                        const unsigned long long* b, int64_t universe, uint32_t* block_sums,
                        uint32_t* prefix, int32_t* members, int* count, hipStream_t st);

// zero the bitmaps region [zero, zero + zero_words), mark ids into bits and
// finalise that set (the top frontier of a step)
int launch_top_set(unsigned long long* zero, int64_t zero_words, unsigned long long* bits,
                   const int64_t* ids, int64_t n, int64_t universe, uint32_t* block_sums,
                   uint32_t* prefix, int32_t* members, int* count, hipStream_t st, int64_t x0,
                   const int* x_n) {
  const int64_t nw = bitset_words(universe);
  if (nw <= kSmallWords) {
    hipLaunchKernelGGL(bits_top_set_kernel, dim3(1), dim3(1024), 0, st, zero, zero_words, bits, ids,
                       n, universe, nw, prefix, members, count, x0, x_n);
    PS_CHECK_LAUNCH();
    return kOk;
  }
  hipLaunchKernelGGL(zero_words_kernel, dim3(grid_for(zero_words, 256, 2048)), dim3(256), 0, st, zero,
                     zero_words);
  PS_CHECK_LAUNCH();
  PS_TRY(launch_mark_i64(bits, ids, n, universe, nullptr, st));
  if (x_n) {
    hipLaunchKernelGGL(bits_mark_range_kernel, dim3(16), dim3(256), 0, st, bits, x0, x_n, universe);
    PS_CHECK_LAUNCH();
  }
  return launch_set_finalize(bits, bits, nullptr, universe, block_sums, prefix, members, count, st);
}

int launch_set_finalize(unsigned long long* dst, const unsigned long long* a,
                        const unsigned long long* b, int64_t universe, uint32_t* block_sums,
                        uint32_t* prefix, int32_t* members, int* count, hipStream_t st) {
  const int64_t nw = bitset_words(universe);
  if (nw <= kSmallWords) {
    hipLaunchKernelGGL(bits_finalize_small_kernel, dim3(1), dim3(1024), 0, st, dst, a, b, nw, prefix,
                       members, count);
    PS_CHECK_LAUNCH();
    return kOk;
  }
  const int nb = (int)bitset_blocks(universe);
  hipLaunchKernelGGL(bits_or_count_kernel, dim3(nb), dim3(kScanBlock), 0, st, dst, a, b, nw,
                     block_sums);
  PS_CHECK_LAUNCH();
  hipLaunchKernelGGL(bits_scan_compact_kernel, dim3(nb), dim3(kScanBlock), 0, st, dst, nw,
                     block_sums, prefix, members, count);
  PS_CHECK_LAUNCH();
  return kOk;
}

}  // namespace ps
