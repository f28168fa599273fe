// Convolution, loss and optimizer kernels for gfx950 (everything of the train
// step that is not a GEMM).
//
//   layer_prep      per-layer index tables (self rows, neighbour slots, weights)
//   agg             importance-weighted neighbour mean (pinsage_model.py:202)
//   csr_*           transpose of the neighbour slots for the backward scatter
//   dq_gather       d(agg) -> d(q) through the transpose, times lrelu'(q)
//   norm_lrelu_bwd  backward of z/||z|| and leaky_relu (pinsage_model.py:209-210)
//   loss_*          max_margin_loss (pinsage_training.py:31-41) fwd+bwd with the
//                   reference's duplicate-gradient semantics, plus monitors
//                   (pinsage_training.py:200-212)
//   adam            torch.optim.Adam step (pinsage_training.py:147,191)
#include "common.h"
#include "conv.h"
#include "bf16split.h"

#include <algorithm>
#include <climits>

namespace ps {

__device__ __forceinline__ int32_t rank_in(const unsigned long long* bits, const uint32_t* prefix,
                                           int64_t v) {
  const unsigned long long w = bits[v >> 6];
  return (int32_t)(prefix[v >> 6] + __popcll(w & ((1ull << (v & 63)) - 1ull)));
}

// ---------------------------------------------------------------- layer prep (conv.h)
// every layer's tables in one launch (each layer's items follow the previous
// layer's: the grid strides over their concatenation)
__global__ void layer_prep_kernel(LayerPreps a) {
  const int T = a.T;
  const int64_t g0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x, gs = (int64_t)gridDim.x * blockDim.x;
  for (int l = 0; l < a.n; ++l) {
    const LayerPrep& p = a.L[l];
    if (p.z) {  // zero the layer below's dY rows: the backward scatter-adds into them
      const int64_t zn4 = (int64_t)(*p.z_rows) * p.z_n / 4;
      float4* z4 = reinterpret_cast<float4*>(p.z);
      for (int64_t i = g0; i < zn4; i += gs) z4[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
  for (int l = 0; l < a.n; ++l) {
    const LayerPrep& p = a.L[l];
    const int64_t FS = (int64_t)(*p.nS), FN = (int64_t)(*p.nN);
    const int64_t total = FS * T + FS + FN + p.n_ids;
    for (int64_t e = g0; e < total; e += gs) {
      if (e < FS * T) {
        const int64_t f = e / T, t = e - f * T;
        const int64_t id = p.S_mem[f];
        const int64_t u = p.nb[id * p.ldT + t];
        p.loc[e] = rank_in(p.N_bits, p.N_pref, u);
        p.wloc[e] = p.wn[id * p.ldT + t];
      } else if (e < FS * T + FS) {
        const int64_t f = e - FS * T;
        const int64_t id = p.S_mem[f];
        p.self_src[f] = p.P_bits ? rank_in(p.P_bits, p.P_pref, id) : (int32_t)id;
      } else if (e < FS * T + FS + FN) {
        const int64_t u = e - FS * T - FS;
        const int64_t id = p.N_mem[u];
        p.q_src[u] = p.P_bits ? rank_in(p.P_bits, p.P_pref, id) : (int32_t)id;
      } else {
        // batch position -> row of the top-layer set (duplicates share a row)
        const int64_t i = e - FS * T - FS - FN;
        p.pos_rank[i] = rank_in(p.S_bits, p.S_pref, p.ids[i]);
      }
    }
  }
}

// ---------------------------------------------------------------- aggregation
// agg[f][:] = sum_t wloc[f,t] * q[loc[f,t]][:]   (weights pre-normalised by the
// row sum in f64, so this is the reference's sum(w*q)/sum(w)).  One wave per
// row, float4 per lane; the T gathered q rows are L2-resident.
template <int VEC>  // float4s per lane per row chunk
__global__ __launch_bounds__(256) void agg_kernel(const float* __restrict__ q, int hid,
                                                  const int32_t* __restrict__ loc,
                                                  const float* __restrict__ wloc, int T,
                                                  const int* __restrict__ nS, int64_t nS_host,
                                                  float* __restrict__ agg) {
  const int64_t F = nS ? (int64_t)(*nS) : nS_host;
  const int lane = threadIdx.x & 63;
  const int64_t wid = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
  const int h4 = hid >> 2;
  // neighbour rows whose loads are in flight together (16 x 2 float4 spill)
  constexpr int U = VEC == 1 ? 16 : 10;  // 10: a fanout-10 row in one round
  // work item = (row, 64*VEC-float4 column chunk): hid 512 at VEC 1 gives two
  // waves per row, each with all of a T <= 16 row's loads in one round
  const int nch = (h4 + 64 * VEC - 1) / (64 * VEC);
  for (int64_t item = wid; item < F * nch; item += nw) {
    const int64_t f = item / nch;
    {
      const int c0 = (int)(item - f * nch) * 64 * VEC;
      float4 a[VEC];
#pragma unroll
      for (int v = 0; v < VEC; ++v) a[v] = make_float4(0.f, 0.f, 0.f, 0.f);
      // the row's slots are read by the lanes (64 at a time) and broadcast, so
      // U neighbour rows' loads issue back to back instead of one index load ->
      // row load round trip per slot; the summation order stays t = 0, 1, ...
      for (int tb = 0; tb < T; tb += 64) {
        const int tn = min(64, T - tb);
        const int myr = lane < tn ? loc[f * T + tb + lane] : 0;
        const float myw = lane < tn ? wloc[f * T + tb + lane] : 0.f;
        for (int t0 = 0; t0 < tn; t0 += U) {
          float4 x[U][VEC];
          float w[U];
#pragma unroll
          for (int u = 0; u < U; ++u) {
            const int t = min(t0 + u, tn - 1);
            const int64_t r = __shfl(myr, t, 64);
            w[u] = t0 + u < tn ? __shfl(myw, t, 64) : 0.f;
            const float4* qr = reinterpret_cast<const float4*>(q + r * hid);
#pragma unroll
            for (int v = 0; v < VEC; ++v) {
              const int c = min(c0 + v * 64 + lane, h4 - 1);
              x[u][v] = qr[c];
            }
          }
          // padded slots select the old sum (a break here made x a scratch array)
#pragma unroll
          for (int u = 0; u < U; ++u) {
            const bool ok = t0 + u < tn;
#pragma unroll
            for (int v = 0; v < VEC; ++v) {
              a[v].x = ok ? fmaf(w[u], x[u][v].x, a[v].x) : a[v].x;
              a[v].y = ok ? fmaf(w[u], x[u][v].y, a[v].y) : a[v].y;
              a[v].z = ok ? fmaf(w[u], x[u][v].z, a[v].z) : a[v].z;
              a[v].w = ok ? fmaf(w[u], x[u][v].w, a[v].w) : a[v].w;
            }
          }
        }
      }
      float4* out = reinterpret_cast<float4*>(agg + f * hid);
#pragma unroll
      for (int v = 0; v < VEC; ++v) {
        const int c = c0 + v * 64 + lane;
        if (c < h4) out[c] = a[v];
      }
    }
  }
}

// XCD-sliced aggregation.  Workgroups are dealt round-robin over the 8 XCDs,
// so block b runs on XCD b % 8; that XCD owns column slice b % 8 (hid / 8
// floats) of q and agg.  Each XCD then gathers only its eighth of the q table
// (U x hid / 8 x 4 B: 2.7 MB at C2 layer 0), which its 4-MiB L2 holds, instead
// of every XCD pulling random whole rows of the full table through the
// Infinity Cache.  A wave covers 64 / SW4 rows (SW4 float4s of the slice per
// row), the T slots summed in order t = 0, 1, ... (bitwise agg_kernel).
constexpr int kXcds = 8;
template <int SW4>
__global__ __launch_bounds__(256) void agg_sliced_kernel(const float* __restrict__ q, int hid,
                                                         const int32_t* __restrict__ loc,
                                                         const float* __restrict__ wloc, int T,
                                                         const int* __restrict__ nS, int64_t nS_host,
                                                         float* __restrict__ agg) {
  constexpr int RPW = 64 / SW4;  // rows per wave pass
  constexpr int UF = 8;          // slots in flight per lane
  const int64_t F = nS ? (int64_t)(*nS) : nS_host;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int slice = blockIdx.x % kXcds;
  const int64_t G = gridDim.x / kXcds, g = blockIdx.x / kXcds;
  const int r_in = lane / SW4, c4 = lane % SW4;
  const int hid4 = hid >> 2;
  const float4* q4 = reinterpret_cast<const float4*>(q) + slice * SW4 + c4;
  for (int64_t rg = g * 4 + wave; rg * RPW < F; rg += G * 4) {
    const int64_t f = rg * RPW + r_in;
    const int64_t fr = f < F ? f : F - 1;
    const int32_t* lr = loc + fr * T;
    const float* wr = wloc + fr * T;
    float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int t0 = 0; t0 < T; t0 += UF) {
      int32_t ix[UF];
      float w[UF];
#pragma unroll
      for (int u = 0; u < UF; ++u) {
        const int t = min(t0 + u, T - 1);
        ix[u] = lr[t];
        w[u] = t0 + u < T ? wr[t] : 0.f;
      }
      float4 x[UF];
#pragma unroll
      for (int u = 0; u < UF; ++u) x[u] = q4[(int64_t)ix[u] * hid4];
#pragma unroll
      for (int u = 0; u < UF; ++u) {
        const bool ok = t0 + u < T;  // padded slots keep the sum (no fma with w = 0)
        a.x = ok ? fmaf(w[u], x[u].x, a.x) : a.x;
        a.y = ok ? fmaf(w[u], x[u].y, a.y) : a.y;
        a.z = ok ? fmaf(w[u], x[u].z, a.z) : a.z;
        a.w = ok ? fmaf(w[u], x[u].w, a.w) : a.w;
      }
    }
    if (f < F) reinterpret_cast<float4*>(agg + f * hid)[slice * SW4 + c4] = a;
  }
}

// ---------------------------------------------------------------- transpose (CSR by q row)
// Popular tracks sit in thousands of neighbour lists, so global per-row
// counters are hot.  When the distinct-neighbour count fits (<= kLdsRows), each
// block counts its contiguous slice of occurrences in an LDS histogram and
// flushes one global atomic per row it touched.  Up to kMaxRanges x kLdsRows
// rows, the rows are cut into ranges of kLdsRows and the work into (range,
// slice of occurrences) items, about two per workgroup: a block reads the slice and histograms
// the occurrences that fall in its range (the slice is read once per range,
// from L2 after the first).  Beyond that, lanes of a wave with the same row
// combine into one global atomic.
constexpr int kLdsRows = 40960;  // 160 KiB: a workgroup may take all of a CU's LDS
constexpr int kMaxRanges = 64;
constexpr int kCsrRangeGrid = 256;  // one 160-KiB workgroup per CU
__global__ __launch_bounds__(1024) void csr_count_kernel(const int32_t* __restrict__ loc,
                                                         const int* __restrict__ nS, int T,
                                                         const int* __restrict__ nN,
                                                         int* __restrict__ cnt,
                                                         float* __restrict__ zero_rows, int zero_n,
                                                         int* __restrict__ nsplit, int max_ranges) {
  extern __shared__ int hist[];
  const int64_t n = (int64_t)(*nS) * T;
  const int U = *nN;
  if (nsplit && blockIdx.x == 0 && threadIdx.x == 0) *nsplit = 0;  // the scan appends to it
  if (zero_rows) {  // the dq output receives atomics at chunk boundaries
    float4* z4 = reinterpret_cast<float4*>(zero_rows);
    const int64_t tot = (int64_t)U * zero_n / 4;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < tot;
         i += (int64_t)gridDim.x * blockDim.x)
      z4[i] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
  if (U <= kLdsRows) {
    for (int u = threadIdx.x; u < U; u += blockDim.x) hist[u] = 0;
    __syncthreads();
    const int64_t per = (n + gridDim.x - 1) / gridDim.x;
    const int64_t e0 = (int64_t)blockIdx.x * per, e1 = min(n, e0 + per);
    for (int64_t e = e0 + threadIdx.x; e < e1; e += blockDim.x) atomicAdd(hist + loc[e], 1);
    __syncthreads();
    for (int u = threadIdx.x; u < U; u += blockDim.x)
      if (hist[u]) atomicAdd(cnt + u, hist[u]);
    return;
  }
  const int R = (U + kLdsRows - 1) / kLdsRows;
  if (R <= max_ranges) {
    // about two items per workgroup: slices of n / ceil(2 grid / R)
    const int64_t S = max((int64_t)1, (int64_t)(2 * gridDim.x + R - 1) / R);
    const int64_t slice = (n + S - 1) / S;
    const int64_t items = (int64_t)R * S;
    for (int64_t it = blockIdx.x; it < items; it += gridDim.x) {
      const int r = (int)(it % R);
      const int u0 = r * kLdsRows, nu = min(kLdsRows, U - u0);
      const int64_t e0 = (it / R) * slice, e1 = min(n, e0 + slice);
      for (int u = threadIdx.x; u < nu; u += blockDim.x) hist[u] = 0;
      __syncthreads();
      for (int64_t e = e0 + threadIdx.x; e < e1; e += blockDim.x) {
        const int u = loc[e] - u0;
        if ((unsigned)u < (unsigned)nu) atomicAdd(hist + u, 1);
      }
      __syncthreads();
      for (int u = threadIdx.x; u < nu; u += blockDim.x)
        if (hist[u]) atomicAdd(cnt + u0 + u, hist[u]);
      __syncthreads();  // the next item zeroes hist
    }
    return;
  }
  const int lane = threadIdx.x & 63;
  for (int64_t base = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) & ~63LL; base < n;
       base += (int64_t)gridDim.x * blockDim.x) {
    const int64_t e = base + lane;
    const int32_t u = e < n ? loc[e] : -1;
    unsigned long long rem = __ballot(e < n);
    while (rem) {
      const int leader = __ffsll((long long)rem) - 1;
      const int32_t v = __shfl(u, leader, 64);
      const unsigned long long m = __ballot(u == v);
      if (lane == leader) atomicAdd(cnt + v, __popcll(m));
      rem &= ~m;
    }
  }
}

// Exclusive scans of cnt[0..*n) into off[0..*n] (off[n] = total) and of the
// per-row chunk counts ceil(cnt/kDqChunk), emitting the chunk list the dq
// kernel walks: chunk = {row u, first occurrence}, at most kDqChunk
// occurrences, never spanning two rows.  cnt is zeroed behind the read (kept
// zero for the next step).  Multi-block form: one block per 1024 rows, each
// block sums its predecessors' totals itself.
#ifndef PS_DQ_CHUNK
#define PS_DQ_CHUNK 16
#endif
constexpr int kDqChunk = PS_DQ_CHUNK;  // <= 16 (the engine's pair blocks), a multiple of 4
constexpr int kDqSplit = 0x100;  // chunk flag: the row's sum is split over several chunks
constexpr int kScanB = 256, kScanPer = 4, kScanChunk = kScanB * kScanPer;
__device__ __forceinline__ int n_chunks(int c) { return (c + kDqChunk - 1) / kDqChunk; }
__device__ __forceinline__ void wave_scan2(int& a, int& b, int lane) {
  for (int o = 1; o < 64; o <<= 1) {
    const int ya = __shfl_up(a, o, 64), yb = __shfl_up(b, o, 64);
    if (lane >= o) {
      a += ya;
      b += yb;
    }
  }
}
// off/cursor/chunks for rows i0 .. i0+per-1 from running totals (p, pc); the
// thread whose range holds index n also writes off[n] and the chunk count
__device__ __forceinline__ void scan_emit(int* __restrict__ cnt, int64_t i0, int per, int64_t n,
                                          int& p, int& pc, int* __restrict__ off,
                                          int* __restrict__ cursor, int* __restrict__ cbase,
                                          int2* __restrict__ chunks,
                                          int* __restrict__ nchunks, int2* __restrict__ split,
                                          int* __restrict__ nsplit) {
  for (int q = 0; q < per; ++q) {
    const int64_t i = i0 + q;
    if (i < n) {
      const int v = cnt[i];
      off[i] = p;
      cursor[i] = p;
      cbase[i] = pc;
      cnt[i] = 0;
      const int nc = n_chunks(v);
      // chunk = {row, occurrences (<= kDqChunk) | kDqSplit if the row spans
      // several chunks}; a split row's chunks are written by csr_fill_kernel's
      // blocks in parallel (one thread here would write thousands for a
      // popular row)
      if (nc == 1) chunks[pc] = make_int2((int)i, v);
      if (nc > 1) split[atomicAdd(nsplit, 1)] = make_int2((int)i, pc);  // order is irrelevant
      p += v;
      pc += nc;
    }
    if (i == n) {
      off[n] = p;
      *nchunks = pc;
    }
  }
}
__global__ __launch_bounds__(kScanB) void scan_block_sums_kernel(const int* __restrict__ cnt,
                                                                 const int* __restrict__ n_dev,
                                                                 int2* __restrict__ bsum) {
  __shared__ int red[2][kScanB / 64];
  const int64_t n = *n_dev;
  const int64_t i0 = (int64_t)blockIdx.x * kScanChunk + threadIdx.x * kScanPer;
  int c = 0, h = 0;
  for (int q = 0; q < kScanPer; ++q)
    if (i0 + q < n) {
      const int v = cnt[i0 + q];
      c += v;
      h += n_chunks(v);
    }
  c = wave_sum_i(c);
  h = wave_sum_i(h);
  if ((threadIdx.x & 63) == 0) {
    red[0][threadIdx.x >> 6] = c;
    red[1][threadIdx.x >> 6] = h;
  }
  __syncthreads();
  if (threadIdx.x == 0)
    bsum[blockIdx.x] = make_int2(red[0][0] + red[0][1] + red[0][2] + red[0][3],
                                 red[1][0] + red[1][1] + red[1][2] + red[1][3]);
}
__global__ __launch_bounds__(kScanB) void scan_apply_kernel(int* __restrict__ cnt,
                                                            const int* __restrict__ n_dev,
                                                            const int2* __restrict__ bsum,
                                                            int* __restrict__ off,
                                                            int* __restrict__ cursor,
                                                            int* __restrict__ cbase,
                                                            int2* __restrict__ chunks,
                                                            int* __restrict__ nchunks,
                                                            int2* __restrict__ split,
                                                            int* __restrict__ nsplit) {
  __shared__ int ws[2][kScanB / 64];
  const int64_t n = *n_dev;
  if ((int64_t)blockIdx.x * kScanChunk > n) return;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  int o = 0, oc = 0;
  for (int i = threadIdx.x; i < (int)blockIdx.x; i += kScanB) {
    const int2 b = bsum[i];
    o += b.x;
    oc += b.y;
  }
  o = wave_sum_i(o);
  oc = wave_sum_i(oc);
  if (lane == 0) {
    ws[0][wv] = o;
    ws[1][wv] = oc;
  }
  __syncthreads();
  const int base = ws[0][0] + ws[0][1] + ws[0][2] + ws[0][3];
  const int basec = ws[1][0] + ws[1][1] + ws[1][2] + ws[1][3];
  __syncthreads();
  const int64_t i0 = (int64_t)blockIdx.x * kScanChunk + threadIdx.x * kScanPer;
  int c = 0, h = 0;
  for (int q = 0; q < kScanPer; ++q)
    if (i0 + q < n) {
      const int v = cnt[i0 + q];
      c += v;
      h += n_chunks(v);
    }
  int inc = c, incc = h;
  wave_scan2(inc, incc, lane);
  if (lane == 63) {
    ws[0][wv] = inc;
    ws[1][wv] = incc;
  }
  __syncthreads();
  int p = base + inc - c, pc = basec + incc - h;
  for (int i = 0; i < wv; ++i) {
    p += ws[0][i];
    pc += ws[1][i];
  }
  scan_emit(cnt, i0, kScanPer, n, p, pc, off, cursor, cbase, chunks, nchunks, split, nsplit);
}
// single-block form, U <= 1024 * 64
__global__ __launch_bounds__(1024) void scan_small_kernel(int* __restrict__ cnt,
                                                          const int* __restrict__ n_dev,
                                                          int* __restrict__ off,
                                                          int* __restrict__ cursor,
                                                          int* __restrict__ cbase,
                                                          int2* __restrict__ chunks,
                                                          int* __restrict__ nchunks,
                                                          int2* __restrict__ split,
                                                          int* __restrict__ nsplit) {
  __shared__ int wsum[2][16];
  const int U = *n_dev;
  const int per = (U + 1023) / 1024;
  const int i0 = threadIdx.x * per;
  int c = 0, h = 0;
  for (int q = 0; q < per; ++q)
    if (i0 + q < U) {
      const int v = cnt[i0 + q];
      c += v;
      h += n_chunks(v);
    }
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  int inc = c, incc = h;
  wave_scan2(inc, incc, lane);
  if (lane == 63) {
    wsum[0][wv] = inc;
    wsum[1][wv] = incc;
  }
  __syncthreads();
  int p = inc - c, pc = incc - h;
  for (int i = 0; i < wv; ++i) {
    p += wsum[0][i];
    pc += wsum[1][i];
  }
  scan_emit(cnt, i0, per, U, p, pc, off, cursor, cbase, chunks, nchunks, split, nsplit);
  // no range holds index U when U == 1024 * per: thread 1023 ends on the totals
  if (threadIdx.x == 1023 && U == 1024 * per) {
    off[U] = p;
    *nchunks = pc;
  }
}

// occurrence (slot e = f T + t) at position pos of row u's range: its
// {source row f, weight} goes to entry (pos - off[u]) % kDqChunk of chunk
// cbase[u] + (pos - off[u]) / kDqChunk, so a dq wave reads its chunk's rows
// and weights with one load
__device__ __forceinline__ void put_occ(int2* __restrict__ occ2, const int* __restrict__ off,
                                        const int* __restrict__ cbase, const float* __restrict__ wloc,
                                        int T, int u, int pos, int64_t e) {
  const int local = pos - off[u];
  occ2[(int64_t)(cbase[u] + local / kDqChunk) * kDqChunk + local % kDqChunk] =
      make_int2((int)(e / T), __float_as_int(wloc[e]));
}

__global__ __launch_bounds__(1024) void csr_fill_kernel(const int32_t* __restrict__ loc,
                                                        const float* __restrict__ wloc,
                                                        const int* __restrict__ nS, int T,
                                                        const int* __restrict__ nN,
                                                        int* __restrict__ cursor,
                                                        const int* __restrict__ off,
                                                        const int* __restrict__ cbase,
                                                        int2* __restrict__ occ2, int max_ranges,
                                                        const int2* __restrict__ split,
                                                        const int* __restrict__ nsplit,
                                                        int2* __restrict__ chunks) {
  extern __shared__ int hist[];
  const int64_t n = (int64_t)(*nS) * T;
  const int U = *nN;
  // the chunk descriptors of the rows split over several chunks (the scan's split list)
  const int ns = *nsplit;
  for (int si = blockIdx.x; si < ns; si += gridDim.x) {
    const int2 sp = split[si];
    const int v = off[sp.x + 1] - off[sp.x], nc = n_chunks(v);
    for (int j = threadIdx.x; j < nc; j += blockDim.x)
      chunks[sp.y + j] = make_int2(sp.x, min(kDqChunk, v - j * kDqChunk) | kDqSplit);
  }
  if (U <= kLdsRows) {
    for (int u = threadIdx.x; u < U; u += blockDim.x) hist[u] = 0;
    __syncthreads();
    const int64_t per = (n + gridDim.x - 1) / gridDim.x;
    const int64_t e0 = (int64_t)blockIdx.x * per, e1 = min(n, e0 + per);
    for (int64_t e = e0 + threadIdx.x; e < e1; e += blockDim.x) atomicAdd(hist + loc[e], 1);
    __syncthreads();
    // reserve this block's slots per row: hist[u] becomes the block's base
    for (int u = threadIdx.x; u < U; u += blockDim.x)
      if (hist[u]) hist[u] = atomicAdd(cursor + u, hist[u]);
    __syncthreads();
    for (int64_t e = e0 + threadIdx.x; e < e1; e += blockDim.x) {
      const int32_t u = loc[e];
      const int pos = atomicAdd(hist + u, 1);
      put_occ(occ2, off, cbase, wloc, T, u, pos, e);
    }
    return;
  }
  const int R = (U + kLdsRows - 1) / kLdsRows;
  if (R <= max_ranges) {  // (range, slice) items as csr_count_kernel's
    // about two items per workgroup: slices of n / ceil(2 grid / R)
    const int64_t S = max((int64_t)1, (int64_t)(2 * gridDim.x + R - 1) / R);
    const int64_t slice = (n + S - 1) / S;
    const int64_t items = (int64_t)R * S;
    for (int64_t it = blockIdx.x; it < items; it += gridDim.x) {
      const int r = (int)(it % R);
      const int u0 = r * kLdsRows, nu = min(kLdsRows, U - u0);
      const int64_t e0 = (it / R) * slice, e1 = min(n, e0 + slice);
      for (int u = threadIdx.x; u < nu; u += blockDim.x) hist[u] = 0;
      __syncthreads();
      for (int64_t e = e0 + threadIdx.x; e < e1; e += blockDim.x) {
        const int u = loc[e] - u0;
        if ((unsigned)u < (unsigned)nu) atomicAdd(hist + u, 1);
      }
      __syncthreads();
      for (int u = threadIdx.x; u < nu; u += blockDim.x)
        if (hist[u]) hist[u] = atomicAdd(cursor + u0 + u, hist[u]);
      __syncthreads();
      for (int64_t e = e0 + threadIdx.x; e < e1; e += blockDim.x) {
        const int u = loc[e] - u0;
        if ((unsigned)u < (unsigned)nu) {
          const int pos = atomicAdd(hist + u, 1);
          put_occ(occ2, off, cbase, wloc, T, u0 + u, pos, e);
        }
      }
      __syncthreads();  // the next item zeroes hist
    }
    return;
  }
  const int lane = threadIdx.x & 63;
  for (int64_t base = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) & ~63LL; base < n;
       base += (int64_t)gridDim.x * blockDim.x) {
    const int64_t e = base + lane;
    const int32_t u = e < n ? loc[e] : -1;
    unsigned long long rem = __ballot(e < n);
    int pos = 0;
    while (rem) {
      const int leader = __ffsll((long long)rem) - 1;
      const int32_t v = __shfl(u, leader, 64);
      const unsigned long long m = __ballot(u == v);
      int b = 0;
      if (lane == leader) b = atomicAdd(cursor + v, __popcll(m));
      b = __shfl(b, leader, 64);
      if (u == v) pos = b + __popcll(m & ((1ull << lane) - 1));
      rem &= ~m;
    }
    if (e < n) put_occ(occ2, off, cbase, wloc, T, u, pos, e);
  }
}

// ---------------------------------------------------------------- canonical CSR order
// The fill claims positions with atomics, so the order of a row's {source row
// f, weight} pairs -- and with it the fp32 summation order of the transposed
// aggregation -- would change from run to run.  Both kernels below sort each
// row's pairs by f (unique within a row: a node's top-T list has distinct
// entries), so the step is bitwise reproducible.  They run on the frontier's
// stream right behind the fill, off the step's critical chain.
//
// Rows of one chunk (<= kDqChunk pairs): one wave per chunk, a bitonic network
// over its 16 lanes (shuffles); empty lanes carry INT_MAX keys.  A row split
// over 2..4 chunks (<= 64 pairs, contiguous from its first chunk) is sorted by
// the wave of its first chunk: every lane holds one pair and its place is the
// number of the row's pairs with a smaller source row.
constexpr int kSortWaveRow = 64;
__global__ __launch_bounds__(256) void csr_sort_chunks_kernel(const int2* __restrict__ chunks,
                                                              const int* __restrict__ nchunks,
                                                              const int* __restrict__ off,
                                                              int2* __restrict__ occ2) {
  const int lane = threadIdx.x & 63;
  const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
  const int nch = *nchunks;
  for (int64_t ci = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; ci < nch; ci += nw) {
    const int2 dsc = chunks[ci];
    const int n = dsc.y & 0xff;
    if (dsc.y & kDqSplit) {
      if (ci > 0 && chunks[ci - 1].x == dsc.x) continue;  // (not the row's first chunk)
      const int nr = off[dsc.x + 1] - off[dsc.x];
      if (nr > kSortWaveRow) continue;  // (csr_sort_rows_kernel)
      const int2 v = lane < nr ? occ2[ci * kDqChunk + lane] : make_int2(INT_MAX, 0);
      int r = 0;
      for (int j = 0; j < nr; ++j) r += __shfl(v.x, j, 64) < v.x;
      __builtin_amdgcn_wave_barrier();
      if (lane < nr) occ2[ci * kDqChunk + r] = v;
      continue;
    }
    if (n < 2) continue;
    int2 v = make_int2(INT_MAX, 0);
    if (lane < n) v = occ2[ci * kDqChunk + lane];
#pragma unroll
    for (int k = 2; k <= kDqChunk; k <<= 1)
#pragma unroll
      for (int j = k >> 1; j > 0; j >>= 1) {
        const int ox = __shfl_xor(v.x, j, 64), oy = __shfl_xor(v.y, j, 64);
        const bool lower = (lane & j) == 0, up = (lane & k) == 0;
        // ascending block: the lower lane keeps the smaller key
        const bool take = (lower == up) ? (ox < v.x) : (ox > v.x);
        if (take) v = make_int2(ox, oy);
      }
    if (lane < n) occ2[ci * kDqChunk + lane] = v;
  }
}

// Rows split over several chunks (the scan's split list {u, first chunk}):
// the row's n pairs are contiguous from occ2[cbase * kDqChunk], and their
// source rows f are distinct.  One block per row ranks every pair by a bitmap
// of the f range (windows of kRankBits): a pair's sorted position is the
// count of set bits below its own, read from per-word popcount prefixes, so it
// writes itself to its place in `tmp` (no comparison sort: O(range / 32 + n)
// per row), then the sorted row is copied back.
constexpr int kRankWords = 16384;                   // bitmap words per window (64 KiB)
constexpr int64_t kRankBits = (int64_t)kRankWords * 32;
constexpr int kRankLds = kRankWords * 4 * 2 + 64;   // bitmap + word prefixes + scan scratch
__global__ __launch_bounds__(1024) void csr_sort_rows_kernel(const int2* __restrict__ split,
                                                             const int* __restrict__ nsplit,
                                                             const int* __restrict__ off, int2* __restrict__ occ2,
                                                             int2* __restrict__ tmp) {
  extern __shared__ unsigned rk[];
  unsigned* bits = rk;                            // [kRankWords]
  unsigned* pref = rk + kRankWords;               // [kRankWords] exclusive popcount prefix
  int* red = reinterpret_cast<int*>(pref + kRankWords);  // [16] wave partials
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int ns = *nsplit;
  for (int si = blockIdx.x; si < ns; si += gridDim.x) {
    const int2 sp = split[si];
    const int n = off[sp.x + 1] - off[sp.x];
    if (n <= kSortWaveRow) continue;  // (sorted by csr_sort_chunks_kernel)
    int2* row = occ2 + (int64_t)sp.y * kDqChunk;
    int2* out = tmp + (int64_t)sp.y * kDqChunk;
    // f range of the row
    int lo = INT_MAX, hi = -1;
    for (int i = tid; i < n; i += blockDim.x) {
      const int f = row[i].x;
      lo = min(lo, f);
      hi = max(hi, f);
    }
    for (int o = 32; o > 0; o >>= 1) {
      lo = min(lo, __shfl_xor(lo, o, 64));
      hi = max(hi, __shfl_xor(hi, o, 64));
    }
    if (lane == 0) red[wv] = lo;
    __syncthreads();
    if (tid == 0) {
      int a = red[0];
      for (int w = 1; w < 16; ++w) a = min(a, red[w]);
      red[0] = a;
    }
    __syncthreads();
    lo = red[0];
    __syncthreads();
    if (lane == 0) red[wv] = hi;
    __syncthreads();
    if (tid == 0) {
      int a = red[0];
      for (int w = 1; w < 16; ++w) a = max(a, red[w]);
      red[0] = a;
    }
    __syncthreads();
    hi = red[0];
    __syncthreads();
    int base = 0;  // pairs placed by earlier windows
    for (int64_t w0 = lo; w0 <= hi; w0 += kRankBits) {
      const int nwords = (int)min((int64_t)kRankWords, (hi - w0) / 32 + 1);
      for (int i = tid; i < nwords; i += blockDim.x) bits[i] = 0u;
      __syncthreads();
      for (int i = tid; i < n; i += blockDim.x) {
        const int64_t b = (int64_t)row[i].x - w0;
        if (b >= 0 && b < (int64_t)nwords * 32) atomicOr(bits + (b >> 5), 1u << (b & 31));
      }
      __syncthreads();
      // exclusive prefix of the words' popcounts: each thread a contiguous run
      const int per = (nwords + (int)blockDim.x - 1) / (int)blockDim.x;
      const int i0 = tid * per;
      int s = 0;
      for (int i = i0; i < min(nwords, i0 + per); ++i) s += __popc(bits[i]);
      int inc = s;
      for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(inc, o, 64);
        if (lane >= o) inc += y;
      }
      if (lane == 63) red[wv] = inc;
      __syncthreads();
      int pre = inc - s;
      for (int w = 0; w < wv; ++w) pre += red[w];
      int total = 0;
      for (int w = 0; w < 16; ++w) total += red[w];
      for (int i = i0; i < min(nwords, i0 + per); ++i) {
        pref[i] = (unsigned)pre;
        pre += __popc(bits[i]);
      }
      __syncthreads();
      for (int i = tid; i < n; i += blockDim.x) {
        const int2 v = row[i];
        const int64_t b = (int64_t)v.x - w0;
        if (b >= 0 && b < (int64_t)nwords * 32) {
          const int wd = (int)(b >> 5);
          const int r = base + (int)pref[wd] + __popc(bits[wd] & ((1u << (b & 31)) - 1u));
          out[r] = v;
        }
      }
      base += total;
      __syncthreads();  // (the next window rewrites bits / pref / red)
    }
    __threadfence_block();
    __syncthreads();
    for (int i = tid; i < n; i += blockDim.x) row[i] = out[i];
    __syncthreads();
  }
}

// dpq[u] = lrelu'(q[u]) * sum over the occurrences (f, t) of u in the slot
// table of w[f][t] * dagg[f]   (the transpose of agg, pinsage_model.py:202).
// One wave per chunk of <= kDqChunk occurrences of ONE row u (chunk list from
// the CSR scan; popular tracks, in thousands of neighbour lists, span many
// chunks).  A chunk is {u, n | split} plus its n {row f, weight} pairs, one
// load each; the wave prefetches its next chunk's pair while it issues this
// chunk's q row and all of its dagg rows at once, so a chunk costs about one
// memory round trip.  A row with one chunk is finished here; a row split over
// several chunks leaves one raw partial per chunk in `part` and
// dq_combine_kernel sums them in chunk order (deterministic, and no
// device-scope float atomics: with per-XCD L2s those run at the memory side
// and serialise on popular rows).
//
// CM (chunk rows, the bottom layer): every chunk writes its MASKED partial,
// lrelu'(q[u]) * sum over its occurrences, to part[ci] and its row's source
// index q_src[u] to csrc[ci].  The mask is elementwise, so u's masked partials
// add up to dpq[u]; the Q weight gradient dpq^T h[q_src] is then the same
// GEMM over chunk rows (h gathered through csrc) and no combine is needed --
// at the bottom layer nothing else reads dpq (no dh below the input features).
// Row-granular write-through store / L2-bypassing load of one float4 of a
// partial row (the split-row tree below: a partial written on one XCD is read
// by a wave on another, and the XCDs' L2s are not coherent; the same hand-off
// as wgrad.hip's split combine).  `row` must be wave-uniform.
typedef int dq_v4i __attribute__((ext_vector_type(4)));
// dpq row elements e .. e + 3 as their hi / mid / lo bf16 planes (plane stride
// ps elements): the split the long-K weight gradient's fp32 form does in
// registers (bf16split.h), so its planes form (wgrad_pl_kernel) gets the same
// products
__device__ __forceinline__ void dq_store_planes(uint16_t* __restrict__ base, int64_t ps, int64_t e, float4 v) {
  unsigned h0, m0, l0, h1, m1, l1;
  split_pair(f32x2{v.x, v.y}, h0, m0, l0);
  split_pair(f32x2{v.z, v.w}, h1, m1, l1);
  *reinterpret_cast<uint2*>(base + e) = make_uint2(h0, h1);
  *reinterpret_cast<uint2*>(base + ps + e) = make_uint2(m0, m1);
  *reinterpret_cast<uint2*>(base + 2 * ps + e) = make_uint2(l0, l1);
}
__device__ __forceinline__ void dq_st_wt(float* row, int i, float4 v) {
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(row, 0, 0x7fffffff, 0x00020000);
  const dq_v4i w{__float_as_int(v.x), __float_as_int(v.y), __float_as_int(v.z), __float_as_int(v.w)};
  __builtin_amdgcn_raw_buffer_store_b128(w, rs, (unsigned)i * 16u, 0, 16);
}
__device__ __forceinline__ float4 dq_ld_wt(const float* row, int i) {
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(row), 0, 0x7fffffff, 0x00020000);
  const dq_v4i y = __builtin_amdgcn_raw_buffer_load_b128(rs, (unsigned)i * 16u, 0, 16);
  return make_float4(__int_as_float(y.x), __int_as_float(y.y), __int_as_float(y.z), __int_as_float(y.w));
}
// Split-row tree (TREE, PINSAGE_DQ_TREE): a row u split over k chunks
// cbase[u] .. cbase[u] + k - 1 is combined by the chunk waves themselves, with
// no dq_combine launch: the chunks are the leaves of a fan-in-8 tree whose node
// (L, g) holds the sum of leaves 8^L g .. 8^L (g + 1) - 1 in part row
// cbase[u] + 8^L g.  A finished node bumps its parent's ticket (level L's
// array, entry cbase[u] + g / 8); the child that arrives last sums the
// parent's children in child order, so every sum has a fixed order whatever
// the timing (deterministic), and the root applies lrelu'(q) and writes
// dpq[u].  Tickets reset themselves.  acc: this chunk's raw partial.
template <int VEC, bool PL3>
__device__ __forceinline__ void dq_tree_leaf(float4 (&acc)[VEC], const float4 (&qv)[VEC], int u, int64_t ci,
                                             int lane, int h4, int hid, const int* __restrict__ off,
                                             const int* __restrict__ cbase, int* __restrict__ tk,
                                             int64_t tk_stride, float* __restrict__ part,
                                             float* __restrict__ dpq, uint16_t* __restrict__ dpq3,
                                             int64_t ps3) {
  const int k = n_chunks(off[u + 1] - off[u]);
  const int64_t cb = cbase[u];
  int64_t g = ci - cb, span = 1, nodes = k;
  float* leaf = part + (int64_t)__builtin_amdgcn_readfirstlane((int)ci) * hid;
#pragma unroll
  for (int v = 0; v < VEC; ++v)
    if (v * 64 + lane < h4) dq_st_wt(leaf, v * 64 + lane, acc[v]);
  for (int L = 0;; ++L) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this node's row is written through
    const int64_t gp = g >> 3;
    const int nch = (int)min<int64_t>(8, nodes - 8 * gp);
    int t = 0;
    if (lane == 0) t = __hip_atomic_fetch_add(tk + L * tk_stride + cb + gp, 1, __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT);
    t = __shfl(t, 0, 64);
    if (t != nch - 1) return;  // a sibling still runs: the last one carries on
    if (lane == 0) __hip_atomic_store(tk + L * tk_stride + cb + gp, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    float4 x[8][VEC];
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const int cc = c < nch ? c : nch - 1;  // (a repeated child: loaded, not added)
      const float* row = part + (cb + span * (8 * gp + cc)) * hid;
#pragma unroll
      for (int v = 0; v < VEC; ++v) x[c][v] = dq_ld_wt(row, min(v * 64 + lane, h4 - 1));
    }
#pragma unroll
    for (int v = 0; v < VEC; ++v) acc[v] = x[0][v];
#pragma unroll
    for (int c = 1; c < 8; ++c)
      if (c < nch)
#pragma unroll
        for (int v = 0; v < VEC; ++v) {
          acc[v].x += x[c][v].x;
          acc[v].y += x[c][v].y;
          acc[v].z += x[c][v].z;
          acc[v].w += x[c][v].w;
        }
    span *= 8;
    nodes = (nodes + 7) >> 3;
    g = gp;
    if (nodes == 1) {  // the root: dpq[u]
      float4* o = reinterpret_cast<float4*>(dpq + (int64_t)u * hid);
#pragma unroll
      for (int v = 0; v < VEC; ++v)
        if (v * 64 + lane < h4) {
          const float4 r = make_float4(acc[v].x * lrelu_grad(qv[v].x), acc[v].y * lrelu_grad(qv[v].y),
                                       acc[v].z * lrelu_grad(qv[v].z), acc[v].w * lrelu_grad(qv[v].w));
          if (PL3) dq_store_planes(dpq3, ps3, (int64_t)u * hid + 4 * (v * 64 + lane), r);
          else o[v * 64 + lane] = r;
        }
      return;
    }
    float* node = part + (int64_t)__builtin_amdgcn_readfirstlane((int)(cb + span * g)) * hid;
#pragma unroll
    for (int v = 0; v < VEC; ++v)
      if (v * 64 + lane < h4) dq_st_wt(node, v * 64 + lane, acc[v]);
  }
}

// PL3 (with TREE; the bottom layer, where only the Q weight gradient reads
// dpq): dpq rows are written as hi / mid / lo bf16 planes (dpq3, plane stride
// ps3) instead of fp32 rows.
template <int VEC, bool CM = false, bool TREE = false, bool PL3 = false>
__global__ __launch_bounds__(256) void dq_chunk_kernel(
    const int2* __restrict__ chunks, const int* __restrict__ nchunks, const int2* __restrict__ occ2,
    const float* __restrict__ dagg, int64_t ld_dagg, const float* __restrict__ q, int hid,
    float* __restrict__ dpq, float* __restrict__ part, const int32_t* __restrict__ q_src = nullptr,
    int32_t* __restrict__ csrc = nullptr, const int* __restrict__ off = nullptr,
    const int* __restrict__ cbase = nullptr, int* __restrict__ tk = nullptr, int64_t tk_stride = 0,
    uint16_t* __restrict__ dpq3 = nullptr, int64_t ps3 = 0) {
  const int lane = threadIdx.x & 63;
  const int64_t wid = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
  const int h4 = hid >> 2;
  const int nch = *nchunks;
  int2 dsc = make_int2(0, 0), oc = make_int2(0, 0);
  if (wid < nch) {
    dsc = chunks[wid];
    if (lane < kDqChunk) oc = occ2[wid * kDqChunk + lane];
  }
  if (!CM && h4 <= 64 * VEC) {
    // One column pass per chunk: each chunk's result is stored only after the
    // NEXT chunk's rows have been issued.  vmcnt counts stores and loads in
    // issue order, so rows loaded behind a store also waited for it: every
    // chunk paid a store round trip before its loads could land.
    float4 pend[VEC];
    float4* pend_o = nullptr;
    int64_t pend_e = -1;  // (PL3) the pending dpq row's first element
    auto store_pend = [&]() __attribute__((always_inline)) {
      if (PL3 && pend_e >= 0) {
#pragma unroll
        for (int v = 0; v < VEC; ++v)
          if (v * 64 + lane < h4) dq_store_planes(dpq3, ps3, pend_e + 4 * (v * 64 + lane), pend[v]);
        pend_e = -1;
      } else if (pend_o) {
#pragma unroll
        for (int v = 0; v < VEC; ++v)
          if (v * 64 + lane < h4) pend_o[v * 64 + lane] = pend[v];
        pend_o = nullptr;
      }
    };
    for (int64_t ci = wid; ci < nch; ci += nw) {
      int2 dsc_n = make_int2(0, 0), oc_n = make_int2(0, 0);
      if (ci + nw < nch) {
        dsc_n = chunks[ci + nw];
        if (lane < kDqChunk) oc_n = occ2[(ci + nw) * kDqChunk + lane];
      }
      const int u = dsc.x, n = dsc.y & 0xff;
      const bool split = (dsc.y & kDqSplit) != 0;
      const int32_t my_row = oc.x;
      const float my_w = __int_as_float(oc.y);
      float4 qv[VEC], x[kDqChunk][VEC];
#pragma unroll
      for (int v = 0; v < VEC; ++v) qv[v] = reinterpret_cast<const float4*>(q + (int64_t)u * hid)[min(v * 64 + lane, h4 - 1)];
      const int ng = (n + 3) >> 2;
#pragma unroll
      for (int g = 0; g < kDqChunk / 4; ++g) {
        if (g < ng) {
#pragma unroll
          for (int jj = 0; jj < 4; ++jj) {
            const int j = 4 * g + jj;
            const int32_t row = __shfl(my_row, min(j, n - 1), 64);
            const float4* dr = reinterpret_cast<const float4*>(dagg + (int64_t)row * ld_dagg);
#pragma unroll
            for (int v = 0; v < VEC; ++v) x[j][v] = dr[min(v * 64 + lane, h4 - 1)];
          }
        }
      }
      store_pend();  // the previous chunk's result, behind this chunk's loads
      float4 acc[VEC];
#pragma unroll
      for (int v = 0; v < VEC; ++v) acc[v] = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int g = 0; g < kDqChunk / 4; ++g) {
        if (g < ng) {
#pragma unroll
          for (int jj = 0; jj < 4; ++jj) {
            const int j = 4 * g + jj;
            const float w = j < n ? __shfl(my_w, j, 64) : 0.f;
#pragma unroll
            for (int v = 0; v < VEC; ++v) {
              acc[v].x = fmaf(w, x[j][v].x, acc[v].x);
              acc[v].y = fmaf(w, x[j][v].y, acc[v].y);
              acc[v].z = fmaf(w, x[j][v].z, acc[v].z);
              acc[v].w = fmaf(w, x[j][v].w, acc[v].w);
            }
          }
        }
      }
      if (TREE && split) {  // this chunk is a leaf of its row's tree (no pending store)
        dq_tree_leaf<VEC, PL3>(acc, qv, u, ci, lane, h4, hid, off, cbase, tk, tk_stride, part, dpq, dpq3, ps3);
        dsc = dsc_n;
        oc = oc_n;
        continue;
      }
#pragma unroll
      for (int v = 0; v < VEC; ++v)
        pend[v] = split ? acc[v]
                        : make_float4(acc[v].x * lrelu_grad(qv[v].x), acc[v].y * lrelu_grad(qv[v].y),
                                      acc[v].z * lrelu_grad(qv[v].z), acc[v].w * lrelu_grad(qv[v].w));
      if (PL3 && !split) pend_e = (int64_t)u * hid;
      else pend_o = reinterpret_cast<float4*>(split ? part + ci * hid : dpq + (int64_t)u * hid);
      dsc = dsc_n;
      oc = oc_n;
    }
    store_pend();
    return;
  }
  for (int64_t ci = wid; ci < nch; ci += nw) {
    int2 dsc_n = make_int2(0, 0), oc_n = make_int2(0, 0);
    if (ci + nw < nch) {  // the next chunk's descriptor and pairs, under this one
      dsc_n = chunks[ci + nw];
      if (lane < kDqChunk) oc_n = occ2[(ci + nw) * kDqChunk + lane];
    }
    const int u = dsc.x, n = dsc.y & 0xff;
    const bool split = !CM && (dsc.y & kDqSplit) != 0;
    if (CM && lane == 0) csrc[ci] = q_src[u];
    const int32_t my_row = oc.x;
    const float my_w = __int_as_float(oc.y);
    for (int c0 = 0; c0 < h4; c0 += 64 * VEC) {
      float4 qv[VEC], x[kDqChunk][VEC];
#pragma unroll
      for (int v = 0; v < VEC; ++v) {
        const int c = min(c0 + v * 64 + lane, h4 - 1);
        qv[v] = reinterpret_cast<const float4*>(q + (int64_t)u * hid)[c];
      }
      // rows in groups of 4 (n is wave-uniform, so the group tests are scalar
      // branches); every load is issued before the first use, and a partial
      // group repeats its last row (a cache hit) instead of branching per row
      const int ng = (n + 3) >> 2;
#pragma unroll
      for (int g = 0; g < kDqChunk / 4; ++g) {
        if (g < ng) {
#pragma unroll
          for (int jj = 0; jj < 4; ++jj) {
            const int j = 4 * g + jj;
            const int32_t row = __shfl(my_row, min(j, n - 1), 64);
            const float4* dr = reinterpret_cast<const float4*>(dagg + (int64_t)row * ld_dagg);
#pragma unroll
            for (int v = 0; v < VEC; ++v) x[j][v] = dr[min(c0 + v * 64 + lane, h4 - 1)];
          }
        }
      }
      float4 acc[VEC];
#pragma unroll
      for (int v = 0; v < VEC; ++v) acc[v] = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int g = 0; g < kDqChunk / 4; ++g) {
        if (g < ng) {
#pragma unroll
          for (int jj = 0; jj < 4; ++jj) {
            const int j = 4 * g + jj;
            const float w = j < n ? __shfl(my_w, j, 64) : 0.f;
#pragma unroll
            for (int v = 0; v < VEC; ++v) {
              acc[v].x = fmaf(w, x[j][v].x, acc[v].x);
              acc[v].y = fmaf(w, x[j][v].y, acc[v].y);
              acc[v].z = fmaf(w, x[j][v].z, acc[v].z);
              acc[v].w = fmaf(w, x[j][v].w, acc[v].w);
            }
          }
        }
      }
      float4* o = reinterpret_cast<float4*>(split || CM ? part + ci * hid : dpq + (int64_t)u * hid);
#pragma unroll
      for (int v = 0; v < VEC; ++v) {
        const int c = c0 + v * 64 + lane;
        if (c < h4)
          o[c] = split ? acc[v]
                       : make_float4(acc[v].x * lrelu_grad(qv[v].x), acc[v].y * lrelu_grad(qv[v].y),
                                     acc[v].z * lrelu_grad(qv[v].z), acc[v].w * lrelu_grad(qv[v].w));
      }
    }
    dsc = dsc_n;
    oc = oc_n;
  }
}

// dpq[u] = lrelu'(q[u]) * (sum of u's chunk partials) for the rows
// dq_chunk_kernel split (the scan's split list: {u, first chunk}).  One
// 1024-thread block per row: wave w sums partials j = w, w + 16, ... with 8
// loads in flight per lane, then the 16 wave sums are added in a fixed order in
// LDS (deterministic).  Popular rows have hundreds of partials, so a row's sum
// is spread over a block rather than one wave.
constexpr int kCombWaves = 16;
__global__ __launch_bounds__(1024) void dq_combine_kernel(const int2* __restrict__ split,
                                                          const int* __restrict__ nsplit,
                                                          const int* __restrict__ off,
                                                          const float* __restrict__ part,
                                                          const float* __restrict__ q, int hid,
                                                          float* __restrict__ dpq) {
  __shared__ float4 red[kCombWaves][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int h4 = hid >> 2;
  const int ns = *nsplit;
  for (int si = blockIdx.x; si < ns; si += gridDim.x) {
    const int2 sp = split[si];
    const int u = sp.x;
    const int64_t ci = sp.y;
    const int k = (off[u + 1] - off[u] + kDqChunk - 1) / kDqChunk;
    for (int c0 = 0; c0 < h4; c0 += 64) {
      const int c = c0 + lane;
      const int cc = min(c, h4 - 1);
      float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
      int j = wv;
      for (; j + 7 * kCombWaves < k; j += 8 * kCombWaves) {
        float4 x[8];
#pragma unroll
        for (int i = 0; i < 8; ++i)
          x[i] = reinterpret_cast<const float4*>(part + (ci + j + i * kCombWaves) * hid)[cc];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          acc.x += x[i].x;
          acc.y += x[i].y;
          acc.z += x[i].z;
          acc.w += x[i].w;
        }
      }
      for (; j < k; j += kCombWaves) {
        const float4 x = reinterpret_cast<const float4*>(part + (ci + j) * hid)[cc];
        acc.x += x.x;
        acc.y += x.y;
        acc.z += x.z;
        acc.w += x.w;
      }
      red[wv][lane] = acc;
      __syncthreads();
      if (wv == 0 && c < h4) {
        float4 t = red[0][lane];
        for (int i = 1; i < kCombWaves; ++i) {
          const float4 x = red[i][lane];
          t.x += x.x;
          t.y += x.y;
          t.z += x.z;
          t.w += x.w;
        }
        const float4 qq = reinterpret_cast<const float4*>(q + (int64_t)u * hid)[c];
        reinterpret_cast<float4*>(dpq + (int64_t)u * hid)[c] =
            make_float4(t.x * lrelu_grad(qq.x), t.y * lrelu_grad(qq.y), t.z * lrelu_grad(qq.z),
                        t.w * lrelu_grad(qq.w));
      }
      __syncthreads();
    }
  }
}

// ---------------------------------------------------------------- L2 norm + lrelu backward
// y = lrelu(p) / ||lrelu(p)||:  dp = lrelu'(y) * (dy - y (y . dy)) / ||.||
// Also zeroes (a) rows [0, *z_rows) x z_n of z (the previous layer's dY,
// about to receive scatter-adds) and (b) zi[0, zi_n) (multiplicity counters of
// the loss, consumed by now) -- work that would otherwise be memset launches.
__global__ __launch_bounds__(256) void norm_lrelu_bwd_kernel(const float* __restrict__ y,
                                                             const float* __restrict__ nrm,
                                                             const float* __restrict__ dy, int n,
                                                             const int* __restrict__ nrows,
                                                             int64_t n_static,
                                                             float* __restrict__ dp,
                                                             float* __restrict__ z, int z_n,
                                                             const int* __restrict__ z_rows,
                                                             int* __restrict__ zi, int64_t zi_n) {
  const int64_t gt = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t gs = (int64_t)gridDim.x * blockDim.x;
  const int64_t R = nrows ? (int64_t)*nrows : n_static;
  const int lane = threadIdx.x & 63;
  const int64_t wid = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t r = wid; r < R; r += nw) {
    float dot = 0.f;
    for (int c = lane; c < n; c += 64) dot += y[r * n + c] * dy[r * n + c];
    dot = wave_sum(dot);
    const float inv = 1.f / nrm[r];
    for (int c = lane; c < n; c += 64) {
      const float yy = y[r * n + c];
      dp[r * n + c] = lrelu_grad(yy) * (dy[r * n + c] - yy * dot) * inv;
    }
  }
  // the zeroing after the rows: loads issued behind stores wait for them
  if (z) {
    const int64_t zn = (int64_t)(*z_rows) * z_n;
    for (int64_t i = gt; i < zn; i += gs) z[i] = 0.f;
  }
  if (zi)
    for (int64_t i = gt; i < zi_n; i += gs) zi[i] = 0;
}

// In-place row L2 normalisation of y [n][out] (the W projection's last step,
// pinsage_model.py:210, for out_dim > 128, where the GEMM's fused L2-norm
// epilogue does not apply): one wave per row; norms[r] = ||y_r||.
__global__ __launch_bounds__(256) void l2norm_rows_kernel(float* __restrict__ y, int64_t n, int out,
                                                          float* __restrict__ norms) {
  const int lane = threadIdx.x & 63;
  const int64_t wid = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t r = wid; r < n; r += nw) {
    float s2 = 0.f;
    for (int c = lane; c < out; c += 64) s2 += y[r * out + c] * y[r * out + c];
    const float nrm = sqrtf(wave_sum(s2));
    for (int c = lane; c < out; c += 64) y[r * out + c] = y[r * out + c] / nrm;
    if (lane == 0 && norms) norms[r] = nrm;
  }
}

int launch_l2norm_rows(float* y, int64_t n, int out, float* norms, hipStream_t st) {
  if (n <= 0) return kOk;
  hipLaunchKernelGGL(l2norm_rows_kernel, dim3(grid_for(n * 64, 256, 4096)), dim3(256), 0, st, y, n, out, norms);
  PS_CHECK_LAUNCH();
  return kOk;
}

// ---------------------------------------------------------------- positions by rank
// The batch positions grouped by their top-set rank, in position order:
// pos_sorted[rank_off[r] .. rank_off[r + 1]) are the positions p with
// pos_rank[p] == r, increasing.  The loss (and the autograd path's output
// gradient) sum a repeated node's per-position gradients in that order
// (deterministic; see det_put below).  One block: a stable LSD radix sort of
// (rank << 16 | position) keys in LDS by the rank's two 7-bit digits.  Each of
// the 16 waves owns a contiguous run of keys and walks it 64 at a time; lanes
// holding the same digit find each other with seven ballots, so a key's place
// is its (digit, wave) base plus the count of same-digit lanes below it --
// stable without atomics.  More than kPosCsrMax positions marks the CSR absent
// (rank_off[0] = -1) and the writers fall back to float atomics.
constexpr int kPosCsrMax = 16384;  // ranks < 2^14: two 7-bit digits
constexpr int kPosDig = 7, kPosBuckets = 1 << kPosDig, kPosWaves = 16;
constexpr int kPosCsrLds = 2 * kPosCsrMax * 4 + kPosBuckets * kPosWaves * 4 + 64;
__device__ __forceinline__ unsigned long long match_digit(int dig, bool valid) {
  unsigned long long m = __ballot(valid);
#pragma unroll
  for (int bit = 0; bit < kPosDig; ++bit) {
    const unsigned long long bb = __ballot((dig >> bit) & 1);
    m &= ((dig >> bit) & 1) ? bb : ~bb;
  }
  return m;
}
__global__ __launch_bounds__(1024) void pos_csr_kernel(const int32_t* __restrict__ pos_rank, int n,
                                                       const int* __restrict__ nS, int* __restrict__ rank_off,
                                                       int32_t* __restrict__ pos_sorted) {
  extern __shared__ unsigned pk[];
  if (n > kPosCsrMax) {
    if (threadIdx.x == 0) rank_off[0] = -1;
    return;
  }
  unsigned* src = pk;
  unsigned* dst = pk + kPosCsrMax;
  int* base = reinterpret_cast<int*>(pk + 2 * kPosCsrMax);  // [bucket][wave]
  int* wsum = base + kPosBuckets * kPosWaves;                // [16] scan scratch
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  for (int i = tid; i < n; i += blockDim.x) src[i] = ((unsigned)pos_rank[i] << 16) | (unsigned)i;
  const int seg = ((n + kPosWaves - 1) / kPosWaves + 63) & ~63;
  const int w0 = min(n, wv * seg), w1 = min(n, w0 + seg);
  const unsigned long long below = (1ull << lane) - 1ull;
  for (int pass = 0; pass < 2; ++pass) {
    const int sh = 16 + kPosDig * pass;
    for (int i = tid; i < kPosBuckets * kPosWaves; i += blockDim.x) base[i] = 0;
    __syncthreads();
    for (int i0 = w0; i0 < w1; i0 += 64) {  // this wave's digit counts (column wv only)
      const int i = i0 + lane;
      const bool valid = i < w1;
      const int dig = valid ? (int)(src[i] >> sh) & (kPosBuckets - 1) : 0;
      const unsigned long long m = match_digit(dig, valid);
      if (valid && (m & below) == 0) base[dig * kPosWaves + wv] += __popcll(m);
    }
    __syncthreads();
    // exclusive scan of the (bucket, wave) counts, two per thread
    const int c0 = base[2 * tid], c1 = base[2 * tid + 1];
    int inc = c0 + c1;
    for (int o = 1; o < 64; o <<= 1) {
      const int y = __shfl_up(inc, o, 64);
      if (lane >= o) inc += y;
    }
    if (lane == 63) wsum[wv] = inc;
    __syncthreads();
    int pre = inc - c0 - c1;
    for (int w = 0; w < wv; ++w) pre += wsum[w];
    base[2 * tid] = pre;
    base[2 * tid + 1] = pre + c0;
    __syncthreads();
    for (int i0 = w0; i0 < w1; i0 += 64) {  // stable placement
      const int i = i0 + lane;
      const bool valid = i < w1;
      const unsigned key = valid ? src[i] : 0u;
      const int dig = (int)(key >> sh) & (kPosBuckets - 1);
      const unsigned long long m = match_digit(dig, valid);
      const int b = valid ? base[dig * kPosWaves + wv] : 0;
      __builtin_amdgcn_wave_barrier();
      if (valid) {
        dst[b + __popcll(m & below)] = key;
        if ((m & below) == 0) base[dig * kPosWaves + wv] = b + __popcll(m);
      }
      __builtin_amdgcn_wave_barrier();
    }
    __syncthreads();
    unsigned* t = src;
    src = dst;
    dst = t;
  }
  // every rank 0..nS gets an offset, the ranks without a position too (the
  // on-the-fly step's virtual nodes: top-set ranks no batch position names)
  for (int i = tid; i < n; i += blockDim.x) {
    const unsigned v = src[i];
    const int r = (int)(v >> 16);
    pos_sorted[i] = (int32_t)(v & 0xffffu);
    const int rp = i == 0 ? -1 : (int)(src[i - 1] >> 16);
    for (int q = rp + 1; q <= r; ++q) rank_off[q] = i;
  }
  const int qe = max(*nS, (int)(src[n - 1] >> 16) + 1);
  for (int q = (int)(src[n - 1] >> 16) + 1 + tid; q <= qe; q += blockDim.x) rank_off[q] = n;
}

int launch_pos_csr(const int32_t* pos_rank, int64_t n, const int* nS, int* rank_off, int32_t* pos_sorted,
                   hipStream_t st) {
  static bool prepared = false;
  if (!prepared) {
    PS_CHECK_HIP(hipFuncSetAttribute((const void*)pos_csr_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                     kPosCsrLds));
    prepared = true;
  }
  if (n <= 0) return kOk;
  hipLaunchKernelGGL(pos_csr_kernel, dim3(1), dim3(1024), n <= kPosCsrMax ? (unsigned)kPosCsrLds : 0u, st, pos_rank,
                     (int)std::min<int64_t>(n, INT32_MAX), nS, rank_off, pos_sorted);
  PS_CHECK_LAUNCH();
  return kOk;
}

// Deterministic accumulation of one position's gradient row x (held by a wave,
// XPL values per lane, column lane + 64 i) into G[grp][r] (row stride d), in
// two passes with no float atomics and no cross-workgroup fences:
//   * the node's only position in the batch (the common case): G row = x;
//   * a repeated node: x goes to Gp[p] (zeros from an inactive triple too), and
//     rep_sum_kernel, launched behind the writer, sums each group's rows in
//     position order (pos_sorted) into G -- bitwise the same on every run.
//   rank_off[0] == -1 (no position CSR): float atomics (order-dependent).
// mode (det_mode): -1 atomics, 0 the only position, 1 a repeated node.  The
// caller loads it with its other operands: read here, behind the row stores
// of an earlier det_put, each load waited for those stores.
__device__ __forceinline__ int det_mode(int ro0, int a0, int a1) { return ro0 < 0 ? -1 : a1 - a0 == 1 ? 0 : 1; }
template <int XPL>
__device__ __forceinline__ void det_put(const float (&x)[XPL], int d, int p, int r, int grp, int mode,
                                        float* __restrict__ G, int64_t S_max, float* __restrict__ Gp, int lane) {
  float* g = G + ((int64_t)grp * S_max + r) * d;
  if (mode < 0) {
#pragma unroll
    for (int i = 0; i < XPL; ++i)
      if (lane + 64 * i < d) atomicAdd(g + lane + 64 * i, x[i]);
    return;
  }
  float* dst = mode == 0 ? g : Gp + (int64_t)p * d;
#pragma unroll
  for (int i = 0; i < XPL; ++i)
    if (lane + 64 * i < d) dst[lane + 64 * i] = x[i];
}

// Second pass: one wave per repeated rank r; G[grp][r] = the sum, in position
// order, of the rows Gp[p] of r's positions p with p % ng == grp (groups with
// no position keep their zero row).  Sixteen rows are in flight at a time
// (their positions one load by lanes 0..15), added in order.
constexpr int kRepBatch = 16;
template <int XPL, int NG>
__global__ __launch_bounds__(256) void rep_sum_kernel(const int* __restrict__ rank_off,
                                                      const int32_t* __restrict__ pos_sorted,
                                                      const int* __restrict__ nS, int d,
                                                      const float* __restrict__ Gp, float* __restrict__ G,
                                                      int64_t S_max) {
  if (rank_off[0] < 0) return;
  const int lane = threadIdx.x & 63;
  const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
  const int64_t R = *nS;
  for (int64_t r = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; r < R; r += nw) {
    const int o0 = rank_off[r], o1 = rank_off[r + 1];
    if (o1 - o0 < 2) continue;
    float acc[NG][XPL];
    bool any[NG];
#pragma unroll
    for (int c = 0; c < NG; ++c) {
      any[c] = false;
#pragma unroll
      for (int i = 0; i < XPL; ++i) acc[c][i] = 0.f;
    }
    for (int o = o0; o < o1; o += kRepBatch) {
      const int my_q = lane < kRepBatch && o + lane < o1 ? pos_sorted[o + lane] : -1;
      int q[kRepBatch];
      float v[kRepBatch][XPL];
#pragma unroll
      for (int u = 0; u < kRepBatch; ++u) q[u] = __shfl(my_q, u, 64);
#pragma unroll
      for (int u = 0; u < kRepBatch; ++u)
#pragma unroll
        for (int i = 0; i < XPL; ++i)
          v[u][i] = q[u] >= 0 && lane + 64 * i < d ? Gp[(int64_t)q[u] * d + lane + 64 * i] : 0.f;
#pragma unroll
      for (int u = 0; u < kRepBatch; ++u) {
        if (q[u] < 0) continue;
        const int c = NG == 1 ? 0 : q[u] % NG;
#pragma unroll
        for (int cc = 0; cc < NG; ++cc)
          if (cc == c) {
            any[cc] = true;
#pragma unroll
            for (int i = 0; i < XPL; ++i) acc[cc][i] += v[u][i];
          }
      }
    }
#pragma unroll
    for (int c = 0; c < NG; ++c)
      if (any[c]) {
        float* g = G + ((int64_t)c * S_max + r) * d;
#pragma unroll
        for (int i = 0; i < XPL; ++i)
          if (lane + 64 * i < d) g[lane + 64 * i] = acc[c][i];
      }
  }
}

// ---------------------------------------------------------------- loss
// One wave per triple b: rows rq, rp, rn of Z (head outputs of the unique top
// nodes).  Per call c in {q, pos, neg} and position b, the reference's
// backward hands the output row the SUM of the gradients of every position of
// that call holding the same node (index_put backward, pinsage_model.py:29 then
// :265), so G[c][rank] accumulates those sums and K[c][rank] the multiplicity;
// dZ = sum_c K[c] * G[c] is formed by the head backward as it loads its rows
// (head.hip), or by dz_combine_kernel for the unfused head.
//
// Two memory round trips per wave: the triple's indices (pos_rank, batch ids),
// then every Z and feature value it needs, into registers (ZPL / FPL values per
// lane and row), before any arithmetic.  The variance monitor's per-block
// column partials come from the query rows already in registers (via LDS);
// loss_monitor_kernel reduces them beside the backward.
template <int ZPL, int FPL>
__global__ __launch_bounds__(256) void loss_triple_kernel(
    const float* __restrict__ Z, int d, const int32_t* __restrict__ pos_rank, int B, float margin,
    const float* __restrict__ feats, int64_t ld_f, int d_in, const int64_t* __restrict__ batch,
    float* __restrict__ G, int* __restrict__ Kc, int64_t S_max, float* __restrict__ part,
    float* __restrict__ colpart, float* __restrict__ hinge, const int* __restrict__ rank_off,
    float* __restrict__ Gp) {
  __shared__ float red[4][4];  // per wave: loss, nfl, sum||h_q||^2, unused
  __shared__ float qrow[4][64 * ZPL];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int b = blockIdx.x * 4 + wv;
  const bool valid = b < B;
  // round 1: indices
  int rq = 0, rp = 0, rn = 0;
  int64_t iq = 0, ip = 0, in = 0;
  const int ro0 = rank_off[0];
  if (valid) {
    rq = pos_rank[3 * b];
    rp = pos_rank[3 * b + 1];
    rn = pos_rank[3 * b + 2];
    if (feats) {
      iq = batch[3 * b];
      ip = batch[3 * b + 1];
      in = batch[3 * b + 2];
    }
  }
  // round 2: rows into registers, with each rank's position count (det_mode;
  // no position CSR: rank_off[0], [1] are read and ignored)
  int mode[3];
  {
    const int rr[3] = {rq, rp, rn};
    int a0[3], a1[3];
#pragma unroll
    for (int c3 = 0; c3 < 3; ++c3) {
      const int at = ro0 >= 0 ? rr[c3] : 0;
      a0[c3] = rank_off[at];
      a1[c3] = rank_off[at + 1];
    }
#pragma unroll
    for (int c3 = 0; c3 < 3; ++c3) mode[c3] = det_mode(ro0, a0[c3], a1[c3]);
  }
  float zq[ZPL], zp[ZPL], zn[ZPL];
#pragma unroll
  for (int i = 0; i < ZPL; ++i) {
    const int c = lane + 64 * i;
    const bool ok = valid && c < d;
    zq[i] = ok ? Z[(int64_t)rq * d + c] : 0.f;
    zp[i] = ok ? Z[(int64_t)rp * d + c] : 0.f;
    zn[i] = ok ? Z[(int64_t)rn * d + c] : 0.f;
  }
  float fq[FPL], fp[FPL], fn[FPL];
#pragma unroll
  for (int i = 0; i < FPL; ++i) {
    const int c = lane + 64 * i;
    const bool ok = valid && feats && c < d_in;
    fq[i] = ok ? feats[iq * ld_f + c] : 0.f;
    fp[i] = ok ? feats[ip * ld_f + c] : 0.f;
    fn[i] = ok ? feats[in * ld_f + c] : 0.f;
  }
  float lossv = 0.f, nflv = 0.f, sq = 0.f;
  {
    // --- max_margin_loss on the model outputs
    float dq_ = 0.f, dp_ = 0.f, dn_ = 0.f, qp = 0.f, qn = 0.f;
#pragma unroll
    for (int i = 0; i < ZPL; ++i) {
      dq_ += zq[i] * zq[i];
      dp_ += zp[i] * zp[i];
      dn_ += zn[i] * zn[i];
      qp += zq[i] * zp[i];
      qn += zq[i] * zn[i];
    }
    dq_ = wave_sum(dq_);
    dp_ = wave_sum(dp_);
    dn_ = wave_sum(dn_);
    qp = wave_sum(qp);
    qn = wave_sum(qn);
    sq = dq_;
    const float nq = fmaxf(sqrtf(dq_), 1e-12f), np = fmaxf(sqrtf(dp_), 1e-12f),
                nn = fmaxf(sqrtf(dn_), 1e-12f);
    const float cqp = qp / (nq * np), cqn = qn / (nq * nn);
    const float ds = cqn - cqp + margin;
    if (valid && hinge && lane == 0) hinge[b] = ds;  // the hinge argument (parity tests read it)
    lossv = (valid && ds >= 0.f) ? ds : 0.f;
    const float g = (valid && ds >= 0.f) ? 1.f / (float)B : 0.f;
    if (g != 0.f) {
      // d/d(normalised rows): q_hat <- g(n_hat - p_hat), p_hat <- -g q_hat,
      // n_hat <- g q_hat; then x_hat = x/||x||: dx = (g_hat - x_hat (x_hat.g_hat)) / ||x||
      float pq = 0.f, pp = 0.f, pn = 0.f;
#pragma unroll
      for (int i = 0; i < ZPL; ++i) {
        const float a = zq[i] / nq, p = zp[i] / np, n = zn[i] / nn;
        pq += a * (g * (n - p));
        pp += p * (-g * a);
        pn += n * (g * a);
      }
      pq = wave_sum(pq);
      pp = wave_sum(pp);
      pn = wave_sum(pn);
      float xq[ZPL], xp[ZPL], xn[ZPL];
#pragma unroll
      for (int i = 0; i < ZPL; ++i) {
        const float a = zq[i] / nq, p = zp[i] / np, n = zn[i] / nn;
        xq[i] = (g * (n - p) - a * pq) / nq;
        xp[i] = (-g * a - p * pp) / np;
        xn[i] = (g * a - n * pn) / nn;
      }
      det_put<ZPL>(xq, d, 3 * b, rq, 0, mode[0], G, S_max, Gp, lane);
      det_put<ZPL>(xp, d, 3 * b + 1, rp, 1, mode[1], G, S_max, Gp, lane);
      det_put<ZPL>(xn, d, 3 * b + 2, rn, 2, mode[2], G, S_max, Gp, lane);
    } else if (valid && ro0 >= 0) {
      // an inactive triple's positions of a repeated node hold zero rows (the
      // ordered sum reads every position of the node)
#pragma unroll
      for (int c3 = 0; c3 < 3; ++c3)
        if (mode[c3] == 1)
#pragma unroll
          for (int i = 0; i < ZPL; ++i)
            if (lane + 64 * i < d) Gp[(int64_t)(3 * b + c3) * d + lane + 64 * i] = 0.f;
    }
    if (valid && lane == 0) {
      atomicAdd(Kc + 0 * S_max + rq, 1);
      atomicAdd(Kc + 1 * S_max + rp, 1);
      atomicAdd(Kc + 2 * S_max + rn, 1);
    }
    // --- monitor: cosine triplet loss on raw features (margin 1e-4)
    if (feats) {
      float fqq = 0.f, fpp = 0.f, fnn = 0.f, fqp = 0.f, fqn = 0.f;
#pragma unroll
      for (int i = 0; i < FPL; ++i) {
        fqq += fq[i] * fq[i];
        fpp += fp[i] * fp[i];
        fnn += fn[i] * fn[i];
        fqp += fq[i] * fp[i];
        fqn += fq[i] * fn[i];
      }
      // (d_in > 64 * FPL: the rest of the row, streamed)
      for (int c = lane + 64 * FPL; valid && c < d_in; c += 64) {
        const float a = feats[iq * ld_f + c], p = feats[ip * ld_f + c], n = feats[in * ld_f + c];
        fqq += a * a;
        fpp += p * p;
        fnn += n * n;
        fqp += a * p;
        fqn += a * n;
      }
      fqq = wave_sum(fqq);
      fpp = wave_sum(fpp);
      fnn = wave_sum(fnn);
      fqp = wave_sum(fqp);
      fqn = wave_sum(fqn);
      // inputs are normalised first (F.normalize), then cosine similarity
      const float aq = fmaxf(sqrtf(fqq), 1e-12f), ap = fmaxf(sqrtf(fpp), 1e-12f),
                  an = fmaxf(sqrtf(fnn), 1e-12f);
      const float hq2 = fqq / (aq * aq), hp2 = fpp / (ap * ap), hn2 = fnn / (an * an);
      const float cp = (fqp / (aq * ap)) / fmaxf(sqrtf(hq2 * hp2), 1e-8f);
      const float cn = (fqn / (aq * an)) / fmaxf(sqrtf(hq2 * hn2), 1e-8f);
      const float v = (1.f - cp) - (1.f - cn) + 1e-4f;
      nflv = (valid && v > 0.f) ? v : 0.f;
    }
  }
  // per-block column sum and sum of squared deviations from the block's own
  // column mean over its (<= 4) query rows (variance monitor; Chan's merge below)
#pragma unroll
  for (int i = 0; i < ZPL; ++i) qrow[wv][lane + 64 * i] = zq[i];
  if (lane == 0) {
    red[wv][0] = lossv;
    red[wv][1] = nflv;
    red[wv][2] = valid ? sq : 0.f;
  }
  __syncthreads();
  const int nb = min(4, B - (int)blockIdx.x * 4);
  for (int c = tid; c < d; c += 256) {
    float s = 0.f;
    for (int k = 0; k < nb; ++k) s += qrow[k][c];
    const float mb = s / (float)nb;
    float m2 = 0.f;
    for (int k = 0; k < nb; ++k) m2 += (qrow[k][c] - mb) * (qrow[k][c] - mb);
    colpart[(int64_t)blockIdx.x * 2 * d + c] = s;
    colpart[(int64_t)blockIdx.x * 2 * d + d + c] = m2;
  }
  if (tid == 0) {
    for (int k = 0; k < 3; ++k) part[(int64_t)blockIdx.x * 4 + k] = red[0][k] + red[1][k] + red[2][k] + red[3][k];
  }
}

// The step's monitors (pinsage_training.py:200-212): one block reduces, in a
// fixed order, the per-block partials of the loss kernel into scal[0] = loss,
// scal[1] = node-feature loss, scal[2] = sum |h_q|^2 and the variance
// (pinsage_training.py:99-103) -- Chan's merge of the per-block (sum, M2)
// column partials, M2 = sum_g M2_g + n_g (mean_g - mean)^2 (deviations, never
// |h|^2 - |mean|^2).  Nothing in the backward reads these: the engine runs it
// beside the backward.
__global__ __launch_bounds__(1024) void loss_monitor_kernel(const float* __restrict__ part,
                                                            int nparts,
                                                            const float* __restrict__ colpart,
                                                            int d, int B, float* __restrict__ scal) {
  __shared__ float cs[1024];
  __shared__ float mean_s[1024];
  __shared__ float wred[16][3];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  float l = 0.f, nf = 0.f, sq = 0.f;
  for (int i = t; i < nparts; i += 1024) {
    l += part[i * 4 + 0];
    nf += part[i * 4 + 1];
    sq += part[i * 4 + 2];
  }
  // column sums of the query rows: thread (grp, c) sums parts grp, grp+ng, ...
  const int ng = 1024 / d, c = t % d, grp = t / d;
  const int64_t ld2 = 2 * (int64_t)d;
  float cv = 0.f;
  if (grp < ng) {
    int g = grp;
    for (; g + 3 * ng < nparts; g += 4 * ng)
      cv += (colpart[g * ld2 + c] + colpart[(g + ng) * ld2 + c]) +
            (colpart[(g + 2 * ng) * ld2 + c] + colpart[(g + 3 * ng) * ld2 + c]);
    for (; g < nparts; g += ng) cv += colpart[g * ld2 + c];
  }
  cs[t] = cv;
  l = wave_sum(l);
  nf = wave_sum(nf);
  sq = wave_sum(sq);
  if (lane == 0) {
    wred[wv][0] = l;
    wred[wv][1] = nf;
    wred[wv][2] = sq;
  }
  __syncthreads();
  if (t < d) {
    float tot = 0.f;
    for (int q = 0; q < ng; ++q) tot += cs[q * d + t];
    mean_s[t] = tot / (float)B;
  }
  __syncthreads();
  float m2 = 0.f;
  if (grp < ng) {
    const float m = mean_s[c];
    for (int g = grp; g < nparts; g += ng) {
      const int n_g = min(4, B - 4 * g);
      const float dm = colpart[g * ld2 + c] / (float)n_g - m;
      m2 += colpart[g * ld2 + d + c] + (float)n_g * dm * dm;
    }
  }
  m2 = wave_sum(m2);
  __syncthreads();
  if (lane == 0) cs[wv] = m2;
  __syncthreads();
  if (t == 0) {
    float lsum = 0.f, nfs = 0.f, sqs = 0.f, ms = 0.f;
    for (int i = 0; i < 16; ++i) {
      lsum += wred[i][0];
      nfs += wred[i][1];
      sqs += wred[i][2];
      ms += cs[i];
    }
    scal[0] = lsum / (float)B;
    scal[1] = nfs / (float)B;
    scal[2] = sqs;
    scal[3] = ms / (float)(B - 1);
  }
}

// dZ[r] = sum_c K[c][r] * G[c][r], and G is zeroed behind the read (the unfused
// head's path; the fused head backward forms dZ itself).  Kc is zeroed by the
// first backward kernel.
__global__ __launch_bounds__(1024) void dz_combine_kernel(float* __restrict__ G,
                                                          const int* __restrict__ Kc, int64_t S_max,
                                                          const int* __restrict__ nS, int d,
                                                          float* __restrict__ dZ) {
  const int64_t S = *nS;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < S * d;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = e / d;
    float v = 0.f;
    for (int c = 0; c < 3; ++c) {
      const int k = Kc[c * S_max + r];
      if (k) {
        v += (float)k * G[c * S_max * d + e];
        G[c * S_max * d + e] = 0.f;
      }
    }
    dZ[e] = v;
  }
}

// ---------------------------------------------------------------- Adam
// torch.optim.Adam step (pinsage_training.py:147,191; torch _single_tensor_adam):
//   m = lerp(m, g, 1-b1); v = b2 v + (1-b2) g^2
//   p -= step_size * m / (sqrt(v) / bc2_sqrt + eps)
// coef = {step_size = lr / (1 - b1^t), bc2_sqrt = sqrt(1 - b2^t)} comes from
// device memory, written by the host beside the batch ids each step (the host
// computes them in double exactly as torch does), so the replayed graph needs
// no step counter on the device.
__device__ __forceinline__ void adam1(float& p, float g, float& m, float& v, float ss, float bc2,
                                      float beta2, float omb1, float omb2, float eps) {
  m = m + omb1 * (g - m);
  v = v * beta2 + omb2 * g * g;
  const float denom = sqrtf(v) / bc2 + eps;
  p = p - ss * (m / denom);
}
__global__ __launch_bounds__(256) void adam_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                   float* __restrict__ m, float* __restrict__ v,
                                                   int64_t n, const float* __restrict__ coef,
                                                   float beta2, float omb1, float omb2, float eps) {
  const float ss = coef[0], bc2 = coef[1];
  // bc2 = sqrt(1 - beta2^t) > 0 on every real step; 0 marks a step the device
  // refused (the on-the-fly sampler's error words, pinsage_fly_gate_adam):
  // parameters and moments stay untouched, as when the reference raises
  if (!(bc2 > 0.f)) return;
  const int64_t n4 = n >> 2;
  float4* p4 = reinterpret_cast<float4*>(p);
  float4* m4 = reinterpret_cast<float4*>(m);
  float4* v4 = reinterpret_cast<float4*>(v);
  const float4* g4 = reinterpret_cast<const float4*>(g);
  const int64_t t0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x, ts = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = t0; i < n4; i += ts) {
    float4 pp = p4[i], mm = m4[i], vv = v4[i];
    const float4 gg = g4[i];
    adam1(pp.x, gg.x, mm.x, vv.x, ss, bc2, beta2, omb1, omb2, eps);
    adam1(pp.y, gg.y, mm.y, vv.y, ss, bc2, beta2, omb1, omb2, eps);
    adam1(pp.z, gg.z, mm.z, vv.z, ss, bc2, beta2, omb1, omb2, eps);
    adam1(pp.w, gg.w, mm.w, vv.w, ss, bc2, beta2, omb1, omb2, eps);
    p4[i] = pp;
    m4[i] = mm;
    v4[i] = vv;
  }
  for (int64_t i = 4 * n4 + t0; i < n; i += ts) adam1(p[i], g[i], m[i], v[i], ss, bc2, beta2, omb1, omb2, eps);
}

// out[i][:] = Z[pos_rank[i]][:]
__global__ void gather_out_kernel(const float* __restrict__ Z, int d, const int32_t* __restrict__ pr,
                                  int64_t n, float* __restrict__ out) {
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n * d;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = e / d, c = e - i * d;
    out[e] = Z[(int64_t)pr[i] * d + c];
  }
}

// get_embeddings' row gather h[idx, :d] (pinsage_model.py:21-23) as an op:
// one wave per output row, float4 columns when rows are 16-B aligned.  Ids
// outside [0, n_h) give a zero row (the caller validates; the reference raises).
__global__ __launch_bounds__(256) void gather_rows_kernel(const float* __restrict__ h, int64_t ldh,
                                                          int64_t n_h, int d, const int64_t* __restrict__ idx,
                                                          int64_t n, float* __restrict__ out, int64_t ldo,
                                                          bool vec) {
  const int lane = threadIdx.x & 63;
  const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t r = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; r < n; r += nw) {
    const int64_t s = idx[r];
    const bool ok = s >= 0 && s < n_h;
    const float* src = h + (ok ? s : 0) * ldh;
    float* dst = out + r * ldo;
    if (vec) {
      for (int c = lane; c < (d >> 2); c += 64)
        reinterpret_cast<float4*>(dst)[c] =
            ok ? reinterpret_cast<const float4*>(src)[c] : make_float4(0.f, 0.f, 0.f, 0.f);
    } else {
      for (int c = lane; c < d; c += 64) dst[c] = ok ? src[c] : 0.f;
    }
  }
}

// one call: G[r] = sum of dout rows at positions of node r (in position order,
// det_put + rep_sum_kernel), K[r] = multiplicity; one wave per position
__global__ __launch_bounds__(256) void dout_accum_kernel(const float* __restrict__ dout, int d,
                                                         const int32_t* __restrict__ pr, int64_t n,
                                                         float* __restrict__ G, int* __restrict__ Kc, int64_t S_max,
                                                         const int* __restrict__ rank_off,
                                                         float* __restrict__ Gp) {
  const int lane = threadIdx.x & 63;
  const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; i < n; i += nw) {
    const int r = pr[i];
    float x[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) x[k] = lane + 64 * k < d ? dout[i * d + lane + 64 * k] : 0.f;
    const int ro0 = rank_off[0], at = ro0 >= 0 ? r : 0;
    det_put<4>(x, d, (int)i, r, 0, det_mode(ro0, rank_off[at], rank_off[at + 1]), G, S_max, Gp, lane);
    if (lane == 0) atomicAdd(Kc + r, 1);
  }
}
__global__ void dz_scale_kernel(const float* __restrict__ G, const int* __restrict__ Kc, int d,
                                const int* __restrict__ nS, float* __restrict__ dZ) {
  const int64_t S = *nS;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < S * d;
       e += (int64_t)gridDim.x * blockDim.x) {
    dZ[e] = (float)Kc[e / d] * G[e];
    ((float*)G)[e] = 0.f;
  }
}

// Split-K reduction: out[m*ld + n] = sum_s part[s*stride + m*N + n] and
// bias_out[m] = sum_s bpart[s*M + m].  A block is 64 float4 columns x 4 slab
// groups: each thread issues its S/4 loads together (the reduction is latency-
// bound otherwise: few outputs, many slabs), then the 4 groups are combined in
// LDS in a fixed order (deterministic).  Blocks >= nb_main do the bias.
__global__ __launch_bounds__(256) void reduce_slabs_2d_kernel(const float* __restrict__ part, int S,
                                                              int64_t stride, int M, int N,
                                                              float* __restrict__ out, int64_t ld,
                                                              const float* __restrict__ bpart,
                                                              float* __restrict__ bias_out,
                                                              int nb_main, AdamSlice ad) {
  __shared__ float4 red[4][64];
  const int j = threadIdx.x & 63, g = threadIdx.x >> 6;
  float ss = 0.f, bc2 = 1.f, omb1 = 0.f, omb2 = 0.f;
  if (ad.coef) {
    ss = ad.coef[0];
    bc2 = ad.coef[1];
    omb1 = (float)(1.0 - ad.beta1);
    omb2 = (float)(1.0 - ad.beta2);
  }
  if ((int)blockIdx.x < nb_main) {
    const int64_t e4 = (int64_t)blockIdx.x * 64 + j;  // float4 index into [M][N]
    const bool ok = e4 * 4 < (int64_t)M * N;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    if (ok) {
      const float4* p4 = reinterpret_cast<const float4*>(part) + e4;
      const int64_t st4 = stride / 4;
      int k = g;
      for (; k + 12 < S; k += 16) {
        const float4 x0 = p4[k * st4], x1 = p4[(k + 4) * st4], x2 = p4[(k + 8) * st4],
                     x3 = p4[(k + 12) * st4];
        acc.x += (x0.x + x1.x) + (x2.x + x3.x);
        acc.y += (x0.y + x1.y) + (x2.y + x3.y);
        acc.z += (x0.z + x1.z) + (x2.z + x3.z);
        acc.w += (x0.w + x1.w) + (x2.w + x3.w);
      }
      for (; k < S; k += 4) {
        const float4 x = p4[k * st4];
        acc.x += x.x;
        acc.y += x.y;
        acc.z += x.z;
        acc.w += x.w;
      }
    }
    red[g][j] = acc;
    __syncthreads();
    if (g == 0 && ok) {
      const float4 a = red[0][j], b = red[1][j], c = red[2][j], d = red[3][j];
      const float4 r = make_float4((a.x + b.x) + (c.x + d.x), (a.y + b.y) + (c.y + d.y),
                                   (a.z + b.z) + (c.z + d.z), (a.w + b.w) + (c.w + d.w));
      const int64_t e = e4 * 4, m = e / N, n = e - m * N, o = m * ld + n;
      *reinterpret_cast<float4*>(out + o) = r;
      if (ad.p && bc2 > 0.f) {  // the slice's Adam step, as adam_kernel would apply it (bc2 0: refused)
        float4 pp = *reinterpret_cast<const float4*>(ad.p + o);
        float4 mm = *reinterpret_cast<const float4*>(ad.m + o);
        float4 vv = *reinterpret_cast<const float4*>(ad.v + o);
        adam1(pp.x, r.x, mm.x, vv.x, ss, bc2, (float)ad.beta2, omb1, omb2, ad.eps);
        adam1(pp.y, r.y, mm.y, vv.y, ss, bc2, (float)ad.beta2, omb1, omb2, ad.eps);
        adam1(pp.z, r.z, mm.z, vv.z, ss, bc2, (float)ad.beta2, omb1, omb2, ad.eps);
        adam1(pp.w, r.w, mm.w, vv.w, ss, bc2, (float)ad.beta2, omb1, omb2, ad.eps);
        *reinterpret_cast<float4*>(ad.p + o) = pp;
        *reinterpret_cast<float4*>(ad.m + o) = mm;
        *reinterpret_cast<float4*>(ad.v + o) = vv;
      }
    }
    return;
  }
  // bias: 64 rows x 4 slab groups per block
  float* redf = reinterpret_cast<float*>(&red[0][0]);
  const int64_t m = (int64_t)(blockIdx.x - nb_main) * 64 + j;
  float acc = 0.f;
  if (m < M)
    for (int k = g; k < S; k += 4) acc += bpart[(int64_t)k * M + m];
  redf[g * 64 + j] = acc;
  __syncthreads();
  if (g == 0 && m < M) {
    const float r = (redf[j] + redf[64 + j]) + (redf[128 + j] + redf[192 + j]);
    bias_out[m] = r;
    if (ad.pb && bc2 > 0.f) adam1(ad.pb[m], r, ad.mb[m], ad.vb[m], ss, bc2, (float)ad.beta2, omb1, omb2, ad.eps);
  }
}

// ---------------------------------------------------------------- host launchers
int launch_gather_out(const float* Z, int d, const int32_t* pr, int64_t n, float* out,
                      hipStream_t st) {
  if (n <= 0) return kOk;
  hipLaunchKernelGGL(gather_out_kernel, dim3(grid_for(n * d, 256)), dim3(256), 0, st, Z, d, pr, n,
                     out);
  PS_CHECK_LAUNCH();
  return kOk;
}

int launch_gather_rows(const float* h, int64_t ldh, int64_t n_h, int d, const int64_t* idx, int64_t n,
                       float* out, int64_t ldo, hipStream_t st) {
  PS_REQUIRE(d >= 0 && n >= 0 && ldh >= d && ldo >= d, kErrArg, "gather_rows: bad sizes");
  if (n == 0 || d == 0) return kOk;
  const bool vec = d % 4 == 0 && ldh % 4 == 0 && ldo % 4 == 0 && (uintptr_t)h % 16 == 0 && (uintptr_t)out % 16 == 0;
  hipLaunchKernelGGL(gather_rows_kernel, dim3(grid_for(n * 64, 256, 8192)), dim3(256), 0, st, h, ldh, n_h, d, idx,
                     n, out, ldo, vec);
  PS_CHECK_LAUNCH();
  return kOk;
}

// autograd: the output rows' cotangents go into the loss's accumulators (G slab
// 0, K slab 0); dZ = K * G is formed by the fused head backward (or here, for
// the unfused head: scale = true)
int launch_dz_from_dout(const float* dout, int d, const int32_t* pr, int64_t n, const int* nS,
                        int64_t S_max, float* G, int* Kc, float* dZ, bool scale, const int* rank_off,
                        const int32_t* pos_sorted, float* Gp, hipStream_t st) {
  PS_REQUIRE(d <= 256, kErrArg, "dz_from_dout: out_dim must be <= 256");
  hipLaunchKernelGGL(dout_accum_kernel, dim3(grid_for(n * 64, 256)), dim3(256), 0, st, dout, d, pr, n, G, Kc, S_max,
                     rank_off, Gp);
  PS_CHECK_LAUNCH();
  hipLaunchKernelGGL((rep_sum_kernel<4, 1>), dim3(grid_for(S_max * 64, 256)), dim3(256), 0, st, rank_off,
                     pos_sorted, nS, d, Gp, G, S_max);
  PS_CHECK_LAUNCH();
  if (scale) {
    hipLaunchKernelGGL(dz_scale_kernel, dim3(grid_for(S_max * d, 256)), dim3(256), 0, st, G, Kc, d, nS,
                       dZ);
    PS_CHECK_LAUNCH();
  }
  return kOk;
}

int launch_reduce_slabs_2d(const float* part, int S, int64_t stride, int M, int N, float* out,
                           int64_t ld, const float* bpart, float* bias_out, const AdamSlice* adam,
                           hipStream_t st) {
  PS_REQUIRE(N % 4 == 0 && ld % 4 == 0 && stride % 4 == 0 &&
                 (reinterpret_cast<uintptr_t>(out) & 15) == 0 &&
                 (reinterpret_cast<uintptr_t>(part) & 15) == 0,
             kErrArg, "reduce_slabs: needs 16-byte aligned rows");
  AdamSlice ad;
  if (adam) {
    ad = *adam;
    PS_REQUIRE(ad.p && ad.m && ad.v && ad.coef && (!bias_out || (ad.pb && ad.mb && ad.vb)) &&
                   ((reinterpret_cast<uintptr_t>(ad.p) | reinterpret_cast<uintptr_t>(ad.m) |
                     reinterpret_cast<uintptr_t>(ad.v)) & 15) == 0,
               kErrArg, "reduce_slabs: Adam slice needs 16-byte aligned state for every output");
  }
  const int nb_main = (int)ceil_div((int64_t)M * N / 4, 64);
  const int nb_bias = bias_out ? (int)ceil_div(M, 64) : 0;
  hipLaunchKernelGGL(reduce_slabs_2d_kernel, dim3(nb_main + nb_bias), dim3(256), 0, st, part, S, stride,
                     M, N, out, ld, bpart, bias_out, nb_main, ad);
  PS_CHECK_LAUNCH();
  return kOk;
}
// one layer's tables: p.* as in LayerPrep, S_max / N_max the set capacities
int launch_layer_preps(const LayerPrep* p, const int64_t* S_max, const int64_t* N_max, int n, int T, hipStream_t st) {
  PS_REQUIRE(n >= 1 && n <= kMaxPrepLayers, kErrArg, "layer_prep: 1..4 layers per launch");
  LayerPreps a;
  a.n = n;
  a.T = T;
  int64_t tot = 0;
  for (int l = 0; l < n; ++l) {
    PS_REQUIRE(!p[l].z || p[l].z_n % 4 == 0, kErrArg, "layer_prep: zeroed rows must be a multiple of 4 wide");
    a.L[l] = p[l];
    tot = std::max(tot, S_max[l] * T + S_max[l] + N_max[l] + p[l].n_ids);
  }
  hipLaunchKernelGGL(layer_prep_kernel, dim3(grid_for(tot, 256)), dim3(256), 0, st, a);
  PS_CHECK_LAUNCH();
  return kOk;
}

int launch_agg(const float* q, int hid, const int32_t* loc, const float* wloc, int T,
               const int* nS, int64_t S_max, float* agg, hipStream_t st) {
  PS_REQUIRE(hid % 4 == 0, kErrArg, "agg: hidden dim must be a multiple of 4");
  if (S_max <= 0) return kOk;
  // opt-in (PINSAGE_AGG_SLICED=1): in the step, where popular q rows repeat and
  // hit L2 anyway, the sliced form measured slower (C2 layer 0 15.9 vs 13.6 us,
  // C4 22.3 vs 19.1 us); on uniformly random slots it is faster (15.6 vs 20.3 us)
  const bool sliced = getenv("PINSAGE_AGG_SLICED") && atoi(getenv("PINSAGE_AGG_SLICED")) != 0;
  if (sliced && (hid == 512 || hid == 256 || hid == 128)) {
    // 4 waves per block, blocks in groups of 8 (one per XCD slice), ~2 passes per wave
    const int rpw = 64 / (hid / 32);
    const int64_t per_block = 4 * rpw * 2;
    const int64_t G = std::max<int64_t>(1, std::min<int64_t>((S_max + per_block - 1) / per_block, 1024));
    const dim3 gr((unsigned)(G * kXcds)), bl(256);
    if (hid == 512) hipLaunchKernelGGL((agg_sliced_kernel<16>), gr, bl, 0, st, q, hid, loc, wloc, T, nS, S_max, agg);
    else if (hid == 256) hipLaunchKernelGGL((agg_sliced_kernel<8>), gr, bl, 0, st, q, hid, loc, wloc, T, nS, S_max, agg);
    else hipLaunchKernelGGL((agg_sliced_kernel<4>), gr, bl, 0, st, q, hid, loc, wloc, T, nS, S_max, agg);
    PS_CHECK_LAUNCH();
    return kOk;
  }
  // hid >= 512: one wave per row (2 float4 per lane per slot, 8 slots in flight);
  // measured faster than two waves per row with all 16 slots in flight
  if (hid >= 512)
    hipLaunchKernelGGL((agg_kernel<2>), dim3(grid_for(S_max * 64, 256, 4096)), dim3(256), 0, st, q, hid,
                       loc, wloc, T, nS, S_max, agg);
  else
    hipLaunchKernelGGL((agg_kernel<1>), dim3(grid_for(S_max * ((hid / 4 + 63) / 64) * 64, 256, 8192)),
                       dim3(256), 0, st, q, hid, loc, wloc, T, nS, S_max, agg);
  PS_CHECK_LAUNCH();
  return kOk;
}

// CSR of the neighbour slots by q row.  cnt must be zero on entry (zeroed once
// by pinsage_engine_init_workspace, then left zero by the scan).  The count
// kernel also zeroes dpq's rows (the dq kernel's atomic targets).
// CSR of the neighbour slots by q row, plus the dq chunk list.  cnt must be
// zero on entry (zeroed once by pinsage_engine_init_workspace, then left zero
// by the scan).
// dynamic LDS above 64 KiB must be allowed per kernel (once, outside capture)
int csr_prepare() {
  static int rc = [] {
    if (hipFuncSetAttribute((const void*)csr_count_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                            kLdsRows * 4) != hipSuccess)
      return (int)kErrHip;
    if (hipFuncSetAttribute((const void*)csr_fill_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                            kLdsRows * 4) != hipSuccess)
      return (int)kErrHip;
    if (hipFuncSetAttribute((const void*)csr_sort_rows_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                            kRankLds) != hipSuccess)
      return (int)kErrHip;
    return (int)kOk;
  }();
  if (rc != kOk) set_error("csr: cannot raise the dynamic LDS limit");
  return rc;
}

int64_t dq_chunk_capacity(int64_t S_max, int T, int64_t N_max);
int launch_csr_build(const int32_t* loc, const float* wloc, const int* nS, int64_t S_max, int T, const int* nN,
                     int64_t N_max, int* cnt, int* bsum, int* off, int* cursor, int* cbase, int2* occ2,
                     int2* chunks, int* nchunks, int2* split, int* nsplit, float* dpq, int hid, hipStream_t st,
                     int2* occ2_tmp) {
  const int lds = (int)std::min<int64_t>(N_max, kLdsRows) * 4;
  // more rows than one histogram: (range, slice) items over a CU-wide grid
  const int gb = N_max > kLdsRows ? kCsrRangeGrid : std::max(1, std::min(128, ceil_div(S_max * T, 2048)));
  // dq writes every row it owns (no atomics), so dpq needs no zeroing
  (void)dpq;
  // PINSAGE_CSR_RANGES: the range cap (0: the per-wave global-atomic path
  // beyond one histogram; A/B and tests)
  const int max_ranges = getenv("PINSAGE_CSR_RANGES") ? atoi(getenv("PINSAGE_CSR_RANGES")) : kMaxRanges;
  hipLaunchKernelGGL(csr_count_kernel, dim3(gb), dim3(1024), lds, st, loc, nS, T, nN, cnt,
                     (float*)nullptr, hid, nsplit, max_ranges);
  PS_CHECK_LAUNCH();
  // one block scans small sets; from ~4k rows on its threads' serial runs
  // (N / 1024 rows each) outlast the two-launch form (C4 layer 1, ~15k rows:
  // 26 us in one block)
  if (N_max <= 4096) {
    hipLaunchKernelGGL(scan_small_kernel, dim3(1), dim3(1024), 0, st, cnt, nN, off, cursor, cbase, chunks,
                       nchunks, split, nsplit);
    PS_CHECK_LAUNCH();
  } else {
    const int nb = ceil_div(N_max + 1, kScanChunk);
    int2* bs = reinterpret_cast<int2*>(bsum);
    hipLaunchKernelGGL(scan_block_sums_kernel, dim3(nb), dim3(kScanB), 0, st, cnt, nN, bs);
    PS_CHECK_LAUNCH();
    hipLaunchKernelGGL(scan_apply_kernel, dim3(nb), dim3(kScanB), 0, st, cnt, nN, bs, off, cursor,
                       cbase, chunks, nchunks, split, nsplit);
    PS_CHECK_LAUNCH();
  }
  hipLaunchKernelGGL(csr_fill_kernel, dim3(gb), dim3(1024), lds, st, loc, wloc, nS, T, nN, cursor, off, cbase,
                     occ2, max_ranges, split, nsplit, chunks);
  PS_CHECK_LAUNCH();
  // canonical pair order (sorted by source row): bitwise-reproducible sums
  if (occ2_tmp) {
    const int64_t max_chunks = dq_chunk_capacity(S_max, T, N_max);
    hipLaunchKernelGGL(csr_sort_chunks_kernel, dim3(grid_for(max_chunks * 64, 256, 2048)), dim3(256), 0, st,
                       chunks, nchunks, off, occ2);
    PS_CHECK_LAUNCH();
    hipLaunchKernelGGL(csr_sort_rows_kernel, dim3(256), dim3(1024), kRankLds, st, split, nsplit, off, occ2,
                       occ2_tmp);
    PS_CHECK_LAUNCH();
  }
  return kOk;
}

// upper bound of the dq chunk list: one partial chunk per row plus full ones
int64_t dq_chunk_capacity(int64_t S_max, int T, int64_t N_max) {
  return N_max + (S_max * T + kDqChunk - 1) / kDqChunk + 1;
}
// upper bound of the split-row list: a split row holds more than kDqChunk slots
int64_t dq_split_capacity(int64_t S_max, int T) { return S_max * T / (kDqChunk + 1) + 1; }

// levels of the split-row tree for rows of up to max_chunks chunks (fan-in 8)
int dq_tree_levels(int64_t max_chunks) {
  int L = 1;
  for (int64_t n = 8; n < max_chunks; n *= 8) ++L;
  return L;
}

int launch_dq_chunks(const int2* chunks, const int* nchunks, int64_t max_chunks, const int2* split,
                     const int* nsplit, int64_t max_split, const int* off, const int2* occ2,
                     const float* dagg, int64_t ld_dagg, const float* q,
                     int hid, float* dpq, float* part, hipStream_t st, const int32_t* q_src,
                     int32_t* csrc, const int* cbase, int* tk, uint16_t* dpq3, int64_t ps3) {
  PS_REQUIRE(hid % 4 == 0, kErrArg, "dq: hidden dim must be a multiple of 4");
  // persistent waves (each prefetches its next chunk); 512 to 4096 blocks
  // measured alike at C2 (round 5), 1024 to 8192 at C2 and C4 (round 6), 2048
  // kept (PINSAGE_DQ_GRID: the cap, A/B)
  static const int grid_cap = getenv("PINSAGE_DQ_GRID") ? std::max(1, atoi(getenv("PINSAGE_DQ_GRID"))) : 2048;
  const int grid = grid_for(max_chunks * 64, 256, grid_cap);
  if (csrc) {  // chunk rows: masked partials in part, no combine
    PS_REQUIRE(q_src, kErrArg, "dq: chunk rows need the rows' source indices");
    if (hid >= 512)
      hipLaunchKernelGGL((dq_chunk_kernel<2, true>), dim3(grid), dim3(256), 0, st, chunks, nchunks, occ2, dagg,
                         ld_dagg, q, hid, dpq, part, q_src, csrc);
    else
      hipLaunchKernelGGL((dq_chunk_kernel<1, true>), dim3(grid), dim3(256), 0, st, chunks, nchunks, occ2, dagg,
                         ld_dagg, q, hid, dpq, part, q_src, csrc);
    PS_CHECK_LAUNCH();
    return kOk;
  }
  // (an XCD-sliced form -- block b on column slice b % 8 of every chunk, so
  // each XCD gathers its eighth of d_agg from its own L2 -- was bitwise this
  // kernel and slower in the step: C2 0.398-0.406 -> 0.408-0.50 ms, C4
  // 0.426-0.431 -> 0.447-0.452, round 6; removed)
  if (tk && cbase && hid <= 512 && dpq3) {  // the same, dpq written as bf16 planes
    if (hid > 256)
      hipLaunchKernelGGL((dq_chunk_kernel<2, false, true, true>), dim3(grid), dim3(256), 0, st, chunks, nchunks,
                         occ2, dagg, ld_dagg, q, hid, dpq, part, nullptr, nullptr, off, cbase, tk, max_chunks, dpq3,
                         ps3);
    else
      hipLaunchKernelGGL((dq_chunk_kernel<1, false, true, true>), dim3(grid), dim3(256), 0, st, chunks, nchunks,
                         occ2, dagg, ld_dagg, q, hid, dpq, part, nullptr, nullptr, off, cbase, tk, max_chunks, dpq3,
                         ps3);
    PS_CHECK_LAUNCH();
    return kOk;
  }
  PS_REQUIRE(!dpq3, kErrArg, "dq: planes output needs the split-row tree and hid <= 512");
  if (tk && cbase && hid <= 512) {  // split rows combined by their own chunks (no combine launch)
    if (hid > 256)
      hipLaunchKernelGGL((dq_chunk_kernel<2, false, true>), dim3(grid), dim3(256), 0, st, chunks, nchunks, occ2,
                         dagg, ld_dagg, q, hid, dpq, part, nullptr, nullptr, off, cbase, tk, max_chunks);
    else
      hipLaunchKernelGGL((dq_chunk_kernel<1, false, true>), dim3(grid), dim3(256), 0, st, chunks, nchunks, occ2,
                         dagg, ld_dagg, q, hid, dpq, part, nullptr, nullptr, off, cbase, tk, max_chunks);
    PS_CHECK_LAUNCH();
    return kOk;
  }
  if (hid >= 512)
    hipLaunchKernelGGL((dq_chunk_kernel<2>), dim3(grid), dim3(256), 0, st, chunks, nchunks, occ2, dagg, ld_dagg,
                       q, hid, dpq, part);
  else
    hipLaunchKernelGGL((dq_chunk_kernel<1>), dim3(grid), dim3(256), 0, st, chunks, nchunks, occ2, dagg, ld_dagg,
                       q, hid, dpq, part);
  PS_CHECK_LAUNCH();
  hipLaunchKernelGGL(dq_combine_kernel, dim3((int)std::max<int64_t>(1, std::min<int64_t>(max_split, 512))),
                     dim3(1024), 0, st, split, nsplit, off, part, q, hid, dpq);
  PS_CHECK_LAUNCH();
  return kOk;
}

int launch_norm_lrelu_bwd(const float* y, const float* nrm, const float* dy, int n,
                          const int* nrows, int64_t max_rows, float* dp, float* z, int z_n,
                          const int* z_rows, int* zi, int64_t zi_n, hipStream_t st) {
  hipLaunchKernelGGL(norm_lrelu_bwd_kernel, dim3(grid_for(max_rows * 64, 256, 4096)), dim3(256), 0,
                     st, y, nrm, dy, n, nrows, max_rows, dp, z, z_n, z_rows, zi, zi_n);
  PS_CHECK_LAUNCH();
  return kOk;
}

int launch_loss(const float* Z, int d, const int32_t* pos_rank, int B, float margin,
                const float* feats, int64_t ld_f, int d_in, const int64_t* batch, float* G, int* Kc,
                int64_t S_max, const int* nS, float* dZ, float* part, float* colpart, float* scal,
                float* hinge, bool combine_dz, bool rep_sum, const int* rank_off, const int32_t* pos_sorted,
                float* Gp, hipStream_t st) {
  // G and Kc are zero on entry (init_workspace; then the head backward (or
  // dz_combine) and the first backward kernel leave them zero)
  PS_REQUIRE(d <= 256, kErrArg, "loss: out_dim must be <= 256");
  PS_REQUIRE(d <= 1024 && 1024 % d == 0, kErrArg, "loss: out_dim must divide 1024");
  const int nblk = ceil_div(B, 4);
  // (features past 64 FPL per lane are streamed after the row stores, one
  // waited round trip per 64 columns: C2's 1024 take 16 per lane instead)
  const int fpl = d_in <= 128 ? 2 : d_in <= 256 ? 4 : d_in <= 512 ? 8 : 16;
#define PS_LOSS(ZP, FP)                                                                           \
  hipLaunchKernelGGL((loss_triple_kernel<ZP, FP>), dim3(nblk), dim3(256), 0, st, Z, d, pos_rank, B, \
                     margin, feats, ld_f, d_in, batch, G, Kc, S_max, part, colpart, hinge, rank_off, Gp)
  if (d <= 128) {
    if (fpl == 2) PS_LOSS(2, 2);
    else if (fpl == 4) PS_LOSS(2, 4);
    else if (fpl == 8) PS_LOSS(2, 8);
    else PS_LOSS(2, 16);
  } else {
    if (fpl == 2) PS_LOSS(4, 2);
    else if (fpl == 4) PS_LOSS(4, 4);
    else if (fpl == 8) PS_LOSS(4, 8);
    else PS_LOSS(4, 16);
  }
#undef PS_LOSS
  PS_CHECK_LAUNCH();
  // rep_sum false: the consumer (the fused head backward, head.hip) sums the
  // repeated ranks' Gp rows itself, in the same order
  PS_REQUIRE(rep_sum || !combine_dz, kErrArg, "loss: dz_combine reads G: the repeated ranks need rep_sum");
  if (rep_sum && d <= 128)
    hipLaunchKernelGGL((rep_sum_kernel<2, 3>), dim3(grid_for(S_max * 64, 256)), dim3(256), 0, st, rank_off,
                       pos_sorted, nS, d, Gp, G, S_max);
  else if (rep_sum)
    hipLaunchKernelGGL((rep_sum_kernel<4, 3>), dim3(grid_for(S_max * 64, 256)), dim3(256), 0, st, rank_off,
                       pos_sorted, nS, d, Gp, G, S_max);
  PS_CHECK_LAUNCH();
  if (combine_dz) {
    hipLaunchKernelGGL(dz_combine_kernel, dim3(grid_for(S_max * d, 1024, 256)), dim3(1024), 0, st, G,
                       Kc, S_max, nS, d, dZ);
    PS_CHECK_LAUNCH();
  }
  return kOk;
}

// The on-the-fly step's virtual nodes (fly.hip): an id repeated inside a call
// computed once per occurrence, every occurrence's conv output getting the
// id's summed cotangent (index_put's backward, pinsage_model.py:257-265).  The
// loss left each call's summed rows in G at the id's rank r with Kc = the
// occurrence count (the table step's K x, all occurrences being one row);
// here the real row keeps K = 1 and virtual node j (rank of x0 + j in the top
// set) gets the same G row with K = 1.  One wave per virtual node.
__global__ void fly_fix_kernel(float* __restrict__ G, int* __restrict__ Kc, int64_t S_max, int d,
                               const unsigned long long* __restrict__ bits, const uint32_t* __restrict__ prefix,
                               const int* __restrict__ n_x, const int64_t* __restrict__ xids, int64_t x0,
                               int64_t unit) {
  const int lane = threadIdx.x & 63;
  const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
  const int64_t nx = *n_x;
  for (int64_t j = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; j < nx; j += nw) {
    const int64_t id = xids[j], xv = x0 + j;
    const int c = (int)(id / unit);
    const int64_t rr = prefix[id >> 6] + __popcll(bits[id >> 6] & ((1ull << (id & 63)) - 1ull));
    const int64_t rx = prefix[xv >> 6] + __popcll(bits[xv >> 6] & ((1ull << (xv & 63)) - 1ull));
    const float* src = G + ((int64_t)c * S_max + rr) * d;
    float* dst = G + ((int64_t)c * S_max + rx) * d;
    for (int k = lane; k < d; k += 64) dst[k] = src[k];
    if (lane == 0) {
      Kc[c * S_max + rx] = 1;
      Kc[c * S_max + rr] = 1;
    }
  }
}

int launch_fly_fix(float* G, int* Kc, int64_t S_max, int d, const unsigned long long* bits, const uint32_t* prefix,
                   const int* n_x, const int64_t* xids, int64_t x0, int64_t unit, int64_t x_cap, const int* nS,
                   float* dZ, bool combine_dz, hipStream_t st) {
  hipLaunchKernelGGL(fly_fix_kernel, dim3(grid_for(x_cap * 64, 256)), dim3(256), 0, st, G, Kc, S_max, d, bits, prefix,
                     n_x, xids, x0, unit);
  PS_CHECK_LAUNCH();
  if (combine_dz) {
    hipLaunchKernelGGL(dz_combine_kernel, dim3(grid_for(S_max * d, 1024, 256)), dim3(1024), 0, st, G, Kc, S_max, nS,
                       d, dZ);
    PS_CHECK_LAUNCH();
  }
  return kOk;
}

// The step's loss arithmetic on outputs given per position (the micro-batched
// step, pinsage_training._train_batch_micro): Z [3][B][d] (call-major), every
// position its own row (no repeated ranks, so the float atomics of det_put
// each add into a zero: exact).  G [3][3B][d]: position (c, b)'s cotangent at
// G[c][c*B + b].  scal: {loss, 0, sum |h_q|^2, variance} -- the same kernels
// and reduction order as pinsage_engine_loss, so the same bits for the same
// rows.  scratch: triplet_loss_scratch_bytes(B, d).
__global__ void triplet_identity_kernel(int32_t* __restrict__ pos_rank, int B, int* __restrict__ rank_off) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < 3 * B; i += gridDim.x * blockDim.x)
    pos_rank[i] = (i % 3) * B + i / 3;  // position 3b + c -> row c*B + b
  if (blockIdx.x == 0 && threadIdx.x == 0) rank_off[0] = -1;  // no position CSR: det_put's atomics
}

int64_t triplet_loss_scratch_bytes(int64_t B, int64_t d) {
  const int64_t nblk = (B + 3) / 4;
  return align_up(3 * B * 4, 256) + align_up(9 * B * 4, 256) + align_up((nblk + 1) * 16, 256) +
         align_up((nblk + 1) * 2 * d * 4, 256) + 256;
}

int launch_loss(const float* Z, int d, const int32_t* pos_rank, int B, float margin, const float* feats, int64_t ld_f,
                int d_in, const int64_t* batch, float* G, int* Kc, int64_t S_max, const int* nS, float* dZ, float* part,
                float* colpart, float* scal, float* hinge, bool combine_dz, bool rep_sum, const int* rank_off,
                const int32_t* pos_sorted, float* Gp, hipStream_t st);
int launch_loss_monitor(const float* part, int nparts, const float* colpart, int d, int B, float* scal,
                        hipStream_t st);

int launch_triplet_loss(const float* Z, int B, int d, float margin, float* G, void* scratch, float* scal,
                        hipStream_t st) {
  PS_REQUIRE(B > 0 && d > 0 && d <= 256 && 1024 % d == 0, kErrArg, "triplet_loss: B > 0, d <= 256 dividing 1024");
  const int64_t nblk = (B + 3) / 4;
  char* p = static_cast<char*>(scratch);
  int32_t* pos_rank = reinterpret_cast<int32_t*>(p);
  p += align_up(3LL * B * 4, 256);
  int* Kc = reinterpret_cast<int*>(p);
  p += align_up(9LL * B * 4, 256);
  float* part = reinterpret_cast<float*>(p);
  p += align_up((nblk + 1) * 16, 256);
  float* colpart = reinterpret_cast<float*>(p);
  p += align_up((nblk + 1) * 2 * d * 4, 256);
  int* rank_off = reinterpret_cast<int*>(p);
  PS_CHECK_HIP(hipMemsetAsync(G, 0, (size_t)9 * B * d * 4, st));
  PS_CHECK_HIP(hipMemsetAsync(Kc, 0, (size_t)9 * B * 4, st));
  hipLaunchKernelGGL(triplet_identity_kernel, dim3((unsigned)std::min<int64_t>((3LL * B + 255) / 256, 1024)),
                     dim3(256), 0, st, pos_rank, B, rank_off);
  PS_CHECK_LAUNCH();
  PS_TRY(launch_loss(Z, d, pos_rank, B, margin, nullptr, 0, 0, nullptr, G, Kc, 3LL * B, nullptr, nullptr, part,
                     colpart, scal, nullptr, false, false, rank_off, nullptr, nullptr, st));
  return launch_loss_monitor(part, (int)nblk, colpart, d, B, scal, st);
}

int launch_loss_monitor(const float* part, int nparts, const float* colpart, int d, int B, float* scal,
                        hipStream_t st) {
  hipLaunchKernelGGL(loss_monitor_kernel, dim3(1), dim3(1024), 0, st, part, nparts, colpart, d, B, scal);
  PS_CHECK_LAUNCH();
  return kOk;
}

int launch_adam(float* p, const float* g, float* m, float* v, int64_t n, const float* coef,
                double beta1, double beta2, float eps, hipStream_t st) {
  PS_REQUIRE(((reinterpret_cast<uintptr_t>(p) | reinterpret_cast<uintptr_t>(g) |
               reinterpret_cast<uintptr_t>(m) | reinterpret_cast<uintptr_t>(v)) & 15) == 0,
             kErrArg, "adam: buffers must be 16-byte aligned");
  hipLaunchKernelGGL(adam_kernel, dim3(grid_for((n + 3) / 4, 256, 2048)), dim3(256), 0, st, p, g, m,
                     v, n, coef, (float)beta2, (float)(1.0 - beta1), (float)(1.0 - beta2), eps);
  PS_CHECK_LAUNCH();
  return kOk;
}

}  // namespace ps
