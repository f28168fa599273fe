// Cosine k-nearest neighbours over an embedding table (the evaluation path
// that consumes PinSage embeddings: baselines.py:69-77 cosine_sim_ab and
// :91-103 knn_from_emb, called by eval.py:112-143 save_knn with k = 1000).
//
//   sim(q, j) = dot(e_q, e_j) / (|e_q| |e_j| + eps)      (fp32, as torch.mm / torch.norm)
//   out[q]    = the k largest sim(q, .) over all rows j, sorted descending
//
// Per batch of query rows: one fp32 MFMA GEMM (launch_gemm: gathered query
// rows x the whole table, K = d) writes the dot products to HBM, then one
// workgroup per query row selects its top k: a threshold from the row's first
// 4096 keys (LDS radix select), ONE pass that keeps every key >= it in per-wave
// LDS segments, a radix select of the k-th key among those candidates, and an
// LDS bitonic sort of the keys >= it.  Rows where that cannot be exact (fewer
// than k candidates, a full segment) take the original path: an MSB-first
// radix select over the whole row on the order-preserving uint32 image of the
// similarity (12 + 12 + 8 bit digits, histograms in LDS), then the same sort.  Exact ties at the
// k-th key keep the lowest column indices; the final order is (sim desc,
// index asc).  The row of dot products stays in the Infinity Cache across the
// select's four passes when the batch is sized to it.
#include <algorithm>

#include "common.h"
#include "gemm.h"

namespace ps {

constexpr int kKnnBlock = 1024;
constexpr int kKnnMaxK = 4096;

__device__ __forceinline__ uint32_t f2key(float x) {
  const uint32_t u = __float_as_uint(x);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float key2f(uint32_t k) {
  return __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k);
}

__global__ void knn_row_norms_kernel(const float* __restrict__ e, int64_t n, int d, int64_t ld,
                                     float* __restrict__ norms) {
  const int lane = threadIdx.x & 63;
  const int64_t row = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (row >= n) return;
  const float* r = e + row * ld;
  // torch.norm on CPU accumulates float rows in double (acc_type<float> = double)
  double s = 0.0;
  for (int c = lane; c < d; c += 64) s += (double)r[c] * (double)r[c];
  s = wave_sum_d(s);
  if (lane == 0) norms[row] = (float)sqrt(s);
}

__global__ void knn_ids_kernel(const int64_t* __restrict__ q, int64_t nq, int64_t n,
                               int32_t* __restrict__ q32, float* __restrict__ qn,
                               const float* __restrict__ norms, int* __restrict__ err) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nq) return;
  int64_t v = q[i];
  if (v < 0 || v >= n) {  // callers validate; clamp so that no access strays
    if (err) atomicExch(err, 1);
    v = 0;
  }
  q32[i] = (int32_t)v;
  qn[i] = norms[v];
}

// one workgroup per query row b: dots[b][0..n) -> top k of sim, sorted
constexpr int kKnnSample = 4096;  // leading keys of a row that set the candidate threshold
constexpr int kKnnSeg = 512;      // candidate slots per wave (16 waves: 8192 per row)

// In-LDS bitonic sort of P (a power of two) (key, index) pairs into the final
// order: key descending, then index ascending.  All threads of the block call it.
__device__ void knn_bitonic(uint32_t* key, int32_t* idx, int P) {
  for (int kk = 2; kk <= P; kk <<= 1) {
    for (int jj = kk >> 1; jj > 0; jj >>= 1) {
      for (int i = threadIdx.x; i < P; i += kKnnBlock) {
        const int l = i ^ jj;
        if (l > i) {
          const uint32_t ka = key[i], kb = key[l];
          const int32_t ia = idx[i], ib = idx[l];
          const bool a_first = ka > kb || (ka == kb && ia < ib);
          const bool up = (i & kk) == 0;
          if (up ? !a_first : a_first) {
            key[i] = kb;
            key[l] = ka;
            idx[i] = ib;
            idx[l] = ia;
          }
        }
      }
      __syncthreads();
    }
  }
}

// The rank-th largest of keys held in LDS (12 + 12 + 8 bit MSB-first radix
// select; `get(i)` reads key i of `cnt`): returns it, and in *need_eq how
// many keys equal to it are within the top `rank`.  All threads call it.
template <class Get>
__device__ uint32_t knn_lds_kth(Get get, int cnt, uint32_t rank, uint32_t* hist, uint32_t* sh,
                                uint32_t* need_eq) {
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  uint32_t prefix = 0, need = rank;
  const int shifts[3] = {20, 8, 0};
  const int widths[3] = {12, 12, 8};
#pragma unroll 1
  for (int p = 0; p < 3; ++p) {
    const int sh_ = shifts[p], nb = 1 << widths[p], hs = sh_ + widths[p];
    for (int i = tid; i < nb; i += kKnnBlock) hist[i] = 0;
    __syncthreads();
    for (int i = tid; i < cnt; i += kKnnBlock) {
      const uint32_t key = get(i);
      if (hs >= 32 || (key >> hs) == prefix) atomicAdd(&hist[(key >> sh_) & (nb - 1)], 1u);
    }
    __syncthreads();
    if (wv == 0) {
      const int per = nb / 64;
      uint32_t s = 0;
      for (int i = 0; i < per; ++i) s += hist[nb - 1 - (lane * per + i)];
      uint32_t inc = s;
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(inc, o, 64);
        if (lane >= o) inc += y;
      }
      const uint32_t before = inc - s;
      if (before < need && need <= inc) {
        uint32_t c = before;
        for (int i = 0; i < per; ++i) {
          const int bin = nb - 1 - (lane * per + i);
          const uint32_t h = hist[bin];
          if (c + h >= need) {
            sh[0] = (prefix << widths[p]) | (uint32_t)bin;
            sh[1] = need - c;
            break;
          }
          c += h;
        }
      }
    }
    __syncthreads();
    prefix = sh[0];
    need = sh[1];
    __syncthreads();
  }
  *need_eq = need;
  return prefix;
}

__global__ __launch_bounds__(kKnnBlock) void knn_select_kernel(
    const float* __restrict__ dots, int64_t n, const float* __restrict__ norms,
    const float* __restrict__ qn, float eps, int k, int P, float* __restrict__ out_w,
    int64_t* __restrict__ out_n) {
  __shared__ uint32_t hist[4096];
  __shared__ uint32_t skey[kKnnMaxK];
  __shared__ int32_t sidx[kKnnMaxK];
  __shared__ uint32_t sh_prefix, sh_need;
  __shared__ int sh_gt, sh_eq;
  __shared__ int wave_cnt[kKnnBlock / 64];

  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int64_t b = blockIdx.x;
  const float* row = dots + b * n;
  const float na = qn[b];
  auto key_of = [&](float dot, float nj) __attribute__((always_inline)) {
    // (|a| |b| + eps) rounded like torch's rank-1 mm then add: no contraction
    return f2key(dot / __fadd_rn(__fmul_rn(na, nj), eps));
  };
  auto key_at = [&](int64_t j) __attribute__((always_inline)) { return key_of(row[j], norms[j]); };
  // rows of n % 4 == 0 floats start 16-byte aligned (the dot rows are n apart)
  const bool vec = (n % 4) == 0;

  // ---- one pass.  A threshold t = a key of the row's leading kKnnSample keys
  // whose rank there lies (with wide slack) below k's expected rank; one pass
  // keeps every key >= t in per-wave LDS segments (no shared counter).  If at
  // least k keys reach t, the k-th largest key does too, so the candidates hold
  // the whole top k and its ties: a radix select over them gives the k-th key,
  // and sorting the keys >= it gives the exact result.  Otherwise (too few,
  // a full segment, or more than kKnnMaxK keys >= the k-th) the 4-pass radix
  // select below runs.
  __shared__ uint32_t ckey[16 * kKnnSeg];
  __shared__ int32_t cidx[16 * kKnnSeg];
  __shared__ int seg_cnt[kKnnBlock / 64];
  __shared__ uint32_t sh2[2];
  {
    const int S = (int)min<int64_t>(n, kKnnSample);
    for (int i = tid; i < S; i += kKnnBlock) skey[i] = key_at(i);
    __syncthreads();
    const double er = (double)k * S / (double)n;
    const uint32_t r = S == n ? (uint32_t)k : (uint32_t)min<double>(S, er * 1.5 + 4.0 * sqrt(er) + 8.0);
    uint32_t dummy;
    const uint32_t t = knn_lds_kth([&](int i) { return skey[i]; }, S, r, hist, sh2, &dummy);
    int cw = 0;  // this wave's candidates (wave-uniform)
    bool over = false;
    uint32_t* const wk = ckey + wv * kKnnSeg;
    int32_t* const wi = cidx + wv * kKnnSeg;
    auto take = [&](uint32_t key, int64_t j, bool valid) __attribute__((always_inline)) {
      const bool c = valid && key >= t;
      const unsigned long long m = __ballot(c);
      if (c) {
        const int slot = cw + __popcll(m & ((1ull << lane) - 1ull));
        if (slot < kKnnSeg) {
          wk[slot] = key;
          wi[slot] = (int32_t)j;
        }
      }
      cw += __popcll(m);
    };
    // block-uniform trip counts: take() uses wave-wide ballots
    const int64_t n16 = vec ? (n / 16) * 16 : 0;
    for (int64_t base = 0; base < n16; base += (int64_t)kKnnBlock * 16) {
      const int64_t j0 = base + (int64_t)tid * 16;
      const bool ok = j0 < n16;
      const int64_t jl = ok ? j0 : 0;
      float4 dv[4], nv[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        dv[u] = *reinterpret_cast<const float4*>(row + jl + 4 * u);
        nv[u] = *reinterpret_cast<const float4*>(norms + jl + 4 * u);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        take(key_of(dv[u].x, nv[u].x), j0 + 4 * u, ok);
        take(key_of(dv[u].y, nv[u].y), j0 + 4 * u + 1, ok);
        take(key_of(dv[u].z, nv[u].z), j0 + 4 * u + 2, ok);
        take(key_of(dv[u].w, nv[u].w), j0 + 4 * u + 3, ok);
      }
    }
    for (int64_t j0 = n16; j0 < n; j0 += kKnnBlock) {
      const int64_t j = j0 + tid;
      take(j < n ? key_at(j) : 0u, j, j < n);
    }
    over = cw > kKnnSeg;
    if (lane == 0) seg_cnt[wv] = over ? -1 : cw;
    __syncthreads();
    int tot = 0;
    bool bad = false;
    for (int w = 0; w < kKnnBlock / 64; ++w) {
      bad |= seg_cnt[w] < 0;
      tot += seg_cnt[w] < 0 ? 0 : seg_cnt[w];
    }
    if (!bad && tot >= k) {
      // candidate i (0 <= i < 16 * kKnnSeg) lives in segment i / kKnnSeg
      auto cand = [&](int i) -> uint32_t {
        const int w = i / kKnnSeg, o = i - w * kKnnSeg;
        return o < seg_cnt[w] ? ckey[i] : 0u;  // key 0 sorts below every real key
      };
      uint32_t need_eq;
      const uint32_t thr = knn_lds_kth(cand, 16 * kKnnSeg, (uint32_t)k, hist, sh2, &need_eq);
      // keys >= thr: the n_gt keys above it plus every tie
      if (tid == 0) sh_gt = 0;
      __syncthreads();
      for (int i0 = 0; i0 < 16 * kKnnSeg; i0 += kKnnBlock) {  // block-uniform: ballots below
        const int i = i0 + tid, w = i / kKnnSeg, o = i - w * kKnnSeg;
        const bool c = o < seg_cnt[w] && ckey[i] >= thr;
        const unsigned long long mm = __ballot(c);
        int base = 0;
        if (lane == 0 && mm) base = atomicAdd(&sh_gt, __popcll(mm));
        base = __shfl(base, 0, 64);
        const int sl = base + __popcll(mm & ((1ull << lane) - 1ull));
        if (c && sl < kKnnMaxK) {
          skey[sl] = ckey[i];
          sidx[sl] = cidx[i];
        }
      }
      __syncthreads();
      const int m = sh_gt;
      if (m <= kKnnMaxK) {
        int PC = 64;
        while (PC < m) PC <<= 1;
        for (int i = m + tid; i < PC; i += kKnnBlock) {
          skey[i] = 0u;
          sidx[i] = 0x7fffffff;
        }
        __syncthreads();
        knn_bitonic(skey, sidx, PC);
        for (int i = tid; i < k; i += kKnnBlock) {
          out_w[b * k + i] = key2f(skey[i]);
          out_n[b * k + i] = sidx[i];
        }
        return;  // block-uniform (m is a shared value read after a barrier)
      }
    }
    __syncthreads();
  }

  // ---- radix select of the k-th largest key: digits of 12, 12 and 8 bits
  uint32_t prefix = 0, need = (uint32_t)k;
  const int shifts[3] = {20, 8, 0};
  const int widths[3] = {12, 12, 8};
#pragma unroll 1
  for (int p = 0; p < 3; ++p) {
    const int sh = shifts[p], nb = 1 << widths[p];
    for (int i = tid; i < nb; i += kKnnBlock) hist[i] = 0;
    __syncthreads();
    const int hs = sh + widths[p];  // bits above this digit must equal the prefix
    auto count = [&](uint32_t key) __attribute__((always_inline)) {
      if (hs >= 32 || (key >> hs) == prefix) atomicAdd(&hist[(key >> sh) & (nb - 1)], 1u);
    };
    // 4 x 16-byte loads of dots and norms in flight per thread (the row is
    // streamed four times: memory-level parallelism, not LDS, bounds a pass)
    const int64_t n16 = vec ? (n / 16) * 16 : 0;
    for (int64_t j0 = (int64_t)tid * 16; j0 < n16; j0 += (int64_t)kKnnBlock * 16) {
      float4 dv[4], nv[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        dv[u] = *reinterpret_cast<const float4*>(row + j0 + 4 * u);
        nv[u] = *reinterpret_cast<const float4*>(norms + j0 + 4 * u);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        count(key_of(dv[u].x, nv[u].x));
        count(key_of(dv[u].y, nv[u].y));
        count(key_of(dv[u].z, nv[u].z));
        count(key_of(dv[u].w, nv[u].w));
      }
    }
    for (int64_t j = n16 + tid; j < n; j += kKnnBlock) count(key_at(j));
    __syncthreads();
    if (wv == 0) {  // scan bins from the top: the bin holding the need-th largest
      const int per = nb / 64;
      uint32_t s = 0;
      for (int i = 0; i < per; ++i) s += hist[nb - 1 - (lane * per + i)];
      // exclusive prefix over lanes (lane 0 = highest bins)
      uint32_t inc = s;
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(inc, o, 64);
        if (lane >= o) inc += y;
      }
      const uint32_t before = inc - s;
      if (before < need && need <= inc) {  // exactly one lane
        uint32_t c = before;
        for (int i = 0; i < per; ++i) {
          const int bin = nb - 1 - (lane * per + i);
          const uint32_t h = hist[bin];
          if (c + h >= need) {
            sh_prefix = (prefix << widths[p]) | (uint32_t)bin;
            sh_need = need - c;
            break;
          }
          c += h;
        }
      }
    }
    __syncthreads();
    prefix = sh_prefix;
    need = sh_need;
    __syncthreads();
  }
  const uint32_t thr = prefix;        // the k-th largest key
  const int need_eq = (int)need;      // how many keys == thr belong to the top k
  const int n_gt = k - need_eq;

  // ---- collect: keys > thr (any order) and the lowest-index need_eq keys == thr
  if (tid == 0) {
    sh_gt = 0;
    sh_eq = 0;
  }
  __syncthreads();
  for (int64_t j0 = 0; j0 < n; j0 += kKnnBlock) {
    const int64_t j = j0 + tid;
    uint32_t key = 0;
    bool gt = false, eq = false;
    if (j < n) {
      key = key_at(j);
      gt = key > thr;
      eq = key == thr;
    }
    if (gt) {
      const int s = atomicAdd(&sh_gt, 1);
      skey[s] = key;
      sidx[s] = (int32_t)j;
    }
    // ordered compaction of the ties (index order within and across chunks)
    const unsigned long long m = __ballot(eq);
    if (lane == 0) wave_cnt[wv] = __popcll(m);
    __syncthreads();
    const int taken = sh_eq;
    if (eq) {
      int r = taken + __popcll(m & ((1ull << lane) - 1ull));
      for (int w = 0; w < wv; ++w) r += wave_cnt[w];
      if (r < need_eq) {
        skey[n_gt + r] = key;
        sidx[n_gt + r] = (int32_t)j;
      }
    }
    __syncthreads();
    if (tid == 0) {
      int t = 0;
      for (int w = 0; w < kKnnBlock / 64; ++w) t += wave_cnt[w];
      sh_eq = taken + t;
    }
    __syncthreads();
    if (sh_eq >= need_eq && sh_gt >= n_gt) break;  // uniform: shared values after a barrier
  }
  // ---- sort (key desc, index asc); pad to P with keys that sort last
  for (int i = k + tid; i < P; i += kKnnBlock) {
    skey[i] = 0u;
    sidx[i] = 0x7fffffff;
  }
  __syncthreads();
  knn_bitonic(skey, sidx, P);
  for (int i = tid; i < k; i += kKnnBlock) {
    out_w[b * k + i] = key2f(skey[i]);
    out_n[b * k + i] = sidx[i];
  }
}

int64_t knn_scratch_bytes(int64_t n, int64_t qb) {
  return align_up(n * 4, 256) + align_up(qb * 4, 256) * 2 + align_up(qb * n * 4, 256) + 256;
}

int launch_knn_cosine(const float* emb, int64_t n, int64_t d, int64_t ld, const int64_t* queries,
                      int64_t nq, int64_t k, float eps, void* scratch, int64_t scratch_bytes,
                      float* out_w, int64_t* out_n, int* err, hipStream_t st) {
  PS_REQUIRE(n > 0 && d > 0 && ld >= d && nq >= 0, kErrArg, "knn: bad sizes");
  PS_REQUIRE(d % 4 == 0, kErrArg, "knn: d must be a multiple of 4");
  PS_REQUIRE(n <= INT32_MAX && d <= INT32_MAX, kErrArg, "knn: table too large");
  PS_REQUIRE(k >= 1 && k <= n && k <= kKnnMaxK, kErrArg, "knn: need 1 <= k <= min(n, 4096)");
  if (nq == 0) return kOk;
  // batch of query rows that fits the scratch
  int64_t qb = std::min<int64_t>(nq, 65535);
  qb = std::min<int64_t>(qb, std::max<int64_t>(1, (scratch_bytes - align_up(n * 4, 256) - 1024) /
                                                     (n * 4 + 8)));
  while (qb > 1 && knn_scratch_bytes(n, qb) > scratch_bytes) --qb;
  PS_REQUIRE(knn_scratch_bytes(n, qb) <= scratch_bytes, kErrWorkspace, "knn: scratch too small");
  char* s = (char*)scratch;
  float* norms = (float*)s;
  s += align_up(n * 4, 256);
  int32_t* q32 = (int32_t*)s;
  s += align_up(qb * 4, 256);
  float* qn = (float*)s;
  s += align_up(qb * 4, 256);
  float* dots = (float*)s;

  hipLaunchKernelGGL(knn_row_norms_kernel, dim3((unsigned)ceil_div(n * 64, 256)), dim3(256), 0, st,
                     emb, n, (int)d, ld, norms);
  PS_CHECK_LAUNCH();
  int P = 64;
  while (P < k) P <<= 1;
  for (int64_t q0 = 0; q0 < nq; q0 += qb) {
    const int64_t m = std::min(qb, nq - q0);
    hipLaunchKernelGGL(knn_ids_kernel, dim3((unsigned)ceil_div(m, 256)), dim3(256), 0, st,
                       queries + q0, m, n, q32, qn, norms, err);
    PS_CHECK_LAUNCH();
    GemmParams p;
    p.M = (int)m;
    p.N = (int)n;
    p.K = (int)d;
    p.a = emb;
    p.lda = ld;
    p.a_idx = q32;
    p.b = emb;
    p.ldb = ld;
    p.c = dots;
    p.ldc = n;
    PS_TRY(launch_gemm(p, st));
    hipLaunchKernelGGL(knn_select_kernel, dim3((unsigned)m), dim3(kKnnBlock), 0, st, dots, n, norms,
                       qn, eps, (int)k, P, out_w + q0 * k, out_n + q0 * k);
    PS_CHECK_LAUNCH();
  }
  return kOk;
}

}  // namespace ps
