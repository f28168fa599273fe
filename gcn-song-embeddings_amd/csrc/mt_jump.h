// MT19937 jump-ahead over GF(2): advance a torch-convention MTState by n draws
// in time independent of n (≈ one Horner pass over a degree-19937 polynomial),
// with the exact end state of n sequential draws.
//
// The untempered outputs obey x[k+624] = x[k+397] ^ f(upper(x[k]), lower(x[k+1])),
// a linear map T on 624-word windows.  T^J = p(T) with p = x^J mod phi, phi the
// characteristic polynomial of the recurrence (degree 19937), so
//   window(t + J) = p(T) window(t)      (Horner: r <- T r, r ^= window(t)).
// phi is recovered once by Berlekamp-Massey from 2 * 19937 output bits;
// x^J mod phi by square-and-shift (squaring in GF(2)[x] is bit spreading), with
// polynomials for exponents rounded down to 1024 cached and the rest applied
// as a shift.  Only the first word of a jumped window has undetermined low bits,
// and it is the already-consumed output: the state is rebuilt with next = 1.
//
// Used by MTState::skip for long skips: torch.randperm(P) consumes P - 1 draws
// per batch (pinsage_training.py:58), which at 10^7 positives costs ~10 ms of
// sequential twisting; the walk's host-side chunk states (MT parity mode) too.
#pragma once
#include <cstdint>
#include <cstring>
#include <map>
#include <mutex>
#include <vector>

namespace ps {
namespace mtjump {

constexpr int kN = 624, kM = 397, kDeg = 19937;
constexpr int kWords = (kDeg + 63) / 64;  // 312 words hold degree < kDeg

using Poly = std::vector<uint64_t>;

inline bool bit(const Poly& p, int64_t i) { return (p[(size_t)(i >> 6)] >> (i & 63)) & 1u; }
inline void flip(Poly& p, int64_t i) { p[(size_t)(i >> 6)] ^= 1ull << (i & 63); }

// circular 624-word window: logical word j is w[(o + j) % kN]
struct Win {
  uint32_t w[kN];
  int o = 0;
};
inline void step(Win& r) {
  const uint32_t a = r.w[r.o], b = r.w[r.o + 1 < kN ? r.o + 1 : 0];
  const int im = r.o + kM < kN ? r.o + kM : r.o + kM - kN;
  const uint32_t y = (a & 0x80000000u) | (b & 0x7fffffffu);
  r.w[r.o] = r.w[im] ^ (y >> 1) ^ ((b & 1u) ? 0x9908b0dfu : 0u);
  r.o = r.o + 1 < kN ? r.o + 1 : 0;
}
inline void xor_in(Win& r, const uint32_t* base) {  // r ^= base (logical order)
  const int head = kN - r.o;
  for (int j = 0; j < head; ++j) r.w[r.o + j] ^= base[j];
  for (int j = head; j < kN; ++j) r.w[j - head] ^= base[j];
}

// reduce q (any length) modulo phi in place, leaving degree < kDeg
inline void reduce(Poly& q, const Poly& phi) {
  const int64_t top = (int64_t)q.size() * 64 - 1;
  for (int64_t i = top; i >= kDeg; --i) {
    if (!bit(q, i)) continue;
    // q ^= phi << (i - kDeg)
    const int64_t sh = i - kDeg, ws = sh >> 6;
    const int bs = (int)(sh & 63);
    for (int k = 0; k <= kWords; ++k) {
      const uint64_t v = phi[(size_t)k];
      if (!v) continue;
      q[(size_t)(k + ws)] ^= v << bs;
      if (bs && (size_t)(k + ws + 1) < q.size()) q[(size_t)(k + ws + 1)] ^= v >> (64 - bs);
    }
  }
  q.resize(kWords);
}
inline Poly sqr_mod(const Poly& p, const Poly& phi) {
  Poly q((size_t)2 * kWords + 2, 0);
  for (int k = 0; k < kWords; ++k) {
    uint64_t v = p[(size_t)k];
    if (!v) continue;
    uint64_t lo = 0, hi = 0;
    for (int b = 0; b < 32; ++b) {
      lo |= ((v >> b) & 1ull) << (2 * b);
      hi |= ((v >> (b + 32)) & 1ull) << (2 * b);
    }
    q[(size_t)2 * k] = lo;
    q[(size_t)2 * k + 1] = hi;
  }
  reduce(q, phi);
  return q;
}
inline Poly shift_mod(Poly p, int64_t k, const Poly& phi) {  // p * x^k mod phi
  while (k > 0) {
    const int64_t kk = k < 4096 ? k : 4096;
    const int64_t ws = kk >> 6;
    const int bs = (int)(kk & 63);
    Poly q((size_t)kWords + (size_t)ws + 2, 0);
    for (int i = 0; i < kWords; ++i) {
      q[(size_t)(i + ws)] ^= p[(size_t)i] << bs;
      if (bs) q[(size_t)(i + ws + 1)] ^= p[(size_t)i] >> (64 - bs);
    }
    reduce(q, phi);
    p.swap(q);
    k -= kk;
  }
  return p;
}

// characteristic polynomial of the recurrence (Berlekamp-Massey on bit 31 of
// the untempered outputs of an arbitrary state)
inline Poly compute_phi() {
  const int n = 2 * kDeg + 64;
  std::vector<uint8_t> s((size_t)n);
  Win r;
  uint32_t x = 5489u;
  for (int i = 0; i < kN; ++i) {
    r.w[i] = x;
    x = 1812433253u * (x ^ (x >> 30)) + (uint32_t)(i + 1);
  }
  for (int i = 0; i < kN; ++i) step(r);  // drop the seeding transient
  for (int i = 0; i < n; ++i) {
    s[(size_t)i] = (uint8_t)(r.w[r.o] >> 31);
    step(r);
  }
  const int W = (n + 63) / 64 + 2;
  // R: bit j = s[i - j] for j >= 1 (bit 0 stays 0), so each discrepancy is the
  // word-parallel parity of C & R
  Poly C((size_t)W, 0), B((size_t)W, 0), R((size_t)W, 0), Tm;
  C[0] = B[0] = 1;
  int L = 0, m = 1;
  auto xor_shift = [&](Poly& dst, const Poly& src, int sh) {  // dst ^= src << sh
    const int ws = sh >> 6, bs = sh & 63;
    for (int k = W - 1; k >= ws; --k) {
      const int a = k - ws;
      uint64_t v = src[(size_t)a] << bs;
      if (bs && a >= 1) v |= src[(size_t)(a - 1)] >> (64 - bs);
      dst[(size_t)k] ^= v;
    }
  };
  for (int i = 0; i < n; ++i) {
    if (i > 0) {
      for (int k = W - 1; k >= 1; --k) R[(size_t)k] = (R[(size_t)k] << 1) | (R[(size_t)(k - 1)] >> 63);
      R[0] = (R[0] << 1) | ((uint64_t)s[(size_t)(i - 1)] << 1);
    }
    uint64_t acc = 0;
    const int lw = L / 64 + 1;
    for (int k = 0; k < lw; ++k) acc ^= C[(size_t)k] & R[(size_t)k];
    const int d = s[(size_t)i] ^ (__builtin_popcountll(acc) & 1);
    if (!d) {
      ++m;
      continue;
    }
    if (2 * L <= i) {
      Tm = C;
      xor_shift(C, B, m);
      L = i + 1 - L;
      B = Tm;
      m = 1;
    } else {
      xor_shift(C, B, m);
      ++m;
    }
  }
  Poly phi((size_t)kWords + 1, 0);
  if (L != kDeg) return Poly();
  for (int i = 0; i <= L; ++i)  // phi(x) = x^L C(1/x)
    if (bit(C, i)) flip(phi, L - i);
  return phi;
}

struct Tables {
  Poly phi;
  std::map<int64_t, Poly> cache;  // x^E mod phi, E a multiple of 1024
  std::mutex mu;
};
inline Tables& tables() {
  static Tables t;
  static std::once_flag once;
  std::call_once(once, [] { t.phi = compute_phi(); });
  return t;
}

// x^J mod phi
inline Poly power(int64_t J) {
  Tables& T = tables();
  const int64_t E = J & ~int64_t(1023);
  Poly base;
  {
    std::lock_guard<std::mutex> lk(T.mu);
    auto it = T.cache.find(E);
    if (it != T.cache.end()) base = it->second;
  }
  if (base.empty()) {
    base.assign((size_t)kWords, 0);
    base[0] = 1;  // x^0
    for (int b = 62; b >= 0; --b) {
      base = sqr_mod(base, T.phi);
      if ((E >> b) & 1) base = shift_mod(base, 1, T.phi);
    }
    std::lock_guard<std::mutex> lk(T.mu);
    if (T.cache.size() > 64) T.cache.clear();
    T.cache[E] = base;
  }
  return shift_mod(base, J - E, T.phi);
}

// Horner evaluation of p(T) over 8-bit digits (most significant first): the
// window lives in a linear buffer (a T step appends one word; the live window
// is the last kN words), so every digit's XOR of a 624-word table entry is one
// contiguous, vectorisable loop; the buffer slides back every kSlide digits.
constexpr int kHornerBuf = kN + 8 * 64;
#if defined(__x86_64__) && !defined(__HIP_DEVICE_COMPILE__)
__attribute__((target_clones("avx2", "default")))
#endif
inline void horner(const uint64_t* p, int deg, const uint32_t* V, uint32_t* b, uint32_t* out) {
  constexpr int Q = 8, kBuf = kHornerBuf;
  for (int i = 0; i < kBuf; ++i) b[i] = 0u;
  int o = 0;  // live window: b[o .. o + kN)
  const int nd = deg / Q + 1;
  for (int d = nd - 1; d >= 0; --d) {
    if (o + kN + Q > kBuf) {
      std::memmove(b, b + o, sizeof(uint32_t) * kN);
      o = 0;
    }
    int mask = 0;
    for (int j = Q - 1; j >= 0; --j) {
      // one T step: x[o + kN] = x[o + kM] ^ f(x[o], x[o + 1]); window moves by one
      const uint32_t y = (b[o] & 0x80000000u) | (b[o + 1] & 0x7fffffffu);
      b[o + kN] = b[o + kM] ^ (y >> 1) ^ ((b[o + 1] & 1u) ? 0x9908b0dfu : 0u);
      ++o;
      const int64_t i = (int64_t)d * Q + j;
      if (i < kDeg && ((p[i >> 6] >> (i & 63)) & 1u)) mask |= 1 << j;
    }
    if (mask) {
      uint32_t* __restrict__ w = b + o;
      const uint32_t* __restrict__ v = V + (size_t)mask * kN;
      for (int i = 0; i < kN; ++i) w[i] ^= v[i];
    }
  }
  std::memcpy(out, b + o, sizeof(uint32_t) * kN);
}

// window(t + J) from window(t) (logical order, word 0 first).  Horner over
// 8-coefficient digits: r <- T^8 r ^ V[digit], V[mask] = sum of T^j window(t)
// over the set bits j of mask (256 precomputed windows), so ~2.5k window XORs
// instead of ~10k.
inline void jump_window(const uint32_t* win, int64_t J, uint32_t* out) {
  constexpr int Q = 8;
  const Poly p = power(J);
  // T^j window(t), j < Q, in logical order
  static thread_local std::vector<uint32_t> V;
  V.assign((size_t)(1 << Q) * kN, 0u);
  {
    Win w;
    std::memcpy(w.w, win, sizeof(w.w));
    w.o = 0;
    uint32_t tj[Q][kN];
    for (int j = 0; j < Q; ++j) {
      for (int i = 0; i < kN; ++i) tj[j][i] = w.w[(w.o + i) % kN];
      step(w);
    }
    for (int mask = 1; mask < (1 << Q); ++mask) {
      const int low = __builtin_ctz((unsigned)mask);
      const uint32_t* prev = &V[(size_t)(mask & (mask - 1)) * kN];
      uint32_t* dst = &V[(size_t)mask * kN];
      for (int i = 0; i < kN; ++i) dst[i] = prev[i] ^ tj[low][i];
    }
  }
  int deg = kDeg - 1;
  while (deg >= 0 && !bit(p, deg)) --deg;
  if (deg < 0) {
    std::memset(out, 0, sizeof(uint32_t) * kN);
    return;
  }
  static thread_local std::vector<uint32_t> buf;
  buf.resize((size_t)kHornerBuf);
  horner(p.data(), deg, V.data(), buf.data(), out);
}

inline bool available() { return !tables().phi.empty(); }

}  // namespace mtjump
}  // namespace ps
