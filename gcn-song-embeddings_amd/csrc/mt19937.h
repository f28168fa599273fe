// Host-side MT19937 with torch's CPU-generator semantics (at::mt19937 and the
// 5056-byte torch.get_rng_state() layout).  The product uses it to reproduce
// the reference's RNG stream exactly (rng_mode "mt19937"):
//   torch.randint(n, ())  -> raw % n             (n < 2^28: one 32-bit draw)
//   torch.rand(())        -> (raw & 0xFFFFFF) * 2^-24 as float
//   torch.randperm(n)     -> Fisher-Yates, one draw per step (n-1 draws)
// (pinsage_model.py:42,45,50; pinsage_training.py:58,74).
#pragma once
#include <cstdint>
#include <cstring>
#if defined(__x86_64__) && !defined(__HIP_DEVICE_COMPILE__)
#include <immintrin.h>
#endif

#include "mt_jump.h"

namespace ps {

#if defined(__x86_64__) && !defined(__HIP_DEVICE_COMPILE__)
// The twist eight words at a time (a batch draw skips ~10^5-10^6 words through
// randperm; the host sampler's speculation must keep pace with a GPU step).
// Dependences in the recurrence are at distance 1 (read-ahead) and 227, so
// 8-wide chunks are exact; runtime-dispatched, scalar otherwise.
inline bool mt_has_avx2() {
  static const bool ok = __builtin_cpu_supports("avx2");
  return ok;
}
__attribute__((target("avx2"))) inline void mt_twist_avx2(uint32_t* s) {
  constexpr int N = 624, M = 397;
  const __m256i up = _mm256_set1_epi32((int)0x80000000u), lo = _mm256_set1_epi32(0x7fffffff);
  const __m256i one = _mm256_set1_epi32(1), mag = _mm256_set1_epi32((int)0x9908b0dfu);
  const __m256i zero = _mm256_setzero_si256();
  auto step8 = [&](int i, int src) __attribute__((target("avx2"))) {
    const __m256i u = _mm256_loadu_si256((const __m256i*)(s + i));
    const __m256i v = _mm256_loadu_si256((const __m256i*)(s + i + 1));
    const __m256i x = _mm256_loadu_si256((const __m256i*)(s + src));
    const __m256i y = _mm256_or_si256(_mm256_and_si256(u, up), _mm256_and_si256(v, lo));
    const __m256i m = _mm256_and_si256(_mm256_sub_epi32(zero, _mm256_and_si256(v, one)), mag);
    _mm256_storeu_si256((__m256i*)(s + i),
                        _mm256_xor_si256(x, _mm256_xor_si256(_mm256_srli_epi32(y, 1), m)));
  };
  auto step1 = [&](int i, int src) {
    const uint32_t y = (s[i] & 0x80000000u) | (s[i + 1] & 0x7fffffffu);
    s[i] = s[src] ^ (y >> 1) ^ ((s[i + 1] & 1u) ? 0x9908b0dfu : 0u);
  };
  int i = 0;
  for (; i + 8 <= N - M; i += 8) step8(i, i + M);
  for (; i < N - M; ++i) step1(i, i + M);
  for (; i + 8 <= N - 1; i += 8) step8(i, i + M - N);
  for (; i < N - 1; ++i) step1(i, i + M - N);
  const uint32_t y = (s[N - 1] & 0x80000000u) | (s[0] & 0x7fffffffu);
  s[N - 1] = s[M - 1] ^ (y >> 1) ^ ((s[0] & 1u) ? 0x9908b0dfu : 0u);
}
#endif

struct MTState {
  static constexpr int N = 624;
  static constexpr int M = 397;
  uint64_t seed = 5489;
  int32_t left = 1;    // draws until the next twist, torch convention (1 = twist due)
  int32_t seeded = 1;
  uint32_t next = 0;   // index of the next state word to temper
  uint32_t s[N];

  static inline uint32_t twist1(uint32_t u, uint32_t v) {
    uint32_t y = (u & 0x80000000u) | (v & 0x7fffffffu);
    return (y >> 1) ^ ((v & 1u) ? 0x9908b0dfu : 0u);
  }
  static inline uint32_t temper(uint32_t y) {
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    return y;
  }
  static void twist_words(uint32_t* s) {
    int i = 0;
    for (; i < N - M; ++i) s[i] = s[i + M] ^ twist1(s[i], s[i + 1]);
    for (; i < N - 1; ++i) s[i] = s[i + M - N] ^ twist1(s[i], s[i + 1]);
    s[N - 1] = s[M - 1] ^ twist1(s[N - 1], s[0]);
  }
  void twist() {
#if defined(__x86_64__) && !defined(__HIP_DEVICE_COMPILE__)
    if (mt_has_avx2()) {
      mt_twist_avx2(s);
    } else {
      twist_words(s);
    }
#else
    twist_words(s);
#endif
    left = N;
    next = 0;
  }
  void seed_with(uint64_t sd) {
    seed = sd;
    seeded = 1;
    s[0] = (uint32_t)(sd & 0xffffffffu);
    for (int j = 1; j < N; ++j) s[j] = 1812433253u * (s[j - 1] ^ (s[j - 1] >> 30)) + (uint32_t)j;
    left = 1;
    next = 0;
  }
  inline uint32_t draw() {
    if (--left == 0) twist();
    return temper(s[next++]);
  }
  // words available without a twist
  inline int64_t avail() const { return (int64_t)left - 1; }
  // Advance by n draws without tempering; same end state as n draw()s.  Long
  // skips jump over GF(2) (mt_jump.h); short ones twist through.
  static constexpr int64_t kJumpMin = int64_t(1) << 21;
  void skip(int64_t n) {
    if (n >= kJumpMin && mtjump::available()) {
      // the array s holds outputs x_b .. x_{b+623}, of which c are consumed;
      // jump the window to start at a skipped output x_{b+J}, J <= c + n - 1,
      // then resume at its second word (next = 1, the first is consumed).  J is
      // rounded down to a multiple of 1024 so that x^J mod phi is a cached
      // power (no per-call shift); the < 1024 draws left are twisted through.
      const int64_t c = 625 - left;
      const int64_t J = (c + n - 1) & ~int64_t(1023);
      uint32_t out[N];
      mtjump::jump_window(s, J, out);
      std::memcpy(s, out, sizeof(s));
      next = 1;
      left = N;
      n -= J + 1 - c;  // draws the jump covered
    }
    while (n > 0) {
      int64_t a = avail();
      if (a == 0) {
        twist();
        left = N + 1;  // pretend the twisting draw has not consumed yet
        a = N;
      }
      int64_t take = n < a ? n : a;
      next += (uint32_t)take;
      left -= (int32_t)take;
      n -= take;
    }
  }

  static constexpr int kTorchBytes = 5056;
  bool from_torch(const uint8_t* b, int64_t nbytes) {
    if (nbytes < 24 + 8 * N) return false;
    uint64_t nx, st;
    std::memcpy(&seed, b + 0, 8);
    std::memcpy(&left, b + 8, 4);
    std::memcpy(&seeded, b + 12, 4);
    std::memcpy(&nx, b + 16, 8);
    next = (uint32_t)nx;
    for (int i = 0; i < N; ++i) {
      std::memcpy(&st, b + 24 + 8 * i, 8);
      s[i] = (uint32_t)st;
    }
    return left > 0 && left <= N + 1 && next <= (uint32_t)N;
  }
  void to_torch(uint8_t* b) const {
    uint64_t nx = next, st;
    std::memcpy(b + 0, &seed, 8);
    std::memcpy(b + 8, &left, 4);
    std::memcpy(b + 12, &seeded, 4);
    std::memcpy(b + 16, &nx, 8);
    for (int i = 0; i < N; ++i) {
      st = s[i];
      std::memcpy(b + 24 + 8 * i, &st, 8);
    }
  }
};

// Device-side chunk descriptor: the state words plus where the next draw comes
// from.  A generator workgroup expands it into a run of raw draws.
struct MTChunk {
  uint32_t s[MTState::N];
  uint32_t next;   // next word index
  uint32_t avail;  // words usable before a twist
  uint32_t pad[2];
};

}  // namespace ps
