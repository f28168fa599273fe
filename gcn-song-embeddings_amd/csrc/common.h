// Shared helpers for the PinSage MI355X (gfx950) kernels and the C-ABI.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <string>

namespace ps {

// ---------------------------------------------------------------- errors
// Every C-ABI entry point returns 0 on success or a negative code; the message
// of the last failure on the calling thread is read with pinsage_last_error().
enum Status : int {
  kOk = 0,
  kErrHip = -1,        // a HIP runtime call failed
  kErrArg = -2,        // invalid argument (shape / size / pointer)
  kErrWorkspace = -3,  // workspace too small
  kErrGraph = -4,      // zero-degree node met by the walk (reference crashes there)
  kErrIndex = -5,      // index out of range (reference raises IndexError)
};

void set_error(const std::string& msg);
const char* last_error();

#define PS_CHECK_HIP(expr)                                                          \
  do {                                                                              \
    hipError_t _e = (expr);                                                         \
    if (_e != hipSuccess) {                                                         \
      ::ps::set_error(std::string(#expr) + ": " + hipGetErrorString(_e) + " @" +    \
                      __FILE__ + ":" + std::to_string(__LINE__));                   \
      return ::ps::kErrHip;                                                         \
    }                                                                               \
  } while (0)

#define PS_CHECK_LAUNCH() PS_CHECK_HIP(hipGetLastError())

#define PS_REQUIRE(cond, code, msg)  \
  do {                               \
    if (!(cond)) {                   \
      ::ps::set_error(msg);          \
      return code;                   \
    }                                \
  } while (0)

#define PS_TRY(expr)            \
  do {                          \
    int _rc = (expr);           \
    if (_rc != 0) return _rc;   \
  } while (0)

// Adam state of one parameter slice (weight [M][N] and optional bias [M]) for
// kernels that apply torch.optim.Adam as they produce the slice's gradient.
// coef = {lr / (1 - beta1^t), sqrt(1 - beta2^t)} on the device (staged per step).
struct AdamSlice {
  float* p = nullptr;   // weight rows (same row stride as the gradient)
  float* m = nullptr;
  float* v = nullptr;
  float* pb = nullptr;  // bias (nullable)
  float* mb = nullptr;
  float* vb = nullptr;
  const float* coef = nullptr;
  // betas as torch holds them (Python floats): 1 - beta is formed in double
  // and rounded once, as torch rounds its `value=1 - beta2` / lerp weight
  double beta1 = 0.9, beta2 = 0.999;
  float eps = 1e-8f;
};

// ---------------------------------------------------------------- device helpers
constexpr int kWave = 64;
constexpr float kSlope = 0.01f;  // nn.functional.leaky_relu default

__device__ __forceinline__ float lrelu(float x) { return x > 0.f ? x : x * kSlope; }
__device__ __forceinline__ float lrelu_grad(float y) { return y > 0.f ? 1.f : kSlope; }

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ int wave_sum_i(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

inline int ceil_div(int64_t a, int64_t b) { return (int)((a + b - 1) / b); }
inline int64_t align_up(int64_t a, int64_t b) { return (a + b - 1) / b * b; }

// Grid for a grid-stride loop over n items (memory-bound kernels: <= 8 blocks/CU).
inline int grid_for(int64_t n, int block, int cap = 2048) {
  int64_t g = (n + block - 1) / block;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (int)g;
}

}  // namespace ps
