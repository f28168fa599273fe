// Per-step host <-> device hand-off of the captured train step
// (pinsage_training._FusedStep), without copy operations between graph
// launches.  The host writes step i's ids and Adam coefficients into slot
// i % R of a pinned ring; the step graph's first kernel reads the slot chosen
// by a device-side step counter (system-scope loads: the ring is host memory)
// and its last kernel publishes the loss scalars into slot i % R2 of a device
// ring and advances the counter.  The host mirrors the counter, so each
// step's returned scalars are views of their own ring entry (valid for R2
// steps), and a step is exactly one graph launch on the stream.
#include "../../include/pinsage_hip.h"
#include "common.h"

namespace ps {

__global__ void step_stage_kernel(const uint64_t* __restrict__ ring, int64_t slot_words, int64_t R,
                                  const int64_t* __restrict__ ctr, int64_t src_word, int64_t n_words,
                                  uint64_t* __restrict__ dst, int64_t coef_word,
                                  uint64_t* __restrict__ coef_dst) {
  const uint64_t* slot = ring + (*ctr % R) * slot_words;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_words;
       i += (int64_t)gridDim.x * blockDim.x)
    dst[i] = __hip_atomic_load(slot + src_word + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  if (coef_dst && blockIdx.x == 0 && threadIdx.x == 0)
    *coef_dst = __hip_atomic_load(slot + coef_word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// one wave: ring_out[ctr % R2][0..n) = scal[0..n), then ctr += 1
__global__ void step_publish_kernel(const float* __restrict__ scal, int n, float* __restrict__ ring_out,
                                    int64_t R2, int64_t* __restrict__ ctr) {
  const int64_t k = *ctr % R2;
  if ((int)threadIdx.x < n) ring_out[k * n + threadIdx.x] = scal[threadIdx.x];
  __syncthreads();
  if (threadIdx.x == 0) *ctr += 1;
}

// one wave that holds the stream for `ticks` of the 100 MHz constant clock
// (measurement only: the launches queued behind it then run back to back, so
// events around them time the GPU work and not the host's enqueue gaps)
__global__ void stream_hold_kernel(uint64_t ticks) {
  const uint64_t t0 = wall_clock64();
  while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
}

}  // namespace ps

using namespace ps;

extern "C" {

int pinsage_step_stage(const void* ring, int64_t slot_bytes, int64_t R, const int64_t* ctr,
                       int64_t src_off, int64_t nbytes, void* dst, int64_t coef_off, void* coef_dst,
                       void* stream) {
  if (!ring || !ctr || R <= 0 || slot_bytes <= 0 || slot_bytes % 8 || src_off % 8 || nbytes % 8 ||
      coef_off % 8 || nbytes < 0 || src_off + nbytes > slot_bytes ||
      (coef_dst && coef_off + 8 > slot_bytes) || (nbytes > 0 && !dst)) {
    set_error("step_stage: bad argument");
    return kErrArg;
  }
  const int64_t words = nbytes / 8;
  hipLaunchKernelGGL(step_stage_kernel, dim3((unsigned)std::max(1, std::min(64, ceil_div(words, 256)))),
                     dim3(256), 0, (hipStream_t)stream, (const uint64_t*)ring, slot_bytes / 8, R, ctr,
                     src_off / 8, words, (uint64_t*)dst, coef_off / 8, (uint64_t*)coef_dst);
  PS_CHECK_LAUNCH();
  return kOk;
}

int pinsage_step_publish(const float* scal, int64_t n, float* ring_out, int64_t R2, int64_t* ctr,
                         void* stream) {
  if (!scal || !ring_out || !ctr || n <= 0 || n > 64 || R2 <= 0) {
    set_error("step_publish: bad argument");
    return kErrArg;
  }
  hipLaunchKernelGGL(step_publish_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, scal, (int)n,
                     ring_out, R2, ctr);
  PS_CHECK_LAUNCH();
  return kOk;
}

int pinsage_stream_hold(int64_t us, void* stream) {
  if (us < 0 || us > 1000000) {
    set_error("stream_hold: us must be in [0, 1e6]");
    return kErrArg;
  }
  hipLaunchKernelGGL(stream_hold_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, (uint64_t)us * 100u);
  PS_CHECK_LAUNCH();
  return kOk;
}

}  // extern "C"
