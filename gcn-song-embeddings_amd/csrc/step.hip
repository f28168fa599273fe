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

#include <chrono>
#include <cstring>
#include <vector>

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

// ------------------------------------------------------------------ the host side of one step
// The per-step host work of _FusedStep in one call: wait for the ring slot's
// previous user, write the Adam coefficients, reuse or stage the step's ids
// (its frontier was computed ahead when the batch equals the predicted one),
// write the next step's predicted ids and launch the captured graphs.  The
// graphs are hipGraphExec_t handles of torch.cuda.CUDAGraph captures
// (raw_cuda_graph_exec), so a step costs one C call besides the launches.
struct Stepper {
  int64_t R = 0, slot_bytes = 0, off_ids = 0, off_next = 0, off_coef = 0, max_ids = 0, n_items = 0;
  uint8_t* ring = nullptr;  // pinned host ring [R][slot_bytes]
  hipGraphExec_t gf[2] = {nullptr, nullptr}, gm[2] = {nullptr, nullptr}, ga[2] = {nullptr, nullptr};
  std::vector<hipEvent_t> ev;
  std::vector<char> ev_live;
  std::vector<int64_t> pending[2];  // ids whose frontier sits in workspace p (empty: none)
  int parity = 0;
  int64_t nstep = 0, hits = 0;
  int64_t wait_ns = 0;    // host time blocked on ring slots (the GPU is behind)
  int64_t launch_ns = 0;  // host time inside hipGraphLaunch
  int64_t call_ns = 0;    // host time inside pinsage_stepper_step
};

}  // extern "C"
namespace {
bool ids_in_range(const int64_t* ids, int64_t n, int64_t n_items) {
  for (int64_t i = 0; i < n; ++i)
    if (ids[i] < 0 || ids[i] >= n_items) return false;
  return true;
}
}  // namespace
extern "C" {

int pinsage_stepper_create(void* ring, int64_t R, int64_t slot_bytes, int64_t off_ids, int64_t off_next,
                           int64_t off_coef, int64_t max_ids, int64_t n_items, pinsage_stepper** out) {
  if (!ring || !out || R <= 0 || max_ids <= 0 || off_ids < 0 || off_next < 0 || off_coef < 0 ||
      off_ids + max_ids * 8 > slot_bytes || off_next + max_ids * 8 > slot_bytes || off_coef + 8 > slot_bytes) {
    set_error("stepper_create: bad argument");
    return kErrArg;
  }
  auto* s = new Stepper();
  s->ring = static_cast<uint8_t*>(ring);
  s->R = R;
  s->slot_bytes = slot_bytes;
  s->off_ids = off_ids;
  s->off_next = off_next;
  s->off_coef = off_coef;
  s->max_ids = max_ids;
  s->n_items = n_items;
  s->ev.assign((size_t)R, nullptr);
  s->ev_live.assign((size_t)R, 0);
  for (auto& e : s->ev) {
    if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) {
      set_error("stepper_create: hipEventCreate failed");
      for (auto& x : s->ev)
        if (x) (void)hipEventDestroy(x);
      delete s;
      return kErrHip;
    }
  }
  *out = reinterpret_cast<pinsage_stepper*>(s);
  return kOk;
}

void pinsage_stepper_destroy(pinsage_stepper* h) {
  auto* s = reinterpret_cast<Stepper*>(h);
  if (!s) return;
  for (auto& e : s->ev)
    if (e) (void)hipEventDestroy(e);
  delete s;
}

int64_t pinsage_stepper_wait_ns(const pinsage_stepper* h) {
  const auto* s = reinterpret_cast<const Stepper*>(h);
  return s ? s->wait_ns : -1;
}

int pinsage_stepper_stats(const pinsage_stepper* h, int64_t* out, int n) {
  const auto* s = reinterpret_cast<const Stepper*>(h);
  if (!s || !out || n < 0) {
    set_error("stepper_stats: bad argument");
    return kErrArg;
  }
  const int64_t v[5] = {s->wait_ns, s->launch_ns, s->call_ns, s->nstep, s->hits};
  for (int i = 0; i < n && i < 5; ++i) out[i] = v[i];
  return kOk;
}

int pinsage_stepper_set_graphs(pinsage_stepper* h, int p, void* gf, void* gm, void* ga) {
  auto* s = reinterpret_cast<Stepper*>(h);
  if (!s || (p != 0 && p != 1) || !gf || !gm) {
    set_error("stepper_set_graphs: bad argument");
    return kErrArg;
  }
  s->gf[p] = (hipGraphExec_t)gf;
  s->gm[p] = (hipGraphExec_t)gm;
  s->ga[p] = (hipGraphExec_t)ga;
  return kOk;
}

int pinsage_stepper_sync_state(pinsage_stepper* h, int parity, int64_t nstep) {
  auto* s = reinterpret_cast<Stepper*>(h);
  if (!s || (parity != 0 && parity != 1) || nstep < 0) {
    set_error("stepper_sync_state: bad argument");
    return kErrArg;
  }
  s->parity = parity;
  s->nstep = nstep;
  s->pending[0].clear();
  s->pending[1].clear();
  return kOk;
}

int pinsage_stepper_step(pinsage_stepper* h, const int64_t* batch, int64_t n_ids, const float* coef,
                         const int64_t* next, void* stream, int64_t* info) {
  auto* s = reinterpret_cast<Stepper*>(h);
  if (!s || !batch || !coef || n_ids <= 0 || n_ids > s->max_ids) {
    set_error("stepper_step: bad argument");
    return kErrArg;
  }
  const int p = s->parity;
  if (!s->gf[p] || !s->gm[p] || (next && !s->ga[p])) {
    set_error("stepper_step: graphs not set");
    return kErrArg;
  }
  hipStream_t st = (hipStream_t)stream;
  using clk = std::chrono::steady_clock;
  auto ns_since = [](clk::time_point t) {
    return std::chrono::duration_cast<std::chrono::nanoseconds>(clk::now() - t).count();
  };
  const auto t_call = clk::now();
  const int64_t k = s->nstep % s->R;
  if (s->ev_live[(size_t)k]) {  // the slot's last user is done
    const auto t0 = clk::now();
    PS_CHECK_HIP(hipEventSynchronize(s->ev[(size_t)k]));
    s->wait_ns += ns_since(t0);
  }
  uint8_t* slot = s->ring + k * s->slot_bytes;
  std::memcpy(slot + s->off_coef, coef, 8);
  const bool hit = (int64_t)s->pending[p].size() == n_ids &&
                   std::memcmp(s->pending[p].data(), batch, (size_t)n_ids * 8) == 0;
  if (!hit) {
    if (!ids_in_range(batch, n_ids, s->n_items)) {
      set_error("stepper_step: batch ids out of range");
      return kErrIndex;
    }
    std::memcpy(slot + s->off_ids, batch, (size_t)n_ids * 8);
    const auto t0 = clk::now();
    PS_CHECK_HIP(hipGraphLaunch(s->gf[p], st));
    s->launch_ns += ns_since(t0);
  } else {
    s->hits++;
  }
  s->pending[p].clear();
  if (next && ids_in_range(next, n_ids, s->n_items)) {
    std::memcpy(slot + s->off_next, next, (size_t)n_ids * 8);
    const auto t0 = clk::now();
    PS_CHECK_HIP(hipGraphLaunch(s->ga[p], st));
    s->launch_ns += ns_since(t0);
    s->pending[1 - p].assign(next, next + n_ids);
  } else {
    const auto t0 = clk::now();
    PS_CHECK_HIP(hipGraphLaunch(s->gm[p], st));
    s->launch_ns += ns_since(t0);
    s->pending[1 - p].clear();
  }
  PS_CHECK_HIP(hipEventRecord(s->ev[(size_t)k], st));
  s->ev_live[(size_t)k] = 1;
  if (info) {
    info[0] = hit ? 1 : 0;
    info[1] = s->nstep;
  }
  s->parity ^= 1;
  s->nstep++;
  s->call_ns += ns_since(t_call);
  return kOk;
}

}  // extern "C"
