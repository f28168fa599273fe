// LDS-DMA helpers shared by the GEMM (gemm.hip) and the aggregation +
// projection kernel (aggw.hip): a 16-B global -> LDS copy per lane issued from
// inline asm, and counted vmcnt waits that retire a ring stage while later
// stages stay in flight.
#pragma once
#include <hip/hip_runtime.h>

namespace ps {

// One 16-B LDS-DMA per lane (global_load_lds_dwordx4; LDS destination = M0 +
// 16 * lane).  Issued from inline asm so that hipcc's waitcnt pass, which does
// not see the counted waits below and drains the whole queue (vmcnt(0)) before
// LDS reads at control-flow joins, leaves the ring alone; the kernel retires
// the DMAs itself with s_waitcnt vmcnt(N) before each stage's barrier.
__device__ __forceinline__ void glds16(const float* g, unsigned lds) {  // lds: LDS byte address
  unsigned saved;
  // M0 is reserved to the compiler: save and restore it around the DMA
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %1\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %2, off\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(saved)
      : "s"(__builtin_amdgcn_readfirstlane(lds)), "v"(g)
      : "memory");
}
// s_waitcnt vmcnt(younger * NG): retire a stage while `younger` later stages
// (NG DMAs per wave each) stay in flight (the immediate must be a constant)
template <int NG, int MAXY>
__device__ __forceinline__ void wait_stage(int younger) {
  static_assert(MAXY * NG <= 63, "vmcnt immediate");
  if constexpr (MAXY >= 4) {
    if (younger >= 4) {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(4 * NG) : "memory");
      return;
    }
  }
  if constexpr (MAXY >= 3) {
    if (younger == 3) {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * NG) : "memory");
      return;
    }
  }
  if constexpr (MAXY >= 2) {
    if (younger == 2) {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * NG) : "memory");
      return;
    }
  }
  if (younger == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NG) : "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

}  // namespace ps
