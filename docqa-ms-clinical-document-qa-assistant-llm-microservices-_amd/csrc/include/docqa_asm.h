// docqa_asm.h -- inline-asm building blocks for LDS-DMA ring pipelines on gfx950
// (cdna_hip_programming.md §5.7).  All vector-memory traffic of a ring issued through
// these helpers is invisible to hipcc's waitcnt pass, so the kernel's own counted
// `s_waitcnt vmcnt(N)` waits are the only ones: with the builtin forms hipcc drains every
// outstanding load (vmcnt(0)) at loop headers and before LDS reads, collapsing the ring
// to one stage in flight.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace docqa {

// plain s_barrier: __syncthreads() carries a release fence whose vmcnt(0) would drain
// the ring; LDS visibility of a DMA'd stage comes from the explicit vmcnt wait before it
__device__ __forceinline__ void ring_barrier() { asm volatile("s_barrier" ::: "memory"); }

__device__ __forceinline__ uint32_t lds_u32(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)p;
}

// one 16-B-per-lane LDS-DMA wave-instruction: lane i writes dst_base + 16 i (dst_base is
// a wave-uniform LDS byte address).  NT: non-temporal policy for once-read streams.
template <bool NT = true>
__device__ __forceinline__ void glds16(const void* gsrc, uint32_t dst_base) {
  unsigned keep;
  if constexpr (NT)
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(gsrc), "s"(dst_base) : "memory");
  else
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(gsrc), "s"(dst_base) : "memory");
}

// 16-B write-through (sc1) global store: the line is not left dirty in this XCD's L2, so a
// consumer in another workgroup of the launch needs no release fence from the producer
// (cdna_hip_programming.md §6 Guideline 16 R1); invisible to hipcc's waitcnt pass (drain
// with an explicit vmcnt wait); s_nop 1 so no later VALU overwrites the data registers
// before the store has read them (§5.7 item 1)
__device__ __forceinline__ void store16_wt(void* p, uint4 v) {
  typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
  const u32x4_t d = {v.x, v.y, v.z, v.w};
  asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(p), "v"(d) : "memory");
}

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" :: "i"(N) : "memory");
}

}  // namespace docqa
