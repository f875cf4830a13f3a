// docqa_common.h -- shared device helpers for the gfx950 (MI355X / CDNA4) kernels.
//
// Everything here is written for wave64 and the CDNA4 MFMA/LDS model:
//  * bf16 is moved as 16-byte vectors (8 elements per lane) -- hipcc does not
//    auto-vectorise bf16 loads (cdna_hip_programming.md Guideline 13);
//  * reductions are wave-level shuffles over 64 lanes, then LDS across waves;
//  * f32 -> bf16 uses the plain cast, which lowers to v_cvt_pk_bf16_f32 on gfx950
//    and keeps NaNs NaN (MI355X_MICROARCH.md, correctness boundaries).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace docqa {

constexpr int kWave = 64;

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef short i16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ float bf2f(uint16_t v) {
  return __uint_as_float(((uint32_t)v) << 16);
}
__device__ __forceinline__ uint16_t f2bf(float f) {
  __bf16 b = (__bf16)f;
  return *reinterpret_cast<uint16_t*>(&b);
}

// unpack 8 bf16 held in a uint4 into floats
__device__ __forceinline__ void unpack8(const uint4& v, float* f) {
  f[0] = __uint_as_float(v.x << 16); f[1] = __uint_as_float(v.x & 0xffff0000u);
  f[2] = __uint_as_float(v.y << 16); f[3] = __uint_as_float(v.y & 0xffff0000u);
  f[4] = __uint_as_float(v.z << 16); f[5] = __uint_as_float(v.z & 0xffff0000u);
  f[6] = __uint_as_float(v.w << 16); f[7] = __uint_as_float(v.w & 0xffff0000u);
}
__device__ __forceinline__ uint32_t pack2(float a, float b) {
  return (uint32_t)f2bf(a) | ((uint32_t)f2bf(b) << 16);
}
__device__ __forceinline__ uint4 pack8(const float* f) {
  uint4 v;
  v.x = pack2(f[0], f[1]); v.y = pack2(f[2], f[3]);
  v.z = pack2(f[4], f[5]); v.w = pack2(f[6], f[7]);
  return v;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
// value of the lane `N` positions up inside its 16-lane DPP row (row_ror:N), no LDS trip
template <int N>
__device__ __forceinline__ float row_ror(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x120 + N, 0xf, 0xf, false));
}

// reduction over an aligned group of `W` lanes (W power of two <= 64).  W <= 16 stays in
// the DPP row (rotations by W/2 .. 1 leave every lane with the group sum) instead of
// ds_bpermute round trips through the LDS crossbar.
template <int W>
__device__ __forceinline__ float group_sum(float v) {
  if constexpr (W == 16) {
    v += row_ror<8>(v);
    v += row_ror<4>(v);
    v += row_ror<2>(v);
    v += row_ror<1>(v);
    return v;
  } else {
#pragma unroll
    for (int o = W / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
  }
}
template <int W>
__device__ __forceinline__ float group_max(float v) {
#pragma unroll
  for (int o = W / 2; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Bijective XCD-aware remap of a linear workgroup id (cdna_hip_programming.md §5,
// "XCD swizzle must be bijective"): blocks b and b+8 share an XCD under the observed
// round-robin dispatch, so give each XCD a contiguous chunk of the logical grid.
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  const int q = nwg / 8, r = nwg % 8;
  const int xcd = orig % 8, idx = orig / 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
}

}  // namespace docqa

// 16-byte alignment of an operand a kernel reads or writes with uint4 / float4 accesses:
// host launchers refuse misaligned views (a storage offset that is not a multiple of
// 8 bf16 / 4 fp32 elements) instead of faulting on the GPU
static inline bool docqa_aligned16(const void* p) {
  return (reinterpret_cast<uintptr_t>(p) & 15u) == 0;
}

#define DOCQA_CHECK_LAUNCH() \
  do { hipError_t e__ = hipGetLastError(); if (e__ != hipSuccess) return (int)e__; } while (0)
