// docqa_norm_row.h -- one row of the decode add_rmsnorm fed by split-K slabs, shared by the
// standalone kernel (norm.hip add_rmsnorm_splitk_kernel, one 256-thread workgroup per row)
// and the persistent decode-layer chain (mgemm.hip, two rows per 512-thread item), so both
// produce the same bits.
//
// x = sum of S fp32 partial slabs P[s][row][:] (the split-K combine fused here instead of a
// separate reduce launch + bf16 round trip), rounded to bf16 before the residual add so the
// result matches projection -> bf16 -> add_rmsnorm bit for bit.
// NS > 0: S == NS at compile time -- every slab, the residual and the weight chunk are
// loaded before the first add, so the row costs one memory latency instead of S + 2
// dependent ones (at 128 decode rows this is latency-bound, not bandwidth-bound).
// tid: 0..255 within the row's thread group; red: 4 floats of LDS private to that group.
// Contains one __syncthreads() (the whole workgroup must call it the same number of times).
#pragma once
#include "docqa_common.h"
#include "docqa_asm.h"

namespace docqa {

// 16 B of fp32 slab; COH: agent-scope loads (sc1: past this XCD's L2) of slabs written by
// other workgroups of the same launch
template <bool COH>
__device__ __forceinline__ float4 slab_load4(const float* p) {
  if constexpr (COH) {
    const unsigned long long* q = reinterpret_cast<const unsigned long long*>(p);
    const unsigned long long lo = __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned long long hi = __hip_atomic_load(q + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return float4{__uint_as_float((unsigned)lo), __uint_as_float((unsigned)(lo >> 32)),
                  __uint_as_float((unsigned)hi), __uint_as_float((unsigned)(hi >> 32))};
  } else {
    return *reinterpret_cast<const float4*>(p);
  }
}

// 8 consecutive slab values at p as two float4: fp32 slabs (two 16-B loads), or bf16 slabs
// (mgemm.hip EPI_PARTIAL16: one 16-B load)
template <bool COH>
__device__ __forceinline__ void slab_load8(const float* p, float4& a, float4& b) {
  a = slab_load4<COH>(p);
  b = slab_load4<COH>(p + 4);
}
template <bool COH>
__device__ __forceinline__ void slab_load8(const uint16_t* p, float4& a, float4& b) {
  static_assert(!COH, "bf16 slabs come from an earlier launch");
  const uint4 u = *reinterpret_cast<const uint4*>(p);
  a = float4{__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u), __uint_as_float(u.y << 16),
             __uint_as_float(u.y & 0xffff0000u)};
  b = float4{__uint_as_float(u.z << 16), __uint_as_float(u.z & 0xffff0000u), __uint_as_float(u.w << 16),
             __uint_as_float(u.w & 0xffff0000u)};
}

// WT: write-through (sc1) stores of the residual and the output, for in-launch consumers
// COH: the slabs come from the same launch (slab_load4)
// PT: the slab element type (float, or uint16_t for bf16 slabs)
template <int NV, int NS, bool WT = false, bool COH = false, typename PT = float>
__device__ __forceinline__ void add_rmsnorm_splitk_row(const PT* __restrict__ P, int S, size_t slab,
                                                       uint16_t* __restrict__ residual,
                                                       const uint16_t* __restrict__ w,
                                                       uint16_t* __restrict__ out, int H, float eps,
                                                       int row, int tid, float* red) {
  const int nchunk = H >> 3;
  uint4* rr = reinterpret_cast<uint4*>(residual + (size_t)row * H);
  const uint4* wr = reinterpret_cast<const uint4*>(w);
  float v[NV][8];
  uint4 rres[NV], wres[NV];
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = tid + 256 * i;
    if (c < nchunk) {
      rres[i] = rr[c];
      wres[i] = wr[c];
    }
  }
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = tid + 256 * i;
    if (c < nchunk) {
      const PT* pr = P + (size_t)row * H + c * 8;
      float4 a, b;
      if constexpr (NS > 0) {
        float4 pa[NS], pb[NS];
#pragma unroll
        for (int sl = 0; sl < NS; ++sl) slab_load8<COH>(pr + sl * slab, pa[sl], pb[sl]);
        a = pa[0];
        b = pb[0];
#pragma unroll
        for (int sl = 1; sl < NS; ++sl) {
          a.x += pa[sl].x; a.y += pa[sl].y; a.z += pa[sl].z; a.w += pa[sl].w;
          b.x += pb[sl].x; b.y += pb[sl].y; b.z += pb[sl].z; b.w += pb[sl].w;
        }
      } else {
        slab_load8<COH>(pr, a, b);
        for (int sl = 1; sl < S; ++sl) {
          float4 a2, b2;
          slab_load8<COH>(pr + sl * slab, a2, b2);
          a.x += a2.x; a.y += a2.y; a.z += a2.z; a.w += a2.w;
          b.x += b2.x; b.y += b2.y; b.z += b2.z; b.w += b2.w;
        }
      }
      const float x8[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
      float r[8];
      unpack8(rres[i], r);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[i][j] = bf2f(f2bf(bf2f(f2bf(x8[j])) + r[j]));
      if constexpr (WT) store16_wt(rr + c, pack8(v[i]));
      else rr[c] = pack8(v[i]);
#pragma unroll
      for (int j = 0; j < 8; ++j) ss += v[i][j] * v[i][j];
    }
  }
  ss = wave_sum(ss);
  if ((tid & 63) == 0) red[tid >> 6] = ss;
  __syncthreads();
  ss = red[0] + red[1] + red[2] + red[3];
  const float inv = rsqrtf(ss / (float)H + eps);
  uint4* orow = reinterpret_cast<uint4*>(out + (size_t)row * H);
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = tid + 256 * i;
    if (c < nchunk) {
      float g[8], o[8];
      unpack8(wres[i], g);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = v[i][j] * inv * g[j];
      if constexpr (WT) store16_wt(orow + c, pack8(o));
      else orow[c] = pack8(o);
    }
  }
}

}  // namespace docqa
