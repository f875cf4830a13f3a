// act.hip -- element-wise activations that sit between library GEMMs:
//   * silu_mul  : SwiGLU  out[t, i] = silu(gu[t, i]) * gu[t, I + i]   (Llama MLP; the
//                 gate and up projections are one fused [H, 2I] GEMM whose output rows
//                 are [gate | up])
//   * bias_gelu : out = gelu_erf(x + bias)  (BERT FFN, when the bias is not fused into
//                 the MFMA GEMM epilogue)
//   * add_bias  : out = x + bias [+ residual]
// All are 16-byte vectorised and grid-strided (cdna_hip_programming.md Guideline 13,
// Guideline 11 grid sizing: <= 2048 blocks, grid-stride the rest).
#include "docqa_common.h"

using namespace docqa;

__device__ __forceinline__ float silu(float x) { return x / (1.f + __expf(-x)); }
__device__ __forceinline__ float gelu_erf(float x) { return 0.5f * x * (1.f + erff(x * 0.70710678118654752f)); }

// IL: gate|up rows interleaved in blocks of 8 (the layout the decode GEMM's fused SwiGLU
// epilogue reads): output chunk c = silu(chunk 2c) * chunk 2c+1 of the row.
template <bool IL>
__global__ __launch_bounds__(256) void silu_mul_kernel(const uint16_t* __restrict__ gu,
                                                       uint16_t* __restrict__ out, int T, int I) {
  // 32-bit index math (T * I / 8 < 2^31 is checked by the launcher): 64-bit integer
  // division is a ~100-instruction software sequence on CDNA.
  const int cpr = I >> 3;  // chunks per row
  const int total = T * cpr;
  for (int idx = blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += gridDim.x * blockDim.x) {
    const int t = idx / cpr;
    const int c = idx - t * cpr;
    const uint4* row = reinterpret_cast<const uint4*>(gu + t * (size_t)(2 * I));
    float g[8], u[8], o[8];
    unpack8(row[IL ? 2 * c : c], g);
    unpack8(row[IL ? 2 * c + 1 : cpr + c], u);
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = silu(g[j]) * u[j];
    reinterpret_cast<uint4*>(out + t * (size_t)I)[c] = pack8(o);
  }
}

// split-K SwiGLU consumer: P [S, T, 2I] fp32 slabs of an 8-interleaved gate|up GEMM ->
// out [T, I] = silu(bf16(sum gate)) * bf16(sum up), slabs summed in slab order (the rounding
// of the fused-epilogue GEMMs: the gate / up values as the bf16 GEMM output).  The gate|up
// projection at prefill sizes whose 256 x 256 tiles cannot fill the chip (the 70B TP-8
// shard: 56 tiles at 512 rows) is split over K into these slabs (pgemm.hip EPI_PARTIAL).
__global__ __launch_bounds__(256) void silu_mul_splitk_kernel(const float* __restrict__ P,
                                                              uint16_t* __restrict__ out, int S, int T, int I) {
  const int cpr = I >> 3;
  const int total = T * cpr;
  const size_t slab4 = (size_t)T * (size_t)(2 * I) / 4;   // one slab in float4
  for (int idx = blockIdx.x * blockDim.x + threadIdx.x; idx < total; idx += gridDim.x * blockDim.x) {
    const int t = idx / cpr;
    const int c = idx - t * cpr;
    const float4* p = reinterpret_cast<const float4*>(P + (size_t)t * (size_t)(2 * I)) + 4 * c;
    float4 v[4] = {p[0], p[1], p[2], p[3]};
    for (int sl = 1; sl < S; ++sl) {
      const float4* q = p + sl * slab4;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float4 w = q[j];
        v[j].x += w.x; v[j].y += w.y; v[j].z += w.z; v[j].w += w.w;
      }
    }
    const float g[8] = {v[0].x, v[0].y, v[0].z, v[0].w, v[1].x, v[1].y, v[1].z, v[1].w};
    const float u[8] = {v[2].x, v[2].y, v[2].z, v[2].w, v[3].x, v[3].y, v[3].z, v[3].w};
    float o[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = silu(bf2f(f2bf(g[j]))) * bf2f(f2bf(u[j]));
    reinterpret_cast<uint4*>(out + (size_t)t * I)[c] = pack8(o);
  }
}

// the same from bf16 slabs (mgemm.hip EPI_PARTIAL16: the batch-256 decode gate|up on 256-wide
// tiles split over K, X re-read half as often as the fused-SwiGLU 128-wide tiles).  NS > 0:
// S known at compile time, every slab load in flight before the first add; sum in fp32 in
// slab order.
template <int NS>
__global__ __launch_bounds__(256) void silu_mul_splitk16_kernel(const uint16_t* __restrict__ P,
                                                                uint16_t* __restrict__ out, int S, int T, int I) {
  const int cpr = I >> 3;
  const int total = T * cpr;
  const size_t slab8 = (size_t)T * (size_t)(2 * I) / 8;   // one slab in uint4
  for (int idx = blockIdx.x * blockDim.x + threadIdx.x; idx < total; idx += gridDim.x * blockDim.x) {
    const int t = idx / cpr;
    const int c = idx - t * cpr;
    const uint4* p = reinterpret_cast<const uint4*>(P + (size_t)t * (size_t)(2 * I)) + 2 * c;
    float g[8], u[8];
    if constexpr (NS > 0) {
      uint4 a[NS], b[NS];
#pragma unroll
      for (int sl = 0; sl < NS; ++sl) {
        a[sl] = p[sl * slab8];
        b[sl] = p[sl * slab8 + 1];
      }
      unpack8(a[0], g);
      unpack8(b[0], u);
#pragma unroll
      for (int sl = 1; sl < NS; ++sl) {
        float g2[8], u2[8];
        unpack8(a[sl], g2);
        unpack8(b[sl], u2);
#pragma unroll
        for (int j = 0; j < 8; ++j) { g[j] += g2[j]; u[j] += u2[j]; }
      }
    } else {
      unpack8(p[0], g);
      unpack8(p[1], u);
      for (int sl = 1; sl < S; ++sl) {
        float g2[8], u2[8];
        unpack8(p[sl * slab8], g2);
        unpack8(p[sl * slab8 + 1], u2);
#pragma unroll
        for (int j = 0; j < 8; ++j) { g[j] += g2[j]; u[j] += u2[j]; }
      }
    }
    float o[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = silu(bf2f(f2bf(g[j]))) * bf2f(f2bf(u[j]));
    reinterpret_cast<uint4*>(out + (size_t)t * I)[c] = pack8(o);
  }
}

template <bool GELU, bool RES>
__global__ __launch_bounds__(256) void bias_act_kernel(const uint16_t* __restrict__ x,
                                                       const uint16_t* __restrict__ bias,
                                                       const uint16_t* __restrict__ res,
                                                       uint16_t* __restrict__ out, int T, int N) {
  const int cpr = N >> 3;
  const int total = T * cpr;
  for (int idx = blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += gridDim.x * blockDim.x) {
    const int c = idx % cpr;
    float v[8], b[8];
    unpack8(reinterpret_cast<const uint4*>(x)[idx], v);
    unpack8(reinterpret_cast<const uint4*>(bias)[c], b);
    if constexpr (RES) {
      float r[8];
      unpack8(reinterpret_cast<const uint4*>(res)[idx], r);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] += r[j];
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = GELU ? gelu_erf(v[j] + b[j]) : v[j] + b[j];
    reinterpret_cast<uint4*>(out)[idx] = pack8(v);
  }
}

static inline int grid_for(size_t work) {
  size_t g = (work + 255) / 256;
  return (int)(g > 2048 ? 2048 : (g == 0 ? 1 : g));
}

int docqa_silu_mul(const void* gu, void* out, int T, int I, int interleaved, hipStream_t s) {
  if (I % 8 != 0 || (long long)T * (I / 8) >= (1LL << 31)) return -1;
  if (T == 0) return 0;
  if (interleaved)
    silu_mul_kernel<true><<<grid_for((size_t)T * (I / 8)), 256, 0, s>>>((const uint16_t*)gu,
                                                                       (uint16_t*)out, T, I);
  else
    silu_mul_kernel<false><<<grid_for((size_t)T * (I / 8)), 256, 0, s>>>((const uint16_t*)gu,
                                                                        (uint16_t*)out, T, I);
  DOCQA_CHECK_LAUNCH();
  return 0;
}

int docqa_silu_mul_splitk(const float* P, void* out, int S, int T, int I, hipStream_t s) {
  if (I % 8 != 0 || S < 1 || (long long)T * (I / 8) >= (1LL << 31)) return -1;
  if (T == 0) return 0;
  if (!docqa_aligned16(P) || !docqa_aligned16(out)) return -1;
  silu_mul_splitk_kernel<<<grid_for((size_t)T * (I / 8)), 256, 0, s>>>(P, (uint16_t*)out, S, T, I);
  DOCQA_CHECK_LAUNCH();
  return 0;
}

int docqa_silu_mul_splitk16(const void* P, void* out, int S, int T, int I, hipStream_t s) {
  if (I % 8 != 0 || S < 1 || (long long)T * (I / 8) >= (1LL << 31)) return -1;
  if (T == 0) return 0;
  if (!docqa_aligned16(P) || !docqa_aligned16(out)) return -1;
  const uint16_t* p = (const uint16_t*)P;
  uint16_t* o = (uint16_t*)out;
  const dim3 g = grid_for((size_t)T * (I / 8));
  switch (S) {
    case 2: silu_mul_splitk16_kernel<2><<<g, 256, 0, s>>>(p, o, S, T, I); break;
    case 4: silu_mul_splitk16_kernel<4><<<g, 256, 0, s>>>(p, o, S, T, I); break;
    default: silu_mul_splitk16_kernel<0><<<g, 256, 0, s>>>(p, o, S, T, I); break;
  }
  DOCQA_CHECK_LAUNCH();
  return 0;
}

int docqa_bias_act(const void* x, const void* bias, const void* res, void* out, int T, int N,
                   int gelu, hipStream_t s) {
  if (N % 8 != 0 || (long long)T * (N / 8) >= (1LL << 31)) return -1;
  if (T == 0) return 0;
  const int g = grid_for((size_t)T * (N / 8));
  const uint16_t *xp = (const uint16_t*)x, *bp = (const uint16_t*)bias, *rp = (const uint16_t*)res;
  uint16_t* op = (uint16_t*)out;
  if (gelu) {
    if (res) bias_act_kernel<true, true><<<g, 256, 0, s>>>(xp, bp, rp, op, T, N);
    else bias_act_kernel<true, false><<<g, 256, 0, s>>>(xp, bp, rp, op, T, N);
  } else {
    if (res) bias_act_kernel<false, true><<<g, 256, 0, s>>>(xp, bp, rp, op, T, N);
    else bias_act_kernel<false, false><<<g, 256, 0, s>>>(xp, bp, rp, op, T, N);
  }
  DOCQA_CHECK_LAUNCH();
  return 0;
}
