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
