// docqa_argmax.h -- greedy-pick helpers shared by the LM-head GEMMs with a fused argmax
// (dgemm.hip <= 192 rows, mgemm.hip / wgemm.hip 193..512 rows): every workgroup leaves one
// (value, id) partial per (row, weight tile); the merge kernel reduces a row's partials.
// Ties go to the lowest id (torch.argmax order); values are compared after bf16 rounding,
// so the pick is the token the unfused bf16 logits would give.
#pragma once
#include <float.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace docqa {

__device__ __forceinline__ void argmax_better(float& bv, int& bi, float v, int i) {
  if (v > bv || (v == bv && i < bi)) { bv = v; bi = i; }
}

}  // namespace docqa

namespace {

// out[row] = id of the row's best partial (an all-NaN row still yields a valid id 0);
// outv[row] (optional) its value, for the vocab-parallel pick across TP ranks.
// 256 threads, 8 partials per thread per round with every load issued before the first
// compare (the batch-1 LM head leaves 2,004 partials: 12.7 us with 64 threads walking them
// one dependent load at a time, profiles/r4_batch1_kernel_stats.txt)
__global__ __launch_bounds__(256) void argmax_merge_kernel(const float* __restrict__ pv,
                                                           const int* __restrict__ pi, int parts,
                                                           int64_t* __restrict__ out, float* __restrict__ outv) {
  __shared__ float sv[4];
  __shared__ int si[4];
  const int row = blockIdx.x, tid = threadIdx.x;
  const float* rv = pv + (size_t)row * parts;
  const int* ri = pi + (size_t)row * parts;
  float bv = -FLT_MAX;
  int bi = 0x7fffffff;
  for (int s0 = 0; s0 < parts; s0 += 256 * 8) {
    float v[8];
    int id[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int s = min(s0 + u * 256 + tid, parts - 1);
      v[u] = rv[s];
      id[u] = ri[s];
    }
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (s0 + u * 256 + tid < parts) docqa::argmax_better(bv, bi, v[u], id[u]);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ov = __shfl_xor(bv, o, 64);
    const int oi = __shfl_xor(bi, o, 64);
    docqa::argmax_better(bv, bi, ov, oi);
  }
  if ((tid & 63) == 0) {
    sv[tid >> 6] = bv;
    si[tid >> 6] = bi;
  }
  __syncthreads();
  if (tid == 0) {
#pragma unroll
    for (int w = 1; w < 4; ++w) docqa::argmax_better(bv, bi, sv[w], si[w]);
    out[row] = bi == 0x7fffffff ? 0 : bi;
    if (outv) outv[row] = bv;
  }
}

}  // namespace
