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
// outv[row] (optional) its value, for the vocab-parallel pick across TP ranks
__global__ __launch_bounds__(64) void argmax_merge_kernel(const float* __restrict__ pv,
                                                          const int* __restrict__ pi, int parts,
                                                          int64_t* __restrict__ out, float* __restrict__ outv) {
  const int row = blockIdx.x;
  float bv = -FLT_MAX;
  int bi = 0x7fffffff;
  for (int s = threadIdx.x; s < parts; s += 64)
    docqa::argmax_better(bv, bi, pv[(size_t)row * parts + s], pi[(size_t)row * parts + s]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ov = __shfl_xor(bv, o, 64);
    const int oi = __shfl_xor(bi, o, 64);
    docqa::argmax_better(bv, bi, ov, oi);
  }
  if (threadIdx.x == 0) {
    out[row] = bi == 0x7fffffff ? 0 : bi;
    if (outv) outv[row] = bv;
  }
}

}  // namespace
