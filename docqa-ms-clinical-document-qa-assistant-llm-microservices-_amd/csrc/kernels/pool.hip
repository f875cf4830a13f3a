// pool.hip -- sentence-embedding pooling for the bi-encoders, fused with the
// L2 normalisation FAISS-L2 retrieval relies on (sentence-transformers MiniLM: masked
// mean pool + normalize; bge: CLS pool + normalize).  Packed varlen input [T, H] with
// cu_seqlens; output fp32 [B, H] (the dtype FAISS stores; semantic-indexer/indexer.py:41
// casts to float32).  One workgroup per sequence, 16 B per lane per token row.
#include "docqa_common.h"

using namespace docqa;

template <bool MEAN>
__global__ __launch_bounds__(128) void pool_l2_kernel(const uint16_t* __restrict__ h,
                                                      const int* __restrict__ cu, int H,
                                                      int normalize, float* __restrict__ out) {
  const int b = blockIdx.x;
  const int s0 = cu[b], s1 = cu[b + 1];
  const int c = threadIdx.x;             // chunk of 8 dims
  const bool act = c * 8 < H;
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (act) {
    if (MEAN) {
      for (int t = s0; t < s1; ++t) {
        float f[8];
        unpack8(reinterpret_cast<const uint4*>(h + (size_t)t * H)[c], f);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += f[j];
      }
      const float inv = s1 > s0 ? 1.f / (float)(s1 - s0) : 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] *= inv;
    } else if (s1 > s0) {
      unpack8(reinterpret_cast<const uint4*>(h + (size_t)s0 * H)[c], acc);
    }
  }
  float ss = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) ss += acc[j] * acc[j];
  ss = wave_sum(ss);
  __shared__ float red[2];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = ss;
  __syncthreads();
  const float tot = red[0] + red[1];
  const float inv = normalize ? 1.f / fmaxf(sqrtf(tot), 1e-12f) : 1.f;
  if (act) {
    float4* o = reinterpret_cast<float4*>(out + (size_t)b * H + c * 8);
    o[0] = make_float4(acc[0] * inv, acc[1] * inv, acc[2] * inv, acc[3] * inv);
    o[1] = make_float4(acc[4] * inv, acc[5] * inv, acc[6] * inv, acc[7] * inv);
  }
}

int docqa_pool_l2(const void* h, const int* cu, int B, int H, int mean, int normalize, float* out,
                  hipStream_t s) {
  if (B == 0) return 0;
  if (H % 8 != 0 || H > 1024) return -1;
  if (mean) pool_l2_kernel<true><<<B, 128, 0, s>>>((const uint16_t*)h, cu, H, normalize, out);
  else pool_l2_kernel<false><<<B, 128, 0, s>>>((const uint16_t*)h, cu, H, normalize, out);
  DOCQA_CHECK_LAUNCH();
  return 0;
}
