// docqa_topk.h -- register top-K selection and the cross-block top-K merge shared by the
// flat kNN and IVF-PQ search kernels.  Smaller is better throughout (inner-product
// scores are negated by the producers); ties break towards the lower candidate id.
#pragma once
#include "docqa_common.h"
#include <float.h>

namespace docqa {

// insertion network over a sorted register list (static indices only: no scratch)
template <int K>
__device__ __forceinline__ void topk_insert(float (&td)[K], int (&ti)[K], float d, int id) {
#pragma unroll
  for (int i = 0; i < K; ++i) {
    const bool sw = d < td[i] || (d == td[i] && id < ti[i]);
    const float nd = sw ? td[i] : d;
    const int ni = sw ? ti[i] : id;
    td[i] = sw ? d : td[i];
    ti[i] = sw ? id : ti[i];
    d = nd;
    id = ni;
  }
}

// Merge nblk partial lists per query: ws_d/ws_i [nq][nblk][K] -> out [nq][k_out].
// Dynamic LDS: topk_merge_lds(K) bytes (128 KB at K = 64).
//   qnorm_src != nullptr: add ||q||^2 (flat L2 produced ||x||^2 - 2 x.q)
//   IP: scores were negated, flip back
//   idmap != nullptr: translate candidate positions to stored 64-bit ids
template <int K, bool IP>
__global__ __launch_bounds__(256) void topk_merge_kernel(
    const float* __restrict__ ws_d, const int* __restrict__ ws_i, int nblk,
    const float* __restrict__ qnorm_src, int d, int k_out, float* __restrict__ out_d,
    int64_t* __restrict__ out_i, int64_t id_offset, const int64_t* __restrict__ idmap) {
  extern __shared__ __attribute__((aligned(16))) unsigned char topk_smem[];
  float* sd = reinterpret_cast<float*>(topk_smem);
  int* si = reinterpret_cast<int*>(topk_smem + 256 * K * sizeof(float));
  __shared__ float qn;
  const int q = blockIdx.x, tid = threadIdx.x;
  float td[K];
  int ti[K];
#pragma unroll
  for (int i = 0; i < K; ++i) { td[i] = FLT_MAX; ti[i] = -1; }
  const size_t base = (size_t)q * nblk * K;
  for (int c = tid; c < nblk * K; c += 256) {
    const float v = ws_d[base + c];
    if (v < td[K - 1]) topk_insert<K>(td, ti, v, ws_i[base + c]);
  }
#pragma unroll
  for (int i = 0; i < K; ++i) { sd[tid * K + i] = td[i]; si[tid * K + i] = ti[i]; }
  if (tid == 0) {
    float s = 0.f;
    if (!IP && qnorm_src)
      for (int c = 0; c < d; ++c) s += qnorm_src[(size_t)q * d + c] * qnorm_src[(size_t)q * d + c];
    qn = s;
  }
  __syncthreads();
  for (int stride = 128; stride > 0; stride >>= 1) {
    if (tid < stride) {
      const int o = tid + stride;
#pragma unroll
      for (int i = 0; i < K; ++i) {
        const float v = sd[o * K + i];
        if (v < td[K - 1]) topk_insert<K>(td, ti, v, si[o * K + i]);
      }
#pragma unroll
      for (int i = 0; i < K; ++i) { sd[tid * K + i] = td[i]; si[tid * K + i] = ti[i]; }
    }
    __syncthreads();
  }
  if (tid == 0) {
    for (int i = 0; i < k_out; ++i) {
      const bool valid = ti[i] >= 0 && td[i] != FLT_MAX;
      out_d[(size_t)q * k_out + i] = valid ? (IP ? -td[i] : td[i] + qn) : (IP ? -FLT_MAX : FLT_MAX);
      out_i[(size_t)q * k_out + i] =
          valid ? (idmap ? idmap[ti[i]] : (int64_t)ti[i]) + id_offset : -1;
    }
  }
}

constexpr size_t topk_merge_lds(int K) { return (size_t)256 * K * 8; }

}  // namespace docqa
