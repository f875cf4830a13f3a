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

// order-preserving uint32 key of a float: a < b  <=>  fkey(a) < fkey(b)
__device__ __forceinline__ uint32_t fkey(float f) {
  const uint32_t b = __float_as_uint(f);
  return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}

// Block-wide top-K of the union of every thread's register list (td, ti: any order,
// FLT_MAX / -1 padding): the K smallest (distance, id) pairs, ties towards the lower id
// (ids compared unsigned, so -1 padding loses every tie), written to out_d / out_i [K] in
// ascending order.  Bisection on the composite key (fkey(distance), id) with block-wide
// counts -- ~32 rounds of K compares and one reduction each (the id round only when the
// K-th distance is tied) -- then one compaction and a rank placement by K threads.  Replaces
// a 256-leaf tree of K-long insertion networks (8 serial levels of K x K compare-swaps:
// at K = 64 it dominated the IVF-PQ scan with exact-refine candidate counts).
// lds: >= topk_select_lds(K) bytes of LDS scratch; every thread of the block must call it.
constexpr size_t topk_select_lds(int K) { return (size_t)K * 8 + 64; }

template <int K, int NT>
__device__ void block_select_topk(const float (&td)[K], const int (&ti)[K], float* __restrict__ out_d,
                                  int* __restrict__ out_i, unsigned char* lds) {
  constexpr int NW = NT / 64;
  static_assert(NT % 64 == 0 && NW <= 8 && K <= NT, "block_select_topk geometry");
  float* cd = reinterpret_cast<float*>(lds);               // [K] compacted candidates
  int* ci = reinterpret_cast<int*>(lds + K * 4);           // [K]
  int* red = reinterpret_cast<int*>(lds + K * 8);          // [NW] partial counts, [NW] fill
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  uint32_t key[K];
#pragma unroll
  for (int i = 0; i < K; ++i) key[i] = fkey(td[i]);
  auto total = [&](int c) -> int {                         // block sum (uniform result)
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
    __syncthreads();                                       // the previous round's reads of red
    if (lane == 0) red[wave] = c;
    __syncthreads();
    int t = 0;
#pragma unroll
    for (int w = 0; w < NW; ++w) t += red[w];
    return t;
  };
  // smallest T with #{key <= T} >= K
  uint32_t lo = 0, hi = 0xffffffffu;
  while (lo < hi) {
    const uint32_t mid = lo + ((hi - lo) >> 1);
    int c = 0;
#pragma unroll
    for (int i = 0; i < K; ++i) c += key[i] <= mid;
    if (total(c) >= K) hi = mid;
    else lo = mid + 1;
  }
  const uint32_t T = lo;
  int cb = 0, ce = 0;
#pragma unroll
  for (int i = 0; i < K; ++i) { cb += key[i] < T; ce += key[i] <= T; }
  const int below = total(cb);
  uint32_t U = 0xffffffffu;
  if (total(ce) > K) {                                     // tied at T: smallest id bound
    uint32_t ilo = 0, ihi = 0xffffffffu;
    while (ilo < ihi) {
      const uint32_t mid = ilo + ((ihi - ilo) >> 1);
      int c = 0;
#pragma unroll
      for (int i = 0; i < K; ++i) c += key[i] == T && (uint32_t)ti[i] <= mid;
      if (below + total(c) >= K) ihi = mid;
      else ilo = mid + 1;
    }
    U = ilo;
  }
  // compaction: the `below` entries under T first (they all fit), then the tied ones up to
  // K -- in one pass a run of FLT_MAX / -1 padding (tied at T when fewer than K entries are
  // real) could take the slots of real entries
  __syncthreads();
  if (tid == 0) red[NW] = 0;
  __syncthreads();
#pragma unroll
  for (int i = 0; i < K; ++i)
    if (key[i] < T) {
      const int p = atomicAdd(&red[NW], 1);
      cd[p] = td[i];
      ci[p] = ti[i];
    }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < K; ++i)
    if (key[i] == T && (uint32_t)ti[i] <= U) {
      const int p = atomicAdd(&red[NW], 1);                // padding duplicates may exceed K
      if (p < K) { cd[p] = td[i]; ci[p] = ti[i]; }
    }
  __syncthreads();
  if (tid < K) {
    const float v = cd[tid];
    const uint32_t kv = fkey(v), iv = (uint32_t)ci[tid];
    int r = 0;
    for (int m = 0; m < K; ++m) {
      const uint32_t km = fkey(cd[m]), im = (uint32_t)ci[m];
      r += km < kv || (km == kv && (im < iv || (im == iv && m < tid)));
    }
    out_d[r] = v;
    out_i[r] = ci[tid];
  }
  __syncthreads();
}

// Merge nblk partial lists per query: ws_d/ws_i [nq][nblk][K] -> out [nq][k_out].
// Dynamic LDS: topk_merge_lds(K) bytes.
//   qnorm_src != nullptr: add ||q||^2 (flat L2 produced ||x||^2 - 2 x.q)
//   IP: scores were negated, flip back
//   idmap != nullptr: translate candidate positions to stored 64-bit ids
template <int K, bool IP>
__global__ __launch_bounds__(256) void topk_merge_kernel(
    const float* __restrict__ ws_d, const int* __restrict__ ws_i, int nblk,
    const float* __restrict__ qnorm_src, int d, int k_out, float* __restrict__ out_d,
    int64_t* __restrict__ out_i, int64_t id_offset, const int64_t* __restrict__ idmap) {
  extern __shared__ __attribute__((aligned(16))) unsigned char topk_smem[];
  float* sd = reinterpret_cast<float*>(topk_smem);                 // [K] merged, ascending
  int* si = reinterpret_cast<int*>(topk_smem + K * 4);
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
  if (tid == 0) {
    float s = 0.f;
    if (!IP && qnorm_src)
      for (int c = 0; c < d; ++c) s += qnorm_src[(size_t)q * d + c] * qnorm_src[(size_t)q * d + c];
    qn = s;
  }
  block_select_topk<K, 256>(td, ti, sd, si, topk_smem + K * 8);
  if (tid < k_out) {
    const float v = sd[tid];
    const int id = si[tid];
    const bool valid = id >= 0 && v != FLT_MAX;
    out_d[(size_t)q * k_out + tid] = valid ? (IP ? -v : v + qn) : (IP ? -FLT_MAX : FLT_MAX);
    out_i[(size_t)q * k_out + tid] = valid ? (idmap ? idmap[id] : (int64_t)id) + id_offset : -1;
  }
}

constexpr size_t topk_merge_lds(int K) { return (size_t)K * 8 + topk_select_lds(K); }

}  // namespace docqa
