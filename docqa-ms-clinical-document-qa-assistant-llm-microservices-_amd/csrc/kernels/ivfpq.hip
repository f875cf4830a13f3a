// ivfpq.hip -- IVF-PQ asymmetric-distance (ADC) search for the 10M-vector
// semantic-indexer configuration (bge-base 768-d, nlist coarse cells, M x 8-bit PQ on
// the residuals), FAISS IndexIVFPQ semantics (by_residual, squared L2).
//
// Work item = (query, probed list), one 256-thread workgroup each:
//   1. residual query r = q - c_list into LDS;
//   2. distance look-up table LUT[m][k] = || r_m - pq[m][k] ||^2, M x 256 fp32 in LDS
//      (the PQ codebook, M*256*dsub floats, is L2-resident and shared by every item);
//   3. stream the list's codes (M bytes per vector, 16-byte loads) from HBM: each lane
//      sums M LDS look-ups per vector and keeps a register top-K (insertion network,
//      skipped wave-wide when no lane improves);
//   4. 256 per-lane lists merge through LDS -> top-K of the item -> workspace.
// A second launch (docqa_topk.h) merges the nprobe lists of each query and maps code
// positions to the stored 64-bit ids.
//
// The coarse step (q vs nlist centroids, top-nprobe) is the flat MFMA kNN kernel.
// Reference parity: the reference only has IndexFlatL2 (semantic-indexer/indexer.py:39);
// IVF-PQ is the BASELINE.json config-2 scale-out of the same search API.
#include "docqa_common.h"
#include "docqa_topk.h"
#include <float.h>
#include <algorithm>

using namespace docqa;

namespace {

template <int K, bool VEC16>
__global__ __launch_bounds__(256) void ivfpq_scan_kernel(
    const float* __restrict__ xq, const float* __restrict__ centroids,
    const float* __restrict__ pq, const uint8_t* __restrict__ codes,
    const int64_t* __restrict__ list_off, const int64_t* __restrict__ probes, int nprobe, int d,
    int M, int dsub, float* __restrict__ ws_d, int* __restrict__ ws_i) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* lut = smem;                 // [M][256]
  float* qr = smem + M * 256;        // [d]
  const int item = blockIdx.x;
  const int q = item / nprobe;
  const int tid = threadIdx.x;
  const int64_t list = probes[item];
  const size_t ob = (size_t)item * K;
  if (list < 0) {
    if (tid < K) { ws_d[ob + tid] = FLT_MAX; ws_i[ob + tid] = -1; }
    return;
  }
  for (int c = tid; c < d; c += 256) qr[c] = xq[(size_t)q * d + c] - centroids[(size_t)list * d + c];
  __syncthreads();
  for (int idx = tid; idx < M * 256; idx += 256) {
    const int m = idx >> 8;
    const float* cen = pq + (size_t)idx * dsub;
    const float* r = qr + m * dsub;
    float s = 0.f;
    for (int j = 0; j < dsub; ++j) {
      const float t = r[j] - cen[j];
      s += t * t;
    }
    lut[idx] = s;
  }
  __syncthreads();

  float td[K];
  int ti[K];
#pragma unroll
  for (int i = 0; i < K; ++i) { td[i] = FLT_MAX; ti[i] = -1; }
  const int64_t lo = list_off[list], hi = list_off[list + 1];
  for (int64_t base = lo; base < hi; base += 256) {
    const int64_t i = base + tid;
    float dist = FLT_MAX;
    if (i < hi) {
      const uint8_t* row = codes + i * M;
      float s = 0.f;
      if constexpr (VEC16) {
        for (int m0 = 0; m0 < M; m0 += 16) {
          const uint4 w = *reinterpret_cast<const uint4*>(row + m0);
          const uint32_t ws[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
          for (int e = 0; e < 4; ++e)
#pragma unroll
            for (int b = 0; b < 4; ++b)
              s += lut[(m0 + e * 4 + b) * 256 + ((ws[e] >> (8 * b)) & 0xff)];
        }
      } else {
        for (int m0 = 0; m0 < M; m0 += 4) {
          const uint32_t w = *reinterpret_cast<const uint32_t*>(row + m0);
#pragma unroll
          for (int b = 0; b < 4; ++b) s += lut[(m0 + b) * 256 + ((w >> (8 * b)) & 0xff)];
        }
      }
      dist = s;
    }
    if (__any(dist < td[K - 1])) {
      if (dist < td[K - 1]) topk_insert<K>(td, ti, dist, (int)i);
    }
  }
  // block top-K of the 256 lane lists (threshold select; LUT region reused)
  __syncthreads();
  float* sd = smem;
  int* si = reinterpret_cast<int*>(smem + K);
  block_select_topk<K, 256>(td, ti, sd, si, reinterpret_cast<unsigned char*>(smem + 2 * K));
  if (tid < K) { ws_d[ob + tid] = sd[tid]; ws_i[ob + tid] = si[tid]; }
}

// PQ encoding of residuals: codes[i][m] = argmin_k || (x_i - c_assign(i))_m - pq[m][k] ||^2.
// One wave per (vector, sub-quantizer) group of 64 candidate centroids x 4 passes.
__global__ __launch_bounds__(256) void pq_encode_kernel(const float* __restrict__ x,
                                                        const float* __restrict__ centroids,
                                                        const int64_t* __restrict__ assign,
                                                        const float* __restrict__ pq, int n, int d,
                                                        int M, int dsub, uint8_t* __restrict__ codes) {
  const int lane = threadIdx.x & 63;
  const long long total = (long long)n * M;
  const long long nwaves = (long long)gridDim.x * 4;
  // grid-stride over (vector, sub-quantizer) pairs: a 10M x 64 encode is 640M wave-tasks,
  // past HIP's 2^32 work-item launch limit if launched flat
  for (long long wave = (long long)blockIdx.x * 4 + (threadIdx.x >> 6); wave < total; wave += nwaves) {
  const int i = (int)(wave / M), m = (int)(wave % M);
  const float* xr = x + (size_t)i * d + m * dsub;
  const float* cr = centroids + (size_t)assign[i] * d + m * dsub;
  float best = FLT_MAX;
  int bi = 0;
  for (int k = lane; k < 256; k += 64) {
    const float* cen = pq + ((size_t)m * 256 + k) * dsub;
    float s = 0.f;
    for (int j = 0; j < dsub; ++j) {
      const float t = xr[j] - cr[j] - cen[j];
      s += t * t;
    }
    if (s < best) { best = s; bi = k; }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ob = __shfl_xor(best, o, 64);
    const int oi = __shfl_xor(bi, o, 64);
    if (ob < best || (ob == best && oi < bi)) { best = ob; bi = oi; }
  }
  if (lane == 0) codes[(size_t)i * M + m] = (uint8_t)bi;
  }
}

}  // namespace

template <int K>
static int launch_scan(const float* xq, const float* cent, const float* pq, const uint8_t* codes,
                       const int64_t* list_off, const int64_t* probes, int nq, int nprobe, int d,
                       int M, float* ws_d, int* ws_i, hipStream_t s) {
  const int dsub = d / M;
  size_t lds = (size_t)(M * 256 + d) * 4;
  const size_t merge = (size_t)K * 8 + topk_select_lds(K);
  if (merge > lds) lds = merge;
  if (lds > 160 * 1024) return -2;
  const int items = nq * nprobe;
  if (M % 16 == 0)
    ivfpq_scan_kernel<K, true><<<items, 256, lds, s>>>(xq, cent, pq, codes, list_off, probes, nprobe, d, M, dsub, ws_d, ws_i);
  else
    ivfpq_scan_kernel<K, false><<<items, 256, lds, s>>>(xq, cent, pq, codes, list_off, probes, nprobe, d, M, dsub, ws_d, ws_i);
  return 0;
}

int docqa_ivfpq_search(const float* xq, const float* centroids, const float* pq,
                       const uint8_t* codes, const int64_t* ids, const int64_t* list_off,
                       const int64_t* probes, int nq, int nprobe, int d, int M, int k,
                       float* ws_d, int* ws_i, float* out_d, int64_t* out_i, hipStream_t s) {
  if (nq == 0) return 0;
  if (d % M != 0 || M % 4 != 0) return -1;
  const int kp = k <= 4 ? 4 : k <= 8 ? 8 : k <= 16 ? 16 : k <= 32 ? 32 : k <= 64 ? 64 : -1;
  int rc;
  switch (kp) {
    case 4: rc = launch_scan<4>(xq, centroids, pq, codes, list_off, probes, nq, nprobe, d, M, ws_d, ws_i, s);
      if (!rc) topk_merge_kernel<4, false><<<nq, 256, topk_merge_lds(4), s>>>(ws_d, ws_i, nprobe, nullptr, d, k, out_d, out_i, 0, ids);
      break;
    case 8: rc = launch_scan<8>(xq, centroids, pq, codes, list_off, probes, nq, nprobe, d, M, ws_d, ws_i, s);
      if (!rc) topk_merge_kernel<8, false><<<nq, 256, topk_merge_lds(8), s>>>(ws_d, ws_i, nprobe, nullptr, d, k, out_d, out_i, 0, ids);
      break;
    case 16: rc = launch_scan<16>(xq, centroids, pq, codes, list_off, probes, nq, nprobe, d, M, ws_d, ws_i, s);
      if (!rc) topk_merge_kernel<16, false><<<nq, 256, topk_merge_lds(16), s>>>(ws_d, ws_i, nprobe, nullptr, d, k, out_d, out_i, 0, ids);
      break;
    case 32: rc = launch_scan<32>(xq, centroids, pq, codes, list_off, probes, nq, nprobe, d, M, ws_d, ws_i, s);
      if (!rc) topk_merge_kernel<32, false><<<nq, 256, topk_merge_lds(32), s>>>(ws_d, ws_i, nprobe, nullptr, d, k, out_d, out_i, 0, ids);
      break;
    case 64: rc = launch_scan<64>(xq, centroids, pq, codes, list_off, probes, nq, nprobe, d, M, ws_d, ws_i, s);
      if (!rc) topk_merge_kernel<64, false><<<nq, 256, topk_merge_lds(64), s>>>(ws_d, ws_i, nprobe, nullptr, d, k, out_d, out_i, 0, ids);
      break;
    default: return -1;
  }
  if (rc) return rc;
  DOCQA_CHECK_LAUNCH();
  return 0;
}

int docqa_pq_encode(const float* x, const float* centroids, const int64_t* assign, const float* pq,
                    int n, int d, int M, uint8_t* codes, hipStream_t s) {
  if (n == 0) return 0;
  if (d % M != 0) return -1;
  const long long waves = (long long)n * M;
  const int blocks = (int)std::min<long long>((waves + 3) / 4, 1 << 16);
  pq_encode_kernel<<<blocks, 256, 0, s>>>(x, centroids, assign, pq, n, d, M, d / M, codes);
  DOCQA_CHECK_LAUNCH();
  return 0;
}
