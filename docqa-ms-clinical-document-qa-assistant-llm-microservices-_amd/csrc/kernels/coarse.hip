// coarse.hip -- IVF coarse quantizer for wide probes: the nprobe nearest of nlist centroids
// per query, for nprobe up to 512 (FAISS IndexIVF's quantizer->search(xq, nprobe) with an
// IndexFlatL2 quantizer; reference index sites semantic-indexer/indexer.py:39,41 and the
// retriever search llm-qa/main.py:101, scaled to the 10M-vector config 2).
//
// The fused kNN kernel (knn.hip) keeps a register top-K per lane, which caps K at 64; the
// operating points with recall@10 >= 0.9 at 10M vectors need nprobe 128..512.  Two kernels:
//   1. distance tiles on MFMA, fp32 in / fp32 accumulate (v_mfma_f32_32x32x2_f32: exact
//      fp32, the quantizer's own arithmetic): 32 queries per workgroup staged in LDS, each
//      wave streams 32-centroid tiles; D[q, c] = ||c||^2 - 2 q.c (||q||^2 does not change a
//      query's probe order) -> a [nq, nlist] fp32 workspace (8 MB at nq 256, nlist 8192);
//   2. per-query selection, one workgroup per query: MSB-first radix select over the
//      order-preserving uint32 image of the distances (4 passes of a 256-bin LDS histogram)
//      finds the K-th smallest key T; keys < T and the lowest-index ties == T are compacted
//      into LDS as (key << 32 | centroid) and bitonic-sorted, so probes come out in
//      ascending distance, ties to the lower centroid id -- deterministic, the order of a
//      stable CPU sort.
#include "docqa_common.h"
#include <float.h>

using namespace docqa;

namespace {

constexpr int kMaxProbe = 512;

__global__ __launch_bounds__(256) void coarse_dist_kernel(const float* __restrict__ cent,
                                                          const float* __restrict__ cnorm, int nlist, int d,
                                                          const float* __restrict__ xq, int nq,
                                                          int rows_per_block, float* __restrict__ D) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int blk = blockIdx.x, q0 = blockIdx.y * 32;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int l32 = lane & 31, hh = lane >> 5;
  float* sq = reinterpret_cast<float*>(smem);
  for (int i = tid; i < 32 * d; i += 256) {
    const int q = i / d, c = i - q * d;
    sq[i] = (q0 + q < nq) ? xq[(size_t)(q0 + q) * d + c] : 0.f;
  }
  __syncthreads();
  const int row_begin = blk * rows_per_block;
  const int row_end = min(nlist, row_begin + rows_per_block);
  const int q = q0 + l32;
  for (int tile = row_begin + wave * 32; tile < row_end; tile += 128) {
    const int my_row = min(tile + l32, nlist - 1);   // clamped A-operand row
    f32x16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
    const float* a_row = cent + (size_t)my_row * d;
    const float* b_row = sq + l32 * d;
    for (int u = 0; u < d; u += 8) {
      const float4 a4 = *reinterpret_cast<const float4*>(a_row + u + 4 * hh);
      const float4 b4 = *reinterpret_cast<const float4*>(b_row + u + 4 * hh);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a4.x, b4.x, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a4.y, b4.y, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a4.z, b4.z, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a4.w, b4.w, acc, 0, 0, 0);
    }
    // lane owns query l32; tile rows (r & 3) + 8 (r >> 2) + 4 hh
    if (q < nq) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = tile + (r & 3) + 8 * (r >> 2) + 4 * hh;
        // cnorm null: the plain product (fp32 x @ W^T -- the PQ pre-rotation)
        if (row < row_end) D[(size_t)q * nlist + row] = cnorm ? cnorm[row] - 2.f * acc[r] : acc[r];
      }
    }
  }
}

__device__ __forceinline__ unsigned order_key(float f) {
  const unsigned u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

__global__ __launch_bounds__(256) void coarse_select_kernel(const float* __restrict__ D, int L, int K,
                                                            int64_t* __restrict__ probes) {
  __shared__ unsigned hist[256];
  __shared__ unsigned long long sel[kMaxProbe];
  __shared__ unsigned s_prefix, s_kleft, s_cnt;
  __shared__ unsigned wtot[4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const float* row = D + (size_t)blockIdx.x * L;
  unsigned prefix = 0, mask = 0, kleft = (unsigned)K;
  // 1. radix select: the K-th smallest key, 8 bits per pass from the top
  for (int shift = 24; shift >= 0; shift -= 8) {
    hist[tid] = 0;
    __syncthreads();
    for (int i = tid; i < L; i += 256) {
      const unsigned key = order_key(row[i]);
      if ((key & mask) == prefix) atomicAdd(&hist[(key >> shift) & 255u], 1u);
    }
    __syncthreads();
    if (tid == 0) {
      unsigned cum = 0, b = 0;
      for (; b < 255u; ++b) {
        if (cum + hist[b] >= kleft) break;
        cum += hist[b];
      }
      s_prefix = prefix | (b << shift);
      s_kleft = kleft - cum;
    }
    __syncthreads();
    prefix = s_prefix;
    kleft = s_kleft;
    mask |= 255u << shift;
  }
  const unsigned T = prefix;          // key of the K-th smallest distance
  // 2. compact: every key < T (K - kleft of them), then the kleft lowest-index keys == T
  if (tid == 0) s_cnt = 0;
  for (int i = tid; i < kMaxProbe; i += 256) sel[i] = ~0ull;
  __syncthreads();
  for (int i = tid; i < L; i += 256) {
    const unsigned key = order_key(row[i]);
    if (key < T) sel[atomicAdd(&s_cnt, 1u)] = ((unsigned long long)key << 32) | (unsigned)i;
  }
  __syncthreads();
  const unsigned lt = s_cnt;          // == K - kleft
  unsigned taken = 0;
  for (int base = 0; base < L && taken < kleft; base += 256) {
    const int i = base + tid;
    const bool eq = i < L && order_key(row[i]) == T;
    const unsigned long long bal = __ballot(eq);
    if (lane == 0) wtot[wave] = (unsigned)__popcll(bal);
    __syncthreads();
    unsigned before = 0, total = 0;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      before += w < wave ? wtot[w] : 0u;
      total += wtot[w];
    }
    const unsigned pos = taken + before + (unsigned)__popcll(bal & ((1ull << lane) - 1ull));
    if (eq && pos < kleft) sel[lt + pos] = ((unsigned long long)T << 32) | (unsigned)i;
    taken += total;
    __syncthreads();
  }
  __syncthreads();
  // 3. bitonic sort of the (padded) selection: ascending key, then centroid id
  int P = 1;
  while (P < K) P <<= 1;
  for (int k = 2; k <= P; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = tid; i < P; i += 256) {
        const int ixj = i ^ j;
        if (ixj > i) {
          const unsigned long long a = sel[i], b = sel[ixj];
          const bool up = (i & k) == 0;
          if ((a > b) == up) { sel[i] = b; sel[ixj] = a; }
        }
      }
      __syncthreads();
    }
  }
  for (int i = tid; i < K; i += 256) probes[(size_t)blockIdx.x * K + i] = (int64_t)(sel[i] & 0xffffffffull);
}

}  // namespace

// out[nq, n] = x[nq, d] @ w[n, d]^T in exact fp32 on the same MFMA tiles (d % 8 == 0): the
// IVF-PQ query pre-rotation x @ R with w = R^T, so the search path runs no library GEMM.
int docqa_fp32_gemm_nt(const float* x, int nq, int d, const float* w, int n, float* out, hipStream_t s) {
  if (nq == 0) return 0;
  if (d % 8 != 0 || n <= 0 || !docqa_aligned16(x) || !docqa_aligned16(w)) return -1;
  const size_t lds = (size_t)32 * d * 4;
  if (lds > 160 * 1024) return -2;
  int nblk = (n + 511) / 512;
  if (nblk > 256) nblk = 256;
  int rpb = (n + nblk - 1) / nblk;
  rpb = (rpb + 127) / 128 * 128;
  nblk = (n + rpb - 1) / rpb;
  coarse_dist_kernel<<<dim3(nblk, (nq + 31) / 32), 256, lds, s>>>(w, nullptr, n, d, x, nq, rpb, out);
  DOCQA_CHECK_LAUNCH();
  return 0;
}

// Workspace: fp32 [nq, nlist].  cent fp32 [nlist, d] (d % 8 == 0), cnorm fp32 [nlist],
// xq fp32 [nq, d] -> probes int64 [nq, nprobe] ascending by distance (ties: lower id).
int docqa_coarse_probes(const float* cent, const float* cnorm, int nlist, int d, const float* xq, int nq,
                        int nprobe, float* ws, int64_t* probes, hipStream_t s) {
  if (nq == 0) return 0;
  if (d % 8 != 0 || nlist <= 0 || nprobe < 1 || nprobe > kMaxProbe || nprobe > nlist) return -1;
  if (!docqa_aligned16(cent) || !docqa_aligned16(xq)) return -1;
  const size_t lds = (size_t)32 * d * 4;
  if (lds > 160 * 1024) return -2;
  // ~512 centroid rows per workgroup (4 tiles per wave), at most 256 row blocks
  int nblk = (nlist + 511) / 512;
  if (nblk > 256) nblk = 256;
  int rpb = (nlist + nblk - 1) / nblk;
  rpb = (rpb + 127) / 128 * 128;
  nblk = (nlist + rpb - 1) / rpb;
  coarse_dist_kernel<<<dim3(nblk, (nq + 31) / 32), 256, lds, s>>>(cent, cnorm, nlist, d, xq, nq, rpb, ws);
  coarse_select_kernel<<<nq, 256, 0, s>>>(ws, nlist, nprobe, probes);
  DOCQA_CHECK_LAUNCH();
  return 0;
}
