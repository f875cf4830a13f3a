// knn.hip -- exact brute-force k-nearest-neighbour search (FAISS IndexFlatL2 /
// IndexFlatIP semantics) with the distance GEMM on MFMA and the top-k fused into it.
//
// Reference parity: FAISS IndexFlatL2 search through the LangChain retriever
// (llm-qa/main.py:101, k=3) over the 649 x 384 fp32 index written by
// semantic-indexer/indexer.py:27,41.  FAISS returns squared L2 distances
// ||x||^2 + ||y||^2 - 2 x.y in ascending order and int64 labels (-1 = missing).
//
// Kernel 1 (grid: row-blocks x query-blocks, 256 threads):
//   * 32 queries per workgroup are staged once in LDS; the database streams from HBM.
//   * each wave takes 32-row database tiles: X = Xb . Xq^T on MFMA
//       fp32 database: v_mfma_f32_32x32x2_f32 (exact fp32, = FAISS fp32 semantics);
//         lane (r, h) loads one float4 of its row = the k-slots of 4 MFMAs, the query
//         operand uses the same dim permutation so the dot product is unchanged.
//       bf16 database: v_mfma_f32_32x32x16_bf16 (16-B row chunks, half the HBM bytes
//         for the 10M-vector shards).
//   * the accumulator puts one query per lane and 16 database rows in registers, so the
//     distance epilogue and the running per-lane top-K (register insertion network,
//     skipped wave-wide when no lane beats its current K-th) need no data movement.
//   * end: the 8 per-query lists (4 waves x 2 lane halves) merge through LDS into one
//     top-K per (query, row-block) -> workspace.
// Kernel 2 (grid nq): merges the row-block lists -> final (D, I) per query.
#include "docqa_common.h"
#include "docqa_topk.h"
#include <float.h>

using namespace docqa;

namespace {

template <int K, bool IP, bool BF16>
__global__ __launch_bounds__(256) void knn_tile_kernel(
    const void* __restrict__ xb, const float* __restrict__ xb_norms, int N, int d,
    const float* __restrict__ xq, int nq, int rows_per_block, float* __restrict__ ws_d,
    int* __restrict__ ws_i, int nblk) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int blk = blockIdx.x, q0 = blockIdx.y * 32;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int l32 = lane & 31, hh = lane >> 5;

  // ---- stage the 32 queries (zero padded) in LDS
  if constexpr (BF16) {
    uint16_t* sq = reinterpret_cast<uint16_t*>(smem);
    for (int i = tid; i < 32 * d; i += 256) {
      const int q = i / d, c = i - q * d;
      sq[i] = (q0 + q < nq) ? f2bf(xq[(size_t)(q0 + q) * d + c]) : 0;
    }
  } else {
    float* sq = reinterpret_cast<float*>(smem);
    for (int i = tid; i < 32 * d; i += 256) {
      const int q = i / d, c = i - q * d;
      sq[i] = (q0 + q < nq) ? xq[(size_t)(q0 + q) * d + c] : 0.f;
    }
  }
  __syncthreads();

  float td[K];
  int ti[K];
#pragma unroll
  for (int i = 0; i < K; ++i) { td[i] = FLT_MAX; ti[i] = -1; }

  const int row_begin = blk * rows_per_block;
  const int row_end = min(N, row_begin + rows_per_block);
  for (int tile = row_begin + wave * 32; tile < row_end; tile += 128) {
    const int my_row = min(tile + l32, N - 1);   // clamped A-operand row
    f32x16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
    if constexpr (BF16) {
      const uint16_t* a_row = reinterpret_cast<const uint16_t*>(xb) + (size_t)my_row * d;
      const uint16_t* b_row = reinterpret_cast<const uint16_t*>(smem) + l32 * d;
      for (int s = 0; s < d; s += 16) {
        uint4 av = *reinterpret_cast<const uint4*>(a_row + s + 8 * hh);
        uint4 bv = *reinterpret_cast<const uint4*>(b_row + s + 8 * hh);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(*reinterpret_cast<bf16x8*>(&av),
                                                      *reinterpret_cast<bf16x8*>(&bv), acc, 0, 0, 0);
      }
    } else {
      const float* a_row = reinterpret_cast<const float*>(xb) + (size_t)my_row * d;
      const float* b_row = reinterpret_cast<const float*>(smem) + l32 * d;
      for (int u = 0; u < d; u += 8) {
        const float4 a4 = *reinterpret_cast<const float4*>(a_row + u + 4 * hh);
        const float4 b4 = *reinterpret_cast<const float4*>(b_row + u + 4 * hh);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a4.x, b4.x, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a4.y, b4.y, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a4.z, b4.z, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a4.w, b4.w, acc, 0, 0, 0);
      }
    }
    // epilogue: lane owns query l32; rows (r&3) + 8(r>>2) + 4hh of the tile
    float dist[16];
    float mn = FLT_MAX;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = tile + (r & 3) + 8 * (r >> 2) + 4 * hh;
      float v;
      if (row < row_end) v = IP ? -acc[r] : xb_norms[row] - 2.f * acc[r];
      else v = FLT_MAX;
      dist[r] = v;
      mn = fminf(mn, v);
    }
    // wave-uniform skip when no lane can improve its list
    if (__any(mn < td[K - 1])) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = tile + (r & 3) + 8 * (r >> 2) + 4 * hh;
        if (dist[r] < td[K - 1]) topk_insert<K>(td, ti, dist[r], row);
      }
    }
  }

  // ---- merge the 8 lists per query through LDS (reuse the query region)
  __syncthreads();
  float* md = reinterpret_cast<float*>(smem);              // [32 q][8 lists][K]
  int* mi = reinterpret_cast<int*>(smem) + 32 * 8 * K;
  const int list = wave * 2 + hh;
#pragma unroll
  for (int i = 0; i < K; ++i) {
    md[(l32 * 8 + list) * K + i] = td[i];
    mi[(l32 * 8 + list) * K + i] = ti[i];
  }
  __syncthreads();
  if (tid < 32 && q0 + tid < nq) {
    const int q = tid;
    int head[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) head[j] = 0;
    const size_t ob = ((size_t)(q0 + q) * nblk + blk) * K;
    for (int i = 0; i < K; ++i) {
      int best = 0;
      float bd = FLT_MAX;
      int bi = 0x7fffffff;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if (head[j] < K) {
          const float v = md[(q * 8 + j) * K + head[j]];
          const int id = mi[(q * 8 + j) * K + head[j]];
          if (v < bd || (v == bd && id < bi)) { bd = v; bi = id; best = j; }
        }
      }
      head[best]++;
      ws_d[ob + i] = bd;
      ws_i[ob + i] = bd == FLT_MAX ? -1 : bi;
    }
  }
}

}  // namespace

int docqa_knn_workspace_blocks(int N) {
  int nblk = (N + 511) / 512;       // >= 512 rows (4 tiles per wave) per block
  if (nblk > 1024) nblk = 1024;
  return nblk < 1 ? 1 : nblk;
}

template <int K, bool IP, bool BF16>
static int launch_knn(const void* xb, const float* norms, int N, int d, const float* xq, int nq,
                      int k, float* ws_d, int* ws_i, int nblk, float* out_d, int64_t* out_i,
                      int64_t id_offset, hipStream_t s) {
  int rpb = (N + nblk - 1) / nblk;
  rpb = (rpb + 127) / 128 * 128;
  const size_t qbytes = (size_t)32 * d * (BF16 ? 2 : 4);
  const size_t mbytes = (size_t)32 * 8 * K * 8;
  const size_t lds = qbytes > mbytes ? qbytes : mbytes;
  if (lds > 160 * 1024) return -2;
  dim3 g1(nblk, (nq + 31) / 32);
  knn_tile_kernel<K, IP, BF16><<<g1, 256, lds, s>>>(xb, norms, N, d, xq, nq, rpb, ws_d, ws_i, nblk);
  topk_merge_kernel<K, IP><<<nq, 256, topk_merge_lds(K), s>>>(ws_d, ws_i, nblk, xq, d, k, out_d, out_i, id_offset, nullptr);
  DOCQA_CHECK_LAUNCH();
  return 0;
}

// ws_d/ws_i: [nq, nblk, Kpad] with Kpad = the template K the call selects (<= 64)
int docqa_knn_kpad(int k) { return k <= 4 ? 4 : k <= 8 ? 8 : k <= 16 ? 16 : k <= 32 ? 32 : k <= 64 ? 64 : -1; }

int docqa_knn(const void* xb, const float* norms, int N, int d, int is_bf16, const float* xq,
              int nq, int k, int metric_ip, float* ws_d, int* ws_i, int nblk, float* out_d,
              int64_t* out_i, int64_t id_offset, hipStream_t s) {
  if (nq == 0) return 0;
  if (d % (is_bf16 ? 16 : 8) != 0 || N <= 0) return -1;
  const int kp = docqa_knn_kpad(k);
#define KNN_CASE(KK)                                                                               \
  case KK:                                                                                         \
    if (metric_ip) {                                                                               \
      return is_bf16 ? launch_knn<KK, true, true>(xb, norms, N, d, xq, nq, k, ws_d, ws_i, nblk,    \
                                                  out_d, out_i, id_offset, s)                      \
                     : launch_knn<KK, true, false>(xb, norms, N, d, xq, nq, k, ws_d, ws_i, nblk,   \
                                                   out_d, out_i, id_offset, s);                    \
    } else {                                                                                       \
      return is_bf16 ? launch_knn<KK, false, true>(xb, norms, N, d, xq, nq, k, ws_d, ws_i, nblk,   \
                                                   out_d, out_i, id_offset, s)                     \
                     : launch_knn<KK, false, false>(xb, norms, N, d, xq, nq, k, ws_d, ws_i, nblk,  \
                                                    out_d, out_i, id_offset, s);                   \
    }
  switch (kp) {
    KNN_CASE(4)
    KNN_CASE(8)
    KNN_CASE(16)
    KNN_CASE(32)
    KNN_CASE(64)
    default: return -1;
  }
#undef KNN_CASE
}
