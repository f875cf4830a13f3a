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
#include <hip/hip_fp16.h>
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

// ---------------------------------------------------------------------------------------
// Precomputed-table ADC scan (FAISS's "precomputed tables" decomposition, taken one step
// further).  For a vector x = c_l + r^ (coarse centroid + PQ reconstruction of the residual)
//     ||q - x||^2 = ||q||^2 - 2 <q, c_l>  +  ||c_l + r^||^2  -  2 sum_m <q_m, pq[m][code_m]>
//                   `---- per (q, list) ---'  `- per vector -'  `---- per query LUT -----'
// so the LUT depends on the QUERY only -- T[q][m][k] = -2 <q_m, pq[m][k]>, computed once per
// query for every probe (pq_lut16_kernel, fp16: 48 KB at M = 96, so two workgroups fit per
// CU) -- the vector term N_i = ||c_l + r^_i||^2 is stored at add time, and the list term is
// one dot product per probe (probe_base_kernel).  The old kernel rebuilt an M x 256 fp32 LUT
// from the 768 KB codebook for every (query, list) item (profiles/r4_ivfpq_bge_10m_coarse_
// kernel.log: 14.8 ms per 256-query batch at nprobe 256 before any top-k work).
// Top-k is threshold-filtered: a lane appends a candidate to an LDS buffer only when it
// beats the current K-th best; when the buffer nears capacity a radix select keeps the K
// best and tightens the threshold -- the per-vector cost no longer grows with K (the old
// K-long register insertion networks made k_factor 4 cost 24.8 vs 14.8 ms).

// T[q][m][k] = -2 <q_m, pq[m][k]> (fp16); grid nq, 256 threads (one per k)
__global__ __launch_bounds__(256) void pq_lut16_kernel(const float* __restrict__ xq, const float* __restrict__ pq,
                                                       int d, int M, __half* __restrict__ lut) {
  extern __shared__ float qv[];
  const int q = blockIdx.x, k = threadIdx.x, dsub = d / M;
  for (int c = k; c < d; c += 256) qv[c] = xq[(size_t)q * d + c];
  __syncthreads();
  for (int m = 0; m < M; ++m) {
    const float* cen = pq + ((size_t)m * 256 + k) * dsub;
    const float* r = qv + m * dsub;
    float s = 0.f;
    for (int j = 0; j < dsub; ++j) s += r[j] * cen[j];
    lut[((size_t)q * M + m) * 256 + k] = __float2half(-2.f * s);
  }
}

// base[q][p] = ||q||^2 - 2 <q, c_probe(q, p)>; grid nq, 256 threads (a wave per probe)
__global__ __launch_bounds__(256) void probe_base_kernel(const float* __restrict__ xq,
                                                         const float* __restrict__ centroids,
                                                         const int64_t* __restrict__ probes, int nprobe, int d,
                                                         float* __restrict__ base) {
  extern __shared__ float qv2[];
  __shared__ float red[4];
  const int q = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  float s = 0.f;
  for (int c = tid; c < d; c += 256) {
    const float v = xq[(size_t)q * d + c];
    qv2[c] = v;
    s += v * v;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  if (lane == 0) red[wave] = s;
  __syncthreads();
  const float qn = red[0] + red[1] + red[2] + red[3];
  for (int p = wave; p < nprobe; p += 4) {
    const int64_t l = probes[(size_t)q * nprobe + p];
    float dot = 0.f;
    if (l >= 0)
      for (int c = lane; c < d; c += 64) dot += qv2[c] * centroids[(size_t)l * d + c];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) dot += __shfl_xor(dot, o, 64);
    if (lane == 0) base[(size_t)q * nprobe + p] = l >= 0 ? qn - 2.f * dot : FLT_MAX;
  }
}

// Radix select over the LDS candidate buffer: keep the K smallest of n entries (ties at
// the K-th distance taken in buffer order), compacted to [0, min(n, K)); returns the K-th
// smallest distance (FLT_MAX when n < K).  Every thread calls it; CAP / 256 entries each.
template <int K, int CAP>
__device__ float buf_select(float* bd, int* bi, int n, int* hist, int* ctl) {
  constexpr int P = CAP / 256;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  float vd[P];
  int vi[P];
  uint32_t key[P];
#pragma unroll
  for (int e = 0; e < P; ++e) {
    const int s = tid + e * 256;
    vd[e] = s < n ? bd[s] : FLT_MAX;
    vi[e] = s < n ? bi[s] : -1;
    key[e] = s < n ? fkey(vd[e]) : 0xffffffffu;
  }
  if (n <= K) {       // nothing to drop (uniform: n is read from LDS by every thread)
    return FLT_MAX;
  }
  uint32_t prefix = 0, mask = 0;
  int need = K;       // rank (1-based) of the wanted key among those matching the prefix
#pragma unroll
  for (int shift = 24; shift >= 0; shift -= 8) {
    hist[tid] = 0;
    __syncthreads();
#pragma unroll
    for (int e = 0; e < P; ++e)
      if ((key[e] & mask) == prefix) atomicAdd(&hist[(key[e] >> shift) & 255], 1);
    __syncthreads();
    // inclusive scan of the 256 bins: per wave (64 bins), then the wave totals
    int v = hist[tid];
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int t = __shfl_up(v, o, 64);
      if (lane >= o) v += t;
    }
    if (lane == 63) ctl[wave] = v;
    __syncthreads();
    int off = 0;
    for (int w = 0; w < wave; ++w) off += ctl[w];
    const int incl = v + off, excl = incl - hist[tid];
    if (excl < need && need <= incl) { ctl[4] = tid; ctl[5] = need - excl; }
    __syncthreads();
    prefix |= (uint32_t)ctl[4] << shift;
    mask |= 255u << shift;
    need = ctl[5];
    __syncthreads();
  }
  const uint32_t T = prefix;   // the K-th smallest key; `need` of the entries equal to it are kept
  if (tid == 0) { ctl[6] = 0; ctl[7] = 0; }
  __syncthreads();
#pragma unroll
  for (int e = 0; e < P; ++e)
    if (key[e] < T) {
      const int p = atomicAdd(&ctl[6], 1);
      bd[p] = vd[e];
      bi[p] = vi[e];
    }
  __syncthreads();
  const int below = ctl[6];
#pragma unroll
  for (int e = 0; e < P; ++e)
    if (key[e] == T) {
      const int t = atomicAdd(&ctl[7], 1);
      if (t < need) {
        bd[below + t] = vd[e];
        bi[below + t] = vi[e];
      }
    }
  __syncthreads();
  return __uint_as_float((T & 0x80000000u) ? (T & 0x7fffffffu) : ~T);
}

template <int K, bool VEC16>
__global__ __launch_bounds__(256) void ivfpq_scan_pt_kernel(
    const __half* __restrict__ lut, const float* __restrict__ base, const float* __restrict__ norms,
    const uint8_t* __restrict__ codes, const int64_t* __restrict__ list_off, const int64_t* __restrict__ probes,
    int nprobe, int pc, int nchunk, int M, float* __restrict__ ws_d, int* __restrict__ ws_i) {
  constexpr int CAP = 1024;
  extern __shared__ __attribute__((aligned(16))) unsigned char pt_smem[];
  __half* slut = reinterpret_cast<__half*>(pt_smem);                  // [M][256]
  float* bd = reinterpret_cast<float*>(pt_smem + (size_t)M * 512);    // [CAP]
  int* bi = reinterpret_cast<int*>(bd + CAP);                          // [CAP]
  int* hist = bi + CAP;                                                // [256]
  int* ctl = hist + 256;                                               // [8] select scratch, [8] count
  const int q = blockIdx.x / nchunk, chunk = blockIdx.x % nchunk;
  const int tid = threadIdx.x;
  {   // the query's LUT -> LDS (16 B per thread per step)
    const uint4* src = reinterpret_cast<const uint4*>(lut + (size_t)q * M * 256);
    uint4* dst = reinterpret_cast<uint4*>(slut);
    for (int c = tid; c < M * 32; c += 256) dst[c] = src[c];
  }
  // insertion counters rotate over three LDS words so one barrier per pass suffices: pass j
  // appends through ctl[8 + j % 3] while thread 0 clears the word pass j + 1 will use (last
  // read after pass j - 2's barrier)
  if (tid < 3) ctl[8 + tid] = 0;
  __syncthreads();
  float thr = FLT_MAX;
  int fill = 0, pass = 0;   // uniform: buffered candidates, passes so far
  const int p0 = chunk * pc, p1 = min(nprobe, p0 + pc);
  for (int p = p0; p < p1; ++p) {
    const int64_t l = probes[(size_t)q * nprobe + p];
    if (l < 0) continue;                                     // uniform
    const float b = base[(size_t)q * nprobe + p];
    const int64_t lo = list_off[l], hi = list_off[l + 1];
    for (int64_t i0 = lo; i0 < hi; i0 += 256) {
      const int64_t i = i0 + tid;
      float dist = FLT_MAX;
      if (i < hi) {
        const uint8_t* row = codes + i * M;
        float s = b + norms[i];
        if constexpr (VEC16) {
          for (int m0 = 0; m0 < M; m0 += 16) {
            const uint4 w = *reinterpret_cast<const uint4*>(row + m0);
            const uint32_t ws[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
            for (int e = 0; e < 4; ++e)
#pragma unroll
              for (int bb = 0; bb < 4; ++bb)
                s += __half2float(slut[(m0 + e * 4 + bb) * 256 + ((ws[e] >> (8 * bb)) & 0xff)]);
          }
        } else {
          for (int m0 = 0; m0 < M; m0 += 4) {
            const uint32_t w = *reinterpret_cast<const uint32_t*>(row + m0);
#pragma unroll
            for (int bb = 0; bb < 4; ++bb) s += __half2float(slut[(m0 + bb) * 256 + ((w >> (8 * bb)) & 0xff)]);
          }
        }
        dist = s;
      }
      int* cnt = ctl + 8 + pass % 3;
      if (dist < thr) {
        const int pos = fill + atomicAdd(cnt, 1);
        bd[pos] = dist;
        bi[pos] = (int)i;
      }
      if (tid == 0) ctl[8 + (pass + 1) % 3] = 0;
      __syncthreads();
      fill += *cnt;
      ++pass;
      if (fill > CAP - 256) {                                // uniform: nearly full
        thr = buf_select<K, CAP>(bd, bi, fill, hist, ctl);
        fill = min(fill, K);
      }
    }
  }
  __syncthreads();
  const int n = fill;
  buf_select<K, CAP>(bd, bi, n, hist, ctl);
  const size_t ob = ((size_t)q * nchunk + chunk) * K;
  if (tid < K) {
    const bool ok = tid < min(n, K);
    ws_d[ob + tid] = ok ? bd[tid] : FLT_MAX;
    ws_i[ob + tid] = ok ? bi[tid] : -1;
  }
}

}  // namespace

// Precomputed-table IVF-PQ search (see ivfpq_scan_pt_kernel): norms [N] = ||c_l + r^_i||^2
// (list-major, like codes); lut_ws: >= nq * M * 256 halves; base_ws: >= nq * nprobe floats;
// ws_d / ws_i: >= nq * nchunk * kpad where nchunk = ceil(nprobe / pc).
int docqa_ivfpq_search_pt(const float* xq, const float* centroids, const float* pq, const uint8_t* codes,
                          const float* norms, const int64_t* ids, const int64_t* list_off, const int64_t* probes,
                          int nq, int nprobe, int d, int M, int k, int pc, void* lut_ws, float* base_ws,
                          float* ws_d, int* ws_i, float* out_d, int64_t* out_i, hipStream_t s) {
  if (nq == 0) return 0;
  if (d % M != 0 || M % 4 != 0 || pc < 1) return -1;
  const int kp = k <= 8 ? 8 : k <= 16 ? 16 : k <= 32 ? 32 : k <= 64 ? 64 : -1;
  if (kp < 0) return -1;
  const size_t lds = (size_t)M * 512 + 1024 * 8 + (256 + 16) * 4;
  if (lds > 160 * 1024) return -2;
  __half* lut = (__half*)lut_ws;
  pq_lut16_kernel<<<nq, 256, d * 4, s>>>(xq, pq, d, M, lut);
  probe_base_kernel<<<nq, 256, d * 4, s>>>(xq, centroids, probes, nprobe, d, base_ws);
  const int nchunk = (nprobe + pc - 1) / pc;
  const int grid = nq * nchunk;
  const bool v16 = M % 16 == 0;
#define DOCQA_PT(K_)                                                                                            \
  do {                                                                                                          \
    if (v16)                                                                                                    \
      ivfpq_scan_pt_kernel<K_, true><<<grid, 256, lds, s>>>(lut, base_ws, norms, codes, list_off, probes, nprobe, \
                                                            pc, nchunk, M, ws_d, ws_i);                          \
    else                                                                                                        \
      ivfpq_scan_pt_kernel<K_, false><<<grid, 256, lds, s>>>(lut, base_ws, norms, codes, list_off, probes,       \
                                                             nprobe, pc, nchunk, M, ws_d, ws_i);                 \
    topk_merge_kernel<K_, false><<<nq, 256, topk_merge_lds(K_), s>>>(ws_d, ws_i, nchunk, nullptr, d, k, out_d,   \
                                                                     out_i, 0, ids);                             \
  } while (0)
  switch (kp) {
    case 8: DOCQA_PT(8); break;
    case 16: DOCQA_PT(16); break;
    case 32: DOCQA_PT(32); break;
    default: DOCQA_PT(64); break;
  }
#undef DOCQA_PT
  DOCQA_CHECK_LAUNCH();
  return 0;
}

namespace {
// Exact re-rank of IVF-PQ candidates (FAISS IndexRefineFlat): per query one workgroup, a
// wave per candidate -- gather the stored vector (fp32 or bf16), squared L2 (IP: inner
// product) to the query, then the k best of the <= 64 candidates by rank counting (ties to
// the lower candidate slot).  out: D [nq, k] (+inf / -inf and id -1 for missing), I [nq, k].
template <bool BF16, bool IP>
__global__ __launch_bounds__(256) void refine_l2_kernel(const void* __restrict__ xb, const float* __restrict__ xq,
                                                        const int64_t* __restrict__ cand, int kc, int d, int k,
                                                        int64_t ntotal, float* __restrict__ out_d,
                                                        int64_t* __restrict__ out_i) {
  extern __shared__ float rq[];
  __shared__ float dist[64];
  const int q = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int c = tid; c < d; c += 256) rq[c] = xq[(size_t)q * d + c];
  __syncthreads();
  for (int j = wave; j < kc; j += 4) {
    const int64_t id = cand[(size_t)q * kc + j];
    float s = 0.f;
    if (id >= 0 && id < ntotal) {
      for (int c = lane; c < d; c += 64) {
        const float x = BF16 ? bf2f(reinterpret_cast<const uint16_t*>(xb)[(size_t)id * d + c])
                             : reinterpret_cast<const float*>(xb)[(size_t)id * d + c];
        if constexpr (IP) {
          s += x * rq[c];
        } else {
          const float t = x - rq[c];
          s += t * t;
        }
      }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    if (lane == 0) dist[j] = (id >= 0 && id < ntotal) ? (IP ? -s : s) : FLT_MAX;
  }
  __syncthreads();
  if (tid < kc) {
    const float v = dist[tid];
    int r = 0;
    for (int j = 0; j < kc; ++j) {
      const float u = dist[j];
      r += u < v || (u == v && j < tid);
    }
    if (r < k) {
      const bool ok = v != FLT_MAX;
      out_d[(size_t)q * k + r] = ok ? (IP ? -v : v) : (IP ? -INFINITY : INFINITY);
      out_i[(size_t)q * k + r] = ok ? cand[(size_t)q * kc + tid] : -1;
    }
  }
  // fewer candidates than k: the rest stays missing
  for (int r = kc + tid; r < k; r += 256) {
    out_d[(size_t)q * k + r] = IP ? -INFINITY : INFINITY;
    out_i[(size_t)q * k + r] = -1;
  }
}
}  // namespace

int docqa_refine_flat(const void* xb, int xb_bf16, int64_t ntotal, const float* xq, const int64_t* cand, int nq,
                      int kc, int d, int k, int ip, float* out_d, int64_t* out_i, hipStream_t s) {
  if (nq == 0) return 0;
  if (kc < 1 || kc > 64 || k < 1) return -1;
  auto* kern = xb_bf16 ? (ip ? refine_l2_kernel<true, true> : refine_l2_kernel<true, false>)
                       : (ip ? refine_l2_kernel<false, true> : refine_l2_kernel<false, false>);
  kern<<<nq, 256, d * 4, s>>>(xb, xq, cand, kc, d, k, ntotal, out_d, out_i);
  DOCQA_CHECK_LAUNCH();
  return 0;
}

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
