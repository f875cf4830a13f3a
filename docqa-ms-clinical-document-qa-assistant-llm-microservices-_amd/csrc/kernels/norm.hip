// norm.hip -- RMSNorm / fused residual-add RMSNorm (Llama) and LayerNorm with fused
// residual add (BERT encoders: MiniLM, bge, the NER token classifier).
//
// Layout: one wave64 per row, 4 rows per 256-thread workgroup.  Each lane owns
// NV 16-byte chunks (8 bf16) of its row, kept in registers between the reduction
// and the normalisation pass, so every byte of the row is read from HBM once and
// written once (memory-bound op: the only lever is bytes and vector width --
// cdna_hip_programming.md Guideline 13 and Appendix B "Reduction").
//
// Reference parity: the reference's encoders are sentence-transformers BERTs
// (semantic-indexer/indexer.py:21, llm-qa/main.py:25) and its generator is a
// llama.cpp Mistral (llm-qa/main.py:69) -- both normalisations live in those
// external engines; these kernels are their MI355X-native replacements.
#include "docqa_common.h"
#include "docqa_norm_row.h"

using namespace docqa;

template <int NV, bool ADD>
__global__ __launch_bounds__(256) void rmsnorm_kernel(const uint16_t* __restrict__ x,
                                                      uint16_t* __restrict__ residual,
                                                      const uint16_t* __restrict__ w,
                                                      uint16_t* __restrict__ out, int rows,
                                                      int H, float eps) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const int nchunk = H >> 3;
  const uint4* xr = reinterpret_cast<const uint4*>(x + (size_t)row * H);
  uint4* rr = reinterpret_cast<uint4*>(residual + (size_t)row * H);
  float v[NV][8];
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = lane + 64 * i;
    if (c < nchunk) {
      unpack8(xr[c], v[i]);
      if constexpr (ADD) {
        float r[8];
        unpack8(rr[c], r);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[i][j] = bf2f(f2bf(v[i][j] + r[j]));  // bf16 residual stream
        rr[c] = pack8(v[i]);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) ss += v[i][j] * v[i][j];
    }
  }
  ss = wave_sum(ss);
  const float inv = rsqrtf(ss / (float)H + eps);
  const uint4* wr = reinterpret_cast<const uint4*>(w);
  uint4* orow = reinterpret_cast<uint4*>(out + (size_t)row * H);
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = lane + 64 * i;
    if (c < nchunk) {
      float g[8], o[8];
      unpack8(wr[c], g);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = v[i][j] * inv * g[j];
      orow[c] = pack8(o);
    }
  }
}

// Few-row variant (decode: rows = batch <= a few thousand): one 256-thread workgroup per
// row so a 64-row step still spreads over 64 CUs with 2 chunks per lane, instead of 16
// workgroups each walking four whole rows.
template <int NV, bool ADD>
__global__ __launch_bounds__(256) void rmsnorm_row_kernel(const uint16_t* __restrict__ x,
                                                          uint16_t* __restrict__ residual,
                                                          const uint16_t* __restrict__ w,
                                                          uint16_t* __restrict__ out, int H,
                                                          float eps) {
  const int row = blockIdx.x;
  const int tid = threadIdx.x;
  const int nchunk = H >> 3;
  const uint4* xr = reinterpret_cast<const uint4*>(x + (size_t)row * H);
  uint4* rr = reinterpret_cast<uint4*>(residual + (size_t)row * H);
  float v[NV][8];
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = tid + 256 * i;
    if (c < nchunk) {
      unpack8(xr[c], v[i]);
      if constexpr (ADD) {
        float r[8];
        unpack8(rr[c], r);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[i][j] = bf2f(f2bf(v[i][j] + r[j]));
        rr[c] = pack8(v[i]);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) ss += v[i][j] * v[i][j];
    }
  }
  __shared__ float red[4];
  ss = wave_sum(ss);
  if ((tid & 63) == 0) red[tid >> 6] = ss;
  __syncthreads();
  ss = red[0] + red[1] + red[2] + red[3];
  const float inv = rsqrtf(ss / (float)H + eps);
  const uint4* wr = reinterpret_cast<const uint4*>(w);
  uint4* orow = reinterpret_cast<uint4*>(out + (size_t)row * H);
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = tid + 256 * i;
    if (c < nchunk) {
      float g[8], o[8];
      unpack8(wr[c], g);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = v[i][j] * inv * g[j];
      orow[c] = pack8(o);
    }
  }
}

// Decode add_rmsnorm fed straight by a split-K projection: x = sum of S fp32 partial slabs
// P[s][row][:] (the skinny GEMM's split-K combine fused here instead of a separate
// reduce launch + bf16 round trip).  x is rounded to bf16 before the residual add so the
// result matches projection -> bf16 -> add_rmsnorm bit for bit.
// NS > 0: S == NS at compile time -- every slab, the residual and the weight chunk are
// loaded before the first add, so the row costs one memory latency instead of S + 2
// dependent ones (at 128 decode rows this kernel is latency-bound, not bandwidth-bound).
template <int NV, int NS, typename PT>
__global__ __launch_bounds__(256) void add_rmsnorm_splitk_kernel(const PT* __restrict__ P,
                                                                 int S, size_t slab,
                                                                 uint16_t* __restrict__ residual,
                                                                 const uint16_t* __restrict__ w,
                                                                 uint16_t* __restrict__ out,
                                                                 int H, float eps) {
  __shared__ float red[4];
  add_rmsnorm_splitk_row<NV, NS>(P, S, slab, residual, w, out, H, eps, blockIdx.x, threadIdx.x, red);
}

// LayerNorm(x [+ residual]) * gamma + beta; optional residual may alias nothing.
template <int NV, bool ADD>
__global__ __launch_bounds__(256) void layernorm_kernel(const uint16_t* __restrict__ x,
                                                        const uint16_t* __restrict__ residual,
                                                        const uint16_t* __restrict__ gamma,
                                                        const uint16_t* __restrict__ beta,
                                                        uint16_t* __restrict__ out, int rows,
                                                        int H, float eps) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const int nchunk = H >> 3;
  const uint4* xr = reinterpret_cast<const uint4*>(x + (size_t)row * H);
  const uint4* rr = reinterpret_cast<const uint4*>(residual + (size_t)row * H);
  float v[NV][8];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = lane + 64 * i;
    if (c < nchunk) {
      unpack8(xr[c], v[i]);
      if constexpr (ADD) {
        float r[8];
        unpack8(rr[c], r);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[i][j] += r[j];
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) s += v[i][j];
    }
  }
  const float mean = wave_sum(s) / (float)H;
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = lane + 64 * i;
    if (c < nchunk) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float d = v[i][j] - mean;
        ss += d * d;
      }
    }
  }
  const float inv = rsqrtf(wave_sum(ss) / (float)H + eps);
  const uint4* gr = reinterpret_cast<const uint4*>(gamma);
  const uint4* br = reinterpret_cast<const uint4*>(beta);
  uint4* orow = reinterpret_cast<uint4*>(out + (size_t)row * H);
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = lane + 64 * i;
    if (c < nchunk) {
      float g[8], b[8], o[8];
      unpack8(gr[c], g);
      unpack8(br[c], b);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = (v[i][j] - mean) * inv * g[j] + b[j];
      orow[c] = pack8(o);
    }
  }
}

template <bool ADD>
static int launch_rms(const void* x, void* res, const void* w, void* out, int rows, int H,
                      float eps, hipStream_t s) {
  dim3 grid((rows + 3) / 4), block(256);
  const int nv = (H / 8 + 63) / 64;
  const uint16_t *xp = (const uint16_t*)x, *wp = (const uint16_t*)w;
  uint16_t *rp = (uint16_t*)res, *op = (uint16_t*)out;
  if (rows <= 2048 && H >= 1024) {  // few rows: one workgroup per row
    const int nvr = (H / 8 + 255) / 256;
    if (nvr <= 1) rmsnorm_row_kernel<1, ADD><<<rows, 256, 0, s>>>(xp, rp, wp, op, H, eps);
    else if (nvr <= 2) rmsnorm_row_kernel<2, ADD><<<rows, 256, 0, s>>>(xp, rp, wp, op, H, eps);
    else if (nvr <= 4) rmsnorm_row_kernel<4, ADD><<<rows, 256, 0, s>>>(xp, rp, wp, op, H, eps);
    else return -1;
    DOCQA_CHECK_LAUNCH();
    return 0;
  }
  if (nv <= 1) rmsnorm_kernel<1, ADD><<<grid, block, 0, s>>>(xp, rp, wp, op, rows, H, eps);
  else if (nv <= 2) rmsnorm_kernel<2, ADD><<<grid, block, 0, s>>>(xp, rp, wp, op, rows, H, eps);
  else if (nv <= 4) rmsnorm_kernel<4, ADD><<<grid, block, 0, s>>>(xp, rp, wp, op, rows, H, eps);
  else if (nv <= 8) rmsnorm_kernel<8, ADD><<<grid, block, 0, s>>>(xp, rp, wp, op, rows, H, eps);
  else if (nv <= 16) rmsnorm_kernel<16, ADD><<<grid, block, 0, s>>>(xp, rp, wp, op, rows, H, eps);
  else return -1;
  DOCQA_CHECK_LAUNCH();
  return 0;
}

int docqa_rmsnorm(const void* x, const void* w, void* out, int rows, int H, float eps,
                  hipStream_t s) {
  if (H % 8 != 0 || rows <= 0) return rows == 0 ? 0 : -1;
  return launch_rms<false>(x, nullptr, w, out, rows, H, eps, s);
}

int docqa_add_rmsnorm(const void* x, void* residual, const void* w, void* out, int rows, int H,
                      float eps, hipStream_t s) {
  if (H % 8 != 0 || rows <= 0) return rows == 0 ? 0 : -1;
  return launch_rms<true>(x, residual, w, out, rows, H, eps, s);
}

template <int NV, typename PT>
static void launch_arns(const PT* P, int S, size_t slab, uint16_t* rp, const uint16_t* wp,
                        uint16_t* op, int rows, int H, float eps, hipStream_t s) {
#define DOCQA_ARNS(NS_) add_rmsnorm_splitk_kernel<NV, NS_, PT><<<rows, 256, 0, s>>>(P, S, slab, rp, wp, op, H, eps)
  switch (S) {
    case 1: DOCQA_ARNS(1); break;
    case 2: DOCQA_ARNS(2); break;
    case 3: DOCQA_ARNS(3); break;
    case 4: DOCQA_ARNS(4); break;
    case 5: DOCQA_ARNS(5); break;
    case 6: DOCQA_ARNS(6); break;
    case 7: DOCQA_ARNS(7); break;
    case 8: DOCQA_ARNS(8); break;
    default: DOCQA_ARNS(0); break;
  }
#undef DOCQA_ARNS
}

template <typename PT>
static int add_rmsnorm_splitk_any(const PT* P, int S, void* residual, const void* w, void* out, int rows, int H,
                                  float eps, hipStream_t s) {
  if (rows == 0) return 0;
  if (H % 8 != 0 || S < 1) return -1;
  const size_t slab = (size_t)rows * H;
  const int nvr = (H / 8 + 255) / 256;
  uint16_t *rp = (uint16_t*)residual, *op = (uint16_t*)out;
  const uint16_t* wp = (const uint16_t*)w;
  if (nvr > 4) return -1;
  if (nvr <= 1) launch_arns<1>(P, S, slab, rp, wp, op, rows, H, eps, s);
  else if (nvr <= 2) launch_arns<2>(P, S, slab, rp, wp, op, rows, H, eps, s);
  else launch_arns<4>(P, S, slab, rp, wp, op, rows, H, eps, s);
  DOCQA_CHECK_LAUNCH();
  return 0;
}

int docqa_add_rmsnorm_splitk(const float* P, int S, void* residual, const void* w, void* out,
                             int rows, int H, float eps, hipStream_t s) {
  return add_rmsnorm_splitk_any(P, S, residual, w, out, rows, H, eps, s);
}

// bf16 slabs (mgemm.hip EPI_PARTIAL16), summed in fp32 in slab order like the fp32 form
int docqa_add_rmsnorm_splitk16(const void* P, int S, void* residual, const void* w, void* out,
                               int rows, int H, float eps, hipStream_t s) {
  return add_rmsnorm_splitk_any((const uint16_t*)P, S, residual, w, out, rows, H, eps, s);
}

int docqa_layernorm(const void* x, const void* residual, const void* g, const void* b, void* out,
                    int rows, int H, float eps, hipStream_t s) {
  if (H % 8 != 0 || rows <= 0) return rows == 0 ? 0 : -1;
  dim3 grid((rows + 3) / 4), block(256);
  const int nv = (H / 8 + 63) / 64;
  const uint16_t *xp = (const uint16_t*)x, *rp = (const uint16_t*)residual,
                 *gp = (const uint16_t*)g, *bp = (const uint16_t*)b;
  uint16_t* op = (uint16_t*)out;
  if (residual) {
    if (nv <= 1) layernorm_kernel<1, true><<<grid, block, 0, s>>>(xp, rp, gp, bp, op, rows, H, eps);
    else if (nv <= 2) layernorm_kernel<2, true><<<grid, block, 0, s>>>(xp, rp, gp, bp, op, rows, H, eps);
    else if (nv <= 4) layernorm_kernel<4, true><<<grid, block, 0, s>>>(xp, rp, gp, bp, op, rows, H, eps);
    else if (nv <= 8) layernorm_kernel<8, true><<<grid, block, 0, s>>>(xp, rp, gp, bp, op, rows, H, eps);
    else return -1;
  } else {
    if (nv <= 1) layernorm_kernel<1, false><<<grid, block, 0, s>>>(xp, rp, gp, bp, op, rows, H, eps);
    else if (nv <= 2) layernorm_kernel<2, false><<<grid, block, 0, s>>>(xp, rp, gp, bp, op, rows, H, eps);
    else if (nv <= 4) layernorm_kernel<4, false><<<grid, block, 0, s>>>(xp, rp, gp, bp, op, rows, H, eps);
    else if (nv <= 8) layernorm_kernel<8, false><<<grid, block, 0, s>>>(xp, rp, gp, bp, op, rows, H, eps);
    else return -1;
  }
  DOCQA_CHECK_LAUNCH();
  return 0;
}
