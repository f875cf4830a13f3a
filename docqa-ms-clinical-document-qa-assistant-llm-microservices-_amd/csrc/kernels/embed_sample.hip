// embed_sample.hip -- token-embedding gathers and the greedy / stochastic samplers.
//
//  * embedding_gather : out[t] = table[ids[t]]              (Llama, vocab 128256)
//  * bert_embed_ln    : LN(word[ids] + pos[p] + type[tt])  (BERT encoders; one wave per
//                       token, fused gather + add + LayerNorm, one HBM pass)
//  * argmax_rows      : greedy decode (temperature 0, as the reference's
//                       ChatOllama(temperature=0) at llm-qa/main.py:69); two-pass split
//                       over the vocab so a small batch still fills 256 CUs
//  * sample_rows      : temperature / top-k / top-p sampling from fp32 logits with a
//                       per-row uniform draw supplied by the caller (graph-capturable:
//                       no RNG state inside the kernel)
#include "docqa_common.h"
#include <float.h>

using namespace docqa;

__global__ __launch_bounds__(256) void embedding_gather_kernel(const int* __restrict__ ids,
                                                               const uint16_t* __restrict__ table,
                                                               uint16_t* __restrict__ out, int H, int V) {
  const int t = blockIdx.x;
  // out-of-range ids (a padded decode slot's stale token) read row 0, never past the table
  const int id = (unsigned)ids[t] < (unsigned)V ? ids[t] : 0;
  const uint4* src = reinterpret_cast<const uint4*>(table + (size_t)id * H);
  uint4* dst = reinterpret_cast<uint4*>(out + (size_t)t * H);
  for (int c = threadIdx.x; c < (H >> 3); c += blockDim.x) dst[c] = src[c];
}

// Llama input: h = table[id] (the residual stream) and x = rmsnorm(h) * w for the first
// layer in one launch, one workgroup per token (decode: one kernel and one boundary fewer
// per step).  Same thread -> chunk map and arithmetic as norm.hip rmsnorm_row_kernel.
template <int NV>
__global__ __launch_bounds__(256) void embed_rmsnorm_kernel(const int* __restrict__ ids,
                                                            const uint16_t* __restrict__ table,
                                                            const uint16_t* __restrict__ w,
                                                            uint16_t* __restrict__ h, uint16_t* __restrict__ x,
                                                            int H, int V, float eps) {
  __shared__ float red[4];
  const int t = blockIdx.x, tid = threadIdx.x, nchunk = H >> 3;
  const int id = (unsigned)ids[t] < (unsigned)V ? ids[t] : 0;
  const uint4* src = reinterpret_cast<const uint4*>(table + (size_t)id * H);
  uint4* hr = reinterpret_cast<uint4*>(h + (size_t)t * H);
  float v[NV][8];
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = tid + 256 * i;
    if (c < nchunk) {
      const uint4 q = src[c];
      hr[c] = q;
      unpack8(q, v[i]);
#pragma unroll
      for (int j = 0; j < 8; ++j) ss += v[i][j] * v[i][j];
    }
  }
  ss = wave_sum(ss);
  if ((tid & 63) == 0) red[tid >> 6] = ss;
  __syncthreads();
  ss = red[0] + red[1] + red[2] + red[3];
  const float inv = rsqrtf(ss / (float)H + eps);
  const uint4* wr = reinterpret_cast<const uint4*>(w);
  uint4* xr = reinterpret_cast<uint4*>(x + (size_t)t * H);
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = tid + 256 * i;
    if (c < nchunk) {
      float g[8], o[8];
      unpack8(wr[c], g);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = v[i][j] * inv * g[j];
      xr[c] = pack8(o);
    }
  }
}

template <int NV>
__global__ __launch_bounds__(256) void bert_embed_ln_kernel(
    const int* __restrict__ ids, const int* __restrict__ pos, const int* __restrict__ tt,
    const uint16_t* __restrict__ wte, const uint16_t* __restrict__ wpe,
    const uint16_t* __restrict__ wtt, const uint16_t* __restrict__ gamma,
    const uint16_t* __restrict__ beta, uint16_t* __restrict__ out, int T, int H, float eps) {
  const int t = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (t >= T) return;
  const int nchunk = H >> 3;
  const uint4* w = reinterpret_cast<const uint4*>(wte + (size_t)ids[t] * H);
  const uint4* p = reinterpret_cast<const uint4*>(wpe + (size_t)pos[t] * H);
  const uint4* y = reinterpret_cast<const uint4*>(wtt + (size_t)(tt ? tt[t] : 0) * H);
  float v[NV][8];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = lane + 64 * i;
    if (c < nchunk) {
      float a[8], b[8];
      unpack8(w[c], v[i]);
      unpack8(p[c], a);
      unpack8(y[c], b);
#pragma unroll
      for (int j = 0; j < 8; ++j) { v[i][j] += a[j] + b[j]; s += v[i][j]; }
    }
  }
  const float mean = wave_sum(s) / (float)H;
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = lane + 64 * i;
    if (c < nchunk) {
#pragma unroll
      for (int j = 0; j < 8; ++j) { const float d = v[i][j] - mean; ss += d * d; }
    }
  }
  const float inv = rsqrtf(wave_sum(ss) / (float)H + eps);
  uint4* o = reinterpret_cast<uint4*>(out + (size_t)t * H);
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = lane + 64 * i;
    if (c < nchunk) {
      float g[8], b[8], r[8];
      unpack8(reinterpret_cast<const uint4*>(gamma)[c], g);
      unpack8(reinterpret_cast<const uint4*>(beta)[c], b);
#pragma unroll
      for (int j = 0; j < 8; ++j) r[j] = (v[i][j] - mean) * inv * g[j] + b[j];
      o[c] = pack8(r);
    }
  }
}

// ---------------------------------------------------------------------------------
// argmax: pass 1 -- each (row, split) workgroup reduces a vocab slice to (max, idx);
// pass 2 -- one wave per row merges the splits.  Ties resolve to the lowest index,
// like torch.argmax.
__device__ __forceinline__ void better(float& bv, int& bi, float v, int i) {
  if (v > bv || (v == bv && i < bi)) { bv = v; bi = i; }
}

template <bool BF16>
__global__ __launch_bounds__(256) void argmax_pass1(const void* __restrict__ logits, int V,
                                                    int ld, int splits, float* __restrict__ pv,
                                                    int* __restrict__ pi) {
  const int row = blockIdx.y, sp = blockIdx.x;
  const int chunk = ((V + splits - 1) / splits + 7) & ~7;
  const int lo = sp * chunk, hi = min(V, lo + chunk);
  float bv = -FLT_MAX;
  int bi = 0x7fffffff;
  if constexpr (BF16) {
    const uint16_t* r = reinterpret_cast<const uint16_t*>(logits) + (size_t)row * ld;
    // vector body (ld and lo are multiples of 8 when V % 8 == 0)
    int i = lo + threadIdx.x * 8;
    for (; i + 8 <= hi; i += 256 * 8) {
      float f[8];
      unpack8(*reinterpret_cast<const uint4*>(r + i), f);
#pragma unroll
      for (int j = 0; j < 8; ++j) better(bv, bi, f[j], i + j);
    }
    for (; i < hi; ++i) better(bv, bi, bf2f(r[i]), i);
  } else {
    const float* r = reinterpret_cast<const float*>(logits) + (size_t)row * ld;
    int i = lo + threadIdx.x * 4;
    for (; i + 4 <= hi; i += 256 * 4) {
      const float4 f = *reinterpret_cast<const float4*>(r + i);
      better(bv, bi, f.x, i); better(bv, bi, f.y, i + 1);
      better(bv, bi, f.z, i + 2); better(bv, bi, f.w, i + 3);
    }
    for (; i < hi; ++i) better(bv, bi, r[i], i);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ov = __shfl_xor(bv, o, 64);
    const int oi = __shfl_xor(bi, o, 64);
    better(bv, bi, ov, oi);
  }
  __shared__ float sv[4];
  __shared__ int si[4];
  if ((threadIdx.x & 63) == 0) { sv[threadIdx.x >> 6] = bv; si[threadIdx.x >> 6] = bi; }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < 4; ++w) better(bv, bi, sv[w], si[w]);
    pv[row * splits + sp] = bv;
    pi[row * splits + sp] = bi;
  }
}

__global__ __launch_bounds__(64) void argmax_pass2(const float* __restrict__ pv,
                                                   const int* __restrict__ pi, int splits,
                                                   int64_t* __restrict__ out) {
  const int row = blockIdx.x;
  float bv = -FLT_MAX;
  int bi = 0x7fffffff;
  for (int s = threadIdx.x; s < splits; s += 64) better(bv, bi, pv[row * splits + s], pi[row * splits + s]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ov = __shfl_xor(bv, o, 64);
    const int oi = __shfl_xor(bi, o, 64);
    better(bv, bi, ov, oi);
  }
  if (threadIdx.x == 0) out[row] = bi == 0x7fffffff ? 0 : bi;   // all-NaN row: a valid id
}

// ---------------------------------------------------------------------------------
// Sampling: one 256-thread workgroup per row.  logits are fp32 (already divided by
// the temperature by the caller or by `inv_temp` here).  top-k is applied by a
// threshold search (bisection on the value range, 24 rounds, no sort); top-p by a
// second bisection on the probability mass of the survivors.  Then an inverse-CDF
// draw with the caller's uniform u[row].
__device__ float block_sum(float v, float* sh) {
  v = wave_sum(v);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
  __syncthreads();
  return sh[0] + sh[1] + sh[2] + sh[3];
}
__device__ float block_max(float v, float* sh) {
  v = wave_max(v);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
  __syncthreads();
  return fmaxf(fmaxf(sh[0], sh[1]), fmaxf(sh[2], sh[3]));
}

__global__ __launch_bounds__(256) void sample_kernel(const float* __restrict__ logits, int V,
                                                     int ld, const float* __restrict__ inv_temp,
                                                     const int* __restrict__ top_k,
                                                     const float* __restrict__ top_p,
                                                     const float* __restrict__ u,
                                                     int64_t* __restrict__ out) {
  __shared__ float sh[4];
  const int row = blockIdx.x;
  const float* r = logits + (size_t)row * ld;
  const float it = inv_temp[row];
  float mx = -FLT_MAX, mn = FLT_MAX;
  for (int i = threadIdx.x; i < V; i += 256) { const float x = r[i] * it; mx = fmaxf(mx, x); mn = fminf(mn, x); }
  mx = block_max(mx, sh);
  mn = -block_max(-mn, sh);
  // top-k threshold: largest th such that count(x >= th) >= k
  float th = -FLT_MAX;
  const int k = top_k[row];
  if (k > 0 && k < V) {
    float lo = mn, hi = mx;
    for (int it2 = 0; it2 < 24; ++it2) {
      const float mid = 0.5f * (lo + hi);
      float c = 0.f;
      for (int i = threadIdx.x; i < V; i += 256) c += (r[i] * it >= mid) ? 1.f : 0.f;
      c = block_sum(c, sh);
      if (c >= (float)k) lo = mid; else hi = mid;
    }
    th = lo;
  }
  float z = 0.f;
  for (int i = threadIdx.x; i < V; i += 256) { const float x = r[i] * it; if (x >= th) z += __expf(x - mx); }
  z = block_sum(z, sh);
  const float p = top_p[row];
  if (p > 0.f && p < 1.f) {
    // smallest threshold set whose mass >= p: bisection on th2 in [th, mx]
    float lo = fmaxf(th, mn), hi = mx;
    for (int it2 = 0; it2 < 24; ++it2) {
      const float mid = 0.5f * (lo + hi);
      float m = 0.f;
      for (int i = threadIdx.x; i < V; i += 256) { const float x = r[i] * it; if (x >= mid) m += __expf(x - mx); }
      m = block_sum(m, sh);
      if (m >= p * z) lo = mid; else hi = mid;
    }
    th = fmaxf(th, lo);
    z = 0.f;
    for (int i = threadIdx.x; i < V; i += 256) { const float x = r[i] * it; if (x >= th) z += __expf(x - mx); }
    z = block_sum(z, sh);
  }
  // inverse CDF, chunked: each thread owns a contiguous slice of the vocab
  const int per = (V + 255) / 256;
  const int lo_i = threadIdx.x * per, hi_i = min(V, lo_i + per);
  float local = 0.f;
  for (int i = lo_i; i < hi_i; ++i) { const float x = r[i] * it; if (x >= th) local += __expf(x - mx); }
  // exclusive prefix over threads via LDS
  __shared__ float pre[256];
  pre[threadIdx.x] = local;
  __syncthreads();
  if (threadIdx.x == 0) {
    float acc = 0.f;
    for (int i = 0; i < 256; ++i) { const float v = pre[i]; pre[i] = acc; acc += v; }
  }
  __syncthreads();
  const float target = u[row] * z;
  __shared__ int chosen;
  if (threadIdx.x == 0) chosen = -1;
  __syncthreads();
  const float start = pre[threadIdx.x];
  if (target >= start && target < start + local) {
    float acc = start;
    int pick = -1;
    for (int i = lo_i; i < hi_i; ++i) {
      const float x = r[i] * it;
      if (x >= th) { acc += __expf(x - mx); pick = i; if (acc > target) break; }
    }
    atomicMax(&chosen, pick);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int c = chosen;
    if (c < 0) {  // numerical edge: fall back to the argmax
      float bv = -FLT_MAX;
      for (int i = 0; i < V; ++i) if (r[i] > bv) { bv = r[i]; c = i; }
    }
    out[row] = c;
  }
}

int docqa_embedding(const int* ids, const void* table, void* out, int T, int H, int V, hipStream_t s) {
  if (T == 0) return 0;
  if (H % 8 != 0 || !docqa_aligned16(table) || !docqa_aligned16(out)) return -1;
  embedding_gather_kernel<<<T, 256, 0, s>>>(ids, (const uint16_t*)table, (uint16_t*)out, H, V);
  DOCQA_CHECK_LAUNCH();
  return 0;
}

int docqa_embed_rmsnorm(const int* ids, const void* table, const void* w, void* h, void* x, int T, int H, int V,
                        float eps, hipStream_t s) {
  if (T == 0) return 0;
  if (H % 8 != 0 || H > 8192 || !docqa_aligned16(table) || !docqa_aligned16(w) || !docqa_aligned16(h) ||
      !docqa_aligned16(x)) return -1;
  const int nv = (H / 8 + 255) / 256;
  if (nv <= 1)
    embed_rmsnorm_kernel<1><<<T, 256, 0, s>>>(ids, (const uint16_t*)table, (const uint16_t*)w, (uint16_t*)h,
                                              (uint16_t*)x, H, V, eps);
  else if (nv == 2)
    embed_rmsnorm_kernel<2><<<T, 256, 0, s>>>(ids, (const uint16_t*)table, (const uint16_t*)w, (uint16_t*)h,
                                              (uint16_t*)x, H, V, eps);
  else
    embed_rmsnorm_kernel<4><<<T, 256, 0, s>>>(ids, (const uint16_t*)table, (const uint16_t*)w, (uint16_t*)h,
                                              (uint16_t*)x, H, V, eps);
  DOCQA_CHECK_LAUNCH();
  return 0;
}

int docqa_bert_embed_ln(const int* ids, const int* pos, const int* tt, const void* wte,
                        const void* wpe, const void* wtt, const void* g, const void* b, void* out,
                        int T, int H, float eps, hipStream_t s) {
  if (T == 0) return 0;
  if (H % 8 != 0 || !docqa_aligned16(wte) || !docqa_aligned16(wpe) || !docqa_aligned16(wtt) ||
      !docqa_aligned16(g) || !docqa_aligned16(b) || !docqa_aligned16(out)) return -1;
  const int nv = (H / 8 + 63) / 64;
  dim3 grid((T + 3) / 4);
#define BE(N) bert_embed_ln_kernel<N><<<grid, 256, 0, s>>>(ids, pos, tt, (const uint16_t*)wte, (const uint16_t*)wpe, (const uint16_t*)wtt, (const uint16_t*)g, (const uint16_t*)b, (uint16_t*)out, T, H, eps)
  if (nv <= 1) BE(1); else if (nv <= 2) BE(2); else if (nv <= 4) BE(4); else return -1;
#undef BE
  DOCQA_CHECK_LAUNCH();
  return 0;
}

int docqa_argmax(const void* logits, int rows, int V, int ld, int is_bf16, float* ws_v, int* ws_i,
                 int splits, int64_t* out, hipStream_t s) {
  if (rows == 0) return 0;
  if (is_bf16 && (V % 8 != 0 || ld % 8 != 0)) return -1;
  if (!is_bf16 && (ld % 4 != 0)) return -1;
  if (!docqa_aligned16(logits)) return -1;
  dim3 g1(splits, rows);
  if (is_bf16) argmax_pass1<true><<<g1, 256, 0, s>>>(logits, V, ld, splits, ws_v, ws_i);
  else argmax_pass1<false><<<g1, 256, 0, s>>>(logits, V, ld, splits, ws_v, ws_i);
  argmax_pass2<<<rows, 64, 0, s>>>(ws_v, ws_i, splits, out);
  DOCQA_CHECK_LAUNCH();
  return 0;
}

int docqa_sample(const float* logits, int rows, int V, int ld, const float* inv_temp,
                 const int* top_k, const float* top_p, const float* u, int64_t* out,
                 hipStream_t s) {
  if (rows == 0) return 0;
  sample_kernel<<<rows, 256, 0, s>>>(logits, V, ld, inv_temp, top_k, top_p, u, out);
  DOCQA_CHECK_LAUNCH();
  return 0;
}

// ---- decode-step state (engine/llm_engine.py:_step_body): one launch each instead of the
// ~15 tiny tensor ops (gather, where, div/mod, casts, copies, adds) a step otherwise
// spends ~60 us of graph time on.
//   slots[i] = valid[i] ? block_tables[i][pos[i] / BS] * BS + pos[i] % BS : -1
__global__ __launch_bounds__(256) void decode_slots_kernel(const int* __restrict__ bt, int maxb,
                                                           const int* __restrict__ pos,
                                                           const int* __restrict__ valid,
                                                           int* __restrict__ slots, int B, int BS) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= B) return;
  const int p = pos[i];
  const int blk = p / BS;
  slots[i] = (valid[i] && blk < maxb) ? bt[(size_t)i * maxb + blk] * BS + (p - blk * BS) : -1;
}

//   out[i] = nxt[i]; tokens[i] = nxt[i]; pos[i] += valid[i]; ctx[i] += valid[i]
__global__ __launch_bounds__(256) void decode_advance_kernel(const int64_t* __restrict__ nxt,
                                                             int64_t* __restrict__ out,
                                                             int* __restrict__ tokens,
                                                             int* __restrict__ pos,
                                                             int* __restrict__ ctx,
                                                             const int* __restrict__ valid, int B) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= B) return;
  const int64_t t = nxt[i];
  const int v = valid[i];
  out[i] = t;
  tokens[i] = (int)t;
  pos[i] += v;
  ctx[i] += v;
}

int docqa_decode_slots(const int* block_tables, int maxb, const int* positions, const int* valid,
                       int* slots, int B, int BS, hipStream_t s) {
  if (B == 0) return 0;
  if (BS <= 0 || maxb <= 0) return -1;
  decode_slots_kernel<<<(B + 255) / 256, 256, 0, s>>>(block_tables, maxb, positions, valid, slots, B, BS);
  DOCQA_CHECK_LAUNCH();
  return 0;
}

int docqa_decode_advance(const int64_t* nxt, int64_t* out, int* tokens, int* positions,
                         int* context_lens, const int* valid, int B, hipStream_t s) {
  if (B == 0) return 0;
  decode_advance_kernel<<<(B + 255) / 256, 256, 0, s>>>(nxt, out, tokens, positions, context_lens, valid, B);
  DOCQA_CHECK_LAUNCH();
  return 0;
}

// token_cls_argmax: the NER token-classification head fused with its argmax
// (SURVEY.md §2.3 "Token-classification head + argmax"; the deid-service's spaCy NER at
// deid-service/anonymizer.py:41-45 is replaced by a BERT token classifier).  logits never
// reach HBM: the [NL, H] head (NL <= 32 label rows, padded) sits in LDS, one 64-wide wave
// owns a token, each lane dots 8 bf16 of the hidden row per step against every label row
// (fp32 accumulate), a reduce-scatter butterfly over the labels, and a wave argmax keeps
// the first maximum (torch.argmax tie rule).  Waves stride over tokens so the head is staged once per block.
template <int NL>
__global__ __launch_bounds__(256) void token_cls_argmax_kernel(
    const uint16_t* __restrict__ h, int ldh, const uint16_t* __restrict__ w,
    const uint16_t* __restrict__ bias, int n_valid, int T, int H, int64_t* __restrict__ out) {
  extern __shared__ uint4 w_lds[];  // [NL][H/8]
  const int H8 = H >> 3;
  const uint4* wg = reinterpret_cast<const uint4*>(w);
  for (int i = threadIdx.x; i < NL * H8; i += blockDim.x) w_lds[i] = wg[i];
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int nwaves = gridDim.x * (blockDim.x >> 6);
  for (int t = blockIdx.x * (blockDim.x >> 6) + wave; t < T; t += nwaves) {
    const uint4* hr = reinterpret_cast<const uint4*>(h + (size_t)t * ldh);
    float acc[NL];
#pragma unroll
    for (int n = 0; n < NL; ++n) acc[n] = 0.f;
    for (int c = lane; c < H8; c += 64) {
      float hf[8];
      unpack8(hr[c], hf);
#pragma unroll
      for (int n = 0; n < NL; ++n) {
        float wf[8];
        unpack8(w_lds[n * H8 + c], wf);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[n] = fmaf(hf[j], wf[j], acc[n]);
      }
    }
    // reduce-scatter butterfly: each xor step halves the label array a lane carries
    // (NL-1 shuffles in total instead of NL full wave_sums), leaving lane `lab`'s label
    // summed over its lane group; the remaining xor steps finish the sum.
    int lab = 0;
#pragma unroll
    for (int st = 0; (NL >> st) > 1; ++st) {
      const int half = NL >> (st + 1);
      const int o = 32 >> st;
      const bool up = (lane & o) != 0;
#pragma unroll
      for (int i = 0; i < half; ++i) {
        const float send = up ? acc[i] : acc[i + half];
        const float keep = up ? acc[i + half] : acc[i];
        acc[i] = keep + __shfl_xor(send, o, 64);
      }
      lab = lab * 2 + (up ? 1 : 0);
    }
#pragma unroll
    for (int o = 32 / NL; o >= 1; o >>= 1) acc[0] += __shfl_xor(acc[0], o, 64);
    float best = lab < n_valid ? acc[0] + bf2f(bias[lab]) : -FLT_MAX;
    int best_i = lab;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {  // wave argmax, lowest label wins ties
      const float ov = __shfl_xor(best, o, 64);
      const int oi = __shfl_xor(best_i, o, 64);
      if (ov > best || (ov == best && oi < best_i)) { best = ov; best_i = oi; }
    }
    if (lane == 0) out[t] = best_i;
  }
}

int docqa_token_cls_argmax(const void* h, int ldh, const void* w, const void* bias, int n_rows,
                           int n_valid, int T, int H, int64_t* out, hipStream_t s) {
  if (T == 0) return 0;
  if (H % 8 != 0 || ldh % 8 != 0 || n_valid < 1 || n_valid > n_rows) return -1;
  if (!docqa_aligned16(h) || !docqa_aligned16(w) || !docqa_aligned16(bias)) return -1;
  int nb = (T + 3) / 4;
  if (nb > 1024) nb = 1024;
  const auto* hp = static_cast<const uint16_t*>(h);
  const auto* wp = static_cast<const uint16_t*>(w);
  const auto* bp = static_cast<const uint16_t*>(bias);
#define TCA(NL)                                                                             \
  do {                                                                                      \
    const size_t lds = (size_t)NL * H * 2;                                                  \
    if (lds > 64 * 1024) return -1;                                                         \
    token_cls_argmax_kernel<NL><<<nb, 256, lds, s>>>(hp, ldh, wp, bp, n_valid, T, H, out); \
  } while (0)
  if (n_rows == 8) TCA(8);
  else if (n_rows == 16) TCA(16);
  else if (n_rows == 32) TCA(32);
  else return -1;
#undef TCA
  DOCQA_CHECK_LAUNCH();
  return 0;
}
