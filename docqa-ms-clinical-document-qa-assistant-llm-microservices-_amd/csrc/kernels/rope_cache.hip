// rope_cache.hip -- fused rotary embedding + paged KV-cache write for the Llama-3
// generator.  One launch per layer replaces three (rope q, rope k, cache scatter):
// it reads the packed QKV projection output once, rotates Q and K in place (the
// prefill attention then reads Q/K/V straight from the packed buffer) and scatters
// the rotated K and the V head into the paged cache
//   k_cache/v_cache : [num_blocks, Hkv, BS, D]  (one (block, head) = BS*D contiguous)
// slot = slot_mapping[token] (block = slot / BS, offset = slot % BS, -1 = padding).
//
// Rotation is Llama's rotate-half form: for i < D/2,
//   x'[i] = x[i]*cos - x[i+D/2]*sin ;  x'[i+D/2] = x[i+D/2]*cos + x[i]*sin
// with cos/sin precomputed in fp32 on the host ([max_pos][D/2 cos | D/2 sin]) so the
// kernel stays memory-bound instead of trig-bound (cdna_hip_programming.md App. B,
// "Element-wise").  Thread mapping: D/8 threads per head, each owning 4 rotation
// pairs (two 8-byte loads); V heads move as one 16-byte chunk per thread.
//
// Reference parity: RoPE lives inside the llama.cpp Mistral served through Ollama
// (llm-qa/main.py:66-69); this is its MI355X-native replacement.
#include "docqa_common.h"

using namespace docqa;

// sum of S fp32 split-K partial slabs at element offset `off`, rounded to bf16 (as the
// unfused projection -> bf16 path would), n = 4 or 8 values.  NS > 0: S == NS known at
// compile time, so every slab load is issued before the first add (one memory latency
// instead of S dependent ones -- the decode consumers are latency-bound at 128 rows);
// NS == 0: runtime S.  Summation order is slab 0, 1, 2, ... either way.
// 4 / 8 slab values at p as float4s: fp32 slabs, or bf16 slabs (mgemm.hip EPI_PARTIAL16)
template <int N>
__device__ __forceinline__ void slab_vals(const float* p, float4* a) {
#pragma unroll
  for (int j = 0; j < N / 4; ++j) a[j] = *reinterpret_cast<const float4*>(p + 4 * j);
}
template <int N>
__device__ __forceinline__ void slab_vals(const uint16_t* p, float4* a) {
  if constexpr (N == 4) {
    const uint2 u = *reinterpret_cast<const uint2*>(p);
    a[0] = float4{__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u), __uint_as_float(u.y << 16),
                  __uint_as_float(u.y & 0xffff0000u)};
  } else {
    const uint4 u = *reinterpret_cast<const uint4*>(p);
    a[0] = float4{__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u), __uint_as_float(u.y << 16),
                  __uint_as_float(u.y & 0xffff0000u)};
    a[1] = float4{__uint_as_float(u.z << 16), __uint_as_float(u.z & 0xffff0000u), __uint_as_float(u.w << 16),
                  __uint_as_float(u.w & 0xffff0000u)};
  }
}

template <int N, int NS, typename PT>
__device__ __forceinline__ void load_partials(const PT* P, int S, size_t slab, size_t off, float* x) {
  float4 a[N / 4];
  if constexpr (NS > 0) {
    float4 p[NS][N / 4];
#pragma unroll
    for (int sl = 0; sl < NS; ++sl) slab_vals<N>(P + sl * slab + off, p[sl]);
#pragma unroll
    for (int j = 0; j < N / 4; ++j) {
      a[j] = p[0][j];
#pragma unroll
      for (int sl = 1; sl < NS; ++sl) {
        a[j].x += p[sl][j].x; a[j].y += p[sl][j].y; a[j].z += p[sl][j].z; a[j].w += p[sl][j].w;
      }
    }
  } else {
    slab_vals<N>(P + off, a);
    for (int sl = 1; sl < S; ++sl) {
      float4 b[N / 4];
      slab_vals<N>(P + sl * slab + off, b);
#pragma unroll
      for (int j = 0; j < N / 4; ++j) {
        a[j].x += b[j].x; a[j].y += b[j].y; a[j].z += b[j].z; a[j].w += b[j].w;
      }
    }
  }
#pragma unroll
  for (int j = 0; j < N / 4; ++j) {
    x[4 * j] = bf2f(f2bf(a[j].x)); x[4 * j + 1] = bf2f(f2bf(a[j].y));
    x[4 * j + 2] = bf2f(f2bf(a[j].z)); x[4 * j + 3] = bf2f(f2bf(a[j].w));
  }
}

// SPLIT: the packed QKV row comes from a split-K decode projection as S fp32 partial slabs
// P[s][t][:] and is written (rotated) into `qkv` -- the combine fused into this pass.
// Grid (T, ceil(heads / heads-per-workgroup)): one head slice per thread and no loop, so
// a 128-token decode batch is 384 workgroups (Llama-3-8B: 48 heads / 16 per workgroup)
// instead of 128 workgroups each walking three passes.
template <bool SPLIT, int NS, typename PT = float>
__global__ __launch_bounds__(256) void rope_cache_kernel(
    uint16_t* __restrict__ qkv, const int* __restrict__ positions,
    const float* __restrict__ cos_sin, const int* __restrict__ slot_mapping,
    uint16_t* __restrict__ k_cache, uint16_t* __restrict__ v_cache, int Hq, int Hkv, int D,
    int row_stride, int BS, const PT* __restrict__ P, int S, size_t slab) {
  const int t = blockIdx.x;
  const int tph = D >> 3;                 // threads per head
  const int heads_per_pass = 256 / tph;
  const int sub = threadIdx.x % tph;
  const int h = blockIdx.y * heads_per_pass + threadIdx.x / tph;
  const int total = Hq + 2 * Hkv;
  if (h >= total) return;
  const int pos = positions[t];
  const int slot = slot_mapping ? slot_mapping[t] : -1;
  const int half = D >> 1;
  uint16_t* hp = qkv + (size_t)t * row_stride + h * D;
  if (h < Hq + Hkv) {
    const int i0 = sub * 4;
    const float* cs = cos_sin + (size_t)pos * D;
    const float4 c = *reinterpret_cast<const float4*>(cs + i0);
    const float4 s = *reinterpret_cast<const float4*>(cs + half + i0);
    float x1[4], x2[4];
    if constexpr (SPLIT) {
      const size_t base = (size_t)t * row_stride + h * D;
      load_partials<4, NS>(P, S, slab, base + i0, x1);
      load_partials<4, NS>(P, S, slab, base + half + i0, x2);
    } else {
      const uint2 a = *reinterpret_cast<const uint2*>(hp + i0);
      const uint2 b = *reinterpret_cast<const uint2*>(hp + half + i0);
      x1[0] = __uint_as_float(a.x << 16); x1[1] = __uint_as_float(a.x & 0xffff0000u);
      x1[2] = __uint_as_float(a.y << 16); x1[3] = __uint_as_float(a.y & 0xffff0000u);
      x2[0] = __uint_as_float(b.x << 16); x2[1] = __uint_as_float(b.x & 0xffff0000u);
      x2[2] = __uint_as_float(b.y << 16); x2[3] = __uint_as_float(b.y & 0xffff0000u);
    }
    const float cc[4] = {c.x, c.y, c.z, c.w}, ss[4] = {s.x, s.y, s.z, s.w};
    float o1[4], o2[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      o1[j] = x1[j] * cc[j] - x2[j] * ss[j];
      o2[j] = x2[j] * cc[j] + x1[j] * ss[j];
    }
    uint2 oa, ob;
    oa.x = pack2(o1[0], o1[1]); oa.y = pack2(o1[2], o1[3]);
    ob.x = pack2(o2[0], o2[1]); ob.y = pack2(o2[2], o2[3]);
    *reinterpret_cast<uint2*>(hp + i0) = oa;
    *reinterpret_cast<uint2*>(hp + half + i0) = ob;
    if (h >= Hq && slot >= 0) {
      const int kh = h - Hq;
      const int blk = slot / BS, off = slot - blk * BS;
      uint16_t* dst = k_cache + (((size_t)blk * Hkv + kh) * BS + off) * D;
      *reinterpret_cast<uint2*>(dst + i0) = oa;
      *reinterpret_cast<uint2*>(dst + half + i0) = ob;
    }
  } else {
    uint4 vv;
    if constexpr (SPLIT) {
      float x8[8];
      load_partials<8, NS>(P, S, slab, (size_t)t * row_stride + h * D + sub * 8, x8);
      vv = pack8(x8);
      *reinterpret_cast<uint4*>(hp + sub * 8) = vv;
    } else {
      if (slot < 0) return;
      vv = *reinterpret_cast<const uint4*>(hp + sub * 8);
    }
    if (slot >= 0) {
      const int vh = h - Hq - Hkv;
      const int blk = slot / BS, off = slot - blk * BS;
      uint16_t* dst = v_cache + (((size_t)blk * Hkv + vh) * BS + off) * D;
      *reinterpret_cast<uint4*>(dst + sub * 8) = vv;
    }
  }
}

static dim3 rope_grid(int T, int Hq, int Hkv, int D) {
  const int hpp = 256 / (D / 8);
  return dim3(T, (Hq + 2 * Hkv + hpp - 1) / hpp);
}

int docqa_rope_cache(void* qkv, const int* positions, const float* cos_sin,
                     const int* slot_mapping, void* k_cache, void* v_cache, int T, int Hq,
                     int Hkv, int D, int row_stride, int BS, hipStream_t s) {
  if (T == 0) return 0;
  if (D % 8 != 0 || (256 % (D / 8)) != 0) return -1;
  rope_cache_kernel<false, 0, float><<<rope_grid(T, Hq, Hkv, D), 256, 0, s>>>(
      (uint16_t*)qkv, positions, cos_sin, slot_mapping, (uint16_t*)k_cache, (uint16_t*)v_cache,
      Hq, Hkv, D, row_stride, BS, nullptr, 0, 0);
  DOCQA_CHECK_LAUNCH();
  return 0;
}

template <typename PT>
static int rope_cache_splitk_any(const PT* P, int S, void* qkv_out, const int* positions, const float* cos_sin,
                                 const int* slot_mapping, void* k_cache, void* v_cache, int T, int Hq, int Hkv,
                                 int D, int row_stride, int BS, hipStream_t s) {
  if (T == 0) return 0;
  if (D % 8 != 0 || (256 % (D / 8)) != 0 || S < 1 || row_stride % 4 != 0) return -1;
  const dim3 grid = rope_grid(T, Hq, Hkv, D);
  const size_t slab = (size_t)T * row_stride;
  uint16_t *q = (uint16_t*)qkv_out, *kc = (uint16_t*)k_cache, *vc = (uint16_t*)v_cache;
#define DOCQA_ROPE_SPLIT(NS_)                                                                      \
  rope_cache_kernel<true, NS_, PT><<<grid, 256, 0, s>>>(q, positions, cos_sin, slot_mapping, kc, vc, \
                                                        Hq, Hkv, D, row_stride, BS, P, S, slab)
  switch (S) {
    case 1: DOCQA_ROPE_SPLIT(1); break;
    case 2: DOCQA_ROPE_SPLIT(2); break;
    case 3: DOCQA_ROPE_SPLIT(3); break;
    case 4: DOCQA_ROPE_SPLIT(4); break;
    case 5: DOCQA_ROPE_SPLIT(5); break;
    case 6: DOCQA_ROPE_SPLIT(6); break;
    case 7: DOCQA_ROPE_SPLIT(7); break;
    case 8: DOCQA_ROPE_SPLIT(8); break;
    default: DOCQA_ROPE_SPLIT(0); break;
  }
#undef DOCQA_ROPE_SPLIT
  DOCQA_CHECK_LAUNCH();
  return 0;
}

// qkv_out [T, row_stride] bf16 <- rope(sum_s P[s]) ; P: [S, T, row_stride] fp32
int docqa_rope_cache_splitk(const float* P, int S, void* qkv_out, const int* positions,
                            const float* cos_sin, const int* slot_mapping, void* k_cache,
                            void* v_cache, int T, int Hq, int Hkv, int D, int row_stride, int BS,
                            hipStream_t s) {
  return rope_cache_splitk_any(P, S, qkv_out, positions, cos_sin, slot_mapping, k_cache, v_cache, T, Hq, Hkv, D,
                               row_stride, BS, s);
}

// the same from bf16 slabs (mgemm.hip EPI_PARTIAL16)
int docqa_rope_cache_splitk16(const void* P, int S, void* qkv_out, const int* positions,
                              const float* cos_sin, const int* slot_mapping, void* k_cache,
                              void* v_cache, int T, int Hq, int Hkv, int D, int row_stride, int BS,
                              hipStream_t s) {
  return rope_cache_splitk_any((const uint16_t*)P, S, qkv_out, positions, cos_sin, slot_mapping, k_cache, v_cache,
                               T, Hq, Hkv, D, row_stride, BS, s);
}

// Token-granular prefix reuse (engine/kv_cache.py TailCache): copy K/V rows [0, m) of a
// source block into the same rows of a destination block, for every layer and both K and
// V, in ONE launch (the per-layer tensor-indexing copies were 64 launches of ~40 us).
// caches: [2 L] device pointers (k_0, v_0, k_1, v_1, ...) to [num_blocks, Hkv, BS, D]
// pools; tab: [n, 3] int32 (src block, dst block, rows m).  Grid (n, 2 L): one workgroup
// per (copy, tensor) moves m rows x Hkv heads, each row D bf16 contiguous, 16 B per lane.
__global__ __launch_bounds__(256) void kv_copy_rows_kernel(const uint64_t* __restrict__ caches,
                                                           const int* __restrict__ tab, int nblocks, int Hkv,
                                                           int BS, int D) {
  const int c = blockIdx.x;
  uint16_t* base = reinterpret_cast<uint16_t*>(caches[blockIdx.y]);
  const int src = tab[3 * c], dst = tab[3 * c + 1], m = tab[3 * c + 2];
  if (src < 0 || src >= nblocks || dst < 0 || dst >= nblocks || m <= 0 || m > BS) return;
  const int cpr = D / 8;                        // 16-B chunks per row
  const int total = Hkv * m * cpr;
  for (int i = threadIdx.x; i < total; i += blockDim.x) {
    const int ch = i % cpr, r = (i / cpr) % m, h = i / (cpr * m);
    const size_t so = (((size_t)src * Hkv + h) * BS + r) * D + ch * 8;
    const size_t dso = (((size_t)dst * Hkv + h) * BS + r) * D + ch * 8;
    *reinterpret_cast<uint4*>(base + dso) = *reinterpret_cast<const uint4*>(base + so);
  }
}

int docqa_kv_copy_rows(const uint64_t* caches, int ntensors, const int* tab, int n, int nblocks, int Hkv, int BS,
                       int D, hipStream_t s) {
  if (n == 0 || ntensors == 0) return 0;
  if (D % 8 != 0 || BS <= 0 || Hkv <= 0 || ntensors > 65535) return -1;
  kv_copy_rows_kernel<<<dim3(n, ntensors), 256, 0, s>>>(caches, tab, nblocks, Hkv, BS, D);
  DOCQA_CHECK_LAUNCH();
  return 0;
}
