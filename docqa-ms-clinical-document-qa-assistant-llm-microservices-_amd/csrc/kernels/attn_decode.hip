// attn_decode.hip -- paged GQA decode attention (one new query token per sequence),
// split-K over the context ("flash-decoding") for the Llama-3 generator.
//
// Cache layout: k_cache/v_cache [num_blocks, Hkv, BS, D] bf16; block_tables [B, maxb].
//
// Kernel 1, grid (max_parts, Hkv, B), 256 threads: one workgroup owns one KV head of one
// sequence over one context slice (adaptive split, below) and serves all G = Hq/Hkv query heads of the
// group, so every K/V byte is read from HBM exactly once per step.  Decode attention is a
// KV-streaming op (~4 FLOP/byte, far below the VALU roof): no MFMA, K/V go straight to
// VGPRs (cdna_hip_programming.md App. B "Attention decode"; the "GEMV / M <= 16" row of
// §5: no LDS round trip), and the whole design is about keeping HBM requests in flight:
//   * a 16-lane group owns one token row (16 lanes x 16 B = one 256-B K row), a wave
//     reads 4 consecutive tokens = 1 KiB contiguous per instruction;
//   * each of the 16 lane groups of the workgroup is an independent stream with its own
//     online-softmax state (m, l, acc[G][8 dims]) -- no barrier inside the token loop;
//   * U=4 tokens per iteration: 4 K rows + 4 V rows (8 x 16-B loads) are issued before
//     any of them is consumed;
//   * the 16 streams merge at the end: 4 lane groups by two xor-shuffles, 4 waves via LDS.
// Output per partition: un-normalised acc + (max, sum) in fp32 workspaces.
// Kernel 2, grid (Hq, B): log-sum-exp merge of the partitions -> bf16 [B, Hq, D].
//
// Graph capture: the split count is a function of (batch, Hkv, max context) only, so a
// captured replay serves every step; the per-sequence slice length is computed on the
// device from the live context length.
//
// Reference parity: decode attention is inside llama.cpp behind Ollama
// (llm-qa/main.py:69, greedy decode loop of RetrievalQA.invoke at llm-qa/main.py:117).
#include "docqa_common.h"
#include "docqa_asm.h"
#include "docqa_cascade.h"
#include "docqa_norm_row.h"
#include <float.h>
#include <stdlib.h>

using namespace docqa;

constexpr int kMinChunk = 64;   // smallest context slice worth a workgroup
// kDecodeGridNote: grids are (KV head, sequence, partition).  Workgroups go to the 8 XCDs
// round-robin by linear id; with partitions fastest, XCD x would receive partition x of
// every sequence and the high partitions are empty for the short contexts of a mixed
// batch (the prefill kernel measured 3.7x from the same reordering).  KV heads fastest
// spreads every sequence over the XCDs, empty partitions are dispatched last.
typedef __attribute__((address_space(3))) i16x4 lds_i16x4;

// KV heads per workgroup of the MFMA decode kernel in the one-partition regime (knob)
static int hpw_knob() {
  static const int v = [] {
    const char* e = getenv("DOCQA_DECODE_HPW");
    return e ? atoi(e) : 1;
  }();
  return v;
}

// ring slots of the MFMA decode kernel (knob): 3 -> 48 KB LDS, 3 workgroups per CU
static int mfma_nsr() {
  static const int v = [] {
    const char* e = getenv("DOCQA_DECODE_NSR");
    return e ? atoi(e) : 4;
  }();
  return v;
}

// MFMA vs VALU decode kernel.  Measured on HBM-resident caches
// (benchmarks/bench_decode_attn.py, profiles/r1_decode_attention_mfma_ab.log): at G = 4 both
// are LDS-DMA-stream bound (~4 TB/s at 320-640 tokens) and the VALU ring kernel is a few %
// ahead; the MFMA kernel wins on long contexts (5.2 vs 4.6 TB/s at 2k tokens) and its
// per-token cost does not grow with G, so it is the default for G >= 8 (Llama-3-70B).
// DOCQA_DECODE_MFMA=1 / 0 forces it on / off.
// VALU ring depth: 3 (3 workgroups/CU, default) or 4 (2 workgroups/CU).  LPT-ordered
// mixed batches, bench_decode_attn.py: B=192 ctx 352 55.4 vs 63.3 us, B=192 ctx 640
// 92.4 vs 102.6, B=128 ctx 352 43.3 vs 45.4 (profiles/r1_decode_ring_nsr.log)
static int ring_nsr() {
  static const int v = [] {
    const char* e = getenv("DOCQA_RING_NSR");
    return e ? atoi(e) : 3;
  }();
  return v == 4 ? 4 : v == 2 ? 2 : 3;
}

static bool mfma_decode_on(int G) {
  static const int v = [] {
    const char* e = getenv("DOCQA_DECODE_MFMA");
    return e ? atoi(e) : -1;
  }();
  return v == 1 || (v < 0 && G >= 8);
}
constexpr float kLog2e = 1.4426950408889634f;

// write-through (agent-scope relaxed = global_store ... sc1) stores and agent-scope loads of
// partials that a last-arriving workgroup of the same launch merges
__device__ __forceinline__ void store4_coh(float* p, const f32x4& v) {
  unsigned long long* q = reinterpret_cast<unsigned long long*>(p);
  __hip_atomic_store(q, (unsigned long long)__float_as_uint(v[0]) | ((unsigned long long)__float_as_uint(v[1]) << 32),
                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(q + 1, (unsigned long long)__float_as_uint(v[2]) | ((unsigned long long)__float_as_uint(v[3]) << 32),
                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void store2_coh(float* p, float a, float b) {
  __hip_atomic_store(reinterpret_cast<unsigned long long*>(p),
                     (unsigned long long)__float_as_uint(a) | ((unsigned long long)__float_as_uint(b) << 32),
                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float4 load2_coh(const float* p) {
  const unsigned long long v =
      __hip_atomic_load(reinterpret_cast<const unsigned long long*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return float4{__uint_as_float((unsigned)v), __uint_as_float((unsigned)(v >> 32)), 0.f, 0.f};
}
template <bool COH>
__device__ __forceinline__ void group_merge_body(const int* __restrict__ mg, const float* __restrict__ ws_acc,
                                                 const float* __restrict__ ws_ml,
                                                 const int* __restrict__ context_lens, int B, int Hkv,
                                                 uint16_t* __restrict__ out, int out_stride, const CascadeIn& ci,
                                                 int kvh, int t);

// Adaptive split: the grid has a fixed number of splits per (sequence, kv head) --
// fixed so a HIP graph captured once serves every step -- and each sequence's context
// is cut into that many equal slices (multiples of 64 tokens), so no workgroup is
// launched for a partition past the end of a short context and long contexts simply get
// longer slices.  The launcher picks the split count from the batch size so that
// B x Hkv x splits fills the 256 CUs (batch 1: many splits; batch 64: few).
__device__ __forceinline__ int split_chunk(int L, int nsplit) {
  int c = (L + nsplit - 1) / nsplit;
  c = (c + kMinChunk - 1) / kMinChunk * kMinChunk;
  return c < kMinChunk ? kMinChunk : c;
}

// Online-softmax attention of one lane group's U token rows (16 lanes x 8 dims each): q.k
// on v_dot2c_f32_bf16 + DPP row reduction, rescale, P.V accumulate in fp32.
template <int G, int U>
__device__ __forceinline__ void attend_rows(const uint4 (&kr)[U], const uint4 (&vr)[U],
                                            const bool (&ok)[U], const bf16x2 (&qv)[G][4],
                                            float qs, float (&m)[G], float (&l)[G],
                                            float (&acc)[G][8]) {
    float s[U][G];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const bf16x2 k0 = __builtin_bit_cast(bf16x2, kr[u].x), k1 = __builtin_bit_cast(bf16x2, kr[u].y);
      const bf16x2 k2 = __builtin_bit_cast(bf16x2, kr[u].z), k3 = __builtin_bit_cast(bf16x2, kr[u].w);
#pragma unroll
      for (int g = 0; g < G; ++g) {
        float d0 = __builtin_amdgcn_fdot2_f32_bf16(k0, qv[g][0], 0.f, false);
        float d1 = __builtin_amdgcn_fdot2_f32_bf16(k2, qv[g][2], 0.f, false);
        d0 = __builtin_amdgcn_fdot2_f32_bf16(k1, qv[g][1], d0, false);
        d1 = __builtin_amdgcn_fdot2_f32_bf16(k3, qv[g][3], d1, false);
        const float d = group_sum<16>(d0 + d1) * qs;
        s[u][g] = ok[u] ? d : -FLT_MAX;
      }
    }
#pragma unroll
    for (int g = 0; g < G; ++g) {
      float mx = m[g];
#pragma unroll
      for (int u = 0; u < U; ++u) mx = fmaxf(mx, s[u][g]);
      const float corr = exp2f(m[g] - mx);
      m[g] = mx;
      l[g] *= corr;
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[g][j] *= corr;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (ok[u]) {
        float vf[8];
        unpack8(vr[u], vf);
#pragma unroll
        for (int g = 0; g < G; ++g) {
          const float p = exp2f(s[u][g] - m[g]);
          l[g] += p;
#pragma unroll
          for (int j = 0; j < 8; ++j) acc[g][j] += p * vf[j];
        }
      }
    }
  }

// Merge the 16 lane-group streams of a workgroup (4 per wave via xor-shuffles, 4 waves
// through LDS) and write the partition result: normalised bf16 output (DIRECT) or the
// un-normalised accumulator + (max, sum) for the merge kernel.
// COH: the partition result is written through to the device-coherent level (agent-scope
// relaxed atomic stores = global_store ... sc1) for a merge inside the same launch
template <int G, int D, bool DIRECT, bool COH = false>
__device__ __forceinline__ void finish_partition(
    float (&m)[G], float (&l)[G], float (&acc)[G][8], float (*s_acc)[G][D], float (*s_m)[G],
    float (*s_l)[G], int tid, int wave, int tg, int chunk, int b, int kvh, int part, int Hkv,
    int max_parts, float* __restrict__ tmp_out, float* __restrict__ tmp_ml,
    uint16_t* __restrict__ out, int out_stride, const CascadeIn& ci) {
  // ---- merge the 4 lane-group streams of the wave (lanes l, l^16, l^32, l^48)
#pragma unroll
  for (int g = 0; g < G; ++g) {
    float M = fmaxf(m[g], __shfl_xor(m[g], 16, 64));
    M = fmaxf(M, __shfl_xor(M, 32, 64));
    const float f = (m[g] == -FLT_MAX) ? 0.f : exp2f(m[g] - M);
    float lv = l[g] * f;
    lv += __shfl_xor(lv, 16, 64);
    lv += __shfl_xor(lv, 32, 64);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float a = acc[g][j] * f;
      a += __shfl_xor(a, 16, 64);
      a += __shfl_xor(a, 32, 64);
      acc[g][j] = a;
    }
    m[g] = M;
    l[g] = lv;
  }
  if (tg == 0) {
#pragma unroll
    for (int g = 0; g < G; ++g) {
#pragma unroll
      for (int j = 0; j < 8; ++j) s_acc[wave][g][chunk * 8 + j] = acc[g][j];
      if (chunk == 0) { s_m[wave][g] = m[g]; s_l[wave][g] = l[g]; }
    }
  }
  __syncthreads();
  // ---- merge the 4 waves, write the partition result
  for (int i = tid; i < G * D; i += 256) {
    const int g = i / D, d = i % D;
    float M = fmaxf(fmaxf(s_m[0][g], s_m[1][g]), fmaxf(s_m[2][g], s_m[3][g]));
    float v = 0.f, lsum = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      const float f = (s_m[w][g] == -FLT_MAX) ? 0.f : exp2f(s_m[w][g] - M);
      v += s_acc[w][g][d] * f;
      lsum += s_l[w][g] * f;
    }
    const int h = kvh * G + g;
    if constexpr (DIRECT) {
      const int np = ci.plen ? cascade_parts(*ci.plen, ci.nchunk) : 0;
      if (np > 0) {   // cascade: fold in the shared-prefix chunk partials
        // every chunk's (max, sum, acc) load is issued before the first is used (indices
        // clamped, extra chunks weighted 0): one memory latency, not 2 x np dependent ones
        const size_t B = gridDim.y, Hq = (size_t)Hkv * G;
        float pm[kCascadeMaxChunks], pl[kCascadeMaxChunks], pa[kCascadeMaxChunks];
#pragma unroll
        for (int c = 0; c < kCascadeMaxChunks; ++c) {
          const size_t r = ((size_t)min(c, np - 1) * B + b) * Hq + h;
          const float2 mlv = *reinterpret_cast<const float2*>(ci.ml + r * 2);
          pm[c] = c < np ? mlv.x : -FLT_MAX;
          pl[c] = mlv.y;
          pa[c] = ci.acc[r * D + d];
        }
        float M2 = M;
#pragma unroll
        for (int c = 0; c < kCascadeMaxChunks; ++c) M2 = fmaxf(M2, pm[c]);
        const float f0 = (M == -FLT_MAX) ? 0.f : exp2f(M - M2);
        v *= f0;
        lsum *= f0;
#pragma unroll
        for (int c = 0; c < kCascadeMaxChunks; ++c) {
          const float f = (pm[c] == -FLT_MAX) ? 0.f : exp2f(pm[c] - M2);
          v += f * pa[c];
          lsum += f * pl[c];
        }
      }
      out[(size_t)b * out_stride + (size_t)h * D + d] = f2bf(lsum > 0.f ? v / lsum : 0.f);
    } else {
      const size_t o = ((size_t)b * (Hkv * G) + h) * max_parts + part;
      if constexpr (COH) {
        __hip_atomic_store(tmp_out + o * D + d, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (d == 0) {
          __hip_atomic_store(tmp_ml + o * 2 + 0, M, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(tmp_ml + o * 2 + 1, lsum, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      } else {
        tmp_out[o * D + d] = v;
        if (d == 0) {
          tmp_ml[o * 2 + 0] = M;
          tmp_ml[o * 2 + 1] = lsum;
        }
      }
    }
  }
}

// Partition merge by the LAST workgroup of a (sequence, KV head) to finish (LAST mode of the
// ring kernel): replaces the paged_decode_reduce launch -- at batch 1 a 6 us kernel on the
// critical path of every layer (profiles/r4_batch1_kernel_stats.txt) -- with one ticket
// atomic and a merge of the G heads by a workgroup that is already resident.
//   * every workgroup writes its partition with write-through stores (finish_partition COH),
//     waits for them, then draws a ticket tick[b Hkv + kvh]; the one drawing np - 1 merges
//     and re-arms the ticket for the next launch (graph replays need no memset);
//   * the merge reads the partitions with agent-scope loads (sc1: past this XCD's L2, so a
//     partition written on another XCD is seen), the (max, sum) pairs through LDS, and the
//     accumulators 8 partitions per round with every load issued before the first use.
// Same arithmetic as paged_decode_reduce (fp32, partitions in index order), so the two
// modes agree bit for bit.
constexpr int kFastMergeParts = 16;

template <int G, int D>
__device__ __forceinline__ bool last_arriver_merge(const float* __restrict__ tmp_out, const float* __restrict__ tmp_ml,
                                                   int* __restrict__ tick, int b, int kvh, int Hkv, int max_parts,
                                                   int Lr, int P, const CascadeIn& ci, uint16_t* __restrict__ out,
                                                   int out_stride) {
  constexpr int MAXP = 64;
  __shared__ int s_last;
  __shared__ float s_w[G][MAXP + kCascadeMaxChunks];
  __shared__ float s_inv[G];
  const int tid = threadIdx.x;
  const int chunk = split_chunk(Lr, max_parts);
  const int np = min(max_parts, (Lr + chunk - 1) / chunk);
  const int nc = ci.plen ? cascade_parts(P, ci.nchunk) : 0;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this workgroup's partition has landed
  __syncthreads();
  if (tid == 0) {
    int* t = tick + (size_t)b * Hkv + kvh;
    const int old = __hip_atomic_fetch_add(t, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = old == np - 1;
    if (s_last) __hip_atomic_store(t, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  if (!s_last) return false;
  const int Hq = Hkv * G;
  const size_t B = gridDim.y;
  if constexpr (G * D <= 512) {
    if (nc == 0 && np <= kFastMergeParts) {
      // up to 16 partitions, no cascade (batch-1 decode at <= 1k tokens): ONE memory round
      // trip -- every (max, sum) pair and accumulator this thread's outputs need is loaded
      // before the first is used; the general path below takes two (pairs into LDS, then
      // the accumulators).  Same fp32 arithmetic in the same partition order.
      constexpr int EPT = (G * D + 255) / 256;
      float pm[EPT][kFastMergeParts], pl[EPT][kFastMergeParts], pa[EPT][kFastMergeParts];
#pragma unroll
      for (int e = 0; e < EPT; ++e) {
        const int i = min(tid + 256 * e, G * D - 1), g = i / D, d = i - g * D, h = kvh * G + g;
        const size_t row = ((size_t)b * Hq + h) * max_parts;
#pragma unroll
        for (int p = 0; p < kFastMergeParts; ++p) {
          const int pp = min(p, np - 1);
          const float4 ml = load2_coh(tmp_ml + (row + pp) * 2);
          pm[e][p] = ml.x;
          pl[e][p] = ml.y;
          pa[e][p] = __hip_atomic_load(tmp_out + (row + pp) * D + d, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      }
#pragma unroll
      for (int e = 0; e < EPT; ++e) {
        const int i = tid + 256 * e;
        if (i >= G * D) break;
        const int g = i / D, d = i - g * D, h = kvh * G + g;
        float M = -FLT_MAX;
#pragma unroll
        for (int p = 0; p < kFastMergeParts; ++p)
          if (p < np) M = fmaxf(M, pm[e][p]);
        float den = 0.f, num = 0.f;
#pragma unroll
        for (int p = 0; p < kFastMergeParts; ++p)
          if (p < np) {
            const float w = exp2f(pm[e][p] - M);
            den += w * pl[e][p];
            num += w * pa[e][p];
          }
        out[(size_t)b * out_stride + (size_t)h * D + d] = f2bf(den > 0.f ? num / den : 0.f);
      }
      return true;
    }
  }
  // (max, sum) of every partition (and cascade chunk) -> LDS
  float* s_pm = &s_w[0][0];                           // reuse: [G][np + nc] maxima first
  __shared__ float s_pl[G][MAXP + kCascadeMaxChunks];
  const int ne = np + nc;
  for (int i = tid; i < G * ne; i += 256) {
    const int g = i / ne, p = i - g * ne, h = kvh * G + g;
    float pm, pl;
    if (p < np) {
      const float* ml = tmp_ml + (((size_t)b * Hq + h) * max_parts + p) * 2;
      pm = __hip_atomic_load(ml, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      pl = __hip_atomic_load(ml + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      const size_t r = ((size_t)(p - np) * B + b) * Hq + h;
      pm = ci.ml[r * 2];
      pl = ci.ml[r * 2 + 1];
    }
    s_pm[g * (MAXP + kCascadeMaxChunks) + p] = pm;
    s_pl[g][p] = pl;
  }
  __syncthreads();
  if (tid < G) {
    const int g = tid;
    float M = -FLT_MAX;
    for (int p = 0; p < ne; ++p) M = fmaxf(M, s_w[g][p]);
    float den = 0.f;
    for (int p = 0; p < ne; ++p) {
      const float pm = s_w[g][p];
      // partitions: exp2(m - M) as paged_decode_reduce; cascade chunks may be empty
      const float w = (p >= np && pm == -FLT_MAX) ? 0.f : exp2f(pm - M);
      s_w[g][p] = w;
      den += w * s_pl[g][p];
    }
    s_inv[g] = den;
  }
  __syncthreads();
  for (int i = tid; i < G * D; i += 256) {
    const int g = i / D, d = i - g * D, h = kvh * G + g;
    const float* src = tmp_out + ((size_t)b * Hq + h) * max_parts * D + d;
    float num = 0.f;
    for (int p0 = 0; p0 < np; p0 += 8) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u)
        v[u] = __hip_atomic_load(src + (size_t)min(p0 + u, np - 1) * D, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (p0 + u < np) num += s_w[g][p0 + u] * v[u];
    }
    for (int c = 0; c < nc; ++c) num += s_w[g][np + c] * ci.acc[(((size_t)c * B + b) * Hq + h) * D + d];
    const float den = s_inv[g];
    out[(size_t)b * out_stride + (size_t)h * D + d] = f2bf(den > 0.f ? num / den : 0.f);
  }
  return true;
}

// DIRECT (one partition per sequence, the batch-64 serving case): the workgroup already
// holds the whole softmax, so it writes the normalised bf16 output itself and the
// partition-merge launch is skipped (one kernel boundary less per layer).
template <int G, int D, int U, bool DIRECT, int OCC = 2>
__global__ __launch_bounds__(256, OCC) void paged_decode_kernel(
    const uint16_t* __restrict__ q, int q_stride, const uint16_t* __restrict__ k_cache,
    const uint16_t* __restrict__ v_cache, const int* __restrict__ block_tables, int maxb,
    const int* __restrict__ context_lens, float* __restrict__ tmp_out,
    float* __restrict__ tmp_ml, int Hkv, int BS, int log2BS, int max_parts, float scale,
    uint16_t* __restrict__ out, int out_stride) {
  static_assert(D == 128, "decode kernel is specialised for head_dim 128");
  const int part = blockIdx.z, kvh = blockIdx.x, b = blockIdx.y;
  const int L = context_lens[b];
  const int slice = split_chunk(L, max_parts);
  const int start = part * slice;
  if (start >= L) {
    if (DIRECT && L <= 0)   // padded slot: defined (zero) output
      for (int i = threadIdx.x; i < G * D; i += 256) out[(size_t)b * out_stride + (size_t)kvh * G * D + i] = 0;
    return;
  }
  const int n = min(L - start, slice);

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int chunk = lane & 15;        // 8-dim chunk of the head
  const int tg = lane >> 4;           // lane group = token stream inside the wave

  __shared__ float s_acc[4][G][D];
  __shared__ float s_m[4][G], s_l[4][G];

  // q stays packed bf16: q.k runs on v_dot2c_f32_bf16 straight from the packed K row
  // (no bf16 -> fp32 unpack of K, half the VALU ops of fp32 FMAs); the softmax scale is
  // applied to the reduced score
  bf16x2 qv[G][4];
  const float qs = scale * kLog2e;
#pragma unroll
  for (int g = 0; g < G; ++g) {
    const uint16_t* qp = q + (size_t)b * q_stride + (size_t)(kvh * G + g) * D;
    const uint4 qq = reinterpret_cast<const uint4*>(qp)[chunk];
    qv[g][0] = __builtin_bit_cast(bf16x2, qq.x);
    qv[g][1] = __builtin_bit_cast(bf16x2, qq.y);
    qv[g][2] = __builtin_bit_cast(bf16x2, qq.z);
    qv[g][3] = __builtin_bit_cast(bf16x2, qq.w);
  }
  const int* bt = block_tables + (size_t)b * maxb;
  const size_t head_off = (size_t)kvh * BS * D + chunk * 8;
  const size_t blk_stride = (size_t)Hkv * BS * D;

  float m[G], l[G], acc[G][8];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    m[g] = -FLT_MAX;
    l[g] = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[g][j] = 0.f;
  }

  // Software pipeline (register double buffer): the K/V rows of step i+1 are in flight
  // while step i's dot products / online softmax / P.V run, so HBM latency is hidden by
  // this wave's own compute instead of only by other waves.
  // Loads are unconditional (tail tokens re-read the slice's last valid row and are
  // masked in compute): a per-element "load or skip" branch makes hipcc wait vmcnt(0)
  // around every load and serialises the stream (guide §5 trap (c)).
  auto load = [&](uint4 (&kr)[U], uint4 (&vr)[U], bool (&ok)[U], int base) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int tok = base + 16 * u;
      ok[u] = tok < n;
      const int t = start + min(tok, n - 1);
      const size_t off = (size_t)bt[t >> log2BS] * blk_stride + head_off +
                         (size_t)(t & (BS - 1)) * D;
      kr[u] = *reinterpret_cast<const uint4*>(k_cache + off);
      vr[u] = *reinterpret_cast<const uint4*>(v_cache + off);
    }
  };
  auto compute = [&](const uint4 (&kr)[U], const uint4 (&vr)[U], const bool (&ok)[U]) {
    attend_rows<G, U>(kr, vr, ok, qv, qs, m, l, acc);
  };

  uint4 kA[U], vA[U], kB[U], vB[U];
  bool okA[U], okB[U];
  int base = wave * 4 + tg;
  if (base < n) load(kA, vA, okA, base);
  while (base < n) {
    const int nb = base + 16 * U;
    if (nb < n) load(kB, vB, okB, nb);
    compute(kA, vA, okA);
    if (nb >= n) break;
    const int nb2 = nb + 16 * U;
    if (nb2 < n) load(kA, vA, okA, nb2);
    compute(kB, vB, okB);
    base = nb2;
  }

  finish_partition<G, D, DIRECT>(m, l, acc, s_acc, s_m, s_l, tid, wave, tg, chunk, b, kvh, part,
                                 Hkv, max_parts, tmp_out, tmp_ml, out, out_stride, CascadeIn{});
}

// LDS-DMA ring variant (BS = 64, D = 128).  The register kernel above is capped by the
// wave-loads a CU can keep in flight (~64 x 1 KB at 2 waves/SIMD, ~17 GB/s per CU at the
// loaded HBM latency).  Here K/V move HBM -> LDS by LDS-DMA (global_load_lds, no VGPR
// cost), 32-token tiles (8 KB K + 8 KB V) through a 4-slot ring with three tiles in
// flight per workgroup, two workgroups per CU; lane groups then read their token rows
// from LDS (ds_read_b128, 1 KB contiguous per wave-instruction: conflict-free) and run the
// same online-softmax math.  Counted vmcnt waits + raw s_barrier as in dgemm.hip.
// FUSED: the step's packed QKV arrives as S fp32 split-K partial slabs of the decode
// projection (FusedQKV); the workgroup sums its G query heads and its KV head, applies
// RoPE (rotate-half partner = lane ^ 8 inside the 16-lane row, one DPP rotate), writes the
// new token's K/V into the paged cache (the workgroup whose slice holds the last token)
// and attends -- replacing the separate rope_cache_splitk launch and the bf16 QKV round
// trip.
struct FusedQKV {
  const float* P;            // [S, B, (Hq + 2 Hkv) D]
  int S;
  const int* positions;      // [B]
  const float* cos_sin;      // [max_pos, D] = [cos(D/2) | sin(D/2)]
  const int* slot_mapping;   // [B], -1: no cache write
  int Hq;
  // bf16 source instead of the slabs: the packed, not yet rotated QKV rows of a library
  // GEMM ([B, q_stride]); P is then null
  const uint16_t* qkv = nullptr;
  int q_stride = 0;
};

// 8 consecutive values of a fused-QKV row at element offset `off`: slab sum (split-K
// projection) or bf16 load (library GEMM output)
__device__ __forceinline__ void fused_row8(const FusedQKV& fz, int b, int W, size_t slab, int off,
                                           float (&x)[8]);

// sum of the S slabs of 8 consecutive values, rounded to bf16 like the unfused path
__device__ __forceinline__ void sum_slabs8(const float* p, int S, size_t slab, float (&x)[8]) {
  float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
  if (S <= 4) {
    // up to 4 slabs (the decode plans' splits): every load issued before the first add --
    // one memory latency instead of S dependent ones; clamped slabs are loaded, not added
    float4 c[3], d[3];
#pragma unroll
    for (int sl = 1; sl < 4; ++sl) {
      const float* q = p + (size_t)min(sl, S - 1) * slab;
      c[sl - 1] = *reinterpret_cast<const float4*>(q);
      d[sl - 1] = *reinterpret_cast<const float4*>(q + 4);
    }
#pragma unroll
    for (int sl = 1; sl < 4; ++sl)
      if (sl < S) {
        a.x += c[sl - 1].x; a.y += c[sl - 1].y; a.z += c[sl - 1].z; a.w += c[sl - 1].w;
        b.x += d[sl - 1].x; b.y += d[sl - 1].y; b.z += d[sl - 1].z; b.w += d[sl - 1].w;
      }
    const float v[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
    for (int j = 0; j < 8; ++j) x[j] = bf2f(f2bf(v[j]));
    return;
  }
  for (int sl = 1; sl < S; ++sl) {
    const float4 c = *reinterpret_cast<const float4*>(p + sl * slab);
    const float4 d = *reinterpret_cast<const float4*>(p + sl * slab + 4);
    a.x += c.x; a.y += c.y; a.z += c.z; a.w += c.w;
    b.x += d.x; b.y += d.y; b.z += d.z; b.w += d.w;
  }
  const float v[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
  for (int j = 0; j < 8; ++j) x[j] = bf2f(f2bf(v[j]));
}

__device__ __forceinline__ void fused_row8(const FusedQKV& fz, int b, int W, size_t slab, int off,
                                           float (&x)[8]) {
  if (fz.P) {
    sum_slabs8(fz.P + (size_t)b * W + off, fz.S, slab, x);
  } else {
    unpack8(*reinterpret_cast<const uint4*>(fz.qkv + (size_t)b * fz.q_stride + off), x);
  }
}

// rotate-half RoPE of one 8-dim chunk (chunk index c of 16, D = 128): partner chunk c ^ 8
// lives 8 lanes away in the same DPP row
__device__ __forceinline__ void rope8(float (&x)[8], int c, const float* cs) {
  float xp[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) xp[j] = row_ror<8>(x[j]);
  const int i0 = (c & 7) * 8;                    // rotation index of dim 0 of this chunk
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float co = cs[i0 + j], si = cs[64 + i0 + j];
    x[j] = c < 8 ? x[j] * co - xp[j] * si : x[j] * co + xp[j] * si;
  }
}

// NSR: ring slots.  4 (64 KB + 8 KB merge scratch: 2 workgroups/CU) or 3 (48 KB with the
// merge scratch aliased onto the drained ring: 3 workgroups/CU -- the same bytes in flight
// per CU spread over more workgroups, so one workgroup's prologue / epilogue overlaps
// the others' streaming and a batch-192 step needs two launch rounds instead of three).
// LAST (split partitions only): the last workgroup of each (sequence, KV head) merges the
// partitions itself (last_arriver_merge; tick: zeroed int32 [B, Hkv]) -- no reduce launch.
template <int G, bool DIRECT, bool FUSED = false, int NSR = 4, bool LAST = false>
__global__ __launch_bounds__(256) void paged_decode_ring_kernel(
    const uint16_t* __restrict__ q, int q_stride, uint16_t* __restrict__ k_cache,
    uint16_t* __restrict__ v_cache, const int* __restrict__ block_tables, int maxb,
    const int* __restrict__ context_lens, float* __restrict__ tmp_out,
    float* __restrict__ tmp_ml, int Hkv, int max_parts, float scale,
    uint16_t* __restrict__ out, int out_stride, FusedQKV fz, CascadeIn ci, int* __restrict__ tick = nullptr) {
  static_assert(!(LAST && DIRECT), "LAST merges split partitions");
  constexpr int D = 128, TT = 32, U = 2;
  static_assert(NSR >= 2 && NSR <= 4, "ring of 2..4 slots");
  constexpr int TILE = TT * D;                   // elements of one K (or V) tile: 8 KB
  constexpr bool ALIAS = NSR <= 3;               // merge scratch on the drained ring
  static_assert(!ALIAS || 4 * G * D * 4 <= NSR * 2 * TILE * 2, "scratch fits the ring");
  __shared__ __attribute__((aligned(16))) uint16_t ring[NSR * 2 * TILE];   // 48 / 64 KB
  __shared__ float s_acc_own[ALIAS ? 1 : 4][ALIAS ? 1 : G][ALIAS ? 1 : D];
  float (*s_acc)[G][D] = ALIAS ? reinterpret_cast<float (*)[G][D]>(ring)
                               : reinterpret_cast<float (*)[G][D]>(&s_acc_own[0][0][0]);
  __shared__ float s_m[4][G], s_l[4][G];
  __shared__ int s_bt[256];                      // block ids of the slice (<= 16k tokens)

  const int part = blockIdx.z, kvh = blockIdx.x, b = ci.order ? ci.order[blockIdx.y] : blockIdx.y;
  const int L = context_lens[b];
  // cascade: keys [0, P) are the shared prefix (attended by the prefix kernel), this
  // kernel covers the sequence's own suffix [P, L); P is a multiple of 64
  const int P = ci.plen ? *ci.plen : 0;
  const int slice = split_chunk(L - P, max_parts);   // multiple of 64
  const int start = P + part * slice;
  if (start >= L) {
    // a row with no keys of its own (a padded decode slot, L = 0) still gets a defined
    // output: zeros, so nothing downstream ever consumes uninitialised memory
    if ((DIRECT || LAST) && L <= P && part == 0)
      for (int i = threadIdx.x; i < G * D; i += 256) out[(size_t)b * out_stride + (size_t)kvh * G * D + i] = 0;
    return;
  }
  const int n = min(L - start, slice);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int chunk = lane & 15, tg = lane >> 4;

  // this slice's block ids -> LDS (ring addressing then needs no vector-memory loads)
  const int nblk = (n + 63) >> 6;
  for (int i = tid; i < nblk; i += 256) s_bt[i] = block_tables[(size_t)b * maxb + (start >> 6) + i];

  bf16x2 qv[G][4];
  const float qs = scale * kLog2e;
  if constexpr (!FUSED) {
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const uint16_t* qp = q + (size_t)b * q_stride + (size_t)(kvh * G + g) * D;
      const uint4 qq = reinterpret_cast<const uint4*>(qp)[chunk];
      asm volatile("" :: "v"(qq.x), "v"(qq.y), "v"(qq.z), "v"(qq.w));   // land q before the ring
      qv[g][0] = __builtin_bit_cast(bf16x2, qq.x);
      qv[g][1] = __builtin_bit_cast(bf16x2, qq.y);
      qv[g][2] = __builtin_bit_cast(bf16x2, qq.z);
      qv[g][3] = __builtin_bit_cast(bf16x2, qq.w);
    }
  }
  __syncthreads();

  float m[G], l[G], acc[G][8];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    m[g] = -FLT_MAX;
    l[g] = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[g][j] = 0.f;
  }

  // FUSED: the step's new token (position L-1) is not read back from the cache -- the
  // workgroup whose slice holds it attends to it from registers -- so the ring can start
  // streaming before the QKV partials are even read
  const bool owns_last = FUSED && (start <= L - 1) && (L - 1 < start + n);
  const int n_ring = owns_last ? n - 1 : n;
  const int ntile = (n_ring + TT - 1) / TT;
  const uint32_t ring_base = lds_u32(ring);
  const size_t head_rows = (size_t)kvh * 64;     // row offset of this head inside a block
  // tile j -> slot j % NSR: 8 KB of K + 8 KB of V = 16 wave-instructions, 4 per wave.
  // Past the last tile the source is clamped (L2 hit into a free slot): every step issues
  // the same number of DMAs, so the counted wait below needs no tail cases.
  auto stage = [&](int j) {
    const int jj = min(j, ntile - 1);
    const int tok0 = jj * TT;                    // start is a multiple of 64
    const size_t row = ((size_t)s_bt[tok0 >> 6] * Hkv) * 64 + head_rows + (tok0 & 63);
    const uint16_t* kp = k_cache + row * D;
    const uint16_t* vp = v_cache + row * D;
    const uint32_t dst = ring_base + (uint32_t)((j % NSR) * 2 * TILE * 2);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int c = i * 4 + wave;                // 1 KB piece of the 8 KB tile
      glds16<true>(kp + c * 512 + lane * 8, dst + c * 1024);
      glds16<true>(vp + c * 512 + lane * 8, dst + TILE * 2 + c * 1024);
    }
  };
  if (ntile > 0) {
    stage(0);
    if constexpr (NSR >= 3) stage(1);
    if constexpr (NSR == 4) stage(2);
  }

  uint4 knew = make_uint4(0, 0, 0, 0), vnew = make_uint4(0, 0, 0, 0);
  if constexpr (FUSED) {
    // q for the G heads of the group and (slice owner) the new K/V: sum of the split-K
    // partial slabs, rounded to bf16, RoPE; the new K/V row also goes to the paged cache
    const int W = (fz.Hq + 2 * Hkv) * D;
    const size_t slab = (size_t)gridDim.y * W;
    const float* cs = fz.cos_sin + (size_t)fz.positions[b] * D;
#pragma unroll
    for (int g = 0; g < G; ++g) {
      float x[8];
      fused_row8(fz, b, W, slab, (kvh * G + g) * D + chunk * 8, x);
      rope8(x, chunk, cs);
      qv[g][0] = __builtin_bit_cast(bf16x2, pack2(x[0], x[1]));
      qv[g][1] = __builtin_bit_cast(bf16x2, pack2(x[2], x[3]));
      qv[g][2] = __builtin_bit_cast(bf16x2, pack2(x[4], x[5]));
      qv[g][3] = __builtin_bit_cast(bf16x2, pack2(x[6], x[7]));
    }
    if (owns_last && wave == 0 && tg == 0) {
      float kx[8], vx[8];
      fused_row8(fz, b, W, slab, (fz.Hq + kvh) * D + chunk * 8, kx);
      rope8(kx, chunk, cs);
      fused_row8(fz, b, W, slab, (fz.Hq + Hkv + kvh) * D + chunk * 8, vx);
      knew = pack8(kx);
      vnew = pack8(vx);
      const int slot = fz.slot_mapping[b];
      if (slot >= 0) {
        const size_t off = (((size_t)(slot >> 6) * Hkv + kvh) * 64 + (slot & 63)) * D + chunk * 8;
        *reinterpret_cast<uint4*>(k_cache + off) = knew;
        *reinterpret_cast<uint4*>(v_cache + off) = vnew;
      }
    }
  }

  for (int i = 0; i < ntile; ++i) {
    wait_vmcnt<4 * (NSR - 2)>();                 // the next NSR-2 tiles (4 DMAs each) may fly
    ring_barrier();                              // tile i visible; slot (i-1) % NSR free
    stage(i + NSR - 1);
    const uint16_t* kt = ring + (i % NSR) * 2 * TILE;
    const uint16_t* vt = kt + TILE;
    uint4 kr[U], vr[U];
    bool ok[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int r = wave * 8 + 4 * u + tg;       // token row of the tile
      ok[u] = i * TT + r < n_ring;
      kr[u] = *reinterpret_cast<const uint4*>(kt + r * D + chunk * 8);
      vr[u] = *reinterpret_cast<const uint4*>(vt + r * D + chunk * 8);
    }
    attend_rows<G, U>(kr, vr, ok, qv, qs, m, l, acc);
  }
  if (owns_last && wave == 0 && tg == 0) {       // the new token, from registers
    const uint4 kr1[1] = {knew}, vr1[1] = {vnew};
    const bool ok1[1] = {true};
    attend_rows<G, 1>(kr1, vr1, ok1, qv, qs, m, l, acc);
  }
  wait_vmcnt<0>();                               // drain the clamped tail DMAs
  if constexpr (ALIAS) __syncthreads();          // every wave done with the ring

  finish_partition<G, D, DIRECT, LAST>(m, l, acc, s_acc, s_m, s_l, tid, wave, tg, chunk, b, kvh, part,
                                       Hkv, max_parts, tmp_out, tmp_ml, out, out_stride, ci);
  if constexpr (LAST)
    last_arriver_merge<G, D>(tmp_out, tmp_ml, tick, b, kvh, Hkv, max_parts, L - P, P, ci, out, out_stride);
}

// ---------------------------------------------------------------------------------------
// MFMA decode attention (GQA, G query heads per KV head, head_dim 128, 64-token blocks).
// The VALU kernels above spend ~10 instructions per (token, head) on 16-lane dot-product
// reductions and per-score exponentials, which leaves them VALU-bound once the context is
// short (profiled: the ring kernel at 63 % VALU-active with 2 waves/SIMD on 340-token
// suffixes).  Here each 32-token K/V tile (same LDS-DMA ring as the ring kernel) feeds:
//   S^T[16 tok x 16 col] = K[16 tok x 128] . Q^T   -- 4 v_mfma_f32_16x16x32_bf16 per 16
//     tokens; the G heads are columns 0..G-1 of the B operand (the rest zero);
//   online softmax on the accumulator: each lane holds 4 tokens of ONE head, a head's 16
//     tokens live on lanes l, l^16, l^32, l^48 (two xor-shuffles per reduction);
//   O^T[dims x 16] += V^T . P^T -- v_mfma_f32_16x16x16_bf16 with P^T taken straight from
//     the S^T accumulator (its layout IS the B operand) and V^T fragments from a
//     ds_read_b64_tr_b16 transposed read of the row-major V tile (cdna_hip_programming.md
//     T10; XOR-swizzled image (b) so the reads are conflict-free).
// Every wave computes S for the whole tile (4 x cheaper than any cross-wave softmax merge)
// and owns 32 of the 128 output dims, so the epilogue needs no LDS reduction at all.
// K tiles are swizzled for the 16-lane ds_read_b128 row reads (slot = chunk ^ (row & 15)).
__device__ __forceinline__ int vswz(int t) { return ((t & 3) << 2) | ((t >> 2) & 3); }

template <int G, bool DIRECT, int HPW = 1, int NSR = 4>
__global__ __launch_bounds__(256) void paged_decode_mfma_kernel(
    const uint16_t* __restrict__ q, int q_stride, const uint16_t* __restrict__ k_cache,
    const uint16_t* __restrict__ v_cache, const int* __restrict__ block_tables, int maxb,
    const int* __restrict__ context_lens, float* __restrict__ tmp_out,
    float* __restrict__ tmp_ml, int Hkv, int max_parts, float scale,
    uint16_t* __restrict__ out, int out_stride, CascadeIn ci) {
  static_assert(G <= 16, "heads are MFMA columns");
  constexpr int D = 128, TT = 32;
  static_assert(NSR == 3 || NSR == 4, "ring of 3 (48 KB: 3 workgroups/CU) or 4 slots");
  constexpr int TILE = TT * D;                   // elements of one K (or V) tile: 8 KB
  __shared__ __attribute__((aligned(16))) uint16_t ring[NSR * 2 * TILE];   // 48 / 64 KB
  __shared__ int s_bt[256];

  // HPW KV heads per workgroup, one after the other through the same ring (the K/V tile
  // stream runs on across the head boundary): 1/HPW of the workgroups -- one launch round
  // at batch 128 -- and the next head's ring fill overlaps the current head's tail.
  const int part = blockIdx.z, kvh0 = blockIdx.x * HPW, b = ci.order ? ci.order[blockIdx.y] : blockIdx.y;
  const int L = context_lens[b];
  const int P = ci.plen ? *ci.plen : 0;
  const int slice = split_chunk(L - P, max_parts);
  const int start = P + part * slice;
  if (start >= L) {
    if (DIRECT && L <= P)
      for (int i = threadIdx.x; i < HPW * G * D; i += 256) out[(size_t)b * out_stride + (size_t)kvh0 * G * D + i] = 0;
    return;
  }
  const int n = min(L - start, slice);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int hl = lane & 15, lg = lane >> 4;      // MFMA column (head) / lane group

  const int nblk = (n + 63) >> 6;
  for (int i = tid; i < nblk; i += 256) s_bt[i] = block_tables[(size_t)b * maxb + (start >> 6) + i];

  // Q^T fragments (B operand of S^T = K Q^T): lane holds Q[head hl][32 ks + 8 lg + j]
  bf16x8 qf[HPW][4];
#pragma unroll
  for (int e = 0; e < HPW; ++e) {
    const uint16_t* qp = q + (size_t)b * q_stride + (size_t)((kvh0 + e) * G + (hl < G ? hl : 0)) * D + lg * 8;
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      uint4 v = hl < G ? *reinterpret_cast<const uint4*>(qp + ks * 32) : make_uint4(0, 0, 0, 0);
      qf[e][ks] = __builtin_bit_cast(bf16x8, v);
    }
  }
  __syncthreads();

  const float qs = scale * kLog2e;
  const int ntile = (n + TT - 1) / TT;           // tiles per head
  const int ntot = HPW * ntile;                  // the workgroup's tile stream
  const uint32_t ring_base = lds_u32(ring);
  const int prow = lane >> 4, pslot = lane & 15;  // DMA piece geometry: 4 rows x 16 slots
  auto stage = [&](int j) {
    const int jj = min(j, ntot - 1);
    const int e = HPW == 1 ? 0 : jj / ntile;
    const int tok0 = (jj - e * ntile) * TT;
    const size_t row0 = ((size_t)s_bt[tok0 >> 6] * Hkv) * 64 + (size_t)(kvh0 + e) * 64 + (tok0 & 63);
    const uint16_t* kp = k_cache + row0 * D;
    const uint16_t* vp = v_cache + row0 * D;
    const uint32_t dst = ring_base + (uint32_t)((j % NSR) * 2 * TILE * 2);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int c = i * 4 + wave;                // 1 KB piece = tile rows 4c .. 4c+3
      const int t = 4 * c + prow;
      glds16<true>(kp + t * D + ((pslot ^ (t & 15)) << 3), dst + c * 1024);
      glds16<true>(vp + t * D + ((pslot ^ vswz(t)) << 3), dst + TILE * 2 + c * 1024);
    }
  };

  // epilogue of one head: lane holds O^T[dim 16 dt + 4 lg + r][head hl], dt = 2 wave + dd
  auto finish = [&](int e, float m, float l, const f32x4 (&acc)[2]) {
    if (hl >= G) return;
    const int h = (kvh0 + e) * G + hl;
    if constexpr (DIRECT) {
      float den = l;
      float o[2][4];
#pragma unroll
      for (int dd = 0; dd < 2; ++dd)
#pragma unroll
        for (int r = 0; r < 4; ++r) o[dd][r] = acc[dd][r];
      const int np = ci.plen ? cascade_parts(P, ci.nchunk) : 0;
      if (np > 0) {   // cascade: fold in the shared-prefix chunk partials
        // (max, sum) of every chunk first (loads issued together), then the accumulators
        // in groups of 4 chunks: bounded registers, 8 loads in flight per group
        const size_t B = gridDim.y, Hq = (size_t)Hkv * G;
        float pm[kCascadeMaxChunks], pl[kCascadeMaxChunks];
#pragma unroll
        for (int c = 0; c < kCascadeMaxChunks; ++c) {
          const size_t r = ((size_t)min(c, np - 1) * B + b) * Hq + h;
          const float2 mlv = *reinterpret_cast<const float2*>(ci.ml + r * 2);
          pm[c] = c < np ? mlv.x : -FLT_MAX;
          pl[c] = mlv.y;
        }
        float M2 = m;
#pragma unroll
        for (int c = 0; c < kCascadeMaxChunks; ++c) M2 = fmaxf(M2, pm[c]);
        const float f0 = exp2f(m - M2);
        den = l * f0;
#pragma unroll
        for (int dd = 0; dd < 2; ++dd)
#pragma unroll
          for (int r = 0; r < 4; ++r) o[dd][r] *= f0;
        for (int c0 = 0; c0 < np; c0 += 4) {
          f32x4 pa[4][2];
#pragma unroll
          for (int cc = 0; cc < 4; ++cc) {
            const size_t r = ((size_t)min(c0 + cc, np - 1) * B + b) * Hq + h;
#pragma unroll
            for (int dd = 0; dd < 2; ++dd)
              pa[cc][dd] = *reinterpret_cast<const f32x4*>(ci.acc + r * D + 16 * (2 * wave + dd) + 4 * lg);
          }
#pragma unroll
          for (int cc = 0; cc < 4; ++cc) {
            float pmc = -FLT_MAX, plc = 0.f;
#pragma unroll
            for (int c = 0; c < kCascadeMaxChunks; ++c)
              if (c == c0 + cc) { pmc = pm[c]; plc = pl[c]; }
            const float f = pmc == -FLT_MAX ? 0.f : exp2f(pmc - M2);
            den += f * plc;
#pragma unroll
            for (int dd = 0; dd < 2; ++dd)
#pragma unroll
              for (int r = 0; r < 4; ++r) o[dd][r] += f * pa[cc][dd][r];
          }
        }
      }
      const float inv = den > 0.f ? 1.f / den : 0.f;
      uint16_t* op = out + (size_t)b * out_stride + (size_t)h * D;
#pragma unroll
      for (int dd = 0; dd < 2; ++dd) {
        uint2 v;
        v.x = pack2(o[dd][0] * inv, o[dd][1] * inv);
        v.y = pack2(o[dd][2] * inv, o[dd][3] * inv);
        *reinterpret_cast<uint2*>(op + 16 * (2 * wave + dd) + 4 * lg) = v;
      }
    } else {
      const size_t o = ((size_t)b * (Hkv * G) + h) * max_parts + part;
#pragma unroll
      for (int dd = 0; dd < 2; ++dd)
        *reinterpret_cast<f32x4*>(tmp_out + o * D + 16 * (2 * wave + dd) + 4 * lg) = acc[dd];
      if (wave == 0 && lg == 0) *reinterpret_cast<float2*>(tmp_ml + o * 2) = make_float2(m, l);
    }
  };

  if (ntot > 0) {
    stage(0);
    stage(1);
    if constexpr (NSR == 4) stage(2);
  }
  float m = -FLT_MAX, l = 0.f;
  f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
  for (int jt = 0; jt < ntot; ++jt) {
    const int e = HPW == 1 ? 0 : jt / ntile;     // head of this tile
    const int i = jt - e * ntile;                // tile within the head
    wait_vmcnt<4 * (NSR - 2)>();                 // the next NSR-2 tiles (4 DMAs each) may fly
    ring_barrier();                              // tile jt visible; slot (jt-1) % NSR free
    stage(jt + NSR - 1);
    const uint16_t* kt = ring + (jt % NSR) * 2 * TILE;
    const uint16_t* vt = kt + TILE;
    // ---- S^T for the two 16-token halves
    f32x4 x[2];
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      x[c] = f32x4{0.f, 0.f, 0.f, 0.f};
      const int t = 16 * c + hl;
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        const bf16x8 a = *reinterpret_cast<const bf16x8*>(kt + t * D + (((4 * ks + lg) ^ (t & 15)) << 3));
        x[c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, qf[e][ks], x[c], 0, 0, 0);
      }
    }
    // ---- online softmax: lane = 4 tokens (16c + 4 lg + r) of head hl
    float mx = -FLT_MAX;
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int tok = i * TT + 16 * c + 4 * lg + r;
        const float v = tok < n ? x[c][r] * qs : -FLT_MAX;
        x[c][r] = v;
        mx = fmaxf(mx, v);
      }
    mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    const float m_new = fmaxf(m, mx);            // a tile always holds >= 1 live token
    const float alpha = exp2f(m - m_new);
    float ps = 0.f;
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float p = x[c][r] == -FLT_MAX ? 0.f : exp2f(x[c][r] - m_new);
        x[c][r] = p;
        ps += p;
      }
    ps += __shfl_xor(ps, 16, 64);
    ps += __shfl_xor(ps, 32, 64);
    l = l * alpha + ps;
    m = m_new;
#pragma unroll
    for (int dd = 0; dd < 2; ++dd) acc[dd] *= alpha;
    // ---- O^T += V^T P^T (this wave's 32 dims)
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      i16x4 pb;
#pragma unroll
      for (int r = 0; r < 4; ++r) pb[r] = (short)f2bf(x[c][r]);
      const int row = 16 * c + 4 * lg + (hl >> 2), pp = hl & 3;
#pragma unroll
      for (int dd = 0; dd < 2; ++dd) {
        const int ch = 2 * (2 * wave + dd) + (pp >> 1);
        const uint16_t* va = vt + row * D + ((ch ^ vswz(row)) << 3) + 4 * (pp & 1);
        const i16x4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4*)va);
        acc[dd] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a, pb, acc[dd], 0, 0, 0);
      }
    }
    if (i == ntile - 1) {                        // head e done: write it, start the next
      finish(e, m, l, acc);
      m = -FLT_MAX;
      l = 0.f;
      acc[0] = f32x4{0.f, 0.f, 0.f, 0.f};
      acc[1] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
  }
  wait_vmcnt<0>();                               // drain the clamped tail DMAs
}

// ---------------------------------------------------------------------------------------
// Grouped decode attention over prefix-cache-shared KV blocks (Llama-3 GQA, G = 4).
// In a RAG batch many rows retrieved the same chunks, and the prefix cache maps identical
// prompt prefixes to the SAME physical KV blocks (a trie of blocks beyond the template
// prefix that cascade attends once).  The per-row kernels re-read such a block once per
// row.  Here a workgroup serves a GROUP of up to 4 rows (groups[4 g .. 4 g + 3], -1 = none:
// the host packs rows with common block prefixes together) for one KV head: the 16 MFMA columns
// are the 4 rows x 4 query heads, so a block shared by k rows of the group is streamed
// once and scored against all their queries in the same MFMAs (the per-row MFMA kernel
// leaves 12 of the 16 columns empty).  Blocks of only some rows are processed with the
// other rows' columns masked; every column keeps its own online softmax, so the result
// is exactly the per-row attention.  The tile list (block, half, row mask) is built in
// LDS by wave 0 -- one lane per block position, a wave prefix sum for the offsets -- and
// then streamed through the same LDS-DMA ring as the MFMA kernel.  Keys [P, L) per row
// (P: the cascade prefix, attended by the prefix kernel and merged here).
constexpr int kGroupMaxPos = 64;     // block positions beyond the cascade prefix (4096 tokens)
// Block-table WIDTH the grouped kernels accept (a table sized for an 8192-token MAX_CONTEXT
// is 128 wide); every ROW must still end within kGroupMaxPos positions of its window start,
// which the caller guarantees (LLMEngine.groups_fit: rows of <= 64 blocks by the end of
// their decode) -- positions past the window would not be attended
constexpr int kGroupMaxTable = 256;

// Diagnostic timeline of the group kernel (off unless docqa_set_decode_trace set a buffer):
// per workgroup 8 int64 -- entry, tile list + Q ready, first tile landed, loop end, exit
// (wall_clock64 ticks, 100 MHz), tiles streamed, HW_ID, XCC_ID.  One scalar load of a null
// pointer per workgroup when off.
__device__ long long* g_group_trace = nullptr;

// Epilogue of one grouped-decode work item (paged_decode_group_kernel, paged_decode_group_wave_
// kernel): lane holds O^T[dim 16 dt + 4 lg + r][column hl], dt = 2 wave + dd, with the
// column's running (m, l).  SPLIT items with a partial slot store it (write-through when the
// launch merges by ticket, the last arriver then merging the group); otherwise the column's
// row is normalised -- folding the cascade-prefix partials when a prefix kernel ran -- and
// stored as bf16.
template <bool SPLIT, int NDT = 2>
__device__ __forceinline__ void group_item_finish(float m, float l, const f32x4 (&acc)[NDT], int part, int crow, int cL,
                                                  int hl, int lg, int wave, int tid, const int* __restrict__ gp,
                                                  const int* __restrict__ merges, int* __restrict__ tick,
                                                  float* __restrict__ ws_acc, float* __restrict__ ws_ml,
                                                  const CascadeIn& ci, const int* __restrict__ context_lens, int B,
                                                  int Hkv, uint16_t* __restrict__ out, int out_stride, int kvh,
                                                  int P) {
  constexpr int G = 4, D = 128;
  if constexpr (SPLIT) {
    if (part >= 0) {   // one partial of a split group: (m, l) + un-normalised O^T
      const size_t cidx = ((size_t)part * Hkv + kvh) * 16 + hl;
      if (crow >= 0) {
        if (tick) {    // merged inside this launch: write-through (sc1) for the last arriver
#pragma unroll
          for (int dd = 0; dd < NDT; ++dd) store4_coh(ws_acc + cidx * D + 16 * (NDT * wave + dd) + 4 * lg, acc[dd]);
          if (wave == 0 && lg == 0) store2_coh(ws_ml + cidx * 2, m, l);
        } else {
#pragma unroll
          for (int dd = 0; dd < NDT; ++dd)
            *reinterpret_cast<f32x4*>(ws_acc + cidx * D + 16 * (NDT * wave + dd) + 4 * lg) = acc[dd];
          if (wave == 0 && lg == 0) *reinterpret_cast<float2*>(ws_ml + cidx * 2) = make_float2(m, l);
        }
      }
      if (tick) {
        // last-arriver merge (no group_split_merge launch): the item drawing the group's
        // last ticket folds its partials and the cascade-prefix chunks, and re-arms it
        __shared__ int s_last;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        const int mi = gp[7];
        if (tid == 0) {
          int* t = tick + (size_t)mi * Hkv + kvh;
          const int old = __hip_atomic_fetch_add(t, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          s_last = old == merges[8 * mi + 5] - 1;
          if (s_last) __hip_atomic_store(t, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        __syncthreads();
        if (s_last)   // thread = (column, 8 dims): 256 of them over the workgroup's 512 / NDT threads
          for (int t = tid; t < 256; t += 512 / NDT)
            group_merge_body<true>(merges + 8 * mi, ws_acc, ws_ml, context_lens, B, Hkv, out, out_stride, ci, kvh, t);
      }
      return;
    }
  }
  if (crow < 0) return;
  const int h = kvh * G + (hl & 3);
  uint16_t* op = out + (size_t)crow * out_stride + (size_t)h * D;
  if (cL <= P) {                                 // a padded decode slot: defined zeros
#pragma unroll
    for (int dd = 0; dd < NDT; ++dd) *reinterpret_cast<uint2*>(op + 16 * (NDT * wave + dd) + 4 * lg) = make_uint2(0, 0);
    return;
  }
  float den = l;
  float o[NDT][4];
#pragma unroll
  for (int dd = 0; dd < NDT; ++dd)
#pragma unroll
    for (int r = 0; r < 4; ++r) o[dd][r] = acc[dd][r];
  const int np = ci.plen ? cascade_parts(P, ci.nchunk) : 0;
  if (np > 0) {   // cascade: fold in the shared-prefix chunk partials of this column's row
    const size_t Hq = (size_t)Hkv * G;
    float pm[kCascadeMaxChunks], pl[kCascadeMaxChunks];
#pragma unroll
    for (int c = 0; c < kCascadeMaxChunks; ++c) {
      const size_t r = ((size_t)min(c, np - 1) * B + crow) * Hq + h;
      const float2 mlv = *reinterpret_cast<const float2*>(ci.ml + r * 2);
      pm[c] = c < np ? mlv.x : -FLT_MAX;
      pl[c] = mlv.y;
    }
    float M2 = m;
#pragma unroll
    for (int c = 0; c < kCascadeMaxChunks; ++c) M2 = fmaxf(M2, pm[c]);
    const float f0 = m == -FLT_MAX ? 0.f : exp2f(m - M2);
    den = l * f0;
#pragma unroll
    for (int dd = 0; dd < NDT; ++dd)
#pragma unroll
      for (int r = 0; r < 4; ++r) o[dd][r] *= f0;
    for (int c0 = 0; c0 < np; c0 += 4) {
      f32x4 pa[4][NDT];
#pragma unroll
      for (int cc = 0; cc < 4; ++cc) {
        const size_t r = ((size_t)min(c0 + cc, np - 1) * B + crow) * Hq + h;
#pragma unroll
        for (int dd = 0; dd < NDT; ++dd)
          pa[cc][dd] = *reinterpret_cast<const f32x4*>(ci.acc + r * D + 16 * (NDT * wave + dd) + 4 * lg);
      }
#pragma unroll
      for (int cc = 0; cc < 4; ++cc) {
        float pmc = -FLT_MAX, plc = 0.f;
#pragma unroll
        for (int c = 0; c < kCascadeMaxChunks; ++c)
          if (c == c0 + cc) { pmc = pm[c]; plc = pl[c]; }
        const float f = pmc == -FLT_MAX ? 0.f : exp2f(pmc - M2);
        den += f * plc;
#pragma unroll
        for (int dd = 0; dd < NDT; ++dd)
#pragma unroll
          for (int r = 0; r < 4; ++r) o[dd][r] += f * pa[cc][dd][r];
      }
    }
  }
  const float inv = den > 0.f ? 1.f / den : 0.f;
#pragma unroll
  for (int dd = 0; dd < NDT; ++dd) {
    uint2 v;
    v.x = pack2(o[dd][0] * inv, o[dd][1] * inv);
    v.y = pack2(o[dd][2] * inv, o[dd][3] * inv);
    *reinterpret_cast<uint2*>(op + 16 * (NDT * wave + dd) + 4 * lg) = v;
  }
}

// SPLIT: `groups` is a work-item list [cap, 8] = (4 row ids, first block position, end
// block position, partial slot or -1, 0): a long group's block positions are split over
// several items (workgroups), each writing an un-normalised partial (m, l, O) for its 16
// columns to ws_ml / ws_acc[slot] that group_split_merge_kernel combines; an item of an
// unsplit group (slot -1) finishes as the plain kernel does.
// FUSE (split plans from block 0, no prefix kernel): the step's packed QKV arrives as the
// projection's fp32 split-K slabs (FusedQKV, q null) -- each workgroup sums and rotates the
// query rows it needs (RoPE partner chunk c ^ 8 is the same lane's ks ^ 2 fragment), and the
// item whose block range holds a row's new token writes that token's rotated K and V into
// the paged cache before any tile is staged: the rope_cache_splitk launch and the bf16 QKV
// round trip disappear.  Same arithmetic as rope_cache_splitk (bf16-rounded slab sums).
template <int NSR = 3, bool SPLIT = false, bool FUSE = false>
__global__ __launch_bounds__(256) void paged_decode_group_kernel(
    const uint16_t* __restrict__ q, int q_stride, const uint16_t* __restrict__ k_cache,
    const uint16_t* __restrict__ v_cache, const int* __restrict__ block_tables, int maxb,
    const int* __restrict__ context_lens, int B, int Hkv, float scale,
    uint16_t* __restrict__ out, int out_stride, const int* __restrict__ groups, CascadeIn ci,
    float* __restrict__ ws_acc = nullptr, float* __restrict__ ws_ml = nullptr,
    const int* __restrict__ merges = nullptr, int* __restrict__ tick = nullptr, FusedQKV fz = FusedQKV{}) {
  constexpr int G = 4, R = 4, D = 128, TT = 32, MAXT = kGroupMaxPos * 8;
  constexpr int TILE = TT * D;                   // elements of one K (or V) tile: 8 KB
  __shared__ __attribute__((aligned(16))) uint16_t ring[NSR * 2 * TILE];
  __shared__ int2 s_tl[MAXT];                    // (block id, pos << 8 | half << 4 | row mask)
  __shared__ int s_nt;

  const int kvh = blockIdx.x, grp = blockIdx.y;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int hl = lane & 15, lg = lane >> 4;      // MFMA column (row slot x head) / lane group
  long long* trace = g_group_trace;
  long long tr0 = 0, tr1 = 0, tr2 = 0, tr3 = 0;
  if (trace && tid == 0) tr0 = wall_clock64();
  const int P = ci.plen ? *ci.plen : 0;          // multiple of 64
  const int* gp = groups + (SPLIT ? 8 : R) * grp;
  int rows[R], Ls[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int row = gp[r];
    rows[r] = row >= 0 && row < B ? row : -1;
    Ls[r] = rows[r] >= 0 ? context_lens[rows[r]] : 0;
  }
  int lo = 0, hi = maxb, part = -1;
  if constexpr (SPLIT) {
    if (rows[0] < 0 && rows[1] < 0 && rows[2] < 0 && rows[3] < 0) return;   // unused item
    lo = gp[4];
    hi = min(gp[5], maxb);
    part = gp[6];
  }
  const int Wq = (fz.Hq + 2 * Hkv) * D;          // FUSE: packed QKV row width
  const size_t fslab = (size_t)B * Wq;            // FUSE: slab stride
  if constexpr (FUSE) {
    // new tokens first: wave 0 the rotated K, wave 1 the V of the group's rows whose last
    // position falls in this item's block range (lane = row slot x 16 + 8-dim chunk)
    if (wave < 2) {
      const int rs = lane >> 4, c = lane & 15;
      const int row = rows[rs], L = Ls[rs];
      const bool mine = row >= 0 && L > 0 && ((L - 1) >> 6) >= lo && ((L - 1) >> 6) < hi;
      const float* src = fz.P + (size_t)max(row, 0) * Wq + (size_t)(fz.Hq + (wave ? Hkv : 0) + kvh) * D + c * 8;
      float x[8];
      sum_slabs8(src, fz.S, fslab, x);
      if (wave == 0) rope8(x, c, fz.cos_sin + (size_t)(row >= 0 ? fz.positions[row] : 0) * D);
      const int slot = row >= 0 ? fz.slot_mapping[row] : -1;
      if (mine && slot >= 0) {
        uint16_t* dst = const_cast<uint16_t*>(wave ? v_cache : k_cache) +
                        (((size_t)(slot >> 6) * Hkv + kvh) * 64 + (slot & 63)) * D + c * 8;
        *reinterpret_cast<uint4*>(dst) = pack8(x);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // landed before any tile is staged
    }
  }

  // ---- tile list: lane j of wave 0 owns block position max(P/64, lo) + j
  if (wave == 0) {
    const int pos = max(P >> 6, lo) + lane;
    int ids[R];
    bool alive[R];
    // the table entries are loaded on the row id alone (in bounds: pos < hi <= maxb), not
    // behind the context length: both loads fly together, one dependent latency fewer
    // before the first tile's DMA
#pragma unroll
    for (int r = 0; r < R; ++r) ids[r] = rows[r] >= 0 && pos < hi ? block_tables[(size_t)rows[r] * maxb + pos] : -1;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      alive[r] = pos < hi && 64 * pos < Ls[r];
      ids[r] = alive[r] ? ids[r] : -1;
    }
    int2 ent[2 * R];
    int cnt = 0;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      bool first = alive[r];
#pragma unroll
      for (int r2 = 0; r2 < r; ++r2) first = first && !(alive[r2] && ids[r2] == ids[r]);
      if (first) {
        int mask = 0, two = 0;
#pragma unroll
        for (int r2 = 0; r2 < R; ++r2)
          if (alive[r2] && ids[r2] == ids[r]) { mask |= 1 << r2; two |= Ls[r2] > 64 * pos + 32; }
#pragma unroll
        for (int h = 0; h < 2; ++h)
          if (h == 0 || two) ent[cnt++] = make_int2(ids[r], (pos << 8) | (h << 4) | mask);
      }
    }
    // exclusive prefix sum of the per-lane counts (tiles stay in position order)
    int off = cnt;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int v = __shfl_up(off, o, 64);
      if (lane >= o) off += v;
    }
    const int total = __shfl(off, 63, 64);
    off -= cnt;
    for (int e = 0; e < cnt; ++e) s_tl[off + e] = ent[e];
    if (lane == 0) s_nt = total;
  }
  // Q^T fragments: column hl = row slot hl / 4, head hl % 4
  const int crow = rows[hl >> 2], cL = Ls[hl >> 2], cbit = 1 << (hl >> 2);
  bf16x8 qf[4];
  if constexpr (FUSE) {
    // fragment ks holds dims 8 (4 ks + lg) ..: ks and ks + 2 are a rotate-half pair
    const float* qb = fz.P + (size_t)max(crow, 0) * Wq + (size_t)(kvh * G + (hl & 3)) * D + lg * 8;
    const float* cs = fz.cos_sin + (size_t)(crow >= 0 ? fz.positions[crow] : 0) * D;
#pragma unroll
    for (int pr = 0; pr < 2; ++pr) {
      float x1[8], x2[8], o1[8], o2[8];
      sum_slabs8(qb + pr * 32, fz.S, fslab, x1);
      sum_slabs8(qb + (pr + 2) * 32, fz.S, fslab, x2);
      const int i0 = (4 * pr + lg) * 8;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float co = cs[i0 + j], si = cs[64 + i0 + j];
        o1[j] = x1[j] * co - x2[j] * si;
        o2[j] = x2[j] * co + x1[j] * si;
      }
      const uint4 a = crow >= 0 ? pack8(o1) : make_uint4(0, 0, 0, 0);
      const uint4 b = crow >= 0 ? pack8(o2) : make_uint4(0, 0, 0, 0);
      qf[pr] = __builtin_bit_cast(bf16x8, a);
      qf[pr + 2] = __builtin_bit_cast(bf16x8, b);
    }
  } else {
    const uint16_t* qp = q + (size_t)max(crow, 0) * q_stride + (size_t)(kvh * G + (hl & 3)) * D + lg * 8;
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const uint4 v = crow >= 0 ? *reinterpret_cast<const uint4*>(qp + ks * 32) : make_uint4(0, 0, 0, 0);
      qf[ks] = __builtin_bit_cast(bf16x8, v);
    }
  }
  __syncthreads();
  const int nt = s_nt;
  if (trace && tid == 0) tr1 = wall_clock64();
  auto trace_out = [&]() {
    if (trace && tid == 0) {
      long long* t = trace + ((size_t)blockIdx.y * gridDim.x + blockIdx.x) * 8;
      t[0] = tr0; t[1] = tr1; t[2] = tr2; t[3] = tr3; t[4] = wall_clock64(); t[5] = nt;
      t[6] = __builtin_amdgcn_s_getreg((31 << 11) | 4);
      t[7] = __builtin_amdgcn_s_getreg(20 | (3 << 11)) & 15;
    }
  };

  const float qs = scale * kLog2e;
  const uint32_t ring_base = lds_u32(ring);
  const int prow = lane >> 4, pslot = lane & 15;  // DMA piece geometry: 4 rows x 16 slots
  auto stage = [&](int j) {
    const int2 e = s_tl[min(j, nt - 1)];
    const int tok0 = ((e.y >> 4) & 1) * TT;
    const size_t row0 = ((size_t)e.x * Hkv + kvh) * 64 + tok0;
    const uint16_t* kp = k_cache + row0 * D;
    const uint16_t* vp = v_cache + row0 * D;
    const uint32_t dst = ring_base + (uint32_t)((j % NSR) * 2 * TILE * 2);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int c = i * 4 + wave;                // 1 KB piece = tile rows 4c .. 4c+3
      const int t = 4 * c + prow;
      glds16<true>(kp + t * D + ((pslot ^ (t & 15)) << 3), dst + c * 1024);
      glds16<true>(vp + t * D + ((pslot ^ vswz(t)) << 3), dst + TILE * 2 + c * 1024);
    }
  };
  if (nt > 0) {
    stage(0);
    stage(1);
    if constexpr (NSR == 4) stage(2);
  }
  float m = -FLT_MAX, l = 0.f;
  f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
  for (int jt = 0; jt < nt; ++jt) {
    wait_vmcnt<4 * (NSR - 2)>();                 // the next NSR-2 tiles (4 DMAs each) may fly
    ring_barrier();                              // tile jt visible; slot (jt-1) % NSR free
    if (trace && tid == 0 && jt == 0) tr2 = wall_clock64();
    stage(jt + NSR - 1);
    const int2 e = s_tl[jt];
    const bool mine = (e.y & cbit) != 0;         // this column's row reads this block
    const int base = (e.y >> 8) * 64 + ((e.y >> 4) & 1) * TT;   // absolute position of token 0
    const uint16_t* kt = ring + (jt % NSR) * 2 * TILE;
    const uint16_t* vt = kt + TILE;
    f32x4 x[2];
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      x[c] = f32x4{0.f, 0.f, 0.f, 0.f};
      const int t = 16 * c + hl;
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        const bf16x8 a = *reinterpret_cast<const bf16x8*>(kt + t * D + (((4 * ks + lg) ^ (t & 15)) << 3));
        x[c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, qf[ks], x[c], 0, 0, 0);
      }
    }
    // ---- per-column online softmax: lane = 4 tokens (16c + 4 lg + r) of column hl
    float mx = -FLT_MAX;
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int tok = base + 16 * c + 4 * lg + r;
        const float v = (mine && tok < cL) ? x[c][r] * qs : -FLT_MAX;
        x[c][r] = v;
        mx = fmaxf(mx, v);
      }
    mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    const float m_new = fmaxf(m, mx);
    const float alpha = m_new == -FLT_MAX ? 1.f : exp2f(m - m_new);
    float ps = 0.f;
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float p = x[c][r] == -FLT_MAX ? 0.f : exp2f(x[c][r] - m_new);
        x[c][r] = p;
        ps += p;
      }
    ps += __shfl_xor(ps, 16, 64);
    ps += __shfl_xor(ps, 32, 64);
    l = l * alpha + ps;
    m = m_new;
#pragma unroll
    for (int dd = 0; dd < 2; ++dd) acc[dd] *= alpha;
    // ---- O^T += V^T P^T (this wave's 32 dims)
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      i16x4 pb;
#pragma unroll
      for (int r = 0; r < 4; ++r) pb[r] = (short)f2bf(x[c][r]);
      const int row = 16 * c + 4 * lg + (hl >> 2), pp = hl & 3;
#pragma unroll
      for (int dd = 0; dd < 2; ++dd) {
        const int ch = 2 * (2 * wave + dd) + (pp >> 1);
        const uint16_t* va = vt + row * D + ((ch ^ vswz(row)) << 3) + 4 * (pp & 1);
        const i16x4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4*)va);
        acc[dd] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a, pb, acc[dd], 0, 0, 0);
      }
    }
  }
  wait_vmcnt<0>();                               // drain the clamped tail DMAs
  if (trace && tid == 0) tr3 = wall_clock64();

  trace_out();
  group_item_finish<SPLIT>(m, l, acc, part, crow, cL, hl, lg, wave, tid, gp, merges, tick, ws_acc, ws_ml, ci,
                           context_lens, B, Hkv, out, out_stride, kvh, P);
}

// Reductions over the four 16-lane rows of a wave (lanes l, l ^ 16, l ^ 32, l ^ 48: the
// 4 lane groups of one MFMA output column) with the gfx950 row-swap permutes -- VALU ops,
// no ds_bpermute round trip through the LDS unit in the softmax's dependent chain.
typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ float rows4_max(float x) {
  const u32x2_t a = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  const float h0 = __uint_as_float(a.x), h1 = __uint_as_float(a.y);
  const float y = h0 > h1 ? h0 : h1;
  const u32x2_t b = __builtin_amdgcn_permlane32_swap(__float_as_uint(y), __float_as_uint(y), false, false);
  const float g0 = __uint_as_float(b.x), g1 = __uint_as_float(b.y);
  return g0 > g1 ? g0 : g1;
}
__device__ __forceinline__ float rows4_sum(float x) {
  const u32x2_t a = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  const float y = __uint_as_float(a.x) + __uint_as_float(a.y);
  const u32x2_t b = __builtin_amdgcn_permlane32_swap(__float_as_uint(y), __float_as_uint(y), false, false);
  return __uint_as_float(b.x) + __uint_as_float(b.y);
}

// Wave-parallel grouped decode (split plans): the same work items as paged_decode_group_
// kernel<NSR, SPLIT = true>, but the four waves of a workgroup stream DIFFERENT 16-token
// quarter tiles of the item (tile j to wave j % 4), each through a private LDS ring of NSRW
// slots fed by its own LDS-DMA and its own counted vmcnt -- no workgroup barrier per tile.
// Why (profiles/r5_group_deep_ab.log, the per-workgroup timeline of the cooperative kernel on
// a real batch-256 step): all four waves of the cooperative kernel compute the SAME 32-token
// Q K^T (8 MFMAs and 8 KB of LDS reads each, 4x redundant), its online softmax, then PV for
// their 32 dims, behind one barrier per tile -- a serial chain of ~2 us per tile per
// workgroup that neither a deeper ring (deep variants: 7 tiles in flight, 1.0 us/tile, but
// one workgroup per CU) nor more workgroups hides.  Here a tile costs one wave 4 Q K^T MFMAs,
// its softmax and 8 PV MFMAs over 4 + 4 KB of LDS; the four per-wave states (m, l, O^T) are
// combined once at the end through LDS, after which every wave owns 32 dims exactly as in
// the cooperative kernel and the shared epilogue (group_item_finish) runs unchanged.
// LDS: 4 waves x NSRW x 8 KB + the 8 KB tile list -> two workgroups per CU at NSRW = 2.
template <int WAVES, int NSRW>
__global__ __launch_bounds__(64 * WAVES) void paged_decode_group_wave_kernel(
    const uint16_t* __restrict__ q, int q_stride, const uint16_t* __restrict__ k_cache,
    const uint16_t* __restrict__ v_cache, const int* __restrict__ block_tables, int maxb,
    const int* __restrict__ context_lens, int B, int Hkv, float scale,
    uint16_t* __restrict__ out, int out_stride, const int* __restrict__ groups, CascadeIn ci,
    float* __restrict__ ws_acc, float* __restrict__ ws_ml, const int* __restrict__ merges, int* __restrict__ tick) {
  constexpr int G = 4, R = 4, D = 128, TQ = 16, MAXT = kGroupMaxPos * 16;
  constexpr int TILE = TQ * D;                   // elements of one K (or V) quarter tile: 4 KB
  constexpr int WSLOT = 2 * TILE;                // K + V of one ring slot
  constexpr int NDT = 8 / WAVES;                 // 16-dim output blocks per wave after the merge
  static_assert(WAVES * NSRW * WSLOT * 2 >= WAVES * 8 * 64 * 16 + WAVES * 16 * 2 * 4, "ring reused by the merge");
  __shared__ __attribute__((aligned(16))) uint16_t ring[WAVES * NSRW * WSLOT];
  __shared__ unsigned s_tl[MAXT];                // block id << 12 | pos << 6 | quarter << 4 | row mask
  __shared__ int s_nt;

  const int kvh = blockIdx.x, grp = blockIdx.y;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int hl = lane & 15, lg = lane >> 4;
  long long* trace = g_group_trace;
  long long tr0 = 0, tr1 = 0, tr2 = 0, tr3 = 0;
  if (trace && tid == 0) tr0 = wall_clock64();
  const int P = ci.plen ? *ci.plen : 0;
  const int* gp = groups + 8 * grp;
  int rows[R], Ls[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int row = gp[r];
    rows[r] = row >= 0 && row < B ? row : -1;
    Ls[r] = rows[r] >= 0 ? context_lens[rows[r]] : 0;
  }
  if (rows[0] < 0 && rows[1] < 0 && rows[2] < 0 && rows[3] < 0) return;   // unused item
  const int lo = gp[4], hi = min(gp[5], maxb), part = gp[6];

  // ---- tile list: lane j of wave 0 owns block position max(P/64, lo) + j; a distinct block
  // yields the quarters any of its rows reaches
  if (wave == 0) {
    const int pos = max(P >> 6, lo) + lane;
    int ids[R], nq[R], mk[R];
#pragma unroll
    for (int r = 0; r < R; ++r) ids[r] = rows[r] >= 0 && pos < hi ? block_tables[(size_t)rows[r] * maxb + pos] : -1;
    bool alive[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      alive[r] = pos < hi && 64 * pos < Ls[r];
      ids[r] = alive[r] ? ids[r] : -1;
    }
    int cnt = 0;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      bool first = alive[r];
#pragma unroll
      for (int r2 = 0; r2 < r; ++r2) first = first && !(alive[r2] && ids[r2] == ids[r]);
      int mask = 0, need = 0;
      if (first) {
#pragma unroll
        for (int r2 = 0; r2 < R; ++r2)
          if (alive[r2] && ids[r2] == ids[r]) {
            mask |= 1 << r2;
            need = max(need, min(4, (Ls[r2] - 64 * pos + TQ - 1) / TQ));
          }
      }
      nq[r] = need;
      mk[r] = mask;
      cnt += need;
    }
    int off = cnt;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int v = __shfl_up(off, o, 64);
      if (lane >= o) off += v;
    }
    const int total = __shfl(off, 63, 64);
    off -= cnt;
#pragma unroll
    for (int r = 0; r < R; ++r)
      for (int h = 0; h < nq[r]; ++h) s_tl[off++] = ((unsigned)ids[r] << 12) | (pos << 6) | (h << 4) | mk[r];
    if (lane == 0) s_nt = total;
  }
  const int crow = rows[hl >> 2], cL = Ls[hl >> 2], cbit = 1 << (hl >> 2);
  bf16x8 qf[4];
  {
    const uint16_t* qp = q + (size_t)max(crow, 0) * q_stride + (size_t)(kvh * G + (hl & 3)) * D + lg * 8;
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const uint4 v = crow >= 0 ? *reinterpret_cast<const uint4*>(qp + ks * 32) : make_uint4(0, 0, 0, 0);
      qf[ks] = __builtin_bit_cast(bf16x8, v);
    }
  }
  __syncthreads();                               // tile list + Q landed (fence drains vmcnt)
  const int nt = s_nt;
  if (trace && tid == 0) tr1 = wall_clock64();

  const float qs = scale * kLog2e;
  const uint32_t wbase = lds_u32(ring) + (uint32_t)(wave * NSRW * WSLOT * 2);
  const int prow = lane >> 4, pslot = lane & 15;
  const int mine_nt = nt > wave ? (nt - wave + WAVES - 1) / WAVES : 0;   // this wave's tiles: wave + WAVES i
  auto stage = [&](int i) {
    const unsigned e = s_tl[wave + WAVES * i];
    const size_t row0 = ((size_t)(e >> 12) * Hkv + kvh) * 64 + ((e >> 4) & 3) * TQ;
    const uint16_t* kp = k_cache + row0 * D;
    const uint16_t* vp = v_cache + row0 * D;
    const uint32_t dst = wbase + (uint32_t)((i % NSRW) * WSLOT * 2);
#pragma unroll
    for (int c = 0; c < 4; ++c) {                // 1 KB piece = tile rows 4c .. 4c+3
      const int t = 4 * c + prow;
      glds16<true>(kp + t * D + ((pslot ^ t) << 3), dst + c * 1024);
      glds16<true>(vp + t * D + ((pslot ^ vswz(t)) << 3), dst + TILE * 2 + c * 1024);
    }
  };
#pragma unroll
  for (int i = 0; i < NSRW - 1; ++i)
    if (i < mine_nt) stage(i);
  float m = -FLT_MAX, l = 0.f;
  f32x4 o8[8];
#pragma unroll
  for (int dt = 0; dt < 8; ++dt) o8[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int i = 0; i < mine_nt; ++i) {
    if (i + NSRW - 1 < mine_nt) {
      stage(i + NSRW - 1);
      wait_vmcnt<8 * (NSRW - 1)>();              // tile i landed; the next NSRW - 1 may fly
    } else {
      wait_vmcnt<0>();
    }
    if (trace && tid == 0 && i == 0) tr2 = wall_clock64();
    const unsigned e = s_tl[wave + WAVES * i];
    const bool mine = (e & cbit) != 0;
    const int base = ((e >> 6) & 63) * 64 + ((e >> 4) & 3) * TQ;
    const uint16_t* kt = ring + (wave * NSRW + i % NSRW) * WSLOT;
    const uint16_t* vt = kt + TILE;
    f32x4 x = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const bf16x8 a = *reinterpret_cast<const bf16x8*>(kt + hl * D + (((4 * ks + lg) ^ hl) << 3));
      x = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, qf[ks], x, 0, 0, 0);
    }
    // ---- per-column online softmax: lane = tokens 4 lg + r of column hl
    float mx = -FLT_MAX;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int tok = base + 4 * lg + r;
      const float v = (mine && tok < cL) ? x[r] * qs : -FLT_MAX;
      x[r] = v;
      mx = fmaxf(mx, v);
    }
    mx = rows4_max(mx);
    const float m_new = fmaxf(m, mx);
    const float alpha = m_new == -FLT_MAX ? 1.f : __builtin_amdgcn_exp2f(m - m_new);
    float ps = 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float p = x[r] == -FLT_MAX ? 0.f : __builtin_amdgcn_exp2f(x[r] - m_new);
      x[r] = p;
      ps += p;
    }
    ps = rows4_sum(ps);
    l = l * alpha + ps;
    m = m_new;
    // ---- O^T += V^T P^T over all 128 dims (8 x 16)
    i16x4 pb;
#pragma unroll
    for (int r = 0; r < 4; ++r) pb[r] = (short)f2bf(x[r]);
    const int row = 4 * lg + (hl >> 2), pp = hl & 3;
#pragma unroll
    for (int dt = 0; dt < 8; ++dt) {
      o8[dt] *= alpha;
      const int ch = 2 * dt + (pp >> 1);
      const uint16_t* va = vt + row * D + ((ch ^ vswz(row)) << 3) + 4 * (pp & 1);
      const i16x4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4*)va);
      o8[dt] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a, pb, o8[dt], 0, 0, 0);
    }
  }
  if (trace && tid == 0) tr3 = wall_clock64();

  // ---- combine the waves' states through LDS (the ring is free once every wave is done):
  // wave w then owns dims 16 (NDT w + dd) + 4 lg + r (NDT = 2 at four waves: as in the
  // cooperative kernel)
  __syncthreads();
  f32x4* s_o = reinterpret_cast<f32x4*>(ring);                       // [wave][dt][lane]
  float* s_ml = reinterpret_cast<float*>(ring) + WAVES * 8 * 64 * 4; // [wave][column][2]
#pragma unroll
  for (int dt = 0; dt < 8; ++dt) s_o[(wave * 8 + dt) * 64 + lane] = o8[dt];
  if (lg == 0) {
    s_ml[(wave * 16 + hl) * 2] = m;
    s_ml[(wave * 16 + hl) * 2 + 1] = l;
  }
  __syncthreads();
  float mw[WAVES], lw[WAVES], M = -FLT_MAX;
#pragma unroll
  for (int u = 0; u < WAVES; ++u) {
    mw[u] = s_ml[(u * 16 + hl) * 2];
    lw[u] = s_ml[(u * 16 + hl) * 2 + 1];
    M = fmaxf(M, mw[u]);
  }
  f32x4 acc[NDT];
#pragma unroll
  for (int dd = 0; dd < NDT; ++dd) acc[dd] = f32x4{0.f, 0.f, 0.f, 0.f};
  float L = 0.f;
#pragma unroll
  for (int u = 0; u < WAVES; ++u) {
    const float f = mw[u] == -FLT_MAX ? 0.f : exp2f(mw[u] - M);
    L += f * lw[u];
#pragma unroll
    for (int dd = 0; dd < NDT; ++dd) acc[dd] += f * s_o[(u * 8 + NDT * wave + dd) * 64 + lane];
  }
  if (trace && tid == 0) {
    long long* t = trace + ((size_t)blockIdx.y * gridDim.x + blockIdx.x) * 8;
    t[0] = tr0; t[1] = tr1; t[2] = tr2; t[3] = tr3; t[4] = wall_clock64(); t[5] = nt;
    t[6] = __builtin_amdgcn_s_getreg((31 << 11) | 4);
    t[7] = __builtin_amdgcn_s_getreg(20 | (3 << 11)) & 15;
  }
  group_item_finish<true, NDT>(M, L, acc, part, crow, cL, hl, lg, wave, tid, gp, merges, tick, ws_acc, ws_ml, ci,
                          context_lens, B, Hkv, out, out_stride, kvh, P);
}

// Combines the partials of every split group (merges [cap, 8] = (4 row ids, first slot,
// slots, 0, 0); slots 0: nothing to merge) with the cascade prefix partials of each column's
// row, then normalises: thread = (column, 8 dims).
// COH: the split partials were written in this launch (write-through) -- agent-scope loads
template <bool COH>
__device__ __forceinline__ void group_merge_body(const int* __restrict__ mg, const float* __restrict__ ws_acc,
                                                 const float* __restrict__ ws_ml,
                                                 const int* __restrict__ context_lens, int B, int Hkv,
                                                 uint16_t* __restrict__ out, int out_stride, const CascadeIn& ci,
                                                 int kvh, int t) {
  constexpr int D = 128;
  const int first = mg[4], np = mg[5];
  if (np <= 0) return;
  const int col = t >> 4, d0 = (t & 15) * 8;
  const int row = mg[col >> 2];
  if (row < 0 || row >= B) return;
  const int Hq = Hkv * 4, h = kvh * 4 + (col & 3);
  uint16_t* op = out + (size_t)row * out_stride + (size_t)h * D + d0;
  const int P = ci.plen ? *ci.plen : 0;
  if (context_lens[row] <= P) {                  // a padded decode slot: defined zeros
    *reinterpret_cast<uint4*>(op) = make_uint4(0, 0, 0, 0);
    return;
  }
  const int nc = ci.plen ? cascade_parts(P, ci.nchunk) : 0;
  // sources 0..np-1: this group's split items, np..np+nc-1: the prefix chunks.  Folded
  // online in batches of 4 whose (m, l) and accumulator loads are all issued before the
  // first use: one memory latency per 4 partials (a max pass followed by a fold pass with
  // one source per iteration left every load exposed: ~2 latencies per partial)
  const int ns = np + nc;
  float M = -FLT_MAX, den = 0.f;
  float num[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int s0 = 0; s0 < ns; s0 += 4) {
    float2 ml[4];
    float4 a0[4], a1[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int s = min(s0 + j, ns - 1);
      const float *pml, *pa;
      if (s < np) {
        const size_t c2 = ((size_t)(first + s) * Hkv + kvh) * 16 + col;
        pml = ws_ml + c2 * 2;
        pa = ws_acc + c2 * D + d0;
        if constexpr (COH) {
          const float4 m4 = load2_coh(pml);
          ml[j] = make_float2(m4.x, m4.y);
          a0[j] = slab_load4<true>(pa);
          a1[j] = slab_load4<true>(pa + 4);
          continue;
        }
      } else {
        const size_t r = ((size_t)(s - np) * B + row) * Hq + h;
        pml = ci.ml + r * 2;
        pa = ci.acc + r * D + d0;
      }
      ml[j] = *reinterpret_cast<const float2*>(pml);
      a0[j] = *reinterpret_cast<const float4*>(pa);
      a1[j] = *reinterpret_cast<const float4*>(pa + 4);
    }
    float bm = M;
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (s0 + j < ns) bm = fmaxf(bm, ml[j].x);
    const float f = M == -FLT_MAX ? 0.f : exp2f(M - bm);   // rescale what is folded so far
    den *= f;
#pragma unroll
    for (int e = 0; e < 8; ++e) num[e] *= f;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float w = (s0 + j >= ns || ml[j].x == -FLT_MAX) ? 0.f : exp2f(ml[j].x - bm);
      den += w * ml[j].y;
      num[0] += w * a0[j].x; num[1] += w * a0[j].y; num[2] += w * a0[j].z; num[3] += w * a0[j].w;
      num[4] += w * a1[j].x; num[5] += w * a1[j].y; num[6] += w * a1[j].z; num[7] += w * a1[j].w;
    }
    M = bm;
  }
  const float inv = den > 0.f ? 1.f / den : 0.f;
#pragma unroll
  for (int e = 0; e < 8; ++e) num[e] *= inv;
  *reinterpret_cast<uint4*>(op) = pack8(num);
}

__global__ __launch_bounds__(256) void group_split_merge_kernel(const int* __restrict__ merges,
                                                                const float* __restrict__ ws_acc,
                                                                const float* __restrict__ ws_ml,
                                                                const int* __restrict__ context_lens, int B,
                                                                int Hkv, uint16_t* __restrict__ out,
                                                                int out_stride, CascadeIn ci) {
  group_merge_body<false>(merges + 8 * blockIdx.y, ws_acc, ws_ml, context_lens, B, Hkv, out, out_stride, ci,
                          blockIdx.x, threadIdx.x);
}

// ---------------------------------------------------------------------------------------
// Persistent grouped decode (plan [3, cap, 8]): the split plan's work items are packed by
// the host into bins of <= kBinItems (LPT by tile count, ops.split_decode_groups(bins=));
// one workgroup per (KV head, bin) streams the tiles of ALL its items through ONE LDS-DMA
// ring.  The split kernel above pays, per ~10-tile item, a block-table round trip (tile
// list), the Q loads and the first DMA's latency before any math, and a ring drain at the
// end (profiles/r2_pmc/group_split_decode.txt: 7.4 tiles per workgroup, waves parked 62 %
// of their cycles).  Here the tile lists of every item of the bin are built up front by the
// four waves together (one latency per workgroup), the ring runs across item boundaries,
// and the next item's Q fragments load under the current item's tiles.  Every item writes
// an un-normalised (m, l, O) partial to its slot; group_split_merge_kernel folds each
// group's items and the cascade prefix chunks, and normalises.
constexpr int kBinItems = 8;
constexpr int kBinMaxTiles = 512;

// workgroups per KV head of the persistent launch: ~3 per CU chip-wide, at least one per
// identity quad (shared with ops.persist_bins)
__host__ __device__ inline int group_persist_bins(int cap, int Hkv) {
  const int a = 768 / (Hkv > 0 ? Hkv : 1), b = (cap + 3) / 4;
  const int nb = a > b ? a : b;
  return nb < cap ? nb : cap;
}

template <int NSR = 3>
__global__ __launch_bounds__(256) void paged_decode_group_persist_kernel(
    const uint16_t* __restrict__ q, int q_stride, const uint16_t* __restrict__ k_cache,
    const uint16_t* __restrict__ v_cache, const int* __restrict__ block_tables, int maxb,
    const int* __restrict__ context_lens, int B, int Hkv, float scale, const int* __restrict__ items,
    const int* __restrict__ bins, CascadeIn ci, float* __restrict__ ws_acc, float* __restrict__ ws_ml) {
  constexpr int G = 4, R = 4, D = 128, TT = 32;
  constexpr int TILE = TT * D;
  __shared__ __attribute__((aligned(16))) uint16_t ring[NSR * 2 * TILE];
  __shared__ int2 s_tl[kBinMaxTiles];           // (block id, item << 16 | pos << 8 | half << 4 | mask)
  __shared__ int s_it[kBinItems][8];            // rows[4], lo, hi, slot, - (all -1: no item)
  __shared__ int s_L[kBinItems][4];             // context lengths of the item rows
  __shared__ int s_cnt[kBinItems];

  const int kvh = blockIdx.x, bin = blockIdx.y;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int hl = lane & 15, lg = lane >> 4;
  const int P = ci.plen ? *ci.plen : 0;          // multiple of 64

  if (tid < kBinItems * 8) {                     // the bin's items -> LDS
    const int j = tid >> 3, f = tid & 7;
    const int it = bins[bin * 8 + j];
    int v = it >= 0 ? items[it * 8 + f] : -1;
    if (f < 4) {
      v = (v >= 0 && v < B) ? v : -1;
      s_L[j][f] = v >= 0 ? context_lens[v] : 0;
    }
    s_it[j][f] = v;
  }
  __syncthreads();
  int nit = 0;
#pragma unroll
  for (int j = 0; j < kBinItems; ++j) nit += s_it[j][6] >= 0 ? 1 : 0;
  if (nit == 0) return;                          // unused bin (uniform)

  // ---- tile lists of items wave and wave + 4: lane = one block position of the item
  int2 ent[2][2 * R];
  int cnt[2], off[2];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int j = wave + 4 * u;
    cnt[u] = 0;
    off[u] = 0;
    if (j < nit) {
      const int lo = s_it[j][4], hi = min(s_it[j][5], maxb);
      const int pos = max(P >> 6, lo) + lane;
      int ids[R];
      bool alive[R];
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const int row = s_it[j][r];
        alive[r] = row >= 0 && pos < hi && 64 * pos < s_L[j][r];
        ids[r] = alive[r] ? block_tables[(size_t)row * maxb + pos] : -1;
      }
#pragma unroll
      for (int r = 0; r < R; ++r) {
        bool first = alive[r];
#pragma unroll
        for (int r2 = 0; r2 < r; ++r2) first = first && !(alive[r2] && ids[r2] == ids[r]);
        if (first) {
          int mask = 0, two = 0;
#pragma unroll
          for (int r2 = 0; r2 < R; ++r2)
            if (alive[r2] && ids[r2] == ids[r]) { mask |= 1 << r2; two |= s_L[j][r2] > 64 * pos + 32; }
#pragma unroll
          for (int h = 0; h < 2; ++h)
            if (h == 0 || two) {
              const int y = (j << 16) | (pos << 8) | (h << 4) | mask;
#pragma unroll
              for (int e = 0; e < 2 * R; ++e)
                if (e == cnt[u]) ent[u][e] = make_int2(ids[r], y);
              cnt[u]++;
            }
        }
      }
      int o = cnt[u];                            // exclusive prefix sum over the lanes
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const int v = __shfl_up(o, d, 64);
        if (lane >= d) o += v;
      }
      if (lane == 63) s_cnt[j] = o;
      off[u] = o - cnt[u];
    }
  }
  __syncthreads();
  int base[kBinItems], NT = 0;
#pragma unroll
  for (int j = 0; j < kBinItems; ++j) {
    base[j] = NT;
    NT += j < nit ? s_cnt[j] : 0;
  }
  NT = min(NT, kBinMaxTiles);                    // the host plans <= kBinMaxTiles per bin
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int j = wave + 4 * u;
    if (j < nit) {
      int b0 = 0;
#pragma unroll
      for (int jj = 0; jj < kBinItems; ++jj)
        if (jj == j) b0 = base[jj];
#pragma unroll
      for (int e = 0; e < 2 * R; ++e)
        if (e < cnt[u] && b0 + off[u] + e < kBinMaxTiles) s_tl[b0 + off[u] + e] = ent[u][e];
    }
  }
  // items without any live tile: an empty partial (the merge reads every slot)
  for (int j = wave; j < nit; j += 4) {
    if (s_cnt[j] == 0) {
      const size_t cidx = ((size_t)s_it[j][6] * Hkv + kvh) * 16 + hl;
#pragma unroll
      for (int dd = 0; dd < 2; ++dd)
        *reinterpret_cast<f32x4*>(ws_acc + cidx * D + 16 * (2 * wave + dd) + 4 * lg) = f32x4{0.f, 0.f, 0.f, 0.f};
      if (lg == 0) *reinterpret_cast<float2*>(ws_ml + cidx * 2) = make_float2(-FLT_MAX, 0.f);
    }
  }
  // first item with tiles and the one after it: Q fragments of the current / next item,
  // loaded before the barrier below (which drains them: nothing the compiler tracks is in
  // flight when the ring loop starts)
  auto next_live = [&](int j) {
    int n = kBinItems;
#pragma unroll
    for (int jj = kBinItems - 1; jj >= 0; --jj)
      if (jj > j && jj < nit && s_cnt[jj] > 0) n = jj;
    return n;
  };
  auto qptr = [&](int j) {
    const int row = j < nit ? s_it[j][hl >> 2] : -1;
    return q + (size_t)max(row, 0) * q_stride + (size_t)(kvh * G + (hl & 3)) * D + lg * 8;
  };
  auto qrow = [&](int j) { return j < nit ? s_it[j][hl >> 2] : -1; };
  int cur = next_live(-1);
  int nxt = next_live(cur);
  bf16x8 qf[4], qn[4];
  {
    const uint16_t* p0 = qptr(cur);
    const uint16_t* p1 = qptr(nxt);
    const bool v0 = qrow(cur) >= 0, v1 = qrow(nxt) >= 0;
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const uint4 a = v0 ? *reinterpret_cast<const uint4*>(p0 + ks * 32) : make_uint4(0, 0, 0, 0);
      const uint4 b = v1 ? *reinterpret_cast<const uint4*>(p1 + ks * 32) : make_uint4(0, 0, 0, 0);
      qf[ks] = __builtin_bit_cast(bf16x8, a);
      qn[ks] = __builtin_bit_cast(bf16x8, b);
    }
  }
  __syncthreads();
  if (NT == 0) return;                           // (uniform) nothing live in this bin
  int cL = s_L[cur][hl >> 2];
  const int cbit = 1 << (hl >> 2);
  // the item after next: its Q goes straight into qn by inline-asm loads (invisible to the
  // compiler's waitcnt pass, which would otherwise drain the ring before the copy); they are
  // issued before a step's DMAs, so the next step's counted vmcnt wait covers them
  auto prefetch_q = [&](int j) {
    const uint16_t* p = qptr(j);
#pragma unroll
    for (int ks = 0; ks < 4; ++ks)
      asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(qn[ks]) : "v"(p + ks * 32) : "memory");
  };

  const float qs = scale * kLog2e;
  const uint32_t ring_base = lds_u32(ring);
  const int prow = lane >> 4, pslot = lane & 15;  // DMA piece geometry: 4 rows x 16 slots
  auto stage = [&](int j) {
    const int2 e = s_tl[min(j, NT - 1)];
    const int tok0 = ((e.y >> 4) & 1) * TT;
    const size_t row0 = ((size_t)e.x * Hkv + kvh) * 64 + tok0;
    const uint16_t* kp = k_cache + row0 * D;
    const uint16_t* vp = v_cache + row0 * D;
    const uint32_t dst = ring_base + (uint32_t)((j % NSR) * 2 * TILE * 2);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int c = i * 4 + wave;                // 1 KB piece = tile rows 4c .. 4c+3
      const int t = 4 * c + prow;
      glds16<true>(kp + t * D + ((pslot ^ (t & 15)) << 3), dst + c * 1024);
      glds16<true>(vp + t * D + ((pslot ^ vswz(t)) << 3), dst + TILE * 2 + c * 1024);
    }
  };
  float m = -FLT_MAX, l = 0.f;
  f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
  auto flush = [&](int j) {                      // partial of item j for this lane's column
    const size_t cidx = ((size_t)s_it[j][6] * Hkv + kvh) * 16 + hl;
#pragma unroll
    for (int dd = 0; dd < 2; ++dd)
      *reinterpret_cast<f32x4*>(ws_acc + cidx * D + 16 * (2 * wave + dd) + 4 * lg) = acc[dd];
    if (wave == 0 && lg == 0) *reinterpret_cast<float2*>(ws_ml + cidx * 2) = make_float2(m, l);
  };
  stage(0);
  stage(1);
  if constexpr (NSR == 4) stage(2);
  for (int jt = 0; jt < NT; ++jt) {
    wait_vmcnt<4 * (NSR - 2)>();                 // the next NSR-2 tiles (4 DMAs each) may fly
    ring_barrier();                              // tile jt visible; slot (jt-1) % NSR free
    const int2 e = s_tl[jt];
    const int it = __builtin_amdgcn_readfirstlane((e.y >> 16) & 7);
    if (it != cur) {                             // item boundary (uniform): flush, switch
      flush(cur);
      cur = it;
      const bool live = qrow(cur) >= 0;
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        asm volatile("" : "+v"(qn[ks]));         // landed: the vmcnt wait above covered it
        qf[ks] = live ? qn[ks] : bf16x8{};
      }
      nxt = next_live(cur);
      prefetch_q(nxt);                           // issued before this step's DMAs
      cL = s_L[cur][hl >> 2];
      m = -FLT_MAX;
      l = 0.f;
      acc[0] = f32x4{0.f, 0.f, 0.f, 0.f};
      acc[1] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    stage(jt + NSR - 1);
    const bool mine = (e.y & cbit) != 0;         // this column's row reads this block
    const int tbase = ((e.y >> 8) & 0xff) * 64 + ((e.y >> 4) & 1) * TT;   // position of token 0
    const uint16_t* kt = ring + (jt % NSR) * 2 * TILE;
    const uint16_t* vt = kt + TILE;
    f32x4 x[2];
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      x[c] = f32x4{0.f, 0.f, 0.f, 0.f};
      const int t = 16 * c + hl;
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        const bf16x8 a = *reinterpret_cast<const bf16x8*>(kt + t * D + (((4 * ks + lg) ^ (t & 15)) << 3));
        x[c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, qf[ks], x[c], 0, 0, 0);
      }
    }
    float mx = -FLT_MAX;
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int tok = tbase + 16 * c + 4 * lg + r;
        const float v = (mine && tok < cL) ? x[c][r] * qs : -FLT_MAX;
        x[c][r] = v;
        mx = fmaxf(mx, v);
      }
    mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    const float m_new = fmaxf(m, mx);
    const float alpha = m_new == -FLT_MAX ? 1.f : exp2f(m - m_new);
    float ps = 0.f;
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float p = x[c][r] == -FLT_MAX ? 0.f : exp2f(x[c][r] - m_new);
        x[c][r] = p;
        ps += p;
      }
    ps += __shfl_xor(ps, 16, 64);
    ps += __shfl_xor(ps, 32, 64);
    l = l * alpha + ps;
    m = m_new;
#pragma unroll
    for (int dd = 0; dd < 2; ++dd) acc[dd] *= alpha;
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      i16x4 pb;
#pragma unroll
      for (int r = 0; r < 4; ++r) pb[r] = (short)f2bf(x[c][r]);
      const int row = 16 * c + 4 * lg + (hl >> 2), pp = hl & 3;
#pragma unroll
      for (int dd = 0; dd < 2; ++dd) {
        const int ch = 2 * (2 * wave + dd) + (pp >> 1);
        const uint16_t* va = vt + row * D + ((ch ^ vswz(row)) << 3) + 4 * (pp & 1);
        const i16x4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4*)va);
        acc[dd] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a, pb, acc[dd], 0, 0, 0);
      }
    }
  }
  flush(cur);
  wait_vmcnt<0>();                               // drain the clamped tail DMAs
}

// forward declaration (defined below with the other cascade launchers)
int docqa_cascade_prefix(const void* qkv, int row_stride, int rows, int Hq, int Hkv, float scale,
                         const void* k_cache, const void* v_cache, const int* prefix_table,
                         const int* plen, int BS, int nchunk, float* acc, float* ml,
                         const int* positions, const float* cos_sin, hipStream_t s);

// Grouped cascade decode: MFMA prefix partials over the shared prompt prefix, then the
// group kernel over each row's keys [*plen, L) with the rows packed by shared blocks
// (groups: [ngroups, 4] row ids, -1 = none; every batch row in exactly one group).
int docqa_paged_decode_cascade_grouped(const void* q, int q_stride, void* k_cache, void* v_cache,
                                       const int* block_tables, int maxb, const int* context_lens,
                                       void* out, int out_stride, int B, int Hq, int Hkv, int BS,
                                       float scale, const int* prefix_table, const int* plen, int nchunk,
                                       float* pacc, float* pml, const int* groups, int ngroups,
                                       hipStream_t s) {
  if (B == 0) return 0;
  if (BS != 64 || maxb > kGroupMaxTable || Hq != 4 * Hkv || nchunk < 1 || nchunk > kCascadeMaxChunks ||
      ngroups < 1)
    return -1;
  int rc = docqa_cascade_prefix(q, q_stride, B, Hq, Hkv, scale, k_cache, v_cache, prefix_table, plen, BS,
                                nchunk, pacc, pml, nullptr, nullptr, s);
  if (rc) return rc;
  const CascadeIn ci{pacc, pml, plen, nchunk, nullptr};
  static const int nsr = [] {   // ring slots (A/B knob): 3 (3 workgroups / CU) or 4 (2)
    const char* e = getenv("DOCQA_GROUP_NSR");
    return e && atoi(e) == 4 ? 4 : 3;
  }();
  if (nsr == 4)
    paged_decode_group_kernel<4><<<dim3(Hkv, ngroups), 256, 0, s>>>(
        (const uint16_t*)q, q_stride, (const uint16_t*)k_cache, (const uint16_t*)v_cache, block_tables, maxb,
        context_lens, B, Hkv, scale, (uint16_t*)out, out_stride, groups, ci);
  else
    paged_decode_group_kernel<3><<<dim3(Hkv, ngroups), 256, 0, s>>>(
        (const uint16_t*)q, q_stride, (const uint16_t*)k_cache, (const uint16_t*)v_cache, block_tables, maxb,
        context_lens, B, Hkv, scale, (uint16_t*)out, out_stride, groups, ci);
  DOCQA_CHECK_LAUNCH();
  return 0;
}

// Shared-prefix (cascade) kernel on a side stream, forked from / joined back to `s` by
// events -- captured into the decode graph as parallel branches -- for launchers whose
// suffix kernel does not read the prefix partials (only their merge does): its workgroups
// fill the CUs the suffix kernel's tail leaves idle.  *join: the event `s` must wait for
// before the merge (nullptr: ran on `s`, DOCQA_CASCADE_FORK=0 or no side stream).
static int cascade_prefix_forked(const void* q, int q_stride, int B, int Hq, int Hkv, float scale, void* k_cache,
                                 void* v_cache, const int* prefix_table, const int* plen, int BS, int nchunk,
                                 float* pacc, float* pml, hipStream_t s, hipEvent_t* join) {
  static const bool fork = [] {
    const char* e = getenv("DOCQA_CASCADE_FORK");
    return !(e && atoi(e) == 0);
  }();
  *join = nullptr;
  hipStream_t side = s;
  hipEvent_t ev_fork = nullptr, ev_join = nullptr;
  if (fork) {
    static hipStream_t streams[64] = {};
    static hipEvent_t evs[64][2] = {};
    int dev = 0;
    if (hipGetDevice(&dev) == hipSuccess && dev >= 0 && dev < 64) {
      // created on the first (eager) call: the engine runs every decode step body once
      // before capturing it, and creation is not a stream operation a capture may contain
      hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
      if (!streams[dev] && hipStreamIsCapturing(s, &cs) == hipSuccess && cs == hipStreamCaptureStatusNone) {
        if (hipStreamCreateWithFlags(&streams[dev], hipStreamNonBlocking) != hipSuccess ||
            hipEventCreateWithFlags(&evs[dev][0], hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&evs[dev][1], hipEventDisableTiming) != hipSuccess)
          streams[dev] = nullptr;
      }
      if (streams[dev] && evs[dev][0] && evs[dev][1]) {
        side = streams[dev];
        ev_fork = evs[dev][0];
        ev_join = evs[dev][1];
      }
    }
  }
  if (side != s) {
    if (hipEventRecord(ev_fork, s) != hipSuccess || hipStreamWaitEvent(side, ev_fork, 0) != hipSuccess) return -3;
  }
  const int rc = docqa_cascade_prefix(q, q_stride, B, Hq, Hkv, scale, k_cache, v_cache, prefix_table, plen, BS,
                                      nchunk, pacc, pml, nullptr, nullptr, side);
  if (rc) return rc;
  if (side != s) {
    if (hipEventRecord(ev_join, side) != hipSuccess) return -3;
    *join = ev_join;
  }
  return 0;
}

// Grouped cascade decode with long groups split over several workgroups: items [cap, 8]
// (see paged_decode_group_kernel SPLIT), merges [cap, 8] (group_split_merge_kernel),
// ws_acc [slots, Hkv, 16, 128] / ws_ml [slots, Hkv, 16, 2] fp32 partials.
// wave-parallel split kernel (paged_decode_group_wave_kernel): DOCQA_GROUP_WAVE=1, or
// docqa_set_group_wave (tests and probes A/B both kernels in one process)
// variants (waves per workgroup x ring slots per wave): 1 = 4 x 2 (the default), 2 = 2 x 3,
// 3 = 2 x 4, 4 = 1 x 4; 0 = the cooperative kernel.  Replayed on a real batch-256 step:
// 69.6 / 81.2-83.7 / 81.4 / 103.7-110.5 us against the cooperative kernel's 98.4 (132
// items) - 111.8 us (profiles/r5_group_wave_variants.log)
static int g_group_wave = -1;
static bool group_wave_on() {
  if (g_group_wave < 0) {
    const char* e = getenv("DOCQA_GROUP_WAVE");
    const int v = e ? atoi(e) : 1;   // default: 4 waves x 2 slots (profiles/r5_group_wave_variants.log)
    g_group_wave = v >= 0 && v <= 4 ? v : 0;
  }
  return g_group_wave > 0;
}

int docqa_set_group_wave(int v) {
  group_wave_on();
  const int was = g_group_wave;
  if (v >= 0) g_group_wave = v <= 4 ? v : 0;
  return was;
}

int docqa_paged_decode_cascade_split(const void* q, int q_stride, void* k_cache, void* v_cache,
                                     const int* block_tables, int maxb, const int* context_lens,
                                     void* out, int out_stride, int B, int Hq, int Hkv, int BS,
                                     float scale, const int* prefix_table, const int* plen, int nchunk,
                                     float* pacc, float* pml, const int* items, const int* merges, int cap,
                                     float* ws_acc, float* ws_ml, int defer, hipStream_t s, int* tick,
                                     int inline_prefix, const float* fP, int fS, const int* positions,
                                     const float* cos_sin, const int* slot_mapping) {
  if (B == 0) return 0;
  if (BS != 64 || maxb > kGroupMaxTable || Hq != 4 * Hkv || nchunk < 1 || nchunk > kCascadeMaxChunks || cap < 1)
    return -1;
  // inline_prefix: no prefix kernel -- the plan's items start at block 0 (built with skip 0),
  // so every group streams the shared template blocks itself (L2 hits after the first group)
  if (inline_prefix && defer) return -1;
  // defer (a plan from ops.split_decode_groups(defer=True)): every item writes a partial
  // and every group has a merge row, so no item reads the prefix partials and the prefix
  // kernel is forked onto a side stream beside the group kernel
  hipEvent_t ev_join = nullptr;
  if (!inline_prefix) {
    const int rc = defer ? cascade_prefix_forked(q, q_stride, B, Hq, Hkv, scale, k_cache, v_cache, prefix_table,
                                                 plen, BS, nchunk, pacc, pml, s, &ev_join)
                         : docqa_cascade_prefix(q, q_stride, B, Hq, Hkv, scale, k_cache, v_cache, prefix_table, plen,
                                                BS, nchunk, pacc, pml, nullptr, nullptr, s);
    if (rc) return rc;
  }
  const CascadeIn ci{pacc, pml, inline_prefix ? nullptr : plen, nchunk, nullptr};
  static const int nsr = [] {   // ring slots (A/B knob): 3 (3 workgroups / CU) or 4 (2)
    const char* e = getenv("DOCQA_GROUP_NSR");
    return e && atoi(e) == 4 ? 4 : 3;
  }();
  // tick (non-deferred plans: the prefix partials are complete before the group kernel):
  // split groups merged by their last item, no merge launch (int32 [cap, Hkv] zeroed,
  // items carry their merge row in column 7)
  int* tk = (tick && !defer) ? tick : nullptr;
  if (fP) {   // QKV slabs straight in: RoPE + new-token cache write in the group kernel
    if (!inline_prefix || defer || fS < 1 || !positions || !cos_sin || !slot_mapping) return -1;
    const FusedQKV fz{fP, fS, positions, cos_sin, slot_mapping, Hq};
    paged_decode_group_kernel<3, true, true><<<dim3(Hkv, cap), 256, 0, s>>>(
        nullptr, 0, (const uint16_t*)k_cache, (const uint16_t*)v_cache, block_tables, maxb, context_lens, B, Hkv,
        scale, (uint16_t*)out, out_stride, items, ci, ws_acc, ws_ml, merges, tk, fz);
    DOCQA_CHECK_LAUNCH();
    if (tk) return 0;
  } else if (group_wave_on()) {
#define DOCQA_WAVE_LAUNCH(W_, N_)                                                                                 \
  paged_decode_group_wave_kernel<W_, N_><<<dim3(Hkv, cap), 64 * W_, 0, s>>>(                                     \
      (const uint16_t*)q, q_stride, (const uint16_t*)k_cache, (const uint16_t*)v_cache, block_tables, maxb,       \
      context_lens, B, Hkv, scale, (uint16_t*)out, out_stride, items, ci, ws_acc, ws_ml, merges, tk)
    switch (g_group_wave) {
      case 2: DOCQA_WAVE_LAUNCH(2, 3); break;
      case 3: DOCQA_WAVE_LAUNCH(2, 4); break;
      case 4: DOCQA_WAVE_LAUNCH(1, 4); break;
      default: DOCQA_WAVE_LAUNCH(4, 2); break;
    }
#undef DOCQA_WAVE_LAUNCH
  } else if (nsr == 4)
    paged_decode_group_kernel<4, true><<<dim3(Hkv, cap), 256, 0, s>>>(
        (const uint16_t*)q, q_stride, (const uint16_t*)k_cache, (const uint16_t*)v_cache, block_tables, maxb,
        context_lens, B, Hkv, scale, (uint16_t*)out, out_stride, items, ci, ws_acc, ws_ml, merges, tk);
  else
    paged_decode_group_kernel<3, true><<<dim3(Hkv, cap), 256, 0, s>>>(
        (const uint16_t*)q, q_stride, (const uint16_t*)k_cache, (const uint16_t*)v_cache, block_tables, maxb,
        context_lens, B, Hkv, scale, (uint16_t*)out, out_stride, items, ci, ws_acc, ws_ml, merges, tk);
  DOCQA_CHECK_LAUNCH();
  if (tk) return 0;
  if (ev_join && hipStreamWaitEvent(s, ev_join, 0) != hipSuccess) return -3;
  // merge rows: at most (cap + 1) / 2 (ops.split_decode_groups guarantees it), so half the
  // grid -- the empty workgroups of the unused merge rows are not free; deferred: one per group
  group_split_merge_kernel<<<dim3(Hkv, defer ? cap : (cap + 1) / 2), 256, 0, s>>>(merges, ws_acc, ws_ml, context_lens, B, Hkv,
                                                          (uint16_t*)out, out_stride, ci);
  DOCQA_CHECK_LAUNCH();
  return 0;
}

// Persistent grouped cascade decode: plan [3, cap, 8] = items (4 rows, first position, end
// position, slot, 0), merges (4 rows, first slot, slots, 0, 0) covering EVERY group, bins
// (<= 8 item indices, -1 = none) -- group_persist_bins(cap, Hkv) of them.
int docqa_paged_decode_cascade_persist(const void* q, int q_stride, void* k_cache, void* v_cache,
                                       const int* block_tables, int maxb, const int* context_lens,
                                       void* out, int out_stride, int B, int Hq, int Hkv, int BS,
                                       float scale, const int* prefix_table, const int* plen, int nchunk,
                                       float* pacc, float* pml, const int* items, const int* merges,
                                       const int* bins, int cap, float* ws_acc, float* ws_ml, hipStream_t s) {
  if (B == 0) return 0;
  if (BS != 64 || maxb > kGroupMaxTable || Hq != 4 * Hkv || nchunk < 1 || nchunk > kCascadeMaxChunks || cap < 1)
    return -1;
  // The group kernel no longer reads the prefix partials (the merge does), so the shared-
  // prefix kernel runs on a side stream beside it (cascade_prefix_forked).
  hipEvent_t ev_join = nullptr;
  const int rc = cascade_prefix_forked(q, q_stride, B, Hq, Hkv, scale, k_cache, v_cache, prefix_table, plen, BS,
                                       nchunk, pacc, pml, s, &ev_join);
  if (rc) return rc;
  const CascadeIn ci{pacc, pml, plen, nchunk, nullptr};
  const int nb = group_persist_bins(cap, Hkv);
  paged_decode_group_persist_kernel<3><<<dim3(Hkv, nb), 256, 0, s>>>(
      (const uint16_t*)q, q_stride, (const uint16_t*)k_cache, (const uint16_t*)v_cache, block_tables, maxb,
      context_lens, B, Hkv, scale, items, bins, ci, ws_acc, ws_ml);
  DOCQA_CHECK_LAUNCH();
  if (ev_join && hipStreamWaitEvent(s, ev_join, 0) != hipSuccess) return -3;
  group_split_merge_kernel<<<dim3(Hkv, cap), 256, 0, s>>>(merges, ws_acc, ws_ml, context_lens, B, Hkv,
                                                          (uint16_t*)out, out_stride, ci);
  DOCQA_CHECK_LAUNCH();
  return 0;
}

int docqa_group_persist_bins(int cap, int Hkv) { return group_persist_bins(cap, Hkv); }

// diagnostics: route the group kernel's per-workgroup timeline into `buf` (int64 [wgs x 8]),
// nullptr turns it off
int docqa_set_decode_trace(long long* buf) {
  return hipMemcpyToSymbol(HIP_SYMBOL(g_group_trace), &buf, sizeof(buf)) == hipSuccess ? 0 : -1;
}

// log-sum-exp merge of a sequence's context partitions (and, cascade, of the shared-prefix
// chunk partials) -> normalised bf16 output
template <int D>
__global__ __launch_bounds__(D) void paged_decode_reduce(const float* __restrict__ tmp_out,
                                                         const float* __restrict__ tmp_ml,
                                                         const int* __restrict__ context_lens,
                                                         uint16_t* __restrict__ out,
                                                         int out_stride, int Hq, int max_parts,
                                                         CascadeIn ci = CascadeIn{}) {
  const int h = blockIdx.x, b = blockIdx.y, d = threadIdx.x;
  const int P = ci.plen ? *ci.plen : 0;
  const int L = context_lens[b] - P;
  if (L <= 0) {   // padded slot: defined (zero) output
    out[(size_t)b * out_stride + (size_t)h * D + d] = 0;
    return;
  }
  const int chunk = split_chunk(L, max_parts);
  const int np = min(max_parts, (L + chunk - 1) / chunk);
  const int nc = ci.plen ? cascade_parts(P, ci.nchunk) : 0;
  const size_t base = ((size_t)b * Hq + h) * max_parts;
  const size_t B = gridDim.y;
  float M = -FLT_MAX;
  for (int p = 0; p < np; ++p) M = fmaxf(M, tmp_ml[(base + p) * 2]);
  for (int c = 0; c < nc; ++c) M = fmaxf(M, ci.ml[((c * B + b) * Hq + h) * 2]);
  float num = 0.f, den = 0.f;
  for (int p = 0; p < np; ++p) {
    const float w = exp2f(tmp_ml[(base + p) * 2] - M);
    num += w * tmp_out[(base + p) * D + d];
    den += w * tmp_ml[(base + p) * 2 + 1];
  }
  for (int c = 0; c < nc; ++c) {
    const size_t r = (c * B + b) * Hq + h;
    const float pm = ci.ml[r * 2];
    const float w = (pm == -FLT_MAX) ? 0.f : exp2f(pm - M);
    num += w * ci.acc[r * D + d];
    den += w * ci.ml[r * 2 + 1];
  }
  out[(size_t)b * out_stride + (size_t)h * D + d] = f2bf(den > 0.f ? num / den : 0.f);
}

int docqa_paged_decode(const void* q, int q_stride, const void* k_cache, const void* v_cache,
                       const int* block_tables, int maxb, const int* context_lens, void* out,
                       int out_stride, float* tmp_out, float* tmp_ml, int B, int Hq, int Hkv,
                       int D, int BS, int max_parts, float scale, const int* order, hipStream_t s) {
  if (B == 0) return 0;
  if (D != 128 || (BS & (BS - 1)) != 0 || Hq % Hkv != 0) return -1;
  CascadeIn oi{};
  oi.order = order;
  int log2BS = 0;
  while ((1 << log2BS) < BS) ++log2BS;
  const int G = Hq / Hkv;
  dim3 grid(Hkv, B, max_parts);   // partitions slowest: see kDecodeGridNote
  const bool direct = max_parts == 1;
  // U (tokens in flight per lane group per buffer) and occupancy: measured on HBM-resident
  // caches (benchmarks/bench_decode_attn.py, profiles/r1_decode_attention_sweep_hbm.log):
  // U=4 at 2 waves/SIMD beats U=3/3 and U=2/4 -- all keep ~64 wave-loads in flight per
  // CU, which at the loaded HBM latency caps one CU near 17 GB/s.  DOCQA_DECODE_U=2 knob.
  static const int u_env = [] {
    const char* e = getenv("DOCQA_DECODE_U");
    return e ? atoi(e) : 0;
  }();
#define DEC_K(GG, UU, DIR)                                                                    \
  paged_decode_kernel<GG, 128, UU, DIR><<<grid, 256, 0, s>>>(                                 \
      (const uint16_t*)q, q_stride, (const uint16_t*)k_cache, (const uint16_t*)v_cache,       \
      block_tables, maxb, context_lens, tmp_out, tmp_ml, Hkv, BS, log2BS, max_parts, scale,   \
      (uint16_t*)out, out_stride)
#define DEC(GG, UU)                                                                           \
  do {                                                                                        \
    if (direct) DEC_K(GG, UU, true);                                                          \
    else DEC_K(GG, UU, false);                                                                \
  } while (0)
  if (mfma_decode_on(G) && BS == 64 && maxb <= 256 && (G == 4 || G == 8)) {
#define DMFMA(GG)                                                                             \
    do {                                                                                      \
      if (direct && Hkv % 2 == 0 && hpw_knob() == 2)                                          \
        paged_decode_mfma_kernel<GG, true, 2><<<dim3(Hkv / 2, B, 1), 256, 0, s>>>(            \
            (const uint16_t*)q, q_stride, (const uint16_t*)k_cache, (const uint16_t*)v_cache, \
            block_tables, maxb, context_lens, tmp_out, tmp_ml, Hkv, max_parts, scale,         \
            (uint16_t*)out, out_stride, oi);                                         \
      else if (direct)                                                                        \
        paged_decode_mfma_kernel<GG, true><<<grid, 256, 0, s>>>(                              \
            (const uint16_t*)q, q_stride, (const uint16_t*)k_cache, (const uint16_t*)v_cache, \
            block_tables, maxb, context_lens, tmp_out, tmp_ml, Hkv, max_parts, scale,         \
            (uint16_t*)out, out_stride, oi);                                         \
      else                                                                                    \
        paged_decode_mfma_kernel<GG, false><<<grid, 256, 0, s>>>(                             \
            (const uint16_t*)q, q_stride, (const uint16_t*)k_cache, (const uint16_t*)v_cache, \
            block_tables, maxb, context_lens, tmp_out, tmp_ml, Hkv, max_parts, scale,         \
            (uint16_t*)out, out_stride, oi);                                         \
    } while (0)
    if (G == 4) DMFMA(4);
    else DMFMA(8);
#undef DMFMA
    if (!direct)
      paged_decode_reduce<128><<<dim3(Hq, B), 128, 0, s>>>(tmp_out, tmp_ml, context_lens,
                                                           (uint16_t*)out, out_stride, Hq,
                                                           max_parts);
    DOCQA_CHECK_LAUNCH();
    return 0;
  }
  static const bool ring_env = [] {
    const char* e = getenv("DOCQA_DECODE_RING");
    return !(e && atoi(e) == 0);
  }();
  if (ring_env && BS == 64 && maxb <= 256) {
#define DRING(GG)                                                                             \
    do {                                                                                      \
      if (direct && ring_nsr() == 2)                                                          \
        paged_decode_ring_kernel<GG, true, false, 2><<<grid, 256, 0, s>>>(                    \
            (const uint16_t*)q, q_stride, (uint16_t*)k_cache, (uint16_t*)v_cache,             \
            block_tables, maxb, context_lens, tmp_out, tmp_ml, Hkv, max_parts, scale,         \
            (uint16_t*)out, out_stride, FusedQKV{}, oi);                                      \
      else if (direct && ring_nsr() == 3)                                                     \
        paged_decode_ring_kernel<GG, true, false, 3><<<grid, 256, 0, s>>>(                    \
            (const uint16_t*)q, q_stride, (uint16_t*)k_cache, (uint16_t*)v_cache,             \
            block_tables, maxb, context_lens, tmp_out, tmp_ml, Hkv, max_parts, scale,         \
            (uint16_t*)out, out_stride, FusedQKV{}, oi);                                      \
      else if (direct)                                                                        \
        paged_decode_ring_kernel<GG, true><<<grid, 256, 0, s>>>(                              \
            (const uint16_t*)q, q_stride, (uint16_t*)k_cache, (uint16_t*)v_cache,             \
            block_tables, maxb, context_lens, tmp_out, tmp_ml, Hkv, max_parts, scale,         \
            (uint16_t*)out, out_stride, FusedQKV{}, oi);                                          \
      else                                                                                    \
        paged_decode_ring_kernel<GG, false><<<grid, 256, 0, s>>>(                             \
            (const uint16_t*)q, q_stride, (uint16_t*)k_cache, (uint16_t*)v_cache,             \
            block_tables, maxb, context_lens, tmp_out, tmp_ml, Hkv, max_parts, scale,         \
            (uint16_t*)out, out_stride, FusedQKV{}, oi);                                          \
    } while (0)
    switch (G) {
      case 1: DRING(1); break;
      case 2: DRING(2); break;
      case 4: DRING(4); break;
      case 8: DRING(8); break;
      default: return -1;
    }
#undef DRING
    if (!direct)
      paged_decode_reduce<128><<<dim3(Hq, B), 128, 0, s>>>(tmp_out, tmp_ml, context_lens,
                                                           (uint16_t*)out, out_stride, Hq,
                                                           max_parts);
    DOCQA_CHECK_LAUNCH();
    return 0;
  }
  switch (G) {
    case 1: DEC(1, 4); break;
    case 2: DEC(2, 4); break;
    case 4:
      if (u_env == 2) DEC(4, 2);
      else DEC(4, 4);
      break;
    case 8: DEC(8, 1); break;
    default: return -1;
  }
#undef DEC
#undef DEC_K
  if (!direct)
    paged_decode_reduce<128><<<dim3(Hq, B), 128, 0, s>>>(tmp_out, tmp_ml, context_lens,
                                                         (uint16_t*)out, out_stride, Hq,
                                                         max_parts);
  DOCQA_CHECK_LAUNCH();
  return 0;
}

// splits per (sequence, kv head): about `target` workgroups in total (default 512 = two
// per CU, all resident at once at this kernel's 3 waves/SIMD -- a second partial round of
// workgroups would leave most CUs idle at the tail), at most 64 splits
int docqa_decode_splits(int B, int Hkv, int max_context) {
  static int target = [] {
    const char* e = getenv("DOCQA_DECODE_WG_TARGET");
    const int v = e ? atoi(e) : 0;
    return v > 0 ? v : 512;
  }();
  int s = (target + B * Hkv - 1) / (B * Hkv);
  const int by_len = (max_context + kMinChunk - 1) / kMinChunk;
  if (s > by_len) s = by_len;
  if (s > 64) s = 64;
  return s < 1 ? 1 : s;
}

// Fused decode step attention: QKV split-K partials [S, B, (Hq + 2 Hkv) * 128] fp32 ->
// RoPE + paged-cache write of the new token + attention (ring kernel, FUSED mode).
int docqa_paged_decode_fused(const float* P, int S, const int* positions, const float* cos_sin,
                             const int* slot_mapping, void* k_cache, void* v_cache,
                             const int* block_tables, int maxb, const int* context_lens, void* out,
                             int out_stride, float* tmp_out, float* tmp_ml, int B, int Hq, int Hkv,
                             int BS, int max_parts, float scale, const int* order, hipStream_t s,
                             int* tick) {
  if (B == 0) return 0;
  if (BS != 64 || maxb > 256 || Hq % Hkv != 0 || S < 1) return -1;
  CascadeIn oi{};
  oi.order = order;
  const int G = Hq / Hkv;
  dim3 grid(Hkv, B, max_parts);   // partitions slowest: see kDecodeGridNote
  const bool direct = max_parts == 1;
  FusedQKV fz{P, S, positions, cos_sin, slot_mapping, Hq};
  const bool last = tick && !direct && max_parts <= 64;
#define DFUSED(GG)                                                                            \
  do {                                                                                        \
    if (last)                                                                                 \
      paged_decode_ring_kernel<GG, false, true, 4, true><<<grid, 256, 0, s>>>(                \
          nullptr, 0, (uint16_t*)k_cache, (uint16_t*)v_cache, block_tables, maxb,             \
          context_lens, tmp_out, tmp_ml, Hkv, max_parts, scale, (uint16_t*)out, out_stride, fz, oi, \
          tick);                                                                              \
    else if (direct)                                                                          \
      paged_decode_ring_kernel<GG, true, true><<<grid, 256, 0, s>>>(                          \
          nullptr, 0, (uint16_t*)k_cache, (uint16_t*)v_cache, block_tables, maxb,             \
          context_lens, tmp_out, tmp_ml, Hkv, max_parts, scale, (uint16_t*)out, out_stride, fz, oi); \
    else                                                                                      \
      paged_decode_ring_kernel<GG, false, true><<<grid, 256, 0, s>>>(                         \
          nullptr, 0, (uint16_t*)k_cache, (uint16_t*)v_cache, block_tables, maxb,             \
          context_lens, tmp_out, tmp_ml, Hkv, max_parts, scale, (uint16_t*)out, out_stride, fz, oi); \
  } while (0)
  switch (G) {
    case 1: DFUSED(1); break;
    case 2: DFUSED(2); break;
    case 4: DFUSED(4); break;
    case 8: DFUSED(8); break;
    default: return -1;
  }
#undef DFUSED
  if (!direct && !last)
    paged_decode_reduce<128><<<dim3(Hq, B), 128, 0, s>>>(tmp_out, tmp_ml, context_lens,
                                                         (uint16_t*)out, out_stride, Hq, max_parts);
  DOCQA_CHECK_LAUNCH();
  return 0;
}

int docqa_cascade_prefix(const void* qkv, int row_stride, int rows, int Hq, int Hkv, float scale,
                         const void* k_cache, const void* v_cache, const int* prefix_table,
                         const int* plen, int BS, int nchunk, float* acc, float* ml,
                         const int* positions, const float* cos_sin, hipStream_t s);
int docqa_rope_cache(void* qkv, const int* positions, const float* cos_sin,
                     const int* slot_mapping, void* k_cache, void* v_cache, int T, int Hq,
                     int Hkv, int D, int row_stride, int BS, hipStream_t s);

// Cascade decode with the step's RoPE + paged-cache write fused in (the batch sizes whose
// QKV projection runs on the library GEMM, > 192 rows): the prefix kernel rotates the
// query rows as it loads them, the ring kernel (FUSED mode, bf16 source) rotates its
// queries, writes the new token's rotated K and V to the cache and attends to it from
// registers -- one launch and one QKV round trip fewer per layer.  Shapes the fused ring
// does not cover (split partitions, MFMA decode) fall back to rope_cache + cascade.
int docqa_paged_decode_cascade(const void* q, int q_stride, void* k_cache, void* v_cache,
                               const int* block_tables, int maxb, const int* context_lens, void* out,
                               int out_stride, float* tmp_out, float* tmp_ml, int B, int Hq, int Hkv,
                               int BS, int max_parts, float scale, const int* prefix_table,
                               const int* plen, int nchunk, float* pacc, float* pml, const int* order,
                               hipStream_t s);

int docqa_paged_decode_cascade_rope(void* qkv, int q_stride, const int* positions,
                                    const float* cos_sin, const int* slot_mapping, void* k_cache,
                                    void* v_cache, const int* block_tables, int maxb,
                                    const int* context_lens, void* out, int out_stride,
                                    float* tmp_out, float* tmp_ml, int B, int Hq, int Hkv, int BS,
                                    int max_parts, float scale, const int* prefix_table,
                                    const int* plen, int nchunk, float* pacc, float* pml,
                                    const int* order, hipStream_t s) {
  if (B == 0) return 0;
  if (BS != 64 || maxb > 256 || Hq != 4 * Hkv || nchunk < 1 || nchunk > kCascadeMaxChunks) return -1;
  if (max_parts != 1 || mfma_decode_on(Hq / Hkv)) {
    const int rc = docqa_rope_cache(qkv, positions, cos_sin, slot_mapping, k_cache, v_cache, B, Hq, Hkv,
                                    128, q_stride, BS, s);
    if (rc) return rc;
    return docqa_paged_decode_cascade(qkv, q_stride, k_cache, v_cache, block_tables, maxb, context_lens, out,
                                      out_stride, tmp_out, tmp_ml, B, Hq, Hkv, BS, max_parts, scale,
                                      prefix_table, plen, nchunk, pacc, pml, order, s);
  }
  int rc = docqa_cascade_prefix(qkv, q_stride, B, Hq, Hkv, scale, k_cache, v_cache, prefix_table, plen,
                                BS, nchunk, pacc, pml, positions, cos_sin, s);
  if (rc) return rc;
  const CascadeIn ci{pacc, pml, plen, nchunk, order};
  FusedQKV fz{nullptr, 0, positions, cos_sin, slot_mapping, Hq};
  fz.qkv = (const uint16_t*)qkv;
  fz.q_stride = q_stride;
  dim3 grid(Hkv, B, 1);
  if (ring_nsr() == 4)
    paged_decode_ring_kernel<4, true, true, 4><<<grid, 256, 0, s>>>(
        nullptr, 0, (uint16_t*)k_cache, (uint16_t*)v_cache, block_tables, maxb, context_lens, tmp_out,
        tmp_ml, Hkv, 1, scale, (uint16_t*)out, out_stride, fz, ci);
  else
    paged_decode_ring_kernel<4, true, true, 3><<<grid, 256, 0, s>>>(
        nullptr, 0, (uint16_t*)k_cache, (uint16_t*)v_cache, block_tables, maxb, context_lens, tmp_out,
        tmp_ml, Hkv, 1, scale, (uint16_t*)out, out_stride, fz, ci);
  DOCQA_CHECK_LAUNCH();
  return 0;
}

// Cascade decode attention (docqa_cascade.h): MFMA prefix partials over the shared prompt
// prefix [0, *plen) for all B rows, then the ring kernel over each suffix [*plen, L) with
// the prefix partials merged before normalisation.  q: post-RoPE rows of the packed QKV
// buffer (row stride q_stride), the step's new K/V already in the cache.
int docqa_paged_decode_cascade(const void* q, int q_stride, void* k_cache, void* v_cache,
                               const int* block_tables, int maxb, const int* context_lens, void* out,
                               int out_stride, float* tmp_out, float* tmp_ml, int B, int Hq, int Hkv,
                               int BS, int max_parts, float scale, const int* prefix_table,
                               const int* plen, int nchunk, float* pacc, float* pml, const int* order,
                               hipStream_t s) {
  if (B == 0) return 0;
  if (BS != 64 || maxb > 256 || Hq != 4 * Hkv || nchunk < 1 || nchunk > kCascadeMaxChunks) return -1;
  int rc = docqa_cascade_prefix(q, q_stride, B, Hq, Hkv, scale, k_cache, v_cache, prefix_table, plen,
                                BS, nchunk, pacc, pml, nullptr, nullptr, s);
  if (rc) return rc;
  const CascadeIn ci{pacc, pml, plen, nchunk, order};
  dim3 grid(Hkv, B, max_parts);   // partitions slowest: see kDecodeGridNote
  if (mfma_decode_on(Hq / Hkv)) {
    if (max_parts == 1 && Hkv % 2 == 0 && hpw_knob() == 2)
      paged_decode_mfma_kernel<4, true, 2><<<dim3(Hkv / 2, B, 1), 256, 0, s>>>(
          (const uint16_t*)q, q_stride, (const uint16_t*)k_cache, (const uint16_t*)v_cache, block_tables, maxb,
          context_lens, tmp_out, tmp_ml, Hkv, max_parts, scale, (uint16_t*)out, out_stride, ci);
    else if (max_parts == 1 && mfma_nsr() == 3)
      paged_decode_mfma_kernel<4, true, 1, 3><<<grid, 256, 0, s>>>(
          (const uint16_t*)q, q_stride, (const uint16_t*)k_cache, (const uint16_t*)v_cache, block_tables, maxb,
          context_lens, tmp_out, tmp_ml, Hkv, max_parts, scale, (uint16_t*)out, out_stride, ci);
    else if (max_parts == 1)
      paged_decode_mfma_kernel<4, true><<<grid, 256, 0, s>>>(
          (const uint16_t*)q, q_stride, (const uint16_t*)k_cache, (const uint16_t*)v_cache, block_tables, maxb,
          context_lens, tmp_out, tmp_ml, Hkv, max_parts, scale, (uint16_t*)out, out_stride, ci);
    else {
      paged_decode_mfma_kernel<4, false><<<grid, 256, 0, s>>>(
          (const uint16_t*)q, q_stride, (const uint16_t*)k_cache, (const uint16_t*)v_cache, block_tables, maxb,
          context_lens, tmp_out, tmp_ml, Hkv, max_parts, scale, (uint16_t*)out, out_stride, ci);
      paged_decode_reduce<128><<<dim3(Hq, B), 128, 0, s>>>(tmp_out, tmp_ml, context_lens, (uint16_t*)out,
                                                           out_stride, Hq, max_parts, ci);
    }
  } else if (max_parts == 1 && ring_nsr() == 2)
    paged_decode_ring_kernel<4, true, false, 2><<<grid, 256, 0, s>>>(
        (const uint16_t*)q, q_stride, (uint16_t*)k_cache, (uint16_t*)v_cache, block_tables, maxb,
        context_lens, tmp_out, tmp_ml, Hkv, max_parts, scale, (uint16_t*)out, out_stride, FusedQKV{}, ci);
  else if (max_parts == 1 && ring_nsr() == 3)
    paged_decode_ring_kernel<4, true, false, 3><<<grid, 256, 0, s>>>(
        (const uint16_t*)q, q_stride, (uint16_t*)k_cache, (uint16_t*)v_cache, block_tables, maxb,
        context_lens, tmp_out, tmp_ml, Hkv, max_parts, scale, (uint16_t*)out, out_stride, FusedQKV{}, ci);
  else if (max_parts == 1)
    paged_decode_ring_kernel<4, true><<<grid, 256, 0, s>>>(
        (const uint16_t*)q, q_stride, (uint16_t*)k_cache, (uint16_t*)v_cache, block_tables, maxb,
        context_lens, tmp_out, tmp_ml, Hkv, max_parts, scale, (uint16_t*)out, out_stride, FusedQKV{}, ci);
  else {
    paged_decode_ring_kernel<4, false><<<grid, 256, 0, s>>>(
        (const uint16_t*)q, q_stride, (uint16_t*)k_cache, (uint16_t*)v_cache, block_tables, maxb,
        context_lens, tmp_out, tmp_ml, Hkv, max_parts, scale, (uint16_t*)out, out_stride, FusedQKV{}, ci);
    paged_decode_reduce<128><<<dim3(Hq, B), 128, 0, s>>>(tmp_out, tmp_ml, context_lens, (uint16_t*)out,
                                                         out_stride, Hq, max_parts, ci);
  }
  DOCQA_CHECK_LAUNCH();
  return 0;
}
