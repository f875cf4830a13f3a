// attn_decode.hip -- paged GQA decode attention (one new query token per sequence),
// split-K over the context ("flash-decoding") for the Llama-3 generator.
//
// Cache layout: k_cache/v_cache [num_blocks, Hkv, BS, D] bf16; block_tables [B, maxb].
//
// Kernel 1, grid (max_parts, Hkv, B), 256 threads: one workgroup owns one KV head of one
// sequence over a P=256-token partition and serves all G = Hq/Hkv query heads of that
// group, so every K/V byte is read from HBM exactly once per step (decode attention is
// a KV-streaming op: ~4 FLOP/byte, far below the VALU roof -- no MFMA needed;
// cdna_hip_programming.md App. B "Attention decode": K/V straight to VGPRs).
//   lane = 16 lanes x 16 B per 256-B K row (D=128), so one wave instruction reads four
//   consecutive tokens = 1 KiB contiguous in the (block, head) slab.
//   phase 1: scores s[g][t] = q_g . k_t  (16-lane shuffle reduce) -> LDS
//   phase 2: per-head max / exp2 / sum over the partition (LDS, whole workgroup)
//   phase 3: acc[g][8 dims] += p[g][t] * v_t, reduced over token groups and waves
// Output per partition: un-normalised acc + (max, sum) in fp32 workspaces.
// Kernel 2, grid (Hq, B): log-sum-exp merge of the partitions -> bf16 [B, Hq, D].
//
// Graph capture: the grid is sized for the maximum context, so a captured replay works
// for any context <= max; partitions past the sequence's length exit immediately.
//
// Reference parity: decode attention is inside llama.cpp behind Ollama
// (llm-qa/main.py:69, greedy decode loop of RetrievalQA.invoke at llm-qa/main.py:117).
#include "docqa_common.h"
#include <float.h>

using namespace docqa;

constexpr int kPart = 256;   // tokens per partition
constexpr float kLog2e = 1.4426950408889634f;

template <int G, int D>
__global__ __launch_bounds__(256) void paged_decode_kernel(
    const uint16_t* __restrict__ q, int q_stride, const uint16_t* __restrict__ k_cache,
    const uint16_t* __restrict__ v_cache, const int* __restrict__ block_tables, int maxb,
    const int* __restrict__ context_lens, float* __restrict__ tmp_out,
    float* __restrict__ tmp_ml, int Hkv, int BS, int log2BS, int max_parts, float scale) {
  static_assert(D == 128, "decode kernel is specialised for head_dim 128");
  const int part = blockIdx.x, kvh = blockIdx.y, b = blockIdx.z;
  const int L = context_lens[b];
  const int start = part * kPart;
  if (start >= L) return;
  const int end = min(L, start + kPart);
  const int n = end - start;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int chunk = lane & 15;        // 8-dim chunk of the head
  const int tg = lane >> 4;           // token sub-group inside the wave (0..3)

  __shared__ float s_p[G][kPart];
  __shared__ float s_red[4][G][D];
  __shared__ float s_stat[2][4][G];

  // q for the G heads of this group, pre-scaled so exp2 can be used
  float qv[G][8];
  const float qs = scale * kLog2e;
#pragma unroll
  for (int g = 0; g < G; ++g) {
    const uint16_t* qp = q + (size_t)b * q_stride + (size_t)(kvh * G + g) * D;
    unpack8(reinterpret_cast<const uint4*>(qp)[chunk], qv[g]);
#pragma unroll
    for (int j = 0; j < 8; ++j) qv[g][j] *= qs;
  }
  const int* bt = block_tables + (size_t)b * maxb;
  const size_t head_off = (size_t)kvh * BS * D;
  const size_t blk_stride = (size_t)Hkv * BS * D;

  // ---- phase 1: scores.  Each wave covers 4 tokens per step, 16 tokens per WG step.
  for (int base = wave * 4; base < n; base += 16 * 2) {
    uint4 kv[2];
    int tok[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      tok[u] = base + u * 16 + tg;
      if (tok[u] < n) {
        const int t = start + tok[u];
        const int blk = bt[t >> log2BS];
        const int off = t & (BS - 1);
        kv[u] = reinterpret_cast<const uint4*>(k_cache + blk * blk_stride + head_off +
                                               (size_t)off * D)[chunk];
      }
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      float kf[8];
      if (tok[u] < n) unpack8(kv[u], kf);
      else {
#pragma unroll
        for (int j = 0; j < 8; ++j) kf[j] = 0.f;
      }
#pragma unroll
      for (int g = 0; g < G; ++g) {
        float d = 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) d += qv[g][j] * kf[j];
        d = group_sum<16>(d);
        if (chunk == 0 && tok[u] < n) s_p[g][tok[u]] = d;
      }
    }
  }
  __syncthreads();

  // ---- phase 2: softmax statistics per head (log2 domain)
  float m[G], l[G];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    float mx = -FLT_MAX;
    for (int i = tid; i < n; i += 256) mx = fmaxf(mx, s_p[g][i]);
    mx = wave_max(mx);
    if (lane == 0) s_stat[0][wave][g] = mx;
  }
  __syncthreads();
#pragma unroll
  for (int g = 0; g < G; ++g)
    m[g] = fmaxf(fmaxf(s_stat[0][0][g], s_stat[0][1][g]), fmaxf(s_stat[0][2][g], s_stat[0][3][g]));
#pragma unroll
  for (int g = 0; g < G; ++g) {
    float sum = 0.f;
    for (int i = tid; i < n; i += 256) {
      const float p = exp2f(s_p[g][i] - m[g]);
      s_p[g][i] = p;
      sum += p;
    }
    sum = wave_sum(sum);
    if (lane == 0) s_stat[1][wave][g] = sum;
  }
  __syncthreads();
#pragma unroll
  for (int g = 0; g < G; ++g)
    l[g] = s_stat[1][0][g] + s_stat[1][1][g] + s_stat[1][2][g] + s_stat[1][3][g];

  // ---- phase 3: P.V
  float acc[G][8];
#pragma unroll
  for (int g = 0; g < G; ++g)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[g][j] = 0.f;
  for (int base = wave * 4; base < n; base += 16 * 2) {
    uint4 vv[2];
    int tok[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      tok[u] = base + u * 16 + tg;
      if (tok[u] < n) {
        const int t = start + tok[u];
        const int blk = bt[t >> log2BS];
        const int off = t & (BS - 1);
        vv[u] = reinterpret_cast<const uint4*>(v_cache + blk * blk_stride + head_off +
                                               (size_t)off * D)[chunk];
      }
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      if (tok[u] < n) {
        float vf[8];
        unpack8(vv[u], vf);
#pragma unroll
        for (int g = 0; g < G; ++g) {
          const float p = s_p[g][tok[u]];
#pragma unroll
          for (int j = 0; j < 8; ++j) acc[g][j] += p * vf[j];
        }
      }
    }
  }
  // reduce over the 4 token sub-groups of the wave (lanes differing in bits 4,5)
#pragma unroll
  for (int g = 0; g < G; ++g)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float v = acc[g][j];
      v += __shfl_xor(v, 16, 64);
      v += __shfl_xor(v, 32, 64);
      acc[g][j] = v;
    }
  if (tg == 0) {
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
      for (int j = 0; j < 8; ++j) s_red[wave][g][chunk * 8 + j] = acc[g][j];
  }
  __syncthreads();
  // write partition result: G*D values, 256 threads
  const int nparts_stride = max_parts;
  for (int i = tid; i < G * D; i += 256) {
    const int g = i / D, d = i % D;
    const float v = s_red[0][g][d] + s_red[1][g][d] + s_red[2][g][d] + s_red[3][g][d];
    const int h = kvh * G + g;
    const size_t o = (((size_t)b * (Hkv * G) + h) * nparts_stride + part);
    tmp_out[o * D + d] = v;
    if (d == 0) {
      tmp_ml[o * 2 + 0] = m[g];
      tmp_ml[o * 2 + 1] = l[g];
    }
  }
}

template <int D>
__global__ __launch_bounds__(D) void paged_decode_reduce(const float* __restrict__ tmp_out,
                                                         const float* __restrict__ tmp_ml,
                                                         const int* __restrict__ context_lens,
                                                         uint16_t* __restrict__ out,
                                                         int out_stride, int Hq, int max_parts) {
  const int h = blockIdx.x, b = blockIdx.y, d = threadIdx.x;
  const int L = context_lens[b];
  const int np = (L + kPart - 1) / kPart;
  const size_t base = ((size_t)b * Hq + h) * max_parts;
  float M = -FLT_MAX;
  for (int p = 0; p < np; ++p) M = fmaxf(M, tmp_ml[(base + p) * 2]);
  float num = 0.f, den = 0.f;
  for (int p = 0; p < np; ++p) {
    const float w = exp2f(tmp_ml[(base + p) * 2] - M);
    num += w * tmp_out[(base + p) * D + d];
    den += w * tmp_ml[(base + p) * 2 + 1];
  }
  out[(size_t)b * out_stride + (size_t)h * D + d] = f2bf(L > 0 ? num / den : 0.f);
}

int docqa_paged_decode(const void* q, int q_stride, const void* k_cache, const void* v_cache,
                       const int* block_tables, int maxb, const int* context_lens, void* out,
                       int out_stride, float* tmp_out, float* tmp_ml, int B, int Hq, int Hkv,
                       int D, int BS, int max_parts, float scale, hipStream_t s) {
  if (B == 0) return 0;
  if (D != 128 || (BS & (BS - 1)) != 0 || Hq % Hkv != 0) return -1;
  int log2BS = 0;
  while ((1 << log2BS) < BS) ++log2BS;
  const int G = Hq / Hkv;
  dim3 grid(max_parts, Hkv, B);
#define DEC(GG)                                                                             \
  paged_decode_kernel<GG, 128><<<grid, 256, 0, s>>>(                                        \
      (const uint16_t*)q, q_stride, (const uint16_t*)k_cache, (const uint16_t*)v_cache,     \
      block_tables, maxb, context_lens, tmp_out, tmp_ml, Hkv, BS, log2BS, max_parts, scale)
  switch (G) {
    case 1: DEC(1); break;
    case 2: DEC(2); break;
    case 4: DEC(4); break;
    case 8: DEC(8); break;
    default: return -1;
  }
#undef DEC
  paged_decode_reduce<128><<<dim3(Hq, B), 128, 0, s>>>(tmp_out, tmp_ml, context_lens,
                                                       (uint16_t*)out, out_stride, Hq,
                                                       max_parts);
  DOCQA_CHECK_LAUNCH();
  return 0;
}

int docqa_decode_part_tokens() { return kPart; }
