// attn_prefill.hip -- causal varlen flash-attention forward on MFMA for the Llama-3
// prefill (and, with causal=0, the bidirectional BERT encoders).
//
// Structure (cdna_hip_programming.md App. B "Fused attention prefill", §3 "An
// accumulator tile as the next MFMA's operand", T10 tr-read, T2 swizzle, T14 split):
//  * workgroup = G query heads (one GQA group sharing a KV head) x WPH waves per head,
//    each wave owning 32 query rows of one head.  KV tiles of 64 keys are staged
//    HBM -> registers -> LDS once per workgroup and shared by all G x WPH waves, so with
//    GQA (Llama-3: 4 query heads per KV head) every K/V tile is fetched once per group
//    instead of once per query head: the prefix-cached RAG prefill (~140 new tokens
//    against ~570 cached keys) was bound by exactly that re-fetch.  Encoders (no GQA):
//    G = 1, WPH = 4 (128 rows of one head).
//  * swapped QK^T: X = S^T = K . Q^T on v_mfma_f32_32x32x16_bf16, so each lane holds one
//    query's scores for 16 keys in registers -> the row max / row sum of the online
//    softmax are in-register plus one cross-half shuffle (no LDS round trip for P).
//  * O^T = V^T . P^T: P^T is exactly X converted to bf16 (the accumulator IS the next
//    MFMA's B operand, no lane movement); V^T fragments come from the row-major V tile
//    with ds_read_b64_tr_b16 (hardware transpose read), XOR-swizzled so the reads are
//    bank-conflict-free.  K is read row-wise with ds_read_b128, swizzled chunk ^ (row&15).
//  * next KV tile's global loads are issued before the current tile's MFMAs and written
//    to LDS after the trailing barrier (async-STAGE split).
//
// Q/K/V are read straight from the packed post-RoPE QKV projection buffer
// [T, (Hq + 2*Hkv) * D]; output is [T, Hq, D] (row stride o_stride).
//
// Reference parity: prefill is inside llama.cpp behind Ollama (llm-qa/main.py:69,117)
// and the MiniLM encoder attention inside sentence-transformers
// (semantic-indexer/indexer.py:37).
#include "docqa_common.h"
#include <stdlib.h>
#include "docqa_cascade.h"
#include <float.h>

using namespace docqa;

namespace {
constexpr int QB = 128;   // query rows per workgroup
constexpr int KB = 64;    // keys per tile
constexpr int kPrefillMaxBT = 512;   // block ids of a paged sequence staged in LDS (else read per tile)
constexpr float kLog2e = 1.4426950408889634f;

typedef __attribute__((address_space(3))) i16x4 lds_i16x4;

// element offset of 16-B chunk `ch` of row `row` in the K / V tiles (XOR swizzles, see
// header; for D=128 both are bank-conflict-free for their read pattern)
template <int D>
__device__ __forceinline__ int k_off(int row, int ch) {
  return row * D + ((ch ^ (row & (D / 8 - 1))) << 3);
}
template <int D>
__device__ __forceinline__ int v_off(int row, int ch) {
  return row * D + ((ch ^ (((row & 3) << 2) & (D / 8 - 1))) << 3);
}

// Paged K/V source for prefix-cached prefill: keys [0, ctx_start[b]) were computed by an
// earlier request (shared prompt prefix, prefix-cache hit) and keys
// [ctx_start[b], ctx_start[b] + L) were just written by the fused RoPE/cache kernel, so
// every key of the sequence is read through the block table from the paged cache.
struct PagedKV {
  const uint16_t* k;
  const uint16_t* v;
  const int* block_tables;
  int maxb;
  const int* ctx_start;
  int BS;
  int log2BS;
};

// PFX (cascade decode, docqa_cascade.h): the query rows are the B sequences of a decode
// step (one new token each, rows of the packed QKV buffer), the keys are one chunk
// (blockIdx.y) of the prompt prefix they all share, read through the shared block table
// (row 0 of pk.block_tables), no causal mask; the epilogue writes the un-normalised
// accumulator and (max, sum) of the chunk instead of normalised bf16 rows.
// G = 4, WPH = 1 (32-row tiles, 4 waves): at most 256 VGPRs so that two workgroups share a
// CU and one's prologue (Q, block ids, first K/V tile: three dependent round trips) runs
// under the other's main loop -- unbounded, hipcc spends ~300 and keeps one per CU
template <int D, bool CAUSAL, bool PAGED, int G, int WPH, bool PFX = false>
__global__ __launch_bounds__(64 * G * WPH, (G == 4 && WPH == 1) ? 2 : 1) void flash_prefill_kernel(
    const uint16_t* __restrict__ qkv, int row_stride, const int* __restrict__ cu_seqlens,
    uint16_t* __restrict__ out, int o_stride, int Hq, int Hkv, float scale, PagedKV pk,
    CascadeOut co) {
  constexpr int NT = 64 * G * WPH;              // threads
  constexpr int QBW = 32 * WPH;                 // query rows per workgroup
  __shared__ __attribute__((aligned(16))) uint16_t smem[2 * KB * D];
  // PAGED: the sequence's block ids, read once into LDS -- the per-tile block-table load
  // was a dependent global round trip ahead of every tile's K/V loads (RAG shapes: 458 ->
  // 442 us; an LDS-DMA ring for the tiles was slower still, profiles/r5_prefill_attn_ring_ab.log)
  __shared__ int s_bt[PAGED ? kPrefillMaxBT : 1];
  uint16_t* sK = smem;
  uint16_t* sV = smem + KB * D;

  // grid (heads, sequences, q-tiles): workgroups are dealt to the 8 XCDs round-robin by
  // linear id, so with q-tiles fastest (the old (q-tile, head, seq) grid) XCD x received
  // q-tile x of every sequence -- in a RAG prefill most sequences have 1-2 tiles of new
  // tokens and one long prompt sets the grid to 8, so XCDs 2..7 got only empty tiles and
  // the work ran on two XCDs (4x slower on the bench's real batches).  Heads fastest
  // spreads every tile over all XCDs, and the empty high tiles are dispatched last.
  // q-tiles in reverse: under the causal mask the last tile of a long prompt attends to
  // the most keys, so the heaviest workgroups are dispatched first (LPT) and the empty
  // tiles past short prompts exit at once
  const int hb = blockIdx.x, b = blockIdx.y, qt = gridDim.z - 1 - blockIdx.z;
  int seq0, L, kv_beg = 0, pfx_end = 0;
  if constexpr (PFX) {
    seq0 = 0;
    L = co.rows;
    const int Lp = *co.plen;
    const int ck = cascade_chunk(Lp, co.nchunk);
    kv_beg = b * ck;                              // this chunk's keys: [kv_beg, pfx_end)
    if (kv_beg >= Lp) return;
    pfx_end = min(Lp, kv_beg + ck);
  } else {
    seq0 = cu_seqlens[b];
    L = cu_seqlens[b + 1] - seq0;
  }
  const int q_start = qt * QBW;
  if (q_start >= L) return;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // G > 1: blockIdx.x is the KV head and wave / WPH picks the query head of its group
  const int h = G > 1 ? hb * G + wave / WPH : hb;
  const int kvh = G > 1 ? hb : h / (Hq / Hkv);
  const int P0 = (PAGED && !PFX) ? pk.ctx_start[b] : 0;   // absolute position of query row 0
  const int Lk = PFX ? pfx_end : P0 + L;         // keys visible to this sequence

  const int l32 = lane & 31, hh = lane >> 5;
  const int q_wave = q_start + (wave % WPH) * 32;   // first query row of this wave
  const int my_q = q_wave + l32;                // this lane's query row (column of X)

  // ---- Q fragments (B operand of S^T = K Q^T): lane holds Q[my_q][16ks + 8hh + j]
  constexpr int NKS = D / 16;   // k-steps of the QK^T product
  constexpr int NDT = D / 32;   // 32-wide dim tiles of O^T
  constexpr int NCH = D / 8;    // 16-B chunks per row
  constexpr int CPT = (KB * NCH + NT - 1) / NT;  // staged chunks per thread per tensor
  bf16x8 qf[NKS];
  {
    const bool ok = my_q < L;
    const uint16_t* qp = qkv + (size_t)(seq0 + (ok ? my_q : 0)) * row_stride + (size_t)h * D;
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
      uint4 v = ok ? *reinterpret_cast<const uint4*>(qp + ks * 16 + hh * 8) : make_uint4(0, 0, 0, 0);
      qf[ks] = *reinterpret_cast<bf16x8*>(&v);
    }
    if constexpr (PFX && D == 128) {
      // fused RoPE (rotate-half): dim d of fragment ks pairs with d + 64 of fragment ks + 4,
      // both in this lane; fp32 rotate, bf16 round -- as rope_cache would have stored them
      if (co.cos_sin && ok) {
        const float* cs = co.cos_sin + (size_t)co.positions[my_q] * D;
#pragma unroll
        for (int ks = 0; ks < NKS / 2; ++ks)
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const int d = ks * 16 + hh * 8 + j;
            const float c = cs[d], sn = cs[64 + d];
            const float x1 = (float)qf[ks][j], x2 = (float)qf[ks + 4][j];
            qf[ks][j] = (__bf16)(x1 * c - x2 * sn);
            qf[ks + 4][j] = (__bf16)(x2 * c + x1 * sn);
          }
      }
    }
  }

  f32x16 o[NDT];
#pragma unroll
  for (int i = 0; i < NDT; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) o[i][r] = 0.f;
  float m_run = -FLT_MAX, l_run = 0.f;
  const float sl2 = scale * kLog2e;

  const int kv_end = CAUSAL ? min(Lk, P0 + q_start + QBW) : Lk;
  const int ntiles = (kv_end + KB - 1) / KB;
  const int t_beg = kv_beg / KB;
  const uint16_t* kbase = qkv + (size_t)seq0 * row_stride + (size_t)(Hq + kvh) * D;
  const uint16_t* vbase = qkv + (size_t)seq0 * row_stride + (size_t)(Hq + Hkv + kvh) * D;

  // staging: KB rows x NCH chunks per tensor, CPT per thread per tensor
  uint4 rk[CPT], rv[CPT];
  // block ids the keys [0, Lk) need; PFX: the shared prefix table (row 0, pk.maxb unset),
  // whose first ceil(Lk / BS) entries all exist (Lk <= the prefix length)
  const int nb_need = PAGED ? (Lk + pk.BS - 1) >> pk.log2BS : 0;
  const bool bt_lds = PAGED && nb_need <= kPrefillMaxBT && (PFX || nb_need <= pk.maxb);
  if constexpr (PAGED) {
    if (bt_lds) {
      const int* btr = pk.block_tables + (size_t)(PFX ? 0 : b) * pk.maxb;
      for (int i = tid; i < nb_need; i += NT) s_bt[i] = btr[i];
      __syncthreads();
    }
  }
  auto load_tile = [&](int t) {
#pragma unroll
    for (int i = 0; i < CPT; ++i) {
      const int idx = tid + NT * i;
      const int row = idx / NCH, ch = idx % NCH;
      const int key = t * KB + row;
      if (idx < KB * NCH && key < Lk) {
        if constexpr (PAGED) {
          const int blk = bt_lds ? s_bt[key >> pk.log2BS]
                                 : pk.block_tables[(size_t)(PFX ? 0 : b) * pk.maxb + (key >> pk.log2BS)];
          const size_t off = (((size_t)blk * Hkv + kvh) * pk.BS + (key & (pk.BS - 1))) * D + ch * 8;
          rk[i] = *reinterpret_cast<const uint4*>(pk.k + off);
          rv[i] = *reinterpret_cast<const uint4*>(pk.v + off);
        } else {
          rk[i] = *reinterpret_cast<const uint4*>(kbase + (size_t)key * row_stride + ch * 8);
          rv[i] = *reinterpret_cast<const uint4*>(vbase + (size_t)key * row_stride + ch * 8);
        }
      } else {
        rk[i] = make_uint4(0, 0, 0, 0);
        rv[i] = make_uint4(0, 0, 0, 0);
      }
    }
  };
  auto store_tile = [&]() {
#pragma unroll
    for (int i = 0; i < CPT; ++i) {
      const int idx = tid + NT * i;
      if (idx >= KB * NCH) break;
      const int row = idx / NCH, ch = idx % NCH;
      *reinterpret_cast<uint4*>(sK + k_off<D>(row, ch)) = rk[i];
      *reinterpret_cast<uint4*>(sV + v_off<D>(row, ch)) = rv[i];
    }
  };

  load_tile(t_beg);
  store_tile();
  __syncthreads();

  // tr-read lane geometry (see header): group gi = lane>>4, q = (lane&15)>>2, p = lane&3
  const int gi = lane >> 4, tq = (lane & 15) >> 2, tp = lane & 3;

  for (int t = t_beg; t < ntiles; ++t) {
    if (t + 1 < ntiles) load_tile(t + 1);
    const int kb = t * KB;
    // a wave whose rows all precede this tile's first key contributes nothing (causal),
    // nor does a wave whose rows all lie past the end of the sequence
    const bool active = (!CAUSAL || (kb <= P0 + q_wave + 31)) && q_wave < L;
    if (active) {
      // ---- S^T for the two 32-key sub-tiles
      f32x16 x[2];
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) {
#pragma unroll
        for (int r = 0; r < 16; ++r) x[kt][r] = 0.f;
        const int row = kt * 32 + l32;
#pragma unroll
        for (int ks = 0; ks < NKS; ++ks) {
          const bf16x8 a = *reinterpret_cast<const bf16x8*>(sK + k_off<D>(row, ks * 2 + hh));
          x[kt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, qf[ks], x[kt], 0, 0, 0);
        }
      }
      // ---- online softmax (log2 domain); keys on registers, query on lane
      float mx = -FLT_MAX;
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int key = kb + kt * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh;
          float s = x[kt][r] * sl2;
          const bool masked = (key >= Lk) || (CAUSAL && key > P0 + my_q);
          s = masked ? -FLT_MAX : s;
          x[kt][r] = s;
          mx = fmaxf(mx, s);
        }
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      const float m_new = fmaxf(m_run, mx);
      const bool dead = (m_new == -FLT_MAX);       // every key so far masked
      const float alpha = dead ? 1.f : exp2f(m_run - m_new);
      float rs = 0.f;
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float p = (dead || x[kt][r] == -FLT_MAX) ? 0.f : exp2f(x[kt][r] - m_new);
          x[kt][r] = p;
          rs += p;
        }
      rs += __shfl_xor(rs, 32, 64);
      l_run = l_run * alpha + rs;
      m_run = m_new;
#pragma unroll
      for (int i = 0; i < NDT; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) o[i][r] *= alpha;

      // ---- O^T += V^T P^T
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) {
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          bf16x8 pb;
#pragma unroll
          for (int j = 0; j < 8; ++j) pb[j] = (__bf16)x[kt][8 * s + j];
          const int krow = kt * 32 + 16 * s + 4 * hh + tq;  // key row for tr-read (first 4)
#pragma unroll
          for (int dt = 0; dt < NDT; ++dt) {
            const int col = dt * 32 + 16 * (gi & 1) + 4 * tp;  // dim column
            const int ch = col >> 3, half = (col & 7);
            const i16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                (lds_i16x4*)(sV + v_off<D>(krow, ch) + half));
            const i16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                (lds_i16x4*)(sV + v_off<D>(krow + 8, ch) + half));
            bf16x8 a;
            const __bf16* lp = reinterpret_cast<const __bf16*>(&lo);
            const __bf16* hp = reinterpret_cast<const __bf16*>(&hi);
#pragma unroll
            for (int j = 0; j < 4; ++j) { a[j] = lp[j]; a[4 + j] = hp[j]; }
            o[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, pb, o[dt], 0, 0, 0);
          }
        }
      }
    }
    __syncthreads();
    if (t + 1 < ntiles) {
      store_tile();
      __syncthreads();
    }
  }

  if constexpr (PFX) {   // chunk partial: un-normalised O and (max, sum) per (row, head)
    // O^T is lane = query row, registers = dims: stored straight, every 16-B store lands in
    // a different row (32 partial 128-B lines per instruction).  Transpose each 32-dim
    // slice through a per-wave LDS scratch instead (the K/V tiles are dead after the
    // loop's last barrier: 8 waves x 32 rows x 128 B fill the 32 KB; 16-B chunk c of row r
    // sits at chunk c ^ (r & 7), so the 8 rows of a store group hit distinct banks) and 8
    // lanes write one row's whole 128-B line.
    static_assert(G * WPH * 32 * 32 * 4 <= 2 * KB * D * 2, "PFX scratch");
    float* scr = reinterpret_cast<float*>(smem) + wave * 32 * 32;
    const int rr = lane >> 3, ch = lane & 7;
    float* ap = co.acc + ((size_t)b * L * Hq + h) * D;
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt) {
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4)
        *reinterpret_cast<float4*>(scr + l32 * 32 + (((2 * g4 + hh) ^ (l32 & 7)) << 2)) =
            make_float4(o[dt][4 * g4 + 0], o[dt][4 * g4 + 1], o[dt][4 * g4 + 2], o[dt][4 * g4 + 3]);
#pragma unroll
      for (int it = 0; it < 4; ++it) {
        const int q = q_wave + it * 8 + rr;
        const float4 v = *reinterpret_cast<const float4*>(scr + (it * 8 + rr) * 32 + ((ch ^ rr) << 2));
        if (q < L) *reinterpret_cast<float4*>(ap + (size_t)q * Hq * D + dt * 32 + ch * 4) = v;
      }
    }
    if (my_q < L && hh == 0)
      *reinterpret_cast<float2*>(co.ml + (((size_t)b * L + my_q) * Hq + h) * 2) = make_float2(m_run, l_run);
    return;
  }
  // ---- epilogue: O[q][dim] = O^T[dim][q] / l
  if (my_q < L) {
    const float inv = l_run > 0.f ? 1.f / l_run : 0.f;
    uint16_t* op = out + (size_t)(seq0 + my_q) * o_stride + (size_t)h * D;
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const int d0 = dt * 32 + 8 * g4 + 4 * hh;
        uint2 v;
        v.x = pack2(o[dt][4 * g4 + 0] * inv, o[dt][4 * g4 + 1] * inv);
        v.y = pack2(o[dt][4 * g4 + 2] * inv, o[dt][4 * g4 + 3] * inv);
        *reinterpret_cast<uint2*>(op + d0) = v;
      }
  }
}
}  // namespace

template <int D, int G, int WPH>
static void launch_prefill(dim3 grid, hipStream_t s, int causal, const void* qkv, int row_stride,
                           const int* cu, void* out, int o_stride, int Hq, int Hkv, float scale,
                           const PagedKV& pk) {
  const uint16_t* q = (const uint16_t*)qkv;
  uint16_t* o = (uint16_t*)out;
  constexpr int NT = 64 * G * WPH;
  const CascadeOut co{};
  if (pk.k) {
    flash_prefill_kernel<D, true, true, G, WPH><<<grid, NT, 0, s>>>(q, row_stride, cu, o, o_stride, Hq, Hkv, scale, pk, co);
  } else if (causal) {
    flash_prefill_kernel<D, true, false, G, WPH><<<grid, NT, 0, s>>>(q, row_stride, cu, o, o_stride, Hq, Hkv, scale, pk, co);
  } else {
    flash_prefill_kernel<D, false, false, G, WPH><<<grid, NT, 0, s>>>(q, row_stride, cu, o, o_stride, Hq, Hkv, scale, pk, co);
  }
}

// G = 4 query heads per KV head (Llama-3 GQA): one workgroup per (32 query rows, KV head)
// with 4 waves (DOCQA_PREFILL_WPH=2: 64 rows, 8 waves); otherwise one workgroup per (128
// rows, query head) with 4 waves
static int prefill_dispatch(hipStream_t s, int B, int max_len, int head_dim, int causal, const void* qkv,
                            int row_stride, const int* cu, void* out, int o_stride, int Hq, int Hkv,
                            float scale, const PagedKV& pk) {
  const bool gqa4 = head_dim == 128 && Hq == 4 * Hkv;
  // waves per query head: 1 (default; 32-row tiles, 4 waves, two workgroups per CU) or 2
  // (64-row tiles, 8 waves, one per CU).  RAG shapes: 443 -> 401 us on the bench mix, 134 ->
  // 84 us at 16 new tokens per prompt, bench prefill 428.7 -> 423.0 ms per batch
  // (profiles/r5_prefill_attn_wph_ab.log)
  static const int wph = [] {
    const char* e = getenv("DOCQA_PREFILL_WPH");
    return e && atoi(e) == 2 ? 2 : 1;
  }();
  // G = 8 (Llama-3-70B: 64 query heads over 8 KV heads; its TP-8 shard: 8 over 1): one
  // 8-wave workgroup per (32 rows, KV head), every K/V tile staged once for all 8 heads --
  // the per-query-head path below re-streamed each tile 8 times
  static const bool gqa8_on = [] {
    const char* e = getenv("DOCQA_PREFILL_GQA8");
    return !(e && atoi(e) == 0);
  }();
  const bool gqa8 = gqa8_on && head_dim == 128 && Hq == 8 * Hkv;
  if (gqa8) {
    dim3 grid(Hkv, B, (max_len + 31) / 32);
    launch_prefill<128, 8, 1>(grid, s, causal, qkv, row_stride, cu, out, o_stride, Hq, Hkv, scale, pk);
  } else if (gqa4 && wph == 1) {
    dim3 grid(Hkv, B, (max_len + 31) / 32);
    launch_prefill<128, 4, 1>(grid, s, causal, qkv, row_stride, cu, out, o_stride, Hq, Hkv, scale, pk);
  } else if (gqa4) {
    dim3 grid(Hkv, B, (max_len + 63) / 64);
    launch_prefill<128, 4, 2>(grid, s, causal, qkv, row_stride, cu, out, o_stride, Hq, Hkv, scale, pk);
  } else {
    dim3 grid(Hq, B, (max_len + QB - 1) / QB);
    switch (head_dim) {
      case 32: launch_prefill<32, 1, 4>(grid, s, causal, qkv, row_stride, cu, out, o_stride, Hq, Hkv, scale, pk); break;
      case 64: launch_prefill<64, 1, 4>(grid, s, causal, qkv, row_stride, cu, out, o_stride, Hq, Hkv, scale, pk); break;
      case 128: launch_prefill<128, 1, 4>(grid, s, causal, qkv, row_stride, cu, out, o_stride, Hq, Hkv, scale, pk); break;
      default: return -1;
    }
  }
  DOCQA_CHECK_LAUNCH();
  return 0;
}

int docqa_flash_prefill(const void* qkv, int row_stride, const int* cu_seqlens, void* out,
                        int o_stride, int B, int max_len, int Hq, int Hkv, int head_dim,
                        float scale, int causal, hipStream_t s) {
  if (B == 0 || max_len == 0) return 0;
  if (Hq % Hkv != 0) return -1;
  PagedKV pk{nullptr, nullptr, nullptr, 0, nullptr, 1, 0};
  return prefill_dispatch(s, B, max_len, head_dim, causal, qkv, row_stride, cu_seqlens, out, o_stride, Hq,
                          Hkv, scale, pk);
}

// Causal prefill of new tokens whose keys (prefix + new) live in the paged cache.
int docqa_flash_prefill_paged(const void* qkv, int row_stride, const int* cu_seqlens, void* out,
                              int o_stride, int B, int max_len, int Hq, int Hkv, int head_dim,
                              float scale, const void* k_cache, const void* v_cache,
                              const int* block_tables, int maxb, const int* ctx_start, int BS,
                              hipStream_t s) {
  if (B == 0 || max_len == 0) return 0;
  if (Hq % Hkv != 0 || (BS & (BS - 1)) != 0 || head_dim != 128) return -1;
  int log2BS = 0;
  while ((1 << log2BS) < BS) ++log2BS;
  PagedKV pk{(const uint16_t*)k_cache, (const uint16_t*)v_cache, block_tables, maxb, ctx_start, BS, log2BS};
  return prefill_dispatch(s, B, max_len, head_dim, 1, qkv, row_stride, cu_seqlens, out, o_stride, Hq, Hkv,
                          scale, pk);
}

// Cascade decode, prefix part: chunk partials of the B decode queries (rows of the packed
// QKV buffer, post-RoPE) against the shared prompt prefix [0, *plen) of the 64-token
// blocks listed in prefix_table.  Llama-3 GQA shape only (head_dim 128, 4 query heads per
// KV head): one workgroup per (64 rows, KV head, key chunk), 8 waves.
int docqa_cascade_prefix(const void* qkv, int row_stride, int rows, int Hq, int Hkv, float scale,
                         const void* k_cache, const void* v_cache, const int* prefix_table,
                         const int* plen, int BS, int nchunk, float* acc, float* ml,
                         const int* positions, const float* cos_sin, hipStream_t s) {
  if (rows == 0) return 0;
  if (Hq != 4 * Hkv || BS != 64 || nchunk < 1) return -1;
  PagedKV pk{(const uint16_t*)k_cache, (const uint16_t*)v_cache, prefix_table, 0, nullptr, BS, 6};
  CascadeOut co{acc, ml, plen, nchunk, rows};
  co.positions = positions;
  co.cos_sin = cos_sin;
  static const int wph = [] {   // waves per head: 2 (64-row tiles) or 1 (32-row tiles, 2x workgroups)
    const char* e = getenv("DOCQA_CASCADE_WPH");
    return e && atoi(e) == 1 ? 1 : 2;
  }();
  if (wph == 1) {
    dim3 grid(Hkv, nchunk, (rows + 31) / 32);
    flash_prefill_kernel<128, false, true, 4, 1, true><<<grid, 256, 0, s>>>(
        (const uint16_t*)qkv, row_stride, nullptr, nullptr, 0, Hq, Hkv, scale, pk, co);
  } else {
    dim3 grid(Hkv, nchunk, (rows + 63) / 64);
    flash_prefill_kernel<128, false, true, 4, 2, true><<<grid, 512, 0, s>>>(
        (const uint16_t*)qkv, row_stride, nullptr, nullptr, 0, Hq, Hkv, scale, pk, co);
  }
  DOCQA_CHECK_LAUNCH();
  return 0;
}
