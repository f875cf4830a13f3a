// wgemm.hip -- mid-M decode GEMM with the weights streamed straight into VGPRs:
// Y[M, N] = X[M, K] . W[N, K]^T at 129..512 decode rows (the bench's 256-question step).
//
// Why a second mid-M kernel (mgemm.hip is the first): at M = 256 the projection is bound
// by the bytes each CU pulls through its vector-memory path (TA/TD), not by HBM
// (profiles/r2_pmc/mgemm_isolated_vs_loaded.txt).  mgemm stages BOTH operands through one
// LDS ring, and its 144 KB of LDS caps the weight tile at 128 columns: every workgroup
// re-reads its K slice of X from L2 once per 128 weight rows, so the X bytes moved are twice
// the weight bytes (3x W through TA in all).  Here
//   * each wave OWNS its weight columns (all 256 rows x CW columns of the output tile), so
//     the weight stream needs no sharing and no LDS: 16-B global loads straight into the
//     MFMA B-fragment registers, 2-3 k-stages ahead in a register ring;
//   * LDS holds only X: a 4-slot ring of [256 x 64] bf16 stages (128 KB), filled by LDS-DMA
//     (global_load_lds 16 B, source-address XOR swizzle -> conflict-free ds_read_b128) and
//     read by every wave (LDS bandwidth is not the limit: 256 KB of reads per stage at
//     256 B/clk vs 2048 MFMA cycles per SIMD);
//   * the tile is 256 rows x 256 columns (8 waves x 32), so X through TA = W through TA
//     (2x W in all instead of 3x);
//   * split-K over the grid for the narrow projections (fp32 slabs [S, M, N] combined by
//     the consumer that exists anyway), and for the fused-SwiGLU gate|up a 2-way split-K
//     whose halves meet in the launch: the first half to finish parks its fp32 partial
//     tile (write-through stores, acc-native layout: 16 B per lane, fully coalesced), the
//     second adds it to its accumulators and runs the SwiGLU epilogue.  The second half
//     only waits on a half that already drew its ticket, i.e. is resident -- no deadlock
//     for any residency; fp32 a + b == b + a, so the result is bitwise independent of
//     which half arrives first.
// Every vector-memory op of the main loop (LDS-DMA and the weight loads) is inline asm, so
// the only vmcnt waits are the loop's counted ones (cdna_hip_programming.md §5 "Projection
// GEMM at M = 256" item 4(b)); the weight registers are "published" after each wait so no
// MFMA that reads them is scheduled above it.
// Shapes: N % BN == 0, K % (S * 64) == 0,
// any M (rows tiled by 256, tail rows clamped on load and never stored).
#include "docqa_common.h"
#include "docqa_asm.h"
#include "docqa_argmax.h"
#include <float.h>

using namespace docqa;

namespace {
constexpr int BM = 256;                  // rows per workgroup (all of an m-tile)
constexpr int BKS = 64;                  // k per stage
constexpr int NSR = 4;                   // X ring slots
constexpr int SLOT = BM * BKS;           // bf16 elements per X slot (32 KB)
constexpr int kTicketOff = NSR * SLOT - 8;   // int slot in the ring's tail for the ticket broadcast
enum { EPI_BF16 = 0, EPI_PARTIAL = 1, EPI_GLU = 2, EPI_ARGMAX = 3 };

__device__ __forceinline__ int swz(int row, int ch) { return row * 64 + ((ch ^ ((row >> 1) & 7)) << 3); }

__device__ __forceinline__ float silu_f(float x) { return x / (1.f + __expf(-x)); }

__device__ __forceinline__ void better(float& bv, int& bi, float v, int i) {
  if (v > bv || (v == bv && i < bi)) { bv = v; bi = i; }
}

// 16-B global load into VGPRs (SGPR base + 32-bit lane offset + immediate), invisible to
// hipcc's waitcnt pass (counted by the loop)
template <bool NT, int IMM>
__device__ __forceinline__ void wload16(bf16x8& d, const uint16_t* sbase, uint32_t voff) {
  if constexpr (NT)
    asm volatile("global_load_dwordx4 %0, %1, %2 offset:%3 nt" : "=v"(d) : "v"(voff), "s"(sbase), "i"(IMM) : "memory");
  else
    asm volatile("global_load_dwordx4 %0, %1, %2 offset:%3" : "=v"(d) : "v"(voff), "s"(sbase), "i"(IMM) : "memory");
}
// one 16-B-per-lane LDS-DMA wave-instruction from SGPR base + 32-bit lane offset
__device__ __forceinline__ void glds16s(const uint16_t* sbase, uint32_t voff, uint32_t dst_base) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(voff), "s"(sbase), "s"(dst_base) : "memory");
}
// LDS fragment read invisible to hipcc's lgkmcnt pass (the loop counts its own window)
__device__ __forceinline__ void lds16(bf16x8& d, uint32_t addr) {
  asm volatile("ds_read_b128 %0, %1" : "=v"(d) : "v"(addr) : "memory");
}
template <int N>
__device__ __forceinline__ void wait_lgkmcnt() {
  asm volatile("s_waitcnt lgkmcnt(%0)" :: "i"(N) : "memory");
}
// 16-B write-through load (L1 bypass) of a slab another workgroup stored with sc1
__device__ __forceinline__ f32x4 load16_sc1(const float* p) {
  f32x4 d;
  asm volatile("global_load_dwordx4 %0, %1, off sc1\n\ts_waitcnt vmcnt(0)" : "=v"(d) : "v"(p) : "memory");
  return d;
}

template <int EPI, int NW, int NJ, bool NT, int LD, bool PK = false>
__global__ __launch_bounds__(NW * 64) void wgemm_kernel(const uint16_t* __restrict__ X,
                                                        const uint16_t* __restrict__ W,
                                                        uint16_t* __restrict__ Y, float* __restrict__ P,
                                                        float* __restrict__ pv, int* __restrict__ pi,
                                                        float* __restrict__ ws, int* __restrict__ tick,
                                                        int* __restrict__ err, int M, int N, int K, int Ks,
                                                        int S, int n_valid) {
  constexpr int CW = NJ * 16;                  // output columns per wave
  constexpr int BN = NW * CW;                  // output columns per workgroup
  constexpr int XI = SLOT * 2 / 1024 / NW;     // 1-KiB LDS-DMA instructions per wave per stage
  constexpr int WI = 2 * NJ;                   // weight loads per wave per stage
  constexpr int PER = XI + WI;
  constexpr int MI = BM / 16;                  // 16-row m-tiles
  static_assert(XI * NW * 1024 == SLOT * 2, "DMA split");
  __shared__ __attribute__((aligned(16))) uint16_t smem[NSR * SLOT];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fq = lane >> 4;
  const int ntiles = N / BN;
  const int slice = blockIdx.x % S, tile = blockIdx.x / S;
  const int m0 = blockIdx.y * BM, kbeg = slice * Ks;
  const int c0 = tile * BN + wave * CW;        // this wave's first output column
  const int nk = Ks / BKS;

  // LDS-DMA sources of X: instruction q of this wave covers tile rows 8 (q NW + wave) ..
  // +7; lane -> physical 16-B chunk pc of row r, source = the logical chunk the swizzle
  // puts there.  Byte offsets from the stage's SGPR base (32-bit: M K, N K < 2^31).
  uint32_t xoff[XI];
#pragma unroll
  for (int q = 0; q < XI; ++q) {
    const int p = (q * NW + wave) * 64 + lane, r = p >> 3, pc = p & 7;
    xoff[q] = (uint32_t)(min(m0 + r, M - 1) * K + ((pc ^ ((r >> 1) & 7)) << 3)) * 2u;
  }
  // weight sources: B fragment (16 rows x 32 k) of n-tile j at k-step ks: lane (fr, fq)
  // holds row c0 + 16 j + fr, k chunk 4 ks + fq (ks: +64 B immediate).  PK: W in the MFMA
  // fragment-major layout of ops.pack_fragments -- [N/16][K/32][64 lanes][8]: the fragment
  // of (n-tile, k-step) is 1 KiB contiguous, so every weight load is one fully coalesced
  // wave-instruction (row-major: 16 rows x 64 B, half lines; ks: +1 KiB immediate)
  uint32_t woff[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    if constexpr (PK) woff[j] = (uint32_t)((((c0 >> 4) + j) * (K >> 5) + (kbeg >> 5)) * 512 + lane * 8) * 2u;
    else woff[j] = (uint32_t)((c0 + j * 16 + fr) * K + fq * 8) * 2u;
  }
  const uint16_t* xbase = X + kbeg;
  const uint16_t* wbase = PK ? W : W + kbeg;

  const uint32_t base = lds_u32(smem);
  typedef bf16x8 WSet[2][NJ];
  auto issue = [&](int t, WSet& wb) {
    const uint32_t slot = base + (uint32_t)((t % NSR) * SLOT * 2);
    const uint16_t* xb = xbase + t * BKS;
    const uint16_t* wb_ = wbase + t * (PK ? 2 * 512 : BKS);
#pragma unroll
    for (int q = 0; q < XI; ++q) glds16s(xb, xoff[q], slot + (uint32_t)((q * NW + wave) * 1024));
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      wload16<NT, 0>(wb[0][j], wb_, woff[j]);
      wload16<NT, PK ? 1024 : 64>(wb[1][j], wb_, woff[j]);
    }
  };

  f32x4 acc[MI][NJ];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // A fragments of a stage in (ks, m-tile) order p = 16 ks + i: lane (fr, fq) reads row
  // 16 i + fr, k chunk 4 ks + fq; a window of AW reads is kept in flight under the MFMAs
  constexpr int AW = 4;
  const uint32_t arow = (uint32_t)fr;
  auto a_addr = [&](uint32_t slot, int p) {
    const int i = p & 15, ch = (p >> 4) * 4 + fq;
    return slot + (uint32_t)swz(i * 16 + (int)arow, ch) * 2u;
  };

  // step t: [stage t's X and W landed: counted vmcnt] [publish W(t)] barrier [issue stage
  // t + LD into X slot (t + LD) % 4 (drained by step t - 4 + LD <= t - 1) and W set
  // (t + LD) % (LD + 1) (drained in step t - 1)] [MFMAs of stage t, A fragments read
  // from LDS AW ahead]
  auto step = [&](int t, WSet& cur, WSet& nxt) {
    const int ahead = min(nk - 1, t + LD - 1) - t;   // stages issued beyond t
    if (LD >= 3 && ahead >= 2) wait_vmcnt<2 * PER>();
    else if (ahead >= 1) wait_vmcnt<PER>();
    else wait_vmcnt<0>();
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int j = 0; j < NJ; ++j) asm volatile("" : "+v"(cur[ks][j]));
    ring_barrier();
    if (t + LD < nk) issue(t + LD, nxt);
    const uint32_t slot = base + (uint32_t)((t % NSR) * SLOT * 2);
    bf16x8 a[AW];
#pragma unroll
    for (int p = 0; p < AW; ++p) lds16(a[p], a_addr(slot, p));
#pragma unroll
    for (int p = 0; p < 32; ++p) {
      // reads issued after A(p): min(p + AW - 1, 31) - p
      constexpr int dummy = 0;
      (void)dummy;
      if (p + AW - 1 <= 31) wait_lgkmcnt<AW - 1>();
      else if (p == 29) wait_lgkmcnt<2>();
      else if (p == 30) wait_lgkmcnt<1>();
      else wait_lgkmcnt<0>();
      bf16x8& ap = a[p % AW];
      asm volatile("" : "+v"(ap));
      const int i = p & 15, ks = p >> 4;
#pragma unroll
      for (int j = 0; j < NJ; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ap, cur[ks][j], acc[i][j], 0, 0, 0);
      if (p + AW < 32) lds16(a[p % AW], a_addr(slot, p + AW));
    }
  };

  WSet w[LD + 1];
#pragma unroll
  for (int u = 0; u < LD; ++u)
    if (u < nk) issue(u, w[u]);
  for (int t = 0; t < nk; t += LD + 1) {
#pragma unroll
    for (int u = 0; u <= LD; ++u)
      if (t + u < nk) step(t + u, w[u], w[(u + LD) % (LD + 1)]);
  }
  wait_vmcnt<0>();
  ring_barrier();   // every wave done with the ring: its head is epilogue scratch now

  if constexpr (EPI == EPI_GLU) {
    if (S == 2) {
      // the two K halves of this tile meet here (see the header)
      const int tix = blockIdx.y * ntiles + tile;
      int* tk = reinterpret_cast<int*>(smem + kTicketOff);
      if (tid == 0) tk[0] = __hip_atomic_fetch_add(&tick[2 * tix], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __syncthreads();
      const int first = tk[0] == 0;
      float* slab = ws + ((size_t)tix * NW + wave) * (MI * NJ * 256) + lane * 4;
      if (first) {
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
          for (int j = 0; j < NJ; ++j) {
            const f32x4 v = acc[i][j];
            store16_wt(slab + (i * NJ + j) * 256,
                       uint4{__float_as_uint(v[0]), __float_as_uint(v[1]), __float_as_uint(v[2]), __float_as_uint(v[3])});
          }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) __hip_atomic_store(&tick[2 * tix + 1], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return;
      }
      if (tid == 0) {
        int it = 0;
        while (__hip_atomic_load(&tick[2 * tix + 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0) {
          if (++it > (1 << 24)) {   // a lost hand-off: report, never hang the GPU
            __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            break;
          }
          __builtin_amdgcn_s_sleep(2);
        }
      }
      __syncthreads();
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[i][j] += load16_sc1(slab + (i * NJ + j) * 256);
      if (tid == 0) {   // both halves are past every use of the words: re-arm for the next launch
        __hip_atomic_store(&tick[2 * tix], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&tick[2 * tix + 1], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }

  // epilogue, 16 rows at a time: accumulators -> per-wave scratch [16][CW + 4] -> re-read so
  // consecutive lanes own consecutive 16-B pieces of a row (coalesced row stores)
  constexpr int SCR = CW + 4;
  float* scr = reinterpret_cast<float*>(smem) + wave * 16 * SCR;
  float bestv[MI];
  int besti[MI];
#pragma unroll
  for (int i = 0; i < MI; ++i) {
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) scr[(fq * 4 + r) * SCR + j * 16 + fr] = acc[i][j][r];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if constexpr (EPI == EPI_ARGMAX) {
      // 4 lanes per row, CW / 4 columns each; the row's best (value, id) after 2 shuffles
      constexpr int CPL = CW / 4;
      const int rr = lane >> 2, cc = (lane & 3) * CPL;
      float bv = -FLT_MAX;
      int bi = 0x7fffffff;
#pragma unroll
      for (int e = 0; e < CPL; e += 4) {
        const float4 t = *reinterpret_cast<const float4*>(scr + rr * SCR + cc + e);
        const float tv[4] = {t.x, t.y, t.z, t.w};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int col = c0 + cc + e + q;
          if (col < n_valid) better(bv, bi, bf2f(f2bf(tv[q])), col);
        }
      }
#pragma unroll
      for (int o = 1; o <= 2; o <<= 1) {
        const float ov = __shfl_xor(bv, o, 64);
        const int oi = __shfl_xor(bi, o, 64);
        better(bv, bi, ov, oi);
      }
      bestv[i] = bv;
      besti[i] = bi;
    } else {
      // EPC: input columns per lane (fp32 slab 4, bf16 8, SwiGLU one 16-column gate|up group)
      constexpr int EPC = EPI == EPI_PARTIAL ? 4 : EPI == EPI_BF16 ? 8 : 16;
      constexpr int LPR = CW / EPC;            // lanes per row
#pragma unroll
      for (int e = lane; e < 16 * LPR; e += 64) {
        const int r = e / LPR, c = (e % LPR) * EPC;
        float v[EPC];
#pragma unroll
        for (int u = 0; u < EPC; u += 4) {
          const float4 t = *reinterpret_cast<const float4*>(scr + r * SCR + c + u);
          v[u] = t.x; v[u + 1] = t.y; v[u + 2] = t.z; v[u + 3] = t.w;
        }
        const int row = m0 + i * 16 + r, col = c0 + c;
        if (row < M) {
          if constexpr (EPI == EPI_PARTIAL) {
            *reinterpret_cast<float4*>(P + ((size_t)slice * M + row) * N + col) = float4{v[0], v[1], v[2], v[3]};
          } else if constexpr (EPI == EPI_BF16) {
            *reinterpret_cast<uint4*>(Y + (size_t)row * N + col) = pack8(v);
          } else {
            float o[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
              const float gv = bf2f(f2bf(v[u])), uv = bf2f(f2bf(v[8 + u]));   // as the bf16 GEMM output
              o[u] = silu_f(gv) * uv;
            }
            *reinterpret_cast<uint4*>(Y + (size_t)row * (N >> 1) + (col >> 1)) = pack8(o);
          }
        }
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
  if constexpr (EPI == EPI_ARGMAX) {
    // merge the NW column waves of each row through LDS: one partial per (row, tile)
    __syncthreads();
    float* rv = reinterpret_cast<float*>(smem);
    int* ri = reinterpret_cast<int*>(smem) + BM * NW;
    if ((lane & 3) == 0) {
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        const int lr = i * 16 + (lane >> 2);
        rv[lr * NW + wave] = bestv[i];
        ri[lr * NW + wave] = besti[i];
      }
    }
    __syncthreads();
    for (int lr = tid; lr < BM; lr += NW * 64) {
      const int row = m0 + lr;
      if (row >= M) continue;
      float bv = rv[lr * NW];
      int bi = ri[lr * NW];
#pragma unroll
      for (int w = 1; w < NW; ++w) better(bv, bi, rv[lr * NW + w], ri[lr * NW + w]);
      pv[(size_t)row * ntiles + tile] = bv;
      pi[(size_t)row * ntiles + tile] = bi;
    }
  }
}

// Variants (``cfg``), weight loads default-policy / non-temporal (cfg + 8); + 16: W in the
// fragment-major layout (pack_fragments; 17, 18, 20, 25 instantiated):
//   1: 8 waves x 32 columns (BN 256, 2 waves / SIMD, 128 accumulator registers), 2 stages ahead
//   2: 8 waves x 16 columns (BN 128), 3 stages ahead
//   3: 8 waves x 32 columns (BN 256), 3 stages ahead
//   4: 4 waves x 32 columns (BN 128, 1 wave / SIMD), 3 stages ahead
constexpr int kNumCfg = 4;
constexpr int kBN[kNumCfg + 1] = {0, 256, 128, 256, 128};

template <int EPI, int NW, int NJ, bool NT, int LD, bool PK = false>
int launch(const uint16_t* x, const uint16_t* w, uint16_t* y, float* p, float* pv, int* pi, float* ws, int* tick,
           int* err, int M, int N, int K, int S, int n_valid, hipStream_t s) {
  constexpr int BN = NW * NJ * 16;
  dim3 grid((N / BN) * S, (M + BM - 1) / BM);
  wgemm_kernel<EPI, NW, NJ, NT, LD, PK><<<grid, NW * 64, 0, s>>>(x, w, y, p, pv, pi, ws, tick, err, M, N, K, K / S, S,
                                                         n_valid);
  DOCQA_CHECK_LAUNCH();
  return 0;
}

template <int EPI>
int launch_cfg(int cfg, const uint16_t* x, const uint16_t* w, uint16_t* y, float* p, float* pv, int* pi, float* ws,
               int* tick, int* err, int M, int N, int K, int S, int n_valid, hipStream_t s) {
  switch (cfg) {
    case 1: return launch<EPI, 8, 2, false, 2>(x, w, y, p, pv, pi, ws, tick, err, M, N, K, S, n_valid, s);
    case 2: return launch<EPI, 8, 1, false, 3>(x, w, y, p, pv, pi, ws, tick, err, M, N, K, S, n_valid, s);
    case 3: return launch<EPI, 8, 2, false, 3>(x, w, y, p, pv, pi, ws, tick, err, M, N, K, S, n_valid, s);
    case 4: return launch<EPI, 4, 2, false, 3>(x, w, y, p, pv, pi, ws, tick, err, M, N, K, S, n_valid, s);
    case 17: return launch<EPI, 8, 2, false, 2, true>(x, w, y, p, pv, pi, ws, tick, err, M, N, K, S, n_valid, s);
    case 18: return launch<EPI, 8, 1, false, 3, true>(x, w, y, p, pv, pi, ws, tick, err, M, N, K, S, n_valid, s);
    case 20: return launch<EPI, 4, 2, false, 3, true>(x, w, y, p, pv, pi, ws, tick, err, M, N, K, S, n_valid, s);
    case 25: return launch<EPI, 8, 2, true, 2, true>(x, w, y, p, pv, pi, ws, tick, err, M, N, K, S, n_valid, s);
    case 9: return launch<EPI, 8, 2, true, 2>(x, w, y, p, pv, pi, ws, tick, err, M, N, K, S, n_valid, s);
    case 10: return launch<EPI, 8, 1, true, 3>(x, w, y, p, pv, pi, ws, tick, err, M, N, K, S, n_valid, s);
    case 11: return launch<EPI, 8, 2, true, 3>(x, w, y, p, pv, pi, ws, tick, err, M, N, K, S, n_valid, s);
    case 12: return launch<EPI, 4, 2, true, 3>(x, w, y, p, pv, pi, ws, tick, err, M, N, K, S, n_valid, s);
    default: return -1;
  }
}

int tile_n(int cfg) {
  const int c = cfg % 8 == 0 ? 0 : cfg % 8;
  return c >= 1 && c <= kNumCfg ? kBN[c] : 0;
}

bool shape_ok(int M, int N, int K, int S, int cfg) {
  const int bn = tile_n(cfg);
  return bn > 0 && M > 0 && S >= 1 && N % bn == 0 && K % (S * BKS) == 0;
}
}  // namespace

constexpr int kDefaultCfg = 1;
int docqa_wgemm_tile_n(int cfg) { return tile_n(cfg == 0 ? kDefaultCfg : cfg); }

// P given: fp32 split-K slabs [S, M, N]; else S == 1 and Y bf16 [M, N]
int docqa_wgemm(const void* X, const void* W, void* Y, float* P, int M, int N, int K, int S, int cfg,
                hipStream_t s) {
  if (cfg == 0) cfg = kDefaultCfg;
  if (M == 0) return 0;
  if (!shape_ok(M, N, K, S, cfg) || (P == nullptr && (S != 1 || Y == nullptr))) return -1;
  if (!docqa_aligned16(X) || !docqa_aligned16(W) || !docqa_aligned16(P ? (void*)P : Y)) return -1;
  const uint16_t *x = (const uint16_t*)X, *w = (const uint16_t*)W;
  if (P) return launch_cfg<EPI_PARTIAL>(cfg, x, w, nullptr, P, nullptr, nullptr, nullptr, nullptr, nullptr, M, N, K,
                                        S, N, s);
  return launch_cfg<EPI_BF16>(cfg, x, w, (uint16_t*)Y, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, M, N, K,
                              1, N, s);
}

// Y[M, N/2] = silu(gate) * up for the 8-interleaved gate|up weight W [N, K]; S = 2: the
// in-launch K-half hand-off through ws (fp32, >= wgemm_glu_ws_floats) and tick (int32
// [2 x m-tiles x N / BN], zero before the first launch; the kernel re-arms it); err: sticky
// int32 error word (lost hand-off)
long long docqa_wgemm_glu_ws_floats(int M, int N, int cfg) {
  const int bn = docqa_wgemm_tile_n(cfg);
  if (bn <= 0) return 0;
  return (long long)((M + BM - 1) / BM) * (N / bn) * BM * bn;
}

int docqa_wgemm_glu(const void* X, const void* W, void* Y, float* ws, int* tick, int* err, int M, int N, int K,
                    int S, int cfg, hipStream_t s) {
  if (cfg == 0) cfg = kDefaultCfg;
  if (M == 0) return 0;
  if ((S != 1 && S != 2) || !shape_ok(M, N, K, S, cfg) || tile_n(cfg) % 16) return -1;
  if (S == 2 && (!ws || !tick || !err || !docqa_aligned16(ws))) return -1;
  if (!docqa_aligned16(X) || !docqa_aligned16(W) || !docqa_aligned16(Y)) return -1;
  return launch_cfg<EPI_GLU>(cfg, (const uint16_t*)X, (const uint16_t*)W, (uint16_t*)Y, nullptr, nullptr, nullptr, ws,
                             tick, err, M, N, K, S, N, s);
}

// out[M] = argmax over the first n_valid columns of bf16(X . W^T) (LM head + greedy pick);
// outv[M] (optional) its value; ws_v / ws_i: [M, N / tile_n] partials
int docqa_wgemm_argmax(const void* X, const void* W, int64_t* out, float* outv, float* ws_v, int* ws_i, int M, int N,
                       int K, int n_valid, int cfg, hipStream_t s) {
  if (cfg == 0) cfg = kDefaultCfg;
  if (M == 0) return 0;
  if (!shape_ok(M, N, K, 1, cfg) || n_valid <= 0 || n_valid > N) return -1;
  if (!docqa_aligned16(X) || !docqa_aligned16(W)) return -1;
  const int rc = launch_cfg<EPI_ARGMAX>(cfg, (const uint16_t*)X, (const uint16_t*)W, nullptr, nullptr, ws_v, ws_i,
                                        nullptr, nullptr, nullptr, M, N, K, 1, n_valid, s);
  if (rc) return rc;
  argmax_merge_kernel<<<M, 256, 0, s>>>(ws_v, ws_i, N / tile_n(cfg), out, outv);
  DOCQA_CHECK_LAUNCH();
  return 0;
}
