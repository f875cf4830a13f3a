// mgemm.hip -- "mid-M" decode GEMM for the Llama generator at batch buckets of 193..512
// rows (the bench's 256-question decode step):  Y[M, N] = X[M, K] . W[N, K]^T.
//
// Between the skinny weight-streaming regime (dgemm.hip, <= 192 rows: X in VGPRs, W through
// an LDS-DMA ring) and a plain large GEMM, a 256-row decode projection is limited by the
// chip's L2 -> LDS traffic, not by HBM: every workgroup re-reads its K slice of X (2 MB at
// K = 4096) from L2, so the X bytes moved are (N / BN) x 2 MB -- for the Llama-3-8B QKV at
// BN = 128 twice the 48 MB of weights (measured: time tracks total L2->LDS bytes, hot or
// cold weights alike; cdna_hip_programming.md §5 "Projection GEMM at M = 256").  The design
// therefore maximises the tile width per workgroup:
//   * one workgroup owns ALL 256 rows x BN weight rows (BN = 128 or 256) x one K slice:
//     the weight tile is streamed from HBM exactly once and X is re-read only N / BN times;
//   * both operands go HBM/L2 -> LDS by LDS-DMA (global_load_lds 16 B, source-address XOR
//     swizzle so the 16-row MFMA fragment reads are bank-conflict-free) into a ring of
//     BKS-deep k-stages (64 at BN = 128: 3 x 48 KB; 32 at BN = 256: 4 x 32 KB) with counted
//     vmcnt waits and raw s_barrier (no __syncthreads: its release fence would drain the
//     ring, §5 "Pipelining across barriers");
//   * the fragments of stage k+1 are read from LDS while the MFMAs of stage k run (two
//     register sets, loop unrolled by two), NSR-2 DMA stages stream behind them;
//   * waves WM (M) x WN (N), each a (256/WM) x (BN/WN) sub-tile of mfma_f32_16x16x32_bf16
//     accumulators;
//   * split-K over the grid with XCD-aware slice placement (one K slice per XCD, so its
//     4 MB L2 holds only that slice of X); the fp32 slabs [S, M, N] are combined by the
//     consumer kernel that exists anyway (add_rmsnorm_splitk / rope_cache_splitk);
//   * epilogues through a per-wave LDS scratch (16 rows at a time) so global stores are
//     full 64-B lane runs: bf16, fp32 split-K slab, fused SwiGLU over the 8-interleaved
//     gate|up rows (the decode GEMM's layout), or the LM head's greedy argmax (per-row max
//     over the tile, ties to the lowest id as torch.argmax, compared in bf16 so it picks
//     the token the unfused bf16 logits would) -- the [M, 128256] logits never reach HBM.
// Shapes: N % BN == 0, K % (S * 2 * BKS) == 0, any M (rows tiled by 256, tail rows clamped
// on load and never stored).
#include "docqa_common.h"
#include "docqa_asm.h"
#include "docqa_norm_row.h"
#include "docqa_argmax.h"
#include <float.h>
#include <stdlib.h>

using namespace docqa;

namespace {
constexpr int BM = 256;
// EPI_PARTIAL16: the split-K slabs [S, M, N] stored as bf16 (half the slab bytes the GEMM
// writes and its consumer reads; each partial rounded once before the consumer's fp32 sum)
enum { EPI_BF16 = 0, EPI_PARTIAL = 1, EPI_GLU = 2, EPI_ARGMAX = 3, EPI_PARTIAL16 = 4 };

// element offset of 16-B chunk `ch` of `row` in a [rows][BKS] bf16 tile: the XOR spreads
// the 16 rows of a fragment read over all 64 banks (128-B rows: pairs of rows share a
// 256-B bank row; 64-B rows: quads do)
template <int BKS>
__device__ __forceinline__ int swz(int row, int ch) {
  if constexpr (BKS == 64) return row * 64 + ((ch ^ ((row >> 1) & 7)) << 3);
  else return row * 32 + ((ch ^ ((row >> 2) & 3)) << 3);
}

__device__ __forceinline__ float silu_f(float x) { return x / (1.f + __expf(-x)); }


__device__ __forceinline__ void better(float& bv, int& bi, float v, int i) {
  if (v > bv || (v == bv && i < bi)) { bv = v; bi = i; }
}

// Epilogue shared by the kernels: accumulators -> per-wave LDS scratch (the drained ring)
// -> bf16 / fp32 split-K slab / fused SwiGLU / LM-head argmax partials.
template <int EPI, int BN, int WM, int WN>
__device__ __forceinline__ void mgemm_epilogue(f32x4 (&acc)[BM / WM / 16][BN / WN / 16], uint16_t* smem,
                                               uint16_t* __restrict__ Y, float* __restrict__ P,
                                               float* __restrict__ pv, int* __restrict__ pi, int M, int N,
                                               int m0, int n0, int slice, int tile, int ntiles, int n_valid) {
  constexpr int WAVES = WM * WN;
  constexpr int MI = BM / WM / 16;
  constexpr int CW = BN / WN;
  constexpr int NJ = CW / 16;
  constexpr int SCR = CW + 4;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fq = lane >> 4;
  const int wm = wave % WM, wn = wave / WM;

  // epilogue, 16 rows at a time: accumulators -> per-wave scratch [16][CW] -> re-read so
  // that consecutive lanes own consecutive 16-B pieces of a row (coalesced row stores)
  float* scr = reinterpret_cast<float*>(smem) + wave * 16 * SCR;
  const int rbase = m0 + wm * (BM / WM), cbase = n0 + wn * CW;
  float bestv[MI];
  int besti[MI];
#pragma unroll
  for (int i = 0; i < MI; ++i) {
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) scr[(fq * 4 + r) * SCR + j * 16 + fr] = acc[i][j][r];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    // EPC: output columns per lane (fp32 slab 4, bf16 8, SwiGLU 16 inputs -> 8 outputs)
    constexpr int EPC = EPI == EPI_PARTIAL ? 4 : (EPI == EPI_BF16 || EPI == EPI_PARTIAL16) ? 8 : 16;
    constexpr int LPR = CW / EPC, RPS = 64 / LPR;          // lanes per row, rows per sweep
    if constexpr (EPI != EPI_ARGMAX) {
#pragma unroll
      for (int it = 0; it < 16 / RPS; ++it) {
        const int r = it * RPS + lane / LPR, c = (lane % LPR) * EPC;
        float v[EPC];
#pragma unroll
        for (int e = 0; e < EPC / 4; ++e) {
          const float4 t = *reinterpret_cast<const float4*>(scr + r * SCR + c + e * 4);
          v[e * 4] = t.x; v[e * 4 + 1] = t.y; v[e * 4 + 2] = t.z; v[e * 4 + 3] = t.w;
        }
        const int row = rbase + i * 16 + r, col = cbase + c;
        if (row < M) {
          if constexpr (EPI == EPI_PARTIAL) {
            float* dst = P + ((size_t)slice * M + row) * N + col;
            *reinterpret_cast<float4*>(dst) = float4{v[0], v[1], v[2], v[3]};
          } else if constexpr (EPI == EPI_BF16) {
            *reinterpret_cast<uint4*>(Y + (size_t)row * N + col) = pack8(v);
          } else if constexpr (EPI == EPI_PARTIAL16) {
            *reinterpret_cast<uint4*>(Y + ((size_t)slice * M + row) * N + col) = pack8(v);
          } else {
            // 16 consecutive columns = one (gate 8, up 8) interleave group
            float o[8];
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              const float gv = bf2f(f2bf(v[e])), uv = bf2f(f2bf(v[8 + e]));   // as the bf16 GEMM output
              o[e] = silu_f(gv) * uv;
            }
            uint16_t* dst = Y + (size_t)row * (N >> 1) + (col >> 1);
            *reinterpret_cast<uint4*>(dst) = pack8(o);
          }
        }
      }
    } else {
      // 4 lanes per row, CW/4 columns each; the row's best (value, id) after 2 shuffles
      constexpr int CPL = CW / 4;
      const int rr = lane >> 2, cc = (lane & 3) * CPL;
      float bv = -FLT_MAX;
      int bi = 0x7fffffff;
#pragma unroll
      for (int e = 0; e < CPL / 4; ++e) {
        const float4 t = *reinterpret_cast<const float4*>(scr + rr * SCR + cc + e * 4);
        const float tv[4] = {t.x, t.y, t.z, t.w};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int col = cbase + cc + e * 4 + q;
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
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
  if constexpr (EPI == EPI_ARGMAX) {
    // merge the WN column waves of each row through LDS, one partial per (row, tile)
    __syncthreads();
    float* rv = reinterpret_cast<float*>(smem);
    int* ri = reinterpret_cast<int*>(smem) + BM * WN;
    if ((lane & 3) == 0) {
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        const int lr = wm * (BM / WM) + i * 16 + (lane >> 2);
        rv[lr * WN + wn] = bestv[i];
        ri[lr * WN + wn] = besti[i];
      }
    }
    __syncthreads();
    for (int lr = tid; lr < BM; lr += WAVES * 64) {
      const int row = m0 + lr;
      if (row >= M) continue;
      float bv = rv[lr * WN];
      int bi = ri[lr * WN];
#pragma unroll
      for (int w = 1; w < WN; ++w) better(bv, bi, rv[lr * WN + w], ri[lr * WN + w]);
      pv[(size_t)row * ntiles + tile] = bv;
      pi[(size_t)row * ntiles + tile] = bi;
    }
  }
}

// PF: fragment prefetch (stage k+1's LDS reads under stage k's MFMAs, two register sets);
// PF = 0 reads each stage's fragments after its barrier (one register set, for the
// 128 x 128-per-wave layout whose two sets would not fit)
// The K loop of one (m-tile, weight tile) over K-stages [kbeg / BKS, kbeg / BKS + nk)
// (nk even, >= 2), accumulating into `acc`; ends with the ring drained and a barrier, so the
// caller may reuse the LDS (epilogue scratch, or the next tile's ring).
template <int BN, int BKS, int NSR, int WM, int WN, int PF>
__device__ __forceinline__ void mgemm_mainloop(uint16_t* smem, const uint16_t* __restrict__ X,
                                               const uint16_t* __restrict__ W, int M, int kbeg, int nk, int m0,
                                               int n0, int ldx, int ldw,
                                               f32x4 (&acc)[BM / WM / 16][BN / WN / 16]) {
  // PF bits 0-1: 1 = fragment prefetch, 0 = none, 2 / 3 = probe-only (no MFMAs / no MFMAs
  // and no fragment reads); bit 2: W stored stage-tiled -- [N / BN][K / BKS][BN][BKS], so a
  // stage's weight tile is one contiguous 16 KiB run instead of BN rows x 128 B at a K x 2 B
  // stride (the DRAM-page probe, scripts/mgemm_floor_probe.py)
  constexpr int MODE = PF & 3;
  constexpr bool WTILE = (PF & 4) != 0;
  constexpr int WAVES = WM * WN;
  constexpr int MI = BM / WM / 16;                      // 16-row m-tiles per wave
  constexpr int CW = BN / WN;                           // output columns per wave
  constexpr int NJ = CW / 16;                           // 16-col n-tiles per wave
  constexpr int KS = BKS / 32;                          // MFMA k-steps per stage
  constexpr int CPR = BKS / 8;                          // 16-B chunks per tile row
  constexpr int RPI = 64 / CPR;                         // tile rows per DMA instruction
  constexpr int A_PER_WAVE = BM / RPI / WAVES;          // 1-KiB DMA instructions per stage
  constexpr int B_PER_WAVE = BN / RPI / WAVES;
  constexpr int PER_STAGE = A_PER_WAVE + B_PER_WAVE;
  constexpr int SLOT = (BM + BN) * BKS;                 // elements per ring slot
  static_assert(NSR >= 2, "ring needs >= 2 slots");
  static_assert(A_PER_WAVE * RPI * WAVES == BM && B_PER_WAVE * RPI * WAVES == BN, "DMA split");
  static_assert(NSR * SLOT * 2 <= 160 * 1024, "LDS");

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fq = lane >> 4;
  const int wm = wave % WM, wn = wave / WM;

  // per-lane DMA sources (k offset added per stage): instruction q covers tile rows
  // RPI q .. RPI q + RPI-1; lane -> physical 16-B chunk, source = the logical chunk the
  // swizzle puts there
  const uint16_t* asrc[A_PER_WAVE];
  const uint16_t* bsrc[B_PER_WAVE];
  auto lchunk = [&](int r, int pc) {
    if constexpr (BKS == 64) return pc ^ ((r >> 1) & 7);
    else return pc ^ ((r >> 2) & 3);
  };
#pragma unroll
  for (int i = 0; i < A_PER_WAVE; ++i) {
    const int p = (i * WAVES + wave) * 64 + lane, r = p / CPR;
    asrc[i] = X + (size_t)min(m0 + r, M - 1) * ldx + kbeg + lchunk(r, p % CPR) * 8;
  }
#pragma unroll
  for (int i = 0; i < B_PER_WAVE; ++i) {
    const int p = (i * WAVES + wave) * 64 + lane, r = p / CPR;
    if constexpr (WTILE)
      bsrc[i] = W + ((size_t)(n0 / BN) * (size_t)(ldw / BKS) + (size_t)(kbeg / BKS)) * (BN * BKS) + r * BKS +
                lchunk(r, p % CPR) * 8;
    else
      bsrc[i] = W + (size_t)(n0 + r) * ldw + kbeg + lchunk(r, p % CPR) * 8;
  }
  const uint32_t base = lds_u32(smem);
  auto stage = [&](int kt) {
    const uint32_t slot = base + (uint32_t)((kt % NSR) * SLOT * 2);
    const int ko = kt * BKS;
#pragma unroll
    for (int i = 0; i < A_PER_WAVE; ++i)
      glds16<false>(asrc[i] + ko, slot + (uint32_t)((i * WAVES + wave) * 1024));
#pragma unroll
    for (int i = 0; i < B_PER_WAVE; ++i)
      glds16<true>(bsrc[i] + (WTILE ? (size_t)kt * (BN * BKS) : (size_t)ko), slot + (uint32_t)(BM * BKS * 2 + (i * WAVES + wave) * 1024));
  };

  // fragments of one stage: [k-step][m-tile] A, [k-step][n-tile] B.  They are read by
  // inline-asm ds_read_b128 (invisible to hipcc's waitcnt pass, which otherwise drains
  // every outstanding LDS read -- the next stage's prefetch included -- before the first
  // MFMA of the current stage) and published by an explicit lgkmcnt(0) that names them
  // (`publish`), so no MFMA reading them can be scheduled above the wait.
  struct Frag { bf16x8 a[KS][MI]; bf16x8 b[KS][NJ]; };
  const uint32_t a_off = (uint32_t)(wm * (BM / WM) + fr), b_off = (uint32_t)(BM + wn * CW + fr);
  auto load_frags = [&](Frag& f, int kt) {
    const uint32_t slot = base + (uint32_t)((kt % NSR) * SLOT * 2);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int ch = ks * 4 + fq;
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const uint32_t ad = slot + (uint32_t)swz<BKS>(b_off + j * 16, ch) * 2;
        asm volatile("ds_read_b128 %0, %1" : "=v"(f.b[ks][j]) : "v"(ad) : "memory");
      }
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        const uint32_t ad = slot + (uint32_t)swz<BKS>(a_off + i * 16, ch) * 2;
        asm volatile("ds_read_b128 %0, %1" : "=v"(f.a[ks][i]) : "v"(ad) : "memory");
      }
    }
  };
  auto publish = [&](Frag& f) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
#pragma unroll
      for (int j = 0; j < NJ; ++j) asm volatile("" : "+v"(f.b[ks][j]));
#pragma unroll
      for (int i = 0; i < MI; ++i) asm volatile("" : "+v"(f.a[ks][i]));
    }
  };
  auto mma = [&](const Frag& f) {
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f.a[ks][i], f.b[ks][j], acc[i][j], 0, 0, 0);
  };
  // Schedule (NSR slots): the fragments of stage kt+1 are read from LDS while the MFMAs of
  // stage kt run, and NSR-2 DMA stages stream behind them.  Step kt: [frags(kt) landed:
  // publish] [DMA(kt+1) landed: vmcnt] barrier [DMA(kt+NSR) into slot kt % NSR, which
  // frags(kt) -- now in registers in every wave -- vacated] [ds_read frags(kt+1)] [MFMA(kt)].
  // The fragment reads are issued on every step (the last one reads a dead slot) so the
  // only control flow in the loop is scalar branches around asm (DMA issue, vmcnt).
  auto step = [&](Frag& cur, Frag& nxt, int kt) {
    publish(cur);
    // DMA stages issued so far: 0 .. min(nk - 1, kt + NSR - 1); kt+1 must have landed
    const int ahead = min(nk - 1, kt + NSR - 1) - (kt + 1);
    if (ahead >= NSR - 2) wait_vmcnt<(NSR - 2) * PER_STAGE>();
    else if (NSR >= 4 && ahead == NSR - 3) wait_vmcnt<(NSR >= 4 ? NSR - 3 : 0) * PER_STAGE>();
    else if (NSR >= 5 && ahead == NSR - 4) wait_vmcnt<(NSR >= 5 ? NSR - 4 : 0) * PER_STAGE>();
    else wait_vmcnt<0>();
    ring_barrier();
    if (kt + NSR < nk) stage(kt + NSR);
    if constexpr (MODE != 3) load_frags(nxt, kt + 1);
    if constexpr (MODE == 1) mma(cur);
    // keep this stage's MFMAs above the next stage's publish wait (hipcc otherwise sinks
    // some of them below it, where they wait for the whole prefetch)
    __builtin_amdgcn_sched_barrier(0);
  };
#pragma unroll
  for (int j = 0; j < NSR; ++j)
    if (j < nk) stage(j);
  // PF 2 / 3: probe-only variants (cfg 8-10) -- the same ring without the MFMAs (2), and
  // without the fragment reads too (3): the transfer floor of the schedule
  if constexpr (MODE != 0) {
    Frag f0, f1;
    if (nk >= NSR) wait_vmcnt<(NSR - 1) * PER_STAGE>();
    else wait_vmcnt<0>();
    ring_barrier();
    load_frags(f0, 0);
    for (int kt = 0; kt < nk; kt += 2) {
      step(f0, f1, kt);
      step(f1, f0, kt + 1);
    }
  } else {
    // plain ring: [DMA(kt) landed] barrier [DMA(kt+NSR-1) into the slot read in step kt-1]
    // [fragments of kt -> MFMAs, k-step by k-step so the compiler overlaps the reads]
    const uint16_t* sbase = smem;
    for (int kt = 0; kt < nk; ++kt) {
      // stages issued so far: 0 .. NSR-1 by the prologue, then one per step from step 1
      const int ahead = min(nk - 1, kt == 0 ? NSR - 1 : kt + NSR - 2) - kt;
      if (ahead >= NSR - 1) wait_vmcnt<(NSR - 1) * PER_STAGE>();
      else if (NSR >= 3 && ahead == NSR - 2) wait_vmcnt<(NSR >= 3 ? NSR - 2 : 0) * PER_STAGE>();
      else wait_vmcnt<0>();
      ring_barrier();
      if (kt + NSR - 1 < nk && kt > 0) stage(kt + NSR - 1);
      const uint16_t* sa = sbase + (kt % NSR) * SLOT;
      const uint16_t* sb = sa + BM * BKS;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const int ch = ks * 4 + fq;
        bf16x8 b[NJ];
#pragma unroll
        for (int j = 0; j < NJ; ++j) b[j] = *reinterpret_cast<const bf16x8*>(sb + swz<BKS>(wn * CW + j * 16 + fr, ch));
#pragma unroll
        for (int i = 0; i < MI; ++i) {
          const bf16x8 a = *reinterpret_cast<const bf16x8*>(sa + swz<BKS>(wm * (BM / WM) + i * 16 + fr, ch));
#pragma unroll
          for (int j = 0; j < NJ; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b[j], acc[i][j], 0, 0, 0);
        }
      }
      // every wave's reads of this slot retire before the next barrier frees it
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
  }
  wait_vmcnt<0>();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  ring_barrier();   // every wave is done reading the ring: reuse it as epilogue scratch
}

// One (m-tile, weight tile, K slice) of the GEMM on the workgroup's LDS ring `smem`
// (NSR * (BM + BN) * BKS bf16): the kernel below runs one per workgroup.
template <int EPI, int BN, int BKS, int NSR, int WM, int WN, int PF = 1>
__device__ __forceinline__ void mgemm_tile(uint16_t* smem, const uint16_t* __restrict__ X,
                                           const uint16_t* __restrict__ W, uint16_t* __restrict__ Y,
                                           float* __restrict__ P, float* __restrict__ pv,
                                           int* __restrict__ pi, int M, int N, int K, int Ks,
                                           int tile, int slice, int m0, int ntiles, int n_valid, int ldx,
                                           int ldw) {
  constexpr int MI = BM / WM / 16, NJ = BN / WN / 16;
  f32x4 acc[MI][NJ];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int n0 = tile * BN;
  mgemm_mainloop<BN, BKS, NSR, WM, WN, PF>(smem, X, W, M, slice * Ks, Ks / BKS, m0, n0, ldx, ldw, acc);
  mgemm_epilogue<EPI, BN, WM, WN>(acc, smem, Y, P, pv, pi, M, N, m0, n0, slice, tile, ntiles, n_valid);
}

template <int EPI, int BN, int BKS, int NSR, int WM, int WN, int PF = 1>
__global__ __launch_bounds__(WM * WN * 64) void mgemm_kernel(const uint16_t* __restrict__ X,
                                                             const uint16_t* __restrict__ W,
                                                             uint16_t* __restrict__ Y,
                                                             float* __restrict__ P,
                                                             float* __restrict__ pv, int* __restrict__ pi,
                                                             int M, int N, int K, int Ks, int S,
                                                             int ntiles, int remap, int n_valid, int ldx,
                                                             int ldw) {
  __shared__ __attribute__((aligned(16))) uint16_t smem[NSR * (BM + BN) * BKS];
  const int L = blockIdx.x;
  int tile, slice;
  if (remap == 1) {            // 8 % S == 0: XCD x runs slice x % S
    const int xcd = L & 7, j = L >> 3;
    slice = xcd % S;
    tile = j * (8 / S) + xcd / S;
  } else if (remap == 2) {     // S % 8 == 0: XCD x runs slices x, x + 8, ...
    const int xcd = L & 7, j = L >> 3, q = S / 8;
    slice = xcd + 8 * (j % q);
    tile = j / q;
  } else {
    tile = L % ntiles;
    slice = L / ntiles;
  }
  mgemm_tile<EPI, BN, BKS, NSR, WM, WN, PF>(smem, X, W, Y, P, pv, pi, M, N, K, Ks, tile, slice, blockIdx.y * BM,
                                            ntiles, n_valid, ldx, ldw);
}

// Variants (``cfg``): the tile width and wave layout
//   1: BN 128, 64-deep stages x 3, waves 2 x 2 (128 x 64 each, 1 wave / SIMD)
//   2: BN 128, 64-deep stages x 3, waves 4 x 2 ( 64 x 64 each, 2 waves / SIMD)
//   3: BN 256, 32-deep stages x 4, waves 2 x 4 (128 x 64 each, 2 waves / SIMD)
//   4: BN 256, 32-deep stages x 4, waves 2 x 2 (128 x 128 each, 1 wave / SIMD)
//   5: BN 256, 64-deep stages x 2, waves 2 x 2 (128 x 128 each, 1 wave / SIMD), no prefetch
//   6: BN 256, 64-deep stages x 2, waves 2 x 4 (128 x 64 each, 2 waves / SIMD), no prefetch
struct Cfg { int bn, bks; };
// (Decoupled X / W rings -- weights DMA'd by half the waves into a deeper ring of their
// own, so the HBM stream can run further ahead than the L2-resident activations -- measured
// no faster: 64-deep stages at (3 X, 4 W) / (2, 6) slots equal or 5-10 % slower than cfg 2,
// 32-deep stages 40-50 % slower: the per-stage barrier + LDS traffic, not the weight
// latency, sets the stage time; profiles/r2_mgemm_probe_dq_rings.log.)
//   7: BN  64, 64-deep stages x 3, waves 4 x 2 ( 64 x 32 each, 2 waves / SIMD): twice the
//      workgroups of cfg 2 for the narrow projections that otherwise fill half the chip
// (Half-depth stages -- BN 128, 32-deep x 6 slots, the same 144 KB ring with 5 stages in
// flight instead of 2 -- measured 1.3-1.6x SLOWER on every projection (QKV S=4 30.2 vs
// 22.6 us, gate|up+SwiGLU 114.5 vs 81.1) and 23 % slower end to end: the stage time is a
// fixed ~1000-cycle cost plus the LDS-DMA bytes, not the bytes in flight over the HBM
// latency; profiles/r2_mgemm_probe_bks32_ring6.log, profiles/r2_ab_mid_cfg8_bks32.log.)
// (Raising the wave priority over each stage's MFMA burst (s_setprio 1 / 0 around mma):
// 3-7 % slower per projection, 1.3 % slower end to end; profiles/r2_mgemm_probe_setprio.log,
// profiles/r2_ab_mid_setprio.log.)
// Probe-only (scripts/mgemm_floor_probe.py): 8 = cfg 2 without MFMAs, 9 = cfg 2 without
// MFMAs and fragment reads (DMA ring + waits + barriers alone), 10 = BN 128 x 32-deep x 6
// slots, DMA alone (5 stages / 120 KB in flight instead of 2 / 96 KB)
// 11 / 12 / 13 / 14 = cfg 2 / 9 / 7 / 6 reading a stage-tiled weight copy (WTILE above:
// [N / BN][K / 64][BN][64])
constexpr int kNumCfg = 14;
constexpr Cfg kCfg[kNumCfg + 1] = {{0, 0}, {128, 64}, {128, 64}, {256, 32}, {256, 32}, {256, 64}, {256, 64},
                                   {64, 64}, {128, 64}, {128, 64}, {128, 32}, {128, 64}, {128, 64}, {64, 64},
                                   {256, 64}};

template <int EPI, int BN, int BKS, int NSR, int WM, int WN, int PF = 1>
int launch(const uint16_t* x, const uint16_t* w, uint16_t* y, float* p, float* pv, int* pi, int M,
           int N, int K, int S, int n_valid, hipStream_t s, int ldx, int ldw) {
  // the epilogue sweeps 16-row slices with (columns per wave) / (columns per lane) lanes per
  // row: the SwiGLU epilogue (16 columns per lane) needs >= 64 columns per wave
  if constexpr (EPI == EPI_GLU && BN / WN < 64) {
    return -1;
  } else {
  const int ntiles = N / BN, Ks = K / S;
  int remap = 0;
  if (S > 1 && 8 % S == 0 && (ntiles * S) % 8 == 0) remap = 1;
  else if (S > 8 && S % 8 == 0) remap = 2;
  dim3 grid(ntiles * S, (M + BM - 1) / BM);
  mgemm_kernel<EPI, BN, BKS, NSR, WM, WN, PF><<<grid, WM * WN * 64, 0, s>>>(x, w, y, p, pv, pi, M, N, K, Ks, S,
                                                                      ntiles, remap, n_valid, ldx, ldw);
  DOCQA_CHECK_LAUNCH();
  return 0;
  }
}

template <int EPI>
int launch_cfg(int cfg, const uint16_t* x, const uint16_t* w, uint16_t* y, float* p, float* pv, int* pi,
               int M, int N, int K, int S, int n_valid, hipStream_t s, int ldx = 0, int ldw = 0) {
  if (ldx <= 0) ldx = K;
  if (ldw <= 0) ldw = K;
  switch (cfg) {
    case 1: return launch<EPI, 128, 64, 3, 2, 2>(x, w, y, p, pv, pi, M, N, K, S, n_valid, s, ldx, ldw);
    case 2: return launch<EPI, 128, 64, 3, 4, 2>(x, w, y, p, pv, pi, M, N, K, S, n_valid, s, ldx, ldw);
    case 3: return launch<EPI, 256, 32, 4, 2, 4>(x, w, y, p, pv, pi, M, N, K, S, n_valid, s, ldx, ldw);
    case 4: return launch<EPI, 256, 32, 4, 2, 2>(x, w, y, p, pv, pi, M, N, K, S, n_valid, s, ldx, ldw);
    case 5: return launch<EPI, 256, 64, 2, 2, 2, 0>(x, w, y, p, pv, pi, M, N, K, S, n_valid, s, ldx, ldw);
    case 6: return launch<EPI, 256, 64, 2, 2, 4, 0>(x, w, y, p, pv, pi, M, N, K, S, n_valid, s, ldx, ldw);
    case 7: return launch<EPI, 64, 64, 3, 4, 2>(x, w, y, p, pv, pi, M, N, K, S, n_valid, s, ldx, ldw);
    case 8: return launch<EPI, 128, 64, 3, 4, 2, 2>(x, w, y, p, pv, pi, M, N, K, S, n_valid, s, ldx, ldw);
    case 9: return launch<EPI, 128, 64, 3, 4, 2, 3>(x, w, y, p, pv, pi, M, N, K, S, n_valid, s, ldx, ldw);
    case 10: return launch<EPI, 128, 32, 6, 4, 2, 3>(x, w, y, p, pv, pi, M, N, K, S, n_valid, s, ldx, ldw);
    case 11: return launch<EPI, 128, 64, 3, 4, 2, 5>(x, w, y, p, pv, pi, M, N, K, S, n_valid, s, ldx, ldw);
    case 12: return launch<EPI, 128, 64, 3, 4, 2, 7>(x, w, y, p, pv, pi, M, N, K, S, n_valid, s, ldx, ldw);
    case 13: return launch<EPI, 64, 64, 3, 4, 2, 5>(x, w, y, p, pv, pi, M, N, K, S, n_valid, s, ldx, ldw);
    case 14: return launch<EPI, 256, 64, 2, 2, 4, 4>(x, w, y, p, pv, pi, M, N, K, S, n_valid, s, ldx, ldw);
    default: return -1;
  }
}

bool shape_ok(int M, int N, int K, int S, int cfg) {
  if (cfg < 1 || cfg > kNumCfg || M <= 0 || S < 1) return false;
  // whole pairs of stages per K slice (the main loop is unrolled by two)
  return N % kCfg[cfg].bn == 0 && K % (S * 2 * kCfg[cfg].bks) == 0;
}
}  // namespace

constexpr int kDefaultCfg = 2;
int docqa_mgemm_tile_n(int cfg) {
  if (cfg == 0) cfg = kDefaultCfg;
  return cfg >= 1 && cfg <= kNumCfg ? kCfg[cfg].bn : 0;
}

// P given: fp32 split-K slabs [S, M, N] (S >= 1, combined by the consumer); else S == 1 and
// Y bf16 [M, N]
int docqa_mgemm(const void* X, const void* W, void* Y, float* P, int M, int N, int K, int S, int cfg,
                hipStream_t s) {
  if (cfg == 0) cfg = kDefaultCfg;
  if (M == 0) return 0;
  if (!shape_ok(M, N, K, S, cfg) || (P == nullptr && (S != 1 || Y == nullptr))) return -1;
  if (!docqa_aligned16(X) || !docqa_aligned16(W) || !docqa_aligned16(P ? (void*)P : Y)) return -1;
  const uint16_t *x = (const uint16_t*)X, *w = (const uint16_t*)W;
  if (P) return launch_cfg<EPI_PARTIAL>(cfg, x, w, nullptr, P, nullptr, nullptr, M, N, K, S, N, s);
  return launch_cfg<EPI_BF16>(cfg, x, w, (uint16_t*)Y, nullptr, nullptr, nullptr, M, N, K, 1, N, s);
}

// bf16 split-K slabs Y [S, M, N] (S >= 1) for the bf16-slab consumers
int docqa_mgemm_slab16(const void* X, const void* W, void* Y, int M, int N, int K, int S, int cfg,
                       hipStream_t s) {
  if (cfg == 0) cfg = kDefaultCfg;
  if (M == 0) return 0;
  if (!shape_ok(M, N, K, S, cfg) || Y == nullptr) return -1;
  if (!docqa_aligned16(X) || !docqa_aligned16(W) || !docqa_aligned16(Y)) return -1;
  return launch_cfg<EPI_PARTIAL16>(cfg, (const uint16_t*)X, (const uint16_t*)W, (uint16_t*)Y, nullptr, nullptr,
                                   nullptr, M, N, K, S, N, s);
}

// Y[M, N/2] = silu(gate) * up for the 8-interleaved gate|up weight W [N, K] (N = 2 I)
int docqa_mgemm_glu(const void* X, const void* W, void* Y, int M, int N, int K, int cfg, hipStream_t s) {
  if (cfg == 0) cfg = kDefaultCfg;
  if (M == 0) return 0;
  if (!shape_ok(M, N, K, 1, cfg) || !docqa_aligned16(X) || !docqa_aligned16(W) || !docqa_aligned16(Y)) return -1;
  return launch_cfg<EPI_GLU>(cfg, (const uint16_t*)X, (const uint16_t*)W, (uint16_t*)Y, nullptr, nullptr, nullptr,
                             M, N, K, 1, N, s);
}

// out[M] = argmax over the first n_valid columns of bf16(X . W^T) (LM head + greedy pick),
// outv[M] (optional) its value; ws_v / ws_i: [M, N / tile_n] partials
int docqa_mgemm_argmax(const void* X, const void* W, int64_t* out, float* outv, float* ws_v, int* ws_i, int M,
                       int N, int K, int n_valid, int cfg, hipStream_t s) {
  if (cfg == 0) cfg = kDefaultCfg;
  if (M == 0) return 0;
  if (!shape_ok(M, N, K, 1, cfg) || n_valid <= 0 || n_valid > N) return -1;
  if (!docqa_aligned16(X) || !docqa_aligned16(W)) return -1;
  const int rc = launch_cfg<EPI_ARGMAX>(cfg, (const uint16_t*)X, (const uint16_t*)W, nullptr, nullptr, ws_v, ws_i,
                                        M, N, K, 1, n_valid, s);
  if (rc) return rc;
  argmax_merge_kernel<<<M, 256, 0, s>>>(ws_v, ws_i, N / kCfg[cfg].bn, out, outv);
  DOCQA_CHECK_LAUNCH();
  return 0;
}

// strided operands (row strides ldx / ldw elements, multiples of 8): the layout probe of the
// decode GEMMs (power-of-two row strides put every row of a stage on one L2 channel?)
int docqa_mgemm_ld(const void* X, int ldx, const void* W, int ldw, void* Y, float* P, int M, int N, int K, int S,
                   int cfg, int glu, hipStream_t s) {
  if (cfg == 0) cfg = kDefaultCfg;
  if (M == 0) return 0;
  if (!shape_ok(M, N, K, S, cfg) || ldx < K || ldw < K || ldx % 8 || ldw % 8) return -1;
  if (!docqa_aligned16(X) || !docqa_aligned16(W)) return -1;
  const uint16_t *x = (const uint16_t*)X, *w = (const uint16_t*)W;
  if (glu) return launch_cfg<EPI_GLU>(cfg, x, w, (uint16_t*)Y, nullptr, nullptr, nullptr, M, N, K, 1, N, s, ldx, ldw);
  if (P) return launch_cfg<EPI_PARTIAL>(cfg, x, w, nullptr, P, nullptr, nullptr, M, N, K, S, N, s, ldx, ldw);
  return launch_cfg<EPI_BF16>(cfg, x, w, (uint16_t*)Y, nullptr, nullptr, nullptr, M, N, K, 1, N, s, ldx, ldw);
}
