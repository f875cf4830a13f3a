// dgemm.hip -- skinny "decode GEMM" for the Llama generator's per-token projections:
//   Y[M, N] = X[M, K] . W[N, K]^T,   M = decode batch (<= 128), weights streamed once.
//
// At M <= 64 a projection is a weight-streaming problem (<= 64 FLOP per weight byte, far
// below the MFMA roof), so the design is about HBM bytes in flight (Little's law: ~8 TB/s x
// a few us of loaded latency = tens of KB per CU), not about tiles:
//   * workgroup = 64 weight rows x all M rows x one K slice.  W streams HBM -> LDS through
//     a 4-stage ring of 128-deep k-blocks filled by LDS-DMA (global_load_lds 16 B, source
//     XOR swizzle so the 16-row B-fragment reads are bank-conflict-free).  In-flight bytes
//     then cost LDS, not VGPRs: 2 workgroups x 3 stages x 16 KB per CU, while a register
//     double buffer (the first version of this kernel) capped M=64 at ~4.2 TB/s;
//   * X (tiny, L2-resident) goes straight to VGPRs, one k-block ahead; each wave owns a
//     disjoint (16 X rows x k-range) piece: 4 m-tiles at M=64, or 1-2 m-tiles with the
//     k-range split across waves (partials summed through LDS at the end);
//   * v_mfma_f32_16x16x32_bf16: A = X fragment, B = 4 weight n-tiles from the ring;
//   * split-K over the grid's y dimension gives >= 256 workgroups for the narrow
//     projections (O: N=4096); slices write fp32 partials reduced by a tiny second kernel,
//     S = 1 writes bf16 directly (gate|up, LM head).
//   * EPI_GLU: the Llama gate|up projection with SwiGLU fused into the epilogue.  The
//     weight rows are interleaved in blocks of 8 (gate 8b..8b+7, then up 8b..8b+7), so one
//     16-wide MFMA n-tile holds matching gate and up columns 8 lanes apart: a DPP row
//     rotate by 8 pairs them and silu(g) * u is written directly -- no [M, 2I] round trip
//     and no separate silu_mul launch.  7 n-tiles per workgroup (112 rows) make the Llama-3-8B
//     shape exactly 256 workgroups = one per CU, and halve the L2 traffic of re-reading X
//     per workgroup (at M = 64 that X traffic, not HBM, was the limiter).
//   * 65..128 rows: each wave owns two 16-row m-tiles over the whole k-block, so every
//     B fragment read from the LDS ring feeds two MFMAs and the weights still stream from
//     HBM exactly once (a second pass over 64-row halves would read them twice).
// Shapes: N % (16 NT) == 0, (K / S) % 512 == 0 (whole 4-stage ring turns), M <= 128
// (M <= 192 with 64-row weight tiles: three m-tiles per wave, no fused SwiGLU).
#include "docqa_common.h"
#include "docqa_asm.h"
#include "docqa_argmax.h"
#include "docqa_norm_row.h"
#include <stdlib.h>
#include <type_traits>

using namespace docqa;

namespace {
constexpr int BN = 64, BKD = 128, NS = 4, MR = 192;   // NS: default ring slots, K granule 4 stages
constexpr int KSTEPS = BKD / 32;               // 16x16x32 k-steps per stage
enum { EPI_BF16 = 0, EPI_PARTIAL = 1, EPI_GLU = 2, EPI_ARGMAX = 3 };
typedef __attribute__((address_space(3))) void lds_void;

// The ring's DMA / X loads are inline asm (docqa_asm.h): the counted waits below are the
// only vmcnt waits of the main loop.

template <int OFF>
__device__ __forceinline__ void gload16(bf16x8& d, const void* p) {
  asm volatile("global_load_dwordx4 %0, %1, off offset:%2" : "=v"(d) : "v"(p), "i"(OFF) : "memory");
}

// wait until at most N vector-memory ops are outstanding, naming the registers that
// become valid so nothing reading them is scheduled above the wait
// the same with the non-temporal hint: once-read weight streams (nt: aux = 2,
// MI355X_MICROARCH.md nt-weights) do not displace the L2 lines the next launch re-reads
template <int OFF>
__device__ __forceinline__ void gload16_nt(bf16x8& d, const void* p) {
  asm volatile("global_load_dwordx4 %0, %1, off offset:%2 nt" : "=v"(d) : "v"(p), "i"(OFF) : "memory");
}

template <int N, int SPW>
__device__ __forceinline__ void wait_vm_n(bf16x8 (&x)[SPW]) {
  if constexpr (SPW == 1)
    asm volatile("s_waitcnt vmcnt(%1)" : "+v"(x[0]) : "i"(N) : "memory");
  else if constexpr (SPW == 2)
    asm volatile("s_waitcnt vmcnt(%2)" : "+v"(x[0]), "+v"(x[1]) : "i"(N) : "memory");
  else if constexpr (SPW == 4)
    asm volatile("s_waitcnt vmcnt(%4)" : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]) : "i"(N) : "memory");
  else if constexpr (SPW == 8)
    asm volatile("s_waitcnt vmcnt(%8)" : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]),
                 "+v"(x[6]), "+v"(x[7]) : "i"(N) : "memory");
  else {
    static_assert(SPW == 12, "X fragment sets of 1, 2, 4, 8 or 12");
    asm volatile("s_waitcnt vmcnt(%12)" : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]),
                 "+v"(x[6]), "+v"(x[7]), "+v"(x[8]), "+v"(x[9]), "+v"(x[10]), "+v"(x[11]) : "i"(N) : "memory");
  }
}

// keep x's registers allocated up to this point (for loads that are drained, never read)
template <int SPW>
__device__ __forceinline__ void keep_live(bf16x8 (&x)[SPW]) {
#pragma unroll
  for (int s = 0; s < SPW; ++s) asm volatile("" : "+v"(x[s]));
}

__device__ __forceinline__ int w_off(int row, int ch) {  // [rows][128] stage, 16 chunks per row
  return row * BKD + ((ch ^ (row & 15)) << 3);
}

__device__ __forceinline__ float silu_f(float x) { return x / (1.f + __expf(-x)); }

// value of the lane 8 positions away inside each 16-lane row (DPP row_ror:8)
__device__ __forceinline__ float row_swap8(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x128, 0xf, 0xf, false));
}

// Wave roles: MT m-tiles of 16 X rows.  MT <= 4: the 4 waves split as (m-tile = wave % MT,
// k-group = wave / MT) so every wave owns a disjoint (rows x k) piece of the product and
// the W stage in LDS (NT 16-row n-tiles) is shared by all of them; KW = 4 / MT k-groups
// are summed through LDS at the end.  MT = 8: wave w owns m-tiles 2w, 2w+1 (MPW = 2) over
// the whole k-block (KW = 1).
// NormArgs (EPI_PARTIAL, few rows): the split-K slabs go out write-through and the LAST
// workgroup of the grid to finish (one ticket word, re-armed by it) runs the residual add +
// RMSNorm over them (docqa_norm_row.h, the add_rmsnorm_splitk arithmetic) -- the batch-1
// O / down projection then needs no add_rmsnorm_splitk launch (4.6 us each at M = 1,
// profiles/r4_batch1_kernel_stats.txt).
struct NormArgs {
  int* tick = nullptr;             // null: plain partial slabs
  uint16_t* residual = nullptr;    // [M, N] bf16, updated in place
  const uint16_t* gamma = nullptr; // [N]
  uint16_t* out = nullptr;         // [M, N] bf16 normed rows
  float eps = 0.f;
};

// XNormIn (batch 1, XN mode): the projection's input row is not read from X but built by
// the workgroup itself from the PREVIOUS projection's split-K slabs -- residual add + RMSNorm
// (the add_rmsnorm_splitk arithmetic, same thread -> chunk map, so the same bits) into LDS,
// while the first weight stages are already streaming.  One workgroup writes the updated
// residual to res_out (a second buffer: the others still read res_in), so the norm launch
// between two decode projections disappears.
struct XNormIn {
  const float* P = nullptr;          // [S, 1, K] fp32 slabs of the previous projection
  int S = 0;                         // 1..64 (up to 4 loaded in parallel)
  const uint16_t* res_in = nullptr;  // [1, K]
  uint16_t* res_out = nullptr;       // [1, K] = res_in + bf16(sum P)
  const uint16_t* gamma = nullptr;   // [K]
  float eps = 0.f;
};
constexpr int kXnMaxK = 4096;

// residual add + RMSNorm of the one input row into sx[0 .. Ks) (k slice [kbeg, kbeg + Ks))
__device__ __forceinline__ void xnorm_prologue(const XNormIn& xn, int K, int kbeg, int Ks, bool writer,
                                               uint16_t* sx, float* red) {
  constexpr int NV = kXnMaxK / 8 / 256;
  const int tid = threadIdx.x, nchunk = K >> 3;
  const uint4* rr = reinterpret_cast<const uint4*>(xn.res_in);
  const uint4* wr = reinterpret_cast<const uint4*>(xn.gamma);
  float v[NV][8];
  uint4 rres[NV], wres[NV];
  float4 pa[NV][4], pb[NV][4];
  // every load (residual, gamma, up to 4 slabs; clamped slabs loaded, not added) before the
  // first use: one memory latency, overlapped with the weight stages issued before
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = min(tid + 256 * i, nchunk - 1);
    rres[i] = rr[c];
    wres[i] = wr[c];
#pragma unroll
    for (int sl = 0; sl < 4; ++sl) {
      const float* q = xn.P + (size_t)min(sl, xn.S - 1) * K + c * 8;
      pa[i][sl] = *reinterpret_cast<const float4*>(q);
      pb[i][sl] = *reinterpret_cast<const float4*>(q + 4);
    }
  }
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = tid + 256 * i;
    if (c < nchunk) {
      float4 a = pa[i][0], b = pb[i][0];
#pragma unroll
      for (int sl = 1; sl < 4; ++sl)
        if (sl < xn.S) {
          a.x += pa[i][sl].x; a.y += pa[i][sl].y; a.z += pa[i][sl].z; a.w += pa[i][sl].w;
          b.x += pb[i][sl].x; b.y += pb[i][sl].y; b.z += pb[i][sl].z; b.w += pb[i][sl].w;
        }
      for (int sl = 4; sl < xn.S; ++sl) {   // more than 4 slabs (small models): in order, serial
        const float* q = xn.P + (size_t)sl * K + c * 8;
        const float4 a2 = *reinterpret_cast<const float4*>(q), b2 = *reinterpret_cast<const float4*>(q + 4);
        a.x += a2.x; a.y += a2.y; a.z += a2.z; a.w += a2.w;
        b.x += b2.x; b.y += b2.y; b.z += b2.z; b.w += b2.w;
      }
      const float x8[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
      float r[8];
      unpack8(rres[i], r);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[i][j] = bf2f(f2bf(bf2f(f2bf(x8[j])) + r[j]));
      if (writer) reinterpret_cast<uint4*>(xn.res_out)[c] = pack8(v[i]);
#pragma unroll
      for (int j = 0; j < 8; ++j) ss += v[i][j] * v[i][j];
    }
  }
  ss = wave_sum(ss);
  if ((tid & 63) == 0) red[tid >> 6] = ss;
  __syncthreads();
  ss = red[0] + red[1] + red[2] + red[3];
  const float inv = rsqrtf(ss / (float)K + xn.eps);
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = tid + 256 * i;
    if (c < nchunk && c * 8 >= kbeg && c * 8 < kbeg + Ks) {
      float g[8], o[8];
      unpack8(wres[i], g);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = v[i][j] * inv * g[j];
      *reinterpret_cast<uint4*>(sx + c * 8 - kbeg) = pack8(o);
    }
  }
  __syncthreads();
}

template <int EPI, int MT, int NT, int NSR, int XA = 2, bool NORM = false, bool XN = false>
__global__ __launch_bounds__(256) void dgemm_kernel(const uint16_t* __restrict__ X,
                                                    const uint16_t* __restrict__ W,
                                                    uint16_t* __restrict__ Y,
                                                    float* __restrict__ P, int M, int N, int K,
                                                    int Ks, int xcd_remap, float* __restrict__ pv = nullptr,
                                                    int* __restrict__ pi = nullptr, int n_valid = 0,
                                                    NormArgs na = NormArgs{}, XNormIn xn = XNormIn{}) {
  static_assert(!NORM || EPI == EPI_PARTIAL, "the fused norm consumes split-K slabs");
  static_assert(!XN || (MT == 1 && XA == 2), "the in-LDS input row is the one-row (batch-1) case");
  constexpr int MPW = MT > 4 ? MT / 4 : 1;       // m-tiles per wave
  constexpr int MTW = MT > 4 ? 4 : MT;           // wave groups along m
  constexpr int KW = 4 / MTW, SPW = KSTEPS / KW;
  constexpr int XR = MPW * SPW;                  // X fragments per wave per stage
  constexpr int XV = XN ? 0 : XR;                // ... of them vector-memory loads
  // vector-memory ops allowed in flight at the top of a step: XN counts exactly the NSR - 2
  // weight stages issued after this step's (deeper XN rings hide the input-row prologue);
  // the X-streaming variants keep the tuned 4-slot count
  constexpr int VW = XN ? (NSR - 2) * NT : 2 * NT + XV;
  constexpr int STAGE = NT * 16 * BKD;           // elements of one W stage (NT x 4 KB)
  static_assert(NSR >= 4, "ring needs >= 4 slots");
  static_assert(MT <= 4 || MT == 8 || MT == 12, "MT in {1, 2, 4, 8, 12}");
  __shared__ __attribute__((aligned(16))) uint16_t sw[NSR * STAGE];   // W ring
  __shared__ __attribute__((aligned(16))) uint16_t sx[XN ? kXnMaxK : 8];  // XN: the input row slice
  __shared__ float xred[4];
  // XCD-aware split-K placement: workgroups are dealt to the 8 XCDs round-robin by linear
  // id, so with the plain (tile, slice) grid every XCD sees every K slice and its 4 MB L2
  // must hold all of X next to the weight stream.  Remapped, XCD x only runs slice x % S:
  // its L2 holds 1/S of X and the re-reads of X by its workgroups hit there.
  int tile = blockIdx.x, slice = blockIdx.y;
  if (xcd_remap) {
    const int S = gridDim.y;
    const int L = blockIdx.x + blockIdx.y * gridDim.x;
    const int xcd = L & 7, j = L >> 3;
    slice = xcd % S;
    tile = j * (8 / S) + xcd / S;
  }
  const int n0 = tile * NT * 16;
  const int kbeg = slice * Ks;
  const int nkb = Ks / BKD;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fq = lane >> 4;
  const int mt = wave % MTW, kg = wave / MTW;
  const uint16_t* xrow[MPW];
#pragma unroll
  for (int mi = 0; mi < MPW; ++mi) {
    const int xr = min((mt * MPW + mi) * 16 + fr, M - 1);
    xrow[mi] = X + (size_t)xr * K + kbeg + kg * SPW * 32 + fq * 8;
  }
  const uint32_t ring = lds_u32(sw);

  f32x4 acc[MPW][NT];
#pragma unroll
  for (int mi = 0; mi < MPW; ++mi)
#pragma unroll
    for (int i = 0; i < NT; ++i) acc[mi][i] = f32x4{0.f, 0.f, 0.f, 0.f};

  // W stage j -> ring slot j % NS: 4 NT wave-instructions of 64 lanes x 16 B, NT per wave,
  // source XOR-swizzled (the DMA destination is lane-linear).  Past the last stage the
  // sources are clamped (L2 hits into free slots / dead X buffers) so that every step
  // issues the same loads unconditionally: a load whose destination is live on one path
  // and not on another lets hipcc hand its registers to other values while the data is
  // still in flight.
  const uint16_t* wsrc[NT];
#pragma unroll
  for (int i = 0; i < NT; ++i) {
    const int p = (i * 4 + wave) * 64 + lane;
    const int r = p >> 4;
    wsrc[i] = W + (size_t)(n0 + r) * K + kbeg + (((p & 15) ^ (r & 15)) << 3);
  }
  auto stage_w = [&](int j) {
    const int koff = min(j, nkb - 1) * BKD;
    const uint32_t dst = ring + (uint32_t)((j % NSR) * STAGE * 2);
#pragma unroll
    for (int i = 0; i < NT; ++i) glds16<true>(wsrc[i] + koff, dst + (uint32_t)((i * 4 + wave) * 1024));
  };
  auto load_x = [&](bf16x8 (&x)[XR], int j) {
    if constexpr (XN) {   // one row, from the prologue's LDS slice (a broadcast read)
      x[0] = *reinterpret_cast<const bf16x8*>(sx + min(j, nkb - 1) * BKD + kg * SPW * 32 + fq * 8);
      return;
    }
#pragma unroll
    for (int mi = 0; mi < MPW; ++mi) {
      const uint16_t* src = xrow[mi] + min(j, nkb - 1) * BKD;
      gload16<0>(x[mi * SPW], src);
      if constexpr (SPW > 1) gload16<64>(x[mi * SPW + 1], src);
      if constexpr (SPW > 2) { gload16<128>(x[mi * SPW + 2], src); gload16<192>(x[mi * SPW + 3], src); }
    }
  };
  auto mma = [&](const bf16x8 (&x)[XR], int j) {
    const uint16_t* src = sw + (j % NSR) * STAGE;
#pragma unroll
    for (int s = 0; s < SPW; ++s) {
      const int ch = (kg * SPW + s) * 4 + fq;
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        const bf16x8 b = *reinterpret_cast<const bf16x8*>(src + w_off(nt * 16 + fr, ch));
#pragma unroll
        for (int mi = 0; mi < MPW; ++mi)
          acc[mi][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x[mi * SPW + s], b, acc[mi][nt], 0, 0, 0);
      }
    }
  };
  // Issue order per wave (R = NSR): W0 .. W(R-4) X0 W(R-3) X1 W(R-2) | step i: X(i+2)
  // W(i+R-1).  At the top of step i the ops issued after X(i) are one W group, X(i+1) and
  // one more W group, so vmcnt(2 NT + XR) retires X(i) and (issued before it) W(i)
  // while R-2 W stages stay in flight; the barrier then publishes stage i to every wave
  // and frees slot (i-1) % R for W(i+R-1).
  bf16x8 x0[XR], x1[XR], x2[XR], x3[XR];
#define RING_STEP(I, XC, XN, NW)                                                        \
  wait_vm_n<NW>(XC);                                                                    \
  ring_barrier();                                                                       \
  load_x(XN, (I) + XA);                                                                 \
  stage_w((I) + NSR - 1);                                                               \
  mma(XC, I);
  if constexpr (XA == 2) {
    if constexpr (XN) {
      // weight stages first, then the input row (its loads overlap theirs; waiting for them
      // retires the stages too -- vmcnt is in order), then the first two X fragments
#pragma unroll
      for (int j = 0; j <= NSR - 2; ++j) stage_w(j);
      xnorm_prologue(xn, K, kbeg, Ks, blockIdx.x == 0 && blockIdx.y == 0, sx, xred);
      load_x(x0, 0);
      load_x(x1, 1);
    } else {
#pragma unroll
      for (int j = 0; j <= NSR - 4; ++j) stage_w(j);
      load_x(x0, 0);
      stage_w(NSR - 3);
      load_x(x1, 1);
      stage_w(NSR - 2);
    }
    // nkb % 4 == 0: a break-free 4-step body keeps each X buffer in one register set (an
    // early exit makes hipcc merge buffers with register copies that read in-flight data)
    for (int i = 0; i < nkb; i += 4) {
      RING_STEP(i, x0, x2, VW)
      RING_STEP(i + 1, x1, x3, VW)
      RING_STEP(i + 2, x2, x0, VW)
      RING_STEP(i + 3, x3, x1, VW)
    }
  } else {
    // X three k-blocks ahead (the 65-128-row case, where X -- not W -- is the longer
    // pole): issue W0 X0 W1 X1 W2 X2 | step i: X(i+3) W(i+3).  W(i) now follows X(i), and
    // the ops after W(i) are X(i+1) W(i+1) X(i+2) W(i+2): vmcnt(2 (NT + XR)) retires both.
    static_assert(NSR == 4, "X-ahead-3 schedule is written for a 4-slot ring");
    stage_w(0);
    load_x(x0, 0);
    stage_w(1);
    load_x(x1, 1);
    stage_w(2);
    load_x(x2, 2);
    for (int i = 0; i < nkb; i += 4) {
      RING_STEP(i, x0, x3, 2 * (NT + XR))
      RING_STEP(i + 1, x1, x0, 2 * (NT + XR))
      RING_STEP(i + 2, x2, x1, 2 * (NT + XR))
      RING_STEP(i + 3, x3, x2, 2 * (NT + XR))
    }
  }
#undef RING_STEP
  // drain the clamped tail loads; naming every X buffer keeps their registers reserved
  // until the data has landed
  wait_vm_n<0>(x0);
  keep_live(x1);
  keep_live(x2);
  keep_live(x3);

  // C/D map of 16x16x32: col = lane & 15 (weight row), row = 4 * (lane >> 4) + r (X row)
  auto store = [&](int row, int col, float v) {
    if constexpr (NORM)
      __hip_atomic_store(P + ((size_t)slice * M + row) * N + col, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else if constexpr (EPI == EPI_PARTIAL) P[((size_t)slice * M + row) * N + col] = v;
    else Y[(size_t)row * N + col] = f2bf(v);
  };
  // SwiGLU pair: gate value at an 8-block's low half, up value 8 columns later
  auto store_glu = [&](int row, int col, float g, float u) {
    const float gb = bf2f(f2bf(g)), ub = bf2f(f2bf(u));   // as the unfused bf16 GEMM output
    Y[(size_t)row * (N >> 1) + ((col >> 4) << 3) + (col & 7)] = f2bf(silu_f(gb) * ub);
  };
  if constexpr (EPI == EPI_ARGMAX) {
    // LM head + greedy pick: the [rows, 64] logit tile through LDS (past the k-group
    // reduction area), 4 lanes per row -> one (value, id) partial per (row, tile)
    constexpr int TP = NT * 16 + 1;
    __syncthreads();                                  // every wave done reading the ring
    float* tl = reinterpret_cast<float*>(sw) + (KW == 1 ? 0 : 4 * NT * 64 * 4);
    if constexpr (KW == 1) {
#pragma unroll
      for (int mi = 0; mi < MPW; ++mi)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
#pragma unroll
          for (int r = 0; r < 4; ++r) tl[((mt * MPW + mi) * 16 + fq * 4 + r) * TP + nt * 16 + fr] = acc[mi][nt][r];
    } else {
      f32x4* red = reinterpret_cast<f32x4*>(sw);      // [wave][nt][lane] = one slot
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) red[(wave * NT + nt) * 64 + lane] = acc[0][nt];
      __syncthreads();
      const float* rf = reinterpret_cast<const float*>(sw);
      for (int idx = tid; idx < MT * NT * 256; idx += 256) {
        const int r = idx & 3, ln = (idx >> 2) & 63, q = idx >> 8;
        const int nt = q % NT, m = q / NT;
        float v = 0.f;
#pragma unroll
        for (int g = 0; g < KW; ++g) v += rf[(((g * MT + m) * NT + nt) * 64 + ln) * 4 + r];
        tl[(m * 16 + (ln >> 4) * 4 + r) * TP + nt * 16 + (ln & 15)] = v;
      }
    }
    __syncthreads();
    const int ntiles = N / (NT * 16);
    for (int rr = tid >> 2; rr < MT * 16; rr += 64) {
      float bv = -FLT_MAX;
      int bi = 0x7fffffff;
      const int c0 = (tid & 3) * (NT * 4);
#pragma unroll 4
      for (int c = c0; c < c0 + NT * 4; ++c) {
        const int col = n0 + c;
        if (col < n_valid) argmax_better(bv, bi, bf2f(f2bf(tl[rr * TP + c])), col);
      }
#pragma unroll
      for (int o = 1; o <= 2; o <<= 1) {
        const float ov = __shfl_xor(bv, o, 64);
        const int oi = __shfl_xor(bi, o, 64);
        argmax_better(bv, bi, ov, oi);
      }
      if ((tid & 3) == 0 && rr < M) {
        pv[(size_t)rr * ntiles + tile] = bv;
        pi[(size_t)rr * ntiles + tile] = bi;
      }
    }
    return;
  }
  if constexpr (KW == 1) {
#pragma unroll
    for (int mi = 0; mi < MPW; ++mi)
#pragma unroll
      for (int nt = 0; nt < NT; ++nt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = (mt * MPW + mi) * 16 + fq * 4 + r, col = n0 + nt * 16 + fr;
          if constexpr (EPI == EPI_GLU) {
            const float u = row_swap8(acc[mi][nt][r]);
            if (row < M && (fr & 8) == 0) store_glu(row, col, acc[mi][nt][r], u);
          } else if (row < M) {
            store(row, col, acc[mi][nt][r]);
          }
        }
  } else {
    // sum the KW k-groups through LDS (ring is free after the last barrier + wait)
    __syncthreads();
    f32x4* red = reinterpret_cast<f32x4*>(sw);        // [wave][nt][lane] = one slot
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) red[(wave * NT + nt) * 64 + lane] = acc[0][nt];
    __syncthreads();
    const float* rf = reinterpret_cast<const float*>(sw);
    auto sum_k = [&](int m, int nt, int ln, int r) {
      float v = 0.f;
#pragma unroll
      for (int g = 0; g < KW; ++g) v += rf[(((g * MT + m) * NT + nt) * 64 + ln) * 4 + r];
      return v;
    };
#pragma unroll
    for (int e = 0; e < MT * NT; ++e) {
      const int idx = e * 256 + tid;                 // (m-tile, nt, lane, r)
      const int r = idx & 3, ln = (idx >> 2) & 63, q = idx >> 8;
      const int nt = q % NT, m = q / NT;
      const int row = m * 16 + (ln >> 4) * 4 + r, col = n0 + nt * 16 + (ln & 15);
      if (row >= M) continue;
      if constexpr (EPI == EPI_GLU) {
        if ((ln & 8) == 0) store_glu(row, col, sum_k(m, nt, ln, r), sum_k(m, nt, ln + 8, r));
      } else {
        store(row, col, sum_k(m, nt, ln, r));
      }
    }
  }
  if constexpr (NORM) {
    __shared__ int s_last;
    __shared__ float red[4];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this workgroup's slab pieces landed
    __syncthreads();
    if (tid == 0) {
      const int old = __hip_atomic_fetch_add(na.tick, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      s_last = old == (int)(gridDim.x * gridDim.y) - 1;
      if (s_last) __hip_atomic_store(na.tick, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    if (!s_last) return;
    const int S = gridDim.y;
    for (int row = 0; row < M; ++row) {
      if (S == 4)
        add_rmsnorm_splitk_row<4, 4, false, true>(P, S, (size_t)M * N, na.residual, na.gamma, na.out, N, na.eps,
                                                  row, tid, red);
      else
        add_rmsnorm_splitk_row<4, 0, false, true>(P, S, (size_t)M * N, na.residual, na.gamma, na.out, N, na.eps,
                                                  row, tid, red);
      __syncthreads();   // red reused by the next row
    }
  }
}

__global__ __launch_bounds__(256) void splitk_reduce_kernel(const float* __restrict__ P,
                                                            uint16_t* __restrict__ Y, int MN, int S) {
  const int i = (blockIdx.x * 256 + threadIdx.x) * 4;
  if (i >= MN) return;
  float4 acc = *reinterpret_cast<const float4*>(P + i);
  for (int s = 1; s < S; ++s) {
    const float4 v = *reinterpret_cast<const float4*>(P + (size_t)s * MN + i);
    acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
  }
  uint2 o;
  o.x = pack2(acc.x, acc.y);
  o.y = pack2(acc.z, acc.w);
  *reinterpret_cast<uint2*>(Y + i) = o;
}
}  // namespace

// split count: enough workgroups for the chip (>= 256), K slices of whole ring turns
int docqa_dgemm_splits(int N, int K) {
  const int tiles = N / BN;
  int s = 1;
  while (tiles * s < 256 && K % (s * 2) == 0 && (K / (s * 2)) % (NS * BKD) == 0)
    s *= 2;
  return s;
}

static int xa_knob() {   // X prefetch distance for 65-128 rows (tuning experiments)
  static const int v = [] {
    const char* e = getenv("DOCQA_DGEMM_XA");
    return e ? atoi(e) : 0;
  }();
  return v;
}

static int xcd_knob() {   // XCD-aware slice placement (A/B experiments): 1 on, 0 off
  static const int v = [] {
    const char* e = getenv("DOCQA_DGEMM_XCD");
    return e ? atoi(e) : 1;
  }();
  return v;
}

template <int EPI, int NT, int NSR = NS>
static void launch_mt(int mt, dim3 grid, hipStream_t s, const uint16_t* x, const uint16_t* w,
                      uint16_t* y, float* p, int M, int N, int K, int Ks, float* pv = nullptr,
                      int* pi = nullptr, int nv = 0) {
  const int S = grid.y;
  const int xr = (xcd_knob() && S > 1 && 8 % S == 0 && (grid.x * S) % 8 == 0) ? 1 : 0;
  if (mt == 1) dgemm_kernel<EPI, 1, NT, NSR><<<grid, 256, 0, s>>>(x, w, y, p, M, N, K, Ks, xr, pv, pi, nv);
  else if (mt == 2) dgemm_kernel<EPI, 2, NT, NSR><<<grid, 256, 0, s>>>(x, w, y, p, M, N, K, Ks, xr, pv, pi, nv);
  else if (mt <= 4) dgemm_kernel<EPI, 4, NT, NSR><<<grid, 256, 0, s>>>(x, w, y, p, M, N, K, Ks, xr, pv, pi, nv);
  else if (mt <= 8) {
    if constexpr (NSR == 4) {
      if (xa_knob() == 3)
        dgemm_kernel<EPI, 8, NT, NSR, 3><<<grid, 256, 0, s>>>(x, w, y, p, M, N, K, Ks, xr, pv, pi, nv);
      else dgemm_kernel<EPI, 8, NT, NSR><<<grid, 256, 0, s>>>(x, w, y, p, M, N, K, Ks, xr, pv, pi, nv);
    } else {
      dgemm_kernel<EPI, 8, NT, NSR><<<grid, 256, 0, s>>>(x, w, y, p, M, N, K, Ks, xr, pv, pi, nv);
    }
  } else if constexpr (NT <= 8 && EPI != EPI_GLU) {
    // 129-192 rows: three m-tiles per wave
    dgemm_kernel<EPI, 12, NT, NSR><<<grid, 256, 0, s>>>(x, w, y, p, M, N, K, Ks, xr, pv, pi, nv);
  }
}

static bool shape_ok(int M, int N, int K, int S, int bn) {
  return M <= MR && N % bn == 0 && S >= 1 && K % S == 0 && (K / S) % (NS * BKD) == 0;
}

int docqa_dgemm(const void* X, const void* W, void* Y, float* partial, int M, int N, int K,
                int S, hipStream_t s) {
  if (M == 0) return 0;
  if (!shape_ok(M, N, K, S, BN) || (S > 1 && !partial)) return -1;
  dim3 grid(N / BN, S);
  const int mt = (M + 15) / 16;
  const uint16_t* x = (const uint16_t*)X;
  const uint16_t* w = (const uint16_t*)W;
  if (S == 1) {
    launch_mt<EPI_BF16, 4>(mt, grid, s, x, w, (uint16_t*)Y, nullptr, M, N, K, K);
  } else {
    launch_mt<EPI_PARTIAL, 4>(mt, grid, s, x, w, nullptr, partial, M, N, K, K / S);
    const int MN = M * N;  // multiple of 4 (N % 64 == 0)
    splitk_reduce_kernel<<<(MN / 4 + 255) / 256, 256, 0, s>>>(partial, (uint16_t*)Y, MN, S);
  }
  DOCQA_CHECK_LAUNCH();
  return 0;
}

// split-K partial slabs only (S >= 1, P: [S, M, N] fp32): the combine is fused into the
// consumer (add_rmsnorm_splitk / rope_cache_splitk)
int docqa_dgemm_partial(const void* X, const void* W, float* P, int M, int N, int K, int S,
                        int tile_rows, hipStream_t s) {
  if (M == 0) return 0;
  if (!P || (tile_rows != 64 && tile_rows != 128) || !shape_ok(M, N, K, S, tile_rows)) return -1;
  const int mt = (M + 15) / 16;
  const uint16_t* x = (const uint16_t*)X;
  const uint16_t* w = (const uint16_t*)W;
  static const int ns_env = [] {   // ring depth knob (tuning experiments)
    const char* e = getenv("DOCQA_DGEMM_NS");
    return e ? atoi(e) : 0;
  }();
  if (tile_rows == 128)   // 1 workgroup per CU (128 KB ring), X re-read half as often
    launch_mt<EPI_PARTIAL, 8>(mt, dim3(N / 128, S), s, x, w, nullptr, P, M, N, K, K / S);
  else if (ns_env == 6)
    launch_mt<EPI_PARTIAL, 4, 6>(mt, dim3(N / 64, S), s, x, w, nullptr, P, M, N, K, K / S);
  else if (ns_env == 8)
    launch_mt<EPI_PARTIAL, 4, 8>(mt, dim3(N / 64, S), s, x, w, nullptr, P, M, N, K, K / S);
  else
    launch_mt<EPI_PARTIAL, 4>(mt, dim3(N / 64, S), s, x, w, nullptr, P, M, N, K, K / S);
  DOCQA_CHECK_LAUNCH();
  return 0;
}

// Few-row split-K projection with the residual add + RMSNorm fused in (NormArgs): P [S, M, N]
// fp32 slabs (scratch), residual [M, N] updated, out [M, N] = rmsnorm(residual) * gamma.
// M <= kNormRows, N <= 8192 (4 chunks of 8 per lane), 64-row weight tiles.
constexpr int kNormRows = 4;
int docqa_dgemm_add_rmsnorm(const void* X, const void* W, float* P, int M, int N, int K, int S, void* residual,
                            const void* gamma, void* out, float eps, int* tick, hipStream_t s) {
  if (M == 0) return 0;
  if (M > kNormRows || N > 8192 || N % 8 || !tick || !P || !shape_ok(M, N, K, S, BN)) return -1;
  NormArgs na{tick, (uint16_t*)residual, (const uint16_t*)gamma, (uint16_t*)out, eps};
  const dim3 grid(N / BN, S);
  const int xr = (xcd_knob() && S > 1 && 8 % S == 0 && (grid.x * S) % 8 == 0) ? 1 : 0;
  dgemm_kernel<EPI_PARTIAL, 1, 4, NS, 2, true><<<grid, 256, 0, s>>>((const uint16_t*)X, (const uint16_t*)W, nullptr,
                                                                    P, M, N, K, K / S, xr, nullptr, nullptr, 0, na);
  DOCQA_CHECK_LAUNCH();
  return 0;
}

// Batch-1 projections whose input row is rmsnorm(res_in + bf16(sum of the previous
// projection's slabs)) * gamma, built in LDS by each workgroup (XNormIn): split-K slabs out
// (the next layer's QKV) or the fused SwiGLU (gate|up).  res_out <- res_in + bf16(sum Pin).
static bool xn_ok(int N, int K, int S, int bn, const XNormIn& xn) {
  return K <= kXnMaxK && xn.S >= 1 && xn.S <= 64 && xn.P && xn.res_in && xn.res_out &&
         xn.gamma && xn.res_in != xn.res_out && shape_ok(1, N, K, S, bn);
}

int docqa_dgemm_partial_xn(const float* Pin, int Sin, const void* res_in, void* res_out, const void* gamma,
                           float eps, const void* W, float* P, int N, int K, int S, hipStream_t s) {
  const XNormIn xn{Pin, Sin, (const uint16_t*)res_in, (uint16_t*)res_out, (const uint16_t*)gamma, eps};
  if (!P || !xn_ok(N, K, S, BN, xn)) return -1;
  const dim3 grid(N / BN, S);
  const int xr = (xcd_knob() && S > 1 && 8 % S == 0 && (grid.x * S) % 8 == 0) ? 1 : 0;
  // (an 8-slot ring to stream on under the input-row prologue measured slower: QKV 17.7 vs
  // 16.4 us, profiles/r4_b1_ab.log)
  dgemm_kernel<EPI_PARTIAL, 1, 4, NS, 2, false, true><<<grid, 256, 0, s>>>(
      nullptr, (const uint16_t*)W, nullptr, P, 1, N, K, K / S, xr, nullptr, nullptr, 0, NormArgs{}, xn);
  DOCQA_CHECK_LAUNCH();
  return 0;
}

int docqa_dgemm_glu_xn(const float* Pin, int Sin, const void* res_in, void* res_out, const void* gamma, float eps,
                       const void* W, void* Y, int N, int K, hipStream_t s) {
  const XNormIn xn{Pin, Sin, (const uint16_t*)res_in, (uint16_t*)res_out, (const uint16_t*)gamma, eps};
  if (xn_ok(N, K, 1, 112, xn) && N / 112 >= 192)
    dgemm_kernel<EPI_GLU, 1, 7, NS, 2, false, true><<<dim3(N / 112), 256, 0, s>>>(
        nullptr, (const uint16_t*)W, (uint16_t*)Y, nullptr, 1, N, K, K, 0, nullptr, nullptr, 0, NormArgs{}, xn);
  else if (xn_ok(N, K, 1, 64, xn))
    dgemm_kernel<EPI_GLU, 1, 4, NS, 2, false, true><<<dim3(N / 64), 256, 0, s>>>(
        nullptr, (const uint16_t*)W, (uint16_t*)Y, nullptr, 1, N, K, K, 0, nullptr, nullptr, 0, NormArgs{}, xn);
  else
    return -1;
  DOCQA_CHECK_LAUNCH();
  return 0;
}

// Y[M, N/2] = silu(gate) * up for the 8-interleaved gate|up weight W [N, K] (N = 2 I)
int docqa_dgemm_glu(const void* X, const void* W, void* Y, int M, int N, int K, hipStream_t s) {
  if (M == 0) return 0;
  if (M > 128) return -1;
  const int mt = (M + 15) / 16;
  const uint16_t* x = (const uint16_t*)X;
  const uint16_t* w = (const uint16_t*)W;
  static const int glu_nt = [] {   // tile-width knob (tuning experiments): 4 -> 64-row tiles
    const char* e = getenv("DOCQA_GLU_NT");
    return e ? atoi(e) : 0;
  }();
  if (glu_nt != 4 && shape_ok(M, N, K, 1, 112) && N / 112 >= 192) {
    launch_mt<EPI_GLU, 7>(mt, dim3(N / 112), s, x, w, (uint16_t*)Y, nullptr, M, N, K, K);
  } else if (shape_ok(M, N, K, 1, 64)) {
    launch_mt<EPI_GLU, 4>(mt, dim3(N / 64), s, x, w, (uint16_t*)Y, nullptr, M, N, K, K);
  } else {
    return -1;
  }
  DOCQA_CHECK_LAUNCH();
  return 0;
}

// LM head + greedy pick at <= 192 rows (batch-1 decode included): out[M] = argmax over the
// first n_valid columns of bf16(X . W^T), outv[M] (optional) the picked value; ws_v / ws_i:
// [M, N / 64] per-tile partials.  The [M, vocab] logits never reach HBM.
int docqa_dgemm_argmax(const void* X, const void* W, int64_t* out, float* outv, float* ws_v, int* ws_i, int M,
                       int N, int K, int n_valid, hipStream_t s) {
  if (M == 0) return 0;
  if (!shape_ok(M, N, K, 1, BN) || n_valid <= 0 || n_valid > N) return -1;
  const int mt = (M + 15) / 16;
  launch_mt<EPI_ARGMAX, 4>(mt, dim3(N / BN), s, (const uint16_t*)X, (const uint16_t*)W, nullptr, nullptr, M, N, K,
                           K, ws_v, ws_i, n_valid);
  argmax_merge_kernel<<<M, 256, 0, s>>>(ws_v, ws_i, N / BN, out, outv);
  DOCQA_CHECK_LAUNCH();
  return 0;
}

// ---------------------------------------------------------------------------------------
// Batch-1 GEMV (one decode row): y[N] = x[K] . W[N, K]^T with NO MFMA and NO LDS ring.  At
// M = 1 the projection is a pure weight stream, and the ring kernel above tops out at
// ~4.3 TB/s there (profiles/r4_b1_decode_gemm_split_probe.log) with two 16-KB stages in
// flight per workgroup.  Here every lane issues ALL of its weight loads at once, straight
// into VGPRs (R weight rows x C 16-B chunks: 32 loads = 128 KB per 256-thread workgroup in
// flight for the 4096-wide projections), then retires them row by row in issue order
// (vmcnt counts loads back in order) into v_dot2_f32_bf16 dot products against the input
// row; the 4 waves split K and meet in LDS.  Workgroup = R output rows x one K slice.
//   * EPI_PARTIAL: fp32 slab P[slice][n] for the split-K consumers (same layout as dgemm);
//   * EPI_GLU: R = 16 rows = one 8-interleaved gate|up group -> 8 SwiGLU outputs, bf16;
//   * XN: the input row is built in LDS from the previous projection's slabs (XNormIn),
//     its loads queued behind the weight loads (the stream is already in flight).
// Shapes: N % R == 0, Ks = K / S with Ks % 2048 == 0 (C = Ks / 2048 chunks per lane), and
// R x C <= 32 loads per lane (the 6-bit vmcnt counter holds at most 63 outstanding).
template <int I, int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for<I + 1, N>(f);
  }
}

template <int R, int C, int EPI, bool XN, bool NTW>
__global__ __launch_bounds__(256) void gemv_kernel(const uint16_t* __restrict__ X, const uint16_t* __restrict__ W,
                                                   uint16_t* __restrict__ Y, float* __restrict__ P, int N, int K,
                                                   int Ks, XNormIn xn, int* __restrict__ pi = nullptr,
                                                   int n_valid = 0) {
  static_assert(EPI == EPI_PARTIAL || (EPI == EPI_GLU && R == 16) || (EPI == EPI_ARGMAX && R == 16),
                "GLU: one 16-row gate|up group; ARGMAX: 16 logits per workgroup");
  static_assert(R * C <= 32, "loads in flight per lane must fit the vmcnt counter");
  __shared__ __attribute__((aligned(16))) uint16_t sx[XN ? kXnMaxK : 8];
  __shared__ float red[4][R];
  __shared__ float xred[4];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int n0 = blockIdx.x * R, slice = blockIdx.y, kbeg = slice * Ks;
  const int kq = Ks >> 2;                         // k per wave
  const int kw = kbeg + wave * kq;                // this wave's k range
  // weight chunk (r, c) of this lane: row n0 + r, k = kw + c * 512 + lane * 8
  bf16x8 w[R][C];
  const uint16_t* wb = W + (size_t)n0 * K + kw + lane * 8;
#pragma unroll
  for (int r = 0; r < R; ++r)
#pragma unroll
    for (int c = 0; c < C; ++c) {
      if constexpr (NTW) gload16_nt<0>(w[r][c], wb + (size_t)r * K + c * 512);
      else gload16<0>(w[r][c], wb + (size_t)r * K + c * 512);
    }
  bf16x8 x[C];
  if constexpr (XN) {
    xnorm_prologue(xn, K, kbeg, Ks, blockIdx.x == 0 && blockIdx.y == 0, sx, xred);
#pragma unroll
    for (int c = 0; c < C; ++c) x[c] = *reinterpret_cast<const bf16x8*>(sx + (kw - kbeg) + c * 512 + lane * 8);
  } else {
#pragma unroll
    for (int c = 0; c < C; ++c) x[c] = *reinterpret_cast<const bf16x8*>(X + kw + c * 512 + lane * 8);
  }
  float acc[R];
  static_for<0, R>([&](auto rc) {
    constexpr int r = decltype(rc)::value;
    // row r's chunks landed: everything issued after them is the later rows' C chunks each
    constexpr int LEFT = (R - 1 - r) * C;
    if constexpr (C == 1) wait_vm_n<LEFT, 1>(*reinterpret_cast<bf16x8(*)[1]>(&w[r][0]));
    else if constexpr (C == 2) wait_vm_n<LEFT, 2>(*reinterpret_cast<bf16x8(*)[2]>(&w[r][0]));
    else if constexpr (C == 4) wait_vm_n<LEFT, 4>(*reinterpret_cast<bf16x8(*)[4]>(&w[r][0]));
    else {
      static_assert(C == 7, "C in {1, 2, 4, 7}");
      asm volatile("s_waitcnt vmcnt(%7)" : "+v"(w[r][0]), "+v"(w[r][1]), "+v"(w[r][2]), "+v"(w[r][3]), "+v"(w[r][4]),
                   "+v"(w[r][5]), "+v"(w[r][6]) : "i"(LEFT) : "memory");
    }
    float a = 0.f;
#pragma unroll
    for (int c = 0; c < C; ++c) {
      const bf16x8 wv = w[r][c], xv = x[c];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const bf16x2 wa = {wv[2 * j], wv[2 * j + 1]}, xa = {xv[2 * j], xv[2 * j + 1]};
        a = __builtin_amdgcn_fdot2_f32_bf16(wa, xa, a, false);
      }
    }
    acc[r] = wave_sum(a);
  });
  if (lane == 0) {
#pragma unroll
    for (int r = 0; r < R; ++r) red[wave][r] = acc[r];
  }
  __syncthreads();
  if constexpr (EPI == EPI_PARTIAL) {
    if (tid < R) P[(size_t)slice * N + n0 + tid] = red[0][tid] + red[1][tid] + red[2][tid] + red[3][tid];
  } else if constexpr (EPI == EPI_ARGMAX) {
    // LM head + greedy pick: the 16 logits (bf16-rounded, as the unfused logits) -> one
    // (value, id) partial per workgroup at P / pi [blockIdx.x] for argmax_merge_kernel
    if (tid < 64) {
      float bv = -FLT_MAX;
      int bi = 0x7fffffff;
      if (tid < R && n0 + tid < n_valid) {
        bv = bf2f(f2bf(red[0][tid] + red[1][tid] + red[2][tid] + red[3][tid]));
        bi = n0 + tid;
      }
#pragma unroll
      for (int o = 1; o < R; o <<= 1) {
        const float ov = __shfl_xor(bv, o, 64);
        const int oi = __shfl_xor(bi, o, 64);
        argmax_better(bv, bi, ov, oi);
      }
      if (tid == 0) {
        P[blockIdx.x] = bv;
        pi[blockIdx.x] = bi;
      }
    }
  } else {
    // gate rows n0 .. n0 + 7, up rows n0 + 8 .. n0 + 15 -> outputs n0 / 2 .. n0 / 2 + 7
    if (tid < 8) {
      const float g = red[0][tid] + red[1][tid] + red[2][tid] + red[3][tid];
      const float u = red[0][tid + 8] + red[1][tid + 8] + red[2][tid + 8] + red[3][tid + 8];
      const float gv = bf2f(f2bf(g)), uv = bf2f(f2bf(u));   // as the bf16 GEMM output
      Y[(n0 >> 1) + tid] = f2bf(silu_f(gv) * uv);
    }
  }
}

// weight-load policy: nt by default (batch-1 p50 454 -> 439 ms, profiles/r6_b1_nt_down_ab.log);
// DOCQA_GEMV_NT=0 for the default policy
static bool gemv_nt() {
  static const bool v = [] {
    const char* e = getenv("DOCQA_GEMV_NT");
    return e ? atoi(e) != 0 : true;
  }();
  return v;
}

template <int EPI, bool XN>
static int launch_gemv(int R, int C, dim3 grid, hipStream_t s, const uint16_t* x, const uint16_t* w, uint16_t* y,
                       float* p, int N, int K, int Ks, const XNormIn& xn) {
  const bool nt = gemv_nt();
#define GEMV_CASE(RR, CC)                                                                                    \
  if (R == RR && C == CC) {                                                                                  \
    if (nt) gemv_kernel<RR, CC, EPI, XN, true><<<grid, 256, 0, s>>>(x, w, y, p, N, K, Ks, xn);               \
    else gemv_kernel<RR, CC, EPI, XN, false><<<grid, 256, 0, s>>>(x, w, y, p, N, K, Ks, xn);                 \
    return 0;                                                                                                \
  }
  if constexpr (EPI == EPI_GLU) {
    GEMV_CASE(16, 1) GEMV_CASE(16, 2)
  } else if constexpr (EPI == EPI_ARGMAX) {
    return -1;   // docqa_gemv_argmax launches its own instantiations
  } else {
    GEMV_CASE(16, 1) GEMV_CASE(16, 2) GEMV_CASE(8, 2) GEMV_CASE(8, 4) GEMV_CASE(4, 4) GEMV_CASE(4, 7)
    GEMV_CASE(8, 1) GEMV_CASE(4, 2) GEMV_CASE(4, 1)
  }
#undef GEMV_CASE
  return -1;
}

// Batch-1 GEMV (see gemv_kernel).  epi 0: fp32 slabs P [S, 1, N]; epi 1: SwiGLU Y [1, N / 2]
// (R = 16, S = 1).  xn (nullable): the input row from the previous projection's slabs.
int docqa_gemv(const void* X, const void* W, void* Y, float* P, int N, int K, int S, int R, int epi,
               const float* Pin, int Sin, const void* res_in, void* res_out, const void* gamma, float eps,
               hipStream_t s) {
  if (S < 1 || K % S || (K / S) % 2048 || N % R || R < 1) return -1;
  const int Ks = K / S, C = Ks / 2048;
  const bool xnm = Pin != nullptr;
  const XNormIn xn{Pin, Sin, (const uint16_t*)res_in, (uint16_t*)res_out, (const uint16_t*)gamma, eps};
  if (xnm && !xn_ok(N, K, 1, R, xn)) return -1;
  if (!xnm && !X) return -1;
  if (epi == 1 ? (R != 16 || S != 1 || !Y) : !P) return -1;
  const dim3 grid(N / R, S);
  const uint16_t* x = (const uint16_t*)X;
  const uint16_t* w = (const uint16_t*)W;
  int rc;
  if (epi == 1)
    rc = xnm ? launch_gemv<EPI_GLU, true>(R, C, grid, s, x, w, (uint16_t*)Y, nullptr, N, K, Ks, xn)
             : launch_gemv<EPI_GLU, false>(R, C, grid, s, x, w, (uint16_t*)Y, nullptr, N, K, Ks, xn);
  else
    rc = xnm ? launch_gemv<EPI_PARTIAL, true>(R, C, grid, s, x, w, nullptr, P, N, K, Ks, xn)
             : launch_gemv<EPI_PARTIAL, false>(R, C, grid, s, x, w, nullptr, P, N, K, Ks, xn);
  if (rc) return rc;
  DOCQA_CHECK_LAUNCH();
  return 0;
}

// Batch-1 LM head + greedy pick on the GEMV: 16 vocabulary rows per workgroup (C = K / 2048
// chunks per lane, nt weight loads), one (value, id) partial each, merged by
// argmax_merge_kernel.  ws_v / ws_i: N / 16 entries.
int docqa_gemv_argmax(const void* X, const void* W, int64_t* out, float* outv, float* ws_v, int* ws_i, int N, int K,
                      int n_valid, hipStream_t s) {
  if (N % 16 || K % 2048 || K / 2048 > 2 || n_valid <= 0 || n_valid > N) return -1;
  const dim3 grid(N / 16);
  const XNormIn xn{};
  const uint16_t* x = (const uint16_t*)X;
  const uint16_t* w = (const uint16_t*)W;
  if (K == 2048)
    gemv_kernel<16, 1, EPI_ARGMAX, false, true><<<grid, 256, 0, s>>>(x, w, nullptr, ws_v, N, K, K, xn, ws_i, n_valid);
  else
    gemv_kernel<16, 2, EPI_ARGMAX, false, true><<<grid, 256, 0, s>>>(x, w, nullptr, ws_v, N, K, K, xn, ws_i, n_valid);
  argmax_merge_kernel<<<1, 256, 0, s>>>(ws_v, ws_i, N / 16, out, outv);
  DOCQA_CHECK_LAUNCH();
  return 0;
}
