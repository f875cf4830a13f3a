// pgemm.hip -- prefill GEMM for the Llama generator (large M: packed prompt tokens)
//   C[M, N] = A[M, K] . W[N, K]^T           (bf16 in, fp32 accumulate, bf16 out)
//   C[M, N/2] = silu(gate) * up             (EPI_GLU: W = the 8-interleaved gate|up rows)
// Replaces hipBLASLt for the prefill QKV / O / gate|up (+ fused SwiGLU) / down projections
// (llm-qa/main.py:117 -> prefill inside Ollama in the reference).
//
// Structure: the 256 x 256 x 64 "8-phase" schedule of cdna_hip_programming.md §5 (T1-T5),
// written for this kernel's own stage / read plan:
//   * 8 waves (512 threads, 1 workgroup per CU): wave (wr, wc) owns rows 128 wr .. +127 x
//     cols 64 wc .. +63 as 2 x 4 x 2 x 2 v_mfma_f32_16x16x32_bf16 accumulators (128 regs);
//   * LDS: two K-tile buffers (even / odd K-tiles) of 64 KiB, each cut into four 16-KiB
//     half-tiles whose rows are chosen so that every half is read in ONE phase window:
//       HA0 = the first 64 rows of both wave rows, HA1 = their last 64 rows,
//       HB0 = the first 32 columns of all four wave columns, HB1 = their last 32;
//   * a K-tile is computed in 4 phases, each one C quadrant x K = 64 = 16 MFMAs per wave:
//       phase 1: read HA0 + HB0 -> (m-half 0, n-half 0)      12 ds_read_b128
//       phase 2: read HB1       -> (0, 1)                     4
//       phase 3: read HA1       -> (1, 1)                     8
//       phase 4: (no reads)     -> (1, 0)                     0  (HB0 fragments kept)
//     so HA0 / HB0 are free again after phase 1, HB1 after phase 2, HA1 after phase 3;
//   * every phase issues ONE half-tile of LDS-DMA (global_load_lds_dwordx4, 2 per wave)
//     for a later K-tile into a half whose last read is >= 2 phases back, and retires the
//     half-tile issued 4 phases earlier with a counted `s_waitcnt vmcnt(8)`: 4 half-tiles
//     (64 KiB per CU) stay in flight across the raw s_barriers, and each is read one phase
//     after the wait that retires it (schedule and proof in the comment at `iteration`);
//   * the two wave rows run staggered by one barrier (ping-pong): while waves 0-3 issue
//     their MFMA burst, waves 4-7 (the other wave of each SIMD) read LDS and issue DMA;
//   * XOR-swizzled half-tiles (16-B chunk ^ ((row >> 1) & 7)), applied to the per-lane DMA
//     SOURCE address (rule 21): the 16-row fragment reads are bank-conflict-free;
//   * XCD-aware bijective block remap + groups of 4 m-tiles so an XCD's concurrent
//     workgroups share A rows and W columns in its L2 (T1);
//   * epilogue through the drained LDS: bf16 tile, fused SwiGLU, or fp32 split-K slabs
//     (decode-sized M: K split over workgroups, one slice per XCD, the slabs combined by
//     the consumer -- RoPE + KV write, add + RMSNorm, or the TP all-reduce);
// Shapes: N % 256 == 0, K % (128 S) == 0, any M (tail rows clamped on load, never stored);
// byte offsets of A and W rows must fit 32 bits (saddr + voffset addressing).
#include "docqa_common.h"
#include "docqa_asm.h"
#include <float.h>

using namespace docqa;

namespace {
constexpr int BM = 256, BN = 256, BK = 64;
constexpr int HALF_B = 128 * BK * 2;     // bytes of one half-tile (16 KiB)
constexpr int BUF_B = 4 * HALF_B;        // bytes of one K-tile buffer (64 KiB)
constexpr int SCR_PITCH = 72;            // epilogue scratch row pitch (bf16), 144 B
constexpr int LDS_B = (2 * BUF_B > 8 * 128 * SCR_PITCH * 2) ? 2 * BUF_B : 8 * 128 * SCR_PITCH * 2;
enum { HA0 = 0, HA1 = 1, HB0 = 2, HB1 = 3 };
enum { EPI_BF16 = 0, EPI_GLU = 1, EPI_PARTIAL = 2 };

// byte offset of logical 16-B chunk `ch` of `row` inside a [128][64] bf16 half-tile
__device__ __forceinline__ uint32_t swz(int row, int ch) {
  return (uint32_t)(row * 128 + ((ch ^ ((row >> 1) & 7)) << 4));
}

__device__ __forceinline__ void sbarrier() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_barrier" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

template <int N>
__device__ __forceinline__ void vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" :: "i"(N) : "memory");
}

// the two 1-KiB LDS-DMA wave-instructions of one half-tile: 64-bit wave-uniform source
// base + per-lane 32-bit byte offsets (saddr form), LDS destinations in M0 (wave-uniform)
__device__ __forceinline__ void glds_pair(const void* sbase, uint32_t v0, uint32_t v1, uint32_t l0,
                                          uint32_t l1) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %4\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %1, %3\n\t"
      "s_mov_b32 m0, %5\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %2, %3\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(v0), "v"(v1), "s"(sbase), "s"(l0), "s"(l1)
      : "memory");
}

__device__ __forceinline__ float silu_f(float x) { return x / (1.f + __expf(-x)); }

// K range [kbeg, kbeg + 128 nit) of the 256 x 256 output tile at (m0, n0) into acc (zeroed
// here), nit >= 1.  Returns with the wave rows re-aligned and every LDS buffer drained, so
// the caller may reuse the LDS as epilogue scratch.
__device__ __forceinline__ void pgemm_mainloop(char* smem, const uint16_t* __restrict__ A,
                                               const uint16_t* __restrict__ W, int M, int K, int m0, int n0,
                                               int kbeg, int nit, f32x4 (&acc)[2][4][2][2]) {
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3;
  const int fr = lane & 15, fk = lane >> 4;
  const uint32_t lds = lds_u32(smem);

  // ---- per-lane DMA source offsets (bytes, k = 0) of the 4 half-tiles x 2 instructions
  uint32_t soff[4][2];
#pragma unroll
  for (int h = 0; h < 4; ++h)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int p = (i * 8 + wave) * 64 + lane;      // physical 16-B chunk of the half-tile
      const int lr = p >> 3;                         // half-tile row 0..127
      const int lc = (p & 7) ^ ((lr >> 1) & 7);      // logical chunk stored there
      int grow;
      if (h == HA0 || h == HA1) {
        grow = min(m0 + (lr >> 6) * 128 + (h == HA1 ? 64 : 0) + (lr & 63), M - 1);
      } else {
        grow = n0 + (lr >> 5) * 64 + (h == HB1 ? 32 : 0) + (lr & 31);
      }
      soff[h][i] = (uint32_t)grow * (uint32_t)(K * 2) + (uint32_t)(lc * 16);
    }
  // stage half-tile h of K-tile kt into buffer kt & 1
  auto stage = [&](int h, int kt) {
    const uint16_t* base = (h == HA0 || h == HA1 ? A : W) + kbeg + kt * BK;
    const uint32_t d = __builtin_amdgcn_readfirstlane(lds + (uint32_t)((kt & 1) * BUF_B + h * HALF_B + wave * 1024));
    glds_pair(base, soff[h][0], soff[h][1], d, d + 8 * 1024);
  };

#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[a][i][b][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  bf16x8 fa[2][4];       // [k-step][m-tile] of the current m-half
  bf16x8 fb[2][2][2];    // [n-half][k-step][n-tile]
  const char* sm = smem;

  auto read_a = [&](int buf, int mh) {
    const char* h = sm + buf * BUF_B + (HA0 + mh) * HALF_B;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 4; ++i)
        fa[ks][i] = *reinterpret_cast<const bf16x8*>(h + swz(wr * 64 + i * 16 + fr, ks * 4 + fk));
  };
  auto read_b = [&](int buf, int nh) {
    const char* h = sm + buf * BUF_B + (HB0 + nh) * HALF_B;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        fb[nh][ks][j] = *reinterpret_cast<const bf16x8*>(h + swz(wc * 32 + j * 16 + fr, ks * 4 + fk));
  };
  auto mma = [&](int mh, int nh) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[mh][i][nh][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[ks][i], fb[nh][ks][j],
                                                                      acc[mh][i][nh][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };

  // One phase: [LDS reads of this phase's fragments] [DMA issue] [counted vmcnt] barrier
  // [MFMA burst] barrier.  The reads' lgkmcnt wait is placed by hipcc before the first
  // MFMA (after the barrier), so the partner wave's burst hides the LDS latency.
#define PGEMM_PHASE(BUF, MH, NH, RA, RB, STAGE_STMT, VM)  \
  {                                                       \
    if (RB) read_b(BUF, NH);                              \
    if (RA) read_a(BUF, MH);                              \
    STAGE_STMT;                                           \
    vmcnt<VM>();                                          \
    sbarrier();                                           \
    mma(MH, NH);                                          \
    sbarrier();                                           \
  }

  // Iteration j computes K-tiles 2j (even buffer E, phases 1-4) and 2j+1 (odd buffer O,
  // phases 5-8).  DMA issue per phase (one half-tile each):
  //   1: O.HB1(2j+1)  2: O.HA1(2j+1)  3: E.HA0(2j+2)  4: E.HB0(2j+2)
  //   5: E.HB1(2j+2)  6: E.HA1(2j+2)  7: O.HA0(2j+3)  8: O.HB0(2j+3)
  // WAR: each destination half was last read >= 2 phases before its issue (E.HA0 / HB0 in
  // phase 1, E.HB1 in 2, E.HA1 in 3; O likewise in 5, 5, 6, 7) -- 2 phases cover the
  // one-barrier stagger of the wave rows.  RAW: vmcnt(8) after each phase's issue retires
  // the half issued 4 phases before, and every half is first read >= 1 phase after the
  // wait that retires it (E.HA0 / HB0 issued in 3 / 4 -> retired by phase 8 -> read in
  // phase 1 of j+1; E.HB1 5 -> 1 -> 2; E.HA1 6 -> 2 -> 3; O.HA0 / HB0 7 / 8 -> 4 -> 5;
  // O.HB1 1 -> 5 -> 6; O.HA1 2 -> 6 -> 7).  The last iteration issues only phases 1-2 and
  // retires with the counts that keep the same guarantees (8, 8, 8, 4, 2, 0, 0, 0).
  // prologue: everything the steady state assumes was issued in iteration -1
  stage(HA0, 0);
  stage(HB0, 0);
  stage(HB1, 0);
  stage(HA1, 0);
  stage(HA0, 1);
  stage(HB0, 1);
  vmcnt<8>();
  sbarrier();
  if (wr == 1) sbarrier();   // stagger: wave row 1 runs one barrier behind

  for (int j = 0; j < nit - 1; ++j) {
    const int kt = 2 * j;
    PGEMM_PHASE(0, 0, 0, 1, 1, stage(HB1, kt + 1), 8)
    PGEMM_PHASE(0, 0, 1, 0, 1, stage(HA1, kt + 1), 8)
    PGEMM_PHASE(0, 1, 1, 1, 0, stage(HA0, kt + 2), 8)
    PGEMM_PHASE(0, 1, 0, 0, 0, stage(HB0, kt + 2), 8)
    PGEMM_PHASE(1, 0, 0, 1, 1, stage(HB1, kt + 2), 8)
    PGEMM_PHASE(1, 0, 1, 0, 1, stage(HA1, kt + 2), 8)
    PGEMM_PHASE(1, 1, 1, 1, 0, stage(HA0, kt + 3), 8)
    PGEMM_PHASE(1, 1, 0, 0, 0, stage(HB0, kt + 3), 8)
  }
  {
    const int kt = 2 * (nit - 1);
    PGEMM_PHASE(0, 0, 0, 1, 1, stage(HB1, kt + 1), 8)
    PGEMM_PHASE(0, 0, 1, 0, 1, stage(HA1, kt + 1), 8)
    PGEMM_PHASE(0, 1, 1, 1, 0, (void)0, 8)
    PGEMM_PHASE(0, 1, 0, 0, 0, (void)0, 4)
    PGEMM_PHASE(1, 0, 0, 1, 1, (void)0, 2)
    PGEMM_PHASE(1, 0, 1, 0, 1, (void)0, 0)
    PGEMM_PHASE(1, 1, 1, 1, 0, (void)0, 0)
    PGEMM_PHASE(1, 1, 0, 0, 0, (void)0, 0)
  }
#undef PGEMM_PHASE
  if (wr == 0) sbarrier();   // re-align the wave rows
  vmcnt<0>();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  sbarrier();                // every wave done with the buffers: reuse LDS as scratch
}

// the tile's epilogue through the drained LDS: bf16 tile, fused SwiGLU, or an fp32 slab
template <int EPI>
__device__ __forceinline__ void pgemm_store(char* smem, f32x4 (&acc)[2][4][2][2], uint16_t* __restrict__ C,
                                            float* __restrict__ P, int M, int N, int m0, int n0, int slice) {
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3;
  const int fr = lane & 15, fk = lane >> 4;

  // ---- epilogue: the wave's 128 x 64 tile -> bf16 scratch [128][SCR_PITCH] -> row stores
  uint16_t* scr = reinterpret_cast<uint16_t*>(smem) + wave * 128 * SCR_PITCH;
  if constexpr (EPI == EPI_BF16) {
#pragma unroll
    for (int mh = 0; mh < 2; ++mh)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int nh = 0; nh < 2; ++nh)
#pragma unroll
          for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r)
              scr[(mh * 64 + i * 16 + fk * 4 + r) * SCR_PITCH + nh * 32 + j * 16 + fr] =
                  f2bf(acc[mh][i][nh][j][r]);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    // 8 lanes per 128-B row segment, 8 rows per sweep
#pragma unroll 4
    for (int it = 0; it < 16; ++it) {
      const int r = it * 8 + (lane >> 3), c = (lane & 7) * 8;
      const int row = m0 + wr * 128 + r;
      const uint4 v = *reinterpret_cast<const uint4*>(scr + r * SCR_PITCH + c);
      if (row < M) *reinterpret_cast<uint4*>(C + (size_t)row * N + n0 + wc * 64 + c) = v;
    }
  } else if constexpr (EPI == EPI_PARTIAL) {
    // fp32 split-K slab P[slice][row][col] (combined by the consumer kernel): each wave's
    // 64-row halves through its own LDS scratch [64][68] so stores are whole 256-B row runs
    float* fs = reinterpret_cast<float*>(smem) + wave * 64 * 68;
    float* Ps = P + (size_t)slice * M * N;
#pragma unroll
    for (int mh = 0; mh < 2; ++mh) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int nh = 0; nh < 2; ++nh)
#pragma unroll
          for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r)
              fs[(i * 16 + fk * 4 + r) * 68 + nh * 32 + j * 16 + fr] = acc[mh][i][nh][j][r];
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll 4
      for (int it = 0; it < 16; ++it) {
        const int r = it * 4 + (lane >> 4), c = (lane & 15) * 4;
        const int row = m0 + wr * 128 + mh * 64 + r;
        const float4 v = *reinterpret_cast<const float4*>(fs + r * 68 + c);
        if (row < M) *reinterpret_cast<float4*>(Ps + (size_t)row * N + n0 + wc * 64 + c) = v;
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
  } else {
    // 16 consecutive GEMM columns = one (gate 8 | up 8) group: lane fr < 8 holds gate[fr],
    // lane fr + 8 the matching up (DPP row rotate by 8 pairs them); 32 outputs per wave row
#pragma unroll
    for (int mh = 0; mh < 2; ++mh)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int nh = 0; nh < 2; ++nh)
#pragma unroll
          for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const float v = acc[mh][i][nh][j][r];
              const float u = row_ror<8>(v);
              if (fr < 8) {
                const float gv = bf2f(f2bf(v)), uv = bf2f(f2bf(u));   // as the bf16 GEMM output
                scr[(mh * 64 + i * 16 + fk * 4 + r) * SCR_PITCH + nh * 16 + j * 8 + fr] = f2bf(silu_f(gv) * uv);
              }
            }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    // 32 outputs (64 B) per row: 4 lanes per row, 16 rows per sweep
#pragma unroll 4
    for (int it = 0; it < 8; ++it) {
      const int r = it * 16 + (lane >> 2), c = (lane & 3) * 8;
      const int row = m0 + wr * 128 + r;
      const uint4 v = *reinterpret_cast<const uint4*>(scr + r * SCR_PITCH + c);
      if (row < M) *reinterpret_cast<uint4*>(C + (size_t)row * (N >> 1) + ((n0 + wc * 64) >> 1) + c) = v;
    }
  }
}

template <int EPI>
__global__ __launch_bounds__(512, 2) void pgemm_kernel(const uint16_t* __restrict__ A,
                                                      const uint16_t* __restrict__ W,
                                                      uint16_t* __restrict__ C, float* __restrict__ P,
                                                      int M, int N, int K, int ntm, int ntn, int S, int Ks) {
  __shared__ __attribute__((aligned(16))) char smem[LDS_B];
  const int nwg = ntm * ntn;
  // split-K (decode-sized M): workgroup -> (tile, K slice).  With S | 8 and whole rounds of
  // 8, the workgroups of one XCD all take the same slice, so that XCD's L2 holds just that
  // slice of A -- re-read by every tile (cf. mgemm.hip)
  int tile_id, slice = 0;
  if (S == 1) {
    tile_id = xcd_remap(blockIdx.x, nwg);
  } else if (8 % S == 0 && (nwg * S) % 8 == 0) {
    const int xcd = blockIdx.x & 7, j = blockIdx.x >> 3;
    slice = xcd % S;
    tile_id = j * (8 / S) + xcd / S;
  } else {
    tile_id = blockIdx.x % nwg;
    slice = blockIdx.x / nwg;
  }
  const int kbeg = slice * Ks;
  const int wg = tile_id;
  // groups of GM m-tiles x all n-tiles: consecutive ids (one XCD's concurrent workgroups)
  // form a GM x (32 / GM) block of output tiles
  constexpr int GM = 4;
  const int per_group = GM * ntn;
  const int grp = wg / per_group, first_m = grp * GM;
  const int gm = min(ntm - first_m, GM);
  const int rem = wg - grp * per_group;
  const int bm = first_m + rem % gm, bn = rem / gm;
  const int m0 = bm * BM, n0 = bn * BN;

  f32x4 acc[2][4][2][2];
  pgemm_mainloop(smem, A, W, M, K, m0, n0, kbeg, Ks / (2 * BK), acc);
  pgemm_store<EPI>(smem, acc, C, P, M, N, m0, n0, slice);
}
}  // namespace

bool docqa_pgemm_ok(int M, int N, int K) {
  if (M <= 0 || N % BN != 0 || K % (2 * BK) != 0) return false;
  // 32-bit per-lane byte offsets: (rows - 1) * K * 2 + 128 must fit
  const uint64_t rows = (uint64_t)(M > N ? M : N);
  return rows * (uint64_t)K * 2ull < (1ull << 32);
}

// epi 0: C [M, N] bf16; epi 1: C [M, N / 2] = silu(gate) * up (8-interleaved gate|up W);
// epi 2: P [S, M, N] fp32 split-K slabs (S >= 1 slices of K / S)
int docqa_pgemm(const void* A, const void* W, void* C, float* P, int M, int N, int K, int S, int epi,
                hipStream_t s) {
  if (M == 0) return 0;
  if (!docqa_pgemm_ok(M, N, K) || S < 1 || K % (S * 2 * BK) != 0) return -1;
  if (epi == EPI_PARTIAL ? P == nullptr : (C == nullptr || S != 1)) return -1;
  if (epi != EPI_BF16 && epi != EPI_GLU && epi != EPI_PARTIAL) return -1;
  if (!docqa_aligned16(A) || !docqa_aligned16(W) || !docqa_aligned16(epi == EPI_PARTIAL ? (void*)P : C)) return -1;
  const int ntm = (M + BM - 1) / BM, ntn = N / BN;
  const uint16_t *a = (const uint16_t*)A, *w = (const uint16_t*)W;
  uint16_t* c = (uint16_t*)C;
  const int grid = ntm * ntn * S, Ks = K / S;
  if (epi == EPI_BF16)
    pgemm_kernel<EPI_BF16><<<grid, 512, 0, s>>>(a, w, c, P, M, N, K, ntm, ntn, S, Ks);
  else if (epi == EPI_GLU)
    pgemm_kernel<EPI_GLU><<<grid, 512, 0, s>>>(a, w, c, P, M, N, K, ntm, ntn, S, Ks);
  else
    pgemm_kernel<EPI_PARTIAL><<<grid, 512, 0, s>>>(a, w, c, P, M, N, K, ntm, ntn, S, Ks);
  DOCQA_CHECK_LAUNCH();
  return 0;
}
