// gemm.hip -- bf16 MFMA GEMM with fused epilogues for the encoder stacks
//   C[M, N] = act(A[M, K] . W[N, K]^T + bias[N]) (+ residual[M, N])
// (nn.Linear layout: weights stored [out, in]).  Epilogues: none, bias, bias+GELU(erf),
// bias+residual, and the Llama SwiGLU over 8-interleaved gate|up rows (prefill shapes whose
// 256 x 256 tiles cannot fill the chip: the 70B TP-8 gate|up shard at <= 1k tokens).  Used by the BERT encoders (MiniLM / bge / clinical-BERT): the FFN-up
// GEMM with its bias+GELU, the QKV and output projections with their biases, so no
// separate element-wise pass re-reads the [tokens, 4H] activations from HBM.
//
// Structure (cdna_hip_programming.md §5 "canonical CDNA GEMM", T1, T2, T14):
//   * 128x128 block tile, BK = 64, 4 waves in 2x2, each wave a 64x64 sub-tile of
//     4x4 v_mfma_f32_16x16x32_bf16 accumulators (64 fp32 registers);
//   * A and W tiles are both row-major [row][k] in LDS (W^T's k-contiguous rows are
//     exactly the B-operand fragments), double-buffered, XOR-swizzled
//     (16-B chunk ^ ((row >> 1) & 7)) so the 16-row ds_read_b128 fragment reads are
//     bank-conflict-free;
//   * register-staged global->LDS copy of tile t+1 issued before the MFMAs of tile t and
//     written after them (async-STAGE split);
//   * XCD-aware bijective block remap so neighbouring tiles share an XCD's L2;
//   * epilogue through LDS: accumulators -> fp32 tile -> coalesced 16-B rows with the
//     bias / GELU / residual applied once per output element.
// Shapes: N % 128 == 0, K % 64 == 0, any M.
#include "docqa_common.h"

using namespace docqa;

namespace {
constexpr int BM = 128, BN = 128, BK = 64;
typedef short i16x8 __attribute__((ext_vector_type(8)));

enum Epi { EPI_NONE = 0, EPI_BIAS = 1, EPI_BIAS_GELU = 2, EPI_BIAS_RES = 3, EPI_GLU = 4 };

__device__ __forceinline__ int sw_off(int row, int ch) {  // element offset in a [128][64] tile
  return row * BK + ((ch ^ ((row >> 1) & 7)) << 3);
}

__device__ __forceinline__ float gelu_erf(float x) {
  return 0.5f * x * (1.f + erff(x * 0.70710678118654752f));
}

template <int EPI>
__global__ __launch_bounds__(256) void gemm_kernel(const uint16_t* __restrict__ A,
                                                   const uint16_t* __restrict__ W,
                                                   const uint16_t* __restrict__ bias,
                                                   const uint16_t* __restrict__ res,
                                                   uint16_t* __restrict__ C, int M, int N, int K) {
  // 64 KB of double-buffered A/W tiles, reused by the epilogue's 4 x 64 x 65 fp32 staging
  __shared__ __attribute__((aligned(16))) uint16_t smem[4 * 64 * 65 * 2];
  const int nbn = N / BN, nbm = (M + BM - 1) / BM;
  const int nwg = nbn * nbm;
  const int wg = xcd_remap(blockIdx.x, nwg);
  const int bm = wg / nbn, bn = wg % nbn;
  const int row0 = bm * BM, col0 = bn * BN;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 1, wc = wave & 1;       // 2x2 waves
  const int fr = lane & 15, fk = lane >> 4;      // fragment row / k-group

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // staging by LDS-DMA (global_load_lds, 16 B per lane): each tensor tile is 128 rows x
  // 8 chunks = 16 wave-instructions of 1 KiB, 4 per wave per tensor.  The LDS image is
  // lane-linear, so the XOR swizzle is applied to the per-lane SOURCE address (rule 21):
  // physical chunk p of the image receives logical chunk (p&7) ^ ((row>>1)&7) of its row.
  typedef __attribute__((address_space(3))) void lds_void;
  auto stage = [&](int kt, int buf) {
    uint16_t* sa = smem + buf * (2 * BM * BK);
    uint16_t* sw = sa + BM * BK;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int p0 = (i * 4 + wave) * 64;          // first physical chunk of this issue
      const int p = p0 + lane;
      const int r = p >> 3;
      const int ch = (p & 7) ^ ((r >> 1) & 7);
      const int gr = min(row0 + r, M - 1);         // tail rows: valid memory, never stored
      __builtin_amdgcn_global_load_lds(A + (size_t)gr * K + kt * BK + ch * 8,
                                       (lds_void*)(sa + p0 * 8), 16, 0, 0);
      __builtin_amdgcn_global_load_lds(W + (size_t)(col0 + r) * K + kt * BK + ch * 8,
                                       (lds_void*)(sw + p0 * 8), 16, 0, 0);
    }
  };

  const int nk = K / BK;
  stage(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < nk) stage(kt + 1, buf ^ 1);   // DMA of tile t+1 overlaps MFMAs of tile t
    const uint16_t* sa = smem + buf * (2 * BM * BK);
    const uint16_t* sw = sa + BM * BK;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {          // two 32-deep MFMA k-steps per BK
      bf16x8 af[4], bf[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = wr * 64 + i * 16 + fr;
        af[i] = *reinterpret_cast<const bf16x8*>(sa + sw_off(r, ks * 4 + fk));
        const int c = wc * 64 + i * 16 + fr;
        bf[i] = *reinterpret_cast<const bf16x8*>(sw + sw_off(c, ks * 4 + fk));
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bf[j], acc[i][j], 0, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  // ---- epilogue: stage the wave's 64x64 fp32 tile in LDS (reuse), then 16-B row stores
  float* st = reinterpret_cast<float*>(smem) + wave * (64 * 65);   // padded rows, 16.6 KB/wave
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        st[(i * 16 + fk * 4 + r) * 65 + j * 16 + fr] = acc[i][j][r];
  __syncthreads();
  if constexpr (EPI == EPI_GLU) {
    // Llama gate|up in the 8-interleaved row layout (decode GEMMs' layout): output columns
    // [16 p, 16 p + 8) are gate, [16 p + 8, 16 p + 16) up; C is [M, N / 2] =
    // silu(gate) * up, each input rounded to bf16 first (as the unfused bf16 GEMM output
    // would be).  Lane -> (row, pair p of the wave's 4)
    for (int it = 0; it < 4; ++it) {
      const int rloc = it * 16 + (lane >> 2), p = lane & 3;
      const int gr = row0 + wr * 64 + rloc;
      if (gr < M) {
        float o[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float g = bf2f(f2bf(st[rloc * 65 + p * 16 + e]));
          const float u = bf2f(f2bf(st[rloc * 65 + p * 16 + 8 + e]));
          o[e] = g / (1.f + __expf(-g)) * u;
        }
        *reinterpret_cast<uint4*>(C + (size_t)gr * (N >> 1) + ((col0 + wc * 64) >> 1) + p * 8) = pack8(o);
      }
    }
    return;
  }
  // each wave writes its own 64 rows x 64 cols: lane -> (row group, 8-col chunk)
  for (int it = 0; it < 8; ++it) {
    const int rloc = it * 8 + (lane >> 3);
    const int cch = lane & 7;
    const int gr = row0 + wr * 64 + rloc;
    const int gc = col0 + wc * 64 + cch * 8;
    if (gr < M) {
      float v[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = st[rloc * 65 + cch * 8 + e];
      if constexpr (EPI != EPI_NONE) {
        float b[8];
        unpack8(*reinterpret_cast<const uint4*>(bias + gc), b);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] += b[e];
      }
      if constexpr (EPI == EPI_BIAS_GELU) {
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = gelu_erf(v[e]);
      }
      if constexpr (EPI == EPI_BIAS_RES) {
        float rr[8];
        unpack8(*reinterpret_cast<const uint4*>(res + (size_t)gr * N + gc), rr);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] += rr[e];
      }
      *reinterpret_cast<uint4*>(C + (size_t)gr * N + gc) = pack8(v);
    }
  }
}
}  // namespace

int docqa_gemm(const void* A, const void* W, const void* bias, const void* res, void* C, int M,
               int N, int K, int epi, hipStream_t s) {
  if (M == 0) return 0;
  if (N % BN != 0 || K % BK != 0) return -1;
  if (epi != EPI_NONE && epi != EPI_GLU && bias == nullptr) return -1;
  if (epi == EPI_BIAS_RES && res == nullptr) return -1;
  const int nwg = (N / BN) * ((M + BM - 1) / BM);
  const uint16_t *a = (const uint16_t*)A, *w = (const uint16_t*)W, *b = (const uint16_t*)bias,
                 *r = (const uint16_t*)res;
  uint16_t* c = (uint16_t*)C;
  switch (epi) {
    case EPI_NONE: gemm_kernel<EPI_NONE><<<nwg, 256, 0, s>>>(a, w, b, r, c, M, N, K); break;
    case EPI_BIAS: gemm_kernel<EPI_BIAS><<<nwg, 256, 0, s>>>(a, w, b, r, c, M, N, K); break;
    case EPI_BIAS_GELU: gemm_kernel<EPI_BIAS_GELU><<<nwg, 256, 0, s>>>(a, w, b, r, c, M, N, K); break;
    case EPI_BIAS_RES: gemm_kernel<EPI_BIAS_RES><<<nwg, 256, 0, s>>>(a, w, b, r, c, M, N, K); break;
    case EPI_GLU: gemm_kernel<EPI_GLU><<<nwg, 256, 0, s>>>(a, w, b, r, c, M, N, K); break;
    default: return -1;
  }
  DOCQA_CHECK_LAUNCH();
  return 0;
}
