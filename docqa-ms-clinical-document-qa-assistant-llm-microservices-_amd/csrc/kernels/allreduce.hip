// allreduce.hip -- tensor-parallel all-reduce over IPC-mapped peer memory for the Llama
// generator's row-parallel projections, with the residual add +
// RMSNorm that follows every such all-reduce fused in.
//
// On one MI355X node the 8 GPUs are fully connected by xGMI (7 point-to-point links per
// GPU).  A ring all-reduce uses one link per direction per step; here every rank reads its
// peers' staging buffers directly, so all 7 links carry data at once:
//
//   ONESHOT (small, latency-bound messages -- decode at small batch):
//     1. each workgroup writes its rows of the local partial (bf16, or the fp32 split-K
//        slabs of the projection summed in registers) into this rank's staging area;
//     2. it publishes the call's epoch into slot [0][wg][rank] of every peer's flag array
//        and waits until its own slots [0][wg][p] reach the epoch (bounded spin);
//     3. it sums its rows over all N staging areas (fp32, the same order on every rank, so
//        every rank gets bit-identical results) -> epilogue.
//   TWOSHOT (larger messages -- prefill, decode at batch >= ~64):
//     1. as above;
//     2'. reduce-scatter: each rank sums only its column chunk [r H/N, (r+1) H/N) of the
//        workgroup's rows over all peers and writes it (bf16) to its result area, publishes
//        slot [1][wg][rank] and waits for slots [1][wg][p];
//     3'. all-gather: it reads every column chunk of its rows from the chunk's owner ->
//        epilogue.  Each rank moves 2 (N-1)/N of the message over xGMI instead of N-1.
//   Epilogue: plain (out = sum) or fused (residual <- bf16(residual + sum) in place,
//   out = rmsnorm(residual) * w: exactly ops.add_rmsnorm), one wave per row.
//
// Synchronisation: one epoch per CALL (a device-side counter read by every workgroup at
// start and advanced by the last workgroup to finish, so a HIP-graph replay advances it),
// staging halves double-buffered by epoch parity, flags compared with >= (a peer may
// already have published the next call's epoch).  A rank reuses a staging half two calls
// later only after every peer has published in the call in between, i.e. after each peer's
// previous kernel -- all its reads of that half -- has completed.  Staging and flags are
// allocated uncached (hipDeviceMallocUncached): remote reads and writes over xGMI bypass
// the caches; flag stores / loads are system-scope release / acquire atomics.  Spins give
// up after a wall-clock bound (``timeout``, host-set: sub-second in deployment) and record
// WHICH peer was late in the error word instead of hanging the GPU (every grid is <= 256
// workgroups of 256 threads: all resident); the longest wait of the call is kept in ctr[2]
// (us) for skew diagnostics.  The host reads the word once per engine step
// (parallel/custom_ar.py) and fails the step loudly.
// Root cause of round 3's spin-limit hits (4 ranks sharing ONE GPU in the tests): with
// HIP's default 4 hardware queues per process the 4 processes oversubscribe the GPU's queue
// slots; the scheduler left one rank's queue unmapped while the other ranks' kernels spun
// on its flags, so it "never arrived" (> 30 s, rank 0 at the first call:
// profiles/r4_ar_skew_default_hwq_tp4_fail.txt).  With one hardware queue per process
// (GPU_MAX_HW_QUEUES=1, set by the shared-GPU tests and bench.py --share-gpu) the longest
// peer wait is ~35 ms (profiles/r4_ar_skew_hwq1_tp.log).  One process per GPU -- the
// deployment -- never shares a queue slot pool with its peers.
#include "docqa_common.h"
#include <stdlib.h>
#include <cstring>

using namespace docqa;

namespace {
constexpr int kMaxRanks = 8;
constexpr int kMaxWG = 256;
constexpr size_t kFlagBytes = (size_t)2 * kMaxWG * kMaxRanks * sizeof(unsigned);

enum { ONESHOT = 0, TWOSHOT = 1, GATHER = 2 };
enum { SRC_BF16 = 0, SRC_F32 = 1 };

struct ArPeers {
  uint16_t* data[kMaxRanks];      // staging data of each rank (2 halves x [in | result])
  unsigned* flags[kMaxRanks];     // [2 phases][kMaxWG][kMaxRanks] epoch slots of each rank
};

struct ArArgs {
  const void* in;                 // bf16 [M, H] or fp32 slabs [S, M, H]
  int S;
  uint16_t* out;                  // [M, H]
  uint16_t* residual;             // fused: [M, H], updated in place
  const uint16_t* w;              // fused: [H]
  float eps;
  int M, H, rank, nranks;
  size_t half_elems;              // elements of one [in | result] area
  unsigned* ctr;                  // [0] epoch of the last call, [1] finished workgroups, [2] max wait (us)
  unsigned* err;                  // first error: 1 | late peer << 1 | phase << 4 | (epoch & 0xffffff) << 8
  unsigned long long timeout;     // wall-clock ticks a workgroup waits for a peer before giving up
  unsigned ticks_per_us;
};

__device__ __forceinline__ void publish(const ArPeers& peers, int phase, int wg, int rank, int nranks,
                                        unsigned epoch) {
  __threadfence_system();
  __syncthreads();
  if ((int)threadIdx.x < nranks)
    __hip_atomic_store(peers.flags[threadIdx.x] + ((size_t)phase * kMaxWG + wg) * kMaxRanks + rank, epoch,
                       __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ __forceinline__ void wait_peers(const ArPeers& peers, int phase, int wg, int rank, int nranks,
                                           unsigned epoch, const ArArgs& a) {
  if ((int)threadIdx.x < nranks) {
    const unsigned* slot = peers.flags[rank] + ((size_t)phase * kMaxWG + wg) * kMaxRanks + threadIdx.x;
    const unsigned long long t0 = wall_clock64();
    unsigned long long t = t0;
    while ((int)(__hip_atomic_load(slot, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) - epoch) < 0) {
      __builtin_amdgcn_s_sleep(2);
      t = wall_clock64();
      if (t - t0 > a.timeout) {
        // keep the FIRST failure's detail: which peer (threadIdx.x), which phase, which call
        atomicCAS(a.err, 0u, 1u | (threadIdx.x << 1) | ((unsigned)phase << 4) | ((epoch & 0xffffffu) << 8));
        break;
      }
    }
    if (t != t0) atomicMax(a.ctr + 2, (unsigned)((t - t0) / a.ticks_per_us));
  }
  __syncthreads();
  __atomic_thread_fence(__ATOMIC_ACQUIRE);   // system scope: no stale peer lines below
}

// residual <- bf16(residual + v) for 8 columns; returns the partial sum of squares
__device__ __forceinline__ float fused_add(const ArArgs& a, size_t off, float* v) {
  float r[8];
  unpack8(*reinterpret_cast<const uint4*>(a.residual + off), r);
  float ss = 0.f;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    v[e] = bf2f(f2bf(v[e] + r[e]));
    ss += v[e] * v[e];
  }
  *reinterpret_cast<uint4*>(a.residual + off) = pack8(v);
  return ss;
}

// out = bf16(residual * inv * w) for one row (residual re-read: this lane wrote it)
__device__ __forceinline__ void fused_norm_row(const ArArgs& a, int row, float inv, int lane) {
  for (int c = lane * 8; c < a.H; c += 512) {
    const size_t off = (size_t)row * a.H + c;
    float r[8], w[8];
    unpack8(*reinterpret_cast<const uint4*>(a.residual + off), r);
    unpack8(*reinterpret_cast<const uint4*>(a.w + c), w);
#pragma unroll
    for (int e = 0; e < 8; ++e) r[e] = r[e] * inv * w[e];
    *reinterpret_cast<uint4*>(a.out + off) = pack8(r);
  }
}

template <int MODE, int SRC, bool FUSED>
__global__ __launch_bounds__(256) void allreduce_kernel(ArArgs a, ArPeers peers) {
  const int wg = blockIdx.x, G = gridDim.x;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const unsigned epoch = a.ctr[0] + 1;
  const size_t half = (size_t)(epoch & 1) * 2 * a.half_elems;   // [in | result] of this call
  const int r0 = (int)((long)a.M * wg / G), r1 = (int)((long)a.M * (wg + 1) / G);
  const int H = a.H;
  uint16_t* mine = peers.data[a.rank] + half;

  // 1. local partial rows -> own staging "in" area (fp32 slabs summed here)
  for (int row = r0 + wave; row < r1; row += 4) {
    for (int c = lane * 8; c < H; c += 512) {
      const size_t off = (size_t)row * H + c;
      if constexpr (SRC == SRC_BF16) {
        *reinterpret_cast<uint4*>(mine + off) = *reinterpret_cast<const uint4*>((const uint16_t*)a.in + off);
      } else {
        const float* P = (const float*)a.in;
        const size_t slab = (size_t)a.M * H;
        float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        for (int s = 0; s < a.S; ++s) {
          const float4 x0 = *reinterpret_cast<const float4*>(P + s * slab + off);
          const float4 x1 = *reinterpret_cast<const float4*>(P + s * slab + off + 4);
          v[0] += x0.x; v[1] += x0.y; v[2] += x0.z; v[3] += x0.w;
          v[4] += x1.x; v[5] += x1.y; v[6] += x1.z; v[7] += x1.w;
        }
        *reinterpret_cast<uint4*>(mine + off) = pack8(v);
      }
    }
  }
  publish(peers, 0, wg, a.rank, a.nranks, epoch);
  wait_peers(peers, 0, wg, a.rank, a.nranks, epoch, a);

  if constexpr (MODE == GATHER) {
    // all-gather of raw 16-B words: out[p] <- rank p's rows (bit-exact copies)
    const size_t n = (size_t)a.M * H;
    for (int p = 0; p < a.nranks; ++p)
      for (int row = r0 + wave; row < r1; row += 4)
        for (int c = lane * 8; c < H; c += 512) {
          const size_t off = (size_t)row * H + c;
          *reinterpret_cast<uint4*>(a.out + p * n + off) = *reinterpret_cast<const uint4*>(peers.data[p] + half + off);
        }
  } else if constexpr (MODE == ONESHOT) {
    // 3. every rank sums its rows over all peers itself (same order everywhere)
    for (int row = r0 + wave; row < r1; row += 4) {
      float ss = 0.f;
      for (int c = lane * 8; c < H; c += 512) {
        const size_t off = (size_t)row * H + c;
        float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        for (int p = 0; p < a.nranks; ++p) {
          float x[8];
          unpack8(*reinterpret_cast<const uint4*>(peers.data[p] + half + off), x);
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] += x[e];
        }
        if constexpr (FUSED) {
          // round the cross-rank sum to bf16 first, as the two-shot path (its reduced chunk
          // is stored bf16), the RCCL fallback and TP = 1 do: bf16(bf16(sum) + residual)
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = bf2f(f2bf(v[e]));
          ss += fused_add(a, off, v);
        } else {
          *reinterpret_cast<uint4*>(a.out + off) = pack8(v);
        }
      }
      if constexpr (FUSED) {
        ss = wave_sum(ss);
        fused_norm_row(a, row, rsqrtf(ss / H + a.eps), lane);
      }
    }
  } else {
    // 2'. reduce-scatter: this rank's column chunk of the workgroup's rows
    const int CH = H / a.nranks, c0 = a.rank * CH;
    uint16_t* res = mine + a.half_elems;
    for (int row = r0 + wave; row < r1; row += 4) {
      for (int c = c0 + lane * 8; c < c0 + CH; c += 512) {
        const size_t off = (size_t)row * H + c;
        float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        for (int p = 0; p < a.nranks; ++p) {
          float x[8];
          unpack8(*reinterpret_cast<const uint4*>(peers.data[p] + half + off), x);
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] += x[e];
        }
        *reinterpret_cast<uint4*>(res + off) = pack8(v);
      }
    }
    publish(peers, 1, wg, a.rank, a.nranks, epoch);
    wait_peers(peers, 1, wg, a.rank, a.nranks, epoch, a);
    // 3'. all-gather of the reduced chunks -> epilogue
    for (int row = r0 + wave; row < r1; row += 4) {
      float ss = 0.f;
      for (int c = lane * 8; c < H; c += 512) {
        const size_t off = (size_t)row * H + c;
        const int owner = c / CH;
        float v[8];
        unpack8(*reinterpret_cast<const uint4*>(peers.data[owner] + half + a.half_elems + off), v);
        if constexpr (FUSED) ss += fused_add(a, off, v);
        else *reinterpret_cast<uint4*>(a.out + off) = pack8(v);
      }
      if constexpr (FUSED) {
        ss = wave_sum(ss);
        fused_norm_row(a, row, rsqrtf(ss / H + a.eps), lane);
      }
    }
  }
  // the last workgroup to finish advances the call epoch (read by the next call's grid)
  __syncthreads();
  if (tid == 0) {
    __threadfence();
    if (atomicAdd(a.ctr + 1, 1u) == (unsigned)G - 1) {
      a.ctr[1] = 0;
      a.ctr[0] = epoch;
      __threadfence();
    }
  }
}

template <int MODE, int SRC, bool FUSED>
int launch(const ArArgs& a, const ArPeers& p, int G, hipStream_t s) {
  allreduce_kernel<MODE, SRC, FUSED><<<G, 256, 0, s>>>(a, p);
  DOCQA_CHECK_LAUNCH();
  return 0;
}
}  // namespace

// staging + flag region of one rank: [flags][2 halves x (in max_elems | result max_elems)]
size_t docqa_ar_region_bytes(size_t max_elems) { return kFlagBytes + 4 * max_elems * sizeof(uint16_t); }

int docqa_ar_alloc(size_t bytes, void** ptr) {
  if (hipExtMallocWithFlags(ptr, bytes, hipDeviceMallocUncached) != hipSuccess) return -1;
  if (hipMemset(*ptr, 0, bytes) != hipSuccess) return -1;
  return hipDeviceSynchronize() == hipSuccess ? 0 : -1;
}

int docqa_ar_free(void* ptr) { return hipFree(ptr) == hipSuccess ? 0 : -1; }

int docqa_ar_ipc_handle(void* ptr, void* handle_out /* 64 B */) {
  hipIpcMemHandle_t h;
  if (hipIpcGetMemHandle(&h, ptr) != hipSuccess) return -1;
  memcpy(handle_out, &h, sizeof(h));
  return 0;
}

int docqa_ar_ipc_open(const void* handle, void** ptr) {
  hipIpcMemHandle_t h;
  memcpy(&h, handle, sizeof(h));
  return hipIpcOpenMemHandle(ptr, h, hipIpcMemLazyEnablePeerAccess) == hipSuccess ? 0 : -1;
}

int docqa_ar_ipc_close(void* ptr) { return hipIpcCloseMemHandle(ptr) == hipSuccess ? 0 : -1; }

// All-reduce (mode 0 / 1) or all-gather (mode 2: out [nranks, M, H], raw 16-bit words) of a
// [M, H] tensor over `nranks` IPC-mapped regions (regions[r]: rank r's region
// as mapped in this process).  in: bf16 [M, H] (S == 0) or fp32 split-K slabs [S, M, H];
// residual / w given: fused add + RMSNorm epilogue (residual updated in place, out = the
// normed rows), else out = the sum.  mode 0 one-shot, 1 two-shot, 2 gather.  ctr: int32 [2]
// zeroed once (+ [2] the longest peer wait in us, [3] spare), err: int32 [1]; timeout_us: how
// long a workgroup waits for a peer before it records the error and gives up.
int docqa_ar_run(const void* in, int S, void* out, void* residual, const void* w, float eps, int M, int H,
                 int rank, int nranks, void* const* regions, size_t max_elems, int mode, unsigned* ctr,
                 unsigned* err, long long timeout_us, hipStream_t s) {
  if (M == 0) return 0;
  if (nranks < 1 || nranks > kMaxRanks || rank < 0 || rank >= nranks || H % 8 != 0 || M < 0) return -1;
  if ((size_t)M * H > max_elems) return -1;
  if (mode == TWOSHOT && (H % (8 * nranks) != 0)) return -1;
  if ((residual == nullptr) != (w == nullptr)) return -1;
  if (mode == GATHER && (S != 0 || residual != nullptr)) return -1;
  if (!docqa_aligned16(in) || !docqa_aligned16(out) || (residual && !docqa_aligned16(residual))) return -1;
  ArPeers peers{};
  for (int r = 0; r < nranks; ++r) {
    peers.flags[r] = (unsigned*)regions[r];
    peers.data[r] = (uint16_t*)((char*)regions[r] + kFlagBytes);
  }
  static int khz = 0;   // the constant wall clock behind wall_clock64() (100 MHz on MI355X)
  if (khz == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) !=
                                                 hipSuccess || khz <= 0)
      khz = 100000;
  }
  if (timeout_us <= 0) timeout_us = 500000;
  const unsigned tpu = (unsigned)(khz / 1000 > 0 ? khz / 1000 : 1);
  ArArgs a{in, S, (uint16_t*)out, (uint16_t*)residual, (const uint16_t*)w, eps, M, H, rank, nranks,
           max_elems, ctr, err, (unsigned long long)timeout_us * tpu, tpu};
  // workgroups: one per few rows (4 waves, one row each at a time), <= kMaxWG, all resident;
  // the same count on every rank (a function of M only)
  // DOCQA_AR_MAX_WG (ranks sharing ONE GPU: tests, --share-gpu): fewer workgroups, so the
  // waiting ranks' spinning workgroups never sit on every CU -- a late rank's next kernel
  // (a 512-register attention wave needs a whole SIMD) would otherwise find no CU to run on
  // until the waiters time out.  Read once; every rank sets the same value.
  static const int max_wg = [] {
    const char* e = getenv("DOCQA_AR_MAX_WG");
    const int v = e ? atoi(e) : 0;
    return v > 0 && v < kMaxWG ? v : kMaxWG;
  }();
  int G = (M + 3) / 4;
  if (G > max_wg) G = max_wg;
  if (G < 1) G = 1;
  const bool fused = residual != nullptr;
  const int src = S > 0 ? SRC_F32 : SRC_BF16;
#define AR_CASE(MD, SR, FU) \
  if (mode == MD && src == SR && fused == FU) return launch<MD, SR, FU>(a, peers, G, s);
  AR_CASE(ONESHOT, SRC_BF16, false)
  AR_CASE(ONESHOT, SRC_BF16, true)
  AR_CASE(ONESHOT, SRC_F32, false)
  AR_CASE(ONESHOT, SRC_F32, true)
  AR_CASE(TWOSHOT, SRC_BF16, false)
  AR_CASE(TWOSHOT, SRC_BF16, true)
  AR_CASE(TWOSHOT, SRC_F32, false)
  AR_CASE(TWOSHOT, SRC_F32, true)
  AR_CASE(GATHER, SRC_BF16, false)
#undef AR_CASE
  return -1;
}
