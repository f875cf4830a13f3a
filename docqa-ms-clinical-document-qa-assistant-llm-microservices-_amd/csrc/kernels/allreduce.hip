// allreduce.hip -- one-shot all-reduce over IPC-mapped peer memory for the generator's
// tensor-parallel decode all-reduces.
//
// TP decode all-reduces are small ([B, hidden] bf16: 1 MB at B = 64, hidden = 8192) and
// latency-bound.  On one MI355X node the 8 GPUs are fully connected by xGMI (7 links per
// GPU), so instead of a ring (one link per step, 2(N-1) hops) every rank reads all peers'
// buffers at once over all links and reduces locally:
//
//   1. each workgroup copies its contiguous slice of the local input into this rank's
//      staging buffer (half `epoch & 1` of a double buffer);
//   2. it publishes `epoch` into slot [wg][rank] of every peer's flag array and waits
//      until its own slots [wg][p] hold `epoch` for every peer p (bounded spin);
//   3. it sums slice `wg` of all N staging buffers (fp32 accumulate) into the output.
//
// Double buffering needs only this one barrier per call: a rank can reuse a staging half
// two calls later only after its peers have signalled in the call in between, i.e. after
// they finished reading it.  Epochs live in device memory (one counter per workgroup),
// so a HIP-graph replay of the kernel advances them correctly.
//
// Memory: staging + flags are allocated uncached (hipDeviceMallocUncached), so remote
// reads/writes over xGMI bypass every cache and need no invalidation; flag stores/loads
// are system-scope atomics.  Spins give up after a bound and raise an error word instead
// of hanging the GPU (the grid is <= one workgroup per CU, all resident).
#include "docqa_common.h"
#include <cstring>

using namespace docqa;

namespace {
constexpr int kMaxRanks = 8;
constexpr int kMaxWG = 128;
constexpr unsigned kSpinLimit = 1u << 24;

struct ArPeers {
  uint16_t* data[kMaxRanks];      // staging buffers (2 halves of `half_elems`)
  unsigned* flags[kMaxRanks];     // [kMaxWG][kMaxRanks] epoch slots
};

__global__ __launch_bounds__(256) void allreduce_oneshot_kernel(
    const uint16_t* __restrict__ in, uint16_t* __restrict__ out, int n, int per_wg, int rank,
    int nranks, size_t half_elems, ArPeers peers, unsigned* __restrict__ epochs,
    unsigned* __restrict__ err) {
  const int wg = blockIdx.x, tid = threadIdx.x;
  const unsigned epoch = epochs[wg] + 1;
  const size_t half = (size_t)(epoch & 1) * half_elems;
  const int lo = wg * per_wg;
  const int hi = min(n, lo + per_wg);

  // 1. local slice -> own staging (16-B vectors; n and per_wg are multiples of 8)
  uint16_t* mine = peers.data[rank] + half;
  for (int i = lo + tid * 8; i < hi; i += 256 * 8)
    *reinterpret_cast<uint4*>(mine + i) = *reinterpret_cast<const uint4*>(in + i);
  __threadfence_system();
  __syncthreads();

  // 2. barrier with the same workgroup on every peer
  if (tid < nranks) {
    __hip_atomic_store(peers.flags[tid] + wg * kMaxRanks + rank, epoch, __ATOMIC_RELEASE,
                       __HIP_MEMORY_SCOPE_SYSTEM);
  }
  if (tid < nranks) {
    const unsigned* slot = peers.flags[rank] + wg * kMaxRanks + tid;
    unsigned spins = 0;
    while (__hip_atomic_load(slot, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) != epoch) {
      __builtin_amdgcn_s_sleep(2);
      if (++spins > kSpinLimit) {
        atomicOr(err, 1u);
        break;
      }
    }
  }
  __syncthreads();
  __atomic_thread_fence(__ATOMIC_ACQUIRE);   // system scope: no stale peer lines below

  // 3. reduce slice `wg` over all ranks
  for (int i = lo + tid * 8; i < hi; i += 256 * 8) {
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int p = 0; p < nranks; ++p) {
      float v[8];
      unpack8(*reinterpret_cast<const uint4*>(peers.data[p] + half + i), v);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += v[j];
    }
    *reinterpret_cast<uint4*>(out + i) = pack8(acc);
  }
  if (tid == 0) epochs[wg] = epoch;
}
}  // namespace

// staging + flag region of one rank: [flags kMaxWG * kMaxRanks u32][2 halves of max_elems]
size_t docqa_ar_region_bytes(size_t max_elems) {
  return (size_t)kMaxWG * kMaxRanks * sizeof(unsigned) + 2 * max_elems * sizeof(uint16_t);
}

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

// regions[r]: rank r's region as mapped in this process (own allocation for r == rank)
int docqa_ar_oneshot(const void* in, void* out, int n, int rank, int nranks,
                     void* const* regions, size_t max_elems, unsigned* epochs, unsigned* err,
                     hipStream_t s) {
  if (n == 0) return 0;
  if (nranks < 1 || nranks > kMaxRanks || n % 8 != 0 || (size_t)n > max_elems) return -1;
  ArPeers peers{};
  const size_t flag_bytes = (size_t)kMaxWG * kMaxRanks * sizeof(unsigned);
  for (int r = 0; r < nranks; ++r) {
    peers.flags[r] = (unsigned*)regions[r];
    peers.data[r] = (uint16_t*)((char*)regions[r] + flag_bytes);
  }
  // workgroups: ~16 KB of payload each, at most kMaxWG (all resident); same on every rank
  int wgs = (n * 2 + 16383) / 16384;
  wgs = wgs < 1 ? 1 : (wgs > kMaxWG ? kMaxWG : wgs);
  int per_wg = (n + wgs - 1) / wgs;
  per_wg = (per_wg + 7) / 8 * 8;
  wgs = (n + per_wg - 1) / per_wg;
  allreduce_oneshot_kernel<<<wgs, 256, 0, s>>>((const uint16_t*)in, (uint16_t*)out, n, per_wg,
                                               rank, nranks, max_elems, peers, epochs, err);
  DOCQA_CHECK_LAUNCH();
  return 0;
}
