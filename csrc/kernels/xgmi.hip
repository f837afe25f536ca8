// Collectives over IPC-mapped peer buffers: every rank copies
// its input into its own exchange buffer, then one kernel per rank reads the peers' buffers straight
// over xGMI (the 8 MI355X of a node are a full mesh: 7 links per GPU are used at once, where a ring
// drives one).  RCCL stays the default (opt-in: PDA_ALLREDUCE=oneshot|twoshot|ring|ipc).
//   * all-reduce one-shot: each rank reads ALL of every peer's buffer and reduces locally —
//     (N-1)·S bytes over the links per rank, one barrier round: latency-optimal for small buckets.
//   * all-reduce two-shot: reduce-scatter then all-gather, both direct over the mesh.  Rank r reduces
//     chunk r (S/N) from all peers into its own exchange buffer, then every rank copies chunk c from
//     rank c — 2·(N-1)/N·S bytes per rank (the ring's volume, but on 7 links at once).
//   * all-reduce ring: the reference tutorial's algorithm (`02 DDP基本概念/02_ddp.ipynb` raw lines
//     33-47): N-1 reduce-scatter steps, each adding the LEFT neighbour's partial of one chunk into the
//     own buffer, then N-1 all-gather steps copying completed chunks from the left neighbour — the
//     same 2·(N-1)/N·S bytes, but one link per step.  Kept as the executable form of the concept and
//     as a correctness cross-check of the direct algorithms (tests compare all three).
//   * all-gather (FSDP parameter gather, X18): each rank reads every peer's shard (pull over 7 links).
//   * reduce-scatter (FSDP gradient shards): rank r reduces chunk r of every peer's full buffer.
//     Element→workgroup mapping is chunk-relative and identical on every rank (grid-stride inside each
//     chunk), so a per-workgroup flag barrier orders exactly the producer/consumer pairs.
//
// Synchronisation: per workgroup, flag barriers between steps (step 0: "my buffer holds this call's
// input"; the last: "I finished reading your buffer", so nobody refills its buffer while a peer still
// reads it).  A barrier of step s stores the value epoch·16 + s into flag slot s mod kXgmiPhases of
// every peer; slot values only ever grow (epochs grow per call), so a rank that runs ahead into a
// later step cannot be mistaken for one that has not arrived.  Flags and exchange buffers are
// uncached device memory (hipDeviceMallocUncached), so stores are visible to peers on other GPUs /
// other XCDs without relying on L2 write-back; the flag stores are release / the spin loads acquire
// at system scope.  Every spin is bounded by a wall-clock deadline: on timeout the kernel records an
// error and exits instead of hanging.  The error word is pinned host memory, so callers (DDP) poll it
// every step without synchronising the device; a communicator that reported a timeout is poisoned
// (its peers' epochs no longer line up).
#include "pda_common.h"
#include "pda_kernels.h"

#include <cstring>

namespace pda {
namespace {

constexpr int kXThreads = 256;

constexpr uint32_t kStepsPerEpoch = 16;  // >= 2*kXgmiMaxRanks - 1 barriers of the ring

__device__ __forceinline__ void flag_barrier(const XgmiArgs& a, int step) {
  __syncthreads();
  const int t = threadIdx.x;
  if (t < a.world) {
    const int slot = ((step % kXgmiPhases) * kXgmiMaxBlocks + blockIdx.x) * kXgmiMaxRanks;
    const uint32_t value = a.epoch * kStepsPerEpoch + (uint32_t)step;
    __threadfence_system();
    __hip_atomic_store(a.flags[t] + slot + a.rank, value, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    const uint32_t* mine = a.flags[a.rank] + slot + t;
    const long long t0 = wall_clock64();
    while (__hip_atomic_load(mine, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) < value) {
      if (wall_clock64() - t0 > a.timeout_ticks) {
        // err lives in host-coherent pinned memory: the host polls it without a device sync.  Keep
        // the FIRST step that timed out (later barriers of the same call time out as a consequence).
        if (__hip_atomic_load(a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) == 0)
          __hip_atomic_store(a.err, 1 + step, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
  }
  __syncthreads();
}

template <typename T>
__global__ void __launch_bounds__(kXThreads) xgmi_oneshot_kernel(XgmiArgs a) {
  flag_barrier(a, 0);
  const int64_t nv = a.n / 8;
  const int64_t stride = (int64_t)gridDim.x * kXThreads;
  for (int64_t v = (int64_t)blockIdx.x * kXThreads + threadIdx.x; v < nv; v += stride) {
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int r = 0; r < a.world; ++r) {
      float x[8];
      load8(reinterpret_cast<const T*>(a.data[r]) + v * 8, x);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += x[j];
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] *= a.scale;
    store8(reinterpret_cast<T*>(a.out) + v * 8, acc);
  }
  flag_barrier(a, 1);
}

// Two-shot: phase 0 barrier (buffers filled) -> reduce-scatter of own chunk (result written into the
// own exchange buffer and the output) -> phase 1 barrier (chunks reduced) -> all-gather of the peers'
// chunks -> phase 2 barrier (done reading peers; they may refill for the next epoch).
template <typename T>
__global__ void __launch_bounds__(kXThreads) xgmi_twoshot_kernel(XgmiArgs a) {
  flag_barrier(a, 0);
  const int64_t nv = a.n / 8;
  const int64_t cv = (nv + a.world - 1) / a.world;  // vectors per chunk
  const int64_t stride = (int64_t)gridDim.x * kXThreads;
  const int64_t lo = (int64_t)a.rank * cv, hi = lo + cv < nv ? lo + cv : nv;
  for (int64_t v = lo + (int64_t)blockIdx.x * kXThreads + threadIdx.x; v < hi; v += stride) {
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int i = 0; i < a.world; ++i) {
      const int r = (a.rank + i) % a.world;  // stagger the peer order so links are not hit in lockstep
      float x[8];
      load8(reinterpret_cast<const T*>(a.data[r]) + v * 8, x);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += x[j];
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] *= a.scale;
    store8(reinterpret_cast<T*>(a.data[a.rank]) + v * 8, acc);
    store8(reinterpret_cast<T*>(a.out) + v * 8, acc);
  }
  flag_barrier(a, 1);
  for (int i = 1; i < a.world; ++i) {
    const int c = (a.rank + i) % a.world;
    const int64_t clo = (int64_t)c * cv, chi = clo + cv < nv ? clo + cv : nv;
    const uint4* src = reinterpret_cast<const uint4*>(a.data[c]);
    uint4* dst = reinterpret_cast<uint4*>(a.out);
    constexpr int kPer = (int)(16 / sizeof(T)) == 8 ? 1 : 2;  // 16-B vectors per 8-element group
    for (int64_t v = clo + (int64_t)blockIdx.x * kXThreads + threadIdx.x; v < chi; v += stride) {
#pragma unroll
      for (int q = 0; q < kPer; ++q) dst[v * kPer + q] = src[v * kPer + q];
    }
  }
  flag_barrier(a, 2);
}

// Ring all-reduce.  Chunk c = [c·cv, (c+1)·cv) vectors of 8 elements.  Reduce-scatter step s
// (barrier s+1 before it): rank r adds the left neighbour's partial of chunk (r-s-1) mod N into its
// own buffer — that partial was completed by the neighbour in step s-1 (or is its input for s = 0);
// after step N-2 rank r owns the full sum of chunk (r+1) mod N, scaled there.  All-gather step s:
// rank r copies chunk (r-s) mod N from the left neighbour, which completed it one step earlier.  The
// output is the own exchange buffer, copied out after the last step.
template <typename T>
__global__ void __launch_bounds__(kXThreads) xgmi_ring_kernel(XgmiArgs a) {
  const int N = a.world, r = a.rank, left = (a.rank + N - 1) % N;
  const int64_t nv = a.n / 8;
  const int64_t cv = (nv + N - 1) / N;
  const int64_t stride = (int64_t)gridDim.x * kXThreads;
  T* own = reinterpret_cast<T*>(a.data[r]);
  const T* lft = reinterpret_cast<const T*>(a.data[left]);
  int step = 0;
  flag_barrier(a, step++);
  for (int s = 0; s < N - 1; ++s) {
    const int c = ((r - s - 1) % N + N) % N;
    const int64_t lo = (int64_t)c * cv, hi = lo + cv < nv ? lo + cv : nv;
    const float sc = s == N - 2 ? a.scale : 1.f;
    for (int64_t v = lo + (int64_t)blockIdx.x * kXThreads + threadIdx.x; v < hi; v += stride) {
      float x[8], y[8];
      load8(lft + v * 8, x);
      load8(own + v * 8, y);
#pragma unroll
      for (int j = 0; j < 8; ++j) y[j] = (x[j] + y[j]) * sc;
      store8(own + v * 8, y);
    }
    flag_barrier(a, step++);
  }
  if (N == 1) {  // (one chunk: this mapping is the chunk-relative one)
    for (int64_t v = (int64_t)blockIdx.x * kXThreads + threadIdx.x; v < nv; v += stride) {
      float y[8];
      load8(own + v * 8, y);
#pragma unroll
      for (int j = 0; j < 8; ++j) y[j] *= a.scale;
      store8(own + v * 8, y);
    }
  }
  constexpr int kPer = (int)(16 / sizeof(T)) == 8 ? 1 : 2;  // 16-B vectors per 8-element group
  for (int s = 0; s < N - 1; ++s) {
    const int c = ((r - s) % N + N) % N;
    const int64_t lo = (int64_t)c * cv, hi = lo + cv < nv ? lo + cv : nv;
    const uint4* src = reinterpret_cast<const uint4*>(lft);
    uint4* dst = reinterpret_cast<uint4*>(own);
    for (int64_t v = lo + (int64_t)blockIdx.x * kXThreads + threadIdx.x; v < hi; v += stride) {
#pragma unroll
      for (int q = 0; q < kPer; ++q) dst[v * kPer + q] = src[v * kPer + q];
    }
    flag_barrier(a, step++);
  }
  // copy out with the chunk-relative mapping of the steps above: every element a workgroup copies it
  // wrote (or read from its neighbour) itself — its barriers order nothing written by OTHER
  // workgroups of this kernel
  const uint4* src = reinterpret_cast<const uint4*>(own);
  uint4* dst = reinterpret_cast<uint4*>(a.out);
  for (int c = 0; c < N; ++c) {
    const int64_t lo = (int64_t)c * cv, hi = lo + cv < nv ? lo + cv : nv;
    for (int64_t v = lo + (int64_t)blockIdx.x * kXThreads + threadIdx.x; v < hi; v += stride) {
#pragma unroll
      for (int q = 0; q < kPer; ++q) dst[v * kPer + q] = src[v * kPer + q];
    }
  }
}

// All-gather: a.n = elements per shard; every rank's exchange buffer holds its shard; out[c·n ...]
// = shard of rank c, pulled from rank c over its link (own shard from the own buffer).
template <typename T>
__global__ void __launch_bounds__(kXThreads) xgmi_allgather_kernel(XgmiArgs a) {
  flag_barrier(a, 0);
  constexpr int kPer = (int)(16 / sizeof(T)) == 8 ? 1 : 2;
  const int64_t nv = a.n / 8;
  const int64_t stride = (int64_t)gridDim.x * kXThreads;
  uint4* dst = reinterpret_cast<uint4*>(a.out);
  for (int i = 0; i < a.world; ++i) {
    const int c = (a.rank + i) % a.world;  // staggered: at any moment the ranks pull from different peers
    const uint4* src = reinterpret_cast<const uint4*>(a.data[c]);
    const int64_t off = (int64_t)c * nv * kPer;
    for (int64_t v = (int64_t)blockIdx.x * kXThreads + threadIdx.x; v < nv; v += stride) {
#pragma unroll
      for (int q = 0; q < kPer; ++q) dst[off + v * kPer + q] = src[v * kPer + q];
    }
  }
  flag_barrier(a, 1);
}

// Reduce-scatter: a.n = elements of the FULL input (world shards); every rank's exchange buffer holds
// its full input; rank r writes scale · sum_p buf_p[chunk r] to out (one shard).
template <typename T>
__global__ void __launch_bounds__(kXThreads) xgmi_reduce_scatter_kernel(XgmiArgs a) {
  flag_barrier(a, 0);
  const int64_t sv = a.n / 8 / a.world;  // vectors per shard
  const int64_t lo = (int64_t)a.rank * sv;
  const int64_t stride = (int64_t)gridDim.x * kXThreads;
  for (int64_t v = (int64_t)blockIdx.x * kXThreads + threadIdx.x; v < sv; v += stride) {
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int i = 0; i < a.world; ++i) {
      const int p = (a.rank + i) % a.world;
      float x[8];
      load8(reinterpret_cast<const T*>(a.data[p]) + (lo + v) * 8, x);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += x[j];
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] *= a.scale;
    store8(reinterpret_cast<T*>(a.out) + v * 8, acc);
  }
  flag_barrier(a, 1);
}

}  // namespace

hipError_t xgmi_alloc(void** p, size_t bytes) {
  PDA_CHECK_HIP(hipExtMallocWithFlags(p, bytes, hipDeviceMallocUncached));
  return hipMemset(*p, 0, bytes);
}

hipError_t xgmi_free(void* p) { return hipFree(p); }

hipError_t xgmi_alloc_error_word(int** host, int** dev) {
  PDA_CHECK_HIP(hipHostMalloc(reinterpret_cast<void**>(host), 64, hipHostMallocMapped | hipHostMallocCoherent));
  std::memset(*host, 0, 64);
  return hipHostGetDevicePointer(reinterpret_cast<void**>(dev), *host, 0);
}

hipError_t xgmi_free_error_word(int* host) { return hipHostFree(host); }

hipError_t xgmi_get_handle(void* p, char* out64) {
  hipIpcMemHandle_t h;
  PDA_CHECK_HIP(hipIpcGetMemHandle(&h, p));
  std::memcpy(out64, h.reserved, HIP_IPC_HANDLE_SIZE);
  return hipSuccess;
}

hipError_t xgmi_open_handle(const char* in64, void** p) {
  hipIpcMemHandle_t h;
  std::memcpy(h.reserved, in64, HIP_IPC_HANDLE_SIZE);
  return hipIpcOpenMemHandle(p, h, hipIpcMemLazyEnablePeerAccess);
}

hipError_t xgmi_close_handle(void* p) { return hipIpcCloseMemHandle(p); }

namespace {
int xgmi_blocks(int64_t vectors) {
  int64_t b = (vectors + kXThreads - 1) / kXThreads;
  if (b > kXgmiMaxBlocks) b = kXgmiMaxBlocks;
  return b < 1 ? 1 : (int)b;
}
}  // namespace

hipError_t xgmi_allreduce(const XgmiArgs& a, bool bf16, hipStream_t st) {
  if (a.world < 1 || a.world > kXgmiMaxRanks || a.n % 8) return hipErrorInvalidValue;
  const int64_t nv = a.n / 8;
  switch (a.algo) {
    case kXgmiTwoShot: {
      const unsigned b = xgmi_blocks((nv + a.world - 1) / a.world);
      if (bf16) xgmi_twoshot_kernel<bf16_t><<<b, kXThreads, 0, st>>>(a);
      else xgmi_twoshot_kernel<float><<<b, kXThreads, 0, st>>>(a);
      break;
    }
    case kXgmiRing: {
      const unsigned b = xgmi_blocks((nv + a.world - 1) / a.world);
      if (bf16) xgmi_ring_kernel<bf16_t><<<b, kXThreads, 0, st>>>(a);
      else xgmi_ring_kernel<float><<<b, kXThreads, 0, st>>>(a);
      break;
    }
    case kXgmiAllGather: {
      const unsigned b = xgmi_blocks(nv);
      if (bf16) xgmi_allgather_kernel<bf16_t><<<b, kXThreads, 0, st>>>(a);
      else xgmi_allgather_kernel<float><<<b, kXThreads, 0, st>>>(a);
      break;
    }
    case kXgmiReduceScatter: {
      if (nv % a.world) return hipErrorInvalidValue;
      const unsigned b = xgmi_blocks(nv / a.world);
      if (bf16) xgmi_reduce_scatter_kernel<bf16_t><<<b, kXThreads, 0, st>>>(a);
      else xgmi_reduce_scatter_kernel<float><<<b, kXThreads, 0, st>>>(a);
      break;
    }
    default: {
      const unsigned b = xgmi_blocks(nv);
      if (bf16) xgmi_oneshot_kernel<bf16_t><<<b, kXThreads, 0, st>>>(a);
      else xgmi_oneshot_kernel<float><<<b, kXThreads, 0, st>>>(a);
    }
  }
  return hipGetLastError();
}

}  // namespace pda
