// All-reduce over IPC-mapped peer buffers: every rank copies its
// bucket into its own exchange buffer, then one kernel per rank reads the peers' buffers straight over
// xGMI (the 8 MI355X of a node are a full mesh: 7 links per GPU are used at once, where a ring drives
// one).  RCCL stays the default (opt-in: PDA_ALLREDUCE=oneshot|twoshot|ipc).
//   * one-shot: each rank reads ALL of every peer's buffer and reduces locally — (N-1)·S bytes over
//     the links per rank, one barrier round: latency-optimal for small buckets.
//   * two-shot: reduce-scatter then all-gather, both direct over the mesh.  Rank r reduces chunk r
//     (S/N) from all peers into its own exchange buffer, then every rank copies chunk c from rank c —
//     2·(N-1)/N·S bytes per rank (the ring's volume, but on 7 links at once): bandwidth-optimal.
//     Element→workgroup mapping is identical on every rank (grid-stride inside each chunk), so the
//     per-workgroup flag barrier between the two phases orders exactly the producer/consumer pairs.
//
// Synchronisation: per workgroup, two flag barriers (phase 0: "my buffer holds epoch e", phase 1:
// "I finished reading your buffer for epoch e", so nobody refills its buffer while a peer still
// reads it).  Flags and exchange buffers are uncached device memory (hipDeviceMallocUncached), so
// stores are visible to peers on other GPUs / other XCDs without relying on L2 write-back; the flag
// stores are release / the spin loads acquire at system scope.  Every spin is bounded by a
// wall-clock deadline: on timeout the kernel records an error and exits instead of hanging.  The error
// word is pinned host memory, so callers (DDP) poll it every step without synchronising the device;
// a communicator that reported a timeout is poisoned (its peers' epochs no longer line up).
#include "pda_common.h"
#include "pda_kernels.h"

#include <cstring>

namespace pda {
namespace {

constexpr int kXThreads = 256;

__device__ __forceinline__ void flag_barrier(const XgmiArgs& a, int phase) {
  __syncthreads();
  const int t = threadIdx.x;
  if (t < a.world) {
    const int slot = (phase * kXgmiMaxBlocks + blockIdx.x) * kXgmiMaxRanks;
    __threadfence_system();
    __hip_atomic_store(a.flags[t] + slot + a.rank, a.epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    const uint32_t* mine = a.flags[a.rank] + slot + t;
    const long long t0 = wall_clock64();
    while (__hip_atomic_load(mine, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) < a.epoch) {
      if (wall_clock64() - t0 > a.timeout_ticks) {
        // err lives in host-coherent pinned memory: the host polls it without a device sync.  Keep
        // the FIRST phase that timed out (later barriers of the same call time out as a consequence).
        if (__hip_atomic_load(a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) == 0)
          __hip_atomic_store(a.err, 1 + phase, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
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

hipError_t xgmi_allreduce(const XgmiArgs& a, bool bf16, hipStream_t st) {
  if (a.world < 1 || a.world > kXgmiMaxRanks || a.n % 8) return hipErrorInvalidValue;
  if (a.algo == 1) {
    const int64_t cv = (a.n / 8 + a.world - 1) / a.world;
    int64_t blocks = (cv + kXThreads - 1) / kXThreads;
    if (blocks > kXgmiMaxBlocks) blocks = kXgmiMaxBlocks;
    if (blocks < 1) blocks = 1;
    if (bf16) xgmi_twoshot_kernel<bf16_t><<<(unsigned)blocks, kXThreads, 0, st>>>(a);
    else xgmi_twoshot_kernel<float><<<(unsigned)blocks, kXThreads, 0, st>>>(a);
    return hipGetLastError();
  }
  int64_t blocks = (a.n / 8 + kXThreads - 1) / kXThreads;
  if (blocks > kXgmiMaxBlocks) blocks = kXgmiMaxBlocks;
  if (blocks < 1) blocks = 1;
  if (bf16) xgmi_oneshot_kernel<bf16_t><<<(unsigned)blocks, kXThreads, 0, st>>>(a);
  else xgmi_oneshot_kernel<float><<<(unsigned)blocks, kXThreads, 0, st>>>(a);
  return hipGetLastError();
}

}  // namespace pda
