// One-shot all-reduce over IPC-mapped peer buffers: every rank
// copies its bucket into its own exchange buffer, then one kernel per rank reads ALL peers' buffers
// straight over xGMI (the 8 MI355X of a node are a full mesh: 7 links per GPU are used at once, where
// a ring drives one) and writes the reduced result locally.  Latency-optimal for small and medium
// buckets; RCCL stays the default (opt-in: PDA_ALLREDUCE=ipc).
//
// Synchronisation: per workgroup, two flag barriers (phase 0: "my buffer holds epoch e", phase 1:
// "I finished reading your buffer for epoch e", so nobody refills its buffer while a peer still
// reads it).  Flags and exchange buffers are uncached device memory (hipDeviceMallocUncached), so
// stores are visible to peers on other GPUs / other XCDs without relying on L2 write-back; the flag
// stores are release / the spin loads acquire at system scope.  Every spin is bounded by a
// wall-clock deadline: on timeout the kernel records an error and exits instead of hanging.
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
        atomicExch(a.err, 1 + phase);
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

}  // namespace

hipError_t xgmi_alloc(void** p, size_t bytes) {
  PDA_CHECK_HIP(hipExtMallocWithFlags(p, bytes, hipDeviceMallocUncached));
  return hipMemset(*p, 0, bytes);
}

hipError_t xgmi_free(void* p) { return hipFree(p); }

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
  int64_t blocks = (a.n / 8 + kXThreads - 1) / kXThreads;
  if (blocks > kXgmiMaxBlocks) blocks = kXgmiMaxBlocks;
  if (blocks < 1) blocks = 1;
  if (bf16) xgmi_oneshot_kernel<bf16_t><<<(unsigned)blocks, kXThreads, 0, st>>>(a);
  else xgmi_oneshot_kernel<float><<<(unsigned)blocks, kXThreads, 0, st>>>(a);
  return hipGetLastError();
}

}  // namespace pda
