// One-shot peer-to-peer all-reduce for small buckets over xGMI (SURVEY.md §2.15
// "custom one-shot P2P all-reduce for <= ~1 M elements"; the reference reaches only
// NCCL/oneCCL/gloo all-reduce: trainer.py:215-219, run_pretrain_mlperf.py:565-567).
//
// Every rank owns one IPC-exported staging buffer (coarse-grained HBM) and one signal
// buffer (uncached, so system-scope atomics are coherent across xGMI).  All ranks map all
// peers' buffers (hipIpcOpenMemHandle).  A call is:
//
//   1. the caller copies its input into its own staging buffer (stream ordered);
//   2. kernel, per block: release fence, write `epoch` into slot [block][rank] of every
//      peer's signal buffer, spin until all `world` slots of its own signal buffer for
//      this block hold `epoch` (barrier-in), acquire fence;
//   3. each block sums its grid-stride share of the elements straight out of the peers'
//      staging buffers (16-byte loads over xGMI, fp32 accumulation, rank order fixed so
//      every rank produces bit-identical results) and writes its own output;
//   4. barrier-out with `epoch` in a second slot bank, so no rank overwrites its
//      staging buffer for the next call while a peer still reads it.
//
// Latency is one kernel: no ring steps, each byte crosses xGMI once per peer on the
// direct link.  The spin loops are bounded in WALL-CLOCK time (the constant-rate device
// clock, `timeout_ticks`; the host sizes it like an RCCL timeout, minutes by default): a
// timed-out wait sets an error word in pinned, host-mapped memory and the kernel exits, so
// a missing peer surfaces on the host (the bucketer reads the word every step without a
// device sync and raises) and never as a hung GPU.
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>
#include <string.h>

#include "common.h"

namespace ct {

constexpr int kMaxRanks = 8;
constexpr int kMaxBlocks = 64;
constexpr int kThreads = 512;
// signal buffer layout (uint32): [2 banks][kMaxBlocks][kMaxRanks] slots, then the error word
constexpr int kSigSlots = 2 * kMaxBlocks * kMaxRanks;

struct P2PArgs {
  const void* data[kMaxRanks];  // staging buffers of every rank (own one included)
  uint32_t* sig[kMaxRanks];     // signal buffers of every rank
  void* out;
  long n;                       // elements
  int rank, world;
  uint32_t epoch;
  uint64_t timeout_ticks;       // wall_clock64() ticks
  uint32_t* err;                // host-mapped error word (fine-grained pinned memory)
};

__device__ inline bool barrier(const P2PArgs& a, int bank, uint32_t value) {
  const int b = blockIdx.x;
  // release: the staging copy (and, at barrier-out, this block's reads) happen-before the flag
  __threadfence_system();
  __syncthreads();
  if (threadIdx.x < a.world) {
    uint32_t* slot = a.sig[threadIdx.x] + (bank * kMaxBlocks + b) * kMaxRanks + a.rank;
    __hip_atomic_store(slot, value, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  __shared__ int ok;
  if (threadIdx.x == 0) ok = 1;
  __syncthreads();
  if (threadIdx.x < a.world) {
    const uint32_t* mine = a.sig[a.rank] + (bank * kMaxBlocks + b) * kMaxRanks + threadIdx.x;
    const uint64_t t0 = wall_clock64();
    while (__hip_atomic_load(mine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != value) {
      if (wall_clock64() - t0 > a.timeout_ticks) {
        ok = 0;
        __hip_atomic_store(a.err, 1u + (uint32_t)bank, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
  }
  __syncthreads();
  // acquire: later loads of peer staging buffers must not hit stale cache lines
  __threadfence_system();
  return ok != 0;
}

template <typename T>
struct Vec;
template <>
struct Vec<float> {
  static constexpr int N = 4;
  using V = float4;
  __device__ static void acc(float (&s)[4], const V& v) { s[0] += v.x; s[1] += v.y; s[2] += v.z; s[3] += v.w; }
  __device__ static V pack(const float (&s)[4]) { return make_float4(s[0], s[1], s[2], s[3]); }
  __device__ static float to_f(float x) { return x; }
  __device__ static float from_f(float x) { return x; }
};
template <>
struct Vec<__hip_bfloat16> {
  static constexpr int N = 8;
  using V = uint4;  // 8 x bf16
  __device__ static void acc(float (&s)[8], const V& v) {
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      s[2 * i] += __uint_as_float(w[i] << 16);
      s[2 * i + 1] += __uint_as_float(w[i] & 0xffff0000u);
    }
  }
  __device__ static uint32_t rne(float f) {
    uint32_t u = __float_as_uint(f);
    return (u + 0x7fffu + ((u >> 16) & 1u)) >> 16;
  }
  __device__ static V pack(const float (&s)[8]) {
    uint32_t w[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) w[i] = rne(s[2 * i]) | (rne(s[2 * i + 1]) << 16);
    return make_uint4(w[0], w[1], w[2], w[3]);
  }
  __device__ static float to_f(__hip_bfloat16 x) { return __bfloat162float(x); }
  __device__ static __hip_bfloat16 from_f(float x) { return __float2bfloat16(x); }
};

template <typename T>
__global__ __launch_bounds__(kThreads) void oneshot_allreduce_kernel(P2PArgs a) {
  using VT = Vec<T>;
  if (!barrier(a, 0, a.epoch)) return;
  const long nv = a.n / VT::N;
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < nv; i += stride) {
    float s[VT::N] = {};
    for (int r = 0; r < a.world; ++r) {
      typename VT::V v = reinterpret_cast<const typename VT::V*>(a.data[r])[i];
      VT::acc(s, v);
    }
    reinterpret_cast<typename VT::V*>(a.out)[i] = VT::pack(s);
  }
  // scalar tail (n not a multiple of the vector width): block 0 only
  if (blockIdx.x == 0) {
    for (long i = nv * VT::N + threadIdx.x; i < a.n; i += blockDim.x) {
      float s = 0.f;
      for (int r = 0; r < a.world; ++r) s += VT::to_f(reinterpret_cast<const T*>(a.data[r])[i]);
      reinterpret_cast<T*>(a.out)[i] = VT::from_f(s);
    }
  }
  barrier(a, 1, a.epoch);
}

}  // namespace ct

extern "C" {

size_t ct_p2p_signal_bytes() { return (ct::kSigSlots + 64) * sizeof(uint32_t); }

int ct_p2p_alloc_signal(void** ptr) {
  const size_t bytes = ct_p2p_signal_bytes();
  if (hipExtMallocWithFlags(ptr, bytes, hipDeviceMallocUncached) != hipSuccess) return 1;
  return hipMemset(*ptr, 0, bytes) == hipSuccess ? 0 : 2;
}

int ct_p2p_alloc(void** ptr, size_t bytes) { return hipMalloc(ptr, bytes) == hipSuccess ? 0 : 1; }

// pinned, host-mapped, coherent word pair: the kernel stores, the host reads without a sync
int ct_p2p_alloc_flag(void** host, void** dev) {
  if (hipHostMalloc(host, 64, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) return 1;
  ::memset(*host, 0, 64);
  return hipHostGetDevicePointer(dev, *host, 0) == hipSuccess ? 0 : 2;
}

int ct_p2p_free_flag(void* host) { return hipHostFree(host) == hipSuccess ? 0 : 1; }

// device wall-clock ticks per second (for the barrier timeout)
long ct_p2p_clock_hz() {
  int dev = 0, khz = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess) return 0;
  return (long)khz * 1000L;
}

int ct_p2p_free(void* ptr) { return hipFree(ptr) == hipSuccess ? 0 : 1; }

int ct_ipc_get(void* ptr, char* out /* HIP_IPC_HANDLE_SIZE bytes */) {
  hipIpcMemHandle_t h;
  if (hipIpcGetMemHandle(&h, ptr) != hipSuccess) return 1;
  ::memcpy(out, &h, sizeof(h));
  return 0;
}

int ct_ipc_handle_size() { return (int)sizeof(hipIpcMemHandle_t); }

int ct_ipc_open(const char* handle, void** ptr) {
  hipIpcMemHandle_t h;
  ::memcpy(&h, handle, sizeof(h));
  return hipIpcOpenMemHandle(ptr, h, hipIpcMemLazyEnablePeerAccess) == hipSuccess ? 0 : 1;
}

int ct_ipc_close(void* ptr) { return hipIpcCloseMemHandle(ptr) == hipSuccess ? 0 : 1; }

// dtype: 0 = fp32, 1 = bf16.  Staging buffers must be 16-byte aligned and hold n elements.
int ct_p2p_allreduce(const void* const* data, uint32_t* const* sig, void* out, long n, int dtype, int rank, int world,
                     uint32_t epoch, uint64_t timeout_ticks, uint32_t* err, int blocks, hipStream_t stream) {
  if (world < 1 || world > ct::kMaxRanks || rank < 0 || rank >= world || n < 0) return 1;
  if (blocks < 1 || blocks > ct::kMaxBlocks) return 2;
  if (!err) return 6;
  ct::P2PArgs a{};
  for (int r = 0; r < world; ++r) {
    if (!data[r] || !sig[r] || (reinterpret_cast<uintptr_t>(data[r]) & 15)) return 3;
    a.data[r] = data[r];
    a.sig[r] = sig[r];
  }
  if (reinterpret_cast<uintptr_t>(out) & 15) return 3;
  a.out = out;
  a.n = n;
  a.rank = rank;
  a.world = world;
  a.epoch = epoch;
  a.timeout_ticks = timeout_ticks;
  a.err = err;
  if (dtype == 0)
    hipLaunchKernelGGL(ct::oneshot_allreduce_kernel<float>, dim3(blocks), dim3(ct::kThreads), 0, stream, a);
  else if (dtype == 1)
    hipLaunchKernelGGL(ct::oneshot_allreduce_kernel<__hip_bfloat16>, dim3(blocks), dim3(ct::kThreads), 0, stream, a);
  else
    return 4;
  return hipGetLastError() == hipSuccess ? 0 : 5;
}

}  // extern "C"
