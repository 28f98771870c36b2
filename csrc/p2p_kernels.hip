// Spin-mode kernels of the hipipc transport; contract in p2p_kernels.h.
//
// These mimic the shape of RCCL's p2p kernels on purpose: the send kernel parks on its
// stream until the receiver's credit (a posted buffer) appears in the shared ring, then
// copies with the whole grid and publishes completion; the wait kernel parks on the receive
// stream until the bytes have landed. Lane 0 of each workgroup polls the ring in host
// memory with system-scope loads (the ring is written by another process's host thread or
// by the peer's kernel), sleeping between polls; the wall clock bounds every wait.
#include "p2p_kernels.h"

#include <algorithm>

namespace dfs {

namespace {

__device__ inline uint64_t ld_sys(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ inline uint32_t ld_sys32(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ inline void set_abort(uint32_t* p) { __hip_atomic_store(p, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM); }

__global__ __launch_bounds__(256) void ipc_send_kernel(IpcSendArgs a) {
  __shared__ uint32_t go;
  __shared__ uint64_t off;
  if (threadIdx.x == 0) {
    const uint64_t t0 = wall_clock64();
    uint32_t ok = 0;
    uint64_t o = 0;
    for (;;) {
      if (ld_sys32(a.abort)) break;
      if (ld_sys(a.posted) > a.seq) {
        ok = 1;
        break;
      }
      if (wall_clock64() - t0 > a.spin_ticks) {
        set_abort(a.abort);
        break;
      }
      __builtin_amdgcn_s_sleep(16);
    }
    if (ok) {
      const IpcSlot* sl = a.slots + (a.seq % kIpcRing);
      o = __hip_atomic_load(&sl->off, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      const uint64_t n = __hip_atomic_load(&sl->n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      if (n != a.n || o > a.peer_bytes || n > a.peer_bytes - o) {  // size mismatch: RCCL would fail too
        set_abort(a.abort);
        ok = 0;
      }
    }
    go = ok;
    off = o;
  }
  __syncthreads();
  if (!go) return;
  uint8_t* dst = a.peer_base + off;
  const uint64_t nv = a.n / 16;
  const uint4* s4 = reinterpret_cast<const uint4*>(a.src);
  uint4* d4 = reinterpret_cast<uint4*>(dst);
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * blockDim.x;
  for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < nv; i += stride) d4[i] = s4[i];
  if (blockIdx.x == 0)
    for (uint64_t i = nv * 16 + threadIdx.x; i < a.n; i += blockDim.x) dst[i] = a.src[i];
  // every storing wave's bytes leave this XCD's L2 before its workgroup is counted
  __threadfence_system();
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t prev = atomicAdd(a.done_ctr, 1u);
    if (prev == gridDim.x - 1) {  // last workgroup: all bytes are out; reset, then publish
      atomicExch(a.done_ctr, 0u);
      __hip_atomic_store(a.landed, a.seq + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

__global__ __launch_bounds__(64) void ipc_wait_kernel(const uint64_t* landed, uint64_t target, uint32_t* abort,
                                                      uint64_t spin_ticks) {
  if (threadIdx.x != 0) return;
  const uint64_t t0 = wall_clock64();
  for (;;) {
    if (ld_sys(landed) >= target || ld_sys32(abort)) return;
    if (wall_clock64() - t0 > spin_ticks) {
      set_abort(abort);
      return;
    }
    __builtin_amdgcn_s_sleep(16);
  }
}

__global__ __launch_bounds__(256) void ipc_copy_kernel(uint8_t* __restrict__ dst, const uint8_t* __restrict__ src,
                                                       uint64_t n) {
  const uint64_t nv = n / 16;
  const uint4* s4 = reinterpret_cast<const uint4*>(src);
  uint4* d4 = reinterpret_cast<uint4*>(dst);
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * blockDim.x;
  uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  // four independent 16-byte loads in flight per lane before their stores
  for (; i + 3 * stride < nv; i += 4 * stride) {
    const uint4 a = s4[i], b = s4[i + stride], c = s4[i + 2 * stride], d = s4[i + 3 * stride];
    d4[i] = a;
    d4[i + stride] = b;
    d4[i + 2 * stride] = c;
    d4[i + 3 * stride] = d;
  }
  for (; i < nv; i += stride) d4[i] = s4[i];
  if (blockIdx.x == 0)
    for (uint64_t k = nv * 16 + threadIdx.x; k < n; k += blockDim.x) dst[k] = src[k];
}

}  // namespace

hipError_t launch_ipc_copy(uint8_t* dst, const uint8_t* src, uint64_t n, hipStream_t s) {
  if (n == 0) return hipSuccess;
  if ((reinterpret_cast<uintptr_t>(dst) | reinterpret_cast<uintptr_t>(src)) % 16) return hipErrorInvalidValue;
  // one 16-byte vector per lane up to 4 MiB (1 MiB: 256 workgroups, one per CU), then
  // grid-stride with four loads in flight
  const uint64_t g = std::min<uint64_t>(1024, std::max<uint64_t>(1, (n + 4095) / 4096));
  hipLaunchKernelGGL(ipc_copy_kernel, dim3(static_cast<unsigned>(g)), dim3(256), 0, s, dst, src, n);
  return hipGetLastError();
}

hipError_t launch_ipc_send(const IpcSendArgs& a, int grid, hipStream_t s) {
  hipLaunchKernelGGL(ipc_send_kernel, dim3(grid), dim3(256), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_ipc_wait(const uint64_t* landed, uint64_t target, uint32_t* abort, uint64_t spin_ticks,
                           hipStream_t s) {
  hipLaunchKernelGGL(ipc_wait_kernel, dim3(1), dim3(64), 0, s, landed, target, abort, spin_ticks);
  return hipGetLastError();
}

uint64_t wall_ticks_per_ms(int device) {
  int khz = 0;
  if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, device) != hipSuccess || khz <= 0) khz = 100000;
  return static_cast<uint64_t>(khz);
}

}  // namespace dfs
