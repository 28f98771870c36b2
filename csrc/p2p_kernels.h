// Device side of the hipipc transport's spin mode (p2p_ipc.cpp): kernels that behave like
// RCCL's point-to-point kernels — they occupy their stream (and the hardware queue it maps
// to) while they wait for the peer — so the replication protocol can be exercised against
// that hazard on a single GPU. Every wait is bounded by the device wall clock and an abort
// word, so a kernel whose peer never shows up still exits.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace dfs {

// Shared-memory ring of one directed channel (receiver -> sender credits, sender ->
// receiver completions). Lives in /dev/shm, mapped by both processes and registered for
// device access; every field a kernel touches is 8-byte aligned.
struct IpcSlot {
  uint64_t off;  // byte offset of the posted buffer in the receiver's arena
  uint64_t n;    // bytes
};

constexpr uint32_t kIpcRing = 4096;

struct alignas(64) IpcRing {
  uint64_t magic;
  uint64_t gen;
  int32_t receiver_pid;
  int32_t pad0;
  alignas(64) uint64_t posted;     // receives posted (count); receiver writes
  alignas(64) uint64_t landed;     // receives whose bytes landed (count); sender writes
  alignas(64) uint64_t enqueued;   // copies the sender queued (count)
  alignas(64) uint32_t abort;      // either side: the channel is dead
  alignas(64) uint32_t doorbell;   // futex word: bumped on every post (both sides)
  alignas(64) uint32_t landed_bell;     // futex word: bumped after `landed` advances or on abort
  uint32_t landed_waiters;              // receivers blocked on landed_bell (wake only if > 0)
  alignas(64) uint32_t sender_attached;
  uint32_t receiver_ready;
  uint64_t warm;                   // generation whose warm-up copy the sender delivered
  uint32_t pull;                   // receiver: 1 = I pull (set before my warm-up is published)
  alignas(64) IpcSlot slots[kIpcRing];
  // receiver pull: the sender offers each slice (offset in ITS arena, length) and the
  // receiver's kernel reads it over xGMI; `landed` then counts the slices the receiver's
  // kernels finished, which is also what completes the sender's op
  alignas(64) uint64_t offered;    // slices offered (count); sender writes
  alignas(64) IpcSlot offers[kIpcRing];
};

struct IpcSendArgs {
  const uint64_t* posted;  // device views of the ring fields
  uint64_t* landed;
  uint32_t* abort;
  const IpcSlot* slots;
  uint64_t seq;
  const uint8_t* src;
  uint8_t* peer_base;
  uint64_t peer_bytes;
  uint64_t n;
  uint32_t* done_ctr;   // device memory, 0 between ops (the last workgroup resets it)
  uint64_t spin_ticks;  // wall-clock ticks a workgroup may wait for credit
};

// Wait for the receiver's credit for op `seq`, copy n bytes into its buffer, publish landed.
hipError_t launch_ipc_send(const IpcSendArgs& a, int grid, hipStream_t s);
// Spin until *landed >= target (or abort, or spin_ticks): the receive side's kernel.
hipError_t launch_ipc_wait(const uint64_t* landed, uint64_t target, uint32_t* abort, uint64_t spin_ticks,
                           hipStream_t s);
// Host-driven mode's copy: n bytes from this device's arena into the peer's (IPC-mapped,
// over xGMI between GPUs) by the waves' own 16-byte loads and stores. Both pointers must be
// 16-byte aligned. A copy-engine hipMemcpyAsync of a 256 KiB slice took ~31 us on average
// (rocprofv3 memory-copy trace, profiles/r5_final); the kernel runs at HBM / link speed.
hipError_t launch_ipc_copy(uint8_t* dst, const uint8_t* src, uint64_t n, hipStream_t s);
// Device wall-clock frequency in ticks per millisecond (hipDeviceAttributeWallClockRate).
uint64_t wall_ticks_per_ms(int device);

}  // namespace dfs
