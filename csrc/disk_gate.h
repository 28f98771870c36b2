// Node-wide admission control for durable block writes (nvme-sync).
//
// Every GPU of a node runs its own ChunkServer process, and with RF=3 each client write
// becomes three write+fdatasync streams that usually land on the same volume. Measured on
// an MI355X box (profiles/archive/r1_disk/disk_sweep_*.json) the volume peaks at 10-30 concurrent
// 1 MiB durable writers (8.5-9.2 GB/s buffered) and collapses to 3-4 GB/s with p99 > 100 ms
// once 60-240 writers pile up — exactly the N=8 replication load. DiskGate caps the number
// of durable writes in flight per filesystem ACROSS processes, each slot held for one
// block's write+flush. Admission is a FIFO ticket semaphore in a /dev/shm page keyed by the
// storage directory's st_dev (futex wait/wake across processes): writers enter strictly in
// arrival order, which is what keeps the RF=3 write tail flat under load (r1's per-slot
// flock queues let late arrivals barge and left unlucky waiters behind long queues). A
// holder that dies mid-write is detected by pid and its capacity reclaimed. The reference
// (dfs/chunkserver/src/chunkserver.rs write_block_async) has no equivalent: each
// spawn_blocking write goes straight to the disk.
#pragma once
#include <condition_variable>
#include <cstdint>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

namespace dfs {

class DiskGate {
 public:
  // `dir` selects the filesystem (its st_dev); slots <= 0 disables the gate.
  DiskGate(const std::string& dir, int slots);
  ~DiskGate();
  bool enabled() const { return shm_ != nullptr; }
  int slots() const { return shm_ ? slots_ : 0; }

  class Slot {
   public:
    Slot() = default;
    Slot(Slot&& o) noexcept : g_(o.g_), i_(o.i_) { o.g_ = nullptr; }
    Slot& operator=(Slot&& o) noexcept;
    ~Slot() { release(); }
    void release();
    bool held() const { return g_ != nullptr; }

   private:
    friend class DiskGate;
    DiskGate* g_ = nullptr;
    int i_ = -1;
  };
  // Blocks until this writer's turn (FIFO across every process of the node; immediately
  // when disabled).
  Slot acquire();
  // One non-blocking pass; `*got` says whether a slot was taken.
  Slot try_acquire(bool* got);
  uint64_t waits() const { return waits_; }

 private:
  int claim(uint64_t ticket);
  void unlock(int i);
  void reap();
  bool admitted(uint64_t ticket) const;
  void* shm_ = nullptr;  // Shared admission state (disk_gate.cpp), one per filesystem and cap
  int slots_ = 0;
  uint64_t waits_ = 0;
};

// DFS_DISK_INFLIGHT (default 12; 0 disables) — the per-filesystem cap used by ChunkStore.
int disk_inflight_default();

}  // namespace dfs
