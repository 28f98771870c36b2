// Node-wide admission control for durable block writes (nvme-sync).
//
// Every GPU of a node runs its own ChunkServer process, and with RF=3 each client write
// becomes three write+fdatasync streams that usually land on the same volume. Measured on
// an MI355X box (profiles/r1_native/disk_sweep_*.json) the volume peaks at 10-30 concurrent
// 1 MiB durable writers (8.5-9.2 GB/s buffered) and collapses to 3-4 GB/s with p99 > 100 ms
// once 60-240 writers pile up — exactly the N=8 replication load. DiskGate caps the number
// of durable writes in flight per filesystem ACROSS processes: `slots` lock files in
// /dev/shm keyed by the storage directory's st_dev, each held with flock() for the duration
// of one block's write+flush. flock locks die with their process, so a crashed chunkserver
// never leaks a slot. The reference (dfs/chunkserver/src/chunkserver.rs write_block_async)
// has no equivalent: each spawn_blocking write goes straight to the disk.
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
  bool enabled() const { return !fds_.empty(); }
  int slots() const { return static_cast<int>(fds_.size()); }

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
  // Blocks until one of the node's slots is free (immediately when disabled).
  Slot acquire();
  // One non-blocking pass; `*got` says whether a slot was taken.
  Slot try_acquire(bool* got);
  uint64_t waits() const { return waits_; }

 private:
  bool take(int i, bool block, Slot* s);
  void unlock(int i);
  std::vector<int> fds_;
  struct Local {  // one holder per slot inside this process (released from any thread)
    std::mutex m;
    std::condition_variable cv;
    bool busy = false;
  };
  std::unique_ptr<Local[]> local_;
  std::string dir_;
  uint64_t next_ = 0, waits_ = 0;
};

// DFS_DISK_INFLIGHT (default 12; 0 disables) — the per-filesystem cap used by ChunkStore.
int disk_inflight_default();

}  // namespace dfs
