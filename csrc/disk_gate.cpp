#include "disk_gate.h"

#include <fcntl.h>
#include <linux/futex.h>
#include <signal.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <climits>
#include <cstdio>
#include <cstdlib>
#include <ctime>

namespace dfs {

namespace {

constexpr uint32_t kMagic = 0x44474631;  // "DGF1"
constexpr int kMaxSlots = 256;

// Shared by every process of the node that writes to one filesystem (a /dev/shm file).
// Admission is a FIFO ticket semaphore: ticket t enters once t < released + slots, so at most
// `slots` durable writes are in flight and waiters are admitted strictly in arrival order
// (no barging, no per-slot queues of unequal length). Holders register (pid, ticket) in a
// table so a waiter can reclaim the capacity of a holder that died mid-write.
struct Shared {
  std::atomic<uint32_t> magic;
  std::atomic<uint32_t> slots;
  std::atomic<uint64_t> next;      // next ticket to hand out
  std::atomic<uint32_t> released;  // exits so far (low 32 bits; futex word)
  uint32_t pad;
  struct Holder {
    std::atomic<int32_t> pid;  // 0 = free
    std::atomic<uint32_t> ticket;
  } holders[kMaxSlots];
};
static_assert(sizeof(std::atomic<uint32_t>) == 4, "futex word");

long futex(std::atomic<uint32_t>* w, int op, uint32_t val, const timespec* ts) {
  return ::syscall(SYS_futex, reinterpret_cast<uint32_t*>(w), op, val, ts, nullptr, 0);
}

bool alive(int32_t pid) { return pid > 0 && (::kill(pid, 0) == 0 || errno == EPERM); }

}  // namespace

int disk_inflight_default() {
  const char* e = std::getenv("DFS_DISK_INFLIGHT");
  return e && *e ? std::atoi(e) : 12;
}

DiskGate::DiskGate(const std::string& dir, int slots) {
  if (slots <= 0) return;
  slots = std::min(slots, kMaxSlots);
  struct stat st {};
  if (::stat(dir.c_str(), &st) != 0) return;
  char name[96];
  std::snprintf(name, sizeof name, "/dev/shm/dfs_diskgate_v2_%llx_%d", static_cast<unsigned long long>(st.st_dev),
                slots);
  int fd = ::open(name, O_RDWR | O_CREAT | O_CLOEXEC, 0666);
  if (fd < 0) return;  // no /dev/shm: run ungated
  if (::ftruncate(fd, sizeof(Shared)) != 0) {
    ::close(fd);
    return;
  }
  void* p = ::mmap(nullptr, sizeof(Shared), PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  ::close(fd);
  if (p == MAP_FAILED) return;
  auto* sh = static_cast<Shared*>(p);
  // a fresh file is all zeros: the first process stamps the slot count (zeros are a valid
  // empty state, so racing initialisers agree)
  uint32_t z = 0;
  if (sh->magic.compare_exchange_strong(z, kMagic)) sh->slots.store(static_cast<uint32_t>(slots));
  shm_ = sh;
  slots_ = static_cast<int>(sh->slots.load() ? sh->slots.load() : static_cast<uint32_t>(slots));
}

DiskGate::~DiskGate() {
  if (shm_) ::munmap(shm_, sizeof(Shared));
}

DiskGate::Slot& DiskGate::Slot::operator=(Slot&& o) noexcept {
  if (this != &o) {
    release();
    g_ = o.g_;
    i_ = o.i_;
    o.g_ = nullptr;
  }
  return *this;
}

void DiskGate::Slot::release() {
  if (g_) g_->unlock(i_);
  g_ = nullptr;
}

// Claim a holder entry for our admitted ticket (at most `slots` are ever admitted at once,
// so one is free unless a crashed holder still occupies it — reclaimed by the waiters).
int DiskGate::claim(uint64_t ticket) {
  auto* sh = static_cast<Shared*>(shm_);
  const int32_t me = static_cast<int32_t>(::getpid());
  for (;;) {
    for (int i = 0; i < kMaxSlots; ++i) {
      int32_t z = 0;
      if (sh->holders[i].pid.compare_exchange_strong(z, me)) {
        sh->holders[i].ticket.store(static_cast<uint32_t>(ticket));
        return i;
      }
    }
    reap();
  }
}

void DiskGate::unlock(int i) {
  auto* sh = static_cast<Shared*>(shm_);
  sh->holders[i].pid.store(0);
  sh->released.fetch_add(1);
  futex(&sh->released, FUTEX_WAKE, INT_MAX, nullptr);
}

// Give back the capacity of holders whose process is gone (crashed mid-write).
void DiskGate::reap() {
  auto* sh = static_cast<Shared*>(shm_);
  for (int i = 0; i < kMaxSlots; ++i) {
    int32_t pid = sh->holders[i].pid.load();
    if (pid != 0 && !alive(pid) && sh->holders[i].pid.compare_exchange_strong(pid, 0)) {
      sh->released.fetch_add(1);
      futex(&sh->released, FUTEX_WAKE, INT_MAX, nullptr);
    }
  }
}

bool DiskGate::admitted(uint64_t ticket) const {
  auto* sh = static_cast<Shared*>(shm_);
  // released is a 32-bit counter: compare in modular arithmetic (tickets in flight << 2^31)
  uint32_t r = sh->released.load();
  return static_cast<int32_t>(static_cast<uint32_t>(ticket) - r) < slots_;
}

DiskGate::Slot DiskGate::try_acquire(bool* got) {
  Slot s;
  *got = shm_ == nullptr;
  if (!shm_) return s;
  auto* sh = static_cast<Shared*>(shm_);
  // take a ticket only if it would be admitted at once (nobody queued ahead of us)
  reap();
  uint64_t t = sh->next.load();
  while (static_cast<int32_t>(static_cast<uint32_t>(t) - sh->released.load()) < slots_) {
    if (sh->next.compare_exchange_weak(t, t + 1)) {
      s.g_ = this;
      s.i_ = claim(t);
      *got = true;
      return s;
    }
  }
  return s;
}

DiskGate::Slot DiskGate::acquire() {
  Slot s;
  if (!shm_) return s;
  auto* sh = static_cast<Shared*>(shm_);
  const uint64_t t = sh->next.fetch_add(1);
  if (!admitted(t)) {
    __atomic_fetch_add(&waits_, 1, __ATOMIC_RELAXED);
    const timespec tick{0, 200 * 1000 * 1000};  // re-check for dead holders every 200 ms
    while (!admitted(t)) {
      uint32_t r = sh->released.load();
      if (admitted(t)) break;
      if (futex(&sh->released, FUTEX_WAIT, r, &tick) != 0 && errno == ETIMEDOUT) reap();
    }
  }
  s.g_ = this;
  s.i_ = claim(t);
  return s;
}

}  // namespace dfs
