#include "disk_gate.h"

#include <fcntl.h>
#include <sys/file.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cerrno>
#include <cstdio>
#include <cstdlib>

namespace dfs {

int disk_inflight_default() {
  const char* e = std::getenv("DFS_DISK_INFLIGHT");
  return e && *e ? std::atoi(e) : 12;
}

DiskGate::DiskGate(const std::string& dir, int slots) {
  if (slots <= 0) return;
  struct stat st {};
  if (::stat(dir.c_str(), &st) != 0) return;
  char name[96];
  std::snprintf(name, sizeof name, "/dev/shm/dfs_diskgate_%llx_%d", static_cast<unsigned long long>(st.st_dev),
                slots);
  dir_ = name;
  if (::mkdir(name, 0777) != 0 && errno != EEXIST) return;
  std::vector<int> fds;
  for (int i = 0; i < slots; ++i) {
    std::string p = dir_ + "/slot_" + std::to_string(i);
    int fd = ::open(p.c_str(), O_RDWR | O_CREAT | O_CLOEXEC, 0666);
    if (fd < 0) {
      for (int f : fds) ::close(f);
      return;  // no /dev/shm: run ungated
    }
    fds.push_back(fd);
  }
  fds_ = std::move(fds);
  local_.reset(new Local[fds_.size()]);
}

DiskGate::~DiskGate() {
  for (int f : fds_) ::close(f);
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

void DiskGate::unlock(int i) {
  ::flock(fds_[i], LOCK_UN);
  {
    std::lock_guard<std::mutex> g(local_[i].m);
    local_[i].busy = false;
  }
  local_[i].cv.notify_one();
}

bool DiskGate::take(int i, bool block, Slot* s) {
  {
    std::unique_lock<std::mutex> lk(local_[i].m);
    if (block) local_[i].cv.wait(lk, [&] { return !local_[i].busy; });
    else if (local_[i].busy) return false;
    local_[i].busy = true;
  }
  int r;
  do r = ::flock(fds_[i], LOCK_EX | (block ? 0 : LOCK_NB));
  while (r != 0 && errno == EINTR);
  if (r != 0) {
    {
      std::lock_guard<std::mutex> g(local_[i].m);
      local_[i].busy = false;
    }
    local_[i].cv.notify_one();
    return false;
  }
  s->g_ = this;
  s->i_ = i;
  return true;
}

DiskGate::Slot DiskGate::try_acquire(bool* got) {
  Slot s;
  *got = fds_.empty();
  if (fds_.empty()) return s;
  const int n = static_cast<int>(fds_.size());
  int start = static_cast<int>(__atomic_fetch_add(&next_, 1, __ATOMIC_RELAXED) % n);
  for (int k = 0; k < n; ++k)
    if (take((start + k) % n, false, &s)) {
      *got = true;
      break;
    }
  return s;
}

DiskGate::Slot DiskGate::acquire() {
  // One non-blocking pass over every slot (rotating start so processes spread out); when
  // the node is saturated, queue on one slot with a blocking flock: K independent FIFO
  // queues, no polling (hundreds of waiters must not burn CPU).
  bool got = false;
  Slot s = try_acquire(&got);
  if (got) return s;
  __atomic_fetch_add(&waits_, 1, __ATOMIC_RELAXED);
  const int i = static_cast<int>(__atomic_fetch_add(&next_, 1, __ATOMIC_RELAXED) % fds_.size());
  while (!take(i, true, &s)) {
  }
  return s;
}

}  // namespace dfs
