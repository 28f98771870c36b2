#include "rccl_engine.h"

#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <chrono>
#include <cstring>
#include <fstream>
#include <thread>

namespace dfs {

namespace {
using Clock = std::chrono::steady_clock;

std::string uid_path(const std::string& dir, int a, int b) {
  return dir + "/rccl_uid_" + std::to_string(a) + "_" + std::to_string(b);
}

bool write_uid(const std::string& path, const ncclUniqueId& id) {
  std::string tmp = path + ".tmp." + std::to_string(::getpid());
  int fd = ::open(tmp.c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0644);
  if (fd < 0) return false;
  bool ok = ::write(fd, id.internal, sizeof(id.internal)) == static_cast<ssize_t>(sizeof(id.internal));
  ::fsync(fd);
  ::close(fd);
  return ok && ::rename(tmp.c_str(), path.c_str()) == 0;
}

bool read_uid(const std::string& path, ncclUniqueId* id, int timeout_ms) {
  auto deadline = Clock::now() + std::chrono::milliseconds(timeout_ms);
  while (Clock::now() < deadline) {
    int fd = ::open(path.c_str(), O_RDONLY);
    if (fd >= 0) {
      ssize_t r = ::read(fd, id->internal, sizeof(id->internal));
      ::close(fd);
      if (r == static_cast<ssize_t>(sizeof(id->internal))) return true;
    }
    std::this_thread::sleep_for(std::chrono::milliseconds(5));
  }
  return false;
}
}  // namespace

RcclEngine::RcclEngine(ChunkStore* store, int rank, int world, std::string dir, int timeout_ms)
    : store_(store), rank_(rank), world_(world), dir_(std::move(dir)), timeout_ms_(timeout_ms) {}

RcclEngine::~RcclEngine() {
  for (auto& kv : pairs_) {
    Pair* p = kv.second.get();
    if (!p->comm) continue;
    bool idle;
    {
      std::lock_guard<std::mutex> g(p->mu);
      idle = p->pending.empty() && !p->broken;
    }
    // A pair with transfers still in flight could block its peer's kernel forever:
    // abort instead of destroy so no wave is left spinning on the device.
    if (idle && hipStreamQuery(p->stream) == hipSuccess) ncclCommDestroy(p->comm);
    else ncclCommAbort(p->comm);
    (void)hipStreamDestroy(p->stream);
  }
}

bool RcclEngine::init(std::string* err) {
  if (world_ <= 1) {
    ready_ = true;
    return true;
  }
  if (!store_->gpu()) {
    *err = "RCCL replication requires a GPU chunk store";
    return false;
  }
  if (hipSetDevice(store_->config().device) != hipSuccess) {
    *err = "hipSetDevice failed";
    return false;
  }
  for (int a = 0; a < world_; ++a)
    for (int b = 0; b < world_; ++b) {
      if (a == b || (a != rank_ && b != rank_)) continue;
      auto p = std::make_unique<Pair>();
      ncclUniqueId uid;
      std::string path = uid_path(dir_, a, b);
      if (a == rank_) {
        if (ncclGetUniqueId(&uid) != ncclSuccess || !write_uid(path, uid)) {
          *err = "failed to publish RCCL unique id " + path;
          return false;
        }
      } else if (!read_uid(path, &uid, timeout_ms_)) {
        *err = "timed out waiting for RCCL unique id " + path;
        return false;
      }
      if (hipStreamCreateWithFlags(&p->stream, hipStreamNonBlocking) != hipSuccess) {
        *err = "hipStreamCreate failed";
        return false;
      }
      ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
      cfg.blocking = 1;
      cfg.minCTAs = 1;
      cfg.maxCTAs = 4;
      ncclResult_t r = ncclCommInitRankConfig(&p->comm, 2, uid, a == rank_ ? 0 : 1, &cfg);
      if (r != ncclSuccess) {
        *err = std::string("ncclCommInitRank(") + std::to_string(a) + "->" + std::to_string(b) +
               "): " + ncclGetErrorString(r);
        return false;
      }
      pairs_[{a, b}] = std::move(p);
    }
  ready_ = true;
  return true;
}

RcclEngine::Pair* RcclEngine::pair(int src, int dst) {
  auto it = pairs_.find({src, dst});
  return it == pairs_.end() ? nullptr : it->second.get();
}

bool RcclEngine::pair_ok(int src, int dst) const {
  auto it = pairs_.find({src, dst});
  return ready_ && it != pairs_.end() && !it->second->broken;
}

bool RcclEngine::wait_event(hipEvent_t ev, Pair* p) {
  auto deadline = Clock::now() + std::chrono::milliseconds(timeout_ms_);
  int spins = 0;
  for (;;) {
    hipError_t q = hipEventQuery(ev);
    if (q == hipSuccess) return true;
    if (q != hipErrorNotReady) return false;
    if (p->broken || Clock::now() > deadline) return false;
    if (++spins < 200) std::this_thread::yield();
    else std::this_thread::sleep_for(std::chrono::microseconds(50));
  }
}

void RcclEngine::abort_pair(int src, int dst) {
  Pair* p = pair(src, dst);
  if (!p) return;
  std::lock_guard<std::mutex> g(p->mu);
  if (p->broken) return;
  p->broken = true;
  if (p->comm) ncclCommAbort(p->comm);
  p->comm = nullptr;
  p->cv.notify_all();
}

int64_t RcclEngine::send(int peer, const std::string& id, uint64_t* size, std::string* err) {
  Pair* p = pair(rank_, peer);
  if (!p || p->broken) {
    *err = "no RCCL path to rank " + std::to_string(peer);
    return -1;
  }
  (void)hipSetDevice(store_->config().device);
  const uint8_t* d = store_->pin_device(id, size);
  if (!d) {
    *err = "block not resident: " + id;
    return -1;
  }
  std::lock_guard<std::mutex> g(p->mu);
  if (p->broken) {
    store_->unpin(id);
    *err = "RCCL pair broken";
    return -1;
  }
  int64_t seq = p->next_seq++;
  hipEvent_t ev;
  (void)hipEventCreateWithFlags(&ev, hipEventDisableTiming);
  if (*size) {
    ncclResult_t r = ncclSend(d, *size, ncclUint8, 1, p->comm, p->stream);
    if (r != ncclSuccess) {
      *err = std::string("ncclSend: ") + ncclGetErrorString(r);
      (void)hipEventDestroy(ev);
      store_->unpin(id);
      return -1;
    }
  }
  (void)hipEventRecord(ev, p->stream);
  p->pending[seq] = Pair::Pending{ev, id};
  bytes_sent_ += *size;
  return seq;
}

bool RcclEngine::wait_send(int peer, int64_t seq, std::string* err) {
  Pair* p = pair(rank_, peer);
  if (!p) return false;
  Pair::Pending pend;
  {
    std::lock_guard<std::mutex> g(p->mu);
    auto it = p->pending.find(seq);
    if (it == p->pending.end()) return true;
    pend = it->second;
  }
  bool ok = wait_event(pend.ev, p);
  if (!ok) {
    *err = "RCCL send to rank " + std::to_string(peer) + " timed out";
    abort_pair(rank_, peer);
  }
  {
    std::lock_guard<std::mutex> g(p->mu);
    p->pending.erase(seq);
  }
  (void)hipEventDestroy(pend.ev);
  store_->unpin(pend.id);
  return ok;
}

WriteResult RcclEngine::recv(int src, int64_t seq, const std::string& id, uint64_t size, uint32_t expected_crc,
                             bool persist_now) {
  WriteResult res;
  Pair* p = pair(src, rank_);
  if (!p || p->broken) {
    res.error = "no RCCL path from rank " + std::to_string(src);
    return res;
  }
  (void)hipSetDevice(store_->config().device);
  DevExtent ext = store_->reserve(size);
  if (ext.off < 0) {
    res.error = "HBM arena full";
    abort_pair(src, rank_);  // the matching send can never be consumed now
    return res;
  }
  hipEvent_t ev;
  (void)hipEventCreateWithFlags(&ev, hipEventDisableTiming);
  {
    std::unique_lock<std::mutex> lk(p->mu);
    bool turn = p->cv.wait_for(lk, std::chrono::milliseconds(timeout_ms_),
                               [&] { return p->broken || p->next_seq == seq; });
    if (!turn || p->broken) {
      lk.unlock();
      (void)hipEventDestroy(ev);
      store_->release(ext);
      res.error = "RCCL receive sequence " + std::to_string(seq) + " from rank " + std::to_string(src) + " timed out";
      abort_pair(src, rank_);
      return res;
    }
    if (size) {
      ncclResult_t r = ncclRecv(ext.ptr, size, ncclUint8, 0, p->comm, p->stream);
      if (r != ncclSuccess) {
        lk.unlock();
        (void)hipEventDestroy(ev);
        store_->release(ext);
        res.error = std::string("ncclRecv: ") + ncclGetErrorString(r);
        abort_pair(src, rank_);
        return res;
      }
    }
    (void)hipEventRecord(ev, p->stream);
    p->next_seq++;
  }
  p->cv.notify_all();
  bool ok = wait_event(ev, p);
  (void)hipEventDestroy(ev);
  if (!ok) {
    res.error = "RCCL receive from rank " + std::to_string(src) + " did not complete";
    abort_pair(src, rank_);
    return res;  // extent intentionally leaked: a late DMA may still land in it
  }
  bytes_recv_ += size;
  return store_->commit_device(id, ext, size, expected_crc, nullptr, persist_now);
}

}  // namespace dfs
