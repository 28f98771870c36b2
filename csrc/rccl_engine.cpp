#include "rccl_engine.h"
#include "trace.h"

#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <chrono>
#include <cstring>
#include <fstream>
#include <thread>
#include <algorithm>

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

// Poll a nonblocking communicator until its pending operation (init or a lazily
// connected first send/recv) finishes. Returns false on error or deadline.
static bool settle(ncclComm_t comm, ncclResult_t r, Clock::time_point deadline, std::string* err,
                   const char* what) {
  while (r == ncclInProgress) {
    if (Clock::now() > deadline) {
      *err = std::string(what) + ": timed out";
      return false;
    }
    std::this_thread::sleep_for(std::chrono::microseconds(200));
    if (ncclCommGetAsyncError(comm, &r) != ncclSuccess) break;
  }
  if (r != ncclSuccess) {
    *err = std::string(what) + ": " + ncclGetErrorString(r);
    return false;
  }
  return true;
}

bool RcclEngine::init(std::string* err) {
  if (world_ <= 1) {
    ready_ = true;
    return true;
  }
  bool ok = init_pairs(err);
  // Every rank publishes its verdict and waits for everyone else's: RCCL is used only if
  // ALL ranks brought up ALL their pairs. A partially working mesh would leave a sender
  // blocked on a receiver that has no communicator, so it is all or nothing.
  std::string mine = dir_ + "/rccl_status_" + std::to_string(rank_);
  {
    std::string tmp = mine + ".tmp";
    int fd = ::open(tmp.c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0644);
    if (fd >= 0) {
      const char c = ok ? '1' : '0';
      (void)!::write(fd, &c, 1);
      ::close(fd);
      (void)::rename(tmp.c_str(), mine.c_str());
    }
  }
  auto deadline = Clock::now() + std::chrono::milliseconds(timeout_ms_);
  bool all = ok;
  for (int r = 0; r < world_ && all; ++r) {
    std::string path = dir_ + "/rccl_status_" + std::to_string(r);
    char c = 0;
    for (;;) {
      int fd = ::open(path.c_str(), O_RDONLY);
      if (fd >= 0) {
        ssize_t n = ::read(fd, &c, 1);
        ::close(fd);
        if (n == 1) break;
      }
      if (Clock::now() > deadline) break;
      std::this_thread::sleep_for(std::chrono::milliseconds(5));
    }
    if (c != '1') {
      all = false;
      if (ok) *err = "rank " + std::to_string(r) + (c == '0' ? " failed RCCL bring-up" : " never reported RCCL status");
    }
  }
  if (!all) {
    for (auto& kv : pairs_) {
      if (kv.second->comm) ncclCommAbort(kv.second->comm);
      kv.second->comm = nullptr;
      if (kv.second->stream) (void)hipStreamDestroy(kv.second->stream);
      kv.second->stream = nullptr;
    }
    pairs_.clear();
    return false;
  }
  ready_ = true;
  return true;
}

bool RcclEngine::init_pairs(std::string* err) {
  if (!store_->gpu()) {
    *err = "RCCL replication requires a GPU chunk store";
    return false;
  }
  if (hipSetDevice(store_->config().device) != hipSuccess) {
    *err = "hipSetDevice failed";
    return false;
  }
  auto deadline = Clock::now() + std::chrono::milliseconds(timeout_ms_);
  // Pairs are brought up in rounds of a round-robin tournament (circle method): in round
  // r every rank meets exactly one partner and the two ordered pairs (lo->hi, hi->lo) are
  // initialised back to back. Every rank walks the same schedule, pairs inside a round are
  // disjoint, so there is no wait cycle, and the critical path is world-1 rounds instead
  // of the world*(world-1) serial steps of a lexicographic order.
  std::vector<std::pair<int, int>> order;
  const int m = world_ % 2 ? world_ + 1 : world_;  // odd world: rank m-1 is a bye
  for (int r = 0; r < m - 1; ++r) {
    int partner = -1;
    for (int x = 0; x < m - 1; ++x) {
      int y = ((2 * r - x) % (m - 1) + (m - 1)) % (m - 1);
      if (y == x) y = m - 1;
      if (x == rank_) partner = y;
      if (y == rank_) partner = x;
    }
    if (partner < 0 || partner >= world_ || partner == rank_) continue;
    int lo = std::min(rank_, partner), hi = std::max(rank_, partner);
    order.emplace_back(lo, hi);
    order.emplace_back(hi, lo);
  }
  for (auto [a, b] : order) {
    auto p = std::make_unique<Pair>();
    ncclUniqueId uid;
    std::string path = uid_path(dir_, a, b);
    if (a == rank_) {
      if (ncclGetUniqueId(&uid) != ncclSuccess || !write_uid(path, uid)) {
        *err = "failed to publish RCCL unique id " + path;
        return false;
      }
    } else {
      int left = static_cast<int>(std::chrono::duration_cast<std::chrono::milliseconds>(deadline - Clock::now()).count());
      if (left <= 0 || !read_uid(path, &uid, left)) {
        *err = "timed out waiting for RCCL unique id " + path;
        return false;
      }
    }
    if (hipStreamCreateWithFlags(&p->stream, hipStreamNonBlocking) != hipSuccess) {
      *err = "hipStreamCreate failed";
      return false;
    }
    // Nonblocking communicator: a peer that never shows up costs a deadline, not a hang.
    ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
    cfg.blocking = 0;
    cfg.minCTAs = 1;
    cfg.maxCTAs = 4;
    ncclResult_t r = ncclCommInitRankConfig(&p->comm, 2, uid, a == rank_ ? 0 : 1, &cfg);
    std::string what = "ncclCommInitRank(" + std::to_string(a) + "->" + std::to_string(b) + ")";
    bool good = p->comm != nullptr && settle(p->comm, r, deadline, err, what.c_str());
    if (!good && p->comm == nullptr && r != ncclInProgress && r != ncclSuccess)
      *err = what + ": " + ncclGetErrorString(r);
    if (good) {
      // Warm-up: one tiny transfer per pair connects the p2p channel (RCCL connects
      // lazily) and proves the path end to end before any block depends on it.
      int32_t* probe = nullptr;
      good = hipMalloc(reinterpret_cast<void**>(&probe), sizeof(int32_t)) == hipSuccess;
      if (good) {
        r = a == rank_ ? ncclSend(probe, 1, ncclInt32, 1, p->comm, p->stream)
                       : ncclRecv(probe, 1, ncclInt32, 0, p->comm, p->stream);
        good = settle(p->comm, r, deadline, err, (what + " warm-up").c_str());
        while (good) {
          hipError_t q = hipStreamQuery(p->stream);
          if (q == hipSuccess) break;
          if (q != hipErrorNotReady || Clock::now() > deadline) {
            *err = what + " warm-up transfer did not complete";
            good = false;
            break;
          }
          std::this_thread::sleep_for(std::chrono::microseconds(100));
        }
        (void)hipFree(probe);
      }
    }
    pairs_[{a, b}] = std::move(p);
    if (!good) return false;
  }
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
  TraceRange tr("dfs.rccl.send");
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
    if (!settle(p->comm, r, Clock::now() + std::chrono::milliseconds(timeout_ms_), err, "ncclSend")) {
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
  TraceRange tr("dfs.rccl.wait_send");
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
  TraceRange tr("dfs.rccl.recv");
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
      std::string rerr;
      if (!settle(p->comm, r, Clock::now() + std::chrono::milliseconds(timeout_ms_), &rerr, "ncclRecv")) {
        lk.unlock();
        (void)hipEventDestroy(ev);
        store_->release(ext);
        res.error = rerr;
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
