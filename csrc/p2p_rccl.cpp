// RCCL-over-xGMI implementation of P2PTransport (contract in p2p_transport.h).
//
// One process per GPU = one ChunkServer = one RCCL rank, but replication needs
// point-to-point traffic between arbitrary pairs with many blocks in flight, not
// collectives over a world communicator. Each directed channel (a->b, `channels` of them per
// direction) is its own 2-rank communicator (a = rank 0) with its own HIP stream: traffic on
// a communicator is then
// unidirectional and strictly FIFO, which is exactly the matching rule the replication
// protocol sequences against; two directions never share a communicator, so a send a->b
// can never queue behind a receive a<-b. On the MI355X full xGMI mesh every such channel
// is a dedicated link (~64 GB/s per direction), so per-pair communicators also map 1:1
// onto the hardware.
//
// Communicators are nonblocking (ncclConfig.blocking = 0): init and lazily connected p2p
// channels are polled against a deadline, so a peer that never shows up costs a timeout,
// not a hung thread. close() is ncclCommAbort — the only way to end an op whose match will
// never be posted.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <chrono>
#include <cstring>
#include <map>
#include <mutex>
#include <thread>
#include <vector>
#include <algorithm>

#include "p2p_transport.h"

namespace dfs {

namespace {

using Clock = std::chrono::steady_clock;

bool settle(ncclComm_t comm, ncclResult_t r, Clock::time_point deadline, std::string* err, const std::string& what) {
  while (r == ncclInProgress) {
    if (Clock::now() > deadline) {
      *err = what + ": timed out";
      return false;
    }
    std::this_thread::sleep_for(std::chrono::microseconds(100));
    if (ncclCommGetAsyncError(comm, &r) != ncclSuccess) break;
  }
  if (r != ncclSuccess) {
    *err = what + ": " + ncclGetErrorString(r);
    return false;
  }
  return true;
}

class RcclTransport final : public P2PTransport {
 public:
  RcclTransport(int device, int rank, int channels) : device_(device), rank_(rank), channels_(channels) {}

  ~RcclTransport() override {
    (void)hipSetDevice(device_);
    std::lock_guard<std::mutex> g(mu_);
    for (auto& kv : links_) {
      Link& l = *kv.second;
      abort_locked(l);
      for (auto* v : {&l.out, &l.in})
        for (auto& c : *v)
          if (c.stream) (void)hipStreamDestroy(c.stream);
    }
    for (hipEvent_t e : free_events_) (void)hipEventDestroy(e);
  }

  const char* name() const override { return "rccl"; }
  bool device_buffers() const override { return true; }
  int channels() const override { return channels_; }

  // one unique id per channel of our direction, concatenated
  std::string make_token(int, uint64_t, std::string* err) override {
    (void)hipSetDevice(device_);
    std::string tok;
    for (int c = 0; c < channels_; ++c) {
      ncclUniqueId id;
      ncclResult_t r = ncclGetUniqueId(&id);
      if (r != ncclSuccess) {
        *err = std::string("ncclGetUniqueId: ") + ncclGetErrorString(r);
        return {};
      }
      tok.append(id.internal, sizeof(id.internal));
    }
    return tok;
  }

  bool open(int peer, uint64_t gen, const std::string& tok_out, const std::string& tok_in, int timeout_ms,
            std::string* err) override {
    const size_t idb = sizeof(ncclUniqueId::internal);
    if (tok_out.size() != idb * channels_ || tok_in.size() != idb * channels_) {
      *err = "malformed RCCL token (or the peers disagree on the channel count)";
      return false;
    }
    (void)hipSetDevice(device_);
    Link& l = link(peer);
    std::lock_guard<std::mutex> g(l.mu);
    abort_locked(l);
    l.out.resize(channels_);
    l.in.resize(channels_);
    for (auto* v : {&l.out, &l.in})
      for (auto& c : *v)
        if (!c.stream && hipStreamCreateWithFlags(&c.stream, hipStreamNonBlocking) != hipSuccess) {
          *err = "hipStreamCreate failed";
          return false;
        }
    auto deadline = Clock::now() + std::chrono::milliseconds(timeout_ms);
    auto init = [&](Chan& c, const std::string& tok, int my, const std::string& what) {
      ncclUniqueId uid;
      std::memcpy(uid.internal, tok.data(), sizeof(uid.internal));
      ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
      cfg.blocking = 0;
      cfg.minCTAs = 1;
      cfg.maxCTAs = 4;
      ncclResult_t r = ncclCommInitRankConfig(&c.comm, 2, uid, my, &cfg);
      if (c.comm == nullptr) {
        *err = what + ": " + ncclGetErrorString(r);
        return false;
      }
      return settle(c.comm, r, deadline, err, what);
    };
    bool ok = true;
    for (int c = 0; ok && c < channels_; ++c) {
      const std::string tag =
          std::to_string(rank_) + "<->" + std::to_string(peer) + " gen " + std::to_string(gen) + " ch " + std::to_string(c);
      const std::string to = tok_out.substr(c * idb, idb), ti = tok_in.substr(c * idb, idb);
      // both ranks bring up channel c's lo->hi communicator first, then hi->lo
      ok = rank_ < peer ? init(l.out[c], to, 0, "init out " + tag) && init(l.in[c], ti, 1, "init in " + tag)
                        : init(l.in[c], ti, 1, "init in " + tag) && init(l.out[c], to, 0, "init out " + tag);
      if (ok) ok = warm_up(l.out[c], l.in[c], deadline, tag, err);
    }
    if (!ok) {
      abort_locked(l);
      return false;
    }
    l.up = true;
    return true;
  }

  void close(int peer) override {
    (void)hipSetDevice(device_);
    Link& l = link(peer);
    std::lock_guard<std::mutex> g(l.mu);
    abort_locked(l);
  }

  bool post_send(int peer, int ch, const void* buf, uint64_t n, P2POp* op, std::string* err) override {
    return post(peer, ch, true, const_cast<void*>(buf), n, op, err);
  }
  bool post_recv(int peer, int ch, void* buf, uint64_t n, P2POp* op, std::string* err) override {
    return post(peer, ch, false, buf, n, op, err);
  }

  int test(P2POp* op) override {
    hipError_t q = hipEventQuery(static_cast<hipEvent_t>(op->event));
    return q == hipSuccess ? 1 : (q == hipErrorNotReady ? 0 : -1);
  }

  void release(P2POp* op) override {
    if (!op->event) return;
    std::lock_guard<std::mutex> g(mu_);
    free_events_.push_back(static_cast<hipEvent_t>(op->event));
    op->event = nullptr;
  }

 private:
  struct Chan {
    ncclComm_t comm = nullptr;
    hipStream_t stream = nullptr;
  };
  struct Link {
    std::mutex mu;  // ops on one communicator are issued by one thread at a time
    std::vector<Chan> out, in;  // one per channel
    bool up = false;
  };

  Link& link(int peer) {
    std::lock_guard<std::mutex> g(mu_);
    auto& l = links_[peer];
    if (!l) l = std::make_unique<Link>();
    return *l;
  }

  static void abort_locked(Link& l) {
    for (auto* v : {&l.out, &l.in})
      for (auto& c : *v)
        if (c.comm) {
          ncclCommAbort(c.comm);
          c.comm = nullptr;
        }
    l.up = false;
  }

  hipEvent_t event() {
    {
      std::lock_guard<std::mutex> g(mu_);
      if (!free_events_.empty()) {
        hipEvent_t e = free_events_.back();
        free_events_.pop_back();
        return e;
      }
    }
    hipEvent_t e = nullptr;
    if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return nullptr;
    return e;
  }

  bool post(int peer, int ch, bool send, void* buf, uint64_t n, P2POp* op, std::string* err) {
    Link& l = link(peer);
    hipEvent_t ev = event();
    if (!ev) {
      *err = "hipEventCreate failed";
      return false;
    }
    std::lock_guard<std::mutex> g(l.mu);
    if (!l.up || ch < 0 || ch >= static_cast<int>(l.out.size())) {
      release_event(ev);
      *err = "RCCL channel down";
      return false;
    }
    Chan& c = send ? l.out[ch] : l.in[ch];
    if (!c.comm) {
      release_event(ev);
      *err = "RCCL channel down";
      return false;
    }
    (void)hipSetDevice(device_);
    ncclResult_t r = send ? ncclSend(buf, n, ncclUint8, 1, c.comm, c.stream) : ncclRecv(buf, n, ncclUint8, 0, c.comm, c.stream);
    if (!settle(c.comm, r, Clock::now() + std::chrono::seconds(5), err, send ? "ncclSend" : "ncclRecv") ||
        hipEventRecord(ev, c.stream) != hipSuccess) {
      release_event(ev);
      return false;
    }
    op->event = ev;
    return true;
  }

  void release_event(hipEvent_t e) {
    std::lock_guard<std::mutex> g(mu_);
    free_events_.push_back(e);
  }

  // One 4-byte transfer each way proves both lazily connected channels end to end.
  bool warm_up(Chan& out, Chan& in, Clock::time_point deadline, const std::string& tag, std::string* err) {
    int32_t* probe = nullptr;
    if (hipMalloc(reinterpret_cast<void**>(&probe), 2 * sizeof(int32_t)) != hipSuccess) {
      *err = "hipMalloc failed";
      return false;
    }
    bool ok = settle(out.comm, ncclSend(probe, 1, ncclInt32, 1, out.comm, out.stream), deadline, err,
                     "warm-up send " + tag) &&
              settle(in.comm, ncclRecv(probe + 1, 1, ncclInt32, 0, in.comm, in.stream), deadline, err,
                     "warm-up recv " + tag);
    for (Chan* c : {&out, &in}) {
      while (ok) {
        hipError_t q = hipStreamQuery(c->stream);
        if (q == hipSuccess) break;
        if (q != hipErrorNotReady || Clock::now() > deadline) {
          *err = "warm-up transfer " + tag + " did not complete";
          ok = false;
          break;
        }
        std::this_thread::sleep_for(std::chrono::microseconds(100));
      }
    }
    // on failure the probe may still be a DMA target until the abort lands: leak it
    if (ok) (void)hipFree(probe);
    return ok;
  }

  int device_, rank_, channels_;
  std::mutex mu_;
  std::map<int, std::unique_ptr<Link>> links_;
  std::vector<hipEvent_t> free_events_;
};

}  // namespace

// One-GPU hardware check of the pieces RcclTransport is built from: a NONBLOCKING
// communicator brought up through settle(), a grouped ncclSend/ncclRecv (a 1-rank
// communicator sends to itself; RCCL refuses two ranks on one GPU, so this is the only
// RCCL p2p a 1-GPU box can run), completion observed through a hipEvent as test() does, the
// bytes compared, then ncclCommAbort while a large transfer is still running (close()'s
// path) and a fresh communicator on the same device afterwards (a pair rebuild).
RcclProbe rccl_loopback_probe(int device, uint64_t bytes, uint64_t abort_bytes, int timeout_ms) {
  RcclProbe out;
  auto fail = [&](const std::string& e) {
    out.error = e;
    return out;
  };
  if (hipSetDevice(device) != hipSuccess) return fail("hipSetDevice");
  int ver = 0;
  ncclGetVersion(&ver);
  out.version = ver;
  hipStream_t s = nullptr;
  if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return fail("hipStreamCreate");
  const uint64_t cap = std::max(bytes, abort_bytes);
  uint8_t *src = nullptr, *dst = nullptr;
  if (hipMalloc(reinterpret_cast<void**>(&src), cap) != hipSuccess ||
      hipMalloc(reinterpret_cast<void**>(&dst), cap) != hipSuccess)
    return fail("hipMalloc");
  std::vector<uint8_t> pat(bytes);
  for (uint64_t i = 0; i < bytes; ++i) pat[i] = static_cast<uint8_t>((i * 2654435761u) >> 13);
  (void)hipMemcpy(src, pat.data(), bytes, hipMemcpyHostToDevice);
  (void)hipMemset(dst, 0, cap);
  hipEvent_t ev = nullptr;
  (void)hipEventCreateWithFlags(&ev, hipEventDisableTiming);
  auto comm_up = [&](ncclComm_t* c, const std::string& what) {
    ncclUniqueId id;
    if (ncclGetUniqueId(&id) != ncclSuccess) {
      out.error = "ncclGetUniqueId";
      return false;
    }
    ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
    cfg.blocking = 0;
    auto t0 = Clock::now();
    ncclResult_t r = ncclCommInitRankConfig(c, 1, id, 0, &cfg);
    bool ok = *c != nullptr && settle(*c, r, t0 + std::chrono::milliseconds(timeout_ms), &out.error, what);
    out.init_ms.push_back(std::chrono::duration<double, std::milli>(Clock::now() - t0).count());
    return ok;
  };
  auto self_xfer = [&](ncclComm_t c, uint64_t n, const std::string& what) {
    ncclGroupStart();
    ncclSend(src, n, ncclUint8, 0, c, s);
    ncclRecv(dst, n, ncclUint8, 0, c, s);
    ncclResult_t r = ncclGroupEnd();
    return settle(c, r, Clock::now() + std::chrono::milliseconds(timeout_ms), &out.error, what) &&
           hipEventRecord(ev, s) == hipSuccess;
  };
  auto wait_event = [&](int ms) {
    auto deadline = Clock::now() + std::chrono::milliseconds(ms);
    for (;;) {
      hipError_t q = hipEventQuery(ev);
      if (q == hipSuccess) return true;
      if (q != hipErrorNotReady || Clock::now() > deadline) return false;
      std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
  };
  ncclComm_t comm = nullptr;
  if (!comm_up(&comm, "init")) return out;
  auto t0 = Clock::now();
  if (!self_xfer(comm, bytes, "grouped self send/recv") || !wait_event(timeout_ms)) {
    if (out.error.empty()) out.error = "self transfer did not complete";
    ncclCommAbort(comm);
    return out;
  }
  out.xfer_ms = std::chrono::duration<double, std::milli>(Clock::now() - t0).count();
  std::vector<uint8_t> got(bytes);
  (void)hipMemcpy(got.data(), dst, bytes, hipMemcpyDeviceToHost);
  out.bytes_ok = got == pat;
  if (abort_bytes) {
    // abort with a large transfer in flight: close()'s path; the stream must drain, bounded
    if (!self_xfer(comm, abort_bytes, "large self send/recv")) return out;
    auto ta = Clock::now();
    ncclCommAbort(comm);
    comm = nullptr;
    out.abort_ms = std::chrono::duration<double, std::milli>(Clock::now() - ta).count();
    out.drained_after_abort = wait_event(timeout_ms);
    // a rebuild: a new communicator on the same device carries bytes again
    ncclComm_t again = nullptr;
    (void)hipMemset(dst, 0, bytes);
    if (comm_up(&again, "re-init") && self_xfer(again, bytes, "self send/recv after abort") && wait_event(timeout_ms)) {
      (void)hipMemcpy(got.data(), dst, bytes, hipMemcpyDeviceToHost);
      out.reinit_ok = got == pat;
    }
    if (again) ncclCommDestroy(again);
  } else {
    ncclCommDestroy(comm);
  }
  (void)hipEventDestroy(ev);
  (void)hipFree(src);
  (void)hipFree(dst);
  (void)hipStreamDestroy(s);
  out.ok = out.bytes_ok && (abort_bytes == 0 || (out.drained_after_abort && out.reinit_ok));
  return out;
}

std::unique_ptr<P2PTransport> make_rccl_transport(int device, int rank, int channels, std::string* err) {
  if (device < 0) {
    *err = "RCCL transport requires a GPU";
    return nullptr;
  }
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || device >= n) {
    *err = "no HIP device " + std::to_string(device);
    return nullptr;
  }
  return std::make_unique<RcclTransport>(device, rank, std::max(1, std::min(channels, kMaxP2PChannels)));
}

}  // namespace dfs
