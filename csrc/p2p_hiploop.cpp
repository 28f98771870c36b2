// In-process device P2PTransport for single-GPU tests ("hiploop").
//
// RCCL refuses two ranks on one GPU, and the test boxes have one GPU, so the device half of
// the replication engine (HBM sources pinned in the store, receive extents, per-slice K1
// checksums while a block lands, commit) would otherwise only ever run on an 8-GPU node.
// This transport gives two engines in ONE process (two ChunkStores on the same GPU) the
// exact RCCL p2p contract: per-direction FIFO matching, nonblocking posts, completion via
// events, and ops that never complete until close(). A matched (send, recv) pair becomes a
// hipMemcpyAsync device-to-device copy on the channel's stream.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <deque>
#include <map>
#include <mutex>
#include <tuple>

#include "p2p_transport.h"

namespace dfs {

namespace {

struct Pending {
  void* buf;
  uint64_t n;
  hipEvent_t ev;
  std::shared_ptr<std::atomic<int>> st;
};

struct Chan {
  std::mutex mu;
  std::deque<Pending> sends, recvs;
  hipStream_t stream = nullptr;
  bool open = false;
};

std::mutex g_mu;
std::map<std::tuple<std::string, int, int, int>, std::shared_ptr<Chan>> g_chans;  // (ns, src, dst, channel)

std::shared_ptr<Chan> chan(const std::string& ns, int src, int dst, int ch) {
  std::lock_guard<std::mutex> g(g_mu);
  auto& c = g_chans[{ns, src, dst, ch}];
  if (!c) c = std::make_shared<Chan>();
  return c;
}

class HipLoopTransport final : public P2PTransport {
 public:
  HipLoopTransport(int device, int rank, std::string ns, int channels)
      : device_(device), rank_(rank), ns_(std::move(ns)), channels_(channels) {}
  ~HipLoopTransport() override {
    for (auto& kv : opened_) close(kv.first);
  }
  const char* name() const override { return "hiploop"; }
  bool device_buffers() const override { return true; }
  int channels() const override { return channels_; }

  std::string make_token(int peer, uint64_t gen, std::string*) override {
    return ns_ + "/" + std::to_string(rank_) + "->" + std::to_string(peer) + "@" + std::to_string(gen);
  }

  bool open(int peer, uint64_t, const std::string&, const std::string&, int, std::string*) override {
    (void)hipSetDevice(device_);
    for (int ch = 0; ch < channels_; ++ch)
      for (auto c : {chan(ns_, rank_, peer, ch), chan(ns_, peer, rank_, ch)}) {
        std::lock_guard<std::mutex> g(c->mu);
        if (!c->stream) (void)hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
        c->open = true;
      }
    opened_[peer] = true;
    return true;
  }

  void close(int peer) override {
    for (int ch = 0; ch < channels_; ++ch)
      for (auto c : {chan(ns_, rank_, peer, ch), chan(ns_, peer, rank_, ch)}) {
        std::lock_guard<std::mutex> g(c->mu);
        c->open = false;
        for (auto* q : {&c->sends, &c->recvs}) {
          for (auto& p : *q) p.st->store(-1);
          q->clear();
        }
      }
  }

  bool post_send(int peer, int ch, const void* buf, uint64_t n, P2POp* op, std::string* err) override {
    return post(chan(ns_, rank_, peer, ch), true, const_cast<void*>(buf), n, op, err);
  }
  bool post_recv(int peer, int ch, void* buf, uint64_t n, P2POp* op, std::string* err) override {
    return post(chan(ns_, peer, rank_, ch), false, buf, n, op, err);
  }

  int test(P2POp* op) override {
    int s = op->state ? op->state->load() : -1;
    if (s <= 0) return s;
    hipError_t q = hipEventQuery(static_cast<hipEvent_t>(op->event));
    return q == hipSuccess ? 1 : (q == hipErrorNotReady ? 0 : -1);
  }

  void release(P2POp* op) override {
    if (op->event) (void)hipEventDestroy(static_cast<hipEvent_t>(op->event));
    op->event = nullptr;
    op->state.reset();
  }

 private:
  bool post(const std::shared_ptr<Chan>& c, bool send, void* buf, uint64_t n, P2POp* op, std::string* err) {
    (void)hipSetDevice(device_);
    hipEvent_t ev = nullptr;
    if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) {
      *err = "hipEventCreate failed";
      return false;
    }
    op->event = ev;
    op->state = std::make_shared<std::atomic<int>>(0);
    std::lock_guard<std::mutex> g(c->mu);
    if (!c->open) {
      *err = "hiploop channel down";
      return false;
    }
    auto& mine = send ? c->sends : c->recvs;
    auto& other = send ? c->recvs : c->sends;
    Pending me{buf, n, ev, op->state};
    if (other.empty()) {
      mine.push_back(me);
      return true;
    }
    Pending them = other.front();
    other.pop_front();
    const Pending& s = send ? me : them;
    const Pending& r = send ? them : me;
    if (s.n != r.n) {  // RCCL would fail the communicator: so do we
      s.st->store(-1);
      r.st->store(-1);
      return true;
    }
    if (s.n) (void)hipMemcpyAsync(r.buf, s.buf, s.n, hipMemcpyDeviceToDevice, c->stream);
    (void)hipEventRecord(s.ev, c->stream);
    (void)hipEventRecord(r.ev, c->stream);
    s.st->store(1);
    r.st->store(1);
    return true;
  }

  int device_, rank_;
  std::string ns_;
  int channels_;
  std::map<int, bool> opened_;
};

}  // namespace

std::unique_ptr<P2PTransport> make_hiploop_transport(int device, int rank, const std::string& ns, int channels) {
  return std::make_unique<HipLoopTransport>(device, rank, ns, std::max(1, std::min(channels, kMaxP2PChannels)));
}

}  // namespace dfs
