// Replication engine; design notes in replication.h.
#include "replication.h"

#include <hip/hip_runtime.h>

#include <unistd.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <random>

#include "crc32.h"
#include "trace.h"
#include "thread_name.h"

namespace dfs {

namespace {

using Clock = std::chrono::steady_clock;

uint64_t ns_since(Clock::time_point t0) {
  return static_cast<uint64_t>(std::chrono::duration_cast<std::chrono::nanoseconds>(Clock::now() - t0).count());
}

enum : uint8_t { kOpen = 1, kReopen = 2 };
enum : uint8_t { kOk = 0, kStale = 1, kNotReady = 2, kError = 3 };

template <class T>
void put(std::string& b, T v) {
  b.append(reinterpret_cast<const char*>(&v), sizeof(T));
}
void put_tok(std::string& b, const std::string& t) {
  put<uint16_t>(b, static_cast<uint16_t>(t.size()));
  b += t;
}
struct Rd {
  const char* p;
  const char* e;
  bool ok = true;
  template <class T>
  T get() {
    T v{};
    if (e - p < static_cast<ptrdiff_t>(sizeof(T))) {
      ok = false;
      return v;
    }
    std::memcpy(&v, p, sizeof(T));
    p += sizeof(T);
    return v;
  }
  std::string tok() {
    uint16_t n = get<uint16_t>();
    if (!ok || e - p < n) {
      ok = false;
      return {};
    }
    std::string s(p, n);
    p += n;
    return s;
  }
};

std::string reply(uint8_t status, uint64_t gen, const std::string& tok = {}) {
  std::string r;
  put<uint8_t>(r, status);
  put<uint64_t>(r, gen);
  put_tok(r, tok);
  return r;
}

}  // namespace

std::unique_ptr<P2PTransport> make_transport(const std::string& name, ChunkStore* store, int rank,
                                             const std::string& ns, int channels, std::string* err) {
  if (channels <= 0) {
    const char* e = std::getenv(name == "rccl" ? "DFS_REPL_CHANNELS_RCCL" : "DFS_REPL_CHANNELS");
    // RCCL: K 2-rank communicators per pair direction (each with its own proxy thread and
    // staging buffers: 2*K*(N-1) per process, 28 at N=8 with K=2); hipipc: K rings
    channels = e && *e ? std::atoi(e) : (name == "rccl" ? 2 : 4);
  }
  if (name == "rccl") return make_rccl_transport(store->config().device, rank, channels, err);
  if (name == "socket") return make_socket_transport(rank, ns, channels);
  if (name == "hiploop" && store->gpu()) return make_hiploop_transport(store->config().device, rank, ns, channels);
  if (name == "hipipc" || name == "hipipc-spin") {
    const char* sp = std::getenv("DFS_IPC_SPIN");
    const bool spin = name == "hipipc-spin" || (sp && std::string(sp) == "1");
    // receiver pull (one copy+checksum kernel per hop, on the receiver) unless DFS_IPC_PULL=0
    const char* pe = std::getenv("DFS_IPC_PULL");
    const bool pull = !spin && store->can_pull() && !(pe && std::string(pe) == "0");
    return make_ipc_transport(store->config().device, rank, ns, store->arena_base(), store->arena_bytes(), spin,
                              channels, err, pull);
  }
  *err = "unknown transport " + name;
  return nullptr;
}

ReplicationEngine::ReplicationEngine(ChunkStore* store, std::unique_ptr<P2PTransport> transport, int rank, int world,
                                     ReplOptions opt)
    : store_(store), t_(std::move(transport)), rank_(rank), world_(world), opt_(opt) {
  channels_ = std::max(1, std::min(opt_.channels, t_->channels()));
  // DFS_REPL_MIN_SLICE_KIB: smallest slice of a pipelined transfer, for every transport (A/B
  // of slicing against per-slice overheads)
  if (const char* e = std::getenv("DFS_REPL_MIN_SLICE_KIB")) {
    const uint64_t kib = std::strtoull(e, nullptr, 10);
    if (kib >= kSliceBytes / 1024) opt_.min_slice = opt_.device_min_slice = std::min<uint64_t>(kib << 10, opt_.max_slice);
  }
  for (int i = 0; i < world_; ++i) {
    peers_.push_back(std::make_unique<Peer>());
    reset_seqs_locked(*peers_.back());
  }
  std::random_device rd;
  incarnation_ = (static_cast<uint64_t>(rd()) << 32) ^ rd() ^ static_cast<uint64_t>(::getpid());
}

ReplicationEngine::~ReplicationEngine() { stop(); }

void ReplicationEngine::set_control(ControlFn fn) { control_ = std::move(fn); }

ReplicationEngine::Peer& ReplicationEngine::peer(int p) { return *peers_.at(static_cast<size_t>(p)); }

void ReplicationEngine::reset_seqs_locked(Peer& P) {
  P.send_seq.assign(channels_, 0);
  P.post_next.assign(channels_, 0);
  P.recv_next.assign(channels_, 0);
  P.load.assign(channels_, 0);
}

void ReplicationEngine::unload(ReplTicket* t) {
  if (!t->loaded) return;
  Peer& P = peer(t->peer);
  std::lock_guard<std::mutex> lk(P.mu);
  // a rebuilt pair started its loads afresh: a ticket of an older generation counts nowhere
  if (P.gen == t->gen && t->ch >= 0 && t->ch < static_cast<int>(P.load.size()) && P.load[t->ch] > 0) P.load[t->ch]--;
  t->loaded = false;
}

void ReplicationEngine::spawn(std::function<void()> fn) {
  {
    std::lock_guard<std::mutex> g(threads_mu_);
    live_threads_++;
  }
  std::thread([this, fn = std::move(fn)] {
    name_thread("repl-ctl");
    fn();
    std::lock_guard<std::mutex> g(threads_mu_);
    if (--live_threads_ == 0) threads_cv_.notify_all();
  }).detach();
}

void ReplicationEngine::start() {
  for (int p = rank_ + 1; p < world_; ++p) {
    Peer& P = peer(p);
    std::lock_guard<std::mutex> g(P.mu);
    if (P.opener) continue;
    P.opener = true;
    spawn([this, p] { opener_loop(p); });
  }
  // Lower ranks open their pairs with us. If we are a restarted process, they may still
  // believe the old pair is up (nothing failed on their side yet): announce the fresh start
  // until each of them has opened a new generation with us.
  for (int p = 0; p < rank_; ++p) spawn([this, p] { request_reopen(p, 0, true); });
}

void ReplicationEngine::request_reopen(int p, uint64_t g, bool fresh) {
  int backoff = 50;
  while (!stop_.load()) {
    {
      Peer& Q = peer(p);
      std::lock_guard<std::mutex> lk(Q.mu);
      if (Q.gen != g || (Q.state != State::Broken && Q.state != State::Down)) return;  // already reopened
    }
    std::string req, rep;
    put<uint8_t>(req, kReopen);
    put<int32_t>(req, rank_);
    put<uint64_t>(req, g);
    put<uint8_t>(req, fresh ? 1 : 0);
    put<uint64_t>(req, incarnation_);
    if (control_ && control_(p, req, &rep) && !fresh) return;
    for (int w = 0; w < backoff && !stop_.load(); w += 10) std::this_thread::sleep_for(std::chrono::milliseconds(10));
    backoff = std::min(backoff * 2, 1000);
  }
}

void ReplicationEngine::stop() {
  if (stop_.exchange(true)) return;
  for (auto& P : peers_) {
    std::lock_guard<std::mutex> g(P->mu);
    P->cv.notify_all();
  }
  std::unique_lock<std::mutex> lk(threads_mu_);
  threads_cv_.wait(lk, [this] { return live_threads_ == 0; });
  lk.unlock();
  for (int p = 0; p < world_; ++p) {
    if (p == rank_) continue;
    t_->close(p);
    // shutting down: nothing of ours will receive again, the store outlives the engine
    std::vector<std::pair<uint64_t, DevExtent>> left;
    {
      std::lock_guard<std::mutex> g(peer(p).mu);
      left.swap(peer(p).parked);
    }
    for (auto& pe : left) store_->release(pe.second);
  }
}

void ReplicationEngine::park(int p, uint64_t gen, const DevExtent& e) {
  Peer& P = peer(p);
  {
    std::lock_guard<std::mutex> lk(P.mu);
    P.parked.emplace_back(gen, e);
  }
  {
    std::lock_guard<std::mutex> lk(st_mu_);
    st_.parked_extents++;
  }
  reap(p);  // the pair may already be up again on a newer generation
}

void ReplicationEngine::reap(int p) {
  Peer& P = peer(p);
  std::vector<DevExtent> free_now;
  {
    std::lock_guard<std::mutex> lk(P.mu);
    if (P.state != State::Up) return;
    for (size_t i = 0; i < P.parked.size();) {
      if (P.parked[i].first < P.gen) {
        free_now.push_back(P.parked[i].second);
        P.parked[i] = P.parked.back();
        P.parked.pop_back();
      } else {
        ++i;
      }
    }
  }
  if (free_now.empty()) return;
  for (auto& e : free_now) store_->release(e);
  std::lock_guard<std::mutex> lk(st_mu_);
  st_.reaped_extents += free_now.size();
}

int ReplicationEngine::wait_ready(int timeout_ms, int give_up_after) {
  auto deadline = Clock::now() + std::chrono::milliseconds(timeout_ms);
  int up = 0;
  for (int p = 0; p < world_; ++p) {
    if (p == rank_) continue;
    Peer& P = peer(p);
    std::unique_lock<std::mutex> lk(P.mu);
    P.cv.wait_until(lk, deadline, [&] {
      return stop_.load() || P.state == State::Up || (give_up_after > 0 && P.failed_opens >= give_up_after);
    });
    if (P.state == State::Up) ++up;
  }
  return up;
}

bool ReplicationEngine::pair_ok(int p) {
  if (p < 0 || p >= world_ || p == rank_) return false;
  Peer& P = peer(p);
  std::lock_guard<std::mutex> g(P.mu);
  return P.state == State::Up;
}

uint64_t ReplicationEngine::generation(int p) {
  Peer& P = peer(p);
  std::lock_guard<std::mutex> g(P.mu);
  return P.gen;
}

uint64_t ReplicationEngine::slice_for(uint64_t n) const {
  const uint64_t mn = t_->device_buffers() ? opt_.device_min_slice : opt_.min_slice;
  uint64_t s = std::min(std::max(n / 4, mn), opt_.max_slice);
  s = (s + kSliceBytes - 1) / kSliceBytes * kSliceBytes;
  uint64_t whole = (n + kSliceBytes - 1) / kSliceBytes * kSliceBytes;
  return std::max<uint64_t>(kSliceBytes, std::min(s, whole));
}

ReplStats ReplicationEngine::stats() {
  std::lock_guard<std::mutex> g(st_mu_);
  return st_;
}

// ------------------------------------------------------------------ pair lifecycle
void ReplicationEngine::opener_loop(int p) {
  if (t_->device_buffers()) (void)hipSetDevice(store_->config().device);
  int backoff_ms = 50;
  Peer& P = peer(p);
  while (!stop_.load()) {
    uint64_t g;
    {
      std::lock_guard<std::mutex> lk(P.mu);
      g = P.gen + 1;
      P.gen = g;
      P.state = State::Opening;
      reset_seqs_locked(P);
      P.cv.notify_all();
    }
    t_->close(p);
    {
      std::lock_guard<std::mutex> lk(st_mu_);
      st_.open_attempts++;
    }
    std::string err, rep;
    std::string tok = t_->make_token(p, g, &err);
    bool ok = !tok.empty() && control_;
    if (ok) {
      std::string req;
      put<uint8_t>(req, kOpen);
      put<int32_t>(req, rank_);
      put<uint64_t>(req, g);
      put_tok(req, tok);
      ok = control_(p, req, &rep);
      if (!ok) err = "peer unreachable";
    }
    bool retry_now = false;
    if (ok) {
      Rd rd{rep.data(), rep.data() + rep.size()};
      uint8_t st = rd.get<uint8_t>();
      uint64_t their = rd.get<uint64_t>();
      std::string peer_tok = rd.tok();
      uint64_t peer_inc = rd.p < rd.e ? rd.get<uint64_t>() : 0;
      if (rd.ok && st == kOk) {
        std::lock_guard<std::mutex> lk(P.mu);
        P.peer_inc = peer_inc;
      }
      if (!rd.ok || st != kOk) {
        ok = false;
        err = st == kStale ? "stale generation" : (st == kNotReady ? "peer not ready" : "peer refused");
        if (st == kStale) {
          std::lock_guard<std::mutex> lk(P.mu);
          P.gen = std::max(P.gen, their);  // restart above the peer's generation
          retry_now = true;
        }
      } else {
        ok = t_->open(p, g, tok, peer_tok, opt_.open_timeout_ms, &err);
      }
    }
    {
      std::lock_guard<std::mutex> lk(P.mu);
      if (P.gen == g) {
        P.state = ok ? State::Up : State::Broken;
        P.last_error = err;
      }
      if (ok) P.opener = false;
      else P.failed_opens++;
      P.cv.notify_all();
    }
    if (ok) {
      {
        std::lock_guard<std::mutex> lk(st_mu_);
        st_.pair_opens++;
      }
      reap(p);
      return;
    }
    t_->close(p);
    if (retry_now) continue;
    for (int waited = 0; waited < backoff_ms && !stop_.load(); waited += 10)
      std::this_thread::sleep_for(std::chrono::milliseconds(10));
    backoff_ms = std::min(backoff_ms * 2, 2000);
  }
  std::lock_guard<std::mutex> lk(P.mu);
  P.opener = false;
}

std::string ReplicationEngine::handle_control(const std::string& req) {
  Rd rd{req.data(), req.data() + req.size()};
  uint8_t kind = rd.get<uint8_t>();
  int32_t from = rd.get<int32_t>();
  uint64_t g = rd.get<uint64_t>();
  std::string tok = kind == kOpen ? rd.tok() : std::string();
  bool fresh = kind == kReopen && rd.p < rd.e && rd.get<uint8_t>() == 1;
  uint64_t inc = kind == kReopen && rd.p < rd.e ? rd.get<uint64_t>() : 0;
  if (!rd.ok || from < 0 || from >= world_ || from == rank_) return reply(kError, 0);
  if (stop_.load()) return reply(kNotReady, 0);
  Peer& P = peer(from);
  if (kind == kReopen) {
    // the higher rank saw generation g fail; we (the initiator) rebuild it
    bool start = false;
    {
      std::lock_guard<std::mutex> lk(P.mu);
      // not ours to open, or a late request about an older generation (a restarted peer
      // announces itself with `fresh`: its generation restarts at 0, ours must be rebuilt)
      if (from < rank_ || (g < P.gen && !fresh)) return reply(kOk, P.gen);
      if (P.opener) return reply(kOk, P.gen);  // a rebuild is already under way
      // a start-up announcement from the very process we are paired with: nothing to redo
      if (fresh && P.state == State::Up && P.peer_inc == inc) return reply(kOk, P.gen);
      if (P.state == State::Up) P.state = State::Broken;
      if (!P.opener) {
        P.opener = true;
        start = true;
      }
      P.cv.notify_all();
    }
    if (start) {
      t_->close(from);
      spawn([this, from] { opener_loop(from); });
    }
    return reply(kOk, g);
  }
  if (kind != kOpen || from > rank_) return reply(kError, 0);  // only the lower rank opens
  {
    std::lock_guard<std::mutex> lk(P.mu);
    if (g <= P.gen) return reply(kStale, P.gen);
    P.gen = g;
    P.state = State::Opening;
    reset_seqs_locked(P);
    P.cv.notify_all();  // receivers waiting under the old generation fail now
  }
  t_->close(from);
  std::string err;
  std::string mine = t_->make_token(from, g, &err);
  if (mine.empty()) {
    std::lock_guard<std::mutex> lk(P.mu);
    if (P.gen == g) P.state = State::Broken;
    return reply(kError, g);
  }
  spawn([this, from, g, mine, tok] {
    if (t_->device_buffers()) (void)hipSetDevice(store_->config().device);
    std::string e;
    bool ok = t_->open(from, g, mine, tok, opt_.open_timeout_ms, &e);
    Peer& Q = peer(from);
    std::unique_lock<std::mutex> lk(Q.mu);
    if (Q.gen == g) {
      Q.state = ok ? State::Up : State::Broken;
      Q.last_error = e;
    }
    if (!ok) Q.failed_opens++;
    Q.cv.notify_all();
    if (ok) {
      std::lock_guard<std::mutex> sg(st_mu_);
      st_.pair_opens++;
    }
    lk.unlock();
    if (ok) reap(from);
  });
  std::string r = reply(kOk, g, mine);
  put<uint64_t>(r, incarnation_);
  return r;
}

void ReplicationEngine::fail_pair(int p, const std::string& why) {
  if (p < 0 || p >= world_ || p == rank_) return;
  uint64_t g;
  {
    std::lock_guard<std::mutex> lk(peer(p).mu);
    g = peer(p).gen;
  }
  fail_pair_gen(p, g, why);
}

void ReplicationEngine::fail_pair_gen(int p, uint64_t gen, const std::string& why) {
  if (p < 0 || p >= world_ || p == rank_) return;
  Peer& P = peer(p);
  uint64_t g;
  bool start = false;
  {
    std::lock_guard<std::mutex> lk(P.mu);
    // already failed / being rebuilt, or the failure belongs to an older generation
    if (P.state != State::Up || P.gen != gen) return;
    P.state = State::Broken;
    P.last_error = why;
    g = P.gen;
    if (rank_ < p && !P.opener) {
      P.opener = true;
      start = true;
    }
    P.cv.notify_all();
  }
  {
    std::lock_guard<std::mutex> lk(st_mu_);
    st_.pair_failures++;
  }
  t_->close(p);  // pending ops of this generation end now (RCCL: ncclCommAbort)
  if (start) {
    spawn([this, p] { opener_loop(p); });
  } else if (rank_ > p) {
    // ask the initiator to rebuild; keep asking until it does (or we stop)
    spawn([this, p, g] { request_reopen(p, g, false); });
  }
}

// ------------------------------------------------------------------ data
bool ReplicationEngine::send(int p, const std::string& id, const uint8_t* host_src, uint64_t n, ReplTicket* t,
                             std::string* err, const StagedSource* staged,
                             const std::function<bool(const ReplTicket&)>& announce) {
  TraceRange tr("dfs.repl.send");
  t->peer = p;
  t->id = id;
  const uint8_t* src = host_src;
  if (staged && (!t_->device_buffers() || !staged->dev || !staged->done || staged->slice == 0 ||
                 staged->done->size() != (n + staged->slice - 1) / staged->slice)) {
    *err = "staged send needs a device transport and one event per slice";
    return false;
  }
  if (staged) {
    (void)hipSetDevice(store_->config().device);
    src = staged->dev;  // not indexed yet: the caller holds the extent
  } else if (t_->device_buffers()) {
    (void)hipSetDevice(store_->config().device);
    uint64_t size = 0;
    src = store_->pin_device(id, &size);
    if (!src) {
      *err = "block not resident: " + id;
      return false;
    }
    t->pinned = true;
    n = size;
  } else if (!src && n) {
    *err = "no host source for " + id;
    return false;
  }
  t->size = n;
  t->slice = staged ? staged->slice : slice_for(n);
  Peer& P = peer(p);
  const auto deadline = Clock::now() + std::chrono::milliseconds(opt_.xfer_timeout_ms);
  // slice k of a staged block: wait (bounded) until the head's copy of it reached HBM
  auto landed = [&](uint64_t k) {
    hipEvent_t ev = (*staged->done)[k];
    for (int spins = 0;; ++spins) {
      hipError_t q = hipEventQuery(ev);
      if (q == hipSuccess) return true;
      if (q != hipErrorNotReady || Clock::now() > deadline) return false;
      if (spins < 64) std::this_thread::yield();
      else std::this_thread::sleep_for(std::chrono::microseconds(5));
    }
  };
  bool failed = false, up = false;
  const auto t0 = Clock::now();
  // a staged block's first slice must be in HBM before the block takes a place in the pair's
  // FIFO: the sequence number is reserved only then, so a transfer whose PCIe staging is still
  // queued (10 writers share the copy engines) does not hold up the transfers behind it. With
  // the number taken first, every send to a peer waited for the slowest staging ahead of it:
  // the 2-rank rehearsal spent 3.2 ms per write in the forward even without a flush (hbm-ack).
  if (staged && n && !landed(0)) {
    *err = "staging of slice 0 did not complete";
    if (t->pinned) store_->unpin(id);
    t->pinned = false;
    return false;
  }
  {
    // only the sequence number is taken under the pair lock; the descriptor write and the
    // slice posts (which may wait for the head's staging) run outside it, so a slow peer
    // socket or a slow PCIe copy never blocks fail_pair_gen / reap / handle_control or the
    // generation checks of other transfers
    std::lock_guard<std::mutex> lk(P.mu);
    if (P.state != State::Up) {
      *err = "pair " + std::to_string(rank_) + "->" + std::to_string(p) + " is not up";
    } else {
      up = true;
      t->gen = P.gen;
      // the least-loaded channel (ties: round robin), so a transfer queues behind as few
      // others as possible
      int best = -1;
      for (int i = 0; i < channels_; ++i) {
        const int c = (P.rr + i) % channels_;
        if (best < 0 || P.load[c] < P.load[best]) best = c;
      }
      P.rr = (best + 1) % channels_;
      t->ch = best;
      t->seq = P.send_seq[best]++;
      P.load[best]++;
      t->loaded = true;
    }
  }
  const uint64_t stage_ns = ns_since(t0);
  uint64_t turn_ns = 0;
  if (up) {
    // each channel is FIFO: transfers post in their channel's sequence order
    const auto t1 = Clock::now();
    {
      std::unique_lock<std::mutex> lk(P.mu);
      if (P.post_next[t->ch] != t->seq) {
        std::lock_guard<std::mutex> sg(st_mu_);
        st_.channel_waits++;
      }
      const bool turn = P.cv.wait_until(lk, deadline, [&] {
        return P.gen != t->gen || P.state != State::Up || P.post_next[t->ch] == t->seq;
      });
      if (!turn || P.gen != t->gen || P.state != State::Up) {
        *err = "pair " + std::to_string(rank_) + "->" + std::to_string(p) + " changed before the send was posted";
        failed = true;  // the sequence number is spent: the pair cannot stay in step
      }
    }
    turn_ns = ns_since(t1);
    if (!failed && announce && !announce(*t)) {
      *err = "descriptor to rank " + std::to_string(p) + " failed";
      failed = true;
    }
    for (uint64_t off = 0; !failed && off < n; off += t->slice) {
      P2POp op;
      if (staged && !landed(off / t->slice)) {
        *err = "staging of slice " + std::to_string(off / t->slice) + " did not complete";
        failed = true;
        break;
      }
      if (!t_->post_send(p, t->ch, src + off, std::min(t->slice, n - off), &op, err)) {
        failed = true;
        break;
      }
      t->ops.push_back(op);
    }
    {
      std::lock_guard<std::mutex> lk(P.mu);
      if (P.gen == t->gen && P.post_next[t->ch] == t->seq) P.post_next[t->ch]++;
      P.cv.notify_all();
    }
    {
      std::lock_guard<std::mutex> sg(st_mu_);
      st_.send_calls++;
      st_.send_stage_ns += stage_ns;
      st_.send_turn_ns += turn_ns;
      st_.send_post_ns += ns_since(t0) - stage_ns - turn_ns;
    }
    if (!failed) return true;  // the pin is held until wait_send / cancel_send
  }
  unload(t);
  for (auto& op : t->ops) t_->release(&op);
  t->ops.clear();
  if (failed) fail_pair_gen(p, t->gen, "post_send failed: " + *err);
  if (t->pinned) store_->unpin(id);
  t->pinned = false;
  return false;
}

bool ReplicationEngine::wait_send(ReplTicket* t, std::string* err) {
  TraceRange tr("dfs.repl.wait_send");
  Peer& P = peer(t->peer);
  const auto t0 = Clock::now();
  auto deadline = t0 + std::chrono::milliseconds(opt_.xfer_timeout_ms);
  bool ok = true;
  int spins = 0;
  for (auto& op : t->ops) {
    for (;;) {
      int r = t_->test(&op);
      if (r == 1) break;
      if (r < 0) {
        ok = false;
        *err = "send failed";
        break;
      }
      if ((++spins & 63) == 0 || spins > 64) {
        std::lock_guard<std::mutex> lk(P.mu);
        if (P.gen != t->gen || P.state != State::Up) {
          ok = false;
          *err = "pair failed during send";
          break;
        }
      }
      if (Clock::now() > deadline) {
        ok = false;
        *err = "send timed out";
        break;
      }
      // a short spin for the common sub-100 us copy, then sleep in the transport (futex)
      if (spins < 64) std::this_thread::yield();
      else if (t_->wait(&op, 2000) != 0) continue;
    }
    if (!ok) break;
  }
  if (!ok) fail_pair_gen(t->peer, t->gen, *err);  // abort before unpinning: no DMA reads a freed extent
  unload(t);
  for (auto& op : t->ops) t_->release(&op);
  t->ops.clear();
  if (t->pinned) store_->unpin(t->id);
  t->pinned = false;
  if (ok) {
    std::lock_guard<std::mutex> lk(st_mu_);
    st_.bytes_sent += t->size;
    st_.blocks_sent++;
    st_.wait_send_ns += ns_since(t0);
    st_.sent_to[t->peer] += t->size;
  }
  return ok;
}

void ReplicationEngine::cancel_send(ReplTicket* t, const std::string& why) {
  fail_pair_gen(t->peer, t->gen, why);
  unload(t);
  for (auto& op : t->ops) t_->release(&op);
  t->ops.clear();
  if (t->pinned) store_->unpin(t->id);
  t->pinned = false;
}

WriteResult ReplicationEngine::recv(int src, uint64_t gen, int ch, int64_t seq, const std::string& id, uint64_t size,
                                    uint64_t slice, uint32_t expected_crc, bool persist_now) {
  TraceRange tr("dfs.repl.recv");
  WriteResult res;
  if (src < 0 || src >= world_ || src == rank_) {
    res.error = "bad source rank";
    return res;
  }
  if (ch < 0 || ch >= channels_) {
    res.error = "bad channel";
    fail_pair_gen(src, gen, res.error);  // the peers disagree on the channel count
    return res;
  }
  if (size && (slice == 0 || slice % kSliceBytes != 0)) {
    res.error = "bad slice size";
    fail_pair_gen(src, gen, res.error);
    return res;
  }
  const bool dev = t_->device_buffers();
  if (dev) (void)hipSetDevice(store_->config().device);
  Peer& P = peer(src);
  DevExtent ext;
  std::vector<uint8_t> host;
  if (dev) {
    ext = store_->reserve(size);
    if (ext.off < 0) {
      res.error = "HBM arena full";
      fail_pair_gen(src, gen, res.error);  // the matching send can never be consumed now
      return res;
    }
  } else {
    host.resize(size);
  }
  uint8_t* dst = dev ? ext.ptr : host.data();
  std::vector<P2POp> ops;
  // receiver pull: our kernels move and checksum the slices as the sender offers them, so
  // the receive's .meta scratch exists before the first slice is posted
  ChunkStore::RecvVerify rv;
  const bool pull = dev && t_->pulls_from(src);
  if (pull && !store_->recv_begin(&rv, ext, size, true, persist_now)) {
    res.error = "no pinned scratch for a pulled receive";
    store_->release(ext);
    fail_pair_gen(src, gen, res.error);  // the sender's offer can never be consumed now
    return res;
  }
  const auto t0 = Clock::now();
  {
    std::unique_lock<std::mutex> lk(P.mu);
    // a descriptor may overtake our side of a bring-up (the sender saw the pair up first):
    // an Opening pair of the same generation is waited for like a sequence turn
    bool turn = P.cv.wait_for(lk, std::chrono::milliseconds(opt_.turn_timeout_ms), [&] {
      return stop_.load() || P.gen != gen || P.state == State::Broken || P.state == State::Down ||
             (P.state == State::Up && P.recv_next[ch] >= seq);
    });
    std::string why;
    bool fail = false;
    if (P.gen != gen) {
      why = "stale pair generation " + std::to_string(gen) + " (now " + std::to_string(P.gen) + ")";
      std::lock_guard<std::mutex> sg(st_mu_);
      st_.stale_generation++;
    } else if ((P.state != State::Up && P.state != State::Opening) || stop_.load()) {
      why = "pair down";
    } else if (!turn) {
      why = "receive turn timeout at seq " + std::to_string(seq) + " of channel " + std::to_string(ch) + " (next " +
            std::to_string(P.recv_next[ch]) + ")";
      fail = true;
      std::lock_guard<std::mutex> sg(st_mu_);
      st_.turn_timeouts++;
    } else if (P.recv_next[ch] != seq) {
      why = "sequence " + std::to_string(seq) + " already consumed";
      fail = true;
    } else {
      std::string err;
      for (uint64_t off = 0; off < size; off += slice) {
        P2POp op;
        const uint64_t len = std::min(slice, size - off);
        if (pull ? !t_->post_recv_pull(src, ch, len, store_->recv_pull(&rv, off, off + len), &op, &err)
                 : !t_->post_recv(src, ch, dst + off, len, &op, &err)) {
          why = "post_recv failed: " + err;
          fail = true;
          break;
        }
        ops.push_back(op);
      }
      if (!fail) {
        P.recv_next[ch]++;
        P.cv.notify_all();
      }
    }
    if (!why.empty()) {
      lk.unlock();
      if (pull) store_->recv_abandon(&rv);
      for (auto& op : ops) t_->release(&op);
      if (fail) fail_pair_gen(src, gen, why);
      // an extent that a posted receive may still write into waits for the pair's rebuild
      if (dev && ops.empty()) store_->release(ext);
      else if (dev) park(src, gen, ext);
      res.error = why;
      return res;
    }
  }
  const auto t1 = Clock::now();
  if (dev && !pull) store_->recv_begin(&rv, ext, size);
  auto deadline = Clock::now() + std::chrono::milliseconds(opt_.xfer_timeout_ms);
  std::string why;
  int spins = 0;
  for (size_t s = 0; s < ops.size() && why.empty(); ++s) {
    for (;;) {
      int r = t_->test(&ops[s]);
      if (r == 1) break;
      if (r < 0) {
        why = "receive failed";
        break;
      }
      if ((++spins & 63) == 0 || spins > 64) {
        std::lock_guard<std::mutex> lk(P.mu);
        if (P.gen != gen || P.state != State::Up) {
          why = "pair failed during receive";
          break;
        }
      }
      if (Clock::now() > deadline) {
        why = "receive timed out";
        break;
      }
      if (spins < 64) std::this_thread::yield();
      else if (t_->wait(&ops[s], 2000) != 0) continue;
    }
    // slice s landed: checksum it on the lane while s+1.. are still on the link (pulled
    // slices were checksummed by the kernel that moved them)
    if (why.empty() && dev && !pull) store_->recv_slice(&rv, s * slice, std::min(size, (s + 1) * slice));
  }
  for (auto& op : ops) t_->release(&op);
  if (!why.empty()) {
    if (dev) store_->recv_abandon(&rv);
    fail_pair_gen(src, gen, why);
    if (dev) park(src, gen, ext);
    res.error = why;
    return res;
  }
  const auto t2 = Clock::now();
  res = dev ? store_->recv_finish(&rv, id, expected_crc, persist_now) : store_->write(id, host.data(), size, expected_crc);
  if (res.ok) {
    std::lock_guard<std::mutex> lk(st_mu_);
    st_.recv_calls++;
    st_.recv_turn_ns += static_cast<uint64_t>(std::chrono::duration_cast<std::chrono::nanoseconds>(t1 - t0).count());
    st_.recv_land_ns += static_cast<uint64_t>(std::chrono::duration_cast<std::chrono::nanoseconds>(t2 - t1).count());
    st_.recv_finish_ns += ns_since(t2);
    st_.bytes_recv += size;
    st_.blocks_recv++;
    st_.recv_from[src] += size;
  }
  return res;
}

}  // namespace dfs
