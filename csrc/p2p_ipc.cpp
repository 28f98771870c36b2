// HIP-IPC implementation of P2PTransport ("hipipc"): the device transport between the
// ChunkServer PROCESSES of one node (contract in p2p_transport.h).
//
// Why not RCCL p2p for this traffic. RCCL's ncclSend/ncclRecv run as kernels that wait on
// the device for their peer. The replication engine keeps many blocks in flight in both
// directions of every pair, on 2*(N-1) channel streams plus the store's lanes, and HIP
// multiplexes those streams onto GPU_MAX_HW_QUEUES (4) hardware queues in order. A receive
// kernel parked at the head of a queue then holds everything queued behind it — including
// the send its own peer is waiting for — and with crossing traffic those waits can close a
// cycle across processes. The channel-level proof in replication.h cannot see that coupling.
//
// This transport keeps every wait on the host, so no kernel ever waits for a peer:
//  * Each rank exports its HBM arena (one hipMalloc) with hipIpcGetMemHandle; the peer maps
//    it once per pair generation (xGMI peer mapping between GPUs, plain HBM when the ranks
//    share one GPU).
//  * Each directed channel (`channels` per direction of a pair, each with its own ring, copy
//    stream, host worker and sequence space) has a ring in /dev/shm created by the RECEIVER: post_recv writes
//    (offset in its arena, length) into slot k and bumps `posted` — the credit.
//  * The SENDER's channel worker matches its k-th posted send with slot k, checks the length
//    (RCCL fails a mismatched pair, so do we), and queues one copy-engine hipMemcpyAsync of
//    the slice straight into the receiver's extent on the channel stream. When the copy's
//    event completes it publishes `landed` = k + 1. A copy never waits for anything, so a
//    hardware queue can hold it only for the copy's own duration.
//  * The receiver's op k completes when `landed` > k (the engine then checksums the slice on
//    a store lane while later slices are still in flight, exactly as with RCCL).
//  * close() raises `abort` on both rings, stops the worker and drains the channel stream
//    (copies always finish), so when it returns no copy of that generation can still land.
//
// Pull mode (make_ipc_transport(..., pull=true): the replication engine asks for it when the
// store runs the matrix-core CRC kernels; DFS_IPC_PULL=0 turns it off) inverts the copy: the
// sender only OFFERS each slice (its offset in the sender's arena) on the ring, and the
// receiver's worker launches one kernel that reads the slice from the peer's mapped arena
// (over xGMI between GPUs), stores it into the posted extent, and writes the slice CRCs (the
// .meta image) to HBM and to pinned host memory (crc_write_copy_kernel, the same kernel that
// takes a client's write over PCIe). That replaces the sender's copy kernel plus the
// receiver's separate checksum pass on arrival: one kernel per hop, no readback. When the
// kernel's event completes the receiver publishes `landed`, which completes both sides' ops.
// The receiver decides per direction (its waves must reach the peer's memory) and tells the
// sender through its inbound ring's `pull` word before its warm-up is published.
//
// Spin mode (make_ipc_transport(..., spin=true); DFS_IPC_SPIN=1) is the RCCL emulation used
// to test the engine against the hazard above: post_send launches a kernel that parks on the
// send stream until the credit appears and then copies with the whole grid; post_recv
// launches a kernel that parks on the receive stream until the bytes landed
// (p2p_kernels.hip). Every such wait is bounded by the device wall clock (DFS_IPC_SPIN_MS)
// and by the abort word, so a kernel whose peer never comes still exits.
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <linux/futex.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <climits>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <map>
#include <mutex>
#include <thread>
#include <vector>

#include "p2p_kernels.h"
#include "p2p_transport.h"
#include "thread_name.h"

namespace dfs {

namespace {

using Clock = std::chrono::steady_clock;

constexpr uint64_t kRingMagic = 0x474e495243504944ull;  // "DIPCRING"
constexpr char kTokMagic[8] = {'D', 'F', 'S', 'I', 'P', 'C', '2', '\0'};
constexpr int kMaxRanks = 64;
constexpr size_t kProbeBytes = 2 * kMaxRanks * 64;  // [0,4096) mailbox per sender; [4096,8192) our patterns

struct TokenWire {
  char magic[8];
  int32_t rank, device, pid;
  uint32_t spin;
  uint64_t gen;
  hipIpcMemHandle_t arena;
  uint64_t arena_bytes;
  hipIpcMemHandle_t probe;
  uint32_t channels;
  uint32_t pad;
  char ring[96];  // shm name prefix of the creator's INBOUND rings (`<prefix>_c<k>`, one per channel)
};

long futex(uint32_t* addr, int op, uint32_t val, const timespec* ts) {
  return ::syscall(SYS_futex, addr, op, val, ts, nullptr, 0);
}

template <class T>
T ld(const T* p) {
  return __atomic_load_n(p, __ATOMIC_ACQUIRE);
}
template <class T>
void st(T* p, T v) {
  __atomic_store_n(p, v, __ATOMIC_RELEASE);
}

// Receivers blocked in wait() sleep on landed_bell; the sender bumps it after publishing
// `landed` (and every abort does), waking only when someone is registered as waiting.
void landed_wake(IpcRing* r) {
  __atomic_fetch_add(&r->landed_bell, 1u, __ATOMIC_SEQ_CST);
  if (__atomic_load_n(&r->landed_waiters, __ATOMIC_SEQ_CST)) futex(&r->landed_bell, FUTEX_WAKE, INT_MAX, nullptr);
}

void ring_wake(IpcRing* r) {
  __atomic_fetch_add(&r->doorbell, 1u, __ATOMIC_SEQ_CST);
  futex(&r->doorbell, FUTEX_WAKE, INT_MAX, nullptr);
  if (__atomic_load_n(&r->abort, __ATOMIC_SEQ_CST)) landed_wake(r);
}

// A send op's completion word (process-local): set, then wake a blocked wait().
void finish_send(const std::shared_ptr<std::atomic<int>>& st, int v) {
  st->store(v, std::memory_order_release);
  ::syscall(SYS_futex, reinterpret_cast<uint32_t*>(st.get()), FUTEX_WAKE_PRIVATE, INT_MAX, nullptr, nullptr, 0);
}

// One process's mapping of a channel ring, registered for device access (spin kernels).
struct RingMap {
  IpcRing* r = nullptr;
  IpcRing* dev = nullptr;
  size_t bytes = 0;
  std::string name;
  bool owner = false;
  ~RingMap() {
    if (dev) (void)hipHostUnregister(r);
    if (r) ::munmap(r, bytes);
    if (owner && !name.empty()) ::shm_unlink(name.c_str());
  }
};

std::shared_ptr<RingMap> map_ring(const std::string& name, bool create, uint64_t gen, std::string* err) {
  const size_t bytes = (sizeof(IpcRing) + 4095) / 4096 * 4096;
  if (create) ::shm_unlink(name.c_str());
  int fd = ::shm_open(name.c_str(), create ? (O_RDWR | O_CREAT | O_EXCL) : O_RDWR, 0600);
  if (fd < 0) {
    *err = "shm_open " + name + ": " + std::strerror(errno);
    return nullptr;
  }
  if (create && ::ftruncate(fd, static_cast<off_t>(bytes)) != 0) {
    *err = "ftruncate " + name + ": " + std::strerror(errno);
    ::close(fd);
    ::shm_unlink(name.c_str());
    return nullptr;
  }
  struct stat sb {};
  if (::fstat(fd, &sb) != 0 || static_cast<size_t>(sb.st_size) < bytes) {
    *err = "ring " + name + " too small";
    ::close(fd);
    return nullptr;
  }
  void* p = ::mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  ::close(fd);
  if (p == MAP_FAILED) {
    *err = std::string("mmap ring: ") + std::strerror(errno);
    if (create) ::shm_unlink(name.c_str());
    return nullptr;
  }
  auto m = std::make_shared<RingMap>();
  m->r = static_cast<IpcRing*>(p);
  m->bytes = bytes;
  m->name = name;
  m->owner = create;
  if (create) {
    std::memset(p, 0, bytes);
    m->r->gen = gen;
    m->r->receiver_pid = ::getpid();
    st(&m->r->magic, kRingMagic);
  } else if (ld(&m->r->magic) != kRingMagic || m->r->gen != gen) {
    *err = "ring " + name + " is not generation " + std::to_string(gen);
    return nullptr;
  }
  void* dev = nullptr;
  if (hipHostRegister(p, bytes, hipHostRegisterMapped) == hipSuccess &&
      hipHostGetDevicePointer(&dev, p, 0) == hipSuccess) {
    m->dev = static_cast<IpcRing*>(dev);
  } else {
    (void)hipGetLastError();
    *err = "hipHostRegister of ring " + name + " failed";
    return nullptr;
  }
  return m;
}

struct SendItem {
  const uint8_t* src = nullptr;
  uint64_t n = 0;
  uint64_t seq = 0;
  std::shared_ptr<std::atomic<int>> st;
  hipEvent_t ev = nullptr;
};

// A receive in pull mode: matched with the sender's seq-th offer, then launched.
struct PullItem {
  uint64_t n = 0;
  uint64_t seq = 0;
  P2PTransport::PullLaunch launch;
  hipEvent_t ev = nullptr;
};

class IpcTransport final : public P2PTransport {
 public:
  IpcTransport(int device, int rank, std::string ns, uint8_t* arena, uint64_t arena_bytes, bool spin, int channels,
               bool pull)
      : device_(device), rank_(rank), ns_(std::move(ns)), arena_(arena), arena_bytes_(arena_bytes), spin_(spin),
        channels_(channels), pull_(pull && !spin) {
    const char* ms = std::getenv("DFS_IPC_SPIN_MS");
    spin_ticks_ = wall_ticks_per_ms(device) * static_cast<uint64_t>(ms ? std::max(1, std::atoi(ms)) : 5000);
  }

  bool init(std::string* err) {
    if (rank_ < 0 || rank_ >= kMaxRanks) {
      *err = "hipipc supports ranks 0.." + std::to_string(kMaxRanks - 1);
      return false;
    }
    (void)hipSetDevice(device_);
    if (hipIpcGetMemHandle(&arena_h_, arena_) != hipSuccess) {
      *err = std::string("hipIpcGetMemHandle(arena): ") + hipGetErrorString(hipGetLastError());
      return false;
    }
    if (hipMalloc(reinterpret_cast<void**>(&probe_), kProbeBytes) != hipSuccess ||
        hipMemset(probe_, 0, kProbeBytes) != hipSuccess || hipIpcGetMemHandle(&probe_h_, probe_) != hipSuccess) {
      *err = "probe buffer / IPC handle failed";
      return false;
    }
    return true;
  }

  ~IpcTransport() override {
    std::vector<int> peers;
    {
      std::lock_guard<std::mutex> g(mu_);
      for (auto& kv : links_) peers.push_back(kv.first);
    }
    for (int p : peers) close(p);
    (void)hipSetDevice(device_);
    std::lock_guard<std::mutex> g(mu_);
    for (auto& kv : links_)
      for (auto& c : kv.second->ch) {
        for (hipStream_t s : {c->send_stream, c->recv_stream})
          if (s) (void)hipStreamDestroy(s);
        if (c->done_ctr) (void)hipFree(c->done_ctr);
      }
    for (hipEvent_t e : free_events_) (void)hipEventDestroy(e);
    if (probe_) (void)hipFree(probe_);
  }

  const char* name() const override { return spin_ ? "hipipc-spin" : "hipipc"; }
  bool device_buffers() const override { return true; }
  int channels() const override { return channels_; }

  // our inbound rings for the pair, one per channel: the token carries their name prefix
  std::string make_token(int peer, uint64_t gen, std::string* err) override {
    if (peer < 0 || peer >= kMaxRanks) {
      *err = "peer rank out of range";
      return {};
    }
    const std::string prefix = "/dfs_ipc_" + ns_ + "_" + std::to_string(rank_) + "_" + std::to_string(peer) + "_" +
                               std::to_string(gen) + "_" + std::to_string(::getpid());
    std::vector<std::shared_ptr<RingMap>> rings;
    for (int c = 0; c < channels_; ++c) {
      auto ring = map_ring(prefix + "_c" + std::to_string(c), true, gen, err);
      if (!ring) return {};
      rings.push_back(ring);
    }
    {
      std::lock_guard<std::mutex> g(mu_);
      made_[peer] = {gen, std::move(rings)};
    }
    TokenWire t{};
    std::memcpy(t.magic, kTokMagic, sizeof t.magic);
    t.rank = rank_;
    t.device = device_;
    t.pid = ::getpid();
    t.spin = spin_ ? 1 : 0;
    t.gen = gen;
    t.arena = arena_h_;
    t.arena_bytes = arena_bytes_;
    t.probe = probe_h_;
    t.channels = static_cast<uint32_t>(channels_);
    std::snprintf(t.ring, sizeof t.ring, "%s", prefix.c_str());
    return std::string(reinterpret_cast<const char*>(&t), sizeof t);
  }

  bool open(int peer, uint64_t gen, const std::string& /*tok_out*/, const std::string& tok_in, int timeout_ms,
            std::string* err) override {
    if (tok_in.size() != sizeof(TokenWire)) {
      *err = "malformed hipipc token";
      return false;
    }
    TokenWire tw;
    std::memcpy(&tw, tok_in.data(), sizeof tw);
    if (std::memcmp(tw.magic, kTokMagic, sizeof tw.magic) != 0 || tw.gen != gen || tw.rank != peer) {
      *err = "hipipc token does not match the pair";
      return false;
    }
    if ((tw.spin != 0) != spin_) {
      *err = "hipipc peers disagree on spin mode";
      return false;
    }
    if (static_cast<int>(tw.channels) != channels_) {
      *err = "hipipc peers disagree on the channel count";
      return false;
    }
    (void)hipSetDevice(device_);
    Link& l = link(peer);
    std::lock_guard<std::mutex> g(l.mu);
    teardown_locked(l);
    std::vector<std::shared_ptr<RingMap>> ins;
    {
      std::lock_guard<std::mutex> mg(mu_);
      auto it = made_.find(peer);
      if (it == made_.end() || it->second.first != gen) {
        *err = "no inbound ring for generation " + std::to_string(gen);
        return false;
      }
      ins = std::move(it->second.second);
      made_.erase(it);
    }
    tw.ring[sizeof tw.ring - 1] = '\0';
    while (static_cast<int>(l.ch.size()) < channels_) l.ch.push_back(std::make_unique<Lane>());
    for (int c = 0; c < channels_; ++c) {
      Lane& ln = *l.ch[c];
      ln.in = ins[c];
      ln.out = map_ring(std::string(tw.ring) + "_c" + std::to_string(c), false, gen, err);
      if (!ln.out) return fail_open(l, err);
      for (hipStream_t* st : {&ln.send_stream, &ln.recv_stream})
        if (!*st && hipStreamCreateWithFlags(st, hipStreamNonBlocking) != hipSuccess) {
          *err = "hipStreamCreate failed";
          return fail_open(l, err);
        }
      if (!ln.done_ctr && hipMalloc(reinterpret_cast<void**>(&ln.done_ctr), sizeof(uint32_t)) != hipSuccess) {
        *err = "hipMalloc failed";
        return fail_open(l, err);
      }
      (void)hipMemsetAsync(ln.done_ctr, 0, sizeof(uint32_t), ln.send_stream);
      ln.send_seq = ln.recv_seq = 0;
    }
    void* pa = nullptr;
    if (hipIpcOpenMemHandle(&pa, tw.arena, hipIpcMemLazyEnablePeerAccess) != hipSuccess) {
      *err = std::string("hipIpcOpenMemHandle(peer arena): ") + hipGetErrorString(hipGetLastError());
      return fail_open(l, err);
    }
    l.peer_arena = static_cast<uint8_t*>(pa);
    l.peer_arena_bytes = tw.arena_bytes;
    void* pp = nullptr;
    if (hipIpcOpenMemHandle(&pp, tw.probe, hipIpcMemLazyEnablePeerAccess) != hipSuccess) {
      *err = std::string("hipIpcOpenMemHandle(peer probe): ") + hipGetErrorString(hipGetLastError());
      return fail_open(l, err);
    }
    l.peer_probe = static_cast<uint8_t*>(pp);
    l.gen = gen;
    // slices are copied by kernel when this device reaches the peer's memory (the same
    // device, or a peer the runtime reports accessible over xGMI); else by the copy engines
    {
      int can = 0;
      l.kernel_copy = tw.device == device_ ||
                      (hipDeviceCanAccessPeer(&can, device_, tw.device) == hipSuccess && can != 0);
      (void)hipGetLastError();
    }
    for (auto& c : l.ch) {
      // our receives from this peer are pulled by our kernels when our waves reach its
      // memory; published before our warm-up, which the peer waits for before reading it
      c->i_pull = pull_ && l.kernel_copy;
      st(&c->in->r->pull, c->i_pull ? 1u : 0u);
      st(&c->in->r->receiver_ready, 1u);
      st(&c->out->r->sender_attached, 1u);
    }
    // warm-up: 64 bytes each way through the peer's exported probe, proving the IPC mapping
    // and the copy path (the same kernel or copy-engine copy the slices take) end to end
    // before the pair is declared up (channel 0's stream and
    // ring; the other channels' rings were mapped above and checked for the generation)
    Lane& c0 = *l.ch[0];
    uint64_t pat[8] = {kRingMagic, gen, static_cast<uint64_t>(rank_), static_cast<uint64_t>(peer), 0, 0, 0, 0};
    uint8_t* mine = probe_ + kMaxRanks * 64 + peer * 64;
    if (hipMemcpyAsync(mine, pat, sizeof pat, hipMemcpyHostToDevice, c0.send_stream) != hipSuccess ||
        copy(l.peer_probe + rank_ * 64, mine, sizeof pat, c0.send_stream, l.kernel_copy) != hipSuccess ||
        hipStreamSynchronize(c0.send_stream) != hipSuccess) {
      *err = "warm-up copy failed";
      return fail_open(l, err);
    }
    st(&c0.out->r->warm, gen);
    ring_wake(c0.out->r);
    auto deadline = Clock::now() + std::chrono::milliseconds(timeout_ms);
    while (ld(&c0.in->r->warm) != gen) {
      if (Clock::now() > deadline || ld(&c0.in->r->abort)) {
        *err = "peer never delivered its warm-up copy";
        return fail_open(l, err);
      }
      std::this_thread::sleep_for(std::chrono::microseconds(200));
    }
    uint64_t got[8] = {};
    if (hipMemcpy(got, probe_ + peer * 64, sizeof got, hipMemcpyDeviceToHost) != hipSuccess || got[0] != kRingMagic ||
        got[1] != gen || got[2] != static_cast<uint64_t>(peer) || got[3] != static_cast<uint64_t>(rank_)) {
      *err = "warm-up bytes did not arrive intact";
      return fail_open(l, err);
    }
    for (auto& c : l.ch) {
      // both sides attached: the ring's name can go (the mappings stay)
      ::shm_unlink(c->in->name.c_str());
      c->in->owner = false;
      c->peer_pulls = !spin_ && ld(&c->out->r->pull) != 0;  // the peer's warm-up came after it
      if (!spin_) {
        c->stop.store(false);
        if (!c->peer_pulls)
          c->worker = std::thread([this, lp = &l, cp = c.get(), out = c->out] {
            name_thread("ipc-chan");
            worker(lp, cp, out);
          });
        if (c->i_pull)
          c->rworker = std::thread([this, lp = &l, cp = c.get(), in = c->in] {
            name_thread("ipc-pull");
            pull_worker(lp, cp, in);
          });
      }
    }
    l.up = true;
    return true;
  }

  void close(int peer) override {
    Link& l = link(peer);
    std::lock_guard<std::mutex> g(l.mu);
    teardown_locked(l);
  }

  bool post_send(int peer, int ch, const void* buf, uint64_t n, P2POp* op, std::string* err) override {
    Link& l = link(peer);
    std::lock_guard<std::mutex> g(l.mu);
    if (!l.up || ch < 0 || ch >= static_cast<int>(l.ch.size())) {
      *err = "hipipc channel down";
      return false;
    }
    Lane& c = *l.ch[ch];
    const uint64_t seq = c.send_seq++;
    op->ctx = c.out;
    op->seq = seq;
    if (spin_) {
      (void)hipSetDevice(device_);
      IpcSendArgs a{&c.out->dev->posted, &c.out->dev->landed, &c.out->dev->abort, c.out->dev->slots, seq,
                    static_cast<const uint8_t*>(buf), l.peer_arena, l.peer_arena_bytes, n, c.done_ctr, spin_ticks_};
      hipEvent_t ev = event();
      if (!ev || launch_ipc_send(a, send_grid(n), c.send_stream) != hipSuccess ||
          hipEventRecord(ev, c.send_stream) != hipSuccess) {
        if (ev) release_event(ev);
        *err = "spin send launch failed";
        return false;
      }
      op->event = ev;
      return true;
    }
    if (c.peer_pulls) {
      // offer the slice: the receiver's kernel reads it from our arena; the op completes
      // when the receiver publishes `landed` past it
      const auto* p = static_cast<const uint8_t*>(buf);
      IpcRing* r = c.out->r;
      if (p < arena_ || static_cast<uint64_t>(p - arena_) > arena_bytes_ || n > arena_bytes_ - (p - arena_)) {
        *err = "send buffer outside the exported arena";
        st(&r->abort, 1u);  // the sequence number is spent: the channel cannot stay in step
        ring_wake(r);
        return false;
      }
      if (seq - ld(&r->landed) >= kIpcRing) {
        *err = "hipipc ring full";
        st(&r->abort, 1u);
        ring_wake(r);
        return false;
      }
      IpcSlot& s = r->offers[seq % kIpcRing];
      __atomic_store_n(&s.off, static_cast<uint64_t>(p - arena_), __ATOMIC_RELAXED);
      __atomic_store_n(&s.n, n, __ATOMIC_RELAXED);
      st(&r->offered, seq + 1);
      ring_wake(r);
      return true;
    }
    op->state = std::make_shared<std::atomic<int>>(0);
    {
      std::lock_guard<std::mutex> q(c.qmu);
      c.pending.push_back(SendItem{static_cast<const uint8_t*>(buf), n, seq, op->state, nullptr});
    }
    ring_wake(c.out->r);
    return true;
  }

  bool pulls_from(int peer) override {
    Link& l = link(peer);
    std::lock_guard<std::mutex> g(l.mu);
    return l.up && !l.ch.empty() && l.ch[0]->i_pull;
  }

  bool post_recv_pull(int peer, int ch, uint64_t n, PullLaunch launch, P2POp* op, std::string* err) override {
    Link& l = link(peer);
    std::lock_guard<std::mutex> g(l.mu);
    if (!l.up || ch < 0 || ch >= static_cast<int>(l.ch.size()) || !l.ch[ch]->i_pull) {
      *err = "hipipc pull channel down";
      return false;
    }
    Lane& c = *l.ch[ch];
    IpcRing* r = c.in->r;
    const uint64_t seq = c.recv_seq;
    if (seq - ld(&r->landed) >= kIpcRing) {
      *err = "hipipc ring full";
      return false;
    }
    c.recv_seq++;
    {
      std::lock_guard<std::mutex> q(c.rqmu);
      c.rpending.push_back(PullItem{n, seq, std::move(launch), nullptr});
    }
    op->ctx = c.in;
    op->seq = seq;
    ring_wake(r);
    return true;
  }

  bool post_recv(int peer, int ch, void* buf, uint64_t n, P2POp* op, std::string* err) override {
    Link& l = link(peer);
    std::lock_guard<std::mutex> g(l.mu);
    if (!l.up || ch < 0 || ch >= static_cast<int>(l.ch.size())) {
      *err = "hipipc channel down";
      return false;
    }
    Lane& c = *l.ch[ch];
    auto* p = static_cast<uint8_t*>(buf);
    if (p < arena_ || static_cast<uint64_t>(p - arena_) > arena_bytes_ || n > arena_bytes_ - (p - arena_)) {
      *err = "receive buffer outside the exported arena";
      return false;
    }
    IpcRing* r = c.in->r;
    const uint64_t seq = c.recv_seq;
    if (seq - ld(&r->landed) >= kIpcRing) {
      *err = "hipipc ring full";
      return false;
    }
    c.recv_seq++;
    IpcSlot& s = r->slots[seq % kIpcRing];
    __atomic_store_n(&s.off, static_cast<uint64_t>(p - arena_), __ATOMIC_RELAXED);
    __atomic_store_n(&s.n, n, __ATOMIC_RELAXED);
    st(&r->posted, seq + 1);  // the credit: the slot is visible before the count
    ring_wake(r);
    op->ctx = c.in;
    op->seq = seq;
    if (spin_) {
      (void)hipSetDevice(device_);
      hipEvent_t ev = event();
      if (!ev || launch_ipc_wait(&c.in->dev->landed, seq + 1, &c.in->dev->abort, spin_ticks_, c.recv_stream) !=
                     hipSuccess ||
          hipEventRecord(ev, c.recv_stream) != hipSuccess) {
        if (ev) release_event(ev);
        st(&r->abort, 1u);  // the credit is out but its waiter is not: the channel is unusable
        *err = "spin wait launch failed";
        return false;
      }
      op->event = ev;
    }
    return true;
  }

  int test(P2POp* op) override {
    if (op->state && !spin_) return op->state->load(std::memory_order_acquire);
    auto* rm = static_cast<RingMap*>(op->ctx.get());
    if (!rm) return -1;
    if (op->event) {
      hipError_t q = hipEventQuery(static_cast<hipEvent_t>(op->event));
      if (q == hipErrorNotReady) return 0;
      if (q != hipSuccess) return -1;
      return ld(&rm->r->landed) > op->seq ? 1 : -1;  // the kernel ended: landed, or gave up
    }
    if (ld(&rm->r->landed) > op->seq) return 1;
    return ld(&rm->r->abort) ? -1 : 0;
  }

  // Blocking completion for the host-driven mode: a send op sleeps on its completion word
  // (the channel worker wakes it), a receive op on the ring's landed_bell (the peer's worker
  // wakes it after publishing `landed`, or on abort). Spin-mode ops poll their event.
  int wait(P2POp* op, int max_us) override {
    int r = test(op);
    if (r != 0 || spin_ || op->event) return r == 0 ? P2PTransport::wait(op, max_us) : r;
    timespec ts{max_us / 1000000, static_cast<long>(max_us % 1000000) * 1000};
    if (op->state) {
      ::syscall(SYS_futex, reinterpret_cast<uint32_t*>(op->state.get()), FUTEX_WAIT_PRIVATE, 0u, &ts, nullptr, 0);
      return test(op);
    }
    auto* rm = static_cast<RingMap*>(op->ctx.get());
    if (!rm) return -1;
    IpcRing* ring = rm->r;
    __atomic_fetch_add(&ring->landed_waiters, 1u, __ATOMIC_SEQ_CST);
    const uint32_t bell = __atomic_load_n(&ring->landed_bell, __ATOMIC_SEQ_CST);
    if (test(op) == 0) futex(&ring->landed_bell, FUTEX_WAIT, bell, &ts);
    __atomic_fetch_sub(&ring->landed_waiters, 1u, __ATOMIC_SEQ_CST);
    return test(op);
  }

  void release(P2POp* op) override {
    if (op->event) release_event(static_cast<hipEvent_t>(op->event));
    op->event = nullptr;
    op->ctx.reset();
    op->state.reset();
  }

 private:
  // One channel of a pair: its two rings (in: we receive, our ring; out: we send, the peer's
  // ring), its copy stream and host worker, its own sequence space.
  struct Lane {
    std::shared_ptr<RingMap> in, out;
    hipStream_t send_stream = nullptr, recv_stream = nullptr;
    uint32_t* done_ctr = nullptr;
    uint64_t send_seq = 0, recv_seq = 0;
    std::mutex qmu;
    std::deque<SendItem> pending;
    std::thread worker;
    std::atomic<bool> stop{false};
    bool i_pull = false;      // our receives on this channel are pulled by our kernels
    bool peer_pulls = false;  // the peer pulls our sends: post_send only offers
    std::mutex rqmu;
    std::deque<PullItem> rpending;  // pull receives not launched yet (rqmu)
    std::thread rworker;
  };
  struct Link {
    std::mutex mu;  // open / close / post
    bool up = false;
    uint64_t gen = 0;
    uint8_t* peer_arena = nullptr;
    uint64_t peer_arena_bytes = 0;
    uint8_t* peer_probe = nullptr;
    bool kernel_copy = false;  // this device's waves may store into the peer's mapping
    std::vector<std::unique_ptr<Lane>> ch;
  };

  Link& link(int peer) {
    std::lock_guard<std::mutex> g(mu_);
    auto& l = links_[peer];
    if (!l) l = std::make_unique<Link>();
    return *l;
  }

  static int send_grid(uint64_t n) {
    uint64_t g = n / (256 * 16 * 4);
    return static_cast<int>(std::min<uint64_t>(64, std::max<uint64_t>(1, g)));
  }

  bool fail_open(Link& l, std::string* /*err*/) {
    teardown_locked(l);
    return false;
  }

  // Abort every ring, stop the workers, drain the streams (copies finish; spin kernels see
  // the abort), unmap the peer. When this returns nothing of the old generation can land.
  void teardown_locked(Link& l) {
    (void)hipSetDevice(device_);
    for (auto& c : l.ch)
      for (auto* m : {c->in.get(), c->out.get()})
        if (m) {
          st(&m->r->abort, 1u);
          ring_wake(m->r);
        }
    for (auto& c : l.ch) {
      if (c->worker.joinable()) {
        c->stop.store(true);
        if (c->out) ring_wake(c->out->r);
        c->worker.join();
      }
      if (c->rworker.joinable()) {
        c->stop.store(true);
        if (c->in) ring_wake(c->in->r);
        c->rworker.join();
      }
      {
        std::lock_guard<std::mutex> q(c->qmu);
        for (auto& it : c->pending) finish_send(it.st, -1);
        c->pending.clear();
      }
      {
        std::lock_guard<std::mutex> q(c->rqmu);
        c->rpending.clear();  // never launched: their ops fail on the abort
      }
      for (hipStream_t s : {c->send_stream, c->recv_stream})
        if (s) (void)hipStreamSynchronize(s);
    }
    if (l.peer_arena) (void)hipIpcCloseMemHandle(l.peer_arena);
    if (l.peer_probe) (void)hipIpcCloseMemHandle(l.peer_probe);
    l.peer_arena = l.peer_probe = nullptr;
    for (auto& c : l.ch) {
      c->in.reset();
      c->out.reset();
      c->i_pull = c->peer_pulls = false;
    }
    l.up = false;
  }

  // Host-driven sender of one channel: match posted sends with the receiver's credits in
  // order, queue the copies, publish `landed` as their events complete (in order: one stream).
  void worker(Link* l, Lane* c, std::shared_ptr<RingMap> out) {
    (void)hipSetDevice(device_);
    IpcRing* r = out->r;
    std::deque<SendItem> inflight;
    int idle = 0;
    bool dead = false;
    while (!c->stop.load() && !dead) {
      bool progress = false;
      for (;;) {
        SendItem it;
        {
          std::lock_guard<std::mutex> q(c->qmu);
          if (c->pending.empty() || ld(&r->posted) <= c->pending.front().seq) break;
          it = c->pending.front();
          c->pending.pop_front();
        }
        const IpcSlot& s = r->slots[it.seq % kIpcRing];
        const uint64_t off = __atomic_load_n(&s.off, __ATOMIC_RELAXED), n = __atomic_load_n(&s.n, __ATOMIC_RELAXED);
        hipEvent_t ev = nullptr;
        if (n != it.n || off > l->peer_arena_bytes || n > l->peer_arena_bytes - off || ld(&r->abort) ||
            (n && copy(l->peer_arena + off, it.src, n, c->send_stream, l->kernel_copy) != hipSuccess) ||
            !(ev = event()) || hipEventRecord(ev, c->send_stream) != hipSuccess) {
          if (ev) release_event(ev);
          finish_send(it.st, -1);
          st(&r->abort, 1u);  // mismatched sizes or a failed copy end the channel (as RCCL would)
          ring_wake(r);
          dead = true;
          break;
        }
        __atomic_fetch_add(&r->enqueued, 1ull, __ATOMIC_RELAXED);
        it.ev = ev;
        inflight.push_back(it);
        progress = true;
      }
      while (!inflight.empty()) {
        hipError_t q = hipEventQuery(inflight.front().ev);
        if (q == hipErrorNotReady) break;
        SendItem& it = inflight.front();
        if (q == hipSuccess) {
          st(&r->landed, it.seq + 1);
          landed_wake(r);
          finish_send(it.st, 1);
        } else {
          finish_send(it.st, -1);
          st(&r->abort, 1u);
          landed_wake(r);
          dead = true;
        }
        release_event(it.ev);
        inflight.pop_front();
        progress = true;
      }
      if (ld(&r->abort)) break;
      if (progress) {
        idle = 0;
        continue;
      }
      if (!inflight.empty()) {  // a copy is on the link: poll its event
        if (++idle < 64) std::this_thread::yield();
        else std::this_thread::sleep_for(std::chrono::microseconds(10));
        continue;
      }
      // nothing to do: sleep until a send is posted here or a credit arrives from the peer
      const uint32_t bell = __atomic_load_n(&r->doorbell, __ATOMIC_ACQUIRE);
      {
        std::lock_guard<std::mutex> q(c->qmu);
        if (!c->pending.empty() && ld(&r->posted) > c->pending.front().seq) continue;
      }
      timespec ts{0, 2'000'000};
      futex(&r->doorbell, FUTEX_WAIT, bell, &ts);
    }
    // stopping: the queued copies still finish (nothing can cancel a DMA); their ops fail
    for (auto& it : inflight) {
      (void)hipEventSynchronize(it.ev);
      finish_send(it.st, -1);
      release_event(it.ev);
    }
  }

  // Receiver of one channel in pull mode: match posted receives with the sender's offers in
  // order, launch each one's copy+checksum kernel on the channel's receive stream, and
  // publish `landed` as their events complete (in order: one stream). A launch sees the
  // peer's bytes only after the offer, and `landed` is published only while the channel is
  // not aborted, checked after the kernel finished: a sender that gave up (abort, then
  // unpinning its extent) cannot have a receive completed over bytes it no longer owned.
  void pull_worker(Link* l, Lane* c, std::shared_ptr<RingMap> in) {
    (void)hipSetDevice(device_);
    IpcRing* r = in->r;
    std::deque<PullItem> inflight;
    int idle = 0;
    bool dead = false;
    auto kill = [&] {
      st(&r->abort, 1u);
      ring_wake(r);
      landed_wake(r);
      dead = true;
    };
    while (!c->stop.load() && !dead) {
      bool progress = false;
      for (;;) {
        PullItem it;
        {
          std::lock_guard<std::mutex> q(c->rqmu);
          if (c->rpending.empty() || ld(&r->offered) <= c->rpending.front().seq) break;
          it = std::move(c->rpending.front());
          c->rpending.pop_front();
        }
        const IpcSlot& s = r->offers[it.seq % kIpcRing];
        const uint64_t off = __atomic_load_n(&s.off, __ATOMIC_RELAXED), n = __atomic_load_n(&s.n, __ATOMIC_RELAXED);
        hipEvent_t ev = nullptr;
        if (n != it.n || off > l->peer_arena_bytes || n > l->peer_arena_bytes - off || ld(&r->abort) ||
            (n && it.launch(l->peer_arena + off, c->recv_stream) != 0) || !(ev = event()) ||
            hipEventRecord(ev, c->recv_stream) != hipSuccess) {
          if (ev) release_event(ev);
          kill();  // mismatched sizes or a failed launch end the channel (as RCCL would)
          inflight.push_back(std::move(it));  // a launch that did queue work drains below
          break;
        }
        __atomic_fetch_add(&r->enqueued, 1ull, __ATOMIC_RELAXED);
        it.ev = ev;
        inflight.push_back(std::move(it));
        progress = true;
      }
      while (!dead && !inflight.empty()) {
        hipError_t q = hipEventQuery(inflight.front().ev);
        if (q == hipErrorNotReady) break;
        PullItem& it = inflight.front();
        if (q == hipSuccess && !__atomic_load_n(&r->abort, __ATOMIC_SEQ_CST)) {
          st(&r->landed, it.seq + 1);
          landed_wake(r);
        } else {
          kill();
          break;
        }
        release_event(it.ev);
        inflight.pop_front();
        progress = true;
      }
      if (dead || ld(&r->abort)) break;
      if (progress) {
        idle = 0;
        continue;
      }
      if (!inflight.empty()) {
        if (++idle < 64) std::this_thread::yield();
        else std::this_thread::sleep_for(std::chrono::microseconds(10));
        continue;
      }
      const uint32_t bell = __atomic_load_n(&r->doorbell, __ATOMIC_ACQUIRE);
      {
        std::lock_guard<std::mutex> q(c->rqmu);
        if (!c->rpending.empty() && ld(&r->offered) > c->rpending.front().seq) continue;
      }
      timespec ts{0, 2'000'000};
      futex(&r->doorbell, FUTEX_WAIT, bell, &ts);
    }
    // stopping: kernels already queued finish (they read the peer's mapping, which stays
    // until teardown unmaps it after this); their receives fail on the abort
    (void)hipStreamSynchronize(c->recv_stream);
    for (auto& it : inflight)
      if (it.ev) release_event(it.ev);
  }

  // One slice into the peer's extent: by kernel (default), or by the copy engines
  // (DFS_IPC_COPY=sdma, the round-4 path), or by the engines when the pointers are not
  // 16-byte aligned or the peer's memory is not reachable from this device's waves.
  static hipError_t copy(uint8_t* dst, const uint8_t* src, uint64_t n, hipStream_t s, bool kernel_ok) {
    static const bool sdma = [] {
      const char* e = std::getenv("DFS_IPC_COPY");
      return e && std::string(e) == "sdma";
    }();
    if (!sdma && kernel_ok && (reinterpret_cast<uintptr_t>(dst) | reinterpret_cast<uintptr_t>(src)) % 16 == 0)
      return launch_ipc_copy(dst, src, n, s);
    return hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToDevice, s);
  }

  hipEvent_t event() {
    {
      std::lock_guard<std::mutex> g(ev_mu_);
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
  void release_event(hipEvent_t e) {
    std::lock_guard<std::mutex> g(ev_mu_);
    free_events_.push_back(e);
  }

  int device_, rank_;
  std::string ns_;
  uint8_t* arena_;
  uint64_t arena_bytes_;
  bool spin_;
  int channels_;
  bool pull_;
  uint64_t spin_ticks_ = 0;
  hipIpcMemHandle_t arena_h_{}, probe_h_{};
  uint8_t* probe_ = nullptr;
  std::mutex mu_;
  std::map<int, std::unique_ptr<Link>> links_;
  // inbound rings (one per channel) awaiting open()
  std::map<int, std::pair<uint64_t, std::vector<std::shared_ptr<RingMap>>>> made_;
  std::mutex ev_mu_;
  std::vector<hipEvent_t> free_events_;
};

}  // namespace

std::unique_ptr<P2PTransport> make_ipc_transport(int device, int rank, const std::string& ns, uint8_t* arena,
                                                 uint64_t arena_bytes, bool spin, int channels, std::string* err,
                                                 bool pull) {
  if (device < 0 || arena == nullptr || arena_bytes == 0) {
    *err = "hipipc transport requires a GPU chunk store";
    return nullptr;
  }
  auto t = std::make_unique<IpcTransport>(device, rank, ns, arena, arena_bytes, spin,
                                          std::max(1, std::min(channels, kMaxP2PChannels)), pull);
  if (!t->init(err)) return nullptr;
  return t;
}

}  // namespace dfs
