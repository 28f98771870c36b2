// Point-to-point byte channels between the ChunkServer ranks of one node — the transport
// under chain/fan-out replication (replication.h).
//
// Contract (what RCCL p2p gives us, and what the CPU test transport reproduces):
//  * between two ranks each direction (a->b, b->a) has `channels()` independent FIFO
//    channels (round 5: several per direction, so one slow transfer — a slice still being
//    staged, a large block — does not hold up the pair's other transfers);
//  * transfers on one channel are matched strictly in post order: the k-th post_send on
//    channel c of a->b lands in the buffer of b's k-th post_recv on channel c from a, and
//    sizes must agree; different channels never wait for each other;
//  * posts never block; completion is observed with test(); an op whose peer never posts
//    the matching op never completes — only close() (ncclCommAbort) ends it;
//  * a channel pair is brought up for a generation by open() on BOTH ranks with the
//    same tokens: the sender of each channel creates its token (make_token) and ships it
//    to the peer over the control plane (the fast-path socket).
//
// Implementations:
//  * RcclTransport  (p2p_rccl.cpp): one 2-rank nonblocking communicator + HIP stream per
//    channel and direction; buffers are HBM pointers of our GPU, each op records a hipEvent.
//  * IpcTransport   (p2p_ipc.cpp): HIP IPC between processes of one node; the receiver
//    publishes each posted buffer (an offset in its exported arena) on a shared-memory ring,
//    the sender's copy kernel writes the slice there and bumps the ring's landed count; or,
//    in pull mode, the sender offers the slice and the receiver's copy+checksum kernel reads it. No
//    kernel ever waits on a peer, so no hardware queue can be held by a peer (see p2p_ipc.cpp).
//  * SocketTransport (p2p_socket.cpp): a UNIX stream socket per direction and a worker
//    thread per direction draining the FIFO of posted ops; buffers are host memory. It is
//    what the multi-process CPU tests run (tests/test_replication.py), so every rule of the
//    replication protocol (sequencing, bounded waits, generations, rebuild) is exercised
//    without GPUs; it also carries fault hooks (drop / stall a channel).
#pragma once
#include <atomic>
#include <chrono>
#include <cstdint>
#include <functional>
#include <memory>
#include <string>
#include <thread>
#include <vector>

namespace dfs {

struct P2POp {
  void* event = nullptr;                        // RCCL: hipEvent_t recorded after the op
  std::shared_ptr<std::atomic<int>> state;      // socket: 0 pending, 1 done, -1 failed
  std::shared_ptr<void> ctx;                    // hipipc: the channel ring the op completes on
  uint64_t seq = 0;                             // hipipc: position of the op on its channel
};

class P2PTransport {
 public:
  virtual ~P2PTransport() = default;
  virtual const char* name() const = 0;
  virtual bool device_buffers() const = 0;  // true: buffers are device (HBM) pointers
  virtual int channels() const = 0;         // independent FIFO channels per direction of a pair

  // Token for the channel rank->peer of generation `gen` (we are its sender). Opaque bytes.
  virtual std::string make_token(int peer, uint64_t gen, std::string* err) = 0;
  // Bring up both channels with `peer`: `tok_out` (ours, rank->peer), `tok_in` (the peer's,
  // peer->rank). Both ranks call it concurrently; returns once both channels passed a
  // warm-up transfer, or false at the deadline.
  virtual bool open(int peer, uint64_t gen, const std::string& tok_out, const std::string& tok_in, int timeout_ms,
                    std::string* err) = 0;
  // Abort both channels with `peer`: pending ops fail or never complete; no waiting.
  virtual void close(int peer) = 0;

  // `ch` in [0, channels()): the channel of the pair the op is matched on
  virtual bool post_send(int peer, int ch, const void* buf, uint64_t n, P2POp* op, std::string* err) = 0;
  virtual bool post_recv(int peer, int ch, void* buf, uint64_t n, P2POp* op, std::string* err) = 0;
  virtual int test(P2POp* op) = 0;  // 1 done, 0 pending, -1 failed
  // test(), but a pending op may block the caller for up to `max_us` first (a futex or event
  // wait where the transport has one, so the engine's waiters sleep instead of polling).
  virtual int wait(P2POp* op, int max_us) {
    int r = test(op);
    if (r != 0) return r;
    std::this_thread::sleep_for(std::chrono::microseconds(max_us < 20 ? max_us : 20));
    return test(op);
  }
  virtual void release(P2POp* op) = 0;

  // Receiver pull (hipipc with DFS_IPC_PULL, the default where this device's waves reach the
  // peer's memory): the receiver moves the bytes itself, with a kernel that also checksums
  // what it moves, instead of the sender's copy plus a separate checksum pass on arrival.
  // pulls_from(peer): the receives from `peer` must be posted with post_recv_pull. `launch`
  // runs on the transport's receive worker once the matching send is offered, with the
  // sender's bytes (a device pointer into the peer's mapped arena) and the channel's stream
  // (a hipStream_t); the op completes once the work it queued there finished. The closure
  // must own what it references: it can outlive the receive that posted it (an abandoned
  // receive's launch may still run until close()).
  using PullLaunch = std::function<int(const uint8_t* src, void* stream)>;  // 0 = queued
  virtual bool pulls_from(int /*peer*/) { return false; }
  virtual bool post_recv_pull(int /*peer*/, int /*ch*/, uint64_t /*n*/, PullLaunch /*launch*/, P2POp* /*op*/,
                              std::string* err) {
    *err = "transport has no receiver pull";
    return false;
  }

  // Test hooks (socket transport only; no-ops elsewhere): the next `n` sends to `peer`
  // vanish (never delivered), or the channel to `peer` stalls for `ms`.
  virtual void debug_drop_sends(int /*peer*/, int /*n*/) {}
  virtual void debug_stall(int /*peer*/, int /*ms*/) {}
};

struct RcclProbe {
  bool ok = false, bytes_ok = false, drained_after_abort = false, reinit_ok = false;
  int version = 0;
  double xfer_ms = 0, abort_ms = 0;
  std::vector<double> init_ms;
  std::string error;
};
// 1-GPU hardware check of RcclTransport's building blocks (p2p_rccl.cpp).
RcclProbe rccl_loopback_probe(int device, uint64_t bytes, uint64_t abort_bytes, int timeout_ms);

constexpr int kMaxP2PChannels = 16;

// device >= 0: RCCL over xGMI on that GPU. Returns nullptr (with *err) if unavailable. Each
// channel costs two 2-rank communicators per pair: at N=8 a process holds 14 x channels.
std::unique_ptr<P2PTransport> make_rccl_transport(int device, int rank, int channels, std::string* err);
// Host-memory transport over abstract UNIX sockets; `ns` keeps test clusters apart.
std::unique_ptr<P2PTransport> make_socket_transport(int rank, const std::string& ns, int channels);
// Single-GPU test transport: engines in ONE process (stores on the same GPU) exchange device
// buffers with the RCCL matching contract, each matched pair a D2D copy (p2p_hiploop.cpp).
std::unique_ptr<P2PTransport> make_hiploop_transport(int device, int rank, const std::string& ns, int channels);
// Same-node device transport between PROCESSES (p2p_ipc.cpp): every rank exports its HBM
// arena over HIP IPC; a matched send is a one-sided copy into the receiver's posted extent
// (xGMI between GPUs, an in-HBM copy when ranks share one GPU). `spin` = RCCL emulation:
// spinning send/wait kernels on the channel streams instead of host-driven copies.
// `pull`: receive by receiver-side kernels (P2PTransport::post_recv_pull) where this device
// reaches the peer's memory; the peer learns it at open() and offers instead of copying.
std::unique_ptr<P2PTransport> make_ipc_transport(int device, int rank, const std::string& ns, uint8_t* arena,
                                                 uint64_t arena_bytes, bool spin, int channels, std::string* err,
                                                 bool pull = false);

}  // namespace dfs
