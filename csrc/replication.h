// Replication engine: moves block payloads between the ChunkServers (GPU ranks) of one node
// over a P2PTransport (RCCL over xGMI in production, sockets in the CPU tests), with the
// control messages (descriptors, pair bring-up) on the fast-path sockets.
//
// Reference behaviour it replaces: the synchronous store-and-forward gRPC chain
// (dfs/chunkserver/src/chunkserver.rs:777-829,1039-1077): each hop fsyncs, then forwards
// the whole block to next_servers[0]; a downstream failure still returns success with a
// smaller replicas_written.
//
// MI355X design:
//  * Fan-out, not a device-side chain. The 8 GPUs of a node form a full xGMI mesh: the
//    head has a dedicated link to every replica, so sending to all replicas at once costs
//    no extra link bandwidth and replaces the chain's per-hop latency with a single hop.
//    Device-side cut-through forwarding (recv slice s on a->b, then send it on b->c) would
//    make b->c's FIFO wait on a->b's; with chains in both directions around the node
//    (A->B->C next to C->A->B) those FIFO couplings close a cycle and deadlock. Fan-out
//    sends depend only on data already resident in HBM, so no cycle can form.
//  * Slice pipelining. A block travels as slices (256 KiB..4 MiB on the socket transport,
//    1..4 MiB on the device transports; multiples of the 512 B checksum slice); the
//    receiver launches the K1 checksum of slice s as soon as it lands,
//    while slice s+1 is still on the link, then folds the slice CRCs into the block CRC.
//  * Sequencing. Each direction of each pair has K FIFO channels (round 5; K = channels,
//    default 4): a transfer takes the least-loaded channel, the sender stamps it with the
//    channel, a per-channel sequence number and the generation of the pair, and the receiver
//    posts its receives in that channel's sequence order (a late descriptor waits its turn,
//    boundedly). One transfer still waiting for its staging or for a late descriptor holds
//    only its own channel; the pair's other transfers pass it on the others.
//  * Bounded failure handling. Any anomaly (descriptor lost, turn timeout, transfer
//    timeout, peer gone) marks the pair broken and aborts its channels at once — waiting
//    receivers wake up and fail fast; the caller falls back (shared-memory staging or the
//    gRPC path). The pair is then REBUILT under a new generation: the lower rank of a pair
//    is its only initiator (no open races), retrying with backoff until the peer answers;
//    the higher rank asks it to when it detects the failure. Blocks in flight under an old
//    generation are refused by generation check instead of being mismatched.
#pragma once
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "chunk_store.h"
#include "p2p_transport.h"

namespace dfs {

struct ReplOptions {
  int open_timeout_ms = 20000;   // one bring-up attempt of a pair
  int turn_timeout_ms = 3000;    // receiver waiting for its sequence turn
  int xfer_timeout_ms = 20000;   // one block transfer once posted
  uint64_t min_slice = 256 << 10;         // host transports (socket): pipelined from 1 MiB up
  // device transports: a 1 MiB block goes in one slice (each slice costs a copy launch, an
  // event and a wake-up on both sides: 4 x 256 KiB took 73 us to land, 1 x 1 MiB 43 us,
  // profiles/r5_repl); pipelining starts at 4 MiB
  uint64_t device_min_slice = 1 << 20;
  uint64_t max_slice = 4 << 20;
  int channels = 4;  // FIFO channels per direction of a pair (capped by the transport's)
};

struct ReplTicket {
  int peer = -1;
  uint64_t gen = 0;
  int ch = 0;         // the pair's channel the transfer is sequenced on
  bool loaded = false;  // counted in the channel's in-flight load
  int64_t seq = -1;
  uint64_t size = 0;
  uint64_t slice = 0;
  std::string id;
  bool pinned = false;
  std::vector<P2POp> ops;
};

// A block the head is still staging into HBM (ChunkStore::SliceStage): slice k may be sent
// once done[k] has completed. The caller keeps `dev` alive until wait_send / cancel_send.
struct StagedSource {
  const uint8_t* dev = nullptr;
  uint64_t slice = 0;
  const std::vector<hipEvent_t>* done = nullptr;
};

// The transport a chunkserver names on its command line: "hipipc" / "hipipc-spin" (HIP IPC
// one-sided copies), "rccl", "socket" (host memory, CPU tests), "hiploop" (one process, tests).
// channels <= 0: DFS_REPL_CHANNELS (default 4), or for RCCL DFS_REPL_CHANNELS_RCCL (default 1:
// each channel costs two communicators per pair). nullptr + *err when unavailable.
std::unique_ptr<P2PTransport> make_transport(const std::string& name, ChunkStore* store, int rank,
                                             const std::string& ns, int channels, std::string* err);

struct ReplStats {
  uint64_t bytes_sent = 0, bytes_recv = 0, blocks_sent = 0, blocks_recv = 0;
  uint64_t pair_failures = 0, pair_opens = 0, open_attempts = 0, turn_timeouts = 0, stale_generation = 0;
  uint64_t channel_waits = 0;  // sends that found their channel's turn taken and waited for it
  uint64_t parked_extents = 0, reaped_extents = 0;  // failed-receive extents held / freed after close
  // where a transfer's time goes (ns summed over transfers; divide by the call counts). Send
  // side: waiting for the staged slice 0, for the channel's turn, posting the slices, and
  // wait_send (the copies landing). Receive side: waiting for the turn and posting, the
  // slices landing (with their per-slice checksums), and recv_finish (verify + index/persist).
  uint64_t send_calls = 0, send_stage_ns = 0, send_turn_ns = 0, send_post_ns = 0, wait_send_ns = 0;
  uint64_t recv_calls = 0, recv_turn_ns = 0, recv_land_ns = 0, recv_finish_ns = 0;
  // bytes of completed transfers by peer rank: what each link carried (multi-GPU diagnosis)
  std::map<int, uint64_t> sent_to, recv_from;
};

class ReplicationEngine {
 public:
  // Sends a control message to `peer`'s fast path and returns its reply (false: unreachable).
  using ControlFn = std::function<bool(int peer, const std::string& req, std::string* reply)>;

  ReplicationEngine(ChunkStore* store, std::unique_ptr<P2PTransport> transport, int rank, int world,
                    ReplOptions opt = {});
  ~ReplicationEngine();
  ReplicationEngine(const ReplicationEngine&) = delete;

  void set_control(ControlFn fn);
  // Starts bringing up every pair this rank initiates (peers with a higher rank).
  void start();
  void stop();
  // Waits until every pair is up, or every pair that is not up has failed `give_up_after`
  // bring-up attempts (a deterministic failure, e.g. two ranks sharing one GPU), or the
  // deadline; returns the number of pairs up. Pairs keep retrying in the background.
  int wait_ready(int timeout_ms, int give_up_after = 3);

  int rank() const { return rank_; }
  int world() const { return world_; }
  const char* transport_name() const { return t_->name(); }
  bool pair_ok(int peer);
  uint64_t generation(int peer);

  // Sender: post `id` (resident in HBM for a device transport; `host_src` otherwise) to
  // `peer` as slices. The ticket carries what the peer's descriptor needs.
  // With `staged` (device transports), slices are posted as the head's staging lands them:
  // the send of slice k overlaps the host-to-device copy of slice k+1.
  // `announce` (optional) runs once the ticket is stamped and BEFORE any slice is posted (the
  // caller sends the peer its descriptor there, so the peer posts its receives while the
  // staged slices are still landing); returning false fails the pair.
  bool send(int peer, const std::string& id, const uint8_t* host_src, uint64_t n, ReplTicket* t, std::string* err,
            const StagedSource* staged = nullptr, const std::function<bool(const ReplTicket&)>& announce = nullptr);
  // Waits (bounded) until the posted slices left; unpins. False = the pair was failed.
  bool wait_send(ReplTicket* t, std::string* err);
  // Abandon a ticket whose descriptor never reached the peer (its sends can never match).
  void cancel_send(ReplTicket* t, const std::string& why);

  // Receiver: post the receive for (src, gen, seq) in order, verify while slices land, commit.
  WriteResult recv(int src, uint64_t gen, int ch, int64_t seq, const std::string& id, uint64_t size, uint64_t slice,
                   uint32_t expected_crc, bool persist_now);
  int channels() const { return channels_; }

  // Control plane (fast-path op 5). Returns the reply payload.
  std::string handle_control(const std::string& req);
  // Fails the pair's CURRENT generation (operator / test hook).
  void fail_pair(int peer, const std::string& why);
  // Fails generation `gen` only: a waiter left over from an aborted generation must not
  // tear down the pair that was rebuilt meanwhile (it just fails its own op).
  void fail_pair_gen(int peer, uint64_t gen, const std::string& why);

  P2PTransport* transport() { return t_.get(); }
  ReplStats stats();
  uint64_t slice_for(uint64_t n) const;

 private:
  enum class State { Down, Opening, Up, Broken };
  struct Peer {
    std::mutex mu;
    std::condition_variable cv;
    State state = State::Down;
    uint64_t gen = 0;
    // per channel: next sequence number to stamp, the one whose slices may be posted next,
    // the one whose receives may be posted next, and transfers posted but not completed
    std::vector<int64_t> send_seq, post_next, recv_next;
    std::vector<int> load;
    int rr = 0;  // round robin among equally loaded channels
    bool opener = false;  // an opener thread is running (initiator side)
    uint64_t peer_inc = 0;  // initiator side: the peer process instance the pair was opened with
    int failed_opens = 0;   // bring-up attempts of this pair that failed (both sides count)
    std::string last_error;
    // Receive extents of failed transfers: a DMA of that generation may still land in them,
    // so they are freed only after the next transport close() of this pair has returned
    // (close() aborts the channels and, for device transports, drains inbound copies).
    std::vector<std::pair<uint64_t, DevExtent>> parked;  // (generation, extent)
  };
  Peer& peer(int p);
  void reset_seqs_locked(Peer& P);
  void unload(ReplTicket* t);
  // Park the receive extent of a failed generation-`gen` transfer. It is freed once a LATER
  // generation of the pair is up: both ranks close() their channels before every open, and
  // the open completes only when both did, so no copy of generation `gen` can land any more
  // (RCCL: both communicators aborted; hipipc: both copy streams drained).
  void park(int p, uint64_t gen, const DevExtent& e);
  // Frees the parked extents of generations older than the pair's current, Up generation.
  void reap(int p);
  void opener_loop(int p);
  void request_reopen(int p, uint64_t gen, bool fresh);
  void spawn(std::function<void()> fn);

  ChunkStore* store_;
  std::unique_ptr<P2PTransport> t_;
  int rank_, world_;
  ReplOptions opt_;
  int channels_ = 1;
  ControlFn control_;
  std::vector<std::unique_ptr<Peer>> peers_;
  std::atomic<bool> stop_{false};
  uint64_t incarnation_ = 0;  // random per engine instance: tells a restarted peer process apart
  std::mutex threads_mu_;
  std::condition_variable threads_cv_;
  int live_threads_ = 0;
  std::mutex st_mu_;
  ReplStats st_;
};

}  // namespace dfs
