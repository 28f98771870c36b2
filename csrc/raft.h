// Native Raft consensus node for the metadata plane (C20-C25).
//
// Semantics follow the reference's simple_raft (dfs/metaserver/src/simple_raft.rs): a
// randomised 1.5-3 s election timeout and 100 ms heartbeats (:758,1161,1190-1207), a NoOp
// on becoming leader (:1367-1408), commit only of current-term entries by (joint)
// majority (:1410-1654), replies answered after apply ("commit-wait", :2430-2456),
// ReadIndex for linearizable reads (:993-1011,1863-1895), snapshots + InstallSnapshot
// (:1033-1158,1454-1534), legacy AddServer/RemoveServer and joint consensus (:2458-2737),
// TimeoutNow leadership transfer (:2740-2825) and the optional snapshot backup PUT to an
// S3 endpoint (:1214-1271). The algorithm is re-derived from the Raft paper, not
// transcribed; `log_[i - first_index()]` arithmetic lives in one place.
//
// Structure (one process = one node, no async runtime):
//   * a ticker thread (heartbeats, election timeouts, snapshot threshold),
//   * a WAL flusher thread: proposals accumulate while an fdatasync is in flight and go
//     out in the next write — leader batching / group commit (P8) without a fixed window,
//   * an applier thread feeding committed entries to the state machine in batches,
//   * per peer: a replicator thread (at most one AppendEntries/InstallSnapshot in flight,
//     re-armed by every broadcast) and an aux thread for RequestVote/TimeoutNow so an
//     election never queues behind a slow append.
// Every RPC handler is a blocking call (`handle`) that persists before it replies.
//
// The state machine and the peer transport are supplied by a Host: the master/config
// state machines, or a Python adapter (tests, interim services). Host calls are never
// made with the node mutex held.
#pragma once
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <random>
#include <set>
#include <string>
#include <thread>
#include <vector>

#include "json.h"
#include "wal.h"

namespace dfs::raft {

enum class Role { Follower = 0, Candidate = 1, Leader = 2 };
const char* role_name(Role r);

// Simple or joint (C_old,new) configuration (reference simple_raft.rs:70-252).
struct ClusterConfig {
  std::map<int, std::string> members;      // Simple, or C_new when joint
  std::map<int, std::string> old_members;  // only meaningful when joint
  bool joint = false;
  int64_t version = 0;

  std::map<int, std::string> all() const;
  bool is_voter(int id) const;
  bool has_joint_majority(const std::set<int>& acks) const;
  Json to_json() const;
  static ClusterConfig from_json(const Json& j);
};

// Result delivery for proposals and reads.
//   code 0: committed and applied (payload = state-machine result, JSON text)
//   code 1: not leader (payload = leader hint, may be empty)
//   code 2: failed (payload = message)
using Done = std::function<void(int code, const std::string& payload)>;

// A state machine implemented natively (master / config state); a Host may delegate to one.
class StateMachine {
 public:
  virtual ~StateMachine() = default;
  virtual std::vector<std::string> apply(const std::vector<std::pair<uint64_t, std::string>>& cmds) = 0;
  virtual std::string snapshot() = 0;
  virtual void restore(const std::string& state) = 0;
};

class Host {
 public:
  virtual ~Host() = default;
  // Apply committed commands in log order. One result per entry: JSON text, or "!msg"
  // for a command the state machine rejected with an error.
  virtual std::vector<std::string> apply(const std::vector<std::pair<uint64_t, std::string>>& cmds) = 0;
  virtual std::string snapshot() = 0;                  // JSON text of the whole state
  virtual void restore(const std::string& state) = 0;  // inverse of snapshot()
  // One request/response to a peer (kind = vote|append|snapshot|timeout_now, JSON
  // bodies). False on a transport failure.
  virtual bool send(const std::string& addr, const std::string& kind, const std::string& body,
                    std::string* reply) = 0;
  virtual void backup(const std::string& url, const std::string& data) {
    (void)url;
    (void)data;
  }
  // Optional native peer path: RPCs to `addr` (a member address) go straight to the peer's
  // native endpoint `endpoint` ("" = back to the default transport); `blocked` addresses
  // are unreachable (partition injection for chaos tests).
  virtual void set_peer_endpoint(const std::string& addr, const std::string& endpoint) {
    (void)addr;
    (void)endpoint;
  }
  virtual void set_blocked(const std::vector<std::string>& addrs) { (void)addrs; }
};

struct Options {
  int id = 1;
  std::map<int, std::string> members;
  std::string client_address;  // what clients are told in leader hints
  std::string dir;
  double election_lo = 1.5, election_hi = 3.0, heartbeat = 0.1;
  bool sync = true;
  uint64_t snapshot_threshold = 10000;
  int max_append_batch = 512;
  // Pre-Vote + leader stickiness (Raft thesis 9.6): a server that cannot win (a joining node
  // with an empty log, a removed or partitioned node) probes with a pre-vote first, and a
  // server that heard from a live leader within election_lo refuses to adopt a newer term
  // from a RequestVote. Leadership transfer (TimeoutNow) bypasses both.
  bool pre_vote = true;
  std::string backup_endpoint, backup_bucket = "dfs-backups";
};

class Node {
 public:
  Node(Options opt, std::shared_ptr<Host> host);
  ~Node();
  Node(const Node&) = delete;
  Node& operator=(const Node&) = delete;

  void start();
  void stop();

  void propose(const std::string& cmd, Done done);  // commit-wait
  bool propose_nowait(const std::string& cmd);       // fire and forget
  void read_index(Done done);
  // Blocking RPC handler: kind = vote|append|snapshot|timeout_now, JSON in and out.
  std::string handle(const std::string& kind, const std::string& body);
  bool transfer_leadership(int target);
  void snapshot_now();

  // Joint-consensus helpers: new servers replicate as non-voters until caught up.
  void add_non_voter(int id, const std::string& addr);
  void drop_non_voter(int id);
  bool caught_up(int id);

  // Introspection (thread-safe snapshots of volatile state).
  Role role() const;
  bool is_leader() const { return role() == Role::Leader; }
  // Leader whose leadership a majority confirmed within election_lo (leader lease): safe to
  // answer without a Raft round trip (deferred block placement, see MasterCore::create_file).
  bool has_lease() const;
  uint64_t term() const;
  int leader_id() const;
  std::string leader_address() const;
  uint64_t commit_index() const;
  uint64_t last_applied() const;
  uint64_t last_index() const;
  uint64_t last_included_index() const;
  size_t votes() const;
  ClusterConfig config() const;
  std::string info_json() const;
  uint64_t wal_syncs() const { return wal_ ? wal_->syncs() : 0; }
  uint64_t wal_bytes() const { return wal_ ? wal_->size_bytes() : 0; }
  int id() const { return opt_.id; }
  Host& host() const { return *host_; }

 private:
  struct Entry {
    uint64_t term;
    std::string cmd;  // JSON text ("\"NoOp\"" or an externally tagged command)
  };
  struct Pending {
    uint64_t term;
    Done done;
  };
  struct ReadWaiter {
    uint64_t index;
    uint64_t need_round;
    Done done;
  };
  struct Peer {
    int id = 0;
    std::thread repl, aux;
    std::condition_variable cv, aux_cv;
    bool want_append = false;
    std::string vote_body;  // pending RequestVote args (empty = none)
    uint64_t vote_term = 0;
    bool vote_pre = false;    // vote_body is a pre-vote of round vote_round
    uint64_t vote_round = 0;
  };
  using Callbacks = std::vector<std::function<void()>>;
  using Clock = std::chrono::steady_clock;

  // log arithmetic (mu_ held)
  uint64_t first_index() const { return last_included_index_ + 1; }
  uint64_t last_index_locked() const { return last_included_index_ + log_.size(); }
  int64_t term_at(uint64_t idx) const;
  const Entry& at(uint64_t idx) const { return log_[idx - first_index()]; }

  // persistence
  void load();
  std::string hs_record() const;
  std::string entry_record(uint64_t idx) const;
  std::string config_record() const;
  std::string snap_path() const { return opt_.dir + "/snapshot.json"; }

  // threads
  void ticker_loop();
  void flusher_loop();
  void applier_loop();
  void repl_loop(Peer* p);
  void aux_loop(Peer* p);
  Peer* peer(int id);  // create on first use (mu_ held)

  // role changes (mu_ held)
  void start_election_locked(bool transfer, std::string* hs, std::string* vote_args);
  void run_election(bool transfer = false);
  void run_pre_vote();
  bool leader_recent_locked() const;  // heard from (or are) a live leader within election_lo
  // a reply or request carried a newer term: step down and persist it
  void observe_term(uint64_t term, const std::string& leader_addr, int leader_id);
  void become_leader_locked();
  bool step_down_locked(uint64_t term, const std::string& leader_addr, int leader_id, Callbacks& cbs);
  void fail_pending_locked(Callbacks& cbs);
  void reset_election_timer_locked();
  std::vector<int> peers_locked() const;
  std::string addr_locked(int id) const;

  // replication (mu_ held)
  uint64_t append_local_locked(const std::string& cmd);
  void broadcast_locked();
  void advance_commit_locked();
  void check_reads_locked(Callbacks& cbs);
  bool replicate_once(Peer* p);  // one RPC; true if the peer wants another round now
  void send_snapshot(Peer* p);

  // RPC handlers
  std::string on_vote(const Json& a);
  std::string on_append(const Json& a);
  std::string on_snapshot(const Json& a);
  std::string on_timeout_now(const Json& a);

  // apply helpers
  std::string apply_membership_locked(const Json& m, Callbacks& cbs);
  void take_snapshot();
  void persist(const std::vector<std::string>& recs);  // wal_order_mu_ held

  Options opt_;
  std::shared_ptr<Host> host_;
  std::unique_ptr<Wal> wal_;

  mutable std::mutex mu_;
  std::mutex wal_order_mu_;  // WAL writes happen in the order their records were built
  std::mutex append_mu_;     // serialises AppendEntries / InstallSnapshot handlers
  std::mutex apply_mu_;      // held while the state machine applies / captures a snapshot / restores
  std::mutex snap_mu_;       // one snapshot file writer at a time (compaction vs InstallSnapshot)
  std::condition_variable flush_cv_, apply_cv_, tick_cv_;

  // persistent state
  uint64_t current_term_ = 0;
  int voted_for_ = -1;
  std::deque<Entry> log_;
  uint64_t last_included_index_ = 0, last_included_term_ = 0;
  ClusterConfig config_;
  // volatile state
  Role role_ = Role::Follower;
  int leader_id_ = -1;
  std::string leader_address_;
  uint64_t commit_index_ = 0, last_applied_ = 0;
  std::map<int, uint64_t> next_index_, match_index_;
  std::set<int> votes_;
  std::map<int, std::string> non_voting_;
  std::map<int, std::pair<uint64_t, int>> catch_up_;  // id -> (match, rounds caught up)
  std::map<uint64_t, Pending> pending_;
  uint64_t unsynced_from_ = 0, durable_index_ = 0;
  uint64_t hb_round_ = 0;
  std::map<int, uint64_t> acked_round_;
  std::map<int, Clock::time_point> ack_at_;  // leader: send time of each follower's latest same-term answer
  std::vector<ReadWaiter> read_waiters_;
  uint64_t leader_noop_index_ = 0;
  Clock::time_point election_deadline_;
  Clock::time_point leader_contact_{};  // last accepted AppendEntries / InstallSnapshot
  uint64_t prevote_round_ = 0;
  std::set<int> prevotes_;
  bool tick_now_ = false;
  std::mt19937_64 rng_;

  std::map<int, std::unique_ptr<Peer>> peers_;
  std::thread ticker_, flusher_, applier_, snapshotter_;
  // compaction runs on its own thread: the applier only requests it (snap_req_, under mu_),
  // so applies stall for the state capture, not for the snapshot file write and WAL rewrite
  std::condition_variable snap_cv_;
  bool snap_req_ = false;
  // compaction pacing (mu_): command bytes applied since the last snapshot's capture, and that
  // snapshot's size; a snapshot is due once the log holds both snapshot_threshold entries and
  // half a snapshot's worth of bytes, so rewriting the state stays proportional to the log's
  // growth however large the namespace is
  uint64_t applied_bytes_since_snap_ = 0, last_snap_bytes_ = 0;
  void snapshot_loop();
  std::atomic<bool> running_{false};
  bool started_ = false;
};

// Disaster recovery from an off-box snapshot backup (the bytes a leader PUT to
// `{endpoint}/{bucket}/master-snapshots/node-{id}/...`, Options::backup_endpoint; the reference
// is upload-only). Seeds an EMPTY node directory with the snapshot: its
// state and (index, term) as the node's snapshot, the current term raised to the snapshot's
// (so entries appended after it keep non-decreasing terms), and no membership, so the
// restored node starts with the members it is given (--peers), not the backed-up cluster's.
// Refuses a directory that already holds a snapshot or Raft log records.
bool restore_snapshot_dir(const std::string& dir, const std::string& payload, std::string* err);

}  // namespace dfs::raft
