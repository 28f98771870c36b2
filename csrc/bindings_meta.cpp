// pybind11 bindings of the native metadata plane (Raft node). The service layer drives a
// node through a handful of non-blocking calls; completions come back through Python
// callables invoked from native threads with the GIL acquired. Every binding that can
// wait on a node mutex releases the GIL first, and no native thread ever waits for the
// GIL while holding a node mutex.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstring>
#include <map>
#include <mutex>
#include <optional>
#include <set>
#include <condition_variable>
#include <functional>
#include <thread>

#include "audit_log.h"
#include "client_fast.h"
#include "client_remote.h"
#include "grpc_client.h"
#include "dfs_pb.h"
#include "grpc_server.h"
#include "localrpc.h"
#include "config_core.h"
#include "master_core.h"
#include "raft.h"
#include "s3_front.h"
#include "s3_policy.h"
#include "tls.h"
#include "trace.h"

namespace py = pybind11;
using namespace dfs;

namespace {

// A Python object that may be dropped on any thread: the decref takes the GIL.
struct PyRef {
  py::object obj;
  explicit PyRef(py::object o) : obj(std::move(o)) {}
  ~PyRef() {
    if (!Py_IsInitialized()) {
      obj.release();  // interpreter gone: leak rather than touch it
      return;
    }
    py::gil_scoped_acquire g;
    obj = py::object();
  }
};

// Host backed by a Python object with apply_batch / snapshot / restore / send / backup.
class PyRaftHost : public raft::Host {
 public:
  PyRaftHost(py::object host, std::shared_ptr<raft::StateMachine> sm)
      : host_(std::make_shared<PyRef>(std::move(host))), sm_(std::move(sm)) {}

  std::vector<std::string> apply(const std::vector<std::pair<uint64_t, std::string>>& cmds) override {
    if (sm_) return sm_->apply(cmds);  // native state machine: no GIL on the apply path
    py::gil_scoped_acquire g;
    try {
      py::list l;
      for (auto& c : cmds) l.append(py::make_tuple(c.first, py::str(c.second)));
      return host_->obj.attr("apply_batch")(l).cast<std::vector<std::string>>();
    } catch (py::error_already_set& e) {
      throw std::runtime_error(e.what());
    }
  }
  std::string snapshot() override {
    if (sm_) return sm_->snapshot();
    py::gil_scoped_acquire g;
    try {
      return host_->obj.attr("snapshot")().cast<std::string>();
    } catch (py::error_already_set& e) {
      throw std::runtime_error(e.what());
    }
  }
  void restore(const std::string& state) override {
    if (sm_) return sm_->restore(state);
    py::gil_scoped_acquire g;
    try {
      host_->obj.attr("restore")(py::str(state));
    } catch (py::error_already_set& e) {
      throw std::runtime_error(e.what());
    }
  }
  bool send(const std::string& addr, const std::string& kind, const std::string& body, std::string* reply) override {
    std::string ep;
    {
      std::lock_guard<std::mutex> lk(peers_mu_);
      if (blocked_.count(addr)) return false;
      auto it = endpoints_.find(addr);
      if (it != endpoints_.end()) ep = it->second;
    }
    if (!ep.empty()) {
      // native peer path: the peer's native gRPC server hands the JSON straight to its node
      // (reference timeouts: 1.5 s per RPC, snapshots get longer)
      GrpcResult r = peers_->call(ep, "/dfs.RaftPeer/" + kind, body, "", kind == "snapshot" ? 30000 : 1500);
      if (!r.transport_ok || r.status != 0) return false;
      *reply = std::move(r.message);
      return true;
    }
    py::gil_scoped_acquire g;
    try {
      py::object r = host_->obj.attr("send")(addr, kind, py::str(body));
      if (r.is_none()) return false;
      *reply = r.cast<std::string>();
      return true;
    } catch (py::error_already_set& e) {
      return false;
    }
  }
  void set_peer_endpoint(const std::string& addr, const std::string& endpoint) override {
    std::lock_guard<std::mutex> lk(peers_mu_);
    if (endpoint.empty()) endpoints_.erase(addr);
    else endpoints_[addr] = endpoint;
  }
  void set_blocked(const std::vector<std::string>& addrs) override {
    std::lock_guard<std::mutex> lk(peers_mu_);
    blocked_ = std::set<std::string>(addrs.begin(), addrs.end());
  }
  void backup(const std::string& url, const std::string& data) override {
    py::gil_scoped_acquire g;
    try {
      host_->obj.attr("backup")(url, py::bytes(data));
    } catch (py::error_already_set& e) {
    }
  }

 private:
  std::shared_ptr<PyRef> host_;
  std::shared_ptr<raft::StateMachine> sm_;
  std::mutex peers_mu_;
  std::map<std::string, std::string> endpoints_;  // member address -> native gRPC endpoint
  std::set<std::string> blocked_;
  std::unique_ptr<GrpcChannelPool> peers_ = std::make_unique<GrpcChannelPool>(1500);

 public:
  // https peers: the native Raft peer RPC runs over TLS (set before the node starts)
  void set_peer_tls(std::shared_ptr<TlsContext> tls) { peers_ = std::make_unique<GrpcChannelPool>(1500, std::move(tls)); }
};

// Read a node property with the GIL released (the getter may wait on the node mutex).
template <class F>
auto unlocked(F f) -> decltype(f()) {
  py::gil_scoped_release r;
  return f();
}

raft::Done py_done(py::object cb) {
  auto ref = std::make_shared<PyRef>(std::move(cb));
  return [ref](int code, const std::string& payload) {
    py::gil_scoped_acquire g;
    try {
      ref->obj(code, py::str(payload));
    } catch (py::error_already_set& e) {
      e.discard_as_unraisable("raft completion callback");
    }
  };
}

// Destroying a node joins its threads, which may need the GIL: never hold it meanwhile.
struct NodeDeleter {
  void operator()(raft::Node* n) const {
    py::gil_scoped_release r;
    delete n;
  }
};

// ---------------- native `dfs_cli benchmark` workers
// The reference's benchmark runs its `concurrency` workers as tokio tasks inside the Rust
// CLI (dfs/client/src/bin/dfs_cli.rs:594-628 write, :633-690 read), each timing one
// client call. These are the same workers as native threads over the native clients, so
// the measured latency is the client call and not Python's thread pool and GIL hand-offs.
// Every op still moves the whole file: a write hashes (CRC + MD5) and ships the caller's
// buffer; a read copies the block out of the transfer slot into a worker-owned buffer
// (like `get_file_content`'s Vec) and, when an expected payload is given, compares it.
struct BenchOut {
  std::vector<int> status;  // FastClient::Status per op
  std::vector<double> lat;  // seconds per op
  std::vector<FastClient::Times> times;
  std::vector<uint64_t> bytes;
  std::string first_error;
  uint64_t mismatches = 0;
  double total_s = 0;
};

// The workers are a persistent pool, like the reference CLI's tokio runtime: created once,
// each keeping its read buffer (pre-touched) across calls. Spawning `concurrency` threads per
// phase and giving each a fresh 1 MiB buffer meant thread stacks and buffers mapped and
// unmapped twice per step, and the page faults and TLB shootdowns of that stalled the other
// workers' copies (measured as 2-8 ms copy stalls of ~10 concurrent writes, r6).
class BenchPool {
 public:
  static BenchPool& get() {
    static BenchPool* p = new BenchPool();  // never destroyed: workers park between calls
    return *p;
  }
  // runs job(worker_buffer) on `n` workers and returns when all have finished
  void run(int n, const std::function<void(std::vector<uint8_t>*)>& job) {
    std::unique_lock<std::mutex> lk(mu_);
    busy_cv_.wait(lk, [&] { return !active_; });  // one run at a time
    while (static_cast<int>(threads_.size()) < n) {
      const int id = static_cast<int>(threads_.size());
      bufs_.push_back(std::make_unique<std::vector<uint8_t>>());
      threads_.emplace_back([this, id] { loop(id); });
      threads_.back().detach();
    }
    job_ = &job;
    want_ = n;
    running_ = n;
    active_ = true;
    ++gen_;
    cv_.notify_all();
    done_cv_.wait(lk, [&] { return running_ == 0; });
    job_ = nullptr;
    active_ = false;
    busy_cv_.notify_one();
  }

 private:
  void loop(int id) {
    uint64_t seen = 0;
    std::unique_lock<std::mutex> lk(mu_);
    for (;;) {
      cv_.wait(lk, [&] { return gen_ != seen; });
      seen = gen_;
      if (id >= want_) continue;
      const auto* job = job_;
      std::vector<uint8_t>* buf = bufs_[id].get();
      lk.unlock();
      (*job)(buf);
      lk.lock();
      if (--running_ == 0) done_cv_.notify_all();
    }
  }
  std::mutex mu_;
  std::condition_variable cv_, done_cv_, busy_cv_;
  std::vector<std::thread> threads_;
  std::vector<std::unique_ptr<std::vector<uint8_t>>> bufs_;
  const std::function<void(std::vector<uint8_t>*)>* job_ = nullptr;
  int want_ = 0, running_ = 0;
  bool active_ = false;
  uint64_t gen_ = 0;
};

template <class Op>
void bench_run(size_t count, int concurrency, BenchOut* out, Op op) {
  out->status.assign(count, 0);
  out->lat.assign(count, 0.0);
  out->times.assign(count, FastClient::Times{});
  out->bytes.assign(count, 0);
  std::atomic<size_t> next{0};
  std::mutex err_mu;
  std::function<void(std::vector<uint8_t>*)> worker = [&](std::vector<uint8_t>* buf) {
    for (size_t i; (i = next.fetch_add(1)) < count;) {
      std::string msg;
      auto t0 = std::chrono::steady_clock::now();
      int st = op(i, &out->times[i], &out->bytes[i], buf, &msg);
      out->lat[i] = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      out->status[i] = st;
      if (st == FastClient::Failed) {
        std::lock_guard<std::mutex> g(err_mu);
        if (out->first_error.empty()) out->first_error = msg;
      }
    }
  };
  auto t0 = std::chrono::steady_clock::now();
  BenchPool::get().run(std::max(1, concurrency), worker);
  out->total_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}

py::tuple bench_result(const BenchOut& o, bool reads) {
  py::list times;
  for (const auto& t : o.times) {
    if (reads) times.append(py::make_tuple(t.getinfo, t.read));
    else times.append(py::make_tuple(t.crc, t.create, t.write, t.md5_wait, t.complete, t.copy, t.acquire));
  }
  return py::make_tuple(o.status, o.lat, o.total_s, times, o.bytes, o.first_error, o.mismatches);
}

struct BufView {
  const uint8_t* p = nullptr;
  size_t n = 0;
};

std::vector<BufView> buf_views(const py::list& bufs) {
  std::vector<BufView> v;
  for (auto h : bufs) {
    if (h.is_none()) {
      v.push_back({});
      continue;
    }
    py::buffer_info bi = py::reinterpret_borrow<py::buffer>(h).request();
    v.push_back({static_cast<const uint8_t*>(bi.ptr), static_cast<size_t>(bi.size * bi.itemsize)});
  }
  return v;
}

// writes: paths[i] <- payloads[i % len(payloads)]; the caller keeps `payloads` alive
template <class C>
py::tuple bench_writes(C& c, const std::vector<std::string>& paths, const py::list& payloads, int concurrency) {
  std::vector<BufView> pv = buf_views(payloads);
  if (pv.empty()) throw std::invalid_argument("no payloads");
  BenchOut o;
  {
    py::gil_scoped_release r;
    bench_run(paths.size(), concurrency, &o,
              [&](size_t i, FastClient::Times* t, uint64_t* nb, std::vector<uint8_t>*, std::string* msg) {
                const BufView& b = pv[i % pv.size()];
                int replicas = 0;
                *nb = b.n;
                return static_cast<int>(c.write(paths[i], b.p, b.n, &replicas, msg, t));
              });
  }
  return bench_result(o, false);
}

// reads: expected[i] (or None) is compared with what paths[i] returned
py::tuple bench_reads_fast(FastClient& c, const std::vector<std::string>& paths, const py::list& expected,
                           int concurrency) {
  std::vector<BufView> ev = buf_views(expected);
  BenchOut o;
  std::atomic<uint64_t> bad{0};
  {
    py::gil_scoped_release r;
    bench_run(paths.size(), concurrency, &o,
              [&](size_t i, FastClient::Times* t, uint64_t* nb, std::vector<uint8_t>* buf, std::string* msg) {
                int64_t slot = -1;
                uint64_t n = 0;
                FastClient::Status st = c.read(paths[i], &slot, &n, msg, t);
                if (st != FastClient::Ok) return static_cast<int>(st);
                if (buf->size() < n) buf->resize(n);  // kept by the pool's worker across calls
                if (n) std::memcpy(buf->data(), c.slot_ptr(slot), n);
                if (slot >= 0) c.release(slot);
                *nb = n;
                if (i < ev.size() && ev[i].p && (ev[i].n != n || std::memcmp(ev[i].p, buf->data(), n) != 0)) bad++;
                return static_cast<int>(st);
              });
  }
  o.mismatches = bad.load();
  return bench_result(o, true);
}

py::tuple bench_reads_remote(RemoteClient& c, const std::vector<std::string>& paths, const py::list& expected,
                             int concurrency) {
  std::vector<BufView> ev = buf_views(expected);
  BenchOut o;
  std::atomic<uint64_t> bad{0};
  {
    py::gil_scoped_release r;
    bench_run(paths.size(), concurrency, &o,
              [&](size_t i, FastClient::Times* t, uint64_t* nb, std::vector<uint8_t>*, std::string* msg) {
                std::string data;  // the reply's payload, owned by this op
                FastClient::Status st = c.read(paths[i], &data, msg, t);
                if (st != FastClient::Ok) return static_cast<int>(st);
                *nb = data.size();
                if (i < ev.size() && ev[i].p &&
                    (ev[i].n != data.size() || std::memcmp(ev[i].p, data.data(), data.size()) != 0))
                  bad++;
                return static_cast<int>(st);
              });
  }
  o.mismatches = bad.load();
  return bench_result(o, true);
}

}  // namespace

void bind_meta(py::module_& m) {
  m.def("raft_has_joint_majority", [](const std::string& config_json, const std::vector<int>& acks) {
    return raft::ClusterConfig::from_json(Json::parse(config_json)).has_joint_majority({acks.begin(), acks.end()});
  }, "the native node's (joint) quorum rule, for tests");
  m.def("pb_roundtrip", [](const std::string& name, py::bytes data) -> py::object {
    std::string in = data, out;
    if (!pb::roundtrip(name, in, &out)) return py::none();
    return py::bytes(out);
  }, "decode `data` as dfs.<name> with the native codec and re-encode it");

  py::class_<raft::StateMachine, std::shared_ptr<raft::StateMachine>>(m, "StateMachine",
                                                                     "a natively applied Raft state machine");
  py::class_<raft::Node, std::unique_ptr<raft::Node, NodeDeleter>>(m, "RaftNode")
      .def(py::init([](int id, std::map<int, std::string> members, std::string client_address, std::string dir,
                       py::object host, double elo, double ehi, double hb, bool sync, uint64_t snapshot_threshold,
                       int max_batch, std::string backup_endpoint, std::string backup_bucket, py::object native_sm,
                       bool pre_vote, bool peer_tls, std::string peer_ca, std::string peer_domain) {
             raft::Options o;
             o.id = id;
             o.members = std::move(members);
             o.client_address = std::move(client_address);
             o.dir = std::move(dir);
             o.election_lo = elo;
             o.election_hi = ehi;
             o.heartbeat = hb;
             o.sync = sync;
             o.snapshot_threshold = snapshot_threshold;
             o.max_append_batch = max_batch;
             o.backup_endpoint = std::move(backup_endpoint);
             o.backup_bucket = std::move(backup_bucket);
             o.pre_vote = pre_vote;
             std::shared_ptr<raft::StateMachine> sm;
             if (!native_sm.is_none()) sm = native_sm.cast<std::shared_ptr<raft::StateMachine>>();
             auto h = std::make_shared<PyRaftHost>(std::move(host), sm);
             if (peer_tls) {
               std::string err;
               auto t = TlsContext::client(peer_ca, peer_domain, &err);
               if (!t) throw std::runtime_error(err);
               h->set_peer_tls(std::move(t));
             }
             return std::unique_ptr<raft::Node, NodeDeleter>(new raft::Node(std::move(o), h));
           }),
           py::arg("id"), py::arg("members"), py::arg("client_address"), py::arg("dir"), py::arg("host"),
           py::arg("election_lo") = 1.5, py::arg("election_hi") = 3.0, py::arg("heartbeat") = 0.1,
           py::arg("sync") = true, py::arg("snapshot_threshold") = 10000, py::arg("max_append_batch") = 512,
           py::arg("backup_endpoint") = "", py::arg("backup_bucket") = "dfs-backups",
           py::arg("native_sm") = py::none(), py::arg("pre_vote") = true, py::arg("peer_tls") = false,
           py::arg("peer_ca") = "", py::arg("peer_domain") = "")
      .def("start", &raft::Node::start, py::call_guard<py::gil_scoped_release>())
      .def("stop", &raft::Node::stop, py::call_guard<py::gil_scoped_release>())
      .def("propose", [](raft::Node& n, std::string cmd, py::object cb) {
        raft::Done d = py_done(std::move(cb));
        py::gil_scoped_release r;
        n.propose(cmd, std::move(d));
      })
      .def("propose_nowait", &raft::Node::propose_nowait, py::call_guard<py::gil_scoped_release>())
      .def("read_index", [](raft::Node& n, py::object cb) {
        raft::Done d = py_done(std::move(cb));
        py::gil_scoped_release r;
        n.read_index(std::move(d));
      })
      .def("handle", &raft::Node::handle, py::call_guard<py::gil_scoped_release>())
      .def("transfer_leadership", &raft::Node::transfer_leadership, py::call_guard<py::gil_scoped_release>())
      .def("snapshot_now", &raft::Node::snapshot_now, py::call_guard<py::gil_scoped_release>())
      .def("add_non_voter", &raft::Node::add_non_voter, py::call_guard<py::gil_scoped_release>())
      .def("drop_non_voter", &raft::Node::drop_non_voter, py::call_guard<py::gil_scoped_release>())
      .def("caught_up", &raft::Node::caught_up, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("has_lease", [](raft::Node& n) { return unlocked([&] { return n.has_lease(); }); })
      .def_property_readonly("role", [](raft::Node& n) {
        raft::Role r;
        {
          py::gil_scoped_release g;
          r = n.role();
        }
        return std::string(raft::role_name(r));
      })
      .def_property_readonly("term", [](raft::Node& n) { return unlocked([&] { return n.term(); }); })
      .def_property_readonly("leader_id", [](raft::Node& n) { return unlocked([&] { return n.leader_id(); }); })
      .def_property_readonly("leader_address", [](raft::Node& n) { return unlocked([&] { return n.leader_address(); }); })
      .def_property_readonly("commit_index", [](raft::Node& n) { return unlocked([&] { return n.commit_index(); }); })
      .def_property_readonly("last_applied", [](raft::Node& n) { return unlocked([&] { return n.last_applied(); }); })
      .def_property_readonly("last_index", [](raft::Node& n) { return unlocked([&] { return n.last_index(); }); })
      .def_property_readonly("last_included_index", [](raft::Node& n) { return unlocked([&] { return n.last_included_index(); }); })
      .def_property_readonly("votes", [](raft::Node& n) { return unlocked([&] { return n.votes(); }); })
      .def_property_readonly("config_json", [](raft::Node& n) {
        std::string s;
        {
          py::gil_scoped_release g;
          s = n.config().to_json().dump();
        }
        return s;
      })
      .def("info_json", &raft::Node::info_json, py::call_guard<py::gil_scoped_release>())
      .def("set_peer_endpoint", [](raft::Node& n, const std::string& addr, const std::string& ep) {
        n.host().set_peer_endpoint(addr, ep);
      })
      .def("set_blocked", [](raft::Node& n, const std::vector<std::string>& addrs) { n.host().set_blocked(addrs); })
      .def_property_readonly("wal_syncs", &raft::Node::wal_syncs)
      .def_property_readonly("wal_bytes", &raft::Node::wal_bytes);
  m.def("raft_restore_snapshot_dir", [](const std::string& dir, const std::string& payload) {
    std::string err;
    const bool ok = raft::restore_snapshot_dir(dir, payload, &err);
    return py::make_tuple(ok, err);
  });

  // ---------------- native shard map (csrc/shard_map.cpp), for parity tests with parallel/sharding.py
  py::class_<ShardMap>(m, "NativeShardMap")
      .def_static("new_range", &ShardMap::new_range)
      .def_static("new_consistent_hash", &ShardMap::new_consistent_hash, py::arg("virtual_nodes") = 100)
      .def_static("from_json", [](const std::string& s) { return ShardMap::from_json(Json::parse(s)); })
      .def("to_json", [](const ShardMap& sm) { return sm.to_json().dump(); })
      .def("add_shard", &ShardMap::add_shard)
      .def("remove_shard", &ShardMap::remove_shard)
      .def("split_shard", &ShardMap::split_shard)
      .def("merge_shards", &ShardMap::merge_shards)
      .def("rebalance_boundary", &ShardMap::rebalance_boundary)
      .def("get_shard", [](const ShardMap& sm, const std::string& key) -> py::object {
        std::string s = sm.get_shard(key);
        if (s.empty()) return py::none();
        return py::str(s);
      })
      .def("get_shards", [](const ShardMap& sm, const std::vector<std::string>& keys) {
        std::vector<std::string> out;
        out.reserve(keys.size());
        for (const auto& k : keys) out.push_back(sm.get_shard(k));
        return out;
      })
      .def("shards", &ShardMap::shards);

  // ---------------- native config-server state machine (C36)
  py::class_<ConfigCore, raft::StateMachine, std::shared_ptr<ConfigCore>>(m, "ConfigCore")
      .def(py::init([]() { return std::make_shared<ConfigCore>(); }))
      .def("apply", [](ConfigCore& c, uint64_t idx, const std::string& cmd) {
        py::gil_scoped_release r;
        return c.apply({{idx, cmd}}).front();
      })
      .def("snapshot", &ConfigCore::snapshot, py::call_guard<py::gil_scoped_release>())
      .def("restore", &ConfigCore::restore, py::call_guard<py::gil_scoped_release>())
      .def("shard_map_json", &ConfigCore::shard_map_json)
      .def("masters_json", &ConfigCore::masters_json)
      .def_property_readonly("version", &ConfigCore::version)
      .def("split_candidates", &ConfigCore::split_candidates, py::arg("n") = 3)
      .def("attach", [](ConfigCore& c, raft::Node& n) { c.attach(&n); }, py::keep_alive<1, 2>())
      .def("detach", &ConfigCore::detach)
      .def("handle", [](ConfigCore& c, const std::string& method, py::bytes req) {
        std::string in = req, out;
        int code;
        {
          py::gil_scoped_release r;
          code = c.handle(method, in, &out);
        }
        return py::make_tuple(code, py::bytes(out));
      })
      .def_property_readonly("requests", &ConfigCore::requests);

  // ConfigService over native HTTP/2 gRPC and the same-host socket: every method and the
  // Raft peer RPC answered by ConfigCore, no Python on any request.
  struct NativeGrpcConfig {
    std::unique_ptr<GrpcServer> srv;
    std::atomic<uint64_t> raft_calls{0};
  };
  py::class_<NativeGrpcConfig>(m, "NativeGrpcConfigServer")
      .def(py::init([](std::shared_ptr<ConfigCore> core, const std::string& host, int port, int workers,
                       const std::string& tls_cert, const std::string& tls_key) {
             auto n = std::make_unique<NativeGrpcConfig>();
             NativeGrpcConfig* self = n.get();
             static const std::string kPrefix = "/dfs.ConfigService/";
             static const std::string kRaft = "/dfs.RaftPeer/";
             n->srv = std::make_unique<GrpcServer>(host, port, [core, self](const GrpcCall& c) -> GrpcReply {
               GrpcReply r;
               RequestScope scope(c.request_id);
               if (c.path.compare(0, kRaft.size(), kRaft) == 0) {
                 r.status = core->raft_rpc(c.path.substr(kRaft.size()), c.message, &r.message);
                 self->raft_calls++;
               } else if (c.path.compare(0, kPrefix.size(), kPrefix) == 0) {
                 r.status = core->handle(c.path.substr(kPrefix.size()), c.message, &r.message);
               } else {
                 r.status = 12;
                 r.message = "unknown service: " + c.path;
               }
               return r;
             }, workers);
             if (!tls_cert.empty()) {
               std::string err;
               auto t = TlsContext::server(tls_cert, tls_key, &err);
               if (!t) throw std::runtime_error(err);
               n->srv->set_tls(std::move(t));
             }
             return n;
           }),
           py::arg("core"), py::arg("host"), py::arg("port"), py::arg("workers") = 16, py::arg("tls_cert") = "",
           py::arg("tls_key") = "")
      .def("start", [](NativeGrpcConfig& n) {
        std::string err;
        bool ok = n.srv->start(&err);
        return py::make_tuple(ok, err);
      })
      .def("stop", [](NativeGrpcConfig& n) {
        py::gil_scoped_release r;
        n.srv->stop();
      })
      .def_property_readonly("port", [](NativeGrpcConfig& n) { return n.srv->port(); })
      .def("stats", [](NativeGrpcConfig& n) {
        py::dict d;
        d["native_grpc_calls"] = n.srv->calls();
        d["native_raft_rpcs"] = n.raft_calls.load();
        return d;
      });

  struct ConfigLocal {  // (LocalRpcServer itself is bound once, as MasterLocalServer)
    std::unique_ptr<LocalRpcServer> srv;
  };
  py::class_<ConfigLocal>(m, "ConfigLocalServer")
      .def(py::init([](const std::string& name, std::shared_ptr<ConfigCore> core) {
             static const std::string kPrefix = "/dfs.ConfigService/";
             LocalRpcServer::Handler h = [core](const std::string& path, const std::string& rid, const std::string& payload,
                                                std::string* out) -> int {
               RequestScope scope(rid);
               if (path.compare(0, kPrefix.size(), kPrefix) != 0) return (*out = "unknown service: " + path, 12);
               return core->handle(path.substr(kPrefix.size()), payload, out);
             };
             auto c = std::make_unique<ConfigLocal>();
             c->srv = std::make_unique<LocalRpcServer>(name, std::move(h));
             return c;
           }))
      .def("start", [](ConfigLocal& s) {
        std::string err;
        bool ok = s.srv->start(&err);
        return py::make_tuple(ok, err);
      })
      .def("stop", [](ConfigLocal& s) {
        py::gil_scoped_release r;
        s.srv->stop();
      })
      .def_property_readonly("requests", [](ConfigLocal& s) { return s.srv->requests(); });

  // ---------------- native master core + same-host RPC listener
  py::class_<MasterCore, raft::StateMachine, std::shared_ptr<MasterCore>>(m, "MasterCore")
      .def(py::init([]() { return std::make_shared<MasterCore>(); }))
      .def("attach", [](MasterCore& c, raft::Node& n) { c.attach(&n); }, py::keep_alive<1, 2>())
      .def("detach", &MasterCore::detach)
      .def("native_method", &MasterCore::native_method)
      .def("handle", [](MasterCore& c, const std::string& method, py::bytes req) {
        std::string in = req, out;
        int code;
        {
          py::gil_scoped_release r;
          code = c.handle(method, in, &out);
        }
        return py::make_tuple(code, py::bytes(out));
      })
      .def("set_shard_map", &MasterCore::set_shard_map, py::call_guard<py::gil_scoped_release>())
      .def("note_shard_map_fresh", &MasterCore::note_shard_map_fresh, py::call_guard<py::gil_scoped_release>())
      .def("set_shard_map_max_age", &MasterCore::set_shard_map_max_age, py::call_guard<py::gil_scoped_release>())
      .def("set_access_stats", &MasterCore::set_access_stats)
      .def("upsert_chunk_server", [](MasterCore& c, const std::string& addr, int64_t last_heartbeat, uint64_t used,
                                     uint64_t avail, uint64_t chunks, const std::string& rack, int32_t gpu_rank,
                                     uint64_t hbm_capacity, uint64_t hbm_used, uint64_t scheduled) {
        ChunkServerStatus st;
        st.address = addr;
        st.last_heartbeat = last_heartbeat;
        st.used_space = used;
        st.available_space = avail;
        st.chunk_count = chunks;
        st.rack_id = rack;
        st.gpu_rank = gpu_rank;
        st.hbm_capacity = hbm_capacity;
        st.hbm_used = hbm_used;
        st.scheduled = scheduled;
        c.upsert_chunk_server(st);
      })
      .def("remove_chunk_server", &MasterCore::remove_chunk_server)
      .def("chunk_servers", [](MasterCore& c) {
        py::list out;
        for (auto& s : c.chunk_servers())
          out.append(py::make_tuple(s.address, s.last_heartbeat, s.used_space, s.available_space, s.chunk_count,
                                    s.rack_id, s.gpu_rank, s.hbm_capacity, s.hbm_used, s.scheduled));
        return out;
      })
      .def("enter_safe_mode", &MasterCore::enter_safe_mode, py::arg("manual") = false)
      .def("exit_safe_mode", &MasterCore::exit_safe_mode)
      .def("should_exit_safe_mode", &MasterCore::should_exit_safe_mode)
      .def("report_blocks", &MasterCore::report_blocks)
      .def("safe_mode_status", [](MasterCore& c) { return c.safe_mode_status().dump(); })
      .def("get_file", [](MasterCore& c, const std::string& path, bool visible_only) -> py::object {
        std::string out;
        if (!c.get_file(path, visible_only, &out)) return py::none();
        return py::bytes(out);
      }, py::arg("path"), py::arg("visible_only") = false)
      .def("contains", &MasterCore::contains)
      .def("under_construction", &MasterCore::under_construction)
      .def("file_count", &MasterCore::file_count)
      .def("paths", &MasterCore::paths, py::arg("prefix") = "", py::arg("visible_only") = false)
      .def("files_pb", [](MasterCore& c, const std::string& prefix) {
        py::list out;
        for (auto& s : c.files_pb(prefix)) out.append(py::bytes(s));
        return out;
      }, py::arg("prefix") = "")
      .def("find_block", [](MasterCore& c, const std::string& id) -> py::object {
        std::string out;
        if (!c.find_block(id, &out)) return py::none();
        return py::bytes(out);
      })
      .def("has_block", &MasterCore::has_block)
      .def("total_blocks", &MasterCore::total_blocks)
      .def("tx_record", &MasterCore::tx_record)
      .def("tx_records", &MasterCore::tx_records)
      .def("tx_lock", &MasterCore::tx_lock)
      .def("shuffling_prefixes", &MasterCore::shuffling_prefixes)
      .def("take_request_counts", &MasterCore::take_request_counts)
      .def("take_gc", &MasterCore::take_gc)
      .def("heal_scan", [](const MasterCore& c, int rf, const std::vector<std::string>& live,
                           const std::map<std::string, std::vector<std::string>>& bad,
                           const std::set<std::pair<std::string, std::string>>& queued) {
        std::vector<MasterCore::HealAction> acts;
        {
          py::gil_scoped_release r;
          acts = c.heal_scan(rf, live, bad, queued);
        }
        py::list out;
        for (auto& a : acts)
          out.append(py::make_tuple(a.reconstruct, a.queue_on, a.block_id, a.target, a.shard_index, a.ec_data,
                                    a.ec_parity, a.sources, a.original_size));
        return out;
      })
      .def("pick_block", [](const MasterCore& c, const std::string& src, const std::string& dst,
                            std::optional<std::string> prefix) {
        py::gil_scoped_release r;
        return c.pick_block(src, dst, prefix ? &*prefix : nullptr);
      }, py::arg("src"), py::arg("dst"), py::arg("prefix") = py::none())
      .def("tiering_scan", [](const MasterCore& c, uint64_t now_ms, uint64_t cold_ms) {
        std::vector<MasterCore::ColdFile> v;
        {
          py::gil_scoped_release r;
          v = c.tiering_scan(now_ms, cold_ms);
        }
        py::list out;
        for (auto& f : v) out.append(py::make_tuple(f.path, f.blocks));
        return out;
      })
      .def("ec_candidates", [](const MasterCore& c, uint64_t now_ms, uint64_t ec_ms) {
        std::vector<std::string> v;
        {
          py::gil_scoped_release r;
          v = c.ec_candidates(now_ms, ec_ms);
        }
        py::list out;
        for (auto& s : v) out.append(py::bytes(s));
        return out;
      })
      .def("snapshot", &MasterCore::snapshot, py::call_guard<py::gil_scoped_release>())
      .def("restore", &MasterCore::restore, py::call_guard<py::gil_scoped_release>())
      .def("apply", [](MasterCore& c, uint64_t idx, const std::string& cmd) {
        return c.apply({{idx, cmd}}).front();  // tests: apply one command outside Raft
      })
      .def("enable_native_2pc", [](MasterCore& c, bool tls, const std::string& ca, const std::string& domain) {
             std::shared_ptr<TlsContext> t;
             if (tls) {
               std::string err;
               t = TlsContext::client(ca, domain, &err);
               if (!t) throw std::runtime_error(err);
             }
             auto pool = std::make_shared<GrpcChannelPool>(5000, std::move(t));
             c.enable_native_2pc([pool](const std::string& target, const std::string& path, const std::string& req,
                                        int timeout_ms) {
               return pool->call(target, path, req, t_request_id, timeout_ms);
             });
           }, py::arg("tls") = false, py::arg("ca") = "", py::arg("domain") = "")
      .def("txn_stats", [](const MasterCore& c) { return c.txn_stats().dump(); })
      .def("queue_command", [](MasterCore& c, const std::string& addr, py::bytes cmd) {
        c.queue_command(addr, std::string(cmd));
      })
      .def("take_commands", [](MasterCore& c, const std::string& addr) {
        py::list out;
        for (auto& s : c.take_commands(addr)) out.append(py::bytes(s));
        return out;
      })
      .def("peek_commands", [](const MasterCore& c) {
        py::dict out;
        for (auto& kv : c.peek_commands()) {
          py::list l;
          for (auto& s : kv.second) l.append(py::bytes(s));
          out[py::str(kv.first)] = l;
        }
        return out;
      })
      .def("bad_blocks", &MasterCore::bad_blocks)
      .def("add_bad_block", &MasterCore::add_bad_block)
      .def("take_ec_reports", &MasterCore::take_ec_reports)
      .def("take_heal_request", &MasterCore::take_heal_request)
      .def_property_readonly("requests", &MasterCore::requests)
      .def_property_readonly("heartbeats", &MasterCore::heartbeats);

  m.def("select_servers_rack_aware", [](MasterCore& c, size_t n, const std::string& preferred) {
    return select_servers_rack_aware(c.chunk_servers(), n, preferred);
  });

  py::class_<LocalRpcServer>(m, "MasterLocalServer")
      .def(py::init([](const std::string& name, std::shared_ptr<MasterCore> core, py::object fallback) {
             auto fb = std::make_shared<PyRef>(std::move(fallback));
             static const std::string kPrefix = "/dfs.MasterService/";
             LocalRpcServer::Handler h = [core, fb](const std::string& path, const std::string& rid,
                                                    const std::string& payload, std::string* out) -> int {
               if (path.compare(0, kPrefix.size(), kPrefix) == 0) {
                 std::string method = path.substr(kPrefix.size());
                 if (core->native_method(method)) {
                   int code = core->handle(method, payload, out);
                   if (code != MasterCore::kDecline) return code;
                   out->clear();
                 }
               }
               // everything else runs the Python service handler on its event loop
               py::gil_scoped_acquire g;
               try {
                 py::tuple r = fb->obj(path, rid, py::bytes(payload));
                 *out = r[1].cast<std::string>();
                 return r[0].cast<int>();
               } catch (py::error_already_set& e) {
                 *out = e.what();
                 return 13;
               }
             };
             return std::make_unique<LocalRpcServer>(name, std::move(h));
           }),
           py::keep_alive<1, 3>())
      .def("start", [](LocalRpcServer& s) {
        std::string err;
        bool ok = s.start(&err);
        return py::make_tuple(ok, err);
      })
      .def("stop", &LocalRpcServer::stop, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("requests", &LocalRpcServer::requests);

  // MasterService over native HTTP/2 gRPC (grpc_server.cpp): the methods MasterCore serves
  // natively (CreateFile, AllocateBlock, CompleteFile, GetFileInfo, ...) never touch Python;
  // the rest run the grpcio handlers through the same fallback as the local listener.
  struct NativeGrpcMaster {
    std::shared_ptr<PyRef> fallback;
    std::unique_ptr<GrpcServer> srv;
    std::atomic<uint64_t> native_calls{0}, fallback_calls{0}, raft_calls{0};
  };
  py::class_<NativeGrpcMaster>(m, "NativeGrpcMasterServer")
      .def(py::init([](std::shared_ptr<MasterCore> core, const std::string& host, int port, py::object fallback,
                       int workers, const std::string& tls_cert, const std::string& tls_key) {
             auto n = std::make_unique<NativeGrpcMaster>();
             n->fallback = std::make_shared<PyRef>(std::move(fallback));
             auto fb = n->fallback;
             NativeGrpcMaster* self = n.get();
             static const std::string kPrefix = "/dfs.MasterService/";
             static const std::string kRaft = "/dfs.RaftPeer/";
             n->srv = std::make_unique<GrpcServer>(host, port, [core, fb, self](const GrpcCall& c) -> GrpcReply {
               if (c.path.compare(0, kRaft.size(), kRaft) == 0) {  // Raft peer RPC: no Python at all
                 GrpcReply r;
                 r.status = core->raft_rpc(c.path.substr(kRaft.size()), c.message, &r.message);
                 self->raft_calls++;
                 return r;
               }
               if (c.path.compare(0, kPrefix.size(), kPrefix) == 0) {
                 std::string method = c.path.substr(kPrefix.size());
                 if (core->native_method(method)) {
                   RequestScope scope(c.request_id);
                   GrpcReply r;
                   r.status = core->handle(method, c.message, &r.message);
                   if (r.status != MasterCore::kDecline) {
                     self->native_calls++;
                     return r;
                   }
                 }
               }
               self->fallback_calls++;
               py::gil_scoped_acquire g;
               try {
                 py::tuple r = fb->obj(c.path, c.request_id, py::bytes(c.message));
                 return GrpcReply{r[0].cast<int>(), r[1].cast<std::string>()};
               } catch (py::error_already_set& e) {
                 return GrpcReply{13, std::string("python handler failed: ") + e.what()};
               }
             }, workers);
             if (!tls_cert.empty()) {
               std::string err;
               auto t = TlsContext::server(tls_cert, tls_key, &err);
               if (!t) throw std::runtime_error(err);
               n->srv->set_tls(std::move(t));
             }
             return n;
           }),
           py::arg("core"), py::arg("host"), py::arg("port"), py::arg("fallback"), py::arg("workers") = 64,
           py::arg("tls_cert") = "", py::arg("tls_key") = "")
      .def("start", [](NativeGrpcMaster& n) {
        std::string err;
        bool ok = n.srv->start(&err);
        return py::make_tuple(ok, err);
      })
      .def("stop", [](NativeGrpcMaster& n) {
        py::gil_scoped_release r;
        n.srv->stop();
      })
      .def_property_readonly("port", [](NativeGrpcMaster& n) { return n.srv->port(); })
      .def("stats", [](NativeGrpcMaster& n) {
        py::dict d;
        d["native_grpc_calls"] = n.srv->calls();
        d["native_grpc_native"] = n.native_calls.load();
        d["native_grpc_fallback"] = n.fallback_calls.load();
        d["native_raft_rpcs"] = n.raft_calls.load();
        return d;
      });

  // ---------------- native S3 front end (csrc/s3_front.cpp)
  // S3 audit log writer (C56): records from the gateway and, through the ingest socket, from
  // the gateway's other workers and the native front, in one HMAC chain
  py::class_<AuditLog>(m, "AuditLog")
      .def(py::init<std::string, int, int, std::string, size_t, int, bool>(), py::arg("path"),
           py::arg("retention_days") = 30, py::arg("batch_size") = 100, py::arg("hmac_secret") = "",
           py::arg("capacity") = 10000, py::arg("flush_interval_ms") = 5000, py::arg("sync") = false)
      .def("log", &AuditLog::log, py::call_guard<py::gil_scoped_release>())
      .def("start_ingest", &AuditLog::start_ingest)
      .def("flush", &AuditLog::flush, py::arg("timeout_ms") = 10000, py::call_guard<py::gil_scoped_release>())
      .def("close", &AuditLog::close, py::call_guard<py::gil_scoped_release>())
      .def("cleanup", &AuditLog::cleanup, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("head", &AuditLog::head)
      .def("stats", [](const AuditLog& a) {
        py::dict d;
        d["total"] = a.total();
        d["dropped"] = a.dropped();
        d["flush_errors"] = a.flush_errors();
        d["committed"] = a.committed();
        d["ingested"] = a.ingested();
        return d;
      });

  // the file-system side of a gateway on another host (front_store.h): private slots, gRPC to
  // the masters and chunkservers
  py::class_<RemoteFrontStore>(m, "RemoteFrontStore")
      .def(py::init([](const std::string& shard_map_json, std::vector<std::string> masters, size_t slots,
                       size_t slot_bytes, const std::string& ca_cert, const std::string& domain_name, bool tls) {
             std::shared_ptr<TlsContext> ctx;
             if (tls) {
               std::string err;
               ctx = TlsContext::client(ca_cert, domain_name, &err);
               if (!ctx) throw std::runtime_error(err);
             }
             return std::make_unique<RemoteFrontStore>(shard_map_json, masters, slots, slot_bytes, 120000, ctx);
           }),
           py::arg("shard_map_json"), py::arg("masters"), py::arg("slots") = 32, py::arg("slot_bytes") = 16u << 20,
           py::arg("ca_cert") = "", py::arg("domain_name") = "", py::arg("tls") = false)
      .def("set_routing", &RemoteFrontStore::set_routing)
      .def("stats", [](RemoteFrontStore& s) {
        py::dict d;
        d["writes"] = s.client().writes();
        d["reads"] = s.client().reads();
        d["connects"] = s.client().connects();
        return d;
      });

  py::class_<S3Front>(m, "S3Front")
      .def(py::init([](py::object client, const std::string& host, int port, const std::string& backend, int workers,
                       bool auth_enabled, const std::string& region, const std::string& access_key,
                       const std::string& secret_key, bool allow_unsigned, const std::string& audit_socket,
                       bool sse_enabled, bool metadata_sidecar, const std::string& policy_epoch,
                       const std::string& tls_cert, const std::string& tls_key, py::bytes sse_kek,
                       std::map<uint32_t, py::bytes> sts_keys, const std::string& iam_config, bool require_tls) {
             S3FrontConfig c;
             c.require_tls = require_tls;
             for (auto& kv : sts_keys) c.sts_keys[kv.first] = std::string(kv.second);
             c.iam_config = iam_config;
             c.sse_kek = std::string(sse_kek);
             c.policy_epoch_path = policy_epoch;
             c.tls_cert = tls_cert;
             c.tls_key = tls_key;
             c.host = host;
             c.port = port;
             c.backend = backend;
             c.workers = workers;
             c.auth_enabled = auth_enabled;
             c.region = region;
             c.access_key = access_key;
             c.secret_key = secret_key;
             c.allow_unsigned_payload = allow_unsigned;
             c.audit_socket = audit_socket;
             c.sse_enabled = sse_enabled;
             c.metadata_sidecar = metadata_sidecar;
             if (py::isinstance<RemoteFrontStore>(client))
               return std::make_unique<S3Front>(c, static_cast<FrontStore*>(client.cast<RemoteFrontStore*>()));
             return std::make_unique<S3Front>(c, client.cast<FastClient*>());
           }),
           py::arg("fast_client"), py::arg("host"), py::arg("port"), py::arg("backend"), py::arg("workers") = 32,
           py::arg("auth_enabled") = false, py::arg("region") = "us-east-1", py::arg("access_key") = "",
           py::arg("secret_key") = "", py::arg("allow_unsigned_payload") = true, py::arg("audit_socket") = "",
           py::arg("sse_enabled") = false, py::arg("metadata_sidecar") = false, py::arg("policy_epoch") = "",
           py::arg("tls_cert") = "", py::arg("tls_key") = "", py::arg("sse_kek") = py::bytes(),
           py::arg("sts_keys") = std::map<uint32_t, py::bytes>(), py::arg("iam_config") = "",
           py::arg("require_tls") = false, py::keep_alive<1, 2>())
      .def("drop_policies", &S3Front::drop_policies, py::call_guard<py::gil_scoped_release>())
      .def("start", [](S3Front& f) {
        std::string err;
        bool ok;
        {
          py::gil_scoped_release r;
          ok = f.start(&err);
        }
        return py::make_tuple(ok, err);
      })
      .def("stop", &S3Front::stop, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("port", &S3Front::port)
      .def("stats", [](S3Front& f) {
        S3FrontStats s = f.stats();
        py::dict d;
        d["connections"] = s.connections;
        d["requests"] = s.requests;
        d["native"] = s.native;
        d["proxied"] = s.proxied;
        d["puts"] = s.puts;
        d["parts"] = s.parts;
        d["gets"] = s.gets;
        d["range_gets"] = s.range_gets;
        d["heads"] = s.heads;
        d["mpu_gets"] = s.mpu_gets;
        d["bytes_in"] = s.bytes_in;
        d["bytes_out"] = s.bytes_out;
        d["auth_native"] = s.auth_native;
        d["policy_native"] = s.policy_native;
        d["audit_sent"] = s.audit_sent;
        d["audit_dropped"] = s.audit_dropped;
        d["tls_handshakes"] = s.tls_handshakes;
        d["tls_failures"] = s.tls_failures;
        d["sse_puts"] = s.sse_puts;
        d["sse_gets"] = s.sse_gets;
        d["iam_native"] = s.iam_native;
        d["lists"] = s.lists;
        d["mpu_completes"] = s.mpu_completes;
        d["mpu_initiates"] = s.mpu_initiates;
        d["deletes"] = s.deletes;
        d["multi_deletes"] = s.multi_deletes;
        d["deleted_keys"] = s.deleted_keys;
        d["mpu_aborts"] = s.mpu_aborts;
        d["copies"] = s.copies;
        d["copy_bytes"] = s.copy_bytes;
        d["chunked_puts"] = s.chunked_puts;
        d["chunk_sigs"] = s.chunk_sigs;
        d["chunk_sig_failures"] = s.chunk_sig_failures;
        d["presigned"] = s.presigned;
        d["bucket_ops"] = s.bucket_ops;
        d["sts_issued"] = s.sts_issued;
        d["standalone_answers"] = s.standalone_answers;
        d["standalone_reasons"] = s.standalone_reasons;
        d["auth_results"] = s.auth_results;
        d["by_status"] = s.by_status;
        d["proxy_reasons"] = s.proxy_reasons;
        return d;
      });

  // ---------------- IAM / bucket policy engine (csrc/s3_policy.cpp; parity tests)
  m.def("s3_wildcard", &s3policy::matches_wildcard);
  m.def("s3_bucket_policy_eval", [](const std::string& doc, std::optional<std::string> principal, const std::string& action,
                                    const std::string& resource) {
    s3policy::BucketPolicy p;
    try {
      p = s3policy::BucketPolicy::parse(doc);
    } catch (const std::exception& e) {
      throw py::value_error(e.what());
    }
    switch (p.evaluate(principal ? &*principal : nullptr, action, resource)) {
      case s3policy::PolicyResult::Allow: return std::string("Allow");
      case s3policy::PolicyResult::ExplicitDeny: return std::string("ExplicitDeny");
      default: return std::string("NotApplicable");
    }
  });
  m.def("s3_iam_eval", [](const std::string& doc, const std::string& action, const std::string& resource,
                          const std::string& role_arn, const std::string& principal_id, std::vector<std::string> groups,
                          std::map<std::string, std::string> claims) {
    s3policy::IamPolicy p;
    try {
      p = s3policy::IamPolicy::parse(doc);
    } catch (const std::exception& e) {
      throw py::value_error(e.what());
    }
    s3policy::Context ctx{principal_id, std::move(groups), std::move(claims)};
    return py::make_tuple(p.evaluate(action, resource, role_arn, ctx), p.can_assume_role(role_arn, ctx));
  });
  m.def("s3_resolve_action", [](const std::string& method, const std::string& path, std::vector<std::string> keys) {
    auto r = s3policy::resolve_action_and_resource(method, path, keys);
    return py::make_tuple(r.first, r.second);
  });

  // ---------------- native client data path (co-located writers/readers)
  py::class_<FastClient>(m, "FastClient")
      .def(py::init<std::string, std::string, size_t, size_t, int>(), py::arg("fastpath_socket"),
           py::arg("local_chunkserver"), py::arg("arena_bytes") = 256u << 20, py::arg("slot_bytes") = 16u << 20,
           py::arg("hash_threads") = 8)
      .def_property_readonly("ok", &FastClient::ok)
      .def_property_readonly("arena_path", &FastClient::arena_path)
      .def_property_readonly("md5_mode", &FastClient::md5_mode)
      .def_property_readonly("writes", &FastClient::writes)
      .def_property_readonly("reads", &FastClient::reads)
      .def("set_host_aliases", &FastClient::set_host_aliases)
      .def("set_routing", &FastClient::set_routing, py::call_guard<py::gil_scoped_release>())
      .def("write", [](FastClient& c, const std::string& path, py::buffer data, const std::string& rid,
                         const std::map<std::string, std::string>& attrs) {
        py::buffer_info bi = data.request();
        int replicas = 0;
        std::string msg;
        FastClient::Times t;
        FastClient::Status st;
        {
          py::gil_scoped_release r;
          st = c.write(path, static_cast<const uint8_t*>(bi.ptr), static_cast<size_t>(bi.size * bi.itemsize),
                       &replicas, &msg, &t, rid, attrs.empty() ? nullptr : &attrs);
        }
        return py::make_tuple(static_cast<int>(st), replicas, msg,
                              py::make_tuple(t.crc, t.create, t.write, t.md5_wait, t.complete));
      }, py::arg("path"), py::arg("data"), py::arg("request_id") = "",
         py::arg("attributes") = std::map<std::string, std::string>())
      .def("read", [](FastClient& c, const std::string& path, const std::string& rid, uint64_t offset,
                        uint64_t length) {
        int64_t slot = -1;
        uint64_t n = 0;
        std::string msg;
        FastClient::Times t;
        FastClient::Status st;
        {
          py::gil_scoped_release r;
          st = c.read(path, &slot, &n, &msg, &t, rid, offset, length);
        }
        py::object data = py::none();
        if (st == FastClient::Ok) {
          PyObject* o = PyBytes_FromStringAndSize(nullptr, static_cast<Py_ssize_t>(n));
          if (!o) throw py::error_already_set();
          data = py::reinterpret_steal<py::object>(o);
          char* dst = PyBytes_AS_STRING(o);
          {
            py::gil_scoped_release r;  // the new object is not visible to anyone else yet
            if (n) std::memcpy(dst, c.slot_ptr(slot), n);
            if (slot >= 0) c.release(slot);
          }
        }
        return py::make_tuple(static_cast<int>(st), data, msg, py::make_tuple(t.getinfo, t.read));
      }, py::arg("path"), py::arg("request_id") = "", py::arg("offset") = 0, py::arg("length") = 0)
      .def("write_ec", [](FastClient& c, const std::string& path, py::buffer data, int k, int m, const std::string& rid) {
        py::buffer_info bi = data.request();
        std::string msg;
        FastClient::Status st;
        {
          py::gil_scoped_release r;
          st = c.write_ec(path, static_cast<const uint8_t*>(bi.ptr), static_cast<size_t>(bi.size * bi.itemsize), k, m,
                          &msg, rid);
        }
        return py::make_tuple(static_cast<int>(st), msg);
      }, py::arg("path"), py::arg("data"), py::arg("k"), py::arg("m"), py::arg("request_id") = "")
      .def_property_readonly("ec_gpu_ops", &FastClient::ec_gpu_ops)
      .def_property_readonly("ec_cpu_ops", &FastClient::ec_cpu_ops)
      .def_property_readonly("ec_degraded_reads", &FastClient::ec_degraded_reads)
      .def_property_readonly("ec_device_writes", &FastClient::ec_device_writes)
      .def_property_readonly("ec_device_reads", &FastClient::ec_device_reads)
      .def_property_readonly("ec_host_fallbacks", &FastClient::ec_host_fallbacks)
      .def("remove", [](FastClient& c, const std::string& path, const std::string& rid) {
        std::string msg;
        FastClient::Status st;
        {
          py::gil_scoped_release r;
          st = c.remove(path, &msg, rid);
        }
        return py::make_tuple(static_cast<int>(st), msg);  // NotHandled: the caller's gRPC path
      }, py::arg("path"), py::arg("request_id") = "")
      .def("bench_writes", &bench_writes<FastClient>, py::arg("paths"), py::arg("payloads"), py::arg("concurrency"))
      .def("bench_reads", &bench_reads_fast, py::arg("paths"), py::arg("expected"), py::arg("concurrency"));

  // ---------------- native remote client (every RPC over gRPC/TCP, client_remote.h)
  py::class_<RemoteClient>(m, "RemoteClient")
      .def(py::init([](int hash_threads, int timeout_ms, bool tls, const std::string& ca, const std::string& domain) {
             std::shared_ptr<TlsContext> t;
             if (tls) {
               std::string err;
               t = TlsContext::client(ca, domain, &err);
               if (!t) throw std::runtime_error(err);
             }
             return std::make_unique<RemoteClient>(hash_threads, timeout_ms, std::move(t));
           }),
           py::arg("hash_threads") = 4, py::arg("timeout_ms") = 120000, py::arg("tls") = false, py::arg("ca_cert") = "",
           py::arg("domain_name") = "")
      .def_property_readonly("writes", &RemoteClient::writes)
      .def_property_readonly("reads", &RemoteClient::reads)
      .def_property_readonly("connects", &RemoteClient::connects)
      .def_property_readonly("hedged", &RemoteClient::hedged)
      .def_property_readonly("ec_degraded_reads", &RemoteClient::ec_degraded_reads)
      .def("write_ec", [](RemoteClient& c, const std::string& path, py::buffer data, int k, int m, const std::string& rid) {
        py::buffer_info bi = data.request();
        std::string msg;
        FastClient::Status st;
        {
          py::gil_scoped_release r;
          st = c.write_ec(path, static_cast<const uint8_t*>(bi.ptr), static_cast<size_t>(bi.size * bi.itemsize), k, m,
                          &msg, rid);
        }
        return py::make_tuple(static_cast<int>(st), msg);
      }, py::arg("path"), py::arg("data"), py::arg("k"), py::arg("m"), py::arg("request_id") = "")
      .def("set_hedge_delay", &RemoteClient::set_hedge_delay)
      .def("set_host_aliases", &RemoteClient::set_host_aliases)
      .def("set_routing", &RemoteClient::set_routing, py::call_guard<py::gil_scoped_release>())
      .def("write", [](RemoteClient& c, const std::string& path, py::buffer data, const std::string& rid,
                         const std::map<std::string, std::string>& attrs) {
        py::buffer_info bi = data.request();
        int replicas = 0;
        std::string msg;
        FastClient::Times t;
        FastClient::Status st;
        {
          py::gil_scoped_release r;
          st = c.write(path, static_cast<const uint8_t*>(bi.ptr), static_cast<size_t>(bi.size * bi.itemsize),
                       &replicas, &msg, &t, rid, attrs.empty() ? nullptr : &attrs);
        }
        return py::make_tuple(static_cast<int>(st), replicas, msg,
                              py::make_tuple(t.crc, t.create, t.write, t.md5_wait, t.complete));
      }, py::arg("path"), py::arg("data"), py::arg("request_id") = "",
         py::arg("attributes") = std::map<std::string, std::string>())
      .def("read", [](RemoteClient& c, const std::string& path, const std::string& rid, uint64_t offset,
                          uint64_t length) {
        std::string out, msg;
        FastClient::Times t;
        FastClient::Status st;
        {
          py::gil_scoped_release r;
          st = c.read(path, &out, &msg, &t, rid, offset, length);
        }
        py::object data = st == FastClient::Ok ? py::object(py::bytes(out)) : py::object(py::none());
        return py::make_tuple(static_cast<int>(st), data, msg, py::make_tuple(t.getinfo, t.read));
      }, py::arg("path"), py::arg("request_id") = "", py::arg("offset") = 0, py::arg("length") = 0)
      .def("bench_writes", &bench_writes<RemoteClient>, py::arg("paths"), py::arg("payloads"), py::arg("concurrency"))
      .def("bench_reads", &bench_reads_remote, py::arg("paths"), py::arg("expected"), py::arg("concurrency"));

  // raw native gRPC unary call (interop tests)
  m.def("grpc_call", [](const std::string& target, const std::string& path, py::bytes req, const std::string& rid,
                        int timeout_ms) {
    static GrpcChannelPool pool;
    std::string in = req;
    GrpcResult r;
    {
      py::gil_scoped_release g;
      r = pool.call(target, path, in, rid, timeout_ms);
    }
    return py::make_tuple(r.transport_ok, r.status, py::bytes(r.message));
  }, py::arg("target"), py::arg("path"), py::arg("request"), py::arg("request_id") = "", py::arg("timeout_ms") = 10000);
}
