// unit_tests — native Tier-1/Tier-2 tests of the C++ runtime, no GPU needed.
//
// SURVEY §4 asks for the reference's in-module unit tests and in-process simulations
// (dfs/metaserver/tests/{raft_logic,membership_change_unit,network_partition}_tests.rs,
// dfs/common/src/{sharding,erasure}.rs tests, chunkserver.rs:1091) to exist natively. This
// binary exercises the runtime objects directly: JSON, shard map, joint-majority math,
// extent allocator, CRC-32 (+ combine / slices), GF(2^8) Reed-Solomon, WAL torn tails,
// the node-wide disk gate, and real Raft nodes (1 and 3 of them) talking over an
// in-memory transport with a partition matrix.
//
//   unit_tests [filter]   -> "ok <name>" / "FAIL <name>: <why>" lines, exit 1 on any failure
#include <fcntl.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <filesystem>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <random>
#include <set>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "audit_json.h"
#include "audit_log.h"
#include "aws_chunked.h"
#include "crc32.h"
#include "disk_gate.h"
#include "extent_alloc.h"
#include "gf256.h"
#include "grpc_client.h"
#include "grpc_server.h"
#include "http_lite.h"
#include "journal.h"
#include "json.h"
#include "lin_checker.h"
#include "master_core.h"
#include "md5_mb.h"
#include "p2p_transport.h"
#include "raft.h"
#include "shard_map.h"
#include "sigv4.h"
#include "sts.h"
#include "wal.h"

using namespace dfs;

namespace {

struct Failure : std::runtime_error {
  using std::runtime_error::runtime_error;
};

#define CHECK(cond)                                                                             \
  do {                                                                                          \
    if (!(cond)) throw Failure(std::string(__FILE__ ":") + std::to_string(__LINE__) + " " #cond); \
  } while (0)

std::vector<std::pair<std::string, std::function<void()>>>& registry() {
  static std::vector<std::pair<std::string, std::function<void()>>> r;
  return r;
}
struct Reg {
  Reg(const char* n, std::function<void()> f) { registry().emplace_back(n, std::move(f)); }
};
#define TEST(name)                         \
  static void name();                      \
  static Reg reg_##name(#name, name);      \
  static void name()

std::string tmpdir(const std::string& tag) {
  std::string d = std::filesystem::temp_directory_path().string() + "/dfs_ut_" + tag + "_" +
                  std::to_string(::getpid());
  std::filesystem::remove_all(d);
  std::filesystem::create_directories(d);
  return d;
}

bool eventually(const std::function<bool()>& f, double secs) {
  auto end = std::chrono::steady_clock::now() + std::chrono::duration<double>(secs);
  while (std::chrono::steady_clock::now() < end) {
    if (f()) return true;
    std::this_thread::sleep_for(std::chrono::milliseconds(10));
  }
  return f();
}

// ------------------------------------------------------------------------------- JSON
TEST(json_roundtrip_keeps_order_types_and_escapes) {
  std::string text =
      R"({"z":1,"a":[true,false,null,-7,2.5,"q\"\\\né"],"m":{"k":"v","n":{}},"big":9007199254740993})";
  Json j = Json::parse(text);
  CHECK(j["z"].as_int() == 1);
  CHECK(j["a"].size() == 6 && j["a"][0].as_bool() && j["a"][2].is_null());
  CHECK(j["a"][3].is_int() && j["a"][3].as_int() == -7);
  CHECK(!j["a"][4].is_int() && j["a"][4].as_double() == 2.5);
  CHECK(j["a"][5].as_string() == "q\"\\\n\xc3\xa9");
  CHECK(j["big"].as_int() == 9007199254740993LL);  // no double rounding
  CHECK(j["missing"].is_null());
  Json k = Json::parse(j.dump());
  CHECK(k == j);
  CHECK(j.dump().find("\"z\"") < j.dump().find("\"a\""));  // insertion order survives
}

TEST(json_copy_on_write_and_set_erase) {
  Json a = Json::object();
  a.set("x", 1);
  Json b = a;
  b.set("x", 2);
  b.set("y", "s");
  CHECK(a["x"].as_int() == 1 && !a.has("y"));
  CHECK(b["x"].as_int() == 2 && b.erase("y") && !b.has("y"));
}

TEST(json_rejects_malformed_text) {
  for (const char* bad : {"{", "[1,]", "{\"a\" 1}", "tru", "\"unterminated", "{} x"}) {
    bool threw = false;
    try {
      Json::parse(bad);
    } catch (const std::exception&) {
      threw = true;
    }
    CHECK(threw);
  }
}

// ------------------------------------------------------------------------------- sharding
TEST(shard_map_range_split_routing) {
  ShardMap m = ShardMap::new_range();
  m.add_shard("shard-0", {});
  CHECK(m.split_shard("/m", "shard-1", {}));
  CHECK(m.split_shard("/t", "shard-2", {}));
  CHECK(m.get_shard("/apple") == "shard-1");
  CHECK(m.get_shard("/mango") == "shard-2");
  CHECK(m.get_shard("/zebra") == "shard-0");
  CHECK(!m.split_shard("/t", "shard-3", {}));
  ShardMap back = ShardMap::from_json(m.to_json());
  for (const char* k : {"/apple", "/mango", "/orange", "/zebra", "/"}) CHECK(back.get_shard(k) == m.get_shard(k));
}

TEST(shard_map_consistent_hash_is_stable_and_minimal_on_removal) {
  ShardMap m = ShardMap::new_consistent_hash(100);
  for (const char* s : {"s1", "s2", "s3"}) m.add_shard(s, {std::string(s) + ":1"});
  std::map<std::string, std::string> before;
  for (int i = 0; i < 2000; ++i) before["/k" + std::to_string(i)] = m.get_shard("/k" + std::to_string(i));
  std::set<std::string> used;
  for (auto& kv : before) used.insert(kv.second);
  CHECK(used.size() == 3);
  m.remove_shard("s2");
  for (auto& kv : before)
    if (kv.second != "s2") CHECK(m.get_shard(kv.first) == kv.second);  // only s2's keys move
  CHECK(m.peers("s1") && (*m.peers("s1"))[0] == "s1:1");
}

// ------------------------------------------------------------------------------- membership
TEST(joint_majority_needs_both_configs) {
  raft::ClusterConfig c;
  c.old_members = {{1, "a"}, {2, "b"}, {3, "c"}};
  c.members = {{3, "c"}, {4, "d"}, {5, "e"}};
  c.joint = true;
  CHECK(!c.has_joint_majority({1, 2}));     // old majority only
  CHECK(!c.has_joint_majority({4, 5}));     // new majority only
  CHECK(c.has_joint_majority({1, 3, 4}));   // both
  CHECK(c.has_joint_majority({1, 2, 4, 5}));
  CHECK(c.is_voter(1) && c.is_voter(5) && !c.is_voter(9));
  raft::ClusterConfig s;
  s.members = {{1, "a"}, {2, "b"}, {3, "c"}, {4, "d"}, {5, "e"}};
  CHECK(!s.has_joint_majority({1, 2}) && s.has_joint_majority({1, 2, 3}));
  raft::ClusterConfig back = raft::ClusterConfig::from_json(c.to_json());
  CHECK(back.joint && back.members == c.members && back.old_members == c.old_members);
}

// ------------------------------------------------------------------------------- allocator
TEST(extent_allocator_first_fit_and_coalescing) {
  ExtentAllocator a(1000);
  int64_t x = a.alloc(100), y = a.alloc(200), z = a.alloc(300);
  CHECK(x == 0 && y == 100 && z == 300 && a.used() == 600);
  CHECK(a.alloc(500) == -1);
  a.free(100, 200);
  CHECK(a.alloc(150) == 100);  // first fit reuses the hole
  a.free(100, 150);
  a.free(0, 100);
  a.free(300, 300);
  CHECK(a.used() == 0 && a.largest_free() == 1000);  // everything coalesced back
}

// ------------------------------------------------------------------------------- CRC
TEST(crc32_golden_combine_and_slices) {
  const char* s = "123456789";
  CHECK(crc32(reinterpret_cast<const uint8_t*>(s), 9) == 0xCBF43926u);
  std::vector<uint8_t> buf(5000);
  std::mt19937 g(1);
  for (auto& b : buf) b = static_cast<uint8_t>(g());
  uint32_t whole = crc32(buf.data(), buf.size());
  uint32_t a = crc32(buf.data(), 1234), b = crc32(buf.data() + 1234, buf.size() - 1234);
  CHECK(crc32_combine(a, b, buf.size() - 1234) == whole);
  std::vector<uint32_t> sl(num_slices(buf.size()));
  crc32_slices(buf.data(), buf.size(), sl.data());
  CHECK(sl.size() == 10);  // 512-byte slices, last one partial
  CHECK(sl[0] == crc32(buf.data(), 512));
  CHECK(crc32_from_slices(sl.data(), buf.size()) == whole);
}

// ------------------------------------------------------------------------------- erasure
TEST(reed_solomon_recovers_any_m_losses) {
  const int k = 4, m = 2;
  const size_t len = 777;
  gf::Matrix enc = gf::rs_matrix(k, m);
  for (int r = 0; r < k; ++r)
    for (int c = 0; c < k; ++c) CHECK(enc[r][c] == (r == c ? 1 : 0));  // systematic
  std::vector<std::vector<uint8_t>> shards(k + m, std::vector<uint8_t>(len));
  std::mt19937 g(7);
  for (int i = 0; i < k; ++i)
    for (auto& b : shards[i]) b = static_cast<uint8_t>(g());
  gf::Matrix parity(enc.begin() + k, enc.end());
  std::vector<const uint8_t*> in;
  std::vector<uint8_t*> out;
  for (int i = 0; i < k; ++i) in.push_back(shards[i].data());
  for (int i = 0; i < m; ++i) out.push_back(shards[k + i].data());
  gf::matmul_cpu(parity, in.data(), out.data(), len);
  for (int l1 = 0; l1 < k + m; ++l1)
    for (int l2 = l1 + 1; l2 < k + m; ++l2) {
      std::vector<int> present, wanted;
      for (int i = 0; i < k + m && static_cast<int>(present.size()) < k; ++i)
        if (i != l1 && i != l2) present.push_back(i);
      for (int w : {l1, l2})
        if (w < k) wanted.push_back(w);
      if (wanted.empty()) continue;
      gf::Matrix rows = gf::rs_decode_rows(k, m, present, wanted);
      std::vector<const uint8_t*> pin;
      for (int p : present) pin.push_back(shards[p].data());
      std::vector<std::vector<uint8_t>> rebuilt(wanted.size(), std::vector<uint8_t>(len));
      std::vector<uint8_t*> pout;
      for (auto& r : rebuilt) pout.push_back(r.data());
      gf::matmul_cpu(rows, pin.data(), pout.data(), len);
      for (size_t w = 0; w < wanted.size(); ++w) CHECK(rebuilt[w] == shards[wanted[w]]);
    }
  gf::Matrix inv = gf::invert(gf::Matrix(enc.begin() + 1, enc.begin() + 1 + k));
  CHECK(gf::multiply(inv, gf::Matrix(enc.begin() + 1, enc.begin() + 1 + k)) == gf::identity(k));
}

// ------------------------------------------------------------------------------- WAL
TEST(wal_replays_records_and_drops_a_torn_tail) {
  std::string d = tmpdir("wal");
  std::string p = d + "/log.wal";
  {
    Wal w(p, true);
    w.append({"one", "two"});
    w.append({std::string(3000, 'x')});
  }
  {
    Wal w(p, false);
    auto r = w.replay();
    CHECK(r.size() == 3 && r[0] == "one" && r[2].size() == 3000);
  }
  // the file is written out with zeros past the last frame (appends flush no metadata)
  const uint64_t end = (8 + 3) + (8 + 3) + (8 + 3000);
  CHECK(std::filesystem::file_size(p) > end);
  std::filesystem::resize_file(p, end - 10);  // crash mid-record
  {
    Wal w(p, false);
    auto r = w.replay();
    CHECK(r.size() == 2 && r[1] == "two");
    w.append({"three"});  // appends after the truncated tail
  }
  Wal w(p, false);
  auto r = w.replay();
  CHECK(r.size() == 3 && r[2] == "three");
  // a batch whose first frame is torn while later ones reached the disk: the later frames
  // must never reappear behind a shorter append that lands on the torn one
  {
    Wal w2(p, false);
    (void)w2.replay();
    w2.append({std::string(100, 'a'), "late-1", "late-2"});
  }
  {
    int fd = ::open(p.c_str(), O_RDWR);
    const uint64_t torn = end - 10 + 0;  // (the valid prefix after the first cut: "one", "two")
    (void)torn;
    // flip a payload byte of the 100-byte frame (it starts after "one", "two", "three")
    const off_t at = static_cast<off_t>((8 + 3) + (8 + 3) + (8 + 5) + 8 + 50);
    char c = 0;
    CHECK(::pread(fd, &c, 1, at) == 1);
    c ^= 0x5a;
    CHECK(::pwrite(fd, &c, 1, at) == 1);
    ::close(fd);
  }
  {
    Wal w3(p, false);
    auto r3 = w3.replay();
    CHECK(r3.size() == 3 && r3[2] == "three");
    w3.append({std::string(100, 'b')});  // the same size as the torn frame
  }
  Wal w4(p, false);
  auto r4 = w4.replay();
  CHECK(r4.size() == 4 && r4[3] == std::string(100, 'b'));
  std::filesystem::remove_all(d);
}

// ------------------------------------------------------------------------------- disk gate
TEST(disk_gate_caps_in_flight_writers) {
  std::string d = tmpdir("gate");
  DiskGate g(d, 3);
  CHECK(g.enabled() && g.slots() == 3);
  std::atomic<int> inflight{0}, peak{0};
  std::vector<std::thread> ts;
  for (int t = 0; t < 12; ++t)
    ts.emplace_back([&] {
      for (int i = 0; i < 20; ++i) {
        DiskGate::Slot s = g.acquire();
        int now = ++inflight;
        int p = peak.load();
        while (now > p && !peak.compare_exchange_weak(p, now)) {
        }
        std::this_thread::sleep_for(std::chrono::microseconds(200));
        --inflight;
      }
    });
  for (auto& t : ts) t.join();
  CHECK(peak.load() <= 3 && peak.load() >= 1);
  // deterministic wait (a loaded or sanitized run can serialize the threads above): with all
  // three slots held, a fourth writer must block until one is released
  {
    const uint64_t w0 = g.waits();
    std::vector<DiskGate::Slot> held;
    for (int k = 0; k < 3; ++k) held.push_back(g.acquire());
    std::atomic<bool> got{false};
    std::thread late([&] {
      DiskGate::Slot s = g.acquire();
      got = true;
    });
    std::this_thread::sleep_for(std::chrono::milliseconds(50));
    CHECK(!got.load());
    held.pop_back();
    late.join();
    CHECK(got.load() && g.waits() > w0);
  }
  std::filesystem::remove_all(d);
}

// ------------------------------------------------------------------------------- Raft
// In-memory cluster: Host::send calls the target node's handle() directly unless the
// partition matrix cuts the link. The state machine is an append-only list of commands.
struct Net {
  std::mutex mu;
  std::map<std::string, raft::Node*> nodes;
  std::set<std::pair<std::string, std::string>> cut;
  void isolate(const std::string& a, const std::vector<std::string>& all) {
    std::lock_guard<std::mutex> g(mu);
    for (auto& b : all)
      if (b != a) cut.insert({a, b}), cut.insert({b, a});
  }
  void heal() {
    std::lock_guard<std::mutex> g(mu);
    cut.clear();
  }
};

struct ListHost : raft::Host {
  std::string self;
  std::shared_ptr<Net> net;
  std::mutex mu;
  std::vector<std::string> applied;
  std::vector<std::string> apply(const std::vector<std::pair<uint64_t, std::string>>& cmds) override {
    std::lock_guard<std::mutex> g(mu);
    std::vector<std::string> out;
    for (auto& c : cmds) {
      if (c.second != "\"NoOp\"") applied.push_back(c.second);
      out.push_back(std::to_string(applied.size()));
    }
    return out;
  }
  std::string snapshot() override {
    std::lock_guard<std::mutex> g(mu);
    Json a = Json::array();
    for (auto& s : applied) a.push_back(s);
    return a.dump();
  }
  void restore(const std::string& state) override {
    std::lock_guard<std::mutex> g(mu);
    applied.clear();
    Json a = Json::parse(state);
    for (size_t i = 0; i < a.size(); ++i) applied.push_back(a[i].as_string());
  }
  bool send(const std::string& addr, const std::string& kind, const std::string& body, std::string* reply) override {
    raft::Node* n = nullptr;
    {
      std::lock_guard<std::mutex> g(net->mu);
      if (net->cut.count({self, addr})) return false;
      auto it = net->nodes.find(addr);
      if (it == net->nodes.end()) return false;
      n = it->second;
    }
    *reply = n->handle(kind, body);
    return true;
  }
  std::vector<std::string> snap() {
    std::lock_guard<std::mutex> g(mu);
    return applied;
  }
};

struct Cluster {
  std::shared_ptr<Net> net = std::make_shared<Net>();
  std::vector<std::shared_ptr<ListHost>> hosts;
  std::vector<std::unique_ptr<raft::Node>> nodes;
  std::vector<std::string> addrs;
  std::string dir;
  explicit Cluster(int n, const std::string& tag) {
    dir = tmpdir(tag);
    std::map<int, std::string> members;
    for (int i = 1; i <= n; ++i) {
      addrs.push_back("n" + std::to_string(i));
      members[i] = addrs.back();
    }
    for (int i = 1; i <= n; ++i) {
      raft::Options o;
      o.id = i;
      o.members = members;
      o.client_address = addrs[i - 1];
      o.dir = dir + "/" + addrs[i - 1];
      o.election_lo = 0.15;
      o.election_hi = 0.3;
      o.heartbeat = 0.03;
      o.sync = false;
      o.snapshot_threshold = 50;
      std::filesystem::create_directories(o.dir);
      auto h = std::make_shared<ListHost>();
      h->self = addrs[i - 1];
      h->net = net;
      hosts.push_back(h);
      nodes.push_back(std::make_unique<raft::Node>(o, h));
      net->nodes[addrs[i - 1]] = nodes.back().get();
    }
    for (auto& nd : nodes) nd->start();
  }
  ~Cluster() {
    for (auto& nd : nodes) nd->stop();
    std::filesystem::remove_all(dir);
  }
  int leader() {
    for (size_t i = 0; i < nodes.size(); ++i)
      if (nodes[i]->is_leader()) return static_cast<int>(i);
    return -1;
  }
  // commit-wait propose on node i; returns the Done code
  int propose(int i, const std::string& cmd, double timeout = 3.0) {
    auto st = std::make_shared<std::pair<std::atomic<int>, std::string>>();
    st->first = -1;
    nodes[i]->propose(cmd, [st](int code, const std::string& p) {
      st->second = p;
      st->first = code;
    });
    eventually([&] { return st->first.load() >= 0; }, timeout);
    return st->first.load();
  }
  // at whichever node leads now: a "not leader" answer (1, nothing appended) is retried at the
  // new leader, so an election that lands right after the first one (a loaded machine) is no
  // failure; any other answer is returned as is
  int propose_at_leader(const std::string& cmd, double timeout = 5.0) {
    int code = -1;
    eventually([&] {
      int l = leader();
      if (l < 0) return false;
      code = propose(l, cmd);
      return code != 1;
    }, timeout);
    return code;
  }
};

TEST(raft_single_node_commits_immediately) {
  Cluster c(1, "raft1");
  CHECK(eventually([&] { return c.leader() == 0; }, 3));
  for (int i = 0; i < 20; ++i) CHECK(c.propose(0, Json("cmd" + std::to_string(i)).dump()) == 0);
  CHECK(c.hosts[0]->snap().size() == 20);
  CHECK(c.nodes[0]->commit_index() == c.nodes[0]->last_applied());
}

TEST(raft_three_nodes_replicate_fail_over_and_reconverge) {
  Cluster c(3, "raft3");
  CHECK(eventually([&] { return c.leader() >= 0; }, 5));
  for (int i = 0; i < 10; ++i) CHECK(c.propose_at_leader(Json("a" + std::to_string(i)).dump()) == 0);
  int l = c.leader();
  CHECK(l >= 0);
  CHECK(eventually([&] {
    for (auto& h : c.hosts)
      if (h->snap().size() != 10) return false;
    return true;
  }, 5));
  // a follower refuses proposals with a leader hint
  int f = (l + 1) % 3;
  CHECK(c.propose(f, Json("x").dump()) == 1);
  // isolate the leader: it cannot commit, the majority elects a new leader and commits
  uint64_t old_term = c.nodes[l]->term();
  c.net->isolate(c.addrs[l], c.addrs);
  CHECK(c.propose(l, Json("lost").dump(), 0.6) != 0);
  int nl = -1;
  CHECK(eventually([&] {
    for (int i = 0; i < 3; ++i)
      if (i != l && c.nodes[i]->is_leader()) nl = i;
    return nl >= 0;
  }, 5));
  CHECK(c.nodes[nl]->term() > old_term);
  for (int i = 0; i < 60; ++i) CHECK(c.propose(nl, Json("b" + std::to_string(i)).dump()) == 0);  // crosses a snapshot
  // heal: the old leader steps down, drops its uncommitted entry and catches up
  c.net->heal();
  CHECK(eventually([&] {
    auto ref = c.hosts[nl]->snap();
    for (auto& h : c.hosts)
      if (h->snap() != ref) return false;
    return ref.size() == 70;
  }, 8));
  for (auto& s : c.hosts[l]->snap()) CHECK(s != "\"lost\"");
  CHECK(!c.nodes[l]->is_leader() || c.nodes[l]->term() > c.nodes[nl]->term());
  CHECK(c.nodes[nl]->last_included_index() > 0);  // compaction happened
}

TEST(raft_read_index_needs_a_majority) {
  Cluster c(3, "raftread");
  CHECK(eventually([&] { return c.leader() >= 0; }, 5));
  int l = c.leader();
  CHECK(c.propose(l, Json("v").dump()) == 0);
  auto read = [&](double t) {
    auto st = std::make_shared<std::atomic<int>>(-1);
    c.nodes[l]->read_index([st](int code, const std::string&) { *st = code; });
    eventually([&] { return st->load() >= 0; }, t);
    return st->load();
  };
  CHECK(read(2) == 0);
  c.net->isolate(c.addrs[l], c.addrs);
  CHECK(read(0.5) != 0);  // a deposed-but-unaware leader must not serve a stale read
  c.net->heal();
}

TEST(raft_leadership_transfer) {
  Cluster c(3, "rafttx");
  CHECK(eventually([&] { return c.leader() >= 0; }, 5));
  int l = c.leader(), target = (l + 1) % 3;
  CHECK(c.propose(l, Json("v").dump()) == 0);
  CHECK(c.nodes[l]->transfer_leadership(target + 1));
  CHECK(eventually([&] { return c.nodes[target]->is_leader(); }, 5));
  CHECK(c.propose(target, Json("after").dump()) == 0);
}

// ------------------------------------------------------------------------------- MasterCore
// The native master state machine on a real single-node Raft, hammered by concurrent
// clients through its hot handlers (the calls the native client makes), while the applier
// and access-stats threads run: under TSan this is the master's race check.
struct SmHost : raft::Host {
  std::shared_ptr<raft::StateMachine> sm;
  std::vector<std::string> apply(const std::vector<std::pair<uint64_t, std::string>>& c) override {
    return sm->apply(c);
  }
  std::string snapshot() override { return sm->snapshot(); }
  void restore(const std::string& s) override { sm->restore(s); }
  bool send(const std::string&, const std::string&, const std::string&, std::string*) override { return false; }
};

TEST(master_core_concurrent_create_complete_read_delete) {
  std::string d = tmpdir("mcore");
  auto core = std::make_shared<MasterCore>();
  auto host = std::make_shared<SmHost>();
  host->sm = core;
  raft::Options o;
  o.id = 1;
  o.members = {{1, "n1"}};
  o.client_address = "n1";
  o.dir = d;
  o.election_lo = 0.05;
  o.election_hi = 0.1;
  o.heartbeat = 0.02;
  o.sync = false;
  o.snapshot_threshold = 200;  // compaction happens during the run
  raft::Node node(o, host);
  node.start();
  CHECK(eventually([&] { return node.is_leader(); }, 3));
  core->attach(&node);
  core->set_access_stats(true, 20);
  core->exit_safe_mode();
  for (int i = 0; i < 4; ++i) {
    ChunkServerStatus st;
    st.address = "cs" + std::to_string(i) + ":1";
    st.last_heartbeat = std::chrono::duration_cast<std::chrono::milliseconds>(
                            std::chrono::system_clock::now().time_since_epoch()).count();
    st.available_space = 1ull << 40;
    st.rack_id = "r" + std::to_string(i % 2);
    core->upsert_chunk_server(st);
  }
  const int threads = 6, per = 25;
  std::atomic<int> failures{0};
  std::vector<std::string> errs(threads);
  std::vector<std::thread> ts;
  for (int t = 0; t < threads; ++t)
    ts.emplace_back([&, t] {
      auto fail = [&](const std::string& why) {
        ++failures;
        errs[t] = why;
      };
      for (int i = 0; i < per; ++i) {
        std::string path = "/t" + std::to_string(t) + "/f" + std::to_string(i), out;
        pb::CreateFileRequest c;
        c.path = path;
        c.allocate_block = true;
        c.defer_create = true;
        c.preferred_chunk_server = "cs" + std::to_string(t % 4) + ":1";
        if (core->handle("CreateFile", c.str(), &out) != MasterCore::OK) return fail("create rpc: " + out);
        pb::CreateFileResponse cr;
        if (!cr.decode(out) || !cr.success || !cr.has_allocation) return fail("create: " + cr.error_message);
        const auto& alloc = cr.allocation;
        if (alloc.chunk_server_addresses.size() != 3) return fail("placement size");
        pb::CompleteFileRequest done;
        done.path = path;
        done.size = 1 + i;
        done.etag_md5 = "etag";
        done.create = true;
        done.blocks.push_back(alloc.block);
        pb::BlockChecksumInfo sum;
        sum.block_id = alloc.block.block_id;
        sum.actual_size = 1 + i;
        done.block_checksums.push_back(sum);
        if (core->handle("CompleteFile", done.str(), &out) != MasterCore::OK) return fail("complete rpc: " + out);
        pb::CompleteFileResponse dr;
        if (!dr.decode(out) || !dr.success) return fail("complete: " + dr.error_message);
        pb::GetFileInfoRequest g;
        g.path = path;
        if (core->handle("GetFileInfo", g.str(), &out) != MasterCore::OK) return fail("info rpc: " + out);
        pb::GetFileInfoResponse gr;
        if (!gr.decode(out) || !gr.found || gr.metadata.size != static_cast<uint64_t>(1 + i)) return fail("info");
        if (i % 3 == 0) {
          pb::DeleteFileRequest del;
          del.path = path;
          if (core->handle("DeleteFile", del.str(), &out) != MasterCore::OK) return fail("delete rpc: " + out);
          pb::DeleteFileResponse dd;
          if (!dd.decode(out) || !dd.success) return fail("delete: " + dd.error_message);
        }
      }
      pb::ListFilesRequest l;
      l.path = "/t" + std::to_string(t) + "/";
      std::string out;
      if (core->handle("ListFiles", l.str(), &out) != MasterCore::OK) return fail("list rpc: " + out);
      pb::ListFilesResponse lr;
      lr.decode(out);
      if (lr.files.size() != static_cast<size_t>(per - (per + 2) / 3)) return fail("list size " + std::to_string(lr.files.size()));
    });
  for (auto& th : ts) th.join();
  for (auto& e : errs)
    if (!e.empty()) throw Failure("worker: " + e);
  CHECK(failures.load() == 0);
  CHECK(core->file_count() == static_cast<size_t>(threads * (per - (per + 2) / 3)));
  CHECK(core->take_gc().size() > 0);  // deleted files' blocks are queued for DELETE commands
  // the snapshot of the live state restores to an identical state machine
  MasterCore copy;
  copy.restore(core->snapshot());
  CHECK(copy.file_count() == core->file_count());
  core->detach();
  node.stop();
  std::filesystem::remove_all(d);
}

// Cross-shard Rename through the native 2PC (MasterCore::rename_2pc + the participant
// handlers): two shards, each a MasterCore on its own single-node Raft, wired together by a
// PeerCall that invokes the other core's handlers in-process. Concurrent renames commit on
// both sides; a taken destination and an unreachable participant abort with the source left
// readable and unpinned. Under TSan this is the 2PC's race check.
struct Shard {
  std::string dir;
  std::shared_ptr<MasterCore> core = std::make_shared<MasterCore>();
  std::shared_ptr<SmHost> host = std::make_shared<SmHost>();
  std::unique_ptr<raft::Node> node;
  explicit Shard(const std::string& tag) {
    dir = tmpdir(tag);
    host->sm = core;
    raft::Options o;
    o.id = 1;
    o.members = {{1, tag}};
    o.client_address = tag;
    o.dir = dir;
    o.election_lo = 0.05;
    o.election_hi = 0.1;
    o.heartbeat = 0.02;
    o.sync = false;
    node = std::make_unique<raft::Node>(o, host);
    node->start();
  }
  ~Shard() {
    core->detach();
    node->stop();
    std::filesystem::remove_all(dir);
  }
  int call(const std::string& method, const std::string& req, std::string* out) { return core->handle(method, req, out); }
  bool create(const std::string& path) {
    std::string out;
    pb::CreateFileRequest c;
    c.path = path;
    if (call("CreateFile", c.str(), &out) != MasterCore::OK) return false;
    pb::CreateFileResponse cr;
    if (!cr.decode(out) || !cr.success) return false;
    pb::CompleteFileRequest d;
    d.path = path;
    d.size = 7;
    d.etag_md5 = "e";
    if (call("CompleteFile", d.str(), &out) != MasterCore::OK) return false;
    pb::CompleteFileResponse dr;
    return dr.decode(out) && dr.success;
  }
  bool visible(const std::string& path) {
    std::string out;
    pb::GetFileInfoRequest g;
    g.path = path;
    pb::GetFileInfoResponse gr;
    return call("GetFileInfo", g.str(), &out) == MasterCore::OK && gr.decode(out) && gr.found;
  }
};

pb::RenameResponse rename_on(Shard& s, const std::string& src, const std::string& dst, int* code) {
  pb::RenameRequest r;
  r.source_path = src;
  r.dest_path = dst;
  std::string out;
  *code = s.call("Rename", r.str(), &out);
  pb::RenameResponse resp;
  if (*code == MasterCore::OK) resp.decode(out);
  return resp;
}

TEST(master_core_native_2pc_rename) {
  Shard a("sa"), b("sb");
  CHECK(eventually([&] { return a.node->is_leader() && b.node->is_leader(); }, 3));
  const std::string map =
      R"({"strategy":{"Range":{"ranges":{"/m":"A","~~~~":"B"}}},"shards":["A","B"],"shard_peers":{"A":["a"],"B":["b"]}})";
  std::atomic<bool> b_down{false};
  auto wire = [&](const std::string& target, const std::string& path, const std::string& req, int) {
    GrpcResult r;
    Shard* s = target == "a" ? &a : (target == "b" && !b_down.load()) ? &b : nullptr;
    if (!s) return r;  // unreachable: transport_ok = false
    const std::string prefix = "/dfs.MasterService/";
    r.transport_ok = true;
    r.status = s->call(path.substr(prefix.size()), req, &r.message);
    return r;
  };
  for (Shard* s : {&a, &b}) {
    s->core->attach(s->node.get());
    s->core->exit_safe_mode();
    s->core->enable_native_2pc(wire);
  }
  a.core->set_shard_map(map, "A");
  b.core->set_shard_map(map, "B");
  const int threads = 4, per = 12;
  for (int t = 0; t < threads; ++t)
    for (int i = 0; i < per; ++i) CHECK(a.create("/a/s" + std::to_string(t) + "_" + std::to_string(i)));
  std::atomic<int> bad{0};
  std::vector<std::thread> ts;
  for (int t = 0; t < threads; ++t)
    ts.emplace_back([&, t] {
      for (int i = 0; i < per; ++i) {
        const std::string sfx = std::to_string(t) + "_" + std::to_string(i);
        int code;
        pb::RenameResponse r = rename_on(a, "/a/s" + sfx, "/z/d" + sfx, &code);
        if (code != MasterCore::OK || !r.success) ++bad;
      }
    });
  for (auto& th : ts) th.join();
  CHECK(bad.load() == 0);
  for (int t = 0; t < threads; ++t)
    for (int i = 0; i < per; ++i) {
      const std::string sfx = std::to_string(t) + "_" + std::to_string(i);
      CHECK(b.visible("/z/d" + sfx));
      CHECK(!a.visible("/a/s" + sfx));
    }
  Json stats = a.core->txn_stats();
  CHECK(stats["native_committed"].as_int() == threads * per);
  Json recs = Json::parse(a.core->tx_records());
  for (auto& kv : recs.fields()) {
    CHECK(kv.second["state"].str() == "Committed");
    CHECK(kv.second["participant_acked"].as_bool());
  }
  // a taken destination: the participant refuses, the coordinator aborts, nothing stays pinned
  CHECK(a.create("/a/keep"));
  CHECK(b.create("/z/taken"));
  int code;
  pb::RenameResponse r = rename_on(a, "/a/keep", "/z/taken", &code);
  CHECK(code == MasterCore::OK && !r.success);
  CHECK(a.visible("/a/keep") && a.core->tx_lock("/a/keep").empty());
  // the participant shard unreachable: prepare fails, abort, the source stays usable
  b_down = true;
  r = rename_on(a, "/a/keep", "/z/new", &code);
  CHECK(code == MasterCore::OK && !r.success && r.error_message == "Cross-shard prepare failed");
  CHECK(a.visible("/a/keep") && a.core->tx_lock("/a/keep").empty());
  r = rename_on(a, "/a/keep", "/a/kept", &code);  // same shard: no 2PC, not blocked
  CHECK(code == MasterCore::OK && r.success && a.visible("/a/kept"));
  CHECK(a.core->txn_stats()["native_aborted"].as_int() == 2);
}

// ------------------------------------------------------------------------------- HTTP side channel
// of the native control-plane processes (http_lite.h): keep-alive requests on one server,
// bodies both ways, 404s, and a client that gives up on a dead port.
TEST(http_lite_server_and_client_round_trip) {
  std::atomic<int> calls{0};
  HttpLiteServer srv("127.0.0.1", 0, [&](const HttpRequest& r) -> HttpResponse {
    calls++;
    if (r.path == "/echo" && r.method == "POST") return HttpResponse{200, "application/json", r.body + "!" + r.query};
    if (r.path == "/health") return HttpResponse{200, "text/plain", "OK"};
    return HttpResponse{404, "text/plain", "Not Found"};
  });
  std::string err;
  CHECK(srv.start(&err));
  const std::string base = "http://127.0.0.1:" + std::to_string(srv.port());
  std::string reply;
  CHECK(http_request("GET", base + "/health", "", "", 2000, &reply) == 200 && reply == "OK");
  std::string big(3 << 20, 'x');
  CHECK(http_request("POST", base + "/echo?q=1", big, "application/json", 5000, &reply) == 200);
  CHECK(reply.size() == big.size() + 4 && reply.compare(reply.size() - 4, 4, "!q=1") == 0);
  CHECK(http_request("GET", base + "/nope", "", "", 2000, &reply) == 404);
  std::vector<std::thread> ts;
  std::atomic<int> ok{0};
  for (int t = 0; t < 8; ++t)
    ts.emplace_back([&] {
      std::string r;
      for (int i = 0; i < 20; ++i) ok += http_request("POST", base + "/echo", "p", "text/plain", 2000, &r) == 200 && r == "p!";
    });
  for (auto& t : ts) t.join();
  CHECK(ok == 160 && calls >= 163);
  srv.stop();
  std::string e2;
  CHECK(http_request("GET", base + "/health", "", "", 500, &reply, &e2) == 0 && !e2.empty());
}

// ------------------------------------------------------------------------ block journal
// (journal.h): the store of record's append / group-commit / retire protocol, replay after
// a crash (the object is dropped without retire_all, as a killed process would leave it).
namespace jt {

std::vector<uint8_t> meta_be_of(const std::vector<uint8_t>& d) {
  std::vector<uint32_t> c(num_slices(d.size()));
  crc32_slices(d.data(), d.size(), c.data());
  std::vector<uint8_t> be(4 * c.size());
  for (size_t i = 0; i < c.size(); ++i) {
    be[4 * i] = c[i] >> 24;
    be[4 * i + 1] = (c[i] >> 16) & 0xff;
    be[4 * i + 2] = (c[i] >> 8) & 0xff;
    be[4 * i + 3] = c[i] & 0xff;
  }
  return be;
}

// reserve -> write (in two pieces, out of order) -> finish -> commit
bool append(BlockJournal& j, const std::string& id, const std::vector<uint8_t>& d, JournalRec* r) {
  std::string err;
  const uint64_t ns = num_slices(d.size());
  if (!j.reserve(d.size(), ns, r, &err)) return false;
  const uint64_t half = d.size() / 2;
  if (!j.write(*r, half, d.data() + half, d.size() - half) || !j.write(*r, 0, d.data(), half)) return false;
  auto be = meta_be_of(d);
  if (!j.finish(r, id, d.size(), crc32(d.data(), d.size()), be.data(), ns)) return false;
  return j.commit(*r);
}

JournalConfig small(const std::string& dir, bool grow) {
  JournalConfig c;
  c.dir = dir;
  c.seg_bytes = 4 << 20;  // 4 parts of 1 MiB
  c.parts = 4;
  c.grow = grow;
  c.max_segs = grow ? 0 : 3;
  c.spares = 2;
  c.reserve_bytes = 0;
  c.idle_fill_ms = 5;
  c.full_timeout_s = 2;
  return c;
}

}  // namespace jt

// 8 writers append and commit concurrently while records are released (exported), segments
// retire, compaction-style relocations keep their LSN and tombstones are committed; a thread
// marks sealed segments meanwhile. After the "crash", replay returns every acknowledged,
// unreleased record with its bytes intact, newest version last, and no deleted id survives.
TEST(journal_concurrent_commit_retire_and_crash_replay) {
  const std::string d = tmpdir("journal_cc");
  std::mutex mu;
  std::map<std::string, std::pair<uint32_t, uint64_t>> live;  // id -> (crc, size) of the acked live version
  std::set<std::string> deleted;
  {
    BlockJournal j(jt::small(d + "/j", true));
    CHECK(j.recover().empty());
    std::atomic<bool> stop{false};
    std::thread marker_thread([&] {
      while (!stop) {
        j.mark_sealed_now();
        j.retire_ready();
        std::this_thread::sleep_for(std::chrono::milliseconds(3));
      }
    });
    std::vector<std::thread> ts;
    std::atomic<int> failures{0};
    for (int t = 0; t < 8; ++t)
      ts.emplace_back([&, t] {
        std::mt19937 rng(1234 + t);
        std::vector<std::pair<std::string, JournalRec>> mine;
        for (int i = 0; i < 40; ++i) {
          std::vector<uint8_t> data(1 + rng() % (200 << 10));
          for (auto& b : data) b = static_cast<uint8_t>(rng());
          const std::string id = "blk-" + std::to_string(t) + "-" + std::to_string(i % 25);  // some rewritten
          JournalRec r;
          if (!jt::append(j, id, data, &r)) {
            failures++;
            continue;
          }
          {
            std::lock_guard<std::mutex> g(mu);
            live[id] = {crc32(data.data(), data.size()), data.size()};
            deleted.erase(id);
          }
          for (auto it = mine.begin(); it != mine.end(); ++it)
            if (it->first == id) {  // the older version is superseded
              j.release(it->second);
              mine.erase(it);
              break;
            }
          mine.emplace_back(id, r);
          if (i % 7 == 3 && !mine.empty()) {  // delete the oldest: tombstone first, then release
            auto victim = mine.front();
            std::string err;
            if (!j.marker(kJrTomb, victim.first, &err)) {
              failures++;
              continue;
            }
            {
              std::lock_guard<std::mutex> g(mu);
              live.erase(victim.first);
              deleted.insert(victim.first);
            }
            j.release(victim.second);
            mine.erase(mine.begin());
          }
        }
      });
    for (auto& t : ts) t.join();
    stop = true;
    marker_thread.join();
    CHECK(failures == 0);
    JournalStats st = j.stats();
    CHECK(st.records == 320 && st.tombstones > 0 && st.sync_rounds > 0);
    CHECK(st.segs_retired > 0);  // releases let old segments retire while writers ran
  }  // dropped without retire_all: what a killed chunkserver leaves
  BlockJournal j2(jt::small(d + "/j", true));
  auto recs = j2.recover();
  std::map<std::string, const ReplayRecord*> last;  // replay is in LSN order: the last one wins
  for (auto& r : recs) last[r.id] = &r;
  for (auto& kv : live) {
    auto it = last.find(kv.first);
    CHECK(it != last.end());
    const ReplayRecord& r = *it->second;
    CHECK(r.type == kJrBlock && r.crc == kv.second.first && r.n == kv.second.second);
    std::vector<uint8_t> back(r.n);
    CHECK(::pread(r.fd(), back.data(), r.n, static_cast<off_t>(r.data_off())) == static_cast<ssize_t>(r.n));
    CHECK(crc32(back.data(), back.size()) == r.crc);
    CHECK(jt::meta_be_of(back) == r.meta_be);
  }
  for (auto& id : deleted) {
    auto it = last.find(id);
    CHECK(it == last.end() || it->second->type == kJrTomb);
  }
  std::filesystem::remove_all(d);
}

// Early writeback (appends written in page-aligned pieces, each handed to writeback at once):
// 4 writers append records of odd sizes, each in two out-of-order writes, and commit; after the
// "crash" every acknowledged record replays with its bytes and .meta image intact.
TEST(journal_early_writeback_appends_replay_intact) {
  const std::string d = tmpdir("journal_ewb");
  std::mutex mu;
  std::map<std::string, uint32_t> acked;
  {
    JournalConfig c = jt::small(d + "/j", true);
    c.early_wb_bytes = 64 << 10;
    BlockJournal j(c);
    CHECK(j.recover().empty());
    std::vector<std::thread> ts;
    std::atomic<int> failures{0};
    for (int t = 0; t < 4; ++t)
      ts.emplace_back([&, t] {
        std::mt19937 rng(77 + t);
        for (int i = 0; i < 30; ++i) {
          std::vector<uint8_t> data(1 + rng() % (300 << 10));
          for (auto& b : data) b = static_cast<uint8_t>(rng());
          const std::string id = "ewb-" + std::to_string(t) + "-" + std::to_string(i);
          JournalRec r;
          if (!jt::append(j, id, data, &r)) {
            failures++;
            continue;
          }
          std::lock_guard<std::mutex> g(mu);
          acked[id] = crc32(data.data(), data.size());
        }
      });
    for (auto& t : ts) t.join();
    CHECK(failures == 0);
  }
  BlockJournal j2(jt::small(d + "/j", true));
  auto recs = j2.recover();
  std::map<std::string, const ReplayRecord*> last;
  for (auto& r : recs) last[r.id] = &r;
  CHECK(acked.size() == 120);
  for (auto& kv : acked) {
    auto it = last.find(kv.first);
    CHECK(it != last.end());
    const ReplayRecord& r = *it->second;
    CHECK(r.type == kJrBlock && r.crc == kv.second);
    std::vector<uint8_t> back(r.n);
    CHECK(::pread(r.fd(), back.data(), r.n, static_cast<off_t>(r.data_off())) == static_cast<ssize_t>(r.n));
    CHECK(crc32(back.data(), back.size()) == r.crc);
    CHECK(jt::meta_be_of(back) == r.meta_be);
  }
  std::filesystem::remove_all(d);
}

// a segment is marked sealed (replay trusts its records without re-reading the
// data) only after its records are flushed: a finished record whose commit has not run yet is
// flushed by the marking itself, before the sealed header.
TEST(journal_marks_a_segment_only_after_flushing_pending_records) {
  const std::string d = tmpdir("journal_mark");
  BlockJournal j(jt::small(d + "/j", true));
  CHECK(j.recover().empty());
  std::vector<uint8_t> data(100 << 10, 0x5a);
  JournalRec r;
  std::string err;
  const uint64_t ns = num_slices(data.size());
  CHECK(j.reserve(data.size(), ns, &r, &err));
  CHECK(j.write(r, 0, data.data(), data.size()));
  auto be = jt::meta_be_of(data);
  CHECK(j.finish(&r, "pending", data.size(), crc32(data.data(), data.size()), be.data(), ns));
  // complete but not committed: marking must flush the part before writing the header
  j.mark_sealed_now();
  JournalStats st = j.stats();
  CHECK(st.segs_marked == 1 && st.mark_preflushes >= 1);
  CHECK(j.commit(r));  // already durable: no new flush round needed
  CHECK(j.stats().sync_rounds == st.sync_rounds);
  std::filesystem::remove_all(d);
}

// a full journal (ring of 3 segments, every record live) still takes tombstones —
// they go into the markers' reserve at the tail of each part — while a block append times out.
TEST(journal_full_still_commits_tombstones) {
  const std::string d = tmpdir("journal_full");
  BlockJournal j(jt::small(d + "/j", false));
  CHECK(j.recover().empty());
  // the ring's 3 segments are created (and written out) by the preparer first
  CHECK(eventually([&] { auto st = j.stats(); return st.segs_total == 3 && st.parts_unready == 0; }, 30));
  std::vector<uint8_t> data(240 << 10, 0x11);
  std::vector<JournalRec> held;
  int n = 0;
  for (;;) {
    JournalRec r;
    std::string err;
    const uint64_t ns = num_slices(data.size());
    if (!j.reserve(data.size(), ns, &r, &err)) {
      CHECK(err.find("journal full") != std::string::npos || err.find("segment") != std::string::npos);
      break;
    }
    CHECK(j.write(r, 0, data.data(), data.size()));
    auto be = jt::meta_be_of(data);
    CHECK(j.finish(&r, "b" + std::to_string(n++), data.size(), crc32(data.data(), data.size()), be.data(), ns));
    CHECK(j.commit(r));
    held.push_back(r);
    CHECK(n < 1000);
  }
  CHECK(n >= 3 * 4 * 3);  // 3 segments x 4 parts x at least 3 records of 244 KiB per 1 MiB part
  for (int i = 0; i < 8; ++i) {
    std::string err;
    CHECK(j.marker(kJrTomb, "b" + std::to_string(i), &err));
  }
  CHECK(j.stats().reserve_markers >= 8);
  // the tombstones replay after the records they cancel
  for (auto& r : held) j.release(r);
  std::filesystem::remove_all(d);
}

// Grow mode keeps `spares` free segments, but while the writers are active a top-up waits for
// their next idle window unless fewer than spares_low are free.
TEST(journal_defers_spare_creation_while_writers_are_active) {
  const std::string d = tmpdir("journal_grow");
  JournalConfig c = jt::small(d + "/j", true);
  c.spares = 4;
  c.spares_low = 2;
  c.idle_fill_ms = 400;  // no gap between two appends counts as idle, even under a sanitizer on a loaded host
  BlockJournal j(c);
  CHECK(j.recover().empty());
  CHECK(eventually([&] { auto s = j.stats(); return s.spares_missing == 0 && s.parts_unready == 0; }, 10));
  const uint64_t segs0 = j.stats().segs_total;
  std::vector<uint8_t> data(300 << 10, 0x22);
  // ~1.5 segments of appends back to back: free drops 4 -> 2 (still >= spares_low)
  auto t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < 18; ++i) {
    JournalRec r;
    CHECK(jt::append(j, "g" + std::to_string(i), data, &r));
  }
  const double active_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  JournalStats mid = j.stats();
  if (active_s < 0.4) {  // the writers never paused for an idle window
    CHECK(mid.segs_total == segs0);  // nothing created while they ran
    CHECK(mid.spares_missing > 0 && mid.parts_unready == 0);
  }
  CHECK(eventually([&] { return j.stats().spares_missing == 0; }, 10));  // topped up once idle
  CHECK(j.stats().grow_deferred >= 1 || active_s >= 0.4);
  std::filesystem::remove_all(d);
}

// ------------------------------------------------------------------ aws-chunked decoding
namespace ac {
struct MemSrc {  // the decoder's source over a byte string (the front reads a socket)
  std::string s;
  size_t pos = 0;
  int line(std::string* out, size_t max) {
    size_t e = s.find("\r\n", pos);
    if (e == std::string::npos) return -1;
    if (max == 0 && e != pos) return -1;
    if (max && e - pos > max) return -1;
    out->assign(s, pos, e - pos);
    pos = e + 2;
    return 1;
  }
  int read(uint8_t* dst, uint64_t n) {
    if (s.size() - pos < n) return -1;
    std::memcpy(dst, s.data() + pos, n);
    pos += n;
    return 1;
  }
  int drain() { return 1; }
};
sigv4::ChunkChain seed_chain() {
  sigv4::ChunkChain c;
  c.key = std::string(32, 'k');
  c.timestamp = "20260101T000000Z";
  c.scope = "20260101/us-east-1/s3/aws4_request";
  c.prev = std::string(64, 'a');
  return c;
}
std::string encode(const std::vector<std::string>& chunks, bool sign) {
  sigv4::ChunkChain c = seed_chain();
  std::string out;
  char hex[32];
  for (auto& ch : chunks) {
    std::snprintf(hex, sizeof hex, "%zx", ch.size());
    out += hex;
    if (sign) out += ";chunk-signature=" + c.next(ch.data(), ch.size());
    out += "\r\n" + ch + "\r\n";
  }
  out += "0";
  if (sign) out += ";chunk-signature=" + c.next("", 0);
  out += "\r\n\r\n";
  return out;
}
}  // namespace ac

// The S3 front's aws-chunked decoder (csrc/aws_chunked.h): framing, the chunk-signature
// chain, and a mutation fuzz — no mutated signed stream ever decodes, nothing overruns `cap`.
TEST(aws_chunked_decode_signature_chain_and_fuzz) {
  std::mt19937 rng(7);
  std::vector<std::string> chunks;
  std::string all;
  for (int i = 0; i < 6; ++i) {
    std::string c(1 + rng() % 3000, '\0');
    for (auto& b : c) b = static_cast<char>(rng());
    chunks.push_back(c);
    all += c;
  }
  std::vector<uint8_t> dst(all.size());
  for (bool sign : {false, true}) {
    ac::MemSrc in{ac::encode(chunks, sign)};
    sigv4::ChunkChain chain = ac::seed_chain();
    auto r = decode_aws_chunked(in, sign ? &chain : nullptr, dst.data(), dst.size());
    CHECK(r.rc == 1 && r.bytes == all.size() && std::memcmp(dst.data(), all.data(), all.size()) == 0);
    CHECK(r.sigs == (sign ? chunks.size() + 1 : 0));
  }
  {  // one byte too small a destination
    ac::MemSrc in{ac::encode(chunks, false)};
    std::vector<uint8_t> small(all.size() - 1);
    CHECK(decode_aws_chunked(in, nullptr, small.data(), small.size()).rc == -1);
  }
  {  // a signed stream without its final signed empty chunk
    std::string e = ac::encode(chunks, true);
    e = e.substr(0, e.rfind("0;chunk-signature="));
    ac::MemSrc in{e};
    sigv4::ChunkChain chain = ac::seed_chain();
    CHECK(decode_aws_chunked(in, &chain, dst.data(), dst.size()).rc != 1);
  }
  {  // a huge declared size cannot wrap the bound check
    ac::MemSrc in{std::string("fffffffffffffff\r\n")};
    CHECK(decode_aws_chunked(in, nullptr, dst.data(), dst.size()).rc == -1);
  }
  const std::string good = ac::encode(chunks, true);
  int accepted = 0;
  for (int it = 0; it < 3000; ++it) {
    std::string m = good;
    const int edits = 1 + static_cast<int>(rng() % 3);
    for (int e = 0; e < edits; ++e) {
      const size_t at = rng() % m.size();
      switch (rng() % 3) {
        case 0: m[at] = static_cast<char>(m[at] ^ (1 + rng() % 255)); break;
        case 1: m.erase(at, 1 + rng() % 8); break;
        default: m.insert(at, 1, static_cast<char>(rng())); break;
      }
      if (m.empty()) m = "x";
    }
    ac::MemSrc in{m};
    sigv4::ChunkChain chain = ac::seed_chain();
    std::vector<uint8_t> out(all.size() + 64);
    auto r = decode_aws_chunked(in, &chain, out.data(), out.size());
    if (r.rc == 1) {
      ++accepted;  // only possible when the edit left the signed content intact
      CHECK(r.bytes == all.size() && std::memcmp(out.data(), all.data(), all.size()) == 0);
    }
  }
  CHECK(accepted < 3000);
}

// ------------------------------------------------------------------ audit log (C56)
// 8 threads log concurrently into small batches; every accepted record is committed exactly
// once, in one HMAC chain, and a new writer on the same directory continues that chain.
TEST(audit_log_concurrent_batches_form_one_chain) {
  const std::string d = tmpdir("audit");
  const std::string secret = "audit-secret";
  auto rec = [](int t, int i) {
    return std::string("{\"timestamp\":\"2026-10-18T00:00:00Z\",\"timestamp_ms\":") + std::to_string(1790000000000LL + i) +
           ",\"request_id\":\"r-" + std::to_string(t) + "-" + std::to_string(i) +
           "\",\"remote_ip\":\"127.0.0.1\",\"user_id\":\"u" + std::to_string(t) +
           "\",\"role_arn\":null,\"action\":\"s3:PutObject\",\"resource\":\"arn:dfs:s3:::b/k\",\"status_code\":200,"
           "\"error_code\":null,\"user_agent\":\"ut\",\"duration_ms\":1.5}";
  };
  {
    AuditLog log(d, 30, 7, secret, 100000, 50, true);
    std::vector<std::thread> ts;
    for (int t = 0; t < 8; ++t)
      ts.emplace_back([&, t] {
        for (int i = 0; i < 60; ++i) CHECK(log.log(rec(t, i)));
      });
    for (auto& t : ts) t.join();
    CHECK(log.flush(10000));
    CHECK(log.committed() == 480 && log.dropped() == 0 && log.flush_errors() == 0);
    log.close();
  }
  std::string head;
  {
    AuditLog log(d, 30, 5, secret, 1000, 50, true);
    for (int i = 0; i < 10; ++i) CHECK(log.log(rec(9, 1000 + i)));
    CHECK(log.flush(10000));
    head = log.head();
    log.close();
  }
  // walk the segments: keys increase, previous_hash links, record_hash = HMAC(canonical)
  std::vector<std::string> segs;
  for (auto& e : std::filesystem::directory_iterator(d))
    if (e.path().extension() == ".log") segs.push_back(e.path().string());
  std::sort(segs.begin(), segs.end());
  std::string prev;
  int64_t last_key = -1;
  int n = 0;
  for (auto& sp : segs) {
    FILE* f = std::fopen(sp.c_str(), "r");
    CHECK(f != nullptr);
    char* line = nullptr;
    size_t cap = 0;
    ssize_t len;
    while ((len = ::getline(&line, &cap, f)) > 0) {
      std::string l(line, static_cast<size_t>(len));
      while (!l.empty() && (l.back() == '\n' || l.back() == '\r')) l.pop_back();
      if (l.empty()) continue;
      const size_t tab = l.find('\t');
      CHECK(tab != std::string::npos);
      const int64_t key = std::stoll(l.substr(0, tab));
      CHECK(key >= last_key);  // monotonic key timestamps (audit.rs)
      last_key = key;
      Json r = Json::parse(l.substr(tab + 1));
      CHECK((prev.empty() ? r["previous_hash"].is_null() || r["previous_hash"].str().empty() : r["previous_hash"].str() == prev));
      CHECK(r["record_hash"].str() == audit::hmac_hex(secret, audit::canonical_json(r, true)));
      prev = r["record_hash"].str();
      ++n;
    }
    std::free(line);
    std::fclose(f);
  }
  CHECK(n == 490 && prev == head);
  std::filesystem::remove_all(d);
}

// ------------------------------------------------------------- socket P2P transport
// Two ranks, 4 channels per direction: concurrent transfers on every channel land in post
// order with their bytes; then the receiver drops the pair mid-stream and every pending op on
// the sender ends (failed or done) instead of hanging; the pair reopens for a new generation.
int wait_op(P2PTransport& t, P2POp* op, double secs) {  // wait() naps 20 us at most: poll
  auto end = std::chrono::steady_clock::now() + std::chrono::duration<double>(secs);
  int r;
  while ((r = t.wait(op, 1000)) == 0 && std::chrono::steady_clock::now() < end) {
  }
  return r;
}

TEST(socket_transport_four_channels_and_a_dropped_peer) {
  const std::string ns = "ut" + std::to_string(::getpid());
  auto a = make_socket_transport(0, ns, 4), b = make_socket_transport(1, ns, 4);
  CHECK(a && b && a->channels() == 4);
  auto open_pair = [&](uint64_t gen) {
    std::string e1, e2;
    const std::string ta = a->make_token(1, gen, &e1), tb = b->make_token(0, gen, &e2);
    CHECK(!ta.empty() && !tb.empty());
    bool ok_a = false, ok_b = false;
    std::thread th([&] { ok_b = b->open(0, gen, tb, ta, 5000, &e2); });
    ok_a = a->open(1, gen, ta, tb, 5000, &e1);
    th.join();
    CHECK(ok_a && ok_b);
  };
  open_pair(1);
  std::mt19937 rng(3);
  const int per = 40;
  std::vector<std::vector<std::string>> sent(4), got(4);
  std::vector<P2POp> sops, rops;
  std::vector<std::vector<char>> rbufs;
  sops.reserve(4 * per);
  rops.reserve(4 * per);
  rbufs.reserve(4 * per);
  for (int i = 0; i < per; ++i)
    for (int ch = 0; ch < 4; ++ch) {
      std::string m(1 + rng() % 70000, '\0');
      for (auto& c : m) c = static_cast<char>(rng());
      sent[ch].push_back(m);
    }
  std::string err;
  for (int ch = 0; ch < 4; ++ch)
    for (int i = 0; i < per; ++i) {
      rbufs.emplace_back(sent[ch][i].size());
      rops.emplace_back();
      CHECK(b->post_recv(0, ch, rbufs.back().data(), rbufs.back().size(), &rops.back(), &err));
    }
  for (int i = 0; i < per; ++i)
    for (int ch = 0; ch < 4; ++ch) {
      sops.emplace_back();
      CHECK(a->post_send(1, ch, sent[ch][i].data(), sent[ch][i].size(), &sops.back(), &err));
    }
  for (auto& op : sops) CHECK(wait_op(*a, &op, 20) == 1);
  for (auto& op : rops) CHECK(wait_op(*b, &op, 20) == 1);
  for (int ch = 0; ch < 4; ++ch)
    for (int i = 0; i < per; ++i) CHECK(std::string(rbufs[ch * per + i].begin(), rbufs[ch * per + i].end()) == sent[ch][i]);
  for (auto& op : sops) a->release(&op);
  for (auto& op : rops) b->release(&op);
  // the peer goes away with sends posted that it never receives
  std::vector<P2POp> pend(8);
  std::string big(1 << 20, 'z');
  for (int i = 0; i < 8; ++i) CHECK(a->post_send(1, i % 4, big.data(), big.size(), &pend[i], &err));
  b->close(0);
  for (auto& op : pend) {
    int r = wait_op(*a, &op, 5);
    if (r == 0) {  // still queued behind a dead socket: close() must end it
      a->close(1);
      r = a->test(&op);
    }
    CHECK(r != 0);
    a->release(&op);
  }
  a->close(1);
  open_pair(2);  // a new generation comes up on both sides
  P2POp s1, r1;
  char out[5] = "ping", in[5] = {0};
  CHECK(b->post_recv(0, 3, in, 4, &r1, &err) && a->post_send(1, 3, out, 4, &s1, &err));
  CHECK(wait_op(*a, &s1, 5) == 1 && wait_op(*b, &r1, 5) == 1 && std::string(in) == "ping");
  a->release(&s1);
  b->release(&r1);
}

// ------------------------------------------------------------------ checker (C49)
TEST(linearizability_checker_self_test) {
  auto fails = lin::self_test();
  for (auto& f : fails) std::printf("  %s\n", f.c_str());
  CHECK(fails.empty());
}

// --------------------------------------------------------------------- OIDC (C15)
// tokens with unknown kids must not drive one outbound discovery + JWKS fetch each.
TEST(oidc_unknown_kid_refetch_is_rate_limited) {
  sts::OidcValidator v("http://127.0.0.1:1", "dfs-client", true);
  auto tok = [](const std::string& kid) {
    auto b64 = [](const std::string& s) {
      static const char* a = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789-_";
      std::string o;
      uint32_t val = 0;
      int bits = -6;
      for (unsigned char c : s) {
        val = ((val << 8) | c) & 0xFFFFFFu;  // at most 24 live bits
        bits += 8;
        while (bits >= 0) {
          o.push_back(a[(val >> bits) & 0x3F]);
          bits -= 6;
        }
      }
      if (bits > -6) o.push_back(a[((val << 8) >> (bits + 8)) & 0x3F]);
      return o;
    };
    return b64("{\"alg\":\"HS256\",\"kid\":\"" + kid + "\"}") + "." + b64("{\"sub\":\"x\"}") + "." + b64("sig");
  };
  sts::Claims c;
  std::string kind, detail;
  std::vector<std::thread> ts;
  for (int i = 0; i < 8; ++i)
    ts.emplace_back([&, i] {
      sts::Claims cc;
      std::string k, dd;
      CHECK(!v.validate(tok("kid-" + std::to_string(i)), &cc, &k, &dd));
    });
  for (auto& t : ts) t.join();
  CHECK(!v.validate(tok("another"), &c, &kind, &detail));
  CHECK(kind == "internal");  // no JWKS at all
  CHECK(v.fetches_failed() == 1 && v.fetches_ok() == 0);  // one attempt for 9 unknown kids
}

// ------------------------------------------------------------------ native gRPC wire
// The HTTP/2 gRPC server and client (nghttp2): 16 threads x 50 unary calls on pooled
// connections, payloads up to 1 MiB each way, request ids carried, an error status passed
// through, and calls to a stopped server failing at the transport instead of hanging.
TEST(grpc_server_and_client_concurrent_unary_calls) {
  GrpcServer srv("127.0.0.1", 0, [](const GrpcCall& c) {
    GrpcReply r;
    if (c.path == "/t.S/Fail") {
      r.status = 9;
      r.message = "Not Leader|x";
      return r;
    }
    r.message.assign(reinterpret_cast<const char*>(c.data()), c.size());
    r.message += "|" + c.request_id;
    return r;
  });
  std::string err;
  CHECK(srv.start(&err));
  const std::string target = "127.0.0.1:" + std::to_string(srv.port());
  GrpcChannelPool pool(10000);
  std::atomic<int> ok{0};
  std::vector<std::thread> ts;
  for (int t = 0; t < 16; ++t)
    ts.emplace_back([&, t] {
      std::mt19937 rng(t);
      for (int i = 0; i < 50; ++i) {
        std::string req(rng() % (i % 10 == 0 ? (1 << 20) : 4096), static_cast<char>('a' + t));
        const std::string rid = "rid-" + std::to_string(t) + "-" + std::to_string(i);
        GrpcResult r = pool.call(target, "/t.S/Echo", req, rid);
        ok += r.transport_ok && r.status == 0 && r.message == req + "|" + rid;
      }
    });
  for (auto& t : ts) t.join();
  CHECK(ok == 800);
  GrpcResult f = pool.call(target, "/t.S/Fail", "x", "rid");
  CHECK(f.transport_ok && f.status == 9 && f.message == "Not Leader|x");
  srv.stop();
  GrpcResult dead = pool.call(target, "/t.S/Echo", "x", "rid", 2000);
  CHECK(!dead.transport_ok || dead.status != 0);
}

// ------------------------------------------------------------------ multi-buffer MD5
// The ETag hash of md5_mb.cpp against OpenSSL: every length class (empty, < 56, 56..63 with a
// second padding block, whole blocks, MiB), 40 messages from 8 submitting threads through 2
// engines, so lanes join and finish at different rounds.
TEST(md5_multibuffer_matches_openssl) {
  std::mt19937 rng(11);
  std::vector<std::vector<uint8_t>> msgs;
  for (size_t n : {0, 1, 3, 55, 56, 57, 63, 64, 65, 119, 120, 127, 128, 1000, 4096, 65535, 1 << 20, (1 << 20) + 17})
    msgs.emplace_back(n);
  while (msgs.size() < 40) msgs.emplace_back(rng() % 300000);
  for (auto& m : msgs)
    for (auto& b : m) b = static_cast<uint8_t>(rng());
  for (auto kind : {Md5MultiBuffer::Kind::Avx512, Md5MultiBuffer::Kind::Scalar})
    for (int lanes : {1, 2, 3}) {
      if (kind == Md5MultiBuffer::Kind::Avx512 && (lanes > 1 || !Md5MultiBuffer::available())) continue;
      Md5MultiBuffer mb(2, kind, lanes);
      std::vector<std::future<std::string>> fs(msgs.size());
      std::vector<std::thread> ts;
      for (int t = 0; t < 8; ++t)
        ts.emplace_back([&, t] {
          for (size_t i = t; i < msgs.size(); i += 8) fs[i] = mb.submit(msgs[i].data(), msgs[i].size());
        });
      for (auto& t : ts) t.join();
      for (size_t i = 0; i < msgs.size(); ++i) CHECK(fs[i].get() == md5_hex_scalar(msgs[i].data(), msgs[i].size()));
      CHECK(mb.messages() == msgs.size());
    }
}

}  // namespace

int main(int argc, char** argv) {
  std::string filter = argc > 1 ? argv[1] : "";
  int failed = 0, ran = 0;
  for (auto& t : registry()) {
    if (!filter.empty() && t.first.find(filter) == std::string::npos) continue;
    ++ran;
    auto t0 = std::chrono::steady_clock::now();
    try {
      t.second();
      std::printf("ok %s (%.2fs)\n", t.first.c_str(),
                  std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
    } catch (const std::exception& e) {
      ++failed;
      std::printf("FAIL %s: %s\n", t.first.c_str(), e.what());
    }
    std::fflush(stdout);
  }
  std::printf("%d/%d passed\n", ran - failed, ran);
  return failed ? 1 : 0;
}
