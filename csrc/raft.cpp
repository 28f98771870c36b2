#include "raft.h"

#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cstdio>
#include <ctime>
#include <fstream>
#include <sstream>

namespace dfs::raft {

namespace {

void mkdirs(const std::string& path) {
  std::string cur;
  for (size_t i = 0; i < path.size(); ++i) {
    cur.push_back(path[i]);
    if ((path[i] == '/' || i + 1 == path.size()) && cur.size() > 1) ::mkdir(cur.c_str(), 0755);
  }
}

bool majority(const std::map<int, std::string>& group, const std::set<int>& acks) {
  size_t n = 0;
  for (int a : acks) n += group.count(a);
  return n > group.size() / 2;
}

Json members_json(const std::map<int, std::string>& m) {
  Json o = Json::object();
  for (auto& kv : m) o.set(std::to_string(kv.first), kv.second);
  return o;
}

std::map<int, std::string> members_from(const Json& j) {
  std::map<int, std::string> out;
  for (auto& kv : j.fields()) out[std::stoi(kv.first)] = kv.second.str();
  return out;
}

bool is_membership(const std::string& cmd) { return cmd.compare(0, 13, "{\"Membership\"") == 0; }

}  // namespace

const char* role_name(Role r) {
  switch (r) {
    case Role::Follower: return "Follower";
    case Role::Candidate: return "Candidate";
    default: return "Leader";
  }
}

// ---------------------------------------------------------------- ClusterConfig
std::map<int, std::string> ClusterConfig::all() const {
  std::map<int, std::string> out;
  if (joint) out = old_members;
  for (auto& kv : members) out[kv.first] = kv.second;
  return out;
}

bool ClusterConfig::is_voter(int id) const { return members.count(id) || (joint && old_members.count(id)); }

bool ClusterConfig::has_joint_majority(const std::set<int>& acks) const {
  if (joint) return majority(old_members, acks) && majority(members, acks);
  return majority(members, acks);
}

Json ClusterConfig::to_json() const {
  Json inner = Json::object(), out = Json::object();
  if (joint) {
    inner.set("old_members", members_json(old_members));
    inner.set("new_members", members_json(members));
    inner.set("version", version);
    out.set("Joint", inner);
  } else {
    inner.set("members", members_json(members));
    inner.set("version", version);
    out.set("Simple", inner);
  }
  return out;
}

ClusterConfig ClusterConfig::from_json(const Json& j) {
  ClusterConfig c;
  if (const Json* jt = j.find("Joint")) {
    c.joint = true;
    c.members = members_from((*jt)["new_members"]);
    c.old_members = members_from((*jt)["old_members"]);
    c.version = (*jt)["version"].as_int();
  } else {
    const Json& s = j["Simple"];
    c.members = members_from(s["members"]);
    c.version = s["version"].as_int();
  }
  return c;
}

// ---------------------------------------------------------------- construction / persistence
Node::Node(Options opt, std::shared_ptr<Host> host)
    : opt_(std::move(opt)), host_(std::move(host)), rng_(std::random_device{}()) {
  mkdirs(opt_.dir);
  config_.members = opt_.members;
  wal_ = std::make_unique<Wal>(opt_.dir + "/raft.wal", opt_.sync);
  load();
}

Node::~Node() { stop(); }

int64_t Node::term_at(uint64_t idx) const {
  if (idx == last_included_index_) return static_cast<int64_t>(last_included_term_);
  if (idx < last_included_index_ || idx > last_index_locked()) return -1;
  return static_cast<int64_t>(at(idx).term);
}

void Node::load() {
  std::ifstream f(snap_path(), std::ios::binary);
  if (f) {
    std::stringstream ss;
    ss << f.rdbuf();
    Json snap = Json::parse(ss.str());
    last_included_index_ = snap["meta"][0].as_u64();
    last_included_term_ = snap["meta"][1].as_u64();
    if (!snap["config"].is_null()) config_ = ClusterConfig::from_json(snap["config"]);
    host_->restore(snap["state"].dump());
    commit_index_ = last_applied_ = last_included_index_;
  }
  for (const std::string& raw : wal_->replay()) {
    Json r = Json::parse(raw);
    const std::string& k = r["k"].as_string();
    if (k == "H") {
      current_term_ = r["term"].as_u64();
      voted_for_ = r["vote"].is_null() ? -1 : static_cast<int>(r["vote"].as_int());
    } else if (k == "E") {
      uint64_t idx = r["i"].as_u64();
      if (idx <= last_included_index_) continue;
      uint64_t pos = idx - first_index();
      if (pos < log_.size()) log_.resize(pos);
      if (pos == log_.size()) log_.push_back(Entry{r["t"].as_u64(), r["c"].dump()});
    } else if (k == "T") {
      uint64_t from = r["from"].as_u64();
      if (from >= first_index() && from - first_index() < log_.size()) log_.resize(from - first_index());
    } else if (k == "C") {
      config_ = ClusterConfig::from_json(r["config"]);
    }
  }
  durable_index_ = last_index_locked();
}

std::string Node::hs_record() const {
  Json r = Json::object();
  r.set("k", "H");
  r.set("term", current_term_);
  r.set("vote", voted_for_ < 0 ? Json() : Json(voted_for_));
  return r.dump();
}

std::string Node::entry_record(uint64_t idx) const {
  const Entry& e = at(idx);
  std::string s = "{\"k\":\"E\",\"i\":" + std::to_string(idx) + ",\"t\":" + std::to_string(e.term) + ",\"c\":";
  s += e.cmd;
  s += "}";
  return s;
}

std::string Node::config_record() const {
  Json r = Json::object();
  r.set("k", "C");
  r.set("config", config_.to_json());
  return r.dump();
}

void Node::persist(const std::vector<std::string>& recs) {
  if (recs.empty()) return;
  try {
    wal_->append(recs);
  } catch (const std::exception& e) {
    std::fprintf(stderr, "raft node %d: WAL append failed: %s\n", opt_.id, e.what());
  }
}

// ---------------------------------------------------------------- lifecycle
void Node::start() {
  {
    std::lock_guard<std::mutex> g(mu_);
    if (started_) return;
    started_ = true;
    running_ = true;
    reset_election_timer_locked();
  }
  ticker_ = std::thread([this] { ticker_loop(); });
  flusher_ = std::thread([this] { flusher_loop(); });
  applier_ = std::thread([this] { applier_loop(); });
  snapshotter_ = std::thread([this] { snapshot_loop(); });
  bool solo;
  {
    std::lock_guard<std::mutex> g(mu_);
    solo = peers_locked().empty() && config_.is_voter(opt_.id);
  }
  if (solo) run_election();  // single-node group: lead immediately
}

void Node::stop() {
  {
    std::lock_guard<std::mutex> g(mu_);
    if (!running_) return;
    running_ = false;
    tick_cv_.notify_all();
    flush_cv_.notify_all();
    apply_cv_.notify_all();
    snap_cv_.notify_all();
    for (auto& kv : peers_) {
      kv.second->cv.notify_all();
      kv.second->aux_cv.notify_all();
    }
  }
  for (std::thread* t : {&ticker_, &flusher_, &applier_, &snapshotter_})
    if (t->joinable()) t->join();
  std::map<int, std::unique_ptr<Peer>> peers;
  {
    std::lock_guard<std::mutex> g(mu_);
    peers.swap(peers_);
  }
  for (auto& kv : peers) {
    if (kv.second->repl.joinable()) kv.second->repl.join();
    if (kv.second->aux.joinable()) kv.second->aux.join();
  }
  Callbacks cbs;
  {
    std::lock_guard<std::mutex> g(mu_);
    fail_pending_locked(cbs);
  }
  for (auto& cb : cbs) cb();
}

Node::Peer* Node::peer(int id) {
  auto it = peers_.find(id);
  if (it != peers_.end()) return it->second.get();
  auto p = std::make_unique<Peer>();
  p->id = id;
  Peer* raw = p.get();
  peers_[id] = std::move(p);
  if (running_) {
    raw->repl = std::thread([this, raw] { repl_loop(raw); });
    raw->aux = std::thread([this, raw] { aux_loop(raw); });
  }
  return raw;
}

std::vector<int> Node::peers_locked() const {
  std::set<int> ids;
  for (auto& kv : config_.all()) ids.insert(kv.first);
  for (auto& kv : non_voting_) ids.insert(kv.first);
  ids.erase(opt_.id);
  return {ids.begin(), ids.end()};
}

std::string Node::addr_locked(int id) const {
  auto all = config_.all();
  auto it = all.find(id);
  if (it != all.end()) return it->second;
  auto nv = non_voting_.find(id);
  return nv == non_voting_.end() ? std::string() : nv->second;
}

void Node::reset_election_timer_locked() {
  std::uniform_real_distribution<double> d(opt_.election_lo, opt_.election_hi);
  election_deadline_ = Clock::now() + std::chrono::microseconds(static_cast<int64_t>(d(rng_) * 1e6));
}

// ---------------------------------------------------------------- elections
void Node::ticker_loop() {
  auto hb = std::chrono::microseconds(static_cast<int64_t>(opt_.heartbeat * 1e6));
  while (running_) {
    bool elect = false;
    {
      std::unique_lock<std::mutex> lk(mu_);
      tick_cv_.wait_for(lk, hb, [&] { return !running_ || tick_now_; });
      tick_now_ = false;
      if (!running_) break;
      if (role_ == Role::Leader) {
        broadcast_locked();
      } else if (Clock::now() >= election_deadline_ && config_.is_voter(opt_.id)) {
        elect = true;
      }
    }
    if (elect && opt_.pre_vote) run_pre_vote();
    else if (elect) run_election(false);
  }
}

void Node::start_election_locked(bool transfer, std::string* hs, std::string* vote_args) {
  role_ = Role::Candidate;
  ++current_term_;
  voted_for_ = opt_.id;
  leader_id_ = -1;
  votes_ = {opt_.id};
  reset_election_timer_locked();
  *hs = hs_record();
  Json a = Json::object();
  a.set("term", current_term_);
  a.set("candidate_id", opt_.id);
  a.set("last_log_index", last_index_locked());
  a.set("last_log_term", term_at(last_index_locked()));
  if (transfer) a.set("transfer", true);
  *vote_args = a.dump();
}

bool Node::has_lease() const {
  std::lock_guard<std::mutex> g(mu_);
  if (role_ != Role::Leader) return false;
  // a majority answered us within election_lo: with pre-vote and leader stickiness none of
  // them votes for anyone else before election_lo passes, so no newer leader exists yet
  const auto horizon = Clock::now() - std::chrono::microseconds(static_cast<int64_t>(opt_.election_lo * 1e6));
  std::set<int> fresh = {opt_.id};
  for (auto& kv : ack_at_)
    if (kv.second >= horizon) fresh.insert(kv.first);
  return config_.has_joint_majority(fresh);
}

bool Node::leader_recent_locked() const {
  if (role_ == Role::Leader) return true;
  if (leader_id_ < 0) return false;
  auto lease = std::chrono::microseconds(static_cast<int64_t>(opt_.election_lo * 1e6));
  return Clock::now() < leader_contact_ + lease;
}

// Pre-vote round: ask the voters whether they WOULD vote for us at term+1, changing no
// state anywhere. Only a majority of yes starts the real election (aux_loop), so a server
// that cannot win never bumps the cluster's term and never unseats a working leader.
void Node::run_pre_vote() {
  {
    std::lock_guard<std::mutex> g(mu_);
    if (!running_ || role_ == Role::Leader) return;
    reset_election_timer_locked();  // no majority of yes: try again after another timeout
    uint64_t round = ++prevote_round_;
    prevotes_ = {opt_.id};
    if (!config_.has_joint_majority(prevotes_)) {
      Json a = Json::object();
      a.set("term", current_term_ + 1);
      a.set("candidate_id", opt_.id);
      a.set("last_log_index", last_index_locked());
      a.set("last_log_term", term_at(last_index_locked()));
      a.set("pre_vote", true);
      std::string args = a.dump();
      for (int p : peers_locked()) {
        if (!config_.is_voter(p)) continue;
        Peer* pp = peer(p);
        pp->vote_body = args;
        pp->vote_term = current_term_;
        pp->vote_pre = true;
        pp->vote_round = round;
        pp->aux_cv.notify_one();
      }
      return;
    }
  }
  run_election(false);  // sole voter
}

void Node::run_election(bool transfer) {
  std::string args;
  uint64_t term;
  {
    std::lock_guard<std::mutex> w(wal_order_mu_);
    std::string hs;
    {
      std::lock_guard<std::mutex> g(mu_);
      if (!running_) return;
      start_election_locked(transfer, &hs, &args);
      term = current_term_;
    }
    persist({hs});
  }
  std::lock_guard<std::mutex> g(mu_);
  if (role_ != Role::Candidate || current_term_ != term) return;
  if (config_.has_joint_majority(votes_)) {
    become_leader_locked();
    return;
  }
  for (int p : peers_locked()) {
    if (!config_.is_voter(p)) continue;
    Peer* pp = peer(p);
    pp->vote_body = args;
    pp->vote_term = term;
    pp->vote_pre = false;
    pp->aux_cv.notify_one();
  }
}

void Node::aux_loop(Peer* p) {
  for (;;) {
    std::string body, addr;
    uint64_t term, round;
    bool pre;
    {
      std::unique_lock<std::mutex> lk(mu_);
      p->aux_cv.wait(lk, [&] { return !running_ || !p->vote_body.empty(); });
      if (!running_) return;
      body.swap(p->vote_body);
      term = p->vote_term;
      pre = p->vote_pre;
      round = p->vote_round;
      addr = addr_locked(p->id);
    }
    std::string reply;
    if (addr.empty() || !host_->send(addr, "vote", body, &reply)) continue;
    Json r;
    try {
      r = Json::parse(reply);
    } catch (const std::exception&) {
      continue;
    }
    uint64_t rt = r["term"].as_u64();
    if (rt > term) {
      observe_term(rt, "", -1);
      continue;
    }
    if (pre) {
      bool start = false;
      {
        std::lock_guard<std::mutex> g(mu_);
        if (role_ != Role::Leader && prevote_round_ == round && current_term_ == term &&
            r["vote_granted"].as_bool()) {
          prevotes_.insert(r.has("peer_id") ? static_cast<int>(r["peer_id"].as_int()) : p->id);
          if (config_.has_joint_majority(prevotes_)) {
            ++prevote_round_;  // late yes votes of this round start nothing more
            start = true;
          }
        }
      }
      if (start) run_election(false);
      continue;
    }
    std::lock_guard<std::mutex> g(mu_);
    if (role_ != Role::Candidate || current_term_ != term || !r["vote_granted"].as_bool()) continue;
    votes_.insert(r.has("peer_id") ? static_cast<int>(r["peer_id"].as_int()) : p->id);
    if (config_.has_joint_majority(votes_)) become_leader_locked();
  }
}

void Node::become_leader_locked() {
  if (role_ == Role::Leader) return;
  role_ = Role::Leader;
  leader_id_ = opt_.id;
  leader_address_ = opt_.client_address;
  uint64_t nxt = last_index_locked() + 1;
  next_index_.clear();
  match_index_.clear();
  ack_at_.clear();
  for (int p : peers_locked()) {
    next_index_[p] = nxt;
    match_index_[p] = 0;
  }
  acked_round_.clear();
  leader_noop_index_ = append_local_locked("\"NoOp\"");
  broadcast_locked();
}

bool Node::step_down_locked(uint64_t term, const std::string& leader_addr, int leader_id, Callbacks& cbs) {
  // The role changes in the same step as the term, so a replicator that still saw
  // Leader can never stamp an AppendEntries with a term this node did not win.
  bool was_leader = role_ == Role::Leader;
  role_ = Role::Follower;
  leader_id_ = leader_id;
  leader_address_ = leader_addr;
  bool changed = false;
  if (term > current_term_) {
    current_term_ = term;
    voted_for_ = -1;
    changed = true;
  }
  reset_election_timer_locked();
  if (was_leader) fail_pending_locked(cbs);
  return changed;
}

void Node::observe_term(uint64_t term, const std::string& leader_addr, int leader_id) {
  Callbacks cbs;
  {
    std::lock_guard<std::mutex> w(wal_order_mu_);
    std::string hs;
    {
      std::lock_guard<std::mutex> g(mu_);
      if (term <= current_term_) return;
      step_down_locked(term, leader_addr, leader_id, cbs);
      hs = hs_record();
    }
    persist({hs});
  }
  for (auto& cb : cbs) cb();
}

void Node::fail_pending_locked(Callbacks& cbs) {
  std::string hint = leader_address_;
  for (auto& kv : pending_) {
    Done d = std::move(kv.second.done);
    cbs.push_back([d, hint] { d(1, hint); });
  }
  pending_.clear();
  for (auto& w : read_waiters_) {
    Done d = std::move(w.done);
    cbs.push_back([d, hint] { d(1, hint); });
  }
  read_waiters_.clear();
}

// ---------------------------------------------------------------- proposals
uint64_t Node::append_local_locked(const std::string& cmd) {
  log_.push_back(Entry{current_term_, cmd});
  uint64_t idx = last_index_locked();
  if (unsynced_from_ == 0) unsynced_from_ = idx;
  flush_cv_.notify_one();
  return idx;
}

void Node::propose(const std::string& cmd, Done done) {
  std::string hint;
  {
    std::lock_guard<std::mutex> g(mu_);
    if (role_ == Role::Leader && running_) {
      uint64_t idx = append_local_locked(cmd);
      pending_[idx] = Pending{current_term_, std::move(done)};
      return;
    }
    hint = leader_address_;
  }
  done(1, hint);
}

bool Node::propose_nowait(const std::string& cmd) {
  std::lock_guard<std::mutex> g(mu_);
  if (role_ != Role::Leader || !running_) return false;
  append_local_locked(cmd);
  return true;
}

void Node::flusher_loop() {
  for (;;) {
    {
      std::unique_lock<std::mutex> lk(mu_);
      flush_cv_.wait(lk, [&] { return !running_ || unsynced_from_ != 0; });
      if (!running_) return;
    }
    uint64_t end = 0;
    {
      std::lock_guard<std::mutex> w(wal_order_mu_);
      std::vector<std::string> recs;
      {
        std::lock_guard<std::mutex> g(mu_);
        if (unsynced_from_ == 0) continue;
        uint64_t start = std::max(unsynced_from_, first_index());
        end = last_index_locked();
        unsynced_from_ = 0;
        for (uint64_t i = start; i <= end; ++i) recs.push_back(entry_record(i));
      }
      persist(recs);
    }
    std::lock_guard<std::mutex> g(mu_);
    durable_index_ = std::max(durable_index_, end);
    if (role_ == Role::Leader) {
      advance_commit_locked();
      broadcast_locked();
    }
  }
}

// ---------------------------------------------------------------- replication
void Node::broadcast_locked() {
  if (role_ != Role::Leader) return;
  ++hb_round_;
  for (int p : peers_locked()) {
    Peer* pp = peer(p);
    pp->want_append = true;
    pp->cv.notify_one();
  }
}

void Node::repl_loop(Peer* p) {
  for (;;) {
    {
      std::unique_lock<std::mutex> lk(mu_);
      p->cv.wait(lk, [&] { return !running_ || p->want_append; });
      if (!running_) return;
      p->want_append = false;
    }
    while (running_ && replicate_once(p)) {
      std::lock_guard<std::mutex> g(mu_);
      p->want_append = false;
    }
  }
}

bool Node::replicate_once(Peer* p) {
  std::string body, addr;
  uint64_t term, prev = 0, nxt, rnd = 0, count = 0;
  bool snap = false;
  {
    std::lock_guard<std::mutex> g(mu_);
    if (role_ != Role::Leader) return false;
    addr = addr_locked(p->id);
    if (addr.empty()) return false;
    term = current_term_;
    auto ni = next_index_.find(p->id);
    nxt = ni == next_index_.end() ? last_index_locked() + 1 : ni->second;
    if (nxt <= last_included_index_) {
      snap = true;
    } else {
      prev = nxt - 1;
      uint64_t last = std::min(last_index_locked(), prev + static_cast<uint64_t>(opt_.max_append_batch));
      count = last - prev;
      rnd = hb_round_;
      body = "{\"term\":" + std::to_string(term) + ",\"leader_id\":" + std::to_string(opt_.id) +
             ",\"prev_log_index\":" + std::to_string(prev) + ",\"prev_log_term\":" + std::to_string(term_at(prev)) +
             ",\"entries\":[";
      for (uint64_t i = nxt; i <= last; ++i) {
        if (i > nxt) body += ",";
        body += "{\"term\":" + std::to_string(at(i).term) + ",\"command\":" + at(i).cmd + "}";
      }
      body += "],\"leader_commit\":" + std::to_string(commit_index_) + ",\"leader_address\":";
      json_escape(opt_.client_address, body);
      body += ",\"round\":" + std::to_string(rnd) + "}";
    }
  }
  if (snap) {
    send_snapshot(p);
    return false;
  }
  std::string reply;
  const Clock::time_point sent_at = Clock::now();
  if (!host_->send(addr, "append", body, &reply)) return false;
  Json r;
  try {
    r = Json::parse(reply);
  } catch (const std::exception&) {
    return false;
  }
  uint64_t rterm = r["term"].as_u64();
  if (rterm > term) {
    observe_term(rterm, "", -1);
    return false;
  }
  Callbacks cbs;
  bool more = false;
  {
    std::lock_guard<std::mutex> g(mu_);
    if (role_ != Role::Leader || current_term_ != term) return false;
    // any same-term answer means this follower still takes us as leader (as of sent_at)
    Clock::time_point& ack = ack_at_[p->id];
    ack = std::max(ack, sent_at);
    if (r["success"].as_bool()) {
      uint64_t m = r.has("match_index") ? r["match_index"].as_u64() : prev + count;
      uint64_t& mi = match_index_[p->id];
      mi = std::max(mi, m);
      next_index_[p->id] = mi + 1;
      uint64_t& ar = acked_round_[p->id];
      ar = std::max(ar, rnd);
      auto cu = catch_up_.find(p->id);
      if (cu != catch_up_.end() && m > cu->second.first) {
        cu->second.first = m;
        cu->second.second++;
      }
      advance_commit_locked();
      check_reads_locked(cbs);
      more = next_index_[p->id] <= last_index_locked();
    } else {
      uint64_t hint = r.has("match_index") ? r["match_index"].as_u64() : (prev ? prev - 1 : 0);
      next_index_[p->id] = std::max<uint64_t>(1, std::min(nxt - 1, hint + 1));
      more = true;
    }
  }
  for (auto& cb : cbs) cb();
  return more;
}

void Node::send_snapshot(Peer* p) {
  std::string data;
  for (int attempt = 0; attempt < 2 && data.empty(); ++attempt) {
    std::ifstream f(snap_path(), std::ios::binary);
    if (f) {
      std::stringstream ss;
      ss << f.rdbuf();
      data = ss.str();
    } else {
      take_snapshot();
    }
  }
  if (data.empty()) return;
  uint64_t lii, lit;
  try {
    Json meta = Json::parse(data)["meta"];  // the file's own meta: it may be newer than ours
    lii = meta[0].as_u64();
    lit = meta[1].as_u64();
  } catch (const std::exception&) {
    return;
  }
  std::string body, addr;
  uint64_t term;
  {
    std::lock_guard<std::mutex> g(mu_);
    if (role_ != Role::Leader) return;
    term = current_term_;
    addr = addr_locked(p->id);
    Json a = Json::object();
    a.set("term", term);
    a.set("leader_id", opt_.id);
    a.set("last_included_index", lii);
    a.set("last_included_term", lit);
    a.set("data", data);
    a.set("leader_address", opt_.client_address);
    body = a.dump();
  }
  std::string reply;
  if (!host_->send(addr, "snapshot", body, &reply)) return;
  Json r;
  try {
    r = Json::parse(reply);
  } catch (const std::exception&) {
    return;
  }
  if (r["term"].as_u64() > term) {
    observe_term(r["term"].as_u64(), "", -1);
    return;
  }
  std::lock_guard<std::mutex> g(mu_);
  if (role_ != Role::Leader || current_term_ != term) return;
  uint64_t& mi = match_index_[p->id];
  mi = std::max(mi, r["last_included_index"].as_u64());
  next_index_[p->id] = mi + 1;
  p->want_append = true;
  p->cv.notify_one();
}

void Node::advance_commit_locked() {
  if (role_ != Role::Leader) return;
  uint64_t new_commit = commit_index_;
  for (uint64_t n = last_index_locked(); n > commit_index_; --n) {
    if (term_at(n) != static_cast<int64_t>(current_term_)) break;  // only current-term entries by count
    std::set<int> acks;
    for (auto& kv : match_index_)
      if (kv.second >= n) acks.insert(kv.first);
    if (durable_index_ >= n) acks.insert(opt_.id);
    if (config_.has_joint_majority(acks)) {
      new_commit = n;
      break;
    }
  }
  if (new_commit > commit_index_) {
    commit_index_ = new_commit;
    apply_cv_.notify_one();
  }
}

// ---------------------------------------------------------------- apply
void Node::applier_loop() {
  struct Item {
    uint64_t idx, term;
    std::string cmd;
  };
  for (;;) {
    {
      std::unique_lock<std::mutex> lk(mu_);
      apply_cv_.wait(lk, [&] { return !running_ || commit_index_ > last_applied_; });
      if (!running_) return;
    }
    std::vector<Item> batch;
    std::unique_lock<std::mutex> al(apply_mu_);
    {
      std::lock_guard<std::mutex> g(mu_);
      if (commit_index_ <= last_applied_) continue;
      uint64_t lo = last_applied_ + 1;
      if (lo < first_index()) {  // an installed snapshot already covers these
        last_applied_ = std::max(last_applied_, last_included_index_);
        continue;
      }
      uint64_t hi = std::min(commit_index_, last_index_locked());
      for (uint64_t i = lo; i <= hi; ++i) batch.push_back(Item{i, at(i).term, at(i).cmd});
    }
    if (batch.empty()) continue;
    std::vector<std::string> results(batch.size(), "null");
    Callbacks cbs;
    size_t i = 0;
    while (i < batch.size()) {
      const std::string& cmd = batch[i].cmd;
      if (cmd == "\"NoOp\"") {
        ++i;
        continue;
      }
      if (is_membership(cmd)) {
        std::lock_guard<std::mutex> w(wal_order_mu_);
        std::string rec;
        {
          std::lock_guard<std::mutex> g(mu_);
          try {
            results[i] = apply_membership_locked(Json::parse(cmd)["Membership"], cbs);
          } catch (const std::exception& e) {
            results[i] = std::string("!") + e.what();
          }
          rec = config_record();
        }
        persist({rec});
        ++i;
        continue;
      }
      size_t j = i;
      std::vector<std::pair<uint64_t, std::string>> run;
      while (j < batch.size() && batch[j].cmd != "\"NoOp\"" && !is_membership(batch[j].cmd)) {
        run.emplace_back(batch[j].idx, batch[j].cmd);
        ++j;
      }
      std::vector<std::string> res;
      try {
        res = host_->apply(run);
      } catch (const std::exception& e) {
        res.assign(run.size(), std::string("!") + e.what());
      }
      for (size_t k = 0; k < run.size(); ++k) results[i + k] = k < res.size() ? res[k] : "null";
      i = j;
    }
    bool snap_due;
    {
      std::lock_guard<std::mutex> g(mu_);
      for (size_t k = 0; k < batch.size(); ++k) {
        auto it = pending_.find(batch[k].idx);
        if (it == pending_.end()) continue;
        Done d = std::move(it->second.done);
        uint64_t pterm = it->second.term;
        pending_.erase(it);
        if (pterm != batch[k].term) {
          std::string hint = leader_address_;
          cbs.push_back([d, hint] { d(1, hint); });
        } else if (!results[k].empty() && results[k][0] == '!') {
          std::string msg = results[k].substr(1);
          cbs.push_back([d, msg] { d(2, msg); });
        } else {
          std::string res = results[k];
          cbs.push_back([d, res] { d(0, res); });
        }
      }
      last_applied_ = std::max(last_applied_, batch.back().idx);
      check_reads_locked(cbs);
      for (auto& e : batch) applied_bytes_since_snap_ += e.cmd.size();
      // (a snapshot every 10,000 entries of a 450k-file namespace rewrote ~the whole state about
      // once a second and held applies during each capture: rename p99 37 ms on the box)
      snap_due = last_applied_ - last_included_index_ > opt_.snapshot_threshold &&
                 2 * applied_bytes_since_snap_ >= last_snap_bytes_;
      if (snap_due && !snap_req_) {
        snap_req_ = true;
        snap_cv_.notify_one();
      }
    }
    al.unlock();
    for (auto& cb : cbs) cb();
  }
}

std::string Node::apply_membership_locked(const Json& m, Callbacks& cbs) {
  std::map<int, std::string> members = config_.members;
  if (const Json* a = m.find("AddServer")) {
    members[static_cast<int>((*a)["server_id"].as_int())] = (*a)["server_address"].str();
    config_ = ClusterConfig{members, {}, false, config_.version + 1};
  } else if (const Json* r = m.find("RemoveServer")) {
    // by node id (the reference removes by list index, simple_raft.rs:2549-2571)
    members.erase(static_cast<int>((*r)["server_id"].as_int()));
    config_ = ClusterConfig{members, {}, false, config_.version + 1};
  } else if (const Json* b = m.find("BeginJointConsensus")) {
    config_ = ClusterConfig{members_from((*b)["new_members"]), members_from((*b)["old_members"]), true,
                            (*b)["version"].as_int()};
  } else if (const Json* f = m.find("FinalizeConfiguration")) {
    config_ = ClusterConfig{members_from((*f)["new_members"]), {}, false, (*f)["version"].as_int()};
  }
  for (int p : peers_locked()) {
    if (config_.is_voter(p)) non_voting_.erase(p);
    if (role_ == Role::Leader && !next_index_.count(p)) {
      next_index_[p] = last_index_locked() + 1;
      match_index_[p] = 0;
    }
  }
  if (role_ == Role::Leader && !config_.is_voter(opt_.id)) step_down_locked(current_term_, "", -1, cbs);
  return config_.to_json().dump();
}

void Node::snapshot_loop() {
  std::unique_lock<std::mutex> g(mu_);
  for (;;) {
    snap_cv_.wait(g, [&] { return snap_req_ || !running_; });
    if (!running_) return;
    g.unlock();
    take_snapshot();
    g.lock();
    snap_req_ = false;  // entries applied meanwhile re-request it on a later batch if still due
  }
}

// Compaction: the state is captured under apply_mu_ (applies wait only for the capture), then
// the snapshot file is written and the WAL rewritten without it; entries applied meanwhile
// stay in the log (idx is the captured index). snap_mu_ keeps an InstallSnapshot from
// interleaving with the file write.
void Node::take_snapshot() {
  std::lock_guard<std::mutex> sl(snap_mu_);
  uint64_t idx, term;
  std::string cfg, state;
  {
    std::lock_guard<std::mutex> al(apply_mu_);
    {
      std::lock_guard<std::mutex> g(mu_);
      idx = last_applied_;
      if (idx == 0 || idx <= last_included_index_) return;
      term = static_cast<uint64_t>(std::max<int64_t>(0, term_at(idx)));
      cfg = config_.to_json().dump();
      applied_bytes_since_snap_ = 0;
    }
    state = host_->snapshot();
  }
  std::string data = "{\"meta\":[" + std::to_string(idx) + "," + std::to_string(term) + "],\"state\":" + state +
                     ",\"config\":" + cfg + "}";
  state.clear();
  {
    std::lock_guard<std::mutex> g(mu_);
    last_snap_bytes_ = data.size();
  }
  atomic_write_file(snap_path(), data, opt_.sync);
  bool leader;
  {
    std::lock_guard<std::mutex> w(wal_order_mu_);
    std::vector<std::string> recs;
    {
      std::lock_guard<std::mutex> g(mu_);
      if (idx > last_included_index_) {
        uint64_t drop = std::min<uint64_t>(idx - first_index() + 1, log_.size());
        log_.erase(log_.begin(), log_.begin() + static_cast<std::ptrdiff_t>(drop));
        last_included_index_ = idx;
        last_included_term_ = term;
      }
      recs.push_back(hs_record());
      recs.push_back(config_record());
      for (uint64_t i = first_index(); i <= last_index_locked(); ++i) recs.push_back(entry_record(i));
      leader = role_ == Role::Leader;
    }
    wal_->reset(recs);
  }
  if (leader && !opt_.backup_endpoint.empty()) {
    std::string ep = opt_.backup_endpoint;
    while (!ep.empty() && ep.back() == '/') ep.pop_back();
    std::string url = ep + "/" + opt_.backup_bucket + "/master-snapshots/node-" + std::to_string(opt_.id) + "/" +
                      std::to_string(static_cast<long long>(std::time(nullptr))) + "--idx" + std::to_string(idx) +
                      ".bin";
    host_->backup(url, data);
  }
}

void Node::snapshot_now() { take_snapshot(); }

// ---------------------------------------------------------------- linearizable reads
void Node::read_index(Done done) {
  Callbacks cbs;
  {
    std::lock_guard<std::mutex> g(mu_);
    if (role_ != Role::Leader || !running_) {
      std::string hint = leader_address_;
      cbs.push_back([done, hint] { done(1, hint); });
    } else {
      // everything committed before this term is at or below our NoOp
      uint64_t idx = std::max(commit_index_, leader_noop_index_);
      bool solo = peers_locked().empty();
      read_waiters_.push_back(ReadWaiter{idx, solo ? 0 : hb_round_ + 1, std::move(done)});
      if (!solo) broadcast_locked();
      check_reads_locked(cbs);
    }
  }
  for (auto& cb : cbs) cb();
}

void Node::check_reads_locked(Callbacks& cbs) {
  if (read_waiters_.empty() || role_ != Role::Leader) return;
  std::vector<ReadWaiter> keep;
  for (auto& w : read_waiters_) {
    bool confirmed = w.need_round == 0;
    if (!confirmed) {
      std::set<int> acks = {opt_.id};
      for (auto& kv : acked_round_)
        if (kv.second >= w.need_round) acks.insert(kv.first);
      confirmed = config_.has_joint_majority(acks);
    }
    if (confirmed && last_applied_ >= w.index) {
      Done d = std::move(w.done);
      std::string idx = std::to_string(w.index);
      cbs.push_back([d, idx] { d(0, idx); });
    } else {
      keep.push_back(std::move(w));
    }
  }
  read_waiters_.swap(keep);
}

// ---------------------------------------------------------------- RPC handlers
std::string Node::handle(const std::string& kind, const std::string& body) {
  Json a = Json::parse(body);
  if (kind == "append") return on_append(a);
  if (kind == "vote") return on_vote(a);
  if (kind == "snapshot") return on_snapshot(a);
  if (kind == "timeout_now") return on_timeout_now(a);
  throw std::runtime_error("unknown raft rpc " + kind);
}

std::string Node::on_vote(const Json& a) {
  Callbacks cbs;
  Json out = Json::object();
  {
    std::lock_guard<std::mutex> w(wal_order_mu_);
    std::vector<std::string> recs;
    {
      std::lock_guard<std::mutex> g(mu_);
      uint64_t t = a["term"].as_u64();
      const bool pre = a["pre_vote"].as_bool();
      const int cand = static_cast<int>(a["candidate_id"].as_int());
      uint64_t my_last = last_index_locked();
      int64_t my_term = term_at(my_last);
      int64_t llt = a["last_log_term"].as_int();
      const bool log_ok = llt > my_term || (llt == my_term && a["last_log_index"].as_u64() >= my_last);
      // a live leader exists: neither a pre-vote nor a newer term from a candidate that is
      // not a leadership transfer target (thesis 4.2.3 / 9.6)
      const bool sticky = opt_.pre_vote && !a["transfer"].as_bool() && t > current_term_ && leader_recent_locked();
      if (pre || sticky) {
        out.set("term", current_term_);
        out.set("vote_granted", pre && !sticky && t > current_term_ && log_ok);
        out.set("peer_id", opt_.id);
        return out.dump();  // no state changed, nothing to persist
      }
      if (t > current_term_ && step_down_locked(t, "", -1, cbs)) recs.push_back(hs_record());
      bool granted = false;
      if (t == current_term_ && (voted_for_ == -1 || voted_for_ == cand)) {
        if (log_ok) {
          granted = true;
          voted_for_ = cand;
          recs.push_back(hs_record());
          reset_election_timer_locked();
        }
      }
      out.set("term", current_term_);
      out.set("vote_granted", granted);
      out.set("peer_id", opt_.id);
    }
    persist(recs);  // the vote is durable before the candidate learns of it
  }
  for (auto& cb : cbs) cb();
  return out.dump();
}

std::string Node::on_append(const Json& a) {
  std::lock_guard<std::mutex> am(append_mu_);
  Callbacks cbs;
  Json out = Json::object();
  {
    std::lock_guard<std::mutex> w(wal_order_mu_);
    std::vector<std::string> recs;
    bool ok = false;
    uint64_t last_new = 0, leader_commit = a["leader_commit"].as_u64();
    {
      std::lock_guard<std::mutex> g(mu_);
      uint64_t t = a["term"].as_u64();
      out.set("peer_id", opt_.id);
      if (t < current_term_) {
        out.set("term", current_term_);
        out.set("success", false);
        out.set("match_index", last_index_locked());
        return out.dump();
      }
      int lid = static_cast<int>(a["leader_id"].as_int(-1));
      if ((t > current_term_ || role_ != Role::Follower) && step_down_locked(t, a["leader_address"].str(), lid, cbs))
        recs.push_back(hs_record());
      leader_id_ = lid;
      leader_address_ = a["leader_address"].str();
      leader_contact_ = Clock::now();
      reset_election_timer_locked();
      uint64_t prev = a["prev_log_index"].as_u64();
      if (prev > last_index_locked()) {
        out.set("match_index", last_index_locked());
      } else if (prev >= last_included_index_ && term_at(prev) != a["prev_log_term"].as_int()) {
        out.set("match_index", std::min(prev ? prev - 1 : 0, commit_index_));
      } else {
        uint64_t idx = prev;
        for (const Json& e : a["entries"].items()) {
          ++idx;
          if (idx <= last_included_index_) continue;
          uint64_t et = e["term"].as_u64();
          if (idx <= last_index_locked()) {
            if (term_at(idx) == static_cast<int64_t>(et)) continue;
            log_.resize(idx - first_index());  // conflict: drop this entry and all after it
            recs.push_back("{\"k\":\"T\",\"from\":" + std::to_string(idx) + "}");
          }
          log_.push_back(Entry{et, e["command"].dump()});
          recs.push_back(entry_record(idx));
        }
        ok = true;
        last_new = prev + a["entries"].size();
      }
      out.set("term", current_term_);
      out.set("success", ok);
    }
    persist(recs);
    if (ok) {
      std::lock_guard<std::mutex> g(mu_);
      durable_index_ = last_index_locked();
      if (leader_commit > commit_index_) {
        commit_index_ = std::max(commit_index_, std::min(leader_commit, last_new));
        apply_cv_.notify_one();
      }
      out.set("match_index", last_new);
    }
  }
  for (auto& cb : cbs) cb();
  return out.dump();
}

std::string Node::on_snapshot(const Json& a) {
  std::lock_guard<std::mutex> am(append_mu_);
  std::lock_guard<std::mutex> sl(snap_mu_);  // not while a compaction writes the snapshot file
  std::unique_lock<std::mutex> al(apply_mu_);
  Callbacks cbs;
  Json out = Json::object();
  out.set("peer_id", opt_.id);
  {
    std::lock_guard<std::mutex> w(wal_order_mu_);
    std::vector<std::string> recs;
    uint64_t lii = a["last_included_index"].as_u64(), lit = a["last_included_term"].as_u64();
    bool install = false;
    {
      std::lock_guard<std::mutex> g(mu_);
      uint64_t t = a["term"].as_u64();
      if (t >= current_term_) {
        int lid = static_cast<int>(a["leader_id"].as_int(-1));
        if ((t > current_term_ || role_ != Role::Follower) &&
            step_down_locked(t, a["leader_address"].str(), lid, cbs))
          recs.push_back(hs_record());
        leader_id_ = lid;
        leader_address_ = a["leader_address"].str();
        leader_contact_ = Clock::now();
        reset_election_timer_locked();
        // a snapshot at or behind what we already applied would roll the state back
        install = lii > last_included_index_ && lii > last_applied_;
      }
    }
    persist(recs);
    if (install) {
      const std::string& data = a["data"].as_string();
      Json snap = Json::parse(data);
      atomic_write_file(snap_path(), data, opt_.sync);
      host_->restore(snap["state"].dump());
      std::vector<std::string> all;
      {
        std::lock_guard<std::mutex> g(mu_);
        if (lii <= last_index_locked() && term_at(lii) == static_cast<int64_t>(lit)) {
          log_.erase(log_.begin(), log_.begin() + static_cast<std::ptrdiff_t>(lii - first_index() + 1));
        } else {
          log_.clear();
        }
        last_included_index_ = lii;
        last_included_term_ = lit;
        if (!snap["config"].is_null()) config_ = ClusterConfig::from_json(snap["config"]);
        commit_index_ = std::max(commit_index_, lii);
        last_applied_ = lii;
        durable_index_ = last_index_locked();
        all.push_back(hs_record());
        all.push_back(config_record());
        for (uint64_t i = first_index(); i <= last_index_locked(); ++i) all.push_back(entry_record(i));
      }
      wal_->reset(all);
    }
    std::lock_guard<std::mutex> g(mu_);
    out.set("term", current_term_);
    out.set("last_included_index", last_included_index_);
  }
  al.unlock();
  for (auto& cb : cbs) cb();
  return out.dump();
}

std::string Node::on_timeout_now(const Json& a) {
  Json out = Json::object();
  bool ok;
  {
    std::lock_guard<std::mutex> g(mu_);
    ok = a["term"].as_u64() >= current_term_ && role_ != Role::Leader && config_.is_voter(opt_.id);
    out.set("term", current_term_);
    out.set("success", ok);
  }
  // start the (transfer) election here and now: handing it to the ticker raced with the old
  // leader's next heartbeat, which re-arms the election timer before the ticker looks
  if (ok) run_election(true);
  return out.dump();
}

bool Node::transfer_leadership(int target) {
  std::string addr, body;
  {
    std::lock_guard<std::mutex> g(mu_);
    if (role_ != Role::Leader || !config_.is_voter(target)) return false;
    addr = addr_locked(target);
    Json a = Json::object();
    a.set("term", current_term_);
    a.set("sender_id", opt_.id);
    body = a.dump();
  }
  std::string reply;
  if (!host_->send(addr, "timeout_now", body, &reply)) return false;
  try {
    return Json::parse(reply)["success"].as_bool();
  } catch (const std::exception&) {
    return false;
  }
}

// ---------------------------------------------------------------- membership helpers
void Node::add_non_voter(int id, const std::string& addr) {
  std::lock_guard<std::mutex> g(mu_);
  non_voting_[id] = addr;
  catch_up_[id] = {0, 0};
  next_index_[id] = last_index_locked() + 1;
  match_index_[id] = 0;
  if (running_) peer(id);
  broadcast_locked();
}

void Node::drop_non_voter(int id) {
  std::lock_guard<std::mutex> g(mu_);
  catch_up_.erase(id);
  if (!config_.is_voter(id)) non_voting_.erase(id);
}

bool Node::caught_up(int id) {
  std::lock_guard<std::mutex> g(mu_);
  auto it = catch_up_.find(id);
  if (it == catch_up_.end()) return true;
  broadcast_locked();
  return it->second.first >= commit_index_ && it->second.second >= 10;
}

// ---------------------------------------------------------------- introspection
Role Node::role() const {
  std::lock_guard<std::mutex> g(mu_);
  return role_;
}
uint64_t Node::term() const {
  std::lock_guard<std::mutex> g(mu_);
  return current_term_;
}
int Node::leader_id() const {
  std::lock_guard<std::mutex> g(mu_);
  return leader_id_;
}
std::string Node::leader_address() const {
  std::lock_guard<std::mutex> g(mu_);
  return leader_address_;
}
uint64_t Node::commit_index() const {
  std::lock_guard<std::mutex> g(mu_);
  return commit_index_;
}
uint64_t Node::last_applied() const {
  std::lock_guard<std::mutex> g(mu_);
  return last_applied_;
}
uint64_t Node::last_index() const {
  std::lock_guard<std::mutex> g(mu_);
  return last_index_locked();
}
uint64_t Node::last_included_index() const {
  std::lock_guard<std::mutex> g(mu_);
  return last_included_index_;
}
size_t Node::votes() const {
  std::lock_guard<std::mutex> g(mu_);
  return votes_.size();
}
ClusterConfig Node::config() const {
  std::lock_guard<std::mutex> g(mu_);
  return config_;
}

std::string Node::info_json() const {
  std::lock_guard<std::mutex> g(mu_);
  Json o = Json::object();
  o.set("node_id", opt_.id);
  o.set("role", role_name(role_));
  o.set("current_term", current_term_);
  o.set("leader_id", leader_id_ < 0 ? Json() : Json(leader_id_));
  o.set("leader_address", leader_address_.empty() ? Json() : Json(leader_address_));
  Json peers = Json::array();
  for (int p : peers_locked()) peers.push_back(addr_locked(p));
  o.set("peers", peers);
  o.set("commit_index", commit_index_);
  o.set("last_applied", last_applied_);
  o.set("log_len", last_index_locked());
  o.set("votes_received", static_cast<uint64_t>(votes_.size()));
  o.set("cluster_config", config_.to_json());
  o.set("wal_bytes", wal_->size_bytes());
  o.set("wal_syncs", wal_->syncs());
  o.set("snapshot_index", last_included_index_);
  return o.dump();
}

bool restore_snapshot_dir(const std::string& dir, const std::string& payload, std::string* err) {
  mkdirs(dir);
  struct stat sb {};
  if (::stat((dir + "/snapshot.json").c_str(), &sb) == 0) {
    *err = dir + " already holds a snapshot";
    return false;
  }
  if (::stat((dir + "/raft.wal").c_str(), &sb) == 0) {
    Wal existing(dir + "/raft.wal", false);
    if (!existing.replay().empty()) {
      *err = dir + " already holds a Raft log";
      return false;
    }
  }
  Json snap;
  try {
    snap = Json::parse(payload);
  } catch (const std::exception& e) {
    *err = std::string("not a snapshot backup (JSON): ") + e.what();
    return false;
  }
  if (!snap.is_object() || !snap["meta"].is_array() || snap["meta"].size() != 2 || !snap["meta"][0].is_int() ||
      !snap["meta"][1].is_int() || !snap["state"].is_object()) {
    *err = "not a snapshot backup: want {\"meta\":[index,term],\"state\":{...}}";
    return false;
  }
  const uint64_t idx = snap["meta"][0].as_u64(), term = snap["meta"][1].as_u64();
  atomic_write_file(dir + "/snapshot.json",
                    "{\"meta\":[" + std::to_string(idx) + "," + std::to_string(term) + "],\"state\":" +
                        snap["state"].dump() + ",\"config\":null}",
                    true);
  Wal w(dir + "/raft.wal", true);
  w.append({"{\"k\":\"H\",\"term\":" + std::to_string(term) + ",\"vote\":null}"});
  return true;
}

}  // namespace dfs::raft
