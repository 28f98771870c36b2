#include "lin_checker.h"

#include <algorithm>
#include <functional>
#include <map>
#include <numeric>
#include <set>
#include <sstream>
#include <unordered_map>
#include <unordered_set>

#include "json.h"

namespace dfs::lin {

namespace {

bool known_op(const std::string& op) { return op == "put" || op == "get" || op == "delete" || op == "rename"; }

Op make_op(const Json& inv, int64_t ret_ts, const std::string& result) {
  Op o;
  o.id = inv["id"].as_int();
  o.client = inv["client"].str();
  o.op = inv["op"].str();
  o.path = inv["path"].str();
  o.src = inv["src"].str();
  o.dst = inv["dst"].str();
  o.data_hash = inv["data_hash"].str();
  o.invoke_ts = inv["ts_ns"].as_int();
  o.return_ts = ret_ts;
  o.result = result;
  return o;
}

using State = std::map<std::string, std::string>;  // path -> content hash

// The sequential specification: applies `op` to `s` (in place when it succeeds) and returns
// the result the specification expects.
std::string apply(State* s, const Op& op, bool* changed) {
  *changed = false;
  if (op.op == "put") {
    if (s->count(op.path)) return "error";
    (*s)[op.path] = op.data_hash;
    *changed = true;
    return "put_ok:" + op.data_hash;
  }
  if (op.op == "get") {
    auto it = s->find(op.path);
    return it == s->end() ? "not_found" : "get_ok:" + it->second;
  }
  if (op.op == "delete") {
    if (!s->erase(op.path)) return "not_found";
    *changed = true;
    return "ok";
  }
  auto it = s->find(op.src);
  if (it == s->end() || s->count(op.dst)) return "error";
  std::string h = it->second;
  s->erase(it);
  (*s)[op.dst] = h;
  *changed = true;
  return "ok";
}

bool matches(const std::string& expected, const Op& op) {
  if (op.ambiguous()) return true;
  if (op.op == "rename" && op.result == "not_found") return expected == "error";
  return expected == op.result;
}

struct BudgetExhausted {};

class Search {
 public:
  Search(const std::vector<Op>& ops, uint64_t budget) : ops_(ops), budget_(budget), done_(ops.size(), false) {}

  bool run() {
    State s;
    return go(&s, 0);
  }
  size_t best_depth() const { return best_.size(); }
  const std::vector<size_t>& best() const { return best_; }

 private:
  std::string memo_key(const State& s) const {
    std::string k(done_.size(), '0');
    for (size_t i = 0; i < done_.size(); ++i)
      if (done_[i]) k[i] = '1';
    for (auto& kv : s) {
      k.push_back('\0');
      k += kv.first;
      k.push_back('\1');
      k += kv.second;
    }
    return k;
  }

  bool go(State* s, size_t placed) {
    if (placed == ops_.size()) return true;
    if (++steps_ > budget_) throw BudgetExhausted{};
    if (!seen_.insert(memo_key(*s)).second) return false;
    if (order_.size() > best_.size()) best_ = order_;
    // an op may be linearized next only if no other pending op returned before it was invoked
    int64_t min_ret = INT64_MAX;
    for (size_t i = 0; i < ops_.size(); ++i)
      if (!done_[i]) min_ret = std::min(min_ret, ops_[i].return_ts);
    for (size_t i = 0; i < ops_.size(); ++i) {
      if (done_[i]) continue;
      const Op& op = ops_[i];
      if (op.invoke_ts > min_ret) continue;
      State next = *s;
      bool changed;
      const std::string exp = apply(&next, op, &changed);
      done_[i] = true;
      order_.push_back(i);
      if (matches(exp, op) && go(&next, placed + 1)) return true;
      // an op with an unknown outcome may also never have taken effect
      if (op.ambiguous() && changed && go(s, placed + 1)) return true;
      order_.pop_back();
      done_[i] = false;
    }
    return false;
  }

  const std::vector<Op>& ops_;
  uint64_t budget_, steps_ = 0;
  std::vector<bool> done_;
  std::vector<size_t> order_, best_;
  std::unordered_set<std::string> seen_;
};

std::vector<std::vector<Op>> components(const std::vector<Op>& ops) {
  std::unordered_map<std::string, std::string> parent;
  std::function<std::string(const std::string&)> find = [&](const std::string& x) -> std::string {
    auto it = parent.find(x);
    if (it == parent.end()) {
      parent[x] = x;
      return x;
    }
    if (it->second == x) return x;
    std::string r = find(it->second);
    parent[x] = r;
    return r;
  };
  for (auto& op : ops) {
    auto ks = op.keys();
    std::string r0 = find(ks[0]);
    for (size_t i = 1; i < ks.size(); ++i) {
      std::string r = find(ks[i]);
      if (r != r0) parent[r] = r0;
    }
  }
  std::map<std::string, std::vector<Op>> groups;
  for (auto& op : ops) groups[find(op.keys()[0])].push_back(op);
  std::vector<std::vector<Op>> out;
  for (auto& g : groups) out.push_back(std::move(g.second));
  return out;
}

std::string key_list(const std::vector<Op>& comp) {
  std::set<std::string> ks;
  for (auto& o : comp)
    for (auto& k : o.keys()) ks.insert(k);
  std::string s = "[";
  for (auto& k : ks) s += (s.size() > 1 ? ", '" : "'") + k + "'";
  return s + "]";
}

}  // namespace

bool parse_history(std::istream& in, std::vector<Op>* ops, std::string* err) {
  std::map<int64_t, Json> invokes;
  std::map<int64_t, Op> done;
  std::string line;
  int no = 0;
  while (std::getline(in, line)) {
    ++no;
    if (line.find_first_not_of(" \t\r\n") == std::string::npos) continue;
    Json e;
    try {
      e = Json::parse(line);
    } catch (const std::exception& ex) {
      *err = "line " + std::to_string(no) + ": " + ex.what();
      return false;
    }
    const std::string t = e["type"].str();
    if (t == "invoke") {
      if (!known_op(e["op"].str())) return (*err = "unknown op '" + e["op"].str() + "'", false);
      invokes[e["id"].as_int()] = e;
    } else if (t == "return") {
      auto it = invokes.find(e["id"].as_int());
      if (it == invokes.end())
        return (*err = "return without matching invoke for id " + std::to_string(e["id"].as_int()), false);
      done[it->first] = make_op(it->second, e["ts_ns"].as_int(), e["result"].str());
      invokes.erase(it);
    } else {
      *err = "unknown entry type '" + t + "' at line " + std::to_string(no);
      return false;
    }
  }
  for (auto& kv : invokes) done[kv.first] = make_op(kv.second, INT64_MAX, "");
  ops->clear();
  for (auto& kv : done) ops->push_back(kv.second);
  return true;
}

std::vector<std::string> check(const std::vector<Op>& ops, uint64_t budget) {
  std::vector<std::string> violations;
  for (auto& comp : components(ops)) {
    std::stable_sort(comp.begin(), comp.end(), [](const Op& a, const Op& b) { return a.invoke_ts < b.invoke_ts; });
    Search s(comp, budget);
    bool ok;
    try {
      ok = s.run();
    } catch (const BudgetExhausted&) {
      violations.push_back("search budget exhausted on " + std::to_string(comp.size()) + " ops over keys " +
                           key_list(comp));
      continue;
    }
    if (ok) continue;
    std::vector<bool> placed(comp.size(), false);
    for (size_t i : s.best()) placed[i] = true;
    const Op* first = nullptr;
    for (size_t i = 0; i < comp.size(); ++i)
      if (!placed[i] && (!first || comp[i].invoke_ts < first->invoke_ts)) first = &comp[i];
    std::string detail;
    if (first) {
      std::string ks;
      for (auto& k : first->keys()) ks += (ks.empty() ? "" : ", ") + std::string("'") + k + "'";
      detail = "; first unlinearizable op: id=" + std::to_string(first->id) + " " + first->op + " (" + ks +
               (first->keys().size() == 1 ? ",)" : ")") + " -> '" + first->result + "'";
    }
    violations.push_back("non-linearizable history over keys " + key_list(comp) + " (" +
                         std::to_string(s.best_depth()) + "/" + std::to_string(comp.size()) + " ops placed)" +
                         detail);
  }
  return violations;
}

std::vector<std::string> self_test() {
  auto inv = [](int id, const char* op, int ts, const std::string& kv, const char* client = "c1") {
    return std::string("{\"id\":") + std::to_string(id) + ",\"client\":\"" + client +
           "\",\"type\":\"invoke\",\"op\":\"" + op + "\",\"ts_ns\":" + std::to_string(ts) + kv + "}";
  };
  auto ret = [](int id, const char* result, int ts, const char* client = "c1") {
    return std::string("{\"id\":") + std::to_string(id) + ",\"client\":\"" + client +
           "\",\"type\":\"return\",\"result\":\"" + result + "\",\"ts_ns\":" + std::to_string(ts) + "}";
  };
  const std::string pa = ",\"path\":\"/a\"", pz = ",\"path\":\"/z\"";
  auto put = [&](const char* h) { return pa + ",\"data_hash\":\"" + h + "\""; };
  const std::string mv = ",\"src\":\"/a\",\"dst\":\"/z\"";
  const std::vector<std::pair<std::string, std::pair<bool, std::vector<std::string>>>> cases = {
      {"sequential_put_get", {true, {inv(1, "put", 1, put("h1")), ret(1, "put_ok:h1", 2), inv(2, "get", 3, pa),
                                     ret(2, "get_ok:h1", 4)}}},
      {"stale_read", {false, {inv(1, "put", 1, put("h1")), ret(1, "put_ok:h1", 2), inv(2, "delete", 3, pa),
                              ret(2, "ok", 4), inv(3, "get", 5, pa), ret(3, "get_ok:h1", 6)}}},
      {"lost_write", {false, {inv(1, "put", 1, put("h1")), ret(1, "put_ok:h1", 2), inv(2, "get", 3, pa),
                              ret(2, "not_found", 4)}}},
      {"duplicated_value", {false, {inv(1, "put", 1, put("h1")), ret(1, "put_ok:h1", 2), inv(2, "put", 3, put("h2")),
                                    ret(2, "put_ok:h2", 4)}}},
      {"concurrent_put_get", {true, {inv(1, "put", 1, put("h1")), inv(2, "get", 2, pa, "c2"),
                                     ret(2, "get_ok:h1", 3, "c2"), ret(1, "put_ok:h1", 4)}}},
      {"rename_moves_value", {true, {inv(1, "put", 1, put("h1")), ret(1, "put_ok:h1", 2), inv(2, "rename", 3, mv),
                                     ret(2, "ok", 4), inv(3, "get", 5, pz), ret(3, "get_ok:h1", 6),
                                     inv(4, "get", 7, pa), ret(4, "not_found", 8)}}},
      {"rename_lost", {false, {inv(1, "put", 1, put("h1")), ret(1, "put_ok:h1", 2), inv(2, "rename", 3, mv),
                               ret(2, "ok", 4), inv(3, "get", 5, pz), ret(3, "not_found", 6)}}},
      {"crashed_put_may_apply", {true, {inv(1, "put", 1, put("h1")), inv(2, "get", 5, pa, "c2"),
                                        ret(2, "get_ok:h1", 6, "c2")}}},
      {"crashed_put_may_not_apply", {true, {inv(1, "put", 1, put("h1")), inv(2, "get", 5, pa, "c2"),
                                            ret(2, "not_found", 6, "c2")}}},
      {"error_is_ambiguous", {true, {inv(1, "delete", 1, pa), ret(1, "error", 2), inv(2, "get", 3, pa),
                                     ret(2, "not_found", 4)}}},
  };
  std::vector<std::string> failures;
  for (auto& c : cases) {
    std::string text;
    for (auto& l : c.second.second) text += l + "\n";
    std::istringstream in(text);
    std::vector<Op> ops;
    std::string err;
    if (!parse_history(in, &ops, &err)) {
      failures.push_back(c.first + ": parse error " + err);
      continue;
    }
    const bool ok = check(ops).empty();
    if (ok != c.second.first)
      failures.push_back(c.first + ": expected " + (c.second.first ? "linearizable" : "violation"));
  }
  return failures;
}

}  // namespace dfs::lin
