// Linearizability checker for DFS histories (C49; reference dfs/client/src/checker.rs), the
// native form of client/checker.py that `dfs_cli check-history` runs.
//
// Input: JSONL invoke/return records (id, client, type, op, path, src, dst, data_hash,
// result, ts_ns); an invoke without a return is a crashed op. Sequential specification, a
// map path -> content hash:
//   put(p, h)    p absent -> store h, "put_ok:h"; p present -> fails (CreateFile refuses)
//   get(p)       "get_ok:h" / "not_found"
//   delete(p)    "ok" (p removed) / "not_found"
//   rename(s,d)  s present and d absent -> moved, "ok"; otherwise it fails
// Ops whose outcome is unknown ("error" results, crashed ops) may or may not have taken
// effect. The search is Wing-Gong-Leung with memoisation over (linearized set, state), run
// per connected component of keys (renames link keys), under a step budget whose exhaustion
// is reported as a violation, never passed silently.
#pragma once
#include <cstdint>
#include <istream>
#include <string>
#include <vector>

namespace dfs::lin {

struct Op {
  int64_t id = 0;
  std::string client, op, path, src, dst, data_hash, result;
  int64_t invoke_ts = 0;
  int64_t return_ts = INT64_MAX;  // INT64_MAX: crashed (no return record)
  bool ambiguous() const { return return_ts == INT64_MAX || result.empty() || result == "error"; }
  std::vector<std::string> keys() const {
    return op == "rename" ? std::vector<std::string>{src, dst} : std::vector<std::string>{path};
  }
};

// Parses a JSONL history; false with *err on a malformed line, an unknown op or type, or a
// return without its invoke.
bool parse_history(std::istream& in, std::vector<Op>* ops, std::string* err);
// Violations (empty: linearizable).
std::vector<std::string> check(const std::vector<Op>& ops, uint64_t budget = 2000000);
// The checker's self-tests (the same cases as client/checker.py): failures, empty when all pass.
std::vector<std::string> self_test();

}  // namespace dfs::lin
