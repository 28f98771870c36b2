// IAM and bucket policy evaluation (see s3_policy.h).
#include "s3_policy.h"

#include <algorithm>
#include <stdexcept>

#include "json.h"

namespace dfs {
namespace s3policy {

namespace {

// Python's `re` works on code points: `?` consumes one UTF-8 sequence, not one byte.
size_t cp_len(unsigned char c) { return c < 0x80 ? 1 : c >= 0xF0 ? 4 : c >= 0xE0 ? 3 : c >= 0xC0 ? 2 : 1; }

std::vector<std::string> as_list(const Json& v) {
  std::vector<std::string> out;
  if (v.is_null()) return out;
  if (v.is_string()) return {v.as_string()};
  if (v.is_array()) {
    for (auto& e : v.items()) out.push_back(e.is_string() ? e.as_string() : e.dump());
    return out;
  }
  return {v.dump()};
}

std::optional<std::vector<std::string>> opt_list(const Json* v) {
  if (!v || v->is_null()) return std::nullopt;
  return as_list(*v);
}

Statement statement(const Json& d) {
  if (!d.is_object() || !d.has("Effect") || !d.has("Action")) throw std::runtime_error("statement needs Effect and Action");
  Statement s;
  s.effect = d["Effect"].str();
  s.actions = as_list(d["Action"]);
  s.resources = opt_list(d.find("Resource"));
  if (const Json* c = d.find("Condition"); c && !c->is_null()) {
    if (!c->is_object()) throw std::runtime_error("Condition must be an object");
    std::map<std::string, std::map<std::string, std::vector<std::string>>> cond;
    for (auto& op : c->fields()) {
      if (!op.second.is_object()) throw std::runtime_error("Condition operator must map keys");
      auto& keys = cond[op.first];
      for (auto& kv : op.second.fields()) keys[kv.first] = as_list(kv.second);
    }
    s.condition = std::move(cond);
  }
  return s;
}

std::vector<Statement> statements(const Json& doc) {
  std::vector<Statement> out;
  const Json& st = doc["Statement"];
  if (!st.is_array()) throw std::runtime_error("Statement must be a list");
  for (auto& s : st.items()) out.push_back(statement(s));
  return out;
}

bool any_match(const std::vector<std::string>& pats, const std::string& v) {
  return std::any_of(pats.begin(), pats.end(), [&](const std::string& p) { return matches_wildcard(p, v); });
}

bool condition_holds(const std::map<std::string, std::map<std::string, std::vector<std::string>>>& cond,
                     const Context& ctx) {
  for (auto& [op, keys] : cond)
    for (auto& [key, expected] : keys) {
      std::vector<std::string> actual;
      if (key == "OIDC_ISSUER:groups") {
        actual = ctx.groups;
      } else if (key.compare(0, 12, "OIDC_ISSUER:") == 0) {
        auto it = ctx.claims.find(key.substr(12));
        if (it != ctx.claims.end()) actual.push_back(it->second);
      }
      auto in = [&](const std::string& a) { return std::find(expected.begin(), expected.end(), a) != expected.end(); };
      if (op == "StringEquals") {
        if (actual.empty() || !in(actual[0])) return false;
      } else if (op == "ForAnyValue:StringEquals") {
        if (!std::any_of(actual.begin(), actual.end(), in)) return false;
      } else {
        return false;  // unknown operators fail closed
      }
    }
  return true;
}

}  // namespace

static bool glob(const std::string& pattern, const std::string& target);

bool matches_wildcard(const std::string& pattern, const std::string& target) {
  if (pattern == "*") return true;
  if (glob(pattern, target)) return true;
  return !target.empty() && target.back() == '\n' && glob(pattern, target.substr(0, target.size() - 1));
}

static bool glob(const std::string& pattern, const std::string& target) {
  // iterative glob with backtracking to the last `*`
  size_t p = 0, t = 0, star = std::string::npos, mark = 0;
  while (t < target.size()) {
    if (p < pattern.size() && pattern[p] == '?') {
      ++p;
      t += cp_len(static_cast<unsigned char>(target[t]));
    } else if (p < pattern.size() && pattern[p] == '*') {
      star = p++;
      mark = t;
    } else if (p < pattern.size() && pattern[p] == target[t]) {
      ++p;
      ++t;
    } else if (star != std::string::npos) {
      p = star + 1;
      mark += cp_len(static_cast<unsigned char>(target[mark]));
      t = mark;
    } else {
      return false;
    }
  }
  if (t > target.size()) return false;
  while (p < pattern.size() && pattern[p] == '*') ++p;
  return p == pattern.size();
}

bool evaluate_statements(const std::vector<Statement>& stmts, const std::string& action, const std::string& resource,
                         const Context& ctx) {
  bool allow = false;
  for (auto& s : stmts) {
    if (!any_match(s.actions, action)) continue;
    if (s.resources && !any_match(*s.resources, resource)) continue;
    if (s.condition && !condition_holds(*s.condition, ctx)) continue;
    if (s.effect == "Deny") return false;
    if (s.effect == "Allow") allow = true;
  }
  return allow;
}

IamPolicy IamPolicy::parse(const std::string& text) {
  Json doc = Json::parse(text);
  IamPolicy out;
  const Json& roles = doc["Roles"];
  if (!roles.is_array()) throw std::runtime_error("IamConfig needs Roles");
  for (auto& r : roles.items()) {
    if (!r.has("RoleName") || !r.has("Arn") || !r.has("AssumeRolePolicyDocument"))
      throw std::runtime_error("role needs RoleName, Arn and AssumeRolePolicyDocument");
    Role role;
    role.name = r["RoleName"].str();
    role.trust = statements(r["AssumeRolePolicyDocument"]);
    if (const Json* pols = r.find("Policies"); pols && pols->is_array())
      for (auto& p : pols->items()) {
        if (!p.has("PolicyName") || !p.has("PolicyDocument")) throw std::runtime_error("policy needs a name and document");
        for (auto& s : statements(p["PolicyDocument"])) role.policy.push_back(std::move(s));
      }
    out.roles_[r["Arn"].str()] = std::move(role);
  }
  return out;
}

bool IamPolicy::can_assume_role(const std::string& role_arn, const Context& ctx) const {
  auto it = roles_.find(role_arn);
  return it != roles_.end() && evaluate_statements(it->second.trust, "sts:AssumeRoleWithWebIdentity", "*", ctx);
}

bool IamPolicy::evaluate(const std::string& action, const std::string& resource, const std::string& role_arn,
                         const Context& ctx) const {
  auto it = roles_.find(role_arn);
  return it != roles_.end() && evaluate_statements(it->second.policy, action, resource, ctx);
}

BucketPolicy BucketPolicy::parse(const std::string& text) {
  Json d = Json::parse(text);
  if (!d.is_object() || !d.has("Version") || !d.has("Statement")) throw std::runtime_error("bucket policy needs Version and Statement");
  if (!d["Statement"].is_array()) throw std::runtime_error("Statement must be a list");
  BucketPolicy out;
  for (auto& s : d["Statement"].items()) {
    if (!s.is_object() || !s.has("Effect") || !s.has("Principal") || !s.has("Action"))
      throw std::runtime_error("statement needs Effect, Principal and Action");
    Stmt st;
    st.effect = s["Effect"].str();
    const Json& p = s["Principal"];
    if (p.is_string() && p.as_string() == "*") {
      st.principals = std::nullopt;
    } else if (p.is_string()) {
      st.principals = std::vector<std::string>{p.as_string()};
    } else if (p.is_object() && p.has("AWS")) {
      st.principals = as_list(p["AWS"]);
    } else {
      throw std::runtime_error("invalid Principal value");
    }
    st.actions = as_list(s["Action"]);
    st.resources = opt_list(s.find("Resource"));
    out.stmts_.push_back(std::move(st));
  }
  return out;
}

PolicyResult BucketPolicy::evaluate(const std::string* arn, const std::string& action, const std::string& resource) const {
  bool allow = false;
  for (auto& s : stmts_) {
    bool who = !s.principals;
    if (s.principals)
      for (auto& p : *s.principals)
        if (p == "*" || (arn && matches_wildcard(p, *arn))) {
          who = true;
          break;
        }
    if (!who || !any_match(s.actions, action)) continue;
    if (s.resources && !any_match(*s.resources, resource)) continue;
    if (s.effect == "Deny") return PolicyResult::ExplicitDeny;
    if (s.effect == "Allow") allow = true;
  }
  return allow ? PolicyResult::Allow : PolicyResult::NotApplicable;
}

std::pair<std::string, std::string> resolve_action_and_resource(const std::string& method_in, const std::string& path,
                                                                const std::vector<std::string>& qk) {
  std::vector<std::string> parts;
  std::string cur;
  for (char c : path) {
    if (c == '/') {
      if (!cur.empty()) parts.push_back(cur);
      cur.clear();
    } else {
      cur.push_back(c);
    }
  }
  if (!cur.empty()) parts.push_back(cur);
  std::string method = method_in;
  for (auto& c : method) c = static_cast<char>(std::toupper(static_cast<unsigned char>(c)));
  if (parts.empty())
    return method == "GET" ? std::make_pair(std::string("s3:ListAllMyBuckets"), std::string("arn:dfs:s3:::*"))
                           : std::make_pair(std::string("s3:Unknown"), std::string("arn:dfs:s3:::*"));
  const bool bucket = parts.size() == 1;
  std::string resource = "arn:dfs:s3:::";
  for (size_t i = 0; i < parts.size(); ++i) resource += (i ? "/" : "") + parts[i];
  auto has = [&](const char* k) { return std::find(qk.begin(), qk.end(), k) != qk.end(); };
  if (method == "POST") {
    if (has("uploads") || has("uploadId")) return {"s3:PutObject", resource};
    if (has("delete")) return {"s3:DeleteObject", resource};
    return {"s3:Unknown", resource};
  }
  using Sub = std::vector<std::pair<const char*, const char*>>;
  static const std::map<std::pair<std::string, bool>, Sub> kSub = {
      {{"GET", true},
       {{"acl", "s3:GetBucketAcl"}, {"tagging", "s3:GetBucketTagging"}, {"policy", "s3:GetBucketPolicy"},
        {"location", "s3:GetBucketLocation"}}},
      {{"GET", false}, {{"acl", "s3:GetObjectAcl"}, {"tagging", "s3:GetObjectTagging"}}},
      {{"PUT", true}, {{"acl", "s3:PutBucketAcl"}, {"tagging", "s3:PutBucketTagging"}, {"policy", "s3:PutBucketPolicy"}}},
      {{"PUT", false}, {{"acl", "s3:PutObjectAcl"}, {"tagging", "s3:PutObjectTagging"}}},
      {{"DELETE", true}, {{"tagging", "s3:DeleteBucketTagging"}, {"policy", "s3:DeleteBucketPolicy"}}},
      {{"DELETE", false}, {{"tagging", "s3:DeleteObjectTagging"}}},
  };
  static const std::map<std::pair<std::string, bool>, const char*> kDefault = {
      {{"GET", true}, "s3:ListBucket"},     {{"GET", false}, "s3:GetObject"},     {{"PUT", true}, "s3:CreateBucket"},
      {{"PUT", false}, "s3:PutObject"},     {{"DELETE", true}, "s3:DeleteBucket"}, {{"DELETE", false}, "s3:DeleteObject"},
      {{"HEAD", true}, "s3:HeadBucket"},    {{"HEAD", false}, "s3:HeadObject"}};
  auto sub = kSub.find({method, bucket});
  if (sub != kSub.end())
    for (auto& [q, act] : sub->second)
      if (has(q)) return {act, resource};
  auto d = kDefault.find({method, bucket});
  if (d == kDefault.end()) return {"s3:Unknown", "arn:dfs:s3:::*"};
  return {d->second, resource};
}

}  // namespace s3policy
}  // namespace dfs
