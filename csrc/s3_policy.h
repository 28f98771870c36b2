// IAM role policies and S3 bucket policies (C13-C14), native twin of
// tests/models/s3_policy.py. Reference: dfs/s3_server/src/auth/
// policy.rs:64-200 (wildcards, IamConfig roles, statements with Condition) and
// auth/bucket_policy.rs (Principal "*" | "<arn glob>" | {"AWS": str|[str]}; Allow /
// ExplicitDeny / NotApplicable), and auth_middleware.rs:400-493 (method/path/query ->
// s3:<Action> + arn:dfs:s3:::<bucket>[/<key>]).
//
// Used by the native S3 front (csrc/s3_front.cpp) so that a bucket with a policy keeps its
// object requests on the native path unless the policy denies them; bound to Python for the
// parity tests (tests/test_s3_policy_native.py).
#pragma once
#include <map>
#include <memory>
#include <optional>
#include <string>
#include <vector>

namespace dfs {
namespace s3policy {

// `*` (any run) and `?` (one character, UTF-8 aware) over the whole string; "*" alone
// matches all. Like the Python engine's `re` pattern, `$` also matches before a final newline.
bool matches_wildcard(const std::string& pattern, const std::string& target);

struct Context {  // EvaluationContext: the caller's OIDC claims (STS sessions)
  std::string principal_id;
  std::vector<std::string> groups;
  std::map<std::string, std::string> claims;
};

struct Statement {
  std::string effect;
  std::vector<std::string> actions;
  std::optional<std::vector<std::string>> resources;  // nullopt: any resource
  // operator -> (key -> expected values); nullopt: no Condition
  std::optional<std::map<std::string, std::map<std::string, std::vector<std::string>>>> condition;
};

// Any matching Deny wins, else any matching Allow; default deny.
bool evaluate_statements(const std::vector<Statement>& stmts, const std::string& action, const std::string& resource,
                         const Context& ctx);

class IamPolicy {  // IamConfig{Roles:[...]}
 public:
  // Throws std::runtime_error on a malformed document.
  static IamPolicy parse(const std::string& json);
  bool can_assume_role(const std::string& role_arn, const Context& ctx) const;
  bool evaluate(const std::string& action, const std::string& resource, const std::string& role_arn,
                const Context& ctx) const;

 private:
  struct Role {
    std::string name;
    std::vector<Statement> trust, policy;  // policy: every statement of every attached policy
  };
  std::map<std::string, Role> roles_;  // by ARN
};

enum class PolicyResult { Allow, ExplicitDeny, NotApplicable };

class BucketPolicy {
 public:
  // Throws std::runtime_error on a malformed document (the gateway then ignores the policy).
  static BucketPolicy parse(const std::string& json);
  // `principal_arn` nullptr: a caller without a role (static access key).
  PolicyResult evaluate(const std::string* principal_arn, const std::string& action, const std::string& resource) const;

 private:
  struct Stmt {
    std::string effect;
    std::optional<std::vector<std::string>> principals;  // nullopt: "*"
    std::vector<std::string> actions;
    std::optional<std::vector<std::string>> resources;
  };
  std::vector<Stmt> stmts_;
};

// (s3:<Action>, arn:dfs:s3:::<bucket>[/<key>]) for an HTTP method, decoded path and the
// query's parameter names.
std::pair<std::string, std::string> resolve_action_and_resource(const std::string& method, const std::string& path,
                                                                const std::vector<std::string>& query_keys);

}  // namespace s3policy
}  // namespace dfs
