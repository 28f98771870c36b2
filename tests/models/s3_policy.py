"""IAM role policies and S3 bucket policies.

* ``matches_wildcard``: ``*`` / ``?`` glob over the whole string (auth/policy.rs:64-78).
* IAM (auth/policy.rs:80-200): ``IamConfig{Roles:[{RoleName, Arn, AssumeRolePolicyDocument,
  Policies:[{PolicyName, PolicyDocument}]}]}``. A statement matches when its Action
  (and Resource, if present) match and every Condition holds; any matching Deny wins,
  otherwise any matching Allow allows; default deny. Conditions: ``StringEquals`` (the
  first actual value must be expected) and ``ForAnyValue:StringEquals`` over
  ``OIDC_ISSUER:groups`` / ``OIDC_ISSUER:<claim>``; unknown operators fail closed.
* Bucket policies (auth/bucket_policy.rs): Principal ``"*"``, ``"<arn glob>"`` or
  ``{"AWS": str|[str]}``; result Allow / ExplicitDeny / NotApplicable.
* ``resolve_action_and_resource``: method/path/query → (``s3:<Action>``,
  ``arn:dfs:s3:::<bucket>[/<key>]``) (s3_server/src/auth_middleware.rs:400-493).
"""
from __future__ import annotations

import json
import re
from dataclasses import dataclass, field
from enum import Enum
from functools import lru_cache


@lru_cache(maxsize=4096)
def _glob_re(pattern: str) -> re.Pattern:
    return re.compile("^" + "".join(".*" if c == "*" else "." if c == "?" else re.escape(c) for c in pattern) + "$",
                      re.S)


def matches_wildcard(pattern: str, target: str) -> bool:
    if pattern == "*":
        return True
    return _glob_re(pattern).match(target) is not None


def _as_list(v) -> list[str]:
    if v is None:
        return []
    return [v] if isinstance(v, str) else [str(x) for x in v]


@dataclass
class EvaluationContext:
    principal_id: str = ""
    groups: list[str] = field(default_factory=list)
    claims: dict[str, str] = field(default_factory=dict)

    def to_json(self) -> dict:
        return {"principal_id": self.principal_id, "groups": list(self.groups), "claims": dict(self.claims)}


@dataclass
class Statement:
    effect: str
    actions: list[str]
    resources: list[str] | None
    condition: dict[str, dict[str, list[str]]] | None = None

    @classmethod
    def from_json(cls, d: dict) -> "Statement":
        if "Effect" not in d or "Action" not in d:
            raise ValueError("statement needs Effect and Action")
        cond = d.get("Condition")
        if cond is not None:
            cond = {op: {k: _as_list(v) for k, v in keys.items()} for op, keys in cond.items()}
        res = d.get("Resource")
        return cls(d["Effect"], _as_list(d["Action"]), None if res is None else _as_list(res), cond)

    def action_matches(self, action: str) -> bool:
        return any(matches_wildcard(p, action) for p in self.actions)

    def resource_matches(self, resource: str) -> bool:
        return self.resources is None or any(matches_wildcard(p, resource) for p in self.resources)


def _condition_holds(cond: dict[str, dict[str, list[str]]], ctx: EvaluationContext) -> bool:
    for op, keys in cond.items():
        for key, expected in keys.items():
            if key == "OIDC_ISSUER:groups":
                actual = list(ctx.groups)
            elif key.startswith("OIDC_ISSUER:"):
                v = ctx.claims.get(key[len("OIDC_ISSUER:"):])
                actual = [v] if v is not None else []
            else:
                actual = []
            if op == "StringEquals":
                if not actual or actual[0] not in expected:
                    return False
            elif op == "ForAnyValue:StringEquals":
                if not any(a in expected for a in actual):
                    return False
            else:
                return False
    return True


def evaluate_statements(stmts, action: str, resource: str, ctx: EvaluationContext) -> bool:
    allow = False
    for s in stmts:
        if not s.action_matches(action) or not s.resource_matches(resource):
            continue
        if s.condition is not None and not _condition_holds(s.condition, ctx):
            continue
        if s.effect == "Deny":
            return False
        if s.effect == "Allow":
            allow = True
    return allow


@dataclass
class Role:
    name: str
    arn: str
    trust: list[Statement]
    policies: list[tuple[str, list[Statement]]]


class PolicyEvaluator:
    def __init__(self, roles: list[Role]):
        self.roles = {r.arn: r for r in roles}

    @classmethod
    def from_json(cls, doc: dict | str) -> "PolicyEvaluator":
        if isinstance(doc, str):
            doc = json.loads(doc)
        roles = []
        for r in doc["Roles"]:
            trust = [Statement.from_json(s) for s in r["AssumeRolePolicyDocument"]["Statement"]]
            pols = [(p["PolicyName"], [Statement.from_json(s) for s in p["PolicyDocument"]["Statement"]])
                    for p in r.get("Policies", [])]
            roles.append(Role(r["RoleName"], r["Arn"], trust, pols))
        return cls(roles)

    @classmethod
    def from_file(cls, path: str) -> "PolicyEvaluator":
        with open(path) as f:
            return cls.from_json(f.read())

    def can_assume_role(self, role_arn: str, ctx: EvaluationContext) -> bool:
        r = self.roles.get(role_arn)
        return r is not None and evaluate_statements(r.trust, "sts:AssumeRoleWithWebIdentity", "*", ctx)

    def evaluate(self, action: str, resource: str, role_arn: str, ctx: EvaluationContext) -> bool:
        r = self.roles.get(role_arn)
        if r is None:
            return False
        return evaluate_statements([s for _, ss in r.policies for s in ss], action, resource, ctx)


# ---------------------------------------------------------------------------- bucket policy
class PolicyResult(Enum):
    ALLOW = "Allow"
    EXPLICIT_DENY = "ExplicitDeny"
    NOT_APPLICABLE = "NotApplicable"


def _principal_patterns(p) -> list[str] | None:
    """None means wildcard principal."""
    if p == "*":
        return None
    if isinstance(p, str):
        return [p]
    if isinstance(p, dict) and "AWS" in p:
        return _as_list(p["AWS"])
    raise ValueError("invalid Principal value")


@dataclass
class BucketStatement:
    effect: str
    principals: list[str] | None
    actions: list[str]
    resources: list[str] | None

    def principal_matches(self, arn: str | None) -> bool:
        if self.principals is None:
            return True
        for p in self.principals:
            if p == "*":
                return True
            if arn is not None and matches_wildcard(p, arn):
                return True
        return False


class BucketPolicy:
    def __init__(self, version: str, statements: list[BucketStatement]):
        self.version, self.statements = version, statements

    @classmethod
    def parse(cls, data: bytes | str) -> "BucketPolicy":
        d = json.loads(data)
        if not isinstance(d, dict) or "Version" not in d or "Statement" not in d:
            raise ValueError("bucket policy needs Version and Statement")
        stmts = []
        for s in d["Statement"]:
            if "Effect" not in s or "Principal" not in s or "Action" not in s:
                raise ValueError("statement needs Effect, Principal and Action")
            res = s.get("Resource")
            stmts.append(BucketStatement(s["Effect"], _principal_patterns(s["Principal"]), _as_list(s["Action"]),
                                         None if res is None else _as_list(res)))
        return cls(str(d["Version"]), stmts)

    def evaluate(self, principal_arn: str | None, action: str, resource: str) -> PolicyResult:
        allow = False
        for s in self.statements:
            if not s.principal_matches(principal_arn):
                continue
            if not any(matches_wildcard(a, action) for a in s.actions):
                continue
            if s.resources is not None and not any(matches_wildcard(r, resource) for r in s.resources):
                continue
            if s.effect == "Deny":
                return PolicyResult.EXPLICIT_DENY
            if s.effect == "Allow":
                allow = True
        return PolicyResult.ALLOW if allow else PolicyResult.NOT_APPLICABLE


# ---------------------------------------------------------------------------- action mapping
_SUB = {
    ("GET", "bucket"): (("acl", "s3:GetBucketAcl"), ("tagging", "s3:GetBucketTagging"),
                        ("policy", "s3:GetBucketPolicy"), ("location", "s3:GetBucketLocation")),
    ("GET", "object"): (("acl", "s3:GetObjectAcl"), ("tagging", "s3:GetObjectTagging")),
    ("PUT", "bucket"): (("acl", "s3:PutBucketAcl"), ("tagging", "s3:PutBucketTagging"),
                        ("policy", "s3:PutBucketPolicy")),
    ("PUT", "object"): (("acl", "s3:PutObjectAcl"), ("tagging", "s3:PutObjectTagging")),
    ("DELETE", "bucket"): (("tagging", "s3:DeleteBucketTagging"), ("policy", "s3:DeleteBucketPolicy")),
    ("DELETE", "object"): (("tagging", "s3:DeleteObjectTagging"),),
}
_DEFAULT = {("GET", "bucket"): "s3:ListBucket", ("GET", "object"): "s3:GetObject",
            ("PUT", "bucket"): "s3:CreateBucket", ("PUT", "object"): "s3:PutObject",
            ("DELETE", "bucket"): "s3:DeleteBucket", ("DELETE", "object"): "s3:DeleteObject",
            ("HEAD", "bucket"): "s3:HeadBucket", ("HEAD", "object"): "s3:HeadObject"}


def resolve_action_and_resource(method: str, path: str, query: dict[str, str]) -> tuple[str, str]:
    parts = [p for p in path.split("/") if p]
    method = method.upper()
    if not parts:
        return ("s3:ListAllMyBuckets", "arn:dfs:s3:::*") if method == "GET" else ("s3:Unknown", "arn:dfs:s3:::*")
    kind = "bucket" if len(parts) == 1 else "object"
    resource = "arn:dfs:s3:::" + "/".join(parts)
    if method == "POST":
        # Only multipart calls are mapped by the reference (auth_middleware.rs:478-486),
        # on any path with a bucket; bucket-level multi-delete maps to DeleteObject.
        if "uploads" in query or "uploadId" in query:
            return "s3:PutObject", resource
        if "delete" in query:
            return "s3:DeleteObject", resource
        return "s3:Unknown", resource
    for q, act in _SUB.get((method, kind), ()):
        if q in query:
            return act, resource
    act = _DEFAULT.get((method, kind))
    if act is None:
        return "s3:Unknown", "arn:dfs:s3:::*"
    return act, resource
