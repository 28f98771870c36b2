"""The native IAM / bucket policy engine (csrc/s3_policy.cpp, used by the native S3 front)
against the Python engine (tests/models/s3_policy.py; reference auth/policy.rs, auth/bucket_policy.rs,
auth_middleware.rs:400-493) on randomized documents, principals, actions and resources."""
import json
import random

import pytest

from rust_hadoop_generated_by_llm_amd import native as N
from tests.models.s3_policy import (BucketPolicy, EvaluationContext, PolicyEvaluator,
                                                             matches_wildcard, resolve_action_and_resource)

lib = N.lib
ALPHA = ["a", "b", "/", ":", "é", "-", "*", "?"]
ACTIONS = ["s3:GetObject", "s3:PutObject", "s3:DeleteObject", "s3:ListBucket", "s3:*", "s3:Get*", "s3:?etObject", "*"]
RESOURCES = ["arn:dfs:s3:::b1/*", "arn:dfs:s3:::b1/a*", "arn:dfs:s3:::b?/x", "arn:dfs:s3:::*", "*", "arn:dfs:s3:::b2"]
PRINCIPALS = ["*", "arn:dfs:iam:::role/r1", "arn:dfs:iam:::role/*", {"AWS": "arn:dfs:iam:::role/r?"},
              {"AWS": ["arn:dfs:iam:::role/x", "*"]}, {"AWS": []}]


def rnd_str(r, n):
    return "".join(r.choice(ALPHA) for _ in range(r.randint(0, n)))


def test_wildcard_matches_python():
    r = random.Random(1)
    for _ in range(20000):
        p, t = rnd_str(r, 6), rnd_str(r, 8).replace("*", "a").replace("?", "b")
        if r.random() < 0.05:
            t += "\n"
        assert lib.s3_wildcard(p, t) == matches_wildcard(p, t), (p, t)


def one_of_or_list(r, xs):
    return r.choice(xs) if r.random() < 0.5 else r.sample(xs, r.randint(1, 3))


def test_bucket_policy_matches_python():
    r = random.Random(2)
    targets = ["arn:dfs:s3:::b1/a1", "arn:dfs:s3:::b1/z", "arn:dfs:s3:::b2", "arn:dfs:s3:::b3/x"]
    for _ in range(400):
        stmts = []
        for _ in range(r.randint(1, 4)):
            st = {"Effect": r.choice(["Allow", "Deny", "Other"]), "Principal": r.choice(PRINCIPALS),
                  "Action": one_of_or_list(r, ACTIONS)}
            if r.random() < 0.7:
                st["Resource"] = one_of_or_list(r, RESOURCES)
            stmts.append(st)
        doc = json.dumps({"Version": "2012-10-17", "Statement": stmts})
        py = BucketPolicy.parse(doc)
        for _ in range(10):
            who = r.choice([None, "arn:dfs:iam:::role/r1", "arn:dfs:iam:::role/x", "arn:dfs:iam:::role/zz"])
            act = r.choice(["s3:GetObject", "s3:PutObject", "s3:DeleteObject", "s3:ListBucket"])
            res = r.choice(targets)
            assert lib.s3_bucket_policy_eval(doc, who, act, res) == py.evaluate(who, act, res).value, (doc, who, act, res)


def test_bucket_policy_rejects_what_python_rejects():
    for bad in ('{"Statement": []}', '{"Version": "1", "Statement": [{"Effect": "Allow", "Action": "s3:*"}]}',
                '{"Version": "1", "Statement": [{"Effect": "Allow", "Principal": 5, "Action": "s3:*"}]}', "not json"):
        with pytest.raises(ValueError):
            BucketPolicy.parse(bad)
        with pytest.raises(ValueError):
            lib.s3_bucket_policy_eval(bad, None, "s3:GetObject", "arn:dfs:s3:::b/k")


def test_iam_policy_matches_python():
    r = random.Random(3)
    conds = [None, {"StringEquals": {"OIDC_ISSUER:groups": ["admins"]}},
             {"ForAnyValue:StringEquals": {"OIDC_ISSUER:groups": ["dev", "ops"]}},
             {"StringEquals": {"OIDC_ISSUER:tenant": "t1"}}, {"StringLike": {"OIDC_ISSUER:tenant": "t*"}}]
    for _ in range(200):
        roles = []
        for i in range(2):
            def stmts(n):
                out = []
                for _ in range(n):
                    st = {"Effect": r.choice(["Allow", "Deny"]), "Action": one_of_or_list(r, ACTIONS + ["sts:*"])}
                    if r.random() < 0.6:
                        st["Resource"] = one_of_or_list(r, RESOURCES)
                    c = r.choice(conds)
                    if c is not None:
                        st["Condition"] = c
                    out.append(st)
                return out
            roles.append({"RoleName": f"r{i}", "Arn": f"arn:dfs:iam:::role/r{i}",
                          "AssumeRolePolicyDocument": {"Statement": stmts(r.randint(1, 2))},
                          "Policies": [{"PolicyName": "p", "PolicyDocument": {"Statement": stmts(r.randint(1, 3))}}]})
        doc = json.dumps({"Roles": roles})
        ev = PolicyEvaluator.from_json(doc)
        for _ in range(8):
            ctx = EvaluationContext(principal_id="u", groups=r.sample(["admins", "dev", "ops", "x"], r.randint(0, 2)),
                                    claims=r.choice([{}, {"tenant": "t1"}, {"tenant": "t2"}]))
            arn = r.choice(["arn:dfs:iam:::role/r0", "arn:dfs:iam:::role/r1", "arn:dfs:iam:::role/none"])
            act = r.choice(["s3:GetObject", "s3:PutObject", "s3:DeleteObject"])
            res = r.choice(["arn:dfs:s3:::b1/a1", "arn:dfs:s3:::b2"])
            got = lib.s3_iam_eval(doc, act, res, arn, ctx.principal_id, ctx.groups, ctx.claims)
            assert tuple(got) == (ev.evaluate(act, res, arn, ctx), ev.can_assume_role(arn, ctx)), (doc, ctx, arn, act, res)


def test_resolve_action_matches_python():
    paths = ["/", "", "/b", "/b/", "/b/k", "/b/k/x/y", "//b//k"]
    qs = [[], ["acl"], ["tagging"], ["policy"], ["location"], ["uploads"], ["uploadId", "partNumber"], ["delete"],
          ["versioning"], ["acl", "tagging"]]
    for m in ("GET", "PUT", "DELETE", "HEAD", "POST", "PATCH", "get"):
        for p in paths:
            for q in qs:
                assert tuple(lib.s3_resolve_action(m, p, q)) == resolve_action_and_resource(m, p, {k: "" for k in q}), \
                    (m, p, q)
