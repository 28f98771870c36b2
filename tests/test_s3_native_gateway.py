"""The S3 gateway as one native executable (csrc/tools/dfs_s3_gateway.cpp): the S3 front end
with no Python behind it, the role the reference's s3-server binary plays
(dfs/s3_server/src/main.rs). Most scenarios are the ones tests/test_s3_gateway.py runs
against the in-process gateways, re-collected here against the executable; the rest cover
what only the executable does on its own (audit chain, STS metrics, SSE, remote store, the
configurations it refuses).
"""
import json
import os
import signal
import subprocess
import time

import pytest
import requests

from rust_hadoop_generated_by_llm_amd.cluster.launcher import ROOT, LocalCluster
from tests.models.s3_audit import SegmentStore, verify_chain

from .test_s3_gateway import (  # noqa: F401  (scenarios and fixtures re-collected here)
    AUDIT_SECRET, IAM_CONFIG, assume, creds_of, jwt, md5q, oidc_issuer, signed,
    test_auth_presigned_urls, test_auth_signed_aws_chunked, test_auth_static_credentials,
    test_bucket_lifecycle, test_bucket_policy_crud, test_copy_and_multi_delete, test_gateway_subprocess,
    test_list_objects_v2_pagination_and_v1, test_native_front_terminates_tls, test_object_put_get_head_metadata,
    test_oidc_sts_policy_flow, test_range_requests, test_sidecar_keys_cannot_be_written_or_deleted)

pytestmark = pytest.mark.slow

EXE = ROOT / "build" / "native" / "dfs_s3_gateway"


class Exe:
    """A dfs_s3_gateway process of the cluster; ``front`` / ``gw`` are None (no in-process
    objects), so the shared scenarios skip their in-process stat checks."""

    front = None
    gw = None

    def __init__(self, cluster, env, name):
        self.cluster, self.name = cluster, name
        self.url = cluster.start_s3(env, name=name)
        self.proc = next(p for p in cluster.procs if p.name == name)
        self.audit_dir = env.get("AUDIT_LOG_DIR", str(cluster.base / f"{name}_audit"))

    def metrics(self) -> str:
        return requests.get(self.url + "/metrics").text

    def stop(self):
        self.cluster.kill(self.name, signal.SIGTERM)


@pytest.fixture(scope="module")
def front():
    return "exe"


@pytest.fixture(scope="module")
def cluster():
    if not EXE.exists():
        pytest.fail(f"{EXE} is not built (python build_native.py)")
    with LocalCluster(n_chunkservers=3, fsync=False) as c:
        yield c


@pytest.fixture(scope="module")
def gw(cluster):
    g = Exe(cluster, {"AUDIT_LOG_ENABLED": "false", "LOCAL_CHUNKSERVER": cluster.cs_addrs[0]}, "s3x")
    yield g
    g.stop()


@pytest.fixture(scope="module")
def authgw(cluster, oidc_issuer, tmp_path_factory):
    d = tmp_path_factory.mktemp("exeauth")
    iam = d / "iam.json"
    iam.write_text(json.dumps(IAM_CONFIG))
    env = {"S3_AUTH_ENABLED": "true", "S3_ACCESS_KEY": "admin", "S3_SECRET_KEY": "admin-secret",
           "OIDC_ISSUER_URL": oidc_issuer["url"], "OIDC_CLIENT_ID": "dfs-client",
           "STS_SIGNING_KEY": "sts-signing-key-0123456789abcdef", "IAM_CONFIG_PATH": str(iam),
           "AUDIT_LOG_DIR": str(d / "audit"), "AUDIT_HMAC_SECRET": AUDIT_SECRET, "AUDIT_LOG_BATCH_SIZE": "1",
           "LOCAL_CHUNKSERVER": cluster.cs_addrs[0]}
    g = Exe(cluster, env, "s3xa")
    yield g
    g.stop()


def _audit_records(g, pred, timeout=15.0):
    deadline = time.time() + timeout
    while True:
        recs = [r for _, r in SegmentStore(g.audit_dir).scan()] if os.path.isdir(g.audit_dir) else []
        if pred(recs) or time.time() > deadline:
            return recs
        time.sleep(0.1)


def _quiesced_count(g, quiet_s=1.0, timeout=20.0):
    """Record count once the audit log has taken no new record for `quiet_s`."""
    deadline = time.time() + timeout
    last, since = -1, time.time()
    while time.time() < deadline:
        n = len(list(SegmentStore(g.audit_dir).scan()))
        if n != last:
            last, since = n, time.time()
        elif time.time() - since >= quiet_s:
            break
        time.sleep(0.1)
    return last


def test_process_is_native(gw):
    """The launcher starts the executable for s3.server: no interpreter in the process."""
    import psutil

    assert gw.proc.info.get("native_gateway") is True and gw.proc.info.get("store") == "shm"
    p = psutil.Process(gw.proc.popen.pid)
    assert os.path.basename(p.exe()) == "dfs_s3_gateway" and not p.children()
    assert requests.get(gw.url + "/health").text == "OK"


def test_errors_answered_natively(gw):
    """What the Python gateway used to answer behind the front: S3 error XML from C++."""
    u = gw.url
    r = requests.get(f"{u}/no-such-bucket-x?list-type=2")
    assert r.status_code == 404 and b"<Code>NoSuchBucket</Code>" in r.content
    r = requests.get(f"{u}/no-such-bucket-x/k")  # as the gateway: an object read only asks for the key
    assert r.status_code == 404 and b"<Code>NoSuchKey</Code>" in r.content
    requests.put(f"{u}/errb")
    r = requests.get(f"{u}/errb/missing")
    assert r.status_code == 404 and b"<Code>NoSuchKey</Code>" in r.content
    assert requests.head(f"{u}/errb/missing").status_code == 404
    r = requests.post(f"{u}/errb/k?uploadId=does-not-exist",
                      data="<CompleteMultipartUpload></CompleteMultipartUpload>")
    assert r.status_code in (400, 404) and (b"NoSuchUpload" in r.content or b"MalformedXML" in r.content)
    r = requests.post(f"{u}/errb?delete", data=b"<Delete><Object>")
    assert r.status_code == 400 and b"MalformedXML" in r.content
    requests.put(f"{u}/errb/small", data=b"0123")
    r = requests.get(f"{u}/errb/small", headers={"Range": "bytes=10-20"})
    assert r.status_code == 416 and b"InvalidRange" in r.content
    m = gw.metrics()
    assert 's3_native_requests_total{method="GET",status="404"}' in m


def test_multipart_roundtrip(gw):
    import xml.etree.ElementTree as ET

    u = gw.url
    requests.put(f"{u}/xmpu")
    r = requests.post(f"{u}/xmpu/big?uploads")
    assert r.status_code == 200, r.text
    uid = next(e.text for e in ET.fromstring(r.content).iter() if e.tag.endswith("UploadId"))
    parts = [os.urandom(5 << 20), os.urandom(777)]
    tags = []
    for i, d in enumerate(parts, 1):
        r = requests.put(f"{u}/xmpu/big?partNumber={i}&uploadId={uid}", data=d)
        assert r.status_code == 200 and r.headers["ETag"] == md5q(d)
        tags.append(r.headers["ETag"])
    body = "<CompleteMultipartUpload>" + "".join(
        f"<Part><PartNumber>{i}</PartNumber><ETag>{t}</ETag></Part>" for i, t in enumerate(tags, 1)) + \
        "</CompleteMultipartUpload>"
    assert requests.post(f"{u}/xmpu/big?uploadId={uid}", data=body).status_code == 200
    blob = b"".join(parts)
    assert requests.get(f"{u}/xmpu/big").content == blob
    r = requests.get(f"{u}/xmpu/big", headers={"Range": f"bytes={(5 << 20) - 5}-{(5 << 20) + 4}"})
    assert r.status_code == 206 and r.content == blob[(5 << 20) - 5:(5 << 20) + 5]
    # an aborted upload leaves nothing behind
    r = requests.post(f"{u}/xmpu/gone?uploads")
    uid2 = next(e.text for e in ET.fromstring(r.content).iter() if e.tag.endswith("UploadId"))
    requests.put(f"{u}/xmpu/gone?partNumber=1&uploadId={uid2}", data=b"p")
    assert requests.delete(f"{u}/xmpu/gone?uploadId={uid2}").status_code == 204
    assert requests.get(f"{u}/xmpu/gone").status_code == 404
    r = requests.put(f"{u}/xmpu/gone?partNumber=2&uploadId={uid2}", data=b"p")
    assert r.status_code == 404 and b"NoSuchUpload" in r.content


def test_list_buckets_and_bucket_ops(gw):
    u = gw.url
    for b in ("lb-one", "lb-two"):
        assert requests.put(f"{u}/{b}").status_code == 200
    r = requests.get(u + "/")
    assert r.status_code == 200 and b"<Name>lb-one</Name>" in r.content and b"<Name>lb-two</Name>" in r.content
    assert requests.head(f"{u}/lb-one").status_code == 200
    assert requests.head(f"{u}/lb-none").status_code == 404
    r = requests.get(f"{u}/lb-one?location")
    assert r.status_code == 200 and b"LocationConstraint" in r.content
    requests.put(f"{u}/lb-two/k", data=b"v")
    r = requests.delete(f"{u}/lb-two")
    assert r.status_code == 409 and b"BucketNotEmpty" in r.content
    assert requests.delete(f"{u}/lb-one").status_code == 204
    assert b"<Name>lb-one</Name>" not in requests.get(u + "/").content


def test_bucket_policy_enforced_without_cache_drop(authgw):
    """PUT/DELETE ?policy bump the shared policy epoch, so the next request sees the change
    (the in-process gateway test had to clear Python's cache by hand)."""
    g = authgw
    signed("PUT", g, "/xguard")
    signed("PUT", g, "/xguard/keep", b"k")
    pol = {"Version": "2012-10-17", "Statement": [{"Effect": "Deny", "Principal": "*", "Action": "s3:DeleteObject",
                                                   "Resource": "arn:dfs:s3:::xguard/*"}]}
    assert signed("PUT", g, "/xguard", json.dumps(pol).encode(), query=[("policy", "")]).status_code == 204
    got = signed("GET", g, "/xguard", query=[("policy", "")])
    assert got.status_code == 200 and json.loads(got.content) == pol
    r = signed("DELETE", g, "/xguard/keep")
    assert r.status_code == 403 and b"AccessDenied" in r.content
    assert signed("DELETE", g, "/xguard", query=[("policy", "")]).status_code == 204
    assert signed("GET", g, "/xguard", query=[("policy", "")]).status_code == 404
    assert signed("DELETE", g, "/xguard/keep").status_code == 204
    assert 'iam_policy_evaluations_total{result="deny",action="s3:DeleteObject"}' in g.metrics()


def test_auth_errors_and_sts_metrics(authgw):
    g = authgw
    r = requests.get(g.url + "/")
    assert r.status_code == 403 and b"AccessDenied" in r.content
    assert assume(g, "not.a.jwt").status_code in (400, 403)
    assert requests.get(g.url + "/", params={"Action": "AssumeRole"}).status_code == 403  # a ListBuckets
    assert requests.post(g.url + "/", data={"Action": "AssumeRole"}).status_code == 400  # InvalidAction
    r = assume(g, jwt())
    assert r.status_code == 200
    ak, sk, tok = creds_of(r)
    assert ak.startswith("ASIA") and signed("GET", g, "/", ak=ak, sk=sk, token=tok).status_code in (200, 403)
    m = g.metrics()
    assert 'iam_sts_requests_total{result="success",error_type="none"}' in m
    assert 'iam_oidc_validations_total{result="success"}' in m
    assert 'iam_oidc_jwks_fetches_total{result="success"} 1' in m or 'iam_oidc_jwks_fetches_total{result="success"}' in m
    assert "iam_auth_requests_total{" in m


def test_audit_chain_written_natively(authgw):
    g = authgw
    assert signed("PUT", g, "/xaud").status_code == 200
    assert signed("PUT", g, "/xaud/o", b"audited").status_code == 200
    assert signed("GET", g, "/xaud/o").content == b"audited"
    assert requests.get(g.url + "/xaud/o").status_code == 403
    assert assume(g, jwt()).status_code == 200

    def done(recs):
        return (any(r["resource"] == "arn:dfs:s3:::xaud/o" and r["action"] == "s3:GetObject" and
                    r["status_code"] == 200 and r["user_id"] == "admin" for r in recs) and
                any(r["resource"] == "arn:dfs:sts:::*" for r in recs) and
                any(r["status_code"] == 403 and r["error_code"] == "AccessDenied" for r in recs))

    recs = _audit_records(g, done)
    assert done(recs), recs[-5:]
    assert any(r["resource"] == "arn:dfs:sts:::*" and r["role_arn"] == "arn:dfs:iam:::role/tenant-a-role"
               for r in recs)
    # the logger writes asynchronously: compare the chain with a quiesced log (no new record
    # for a second; every request above has returned), scanned again after the verification
    quiet = _quiesced_count(g)
    n, errs = verify_chain(SegmentStore(g.audit_dir), AUDIT_SECRET)
    after = [r for _, r in SegmentStore(g.audit_dir).scan()]
    assert errs == [] and n == len(after) == quiet >= len(recs)


def test_sse_at_rest(cluster):
    g = Exe(cluster, {"SSE_MASTER_KEY": "ab" * 32, "AUDIT_LOG_ENABLED": "false",
                      "LOCAL_CHUNKSERVER": cluster.cs_addrs[0]}, "s3xsse")
    try:
        u = g.url
        requests.put(f"{u}/xsse")
        data = os.urandom(300_001)
        r = requests.put(f"{u}/xsse/obj", data=data)
        assert r.status_code == 200 and r.headers.get("x-amz-server-side-encryption") == "AES256"
        got = requests.get(f"{u}/xsse/obj")
        assert got.content == data and got.headers.get("x-amz-server-side-encryption") == "AES256"
        r = requests.get(f"{u}/xsse/obj", headers={"Range": "bytes=1000-1999"})
        assert r.status_code == 206 and r.content == data[1000:2000]
        assert requests.put(f"{u}/xsse/copy", headers={"x-amz-copy-source": "/xsse/obj"}).status_code == 200
        assert requests.get(f"{u}/xsse/copy").content == data
        c = cluster.client()
        raw = c.get_file_content("/xsse/obj")
        assert raw != data and data[:64] not in raw
        assert c.get_file_content("/xsse/copy") != raw  # a fresh data key per object
    finally:
        g.stop()


def test_remote_store_gateway(cluster):
    """No chunkserver on the gateway's host: the executable's front speaks gRPC to the
    chunkservers (RemoteFrontStore)."""
    g = Exe(cluster, {"AUDIT_LOG_ENABLED": "false"}, "s3xr")
    try:
        assert g.proc.info.get("store") == "grpc"
        u = g.url
        assert requests.put(f"{u}/xrem").status_code == 200
        data = os.urandom((3 << 20) + 5)
        assert requests.put(f"{u}/xrem/o", data=data).status_code == 200
        assert requests.get(f"{u}/xrem/o").content == data
        assert b"<Key>o</Key>" in requests.get(f"{u}/xrem?list-type=2").content
        assert requests.delete(f"{u}/xrem/o").status_code == 204
    finally:
        g.stop()


def test_reference_sidecar_layout_served_natively(cluster):
    """The reference gateway's object layout (handlers.rs:984-1006,1058-1079): headers in a
    sidecar DFS file `<key>.meta` = {"headers": {...}}. The executable reads it for objects
    without attributes (GET, HEAD, listings, CopyObject, multipart objects the reference
    completed: numbered parts, no recorded layout) and, with S3_METADATA_SIDECAR=true, writes
    it for PUT, CopyObject and CompleteMultipartUpload — with no hand-off to any backend."""
    import json
    import xml.etree.ElementTree as ET

    c = cluster.client()
    g = Exe(cluster, {"AUDIT_LOG_ENABLED": "false", "S3_METADATA_SIDECAR": "true",
                      "LOCAL_CHUNKSERVER": cluster.cs_addrs[0]}, "s3xside")
    try:
        u = g.url
        assert requests.put(f"{u}/refside").status_code == 200
        # objects the reference wrote: plain file + sidecar
        c.create_file_from_buffer(b"legacy bytes", "/refside/legacy")
        c.create_file_from_buffer(json.dumps({"headers": {"ETag": '"abc"', "x-amz-meta-old": "1",
                                                          "Content-Type": "text/old"}}).encode(), "/refside/legacy.meta")
        r = requests.get(f"{u}/refside/legacy")
        assert r.content == b"legacy bytes" and r.headers["ETag"] == '"abc"'
        assert r.headers["x-amz-meta-old"] == "1" and r.headers["Content-Type"] == "text/old"
        assert requests.head(f"{u}/refside/legacy").headers["x-amz-meta-old"] == "1"
        # a multipart object completed by the reference: numbered parts, a bare marker, a sidecar
        p1, p2 = os.urandom(70_000), os.urandom(1234)
        c.create_file_from_buffer(p1, "/refside/big/1")
        c.create_file_from_buffer(p2, "/refside/big/2")
        c.create_file_from_buffer(b"", "/refside/big/.s3_mpu_completed")
        c.create_file_from_buffer(json.dumps({"headers": {"ETag": '"mpu-2"'}}).encode(), "/refside/big.meta")
        r = requests.get(f"{u}/refside/big")
        assert r.content == p1 + p2 and r.headers["ETag"] == '"mpu-2"'
        r = requests.get(f"{u}/refside/big", headers={"Range": "bytes=69990-70009"})
        assert r.status_code == 206 and r.content == (p1 + p2)[69990:70010]
        lst = ET.fromstring(requests.get(f"{u}/refside?list-type=2").content)
        ns = lst.tag.split("}")[0] + "}" if lst.tag.startswith("{") else ""
        got = {e.find(ns + "Key").text: (e.find(ns + "ETag").text, int(e.find(ns + "Size").text))
               for e in lst.findall(ns + "Contents")}
        assert got["legacy"] == ('"abc"', 12) and got["big"] == ('"mpu-2"', len(p1) + len(p2))
        # writes with S3_METADATA_SIDECAR=true also leave the reference's sidecar
        body = os.urandom(5000)
        r = requests.put(f"{u}/refside/new", data=body, headers={"x-amz-meta-a": "b", "Content-Type": "text/n"})
        assert r.status_code == 200
        side = json.loads(c.get_file_content("/refside/new.meta"))
        assert side == {"headers": {"ETag": r.headers["ETag"], "x-amz-meta-a": "b", "Content-Type": "text/n"}}
        assert c.get_file_info("/refside/new").attributes["ETag"] == r.headers["ETag"]
        # CopyObject of a sidecar-described source keeps its headers (COPY directive)
        r = requests.put(f"{u}/refside/copy", headers={"x-amz-copy-source": "/refside/legacy"})
        assert r.status_code == 200
        r = requests.get(f"{u}/refside/copy")
        assert r.content == b"legacy bytes" and r.headers["x-amz-meta-old"] == "1"
        assert json.loads(c.get_file_content("/refside/copy.meta"))["headers"]["x-amz-meta-old"] == "1"
        # multipart completion writes the sidecar of the object too
        up = ET.fromstring(requests.post(f"{u}/refside/mp?uploads").content)
        uid = next(e.text for e in up.iter() if e.tag.endswith("UploadId"))
        e1 = requests.put(f"{u}/refside/mp?partNumber=1&uploadId={uid}", data=b"q" * 6000).headers["ETag"]
        done = ("<CompleteMultipartUpload><Part><PartNumber>1</PartNumber><ETag>" + e1 +
                "</ETag></Part></CompleteMultipartUpload>")
        r = requests.post(f"{u}/refside/mp?uploadId={uid}", data=done)
        assert r.status_code == 200
        assert json.loads(c.get_file_content("/refside/mp.meta"))["headers"]["ETag"].endswith('-1"')
        # DELETE removes the sidecar with the object
        assert requests.delete(f"{u}/refside/new").status_code == 204
        assert not c.exists("/refside/new.meta")
        handoffs = [ln for ln in g.metrics().splitlines()
                    if ln.startswith("s3_native_handoffs_total") and not ln.rstrip().endswith(" 0")]
        assert handoffs == [], handoffs
    finally:
        g.stop()
        c.close()


def test_follows_master_leader_changes():
    """A Raft group of three masters: the executable's shared-memory client reaches only its
    shard's first peer, so calls it declines (that peer not leading, or dead) go over gRPC
    with leader following, the body still in the shared slot; the gateway keeps serving
    across a leader kill (reference: the client follows Not Leader hints, mod.rs)."""
    from rust_hadoop_generated_by_llm_amd.models import proto as pb
    from rust_hadoop_generated_by_llm_amd.utils.rpc import ChannelPool

    with LocalCluster(n_chunkservers=3, masters_per_shard=3, fsync=False) as cl:
        g = Exe(cl, {"AUDIT_LOG_ENABLED": "false", "LOCAL_CHUNKSERVER": cl.cs_addrs[0]}, "s3ha")
        u = g.url
        assert requests.put(f"{u}/ha").status_code == 200
        before = os.urandom(200_000)
        assert requests.put(f"{u}/ha/before", data=before).status_code == 200
        pool = ChannelPool()
        leader = None
        for m in cl.master_addrs:
            if pool.call(m, "MasterService", "GetClusterInfo", pb.GetClusterInfoRequest()).role == "Leader":
                leader = m
        assert leader is not None
        cl.kill(f"master_shard-0_{cl.master_addrs.index(leader) + 1}")
        after = os.urandom(300_000)
        deadline = time.time() + 30
        while requests.put(f"{u}/ha/after", data=after).status_code != 200:
            assert time.time() < deadline, "no write accepted after the leader was killed"
            time.sleep(0.3)
        assert requests.get(f"{u}/ha/before").content == before
        assert requests.get(f"{u}/ha/after").content == after
        keys = requests.get(f"{u}/ha?list-type=2").content
        assert b"<Key>before</Key>" in keys and b"<Key>after</Key>" in keys
        assert requests.delete(f"{u}/ha/before").status_code == 204
        m = g.metrics()
        fb = int(float(next(ln for ln in m.splitlines() if ln.startswith("s3_native_store_fallbacks_total")).split()[-1]))
        assert fb > 0
        pool.close()
