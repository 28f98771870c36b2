"""TEST MODEL (not part of the product): the Python S3 gateway, kept as an executable model of
the native gateway (csrc/s3_front.cpp, csrc/tools/dfs_s3_gateway.cpp) for the A/B tests.
The product's gateway process is dfs_s3_gateway.

S3-compatible HTTP gateway over the DFS (C52-C57).

Reference: dfs/s3_server/src/{main.rs, handlers.rs, auth_middleware.rs, sts_handler.rs,
state.rs}. Path-style addressing only (``/{bucket}/{key}``) and the same on-DFS layout, so
data written through either implementation is readable by the other:

* bucket = marker file ``/{bucket}/.s3keep``; bucket policy = ``/{bucket}/.s3_bucket_policy``;
* object = DFS file ``/{bucket}/{key}``; its headers (``ETag``, ``Content-Type``,
  ``x-amz-meta-*``, ``x-amz-sse-encrypted-dek``) travel in the same CompleteFile as
  ``FileMetadata.attributes`` (extension field), so a PUT is one DFS file write and a GET
  one GetFileInfo + one read. The reference keeps them in a sidecar file
  ``/{bucket}/{key}.meta`` (``{"headers": {...}}``): sidecars are still READ when an object
  has no attributes (data written by the reference), and ``S3_METADATA_SIDECAR=true`` also
  WRITES them, for a bucket the reference gateway must read back;
* multipart upload = ``/.s3_mpu/{uploadId}/{n}`` (part ETag = the part file's etag_md5);
  completion renames parts to ``/{bucket}/{key}/{n}`` (cross-shard renames go through the
  masters' 2PC) and writes ``/{bucket}/{key}/.s3_mpu_completed`` carrying the object
  attributes, ETag ``md5(concat(part md5s))-N``.

Deliberate fixes over the reference (each noted at its site): Range GETs learn the size
from ``GetFileInfo`` instead of downloading the whole object; suffix ranges
(``bytes=-N``) and unsatisfiable ranges (416) follow RFC 7233; multi-delete is also
accepted at the bucket level (what AWS SDKs send); object deletion only removes
``{key}/`` children, not every key sharing the prefix; v1 listings honour marker /
max-keys; v2 listings hide multipart parts; aws-chunked bodies of signed requests have
their chunk-signature chain verified; bucket-policy documents are cached for a second.

The gateway is an asyncio (aiohttp) server; DFS client calls are blocking gRPC calls and
run on a thread pool so one slow read never stalls other requests.
"""
from __future__ import annotations

import argparse
import asyncio
import hashlib
import json
import logging
import os
import shutil
import signal
import socket
import ssl
import struct
import tempfile
import threading
import time
import uuid
from concurrent.futures import ThreadPoolExecutor
from datetime import datetime, timezone
from email.utils import formatdate
from urllib.parse import parse_qsl, unquote

from aiohttp import web

from rust_hadoop_generated_by_llm_amd.client.client import Client, DfsError
from rust_hadoop_generated_by_llm_amd.parallel.sharding import ShardMap
from rust_hadoop_generated_by_llm_amd.utils.metrics import Registry
from tests.models import s3_xml as X
from tests.models.s3_audit import AuditLogger, make_record
from rust_hadoop_generated_by_llm_amd.s3.auth import sigv4
from rust_hadoop_generated_by_llm_amd.s3.auth.errors import AuthError
from tests.models.s3_identity import (EnvCredentialProvider, OidcValidator, SseManager, StsSessionData, StsTokenManager,
                            parse_sse_master_key, random_alnum)
from tests.models.s3_policy import BucketPolicy, PolicyEvaluator, PolicyResult, resolve_action_and_resource

log = logging.getLogger("dfs.s3")

EMPTY_ETAG = '"d41d8cd98f00b204e9800998ecf8427e"'
DEFAULT_DATE = "2025-01-01T00:00:00.000Z"
MAX_BODY = 1 << 30
HIDDEN_SUFFIXES = (".s3keep", ".s3_mpu_completed", ".meta", ".s3_bucket_policy")


def reserved_key(key: str) -> bool:
    """Keys that would collide with the gateway's sidecar files on the DFS namespace."""
    return key.endswith(HIDDEN_SUFFIXES)
MPU_ROOT = "/.s3_mpu"


def _http_date(ms: int | None) -> str:
    if not ms:
        return "Wed, 01 Jan 2025 00:00:00 GMT"
    return formatdate(ms / 1000.0, usegmt=True)


def _iso_ms(ms: int | None) -> str:
    if not ms:
        return DEFAULT_DATE
    return datetime.fromtimestamp(ms // 1000, tz=timezone.utc).strftime("%Y-%m-%dT%H:%M:%S.000Z")


def parse_range(value: str | None, size: int):
    """Returns None (no/ignored range), (start, end) inclusive, or "unsatisfiable"."""
    if not value or not value.startswith("bytes="):
        return None
    spec = value[6:].strip()
    if "," in spec or "-" not in spec:
        return None
    a, b = spec.split("-", 1)
    try:
        if a == "":
            n = int(b)
            if n <= 0:
                return "unsatisfiable"
            return (max(0, size - n), size - 1) if size > 0 else "unsatisfiable"
        start = int(a)
        end = int(b) if b else size - 1
    except ValueError:
        return None
    if start >= size or start < 0:
        return "unsatisfiable"
    end = min(end, size - 1)
    if end < start:
        return None
    return start, end


class S3Config:
    def __init__(self, env: dict | None = None):
        env = dict(os.environ if env is None else env)
        self.env = env
        self.master_addr = env.get("MASTER_ADDR", "http://127.0.0.1:8081")
        self.config_servers = [s for s in env.get("CONFIG_SERVERS", "").split(",") if s]
        self.ca_cert = env.get("CA_CERT")
        self.domain_name = env.get("DOMAIN_NAME")
        self.shard_config = env.get("SHARD_CONFIG")
        self.auth_enabled = env.get("S3_AUTH_ENABLED", "") == "true"
        self.region = env.get("S3_REGION", "us-east-1")
        self.require_tls = env.get("S3_REQUIRE_TLS", "") == "true"
        self.allow_unsigned_payload = env.get("S3_ALLOW_UNSIGNED_PAYLOAD", "true") == "true"
        self.oidc_issuer = env.get("OIDC_ISSUER_URL")
        self.oidc_client_id = env.get("OIDC_CLIENT_ID")
        self.oidc_allow_hs256 = env.get("OIDC_ALLOW_HS256", "") == "true"
        self.sts_signing_key = env.get("STS_SIGNING_KEY")
        self.iam_config_path = env.get("IAM_CONFIG_PATH")
        self.audit_enabled = env.get("AUDIT_LOG_ENABLED", "true") == "true"
        self.audit_dir = env.get("AUDIT_LOG_DIR", "/tmp/s3_audit_log")
        self.audit_retention_days = int(env.get("AUDIT_LOG_RETENTION_DAYS", "30") or 30)
        self.audit_batch_size = int(env.get("AUDIT_LOG_BATCH_SIZE", "100") or 100)
        self.audit_hmac_secret = env.get("AUDIT_HMAC_SECRET")
        self.sse_master_key = env.get("SSE_MASTER_KEY")
        self.port = int(env.get("PORT", "9000") or 9000)
        self.tls_cert = env.get("TLS_CERT")
        self.tls_key = env.get("TLS_KEY")
        self.local_chunkserver = env.get("LOCAL_CHUNKSERVER")
        self.metadata_sidecar = env.get("S3_METADATA_SIDECAR", "") == "true"


class _AuthOk:
    __slots__ = ("user_id", "role_arn", "ctx", "chunk_verifier")

    def __init__(self, user_id="anonymous", role_arn=None, ctx=None, chunk_verifier=None):
        self.user_id, self.role_arn, self.ctx, self.chunk_verifier = user_id, role_arn, ctx, chunk_verifier


class PolicyEpoch:
    """Bucket-policy change counter shared by every process of one gateway (the forked
    aiohttp workers and the native front): a worker that stores or deletes a bucket policy
    bumps it, and every cache that saw an older value drops its entries at once instead of
    serving the old policy for up to its TTL. File-backed (an 8-byte counter in a page that
    each process maps shared); without a file it is a process-local counter."""

    def __init__(self, path: str | None = None):
        import mmap

        self.path = path
        self._local = 0
        self._mm = None
        if path:
            if not os.path.exists(path):
                with open(path, "wb") as f:
                    f.write(b"\0" * 4096)
            fd = os.open(path, os.O_RDWR)
            try:
                self._mm = mmap.mmap(fd, 4096, mmap.MAP_SHARED, mmap.PROT_READ | mmap.PROT_WRITE)
            finally:
                os.close(fd)

    def get(self) -> int:
        if self._mm is None:
            return self._local
        return struct.unpack_from("<Q", self._mm, 0)[0]

    def bump(self) -> None:
        # strictly increasing across processes: the system-wide monotonic clock, at least +1
        nxt = max(self.get() + 1, time.monotonic_ns())
        if self._mm is None:
            self._local = nxt
        else:
            struct.pack_into("<Q", self._mm, 0, nxt)


class S3Gateway:
    def __init__(self, client: Client, cfg: S3Config | None = None, *, registry: Registry | None = None,
                 credential_provider=None, oidc: OidcValidator | None = None, sts: StsTokenManager | None = None,
                 iam: PolicyEvaluator | None = None, audit: AuditLogger | None = None, sse: SseManager | None = None,
                 workers: int = 64):
        self.client = client
        self.cfg = cfg or S3Config({})
        self.registry = registry or Registry()
        self.creds = credential_provider or EnvCredentialProvider(self.cfg.env)
        self.key_cache = sigv4.SigningKeyCache()
        self.oidc, self.sts, self.iam, self.audit, self.sse = oidc, sts, iam, audit, sse
        self.pool = ThreadPoolExecutor(max_workers=workers, thread_name_prefix="s3-dfs")
        self._policy_cache: dict[str, tuple[float, BucketPolicy | None]] = {}
        self.policy_ttl = 1.0
        self.policy_epoch = PolicyEpoch()
        self._policy_epoch_seen = self.policy_epoch.get()
        self.front = None  # the native front when it runs in this process (drop_policies on change)
        self.front_store = None  # its RemoteFrontStore when no chunkserver is co-located
        r = self.registry
        self.m_requests = r.counter("s3_requests_total", "Total number of S3 requests", ("method", "path", "status"))
        self.m_auth = r.counter("iam_auth_requests_total", "Total authentication attempts", ("result", "error_type"))
        self.m_auth_dur = r.histogram("iam_auth_duration_seconds", "Authentication latency", ("result",))
        self.m_policy = r.counter("iam_policy_evaluations_total", "Policy evaluations", ("result", "action"))
        self.m_policy_dur = r.histogram("iam_policy_evaluation_duration_seconds", "Policy evaluation latency")
        self.m_sts = r.counter("iam_sts_requests_total", "STS requests", ("result", "error_type"))
        self.m_sts_dur = r.histogram("iam_sts_token_duration_seconds", "STS token issuance latency")
        self.m_sts_active = r.gauge("iam_sts_active_sessions_gauge", "Active STS sessions")
        self.m_oidc = r.counter("iam_oidc_validations_total", "Total OIDC token validations", ("result",))
        self.m_jwks = r.counter("iam_oidc_jwks_fetches_total", "Total JWKS fetch attempts", ("result",))
        self.m_jwks_dur = r.histogram("iam_oidc_jwks_fetch_duration_seconds", "JWKS fetch latency")
        self.m_jwks_last = r.gauge("iam_oidc_jwks_last_fetch_timestamp", "Last successful JWKS fetch (unix s)")
        self._sts_sessions: list[float] = []
        self.m_client_fallbacks = r.gauge("dfs_client_native_fallbacks", "Gateway DFS-client operations that left "
                                          "the native client for the Python path, by reason", ("reason",))

    # ------------------------------------------------------------------ plumbing
    async def run(self, fn, *args):
        return await asyncio.get_running_loop().run_in_executor(self.pool, fn, *args)

    def app(self) -> web.Application:
        app = web.Application(client_max_size=MAX_BODY + (1 << 20))
        app.router.add_get("/health", self.h_health)
        app.router.add_get("/metrics", self.h_metrics)
        app.router.add_route("*", "/{tail:.*}", self.dispatch)
        app.on_cleanup.append(self._cleanup)
        app.on_startup.append(self._warm)
        if self.oidc is not None:
            app.on_startup.append(self._start_jwks_refresh)
        return app

    async def _cleanup(self, _app) -> None:
        if getattr(self, "_jwks_task", None):
            self._jwks_task.cancel()
        if self.audit is not None:
            await self.run(self.audit.close)
        self.pool.shutdown(wait=False)

    async def _warm(self, _app) -> None:
        """Before serving: one tiny write + delete through the DFS client, so its channels,
        its shared-memory arena and the co-located chunkserver's mapping (and GPU pinning) of
        that arena exist before the first request instead of stalling it."""
        if not self.client.local_chunkserver:
            return

        def work():
            p = f"{MPU_ROOT}/.warm-{os.getpid()}-{uuid.uuid4().hex[:8]}"
            try:
                self.client.create_file_from_buffer(b"w", p)
                self.client.delete_file(p)
            except DfsError as e:
                log.info("client warm-up skipped: %s", e)
        await self.run(work)

    async def _start_jwks_refresh(self, _app) -> None:
        async def loop():
            while True:
                t0 = time.monotonic()
                try:
                    await self.run(self.oidc.fetch_jwks)
                    self.m_jwks.inc(labels={"result": "success"})
                    self.m_jwks_last.set(time.time())
                except AuthError as e:
                    self.m_jwks.inc(labels={"result": "failure"})
                    log.warning("JWKS refresh failed: %s", e)
                self.m_jwks_dur.observe(time.monotonic() - t0)
                await asyncio.sleep(3600)
        self._jwks_task = asyncio.get_running_loop().create_task(loop())

    async def h_health(self, _req):
        return web.Response(text="OK")

    async def h_metrics(self, _req):
        now = time.time()
        self._sts_sessions = [t for t in self._sts_sessions if t > now]
        self.m_sts_active.set(len(self._sts_sessions))
        for reason, n in dict(getattr(self.client, "native_fallbacks", {})).items():
            self.m_client_fallbacks.set(n, labels={"reason": reason})
        lines = []
        for m in self.registry._metrics:  # noqa: SLF001 - registry is ours
            lines.extend(m.render())
        return web.Response(text="\n".join(lines) + "\n", content_type="text/plain")

    @staticmethod
    def xml(status: int, body: str, headers: dict | None = None) -> web.Response:
        return web.Response(status=status, body=body.encode(), headers={"Content-Type": "application/xml",
                                                                        **(headers or {})})

    @staticmethod
    def empty(status: int, headers: dict | None = None) -> web.Response:
        return web.Response(status=status, headers=headers)

    def s3_error(self, status: int, code: str, message: str, resource: str = "") -> web.Response:
        return self.xml(status, X.error(code, message, resource))

    # ------------------------------------------------------------------ entry point
    async def dispatch(self, request: web.Request) -> web.StreamResponse:
        raw_query = request.rel_url.raw_query_string
        query = sigv4.parse_query(raw_query)
        path = request.rel_url.path  # decoded
        bucket_label = path.lstrip("/").split("/", 1)[0] or "/"
        if path in ("", "/") and (query.get("Action") == "AssumeRoleWithWebIdentity" or
                                  (request.method == "POST" and request.content_type ==
                                   "application/x-www-form-urlencoded")):
            resp = await self.handle_sts(request, query)
            self.m_requests.inc(labels={"method": request.method, "path": "/", "status": resp.status})
            return resp
        started = time.time()
        auth = None
        if self.cfg.auth_enabled:
            auth = await self.authenticate(request, query, raw_query, started)
            if isinstance(auth, web.Response):
                self.m_requests.inc(labels={"method": request.method, "path": bucket_label, "status": auth.status})
                return auth
        try:
            resp = await self.route(request, path, query, auth)
        except DfsError as e:
            log.warning("%s %s failed: %s", request.method, path, e)
            resp = self.s3_error(500, "InternalError", str(e), path)
        if auth is not None:
            self._audit(request, query, started, auth.user_id, auth.role_arn, resp.status, None)
        self.m_requests.inc(labels={"method": request.method, "path": bucket_label, "status": resp.status})
        return resp

    async def route(self, request: web.Request, path: str, query: dict, auth: _AuthOk | None):
        m = request.method
        p = path.lstrip("/")
        if not p:
            return await self.list_buckets() if m == "GET" else self.empty(405)
        bucket, _, key = p.partition("/")
        body = b""
        if m in ("PUT", "POST"):
            body = await request.read()
            body = self._maybe_decode_chunked(request, body, auth)
            if body is None:
                return self.s3_error(403, "SignatureDoesNotMatch", "aws-chunked signature chain is invalid")
        if not key:
            if "policy" in query:
                if m == "GET":
                    return await self.get_bucket_policy(bucket)
                if m == "PUT":
                    return await self.put_bucket_policy(bucket, body)
                if m == "DELETE":
                    return await self.delete_bucket_policy(bucket)
                return self.empty(405)
            if m == "POST" and "delete" in query:
                return await self.delete_objects(bucket, body)
            if m == "PUT":
                return await self.create_bucket(bucket)
            if m == "DELETE":
                return await self.delete_bucket(bucket)
            if m == "HEAD":
                return await self.head_bucket(bucket)
            if m == "GET":
                if "location" in query:
                    return self.xml(200, f"<LocationConstraint>{self.cfg.region}</LocationConstraint>")
                return await self.list_objects(bucket, query, v2=query.get("list-type") == "2")
            return self.empty(405)
        if reserved_key(key):
            # object keys must not address the gateway's own sidecar files: a PUT/DELETE of
            # `.s3_bucket_policy` would replace or drop the bucket policy, `<k>.meta` another
            # object's headers and SSE key
            return self.s3_error(400, "InvalidArgument", f"object key {key!r} is reserved")
        if m == "POST" and "uploads" in query:
            return await self.initiate_mpu(bucket, key)
        if m == "POST" and "delete" in query:
            return await self.delete_objects(bucket, body)
        upload_id = query.get("uploadId")
        if upload_id is not None:
            if "/" in upload_id or upload_id in ("", ".", ".."):
                return self.s3_error(400, "InvalidArgument", "bad uploadId")
            if m == "PUT" and "partNumber" in query:
                try:
                    n = int(query["partNumber"])
                except ValueError:
                    return self.s3_error(400, "InvalidArgument", "bad partNumber")
                if not 1 <= n <= 10000:
                    return self.s3_error(400, "InvalidArgument", "partNumber must be 1..10000")
                return await self.upload_part(upload_id, n, body)
            if m == "POST":
                return await self.complete_mpu(bucket, key, upload_id, body)
            if m == "DELETE":
                return await self.abort_mpu(upload_id)
        if m == "PUT" and "x-amz-copy-source" in request.headers:
            return await self.copy_object(bucket, key, request.headers["x-amz-copy-source"], request.headers)
        if m == "PUT":
            return await self.put_object(bucket, key, body, request.headers)
        if m == "GET":
            return await self.get_object(bucket, key, request.headers)
        if m == "HEAD":
            return await self.head_object(bucket, key)
        if m == "DELETE":
            return await self.delete_object(bucket, key)
        return self.empty(405)

    def _maybe_decode_chunked(self, request, body: bytes, auth: _AuthOk | None) -> bytes | None:
        sha = request.headers.get("x-amz-content-sha256", "")
        enc = request.headers.get("Content-Encoding", "")
        if not (sha.startswith("STREAMING-") or "aws-chunked" in enc):
            return body
        verifier = auth.chunk_verifier if (auth is not None and sha == "STREAMING-AWS4-HMAC-SHA256-PAYLOAD") else None
        try:
            return sigv4.decode_chunked(body, verifier)
        except sigv4.ChunkedDecodeError as e:
            log.warning("aws-chunked decode failed: %s", e)
            return None

    # ------------------------------------------------------------------ auth (C54)
    def _audit(self, request, query, started, user_id, role_arn, status, error_code, action=None, resource=None):
        if self.audit is None:
            return
        if action is None:
            action, resource = resolve_action_and_resource(request.method, request.rel_url.path, query)
        peer = request.transport.get_extra_info("peername") if request.transport else None
        ip = peer[0] if peer else (request.headers.get("x-real-ip") or
                                   (request.headers.get("x-forwarded-for", "").split(",")[0].strip() or "unknown"))
        self.audit.log(make_record(request_id=request.headers.get("x-request-id") or str(uuid.uuid4()),
                                   remote_ip=ip, user_id=user_id, role_arn=role_arn, action=action,
                                   resource=resource, status_code=status, error_code=error_code,
                                   user_agent=request.headers.get("User-Agent"),
                                   duration_ms=int((time.time() - started) * 1000)))

    def _auth_fail(self, request, query, started, err: AuthError, user_id="anonymous", role_arn=None,
                   audit_code: str | None = None) -> web.Response:
        self.m_auth.inc(labels={"result": "failure", "error_type": err.error_type})
        self.m_auth_dur.observe(time.time() - started, labels={"result": "failure"})
        resp = web.Response(status=err.status, body=err.xml().encode(), headers={"Content-Type": "application/xml"})
        self._audit(request, query, started, user_id, role_arn, resp.status, audit_code or err.code)
        return resp

    async def authenticate(self, request: web.Request, query: dict, raw_query: str, started: float):
        h = request.headers
        if self.cfg.require_tls and not (request.secure or h.get("X-Forwarded-Proto") == "https"):
            return self._auth_fail(request, query, started, AuthError("insecure_transport"))
        presigned = "X-Amz-Expires" in query and "X-Amz-Algorithm" in query
        try:
            cred = sigv4.parse_credentials(h, query)
        except AuthError as e:
            return self._auth_fail(request, query, started, e)
        user = cred.access_key
        req_time = sigv4.parse_amz_time(cred.timestamp)
        now = datetime.now(timezone.utc)
        if presigned:
            if req_time is None:
                return self._auth_fail(request, query, started, AuthError("missing_auth"), user,
                                       audit_code="InvalidArgument")
            try:
                expires = int(query.get("X-Amz-Expires", ""))
            except ValueError:
                expires = 0
            if expires <= 0:
                return self._auth_fail(request, query, started, AuthError("missing_auth"), user,
                                       audit_code="InvalidArgument")
            if expires > sigv4.MAX_PRESIGN_EXPIRES:
                return self._auth_fail(request, query, started, AuthError("missing_auth"), user,
                                       audit_code="AuthorizationQueryParametersError")
            if sigv4.presigned_is_expired(cred.timestamp, expires, now):
                return self._auth_fail(request, query, started, AuthError("expired_token"), user)
        elif req_time is not None and abs((now - req_time).total_seconds()) / 60.0 > sigv4.MAX_SKEW_MINUTES:
            return self._auth_fail(request, query, started, AuthError("clock_skew"), user)
        if cred.region != self.cfg.region or cred.service != "s3":
            return self._auth_fail(request, query, started, AuthError("invalid_scope"), user)
        token = h.get("x-amz-security-token") or query.get("X-Amz-Security-Token")
        role_arn = ctx = None
        if token:
            if self.sts is None:
                return self._auth_fail(request, query, started, AuthError("internal", "STS is not enabled"), user)
            try:
                sess = self.sts.decrypt_token(token)
            except AuthError as e:
                return self._auth_fail(request, query, started, e, user)
            role_arn = sess.role_arn
            if sess.expiration < int(time.time()):
                return self._auth_fail(request, query, started, AuthError("expired_token"), user, role_arn)
            secret = sess.temp_secret_key
            ctx = sess.claims.to_policy_context()
        else:
            secret = self.creds.get_secret_key(cred.access_key)
            if secret is None:
                return self._auth_fail(request, query, started, AuthError("invalid_access_key"), user)
        # STS sessions derive keys from their per-session secret: never share a cache slot
        # between a session and a static key with the same access-key id.
        cache_id = cred.access_key if not token else f"{cred.access_key}#{hashlib.sha256(token.encode()).hexdigest()}"
        skey = self.key_cache.get(cache_id, cred.date)
        if skey is None:
            skey = sigv4.derive_signing_key(secret, cred.date, cred.region, cred.service)
            self.key_cache.insert(cache_id, cred.date, skey)
        inp = sigv4.build_signing_input(request.method, request.rel_url.raw_path,
                                        sigv4.normalize_query_string(raw_query), h, cred)
        if inp.payload_hash == sigv4.UNSIGNED_PAYLOAD and not self.cfg.allow_unsigned_payload and not presigned:
            return self._auth_fail(request, query, started, AuthError("missing_auth"), user, role_arn)
        try:
            sigv4.verify_signature_with_key(inp, cred, skey)
        except AuthError as e:
            log.info("signature mismatch for %s: %s", user, e.detail)
            return self._auth_fail(request, query, started, e, user, role_arn)
        self.m_auth.inc(labels={"result": "success", "error_type": "none"})
        self.m_auth_dur.observe(time.time() - started, labels={"result": "success"})
        action, resource = resolve_action_and_resource(request.method, request.rel_url.path, query)
        if role_arn is not None and self.iam is not None and ctx is not None:
            t0 = time.perf_counter()
            allowed = self.iam.evaluate(action, resource, role_arn, ctx)
            self.m_policy_dur.observe(time.perf_counter() - t0)
            self.m_policy.inc(labels={"result": "allow" if allowed else "deny", "action": action})
            if not allowed:
                return self._auth_fail(request, query, started, AuthError("missing_auth"), user, role_arn,
                                       audit_code="AccessDenied")
        if "policy" not in query:
            bucket = request.rel_url.path.lstrip("/").split("/", 1)[0]
            if bucket:
                pol = await self._bucket_policy(bucket)
                if pol is not None and pol.evaluate(role_arn, action, resource) is PolicyResult.EXPLICIT_DENY:
                    self.m_policy.inc(labels={"result": "deny", "action": action})
                    return self._auth_fail(request, query, started, AuthError("missing_auth"), user, role_arn,
                                           audit_code="AccessDenied")
        verifier = sigv4.ChunkVerifier(skey, cred.timestamp, cred.scope, cred.signature)
        return _AuthOk(user, role_arn, ctx, verifier)

    def _policy_changed(self, bucket: str) -> None:
        self._policy_cache.pop(bucket, None)
        self.policy_epoch.bump()
        if self.front is not None:
            self.front.drop_policies()

    async def _bucket_policy(self, bucket: str) -> BucketPolicy | None:
        ep = self.policy_epoch.get()
        if ep != self._policy_epoch_seen:  # another worker changed a policy
            self._policy_cache.clear()
            self._policy_epoch_seen = ep
        ent = self._policy_cache.get(bucket)
        now = time.monotonic()
        if ent is not None and ent[0] > now:
            return ent[1]
        path = f"/{bucket}/.s3_bucket_policy"

        def load():
            try:
                return BucketPolicy.parse(self.client.get_file_content(path))
            except (DfsError, ValueError, json.JSONDecodeError):
                return None
        pol = await self.run(load)
        if self.policy_epoch.get() == ep:  # not cached when a change raced the fetch
            if len(self._policy_cache) >= 4096:
                self._policy_cache.clear()
            self._policy_cache[bucket] = (now + self.policy_ttl, pol)
        return pol

    # ------------------------------------------------------------------ STS (C55)
    async def handle_sts(self, request: web.Request, query: dict) -> web.Response:
        started = time.time()
        t0 = time.perf_counter()
        params = dict(query)
        if request.method == "POST" and request.content_type == "application/x-www-form-urlencoded":
            params.update(parse_qsl((await request.read()).decode("utf-8", "replace"), keep_blank_values=True))
        action = params.get("Action", "Unknown")

        def fail(status, code, message, user="anonymous", role=None):
            self.m_sts.inc(labels={"result": "failure", "error_type": code})
            self._audit(request, query, started, user, role, status, code, action, "arn:dfs:sts:::*")
            return self.xml(status, X.sts_error(code, message))

        if action != "AssumeRoleWithWebIdentity":
            self.m_sts.inc(labels={"result": "failure", "error_type": "InvalidAction"})
            self._audit(request, query, started, "anonymous", None, 400, "InvalidAction", action, "arn:dfs:sts:::*")
            return self.empty(400)
        if self.oidc is None:
            return fail(500, "OIDC_NOT_ENABLED", "OIDC validation is not enabled on this server.")
        if self.sts is None:
            return fail(500, "STS_NOT_ENABLED", "STS is not enabled on this server.")
        if self.iam is None:
            return fail(500, "IAM_NOT_ENABLED", "IAM policy evaluation is not enabled on this server.")
        token = params.get("WebIdentityToken")
        if not token:
            return fail(400, "MissingToken", "WebIdentityToken is required")
        role_arn = params.get("RoleArn")
        if not role_arn:
            return fail(400, "MissingRole", "RoleArn is required")
        try:
            claims = await self.run(self.oidc.validate_token, token)
            self.m_oidc.inc(labels={"result": "success"})
        except AuthError as e:
            self.m_oidc.inc(labels={"result": "failure"})
            return fail(403, "InvalidIdentityToken", str(e), role=role_arn)
        if not self.iam.can_assume_role(role_arn, claims.to_policy_context()):
            return fail(403, "AccessDenied", "User is not authorized to assume this role.", claims.sub, role_arn)
        try:
            duration = int(params.get("DurationSeconds", "3600"))
        except ValueError:
            return fail(400, "ValidationError", "DurationSeconds must be an integer", claims.sub, role_arn)
        if not 1 <= duration <= 43200:
            return fail(400, "ValidationError", "DurationSeconds must be in [1, 43200]", claims.sub, role_arn)
        exp = int(time.time()) + duration
        secret = random_alnum(40)
        akid = ("ASIA" + uuid.uuid4().hex[:16]).upper()
        try:
            tok = self.sts.generate_token(StsSessionData(role_arn, secret, exp, claims))
        except AuthError as e:
            return fail(500, "InternalError", str(e), claims.sub, role_arn)
        role_name = role_arn.rsplit("/", 1)[-1] or "role"
        session = params.get("RoleSessionName", "session")
        self.m_sts.inc(labels={"result": "success", "error_type": "none"})
        self.m_sts_dur.observe(time.perf_counter() - t0)
        self._sts_sessions.append(float(exp))
        self._audit(request, query, started, claims.sub, role_arn, 200, None, action, "arn:dfs:sts:::*")
        expiration = datetime.fromtimestamp(exp, tz=timezone.utc).strftime("%Y-%m-%dT%H:%M:%SZ")
        return self.xml(200, X.sts_result(akid, secret, tok, expiration, claims.sub, f"{role_name}:{session}",
                                          f"arn:dfs:sts:::assumed-role/{role_name}/{session}"))

    # ------------------------------------------------------------------ buckets
    async def list_buckets(self) -> web.Response:
        files = await self.run(self.client.list_all_files, "/")
        names = sorted({f.strip("/").split("/", 1)[0] for f in files} - {"", ".s3_mpu"})
        return self.xml(200, X.list_all_my_buckets([(n, DEFAULT_DATE) for n in names]))

    async def create_bucket(self, bucket: str) -> web.Response:
        try:
            await self.run(self.client.create_file_from_buffer, b"", f"/{bucket}/.s3keep")
        except DfsError as e:
            if "already exists" in str(e):
                return self.empty(409)
            raise
        return self.empty(200, {"Location": f"/{bucket}"})

    async def delete_bucket(self, bucket: str) -> web.Response:
        files = await self.run(self.client.list_all_files, f"/{bucket}/")
        if files and any(not f.endswith((".s3keep", ".s3_bucket_policy")) for f in files):
            return self.xml(409, X.error("BucketNotEmpty", "The bucket you tried to delete is not empty", bucket))
        if not files:
            return self.xml(404, X.error("NoSuchBucket", "The specified bucket does not exist", bucket))
        for f in files:
            await self.run(self._delete_quiet, f)
        self._policy_changed(bucket)
        return self.empty(204)

    async def head_bucket(self, bucket: str) -> web.Response:
        if await self.run(self.client.exists, f"/{bucket}/.s3keep"):
            return self.empty(200)
        files = await self.run(self.client.list_all_files, f"/{bucket}/")
        return self.empty(200 if files else 404)

    def _delete_quiet(self, path: str) -> bool:
        try:
            self.client.delete_file(path)
            return True
        except DfsError:
            return False

    # ------------------------------------------------------------------ bucket policy
    async def get_bucket_policy(self, bucket: str) -> web.Response:
        try:
            data = await self.run(self.client.get_file_content, f"/{bucket}/.s3_bucket_policy")
            json.loads(data)
        except (DfsError, ValueError):
            return self.xml(404, X.error("NoSuchBucketPolicy", "The bucket policy does not exist", BucketName=bucket))
        return web.Response(status=200, body=data, headers={"Content-Type": "application/json"})

    async def put_bucket_policy(self, bucket: str, body: bytes) -> web.Response:
        try:
            BucketPolicy.parse(body)
        except (ValueError, KeyError, TypeError):
            return self.xml(400, "<Error><Code>MalformedPolicy</Code><Message>Bucket policy must be valid JSON"
                                 "</Message></Error>")
        path = f"/{bucket}/.s3_bucket_policy"
        try:
            await self.run(self._put_replace, body, path)
        except DfsError:
            return self.xml(500, "<Error><Code>InternalError</Code><Message>Failed to store bucket policy"
                                 "</Message></Error>")
        self._policy_changed(bucket)
        return self.empty(204)

    async def delete_bucket_policy(self, bucket: str) -> web.Response:
        await self.run(self._delete_quiet, f"/{bucket}/.s3_bucket_policy")
        self._policy_changed(bucket)
        return self.empty(204)

    # ------------------------------------------------------------------ objects
    def _put_replace(self, data: bytes, path: str, attributes: dict | None = None, md5: str | None = None) -> None:
        try:
            self.client.create_file_from_buffer(data, path, attributes, md5)
        except DfsError as e:
            if "already exists" not in str(e):
                raise
            self.client.delete_file(path)
            self.client.create_file_from_buffer(data, path, attributes, md5)

    def _put_object_file(self, data: bytes, path: str, headers: dict, md5: str | None = None) -> None:
        """The object file with its headers as attributes (+ the reference's sidecar when
        S3_METADATA_SIDECAR=true)."""
        self._put_replace(data, path, headers, md5)
        if self.cfg.metadata_sidecar:
            self._write_meta(path, headers)

    def _write_meta(self, path: str, headers: dict) -> None:
        meta = json.dumps({"headers": headers}, separators=(",", ":")).encode()
        self._delete_quiet(path + ".meta")
        try:
            self.client.create_file_from_buffer(meta, path + ".meta")
        except DfsError as e:
            log.warning("failed to write object metadata for %s: %s", path, e)

    def _meta_of(self, path: str, info) -> dict:
        """Object headers: the file's attributes, else the reference's sidecar."""
        if info is not None and info.attributes:
            return dict(info.attributes)
        return self._read_meta(path)

    def _mpu_marker_meta(self, path: str) -> dict:
        info = self.client.get_file_info(path + "/.s3_mpu_completed")
        return self._meta_of(path, info) if info is not None else {}

    def _read_meta(self, path: str) -> dict:
        try:
            d = json.loads(self.client.get_file_content(path + ".meta"))
            h = d.get("headers", {})
            return h if isinstance(h, dict) else {}
        except (DfsError, ValueError, AttributeError):
            return {}

    async def put_object(self, bucket: str, key: str, body: bytes, headers) -> web.Response:
        path = f"/{bucket}/{key}"
        md5 = await self.run(lambda: hashlib.md5(body).hexdigest())  # GIL released while hashing
        etag = f'"{md5}"'
        dek = None
        data = body
        if self.sse is not None:
            data, dek = await self.run(self.sse.encrypt_object, body)
        meta = {"ETag": etag}
        for k, v in headers.items():
            lk = k.lower()
            if lk.startswith("x-amz-meta-"):
                meta[lk] = v
        if "Content-Type" in headers:
            meta["Content-Type"] = headers["Content-Type"]
        if dek is not None:
            meta["x-amz-sse-encrypted-dek"] = dek
        # the stored bytes' MD5 is the client's etag_md5: ours when they are the plaintext
        await self.run(self._put_object_file, data, path, meta, None if dek is not None else md5)
        out = {"ETag": etag}
        if dek is not None:
            out["x-amz-server-side-encryption"] = "AES256"
        return self.empty(200, out)

    def _mpu_parts(self, path: str) -> list[tuple[int, str]] | None:
        """Parts of a completed multipart object, or None if ``path`` is not one."""
        files = self.client.list_all_files(path + "/")
        if path + "/.s3_mpu_completed" not in files:
            return None
        parts = []
        for f in files:
            name = f[len(path) + 1:]
            if name.isdigit():
                parts.append((int(name), f))
        return sorted(parts)

    def _object_headers(self, meta: dict, info) -> tuple[dict, str | None]:
        etag = f'"{info.etag_md5}"' if info is not None and info.etag_md5 else EMPTY_ETAG
        out = {"Last-Modified": _http_date(info.created_at_ms if info is not None else None),
               "Accept-Ranges": "bytes"}
        dek = None
        for k, v in meta.items():
            if k == "ETag":
                etag = v
            elif k == "x-amz-sse-encrypted-dek":
                dek = v
            elif k.startswith("x-amz-meta-") or k == "Content-Type":
                out[k] = v
        out["ETag"] = etag
        out.setdefault("Content-Type", "application/octet-stream")
        if dek is not None:
            out["x-amz-server-side-encryption"] = "AES256"
        return out, dek

    def _decrypt(self, data: bytes, dek: str | None) -> bytes:
        if dek is None or self.sse is None:
            return data
        return self.sse.decrypt_object(data, dek)

    def _range_response(self, data_fn, size: int, rng, headers: dict) -> web.Response:
        if rng == "unsatisfiable":
            return self.xml(416, X.error("InvalidRange", "The requested range is not satisfiable"),
                            {"Content-Range": f"bytes */{size}"})
        if rng is None:
            return web.Response(status=200, body=data_fn(0, size), headers=headers)
        s, e = rng
        headers["Content-Range"] = f"bytes {s}-{e}/{size}"
        return web.Response(status=206, body=data_fn(s, e - s + 1), headers=headers)

    async def get_object(self, bucket: str, key: str, req_headers) -> web.Response:
        path = f"/{bucket}/{key}"
        info = await self.run(self.client.get_file_info, path)
        if info is None:
            parts = await self.run(self._mpu_parts, path)
            meta = await self.run(self._mpu_marker_meta, path) if parts is not None else {}
            if parts is None:
                return self.xml(404, X.error("NoSuchKey", "The specified key does not exist.", path))
            headers, dek = self._object_headers(meta, None)
            if dek is not None:
                try:
                    chunks = await asyncio.gather(*[self.run(self.client.get_file_content, p) for _, p in parts])
                    data = b"".join([await self.run(self._decrypt, c, dek) for c in chunks])
                except AuthError:
                    return self.s3_error(500, "InternalError", "SSE decryption failed")
                return self._range_response(lambda o, n: data[o:o + n], len(data),
                                            parse_range(req_headers.get("Range"), len(data)), headers)
            return await self._mpu_range(parts, meta, req_headers.get("Range"), headers)
        size = int(info.size)
        rng_hdr = req_headers.get("Range")
        rng = parse_range(rng_hdr, size)
        # Start the (range) read at once (with the metadata just fetched, no second
        # GetFileInfo); an SSE object needs the whole ciphertext, fetched below once the
        # DEK is known. Objects without attributes load the reference's sidecar meanwhile.
        if isinstance(rng, tuple):
            s, e = rng
            data_fut = asyncio.ensure_future(self.run(self.client.read_file_range, path, s, e - s + 1, info))
        elif rng is None and size > 0:
            data_fut = asyncio.ensure_future(self.run(self.client.get_file_content, path, info))
        else:
            data_fut = None
        meta = dict(info.attributes) if info.attributes else await self.run(self._read_meta, path)
        headers, dek = self._object_headers(meta, info)
        if dek is not None and self.sse is not None:
            if data_fut is not None:
                data_fut.cancel()
            try:
                raw = await self.run(self.client.get_file_content, path, info)
                plain = await self.run(self._decrypt, raw, dek)
            except AuthError:
                return self.s3_error(500, "InternalError", "SSE decryption failed")
            return self._range_response(lambda o, n: plain[o:o + n], len(plain), parse_range(rng_hdr, len(plain)),
                                        headers)
        if rng == "unsatisfiable":
            return self._range_response(None, size, rng, headers)
        body = await data_fut if data_fut is not None else b""
        if isinstance(rng, tuple):
            headers["Content-Range"] = f"bytes {rng[0]}-{rng[1]}/{size}"
            return web.Response(status=206, body=body, headers=headers)
        return web.Response(status=200, body=body, headers=headers)

    async def _mpu_range(self, parts, meta: dict, rng_hdr, headers: dict) -> web.Response:
        """GET (or Range GET) of a multipart object: only the parts overlapping the range are
        read, each with a ranged read, in parallel (a Parquet footer or column-chunk request
        touches one part, not the whole object)."""
        sizes = _mpu_layout(meta, [n for n, _ in parts])
        if sizes is None:  # completed before the layout attribute existed: ask the master
            infos = await asyncio.gather(*[self.run(self.client.get_file_info, p) for _, p in parts])
            sizes = [int(i.size) if i is not None else 0 for i in infos]
        total = sum(sizes)
        rng = parse_range(rng_hdr, total)
        if rng == "unsatisfiable":
            return self._range_response(None, total, rng, headers)
        s, e = rng if isinstance(rng, tuple) else (0, total - 1)
        reads, pos = [], 0
        for (_, p), sz in zip(parts, sizes):
            lo, hi = max(s, pos), min(e + 1, pos + sz)
            if lo == pos and hi == pos + sz:  # whole part: the client's native fast read
                reads.append(self.run(self.client.get_file_content, p))
            elif lo < hi:
                reads.append(self.run(self.client.read_file_range, p, lo - pos, hi - lo))
            pos += sz
        body = b"".join(await asyncio.gather(*reads)) if reads else b""
        if isinstance(rng, tuple):
            headers["Content-Range"] = f"bytes {s}-{e}/{total}"
            return web.Response(status=206, body=body, headers=headers)
        return web.Response(status=200, body=body, headers=headers)

    async def head_object(self, bucket: str, key: str) -> web.Response:
        path = f"/{bucket}/{key}"
        info = await self.run(self.client.get_file_info, path)
        if info is None:
            parts = await self.run(self._mpu_parts, path)
            if parts is not None:
                meta = await self.run(self._mpu_marker_meta, path)
                headers, _ = self._object_headers(meta, None)
                headers["Last-Modified"] = formatdate(usegmt=True)
                headers["Content-Length"] = str(meta.get("x-dfs-mpu-size", 0))
                return self.empty(200, headers)
            if path.endswith("/") and await self.run(self.client.list_all_files, path):
                return self.empty(200, {"Content-Length": "0"})
            return self.empty(404)
        meta = await self.run(self._meta_of, path, info)
        headers, _ = self._object_headers(meta, info)
        headers["Content-Length"] = str(info.size)
        return self.empty(200, headers)

    async def delete_object(self, bucket: str, key: str) -> web.Response:
        path = f"/{bucket}/{key}"

        def work():
            self._delete_quiet(path)
            # children of a multipart object live under "{key}/" (the reference matched the
            # bare prefix, which also deleted sibling keys such as "{key}2")
            for f in self.client.list_all_files(path + "/"):
                self._delete_quiet(f)
            self._delete_quiet(path + ".meta")
        await self.run(work)
        return self.empty(204)

    async def delete_objects(self, bucket: str, body: bytes) -> web.Response:
        try:
            keys, quiet = X.parse_delete_request(body)
        except Exception:  # noqa: BLE001 - any malformed XML
            return self.s3_error(400, "MalformedXML", "The XML you provided was not well-formed")

        def one(k: str):
            if reserved_key(k):
                return k, ("InvalidArgument", f"object key {k!r} is reserved")
            path = f"/{bucket}/{k}"
            try:
                self.client.delete_file(path)
            except DfsError as e:
                if "not found" not in str(e).lower():
                    return k, ("InternalError", str(e))
            self._delete_quiet(path + ".meta")
            return k, None
        results = await asyncio.gather(*[self.run(one, k) for k in keys])
        deleted = [k for k, err in results if err is None]
        errors = [(k, c, m) for k, err in results if err is not None for c, m in [err]]
        return self.xml(200, X.delete_result(deleted, errors, quiet))

    async def copy_object(self, bucket: str, key: str, source: str, req_headers) -> web.Response:
        src = unquote(source.split("?", 1)[0])
        src_path = src if src.startswith("/") else "/" + src
        if reserved_key(src_path):
            return self.s3_error(400, "InvalidArgument", "copy source is reserved")
        dest = f"/{bucket}/{key}"

        def load_source():
            info = self.client.get_file_info(src_path)
            if info is not None:
                meta = self._meta_of(src_path, info)
                dek = meta.get("x-amz-sse-encrypted-dek")
                return self._decrypt(self.client.get_file_content(src_path, info), dek), meta
            parts = self._mpu_parts(src_path)
            if parts is None:
                return None, {}
            meta = self._mpu_marker_meta(src_path)
            dek = meta.get("x-amz-sse-encrypted-dek")
            return b"".join(self._decrypt(self.client.get_file_content(p), dek) for _, p in parts), meta
        try:
            data, src_meta = await self.run(load_source)
        except AuthError:
            return self.s3_error(500, "InternalError", "SSE decryption failed")
        if data is None:
            return self.xml(404, X.error("NoSuchKey", "The specified key does not exist.", src_path))
        md5 = await self.run(lambda: hashlib.md5(data).hexdigest())
        etag = f'"{md5}"'
        dek = None
        payload = data
        if self.sse is not None:
            payload, dek = await self.run(self.sse.encrypt_object, data)
        meta = {"ETag": etag}
        if req_headers.get("x-amz-metadata-directive", "COPY").upper() == "REPLACE":
            meta.update({k.lower(): v for k, v in req_headers.items() if k.lower().startswith("x-amz-meta-")})
        else:
            meta.update({k: v for k, v in src_meta.items() if k.startswith("x-amz-meta-") or k == "Content-Type"})
        if dek is not None:
            meta["x-amz-sse-encrypted-dek"] = dek
        await self.run(self._put_object_file, payload, dest, meta, None if dek is not None else md5)
        return self.xml(200, X.copy_object(datetime.now(timezone.utc).isoformat(), etag))

    # ------------------------------------------------------------------ listings
    async def list_objects(self, bucket: str, q: dict, v2: bool) -> web.Response:
        prefix = q.get("prefix", "")
        delim = q.get("delimiter") or None
        try:
            max_keys = max(0, min(int(q.get("max-keys", "1000")), 1000))
        except ValueError:
            return self.s3_error(400, "InvalidArgument", "max-keys must be an integer")
        marker = (q.get("continuation-token") or q.get("start-after") or "") if v2 else q.get("marker", "")
        bp = f"/{bucket}/"
        # one ListFiles round per shard with every file's metadata (the with_metadata
        # extension) instead of a GetFileInfo per listed key
        infos = await self.run(self.client.list_all_files_with_metadata, bp)
        files = list(infos)
        if not files and not await self.run(self.client.exists, bp + ".s3keep"):
            return self.xml(404, X.error("NoSuchBucket", "The specified bucket does not exist", bucket))
        fileset = set(files)
        mpu_dirs = {f[:-len("/.s3_mpu_completed")] for f in files if f.endswith("/.s3_mpu_completed")}
        entries: dict[str, str | None] = {}  # key -> full path (None for MPU objects)
        for f in files:
            if not f.startswith(bp) or f.endswith(HIDDEN_SUFFIXES):
                continue
            parent = f.rsplit("/", 1)[0]
            if parent in mpu_dirs:
                continue
            entries[f[len(bp):]] = f
        for d in mpu_dirs:
            if d.startswith(bp):
                entries[d[len(bp):]] = None
        keys = sorted(k for k in entries if k.startswith(prefix) and k > marker)
        objects, cps, seen = [], [], set()
        truncated = False
        next_marker = None
        count = 0
        for k in keys:
            if delim:
                i = k.find(delim, len(prefix))
                if i >= 0:
                    cp = k[:i + len(delim)]
                    if cp in seen:
                        continue
                    if count >= max_keys:
                        truncated = True
                        break
                    seen.add(cp)
                    cps.append(cp)
                    count += 1
                    next_marker = cp
                    continue
            if count >= max_keys:
                truncated = True
                break
            objects.append(k)
            count += 1
            next_marker = k

        def describe(k: str) -> dict:
            p = entries[k]
            if p is None:
                mk = infos.get(bp + k + "/.s3_mpu_completed")
                meta = self._meta_of(bp + k, mk) if mk is not None else self._mpu_marker_meta(bp + k)
                return {"key": k, "last_modified": DEFAULT_DATE, "etag": meta.get("ETag", '"000-MPU"'),
                        "size": int(meta.get("x-dfs-mpu-size", 0))}
            info = infos.get(p)
            etag = EMPTY_ETAG
            size, lm = 0, DEFAULT_DATE
            if info is not None:
                size = int(info.size)
                if info.etag_md5:
                    etag = f'"{info.etag_md5}"'
                lm = _iso_ms(info.created_at_ms)
            if info is not None and info.attributes:
                etag = info.attributes.get("ETag", etag)
            elif p + ".meta" in fileset:
                meta = self._read_meta(p)
                etag = meta.get("ETag", etag)
            return {"key": k, "last_modified": lm, "etag": etag, "size": size}
        described = await asyncio.gather(*[self.run(describe, k) for k in objects])
        if v2:
            return self.xml(200, X.list_bucket_v2(bucket, prefix, described, cps, max_keys, truncated, count,
                                                  q.get("continuation-token"),
                                                  next_marker if truncated else None, q.get("start-after")))
        return self.xml(200, X.list_bucket_v1(bucket, prefix, described, cps, q.get("marker", ""), max_keys,
                                              truncated, next_marker if truncated and delim else None))

    # ------------------------------------------------------------------ multipart (C53)
    async def initiate_mpu(self, bucket: str, key: str) -> web.Response:
        upload_id = str(uuid.uuid4())
        await self.run(self.client.create_file_from_buffer, b"", f"{MPU_ROOT}/{upload_id}/.s3keep")
        return self.xml(200, X.initiate_mpu(bucket, key, upload_id))

    async def upload_part(self, upload_id: str, n: int, body: bytes) -> web.Response:
        if not await self.run(self.client.exists, f"{MPU_ROOT}/{upload_id}/.s3keep"):
            return self.xml(404, X.error("NoSuchUpload", "The specified upload does not exist.", upload_id))
        part = f"{MPU_ROOT}/{upload_id}/{n}"
        md5 = await self.run(lambda: hashlib.md5(body).hexdigest())
        await self.run(self._put_replace, body, part, None, md5)  # part ETag = its etag_md5
        return self.empty(200, {"ETag": f'"{md5}"'})

    async def complete_mpu(self, bucket: str, key: str, upload_id: str, body: bytes) -> web.Response:
        mpu_dir = f"{MPU_ROOT}/{upload_id}"
        try:
            requested = X.parse_complete_mpu(body)
        except Exception:  # noqa: BLE001
            return self.s3_error(400, "MalformedXML", "The XML you provided was not well-formed")
        dest = f"/{bucket}/{key}"

        def work():
            files = self.client.list_all_files(mpu_dir + "/")
            if mpu_dir + "/.s3keep" not in files:
                return "nosuchupload"
            have: dict[int, str] = {}
            sizes: dict[int, int] = {}
            part_files = [f for f in files if f[len(mpu_dir) + 1:].isdigit()]
            for f, info in zip(part_files, self.client._exec.map(self.client.get_file_info, part_files)):
                if info is not None:
                    n = int(f[len(mpu_dir) + 1:])
                    have[n], sizes[n] = f'"{info.etag_md5}"', int(info.size)
            if requested:
                nums = []
                for num, et in requested:
                    if num not in have or (et and et.strip('"') != have[num].strip('"')):
                        return "invalidpart"
                    nums.append(num)
                if nums != sorted(set(nums)):
                    return "invalidorder"
            else:
                nums = sorted(have)
            md5s = b"".join(bytes.fromhex(have[n].strip('"')) for n in nums)
            final_etag = f'"{hashlib.md5(md5s).hexdigest()}-{len(nums)}"'
            total = sum(sizes[n] for n in nums)
            meta = {"ETag": final_etag, "x-dfs-mpu-size": str(total),
                    "x-dfs-mpu-layout": ",".join(f"{n}:{sizes[n]}" for n in nums)}
            # replace whatever object was at the destination (plain file or older MPU)
            self._delete_quiet(dest)
            for f in self.client.list_all_files(dest + "/"):
                self._delete_quiet(f)
            self.client.create_file_from_buffer(b"", dest + "/.s3_mpu_completed", meta)
            for n in nums:
                self.client.rename_file(f"{mpu_dir}/{n}", f"{dest}/{n}")
            for f in files:
                if f.endswith(".etag") or f == mpu_dir + "/.s3keep" or \
                        (f[len(mpu_dir) + 1:].isdigit() and int(f[len(mpu_dir) + 1:]) not in nums):
                    self._delete_quiet(f)
            if self.cfg.metadata_sidecar:
                self._write_meta(dest, meta)
            return final_etag
        res = await self.run(work)
        if res == "nosuchupload":
            return self.xml(404, X.error("NoSuchUpload", "The specified upload does not exist.", upload_id))
        if res in ("invalidpart", "invalidorder"):
            code = "InvalidPart" if res == "invalidpart" else "InvalidPartOrder"
            return self.xml(400, X.error(code, "One or more of the specified parts could not be found or the "
                                               "specified entity tag might not have matched.", upload_id))
        return self.xml(200, X.complete_mpu(f"http://localhost:{self.cfg.port}/{bucket}/{key}", bucket, key, res))

    async def abort_mpu(self, upload_id: str) -> web.Response:
        def work():
            for f in self.client.list_all_files(f"{MPU_ROOT}/{upload_id}/"):
                self._delete_quiet(f)
        await self.run(work)
        return self.empty(204)


# ---------------------------------------------------------------------------- main
def _mpu_layout(meta: dict, nums: list[int]) -> list[int] | None:
    """Part sizes from the completion marker's x-dfs-mpu-layout ("n:size,..."), if it
    describes exactly these parts."""
    try:
        pairs = [tuple(int(x) for x in kv.split(":")) for kv in meta["x-dfs-mpu-layout"].split(",") if kv]
    except (KeyError, ValueError):
        return None
    if [n for n, _ in pairs] != list(nums):
        return None
    return [sz for _, sz in pairs]


class ForwardingAudit:
    """Audit sink of gateway worker processes 1..N-1: records go as datagrams over a UNIX
    socket to worker 0, whose AuditLogger owns the store, so one hash chain covers every
    worker. Like AuditLogger.log it never blocks: a full socket counts a drop."""

    def __init__(self, path: str, registry: Registry):
        self.path = path
        self.sock = socket.socket(socket.AF_UNIX, socket.SOCK_DGRAM)
        self.sock.setblocking(False)
        self.m_dropped = registry.counter("audit_log_dropped_total",
                                          "Total number of audit logs dropped due to full buffer")

    def log(self, rec: dict) -> None:
        try:
            self.sock.sendto(json.dumps(rec, separators=(",", ":")).encode(), self.path)
        except OSError:
            self.m_dropped.inc()

    def flush(self, timeout: float = 10.0) -> bool:
        return True

    def close(self) -> None:
        self.sock.close()


def _audit_ingest(sock: socket.socket, audit: AuditLogger) -> None:
    while True:
        try:
            data = sock.recv(1 << 16)
        except OSError:
            return
        try:
            audit.log(json.loads(data))
        except ValueError:
            log.warning("malformed audit datagram dropped")


def build_gateway(cfg: S3Config, client: Client | None = None, audit_sink=None) -> S3Gateway:
    if client is None:
        client = Client([cfg.master_addr], cfg.config_servers, ca_cert=cfg.ca_cert, domain_name=cfg.domain_name,
                        local_chunkserver=cfg.local_chunkserver)
        if cfg.shard_config:
            client.set_shard_map(ShardMap.load_config_file(cfg.shard_config))
    registry = Registry()
    oidc = OidcValidator(cfg.oidc_issuer, cfg.oidc_client_id, allow_hs256=cfg.oidc_allow_hs256) \
        if cfg.oidc_issuer and cfg.oidc_client_id else None
    sts = StsTokenManager.from_signing_key(cfg.sts_signing_key) if cfg.sts_signing_key else None
    iam = None
    if cfg.iam_config_path:
        try:
            iam = PolicyEvaluator.from_file(cfg.iam_config_path)
        except (OSError, ValueError, KeyError) as e:
            log.error("failed to load IAM config %s: %s", cfg.iam_config_path, e)
    audit = None
    if cfg.audit_enabled and audit_sink is not None:
        audit = audit_sink(registry)
    elif cfg.audit_enabled:
        if cfg.audit_hmac_secret and len(cfg.audit_hmac_secret) >= 16:
            audit = AuditLogger(cfg.audit_dir, cfg.audit_retention_days, cfg.audit_batch_size,
                                cfg.audit_hmac_secret, registry=registry)
        else:
            log.warning("audit logging disabled: AUDIT_HMAC_SECRET must be set and at least 16 characters")
    sse = None
    if cfg.sse_master_key:
        try:
            sse = SseManager(parse_sse_master_key(cfg.sse_master_key))
        except ValueError as e:
            log.error("SSE disabled: %s", e)
    return S3Gateway(client, cfg, registry=registry, oidc=oidc, sts=sts, iam=iam, audit=audit, sse=sse)


def _die_with_parent() -> None:
    try:
        import ctypes

        ctypes.CDLL("libc.so.6", use_errno=True).prctl(1, signal.SIGTERM)  # PR_SET_PDEATHSIG
    except OSError:
        pass


def native_front_wanted(cfg: S3Config) -> bool:
    """The native front end (csrc/s3_front.cpp) serves the object data path. Co-located with a
    chunkserver its native client moves bodies through that server's pinned shared memory; a
    gateway on another host (no LOCAL_CHUNKSERVER) gives it a RemoteFrontStore, which speaks
    gRPC to the masters and chunkservers (csrc/front_store.h). It terminates TLS itself
    (TLS_CERT / TLS_KEY, OpenSSL), like the reference binds rustls directly (main.rs:263-274);
    the aiohttp workers behind it then listen on a private UNIX socket in plain HTTP."""
    if cfg.env.get("S3_NATIVE_FRONT", "true") != "true":
        return False
    try:
        from rust_hadoop_generated_by_llm_amd.native import lib  # noqa: F401
    except Exception:  # noqa: BLE001 - no extension: the Python gateway serves everything
        return False
    return True


def native_front_auth(gw: S3Gateway) -> dict:
    """What the native front needs to verify STS-session requests itself: the token keys by
    KID and the IAM role document (only when the gateway loaded it)."""
    out: dict = {"sts_keys": dict(gw.sts.keys) if gw.sts is not None else {}, "iam_config": ""}
    if gw.iam is not None and gw.cfg.iam_config_path:
        with open(gw.cfg.iam_config_path) as f:
            out["iam_config"] = f.read()
    return out


def start_native_front(gw: S3Gateway, host: str, port: int, backend: str, audit_socket: str,
                       policy_epoch: str = ""):
    """Worker 0 runs the native front on the public port; it hands what it does not serve to
    the aiohttp workers on `backend` and sends its audit records to `audit_socket`."""
    from rust_hadoop_generated_by_llm_amd.native import lib

    cfg = gw.cfg
    creds = gw.creds
    store = gw.client._fast
    if store is None:
        # not co-located: private slots, every master / chunkserver call over gRPC (TLS when
        # the gateway's client uses it), routed by the gateway client's shard map
        store = lib.RemoteFrontStore("", [], slots=int(cfg.env.get("S3_FRONT_SLOTS", "32") or 32),
                                     slot_bytes=int(cfg.env.get("S3_FRONT_SLOT_MB", "16") or 16) << 20,
                                     ca_cert=cfg.ca_cert or "", domain_name=cfg.domain_name or "",
                                     tls=bool(gw.client.tls))
        gw.client.add_native_routing(store)
        gw.front_store = store
    front = lib.S3Front(store, host, port, backend,
                        workers=int(cfg.env.get("S3_FRONT_THREADS", "32") or 32),
                        auth_enabled=cfg.auth_enabled, region=cfg.region,
                        access_key=getattr(creds, "access_key", None) or "",
                        secret_key=getattr(creds, "secret_key", None) or "",
                        allow_unsigned_payload=cfg.allow_unsigned_payload,
                        audit_socket=audit_socket if (cfg.auth_enabled and gw.audit is not None) else "",
                        sse_enabled=gw.sse is not None, metadata_sidecar=cfg.metadata_sidecar,
                        policy_epoch=policy_epoch or (gw.policy_epoch.path or ""),
                        tls_cert=cfg.tls_cert or "" if (cfg.tls_cert and cfg.tls_key) else "",
                        tls_key=cfg.tls_key or "" if (cfg.tls_cert and cfg.tls_key) else "",
                        sse_kek=gw.sse.kek if gw.sse is not None else b"",
                        require_tls=cfg.require_tls, **native_front_auth(gw))
    ok, err = front.start()
    if not ok:
        raise RuntimeError(f"native S3 front end failed to start: {err}")
    gw.front = front
    if gw.client._fast is None:
        log.info("native front end for a gateway without a co-located chunkserver: gRPC to masters and chunkservers")
    return front


def main(argv: list[str] | None = None) -> int:
    """One listening socket shared by S3_WORKERS processes (default 4), forked before any
    gRPC channel or thread exists; each runs its own event loop and DFS client, so request
    handling scales past one interpreter lock. Worker 0 owns the audit store.

    Co-located with a chunkserver (LOCAL_CHUNKSERVER), worker 0 also runs the native front
    end on the public port and the workers' shared socket becomes a private UNIX socket that
    only the front hands requests to (S3_NATIVE_FRONT=false keeps the Python-only layout)."""
    ap = argparse.ArgumentParser(prog="s3_server", description="S3-compatible gateway over the DFS")
    ap.add_argument("--port", type=int, default=None)
    ap.add_argument("--host", default="0.0.0.0")
    ap.add_argument("--workers", type=int, default=None)
    a = ap.parse_args(argv)
    logging.basicConfig(level=os.environ.get("LOG_LEVEL", "INFO"),
                        format="%(asctime)s %(levelname)s %(name)s %(message)s")
    cfg = S3Config()
    if a.port is not None:
        cfg.port = a.port
    workers = max(1, a.workers if a.workers is not None else int(os.environ.get("S3_WORKERS", "4") or 4))
    native = native_front_wanted(cfg)
    private_dir = tempfile.mkdtemp(prefix="s3gw-")
    backend_path = os.path.join(private_dir, "backend.sock")
    if native:
        lsock = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
        lsock.bind(backend_path)
    else:
        lsock = socket.socket(socket.AF_INET6 if ":" in a.host else socket.AF_INET, socket.SOCK_STREAM)
        lsock.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
        lsock.bind((a.host, cfg.port))
    lsock.listen(1024)
    ingest_path = ingest = None
    if (workers > 1 or native) and cfg.audit_enabled:
        ingest_path = os.path.join(private_dir, "ingest.sock")
        ingest = socket.socket(socket.AF_UNIX, socket.SOCK_DGRAM)
        ingest.bind(ingest_path)
        ingest.setsockopt(socket.SOL_SOCKET, socket.SO_RCVBUF, 8 << 20)
    epoch_path = os.path.join(private_dir, "policy_epoch")
    PolicyEpoch(epoch_path)  # created before the fork: every worker maps the same page
    children = []
    worker_id = 0
    for i in range(1, workers):
        pid = os.fork()
        if pid == 0:
            worker_id = i
            children = []
            _die_with_parent()
            if ingest is not None:
                ingest.close()
            break
        children.append(pid)
    sink = None
    if worker_id > 0 and ingest_path:
        sink = lambda reg: ForwardingAudit(ingest_path, reg)  # noqa: E731
    gw = build_gateway(cfg, audit_sink=sink)
    gw.policy_epoch = PolicyEpoch(epoch_path)
    gw._policy_epoch_seen = gw.policy_epoch.get()
    if worker_id == 0 and ingest is not None and gw.audit is not None:
        if hasattr(gw.audit, "start_ingest"):  # native writer: a C++ thread receives the datagrams
            gw.audit.start_ingest(ingest)
        else:
            threading.Thread(target=_audit_ingest, args=(ingest, gw.audit), name="audit-ingest",
                             daemon=True).start()
    ssl_ctx = None
    if cfg.tls_cert and cfg.tls_key and not native:  # with the front, TLS ends there
        ssl_ctx = ssl.create_default_context(ssl.Purpose.CLIENT_AUTH)
        ssl_ctx.load_cert_chain(cfg.tls_cert, cfg.tls_key)
    front = None
    if worker_id == 0 and native:
        front = start_native_front(gw, a.host, cfg.port, backend_path, ingest_path or "", epoch_path)
    if worker_id == 0:
        log.info("S3 gateway on %s:%d (workers=%d, auth=%s, sse=%s, audit=%s, native front=%s)", a.host, cfg.port,
                 workers, cfg.auth_enabled, gw.sse is not None, gw.audit is not None, front is not None)
    ready = os.environ.get("DFS_READY_FILE") if worker_id == 0 else None

    async def on_start(_app):
        if ready:
            with open(ready, "w") as f:
                json.dump({"port": cfg.port, "workers": workers, "native_front": front is not None}, f)
    app = gw.app()
    app.on_startup.append(on_start)
    try:
        web.run_app(app, sock=lsock, ssl_context=ssl_ctx, print=None, access_log=None)
    finally:
        if front is not None:
            front.stop()
        for pid in children:
            try:
                os.kill(pid, signal.SIGTERM)
            except ProcessLookupError:
                pass
        for pid in children:
            try:
                os.waitpid(pid, 0)
            except ChildProcessError:
                pass
        if worker_id == 0:
            shutil.rmtree(private_dir, ignore_errors=True)
    if worker_id > 0:
        os._exit(0)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())

