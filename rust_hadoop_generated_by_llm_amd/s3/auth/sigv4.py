"""AWS Signature Version 4: verification (server) and signing (client/CLI).

Behavioural parity with the reference:
* credential parsing from the ``Authorization`` header or presigned query parameters
  (dfs/common/src/auth/mod.rs:110-221);
* canonical request / string-to-sign / signing-key derivation / constant-time compare
  (auth/signing.rs:9-123);
* RFC 3986 ``uri_encode`` (auth/encoding.rs:1-20);
* canonical query normalisation that drops ``X-Amz-Signature`` and sorts by (key, value)
  on the *raw* pairs (s3_server/src/auth_middleware.rs:676-716);
* signing-key LRU cache keyed by (access key, date), 100 entries, 24 h TTL (auth/cache.rs);
* aws-chunked payload chain verification (auth/chunked.rs:1-60) and decoding
  (s3_server/src/handlers.rs:291-320);
* presigned URL generation (auth/presign.rs:17-88).

URI encoding, query normalisation, the canonical request, the signing-key chain and the
constant-time signature check run natively (csrc/sigv4.cpp on OpenSSL); the aws-chunked
chain and the client-side helpers use :mod:`hashlib`/:mod:`hmac`.
"""
from __future__ import annotations

import hashlib
import hmac
import threading
import time
from collections import OrderedDict
from dataclasses import dataclass, field
from datetime import datetime, timezone
from urllib.parse import parse_qsl, unquote

from ...native import lib as _native
from .errors import AuthError

ALGORITHM = "AWS4-HMAC-SHA256"
UNSIGNED_PAYLOAD = "UNSIGNED-PAYLOAD"
EMPTY_SHA256 = "e3b0c44298fc1c149afbf4c8996fb92427ae41e4649b934ca495991b7852b855"
MAX_PRESIGN_EXPIRES = 604_800
MAX_SKEW_MINUTES = 15

@dataclass
class ParsedCredentials:
    access_key: str
    date: str
    region: str
    service: str
    signed_headers: list[str]
    signature: str
    timestamp: str

    @property
    def scope(self) -> str:
        return f"{self.date}/{self.region}/{self.service}/aws4_request"


@dataclass
class SigningInput:
    method: str
    path: str
    query_string: str
    headers: "OrderedDict[str, list[str]]" = field(default_factory=OrderedDict)
    signed_headers_list: str = ""
    payload_hash: str = UNSIGNED_PAYLOAD


def uri_encode(s: str, encode_slash: bool = True) -> str:
    return _native.sigv4_uri_encode(s, encode_slash)


def _split_cred(cred: str) -> list[str]:
    parts = cred.split("/")
    if len(parts) < 5 or parts[4] != "aws4_request":
        raise AuthError("missing_auth", "malformed credential scope")
    return parts


def parse_credentials(headers, query: dict[str, str]) -> ParsedCredentials:
    """``headers`` is any case-insensitive mapping with ``.get`` (aiohttp CIMultiDict)."""
    auth = headers.get("Authorization")
    if auth is not None:
        if not auth.startswith(ALGORITHM):
            raise AuthError("missing_auth", "unsupported authorization scheme")
        parts = [p.strip() for p in auth.split(",")]
        if len(parts) < 3:
            raise AuthError("missing_auth", "malformed authorization header")
        cred_entry = next((t for t in parts[0].split() if t.startswith("Credential=")), None)
        if cred_entry is None:
            raise AuthError("missing_auth", "missing Credential")
        cred = _split_cred(cred_entry.split("=", 1)[1])
        try:
            sh = parts[1].split("=", 1)[1].strip()
            sig = parts[2].split("=", 1)[1].strip()
        except IndexError as e:
            raise AuthError("missing_auth", "malformed authorization header") from e
        ts = headers.get("x-amz-date") or headers.get("Date")
        if ts is None:
            raise AuthError("missing_auth", "missing x-amz-date")
        return ParsedCredentials(cred[0], cred[1], cred[2], cred[3],
                                 [h.strip() for h in sh.split(";") if h.strip()], sig, ts)
    algo = query.get("X-Amz-Algorithm")
    if algo is not None:
        if algo != ALGORITHM:
            raise AuthError("missing_auth", "unsupported algorithm")
        try:
            cred = _split_cred(query["X-Amz-Credential"])
            sh = query["X-Amz-SignedHeaders"]
            sig = query["X-Amz-Signature"]
            ts = query["X-Amz-Date"]
        except KeyError as e:
            raise AuthError("missing_auth", f"missing {e.args[0]}") from e
        return ParsedCredentials(cred[0], cred[1], cred[2], cred[3], sh.split(";"), sig, ts)
    raise AuthError("missing_auth", "no credentials")


def parse_query(raw: str) -> dict[str, str]:
    return dict(parse_qsl(raw, keep_blank_values=True))


def normalize_query_string(raw: str) -> str:
    return _native.sigv4_normalize_query(raw)


def _canon_headers(inp: SigningInput) -> list[tuple[str, str]]:
    return [(name, ",".join(values)) for name, values in inp.headers.items()]


def canonical_request(inp: SigningInput) -> str:
    return _native.sigv4_canonical_request(inp.method, inp.path, inp.query_string, _canon_headers(inp),
                                           inp.signed_headers_list, inp.payload_hash)


def string_to_sign(timestamp: str, scope: str, creq: str) -> str:
    return f"{ALGORITHM}\n{timestamp}\n{scope}\n{hashlib.sha256(creq.encode()).hexdigest()}"


def derive_signing_key(secret: str, date: str, region: str, service: str) -> bytes:
    return _native.sigv4_signing_key(secret, date, region, service)


def calculate_signature(signing_key: bytes, sts: str) -> str:
    return _native.sigv4_signature(signing_key, sts)


def verify_signature_with_key(inp: SigningInput, cred: ParsedCredentials, signing_key: bytes) -> None:
    ok, creq = _native.sigv4_verify(inp.method, inp.path, inp.query_string, _canon_headers(inp),
                                    inp.signed_headers_list, inp.payload_hash, cred.timestamp, cred.scope,
                                    signing_key, cred.signature)
    if not ok:
        raise AuthError("signature_mismatch", f"canonical request:\n{creq}")


def verify_signature(inp: SigningInput, cred: ParsedCredentials, secret: str) -> None:
    verify_signature_with_key(inp, cred, derive_signing_key(secret, cred.date, cred.region, cred.service))


def build_signing_input(method: str, raw_path: str, normalized_query: str, headers, cred: ParsedCredentials
                        ) -> SigningInput:
    """Canonical headers from the request: every value whitespace-collapsed, duplicates
    comma-joined, names lower-cased and sorted (auth_middleware.rs:676-716)."""
    names = sorted({h.lower() for h in cred.signed_headers})
    canon: OrderedDict[str, list[str]] = OrderedDict()
    for n in names:
        vals = [" ".join(v.split()) for v in headers.getall(n, [])] if hasattr(headers, "getall") else \
            ([" ".join(headers[n].split())] if n in headers else [])
        canon[n] = [",".join(vals)]
    payload = headers.get("x-amz-content-sha256") or UNSIGNED_PAYLOAD
    return SigningInput(method, raw_path, normalized_query, canon, ";".join(names), payload)


def parse_amz_time(ts: str) -> datetime | None:
    for fmt in ("%Y%m%dT%H%M%SZ",):
        try:
            return datetime.strptime(ts, fmt).replace(tzinfo=timezone.utc)
        except ValueError:
            pass
    try:
        d = datetime.fromisoformat(ts.replace("Z", "+00:00"))
        return d if d.tzinfo else d.replace(tzinfo=timezone.utc)
    except ValueError:
        return None


def presigned_is_expired(ts: str, expires_secs: int, now: datetime | None = None) -> bool:
    t = parse_amz_time(ts)
    if t is None:
        return True
    now = now or datetime.now(timezone.utc)
    age = (now - t).total_seconds()
    # a URL dated more than the 15-minute clock-skew window ahead is not valid yet (and would
    # otherwise outlive the 7-day cap)
    return age > expires_secs or -age > 15 * 60


class SigningKeyCache:
    """LRU of derived signing keys keyed by (access key, date); 24 h TTL (auth/cache.rs)."""

    def __init__(self, capacity: int = 100, ttl: float = 86400.0):
        self.capacity = max(1, capacity)
        self.ttl = ttl
        self._d: OrderedDict[tuple[str, str], tuple[bytes, float]] = OrderedDict()
        self._lock = threading.Lock()

    def get(self, access_key: str, date: str) -> bytes | None:
        k = (access_key, date)
        with self._lock:
            e = self._d.get(k)
            if e is None:
                return None
            if e[1] <= time.monotonic():
                del self._d[k]
                return None
            self._d.move_to_end(k)
            return e[0]

    def insert(self, access_key: str, date: str, key: bytes) -> None:
        with self._lock:
            self._d[(access_key, date)] = (key, time.monotonic() + self.ttl)
            self._d.move_to_end((access_key, date))
            while len(self._d) > self.capacity:
                self._d.popitem(last=False)

    def __len__(self) -> int:
        return len(self._d)


class ChunkVerifier:
    """Per-chunk signature chain of ``STREAMING-AWS4-HMAC-SHA256-PAYLOAD`` bodies."""

    def __init__(self, signing_key: bytes, timestamp: str, scope: str, seed_signature: str):
        self.key, self.ts, self.scope, self.prev = signing_key, timestamp, scope, seed_signature

    def expected(self, chunk: bytes) -> str:
        sts = (f"{ALGORITHM}-PAYLOAD\n{self.ts}\n{self.scope}\n{self.prev}\n{EMPTY_SHA256}\n"
               f"{hashlib.sha256(chunk).hexdigest()}")
        return calculate_signature(self.key, sts)

    def verify_chunk(self, chunk: bytes, signature: str) -> bool:
        exp = self.expected(chunk)
        if len(exp) == len(signature) and hmac.compare_digest(exp.encode(), signature.encode()):
            self.prev = exp
            return True
        return False


class ChunkedDecodeError(ValueError):
    pass


def decode_chunked(body: bytes, verifier: ChunkVerifier | None = None) -> bytes:
    """Decode an aws-chunked body (``<hex>[;chunk-signature=<sig>]\\r\\n<data>\\r\\n``...,
    terminated by a zero-size chunk and optional trailers). With a verifier every chunk
    signature, including the final empty chunk's, must chain correctly."""
    out = bytearray()
    pos = 0
    n = len(body)
    mv = memoryview(body)
    final = False
    while pos < n:
        eol = body.find(b"\r\n", pos)
        if eol < 0:
            break
        header = bytes(mv[pos:eol]).decode("latin-1")
        size_s, _, ext = header.partition(";")
        try:
            size = int(size_s.strip() or "0", 16)
        except ValueError as e:
            raise ChunkedDecodeError(f"bad chunk header {header!r}") from e
        pos = eol + 2
        if size > n - pos:
            raise ChunkedDecodeError("truncated chunk")
        chunk = mv[pos:pos + size]
        if verifier is not None:
            sig = ext.split("chunk-signature=", 1)[1].strip() if "chunk-signature=" in ext else ""
            if not verifier.verify_chunk(bytes(chunk), sig):
                raise ChunkedDecodeError("chunk signature mismatch")
        if size == 0:
            final = True
            break
        out += chunk
        pos += size + 2
    if verifier is not None and not final:  # a signed stream ends with its signed empty chunk
        raise ChunkedDecodeError("chunk signature chain ends early")
    return bytes(out)


# ---------------------------------------------------------------------------- client side
def amz_now() -> tuple[str, str]:
    now = datetime.now(timezone.utc)
    return now.strftime("%Y%m%d"), now.strftime("%Y%m%dT%H%M%SZ")


def canonical_query_from_params(params: list[tuple[str, str]]) -> str:
    enc = sorted((uri_encode(k), uri_encode(v)) for k, v in params)
    return "&".join(f"{k}={v}" for k, v in enc)


def object_path(bucket: str, key: str = "") -> str:
    p = "/" + uri_encode(bucket)
    if key:
        p += "/" + "/".join(uri_encode(seg) for seg in key.split("/"))
    return p


def generate_presigned_url(endpoint: str, bucket: str, key: str, method: str, access_key: str, secret_key: str,
                           region: str = "us-east-1", expires_secs: int = 3600, *, now: tuple[str, str] | None = None
                           ) -> str:
    date, dt = now or amz_now()
    scope = f"{date}/{region}/s3/aws4_request"
    params = [("X-Amz-Algorithm", ALGORITHM), ("X-Amz-Credential", f"{access_key}/{scope}"),
              ("X-Amz-Date", dt), ("X-Amz-Expires", str(expires_secs)), ("X-Amz-SignedHeaders", "host")]
    cq = canonical_query_from_params(params)
    host = endpoint.split("://", 1)[-1].rstrip("/")
    path = object_path(bucket, key)
    inp = SigningInput(method.upper(), path, cq, OrderedDict(host=[host]), "host", UNSIGNED_PAYLOAD)
    sig = calculate_signature(derive_signing_key(secret_key, date, region, "s3"),
                              string_to_sign(dt, scope, canonical_request(inp)))
    return f"{endpoint.rstrip('/')}{path}?{cq}&X-Amz-Signature={sig}"


def sign_headers(method: str, url_path: str, query: list[tuple[str, str]] | str, host: str, body: bytes | None,
                 access_key: str, secret_key: str, region: str = "us-east-1", *, extra_headers: dict | None = None,
                 unsigned_payload: bool = False, session_token: str | None = None,
                 now: tuple[str, str] | None = None) -> dict[str, str]:
    """Headers (Authorization, x-amz-date, x-amz-content-sha256, ...) for a header-signed
    request; ``url_path`` must already be URI-encoded exactly as it is sent."""
    date, dt = now or amz_now()
    payload = UNSIGNED_PAYLOAD if unsigned_payload else hashlib.sha256(body or b"").hexdigest()
    hdrs = {"host": host, "x-amz-date": dt, "x-amz-content-sha256": payload}
    if session_token:
        hdrs["x-amz-security-token"] = session_token
    for k, v in (extra_headers or {}).items():
        hdrs[k.lower()] = v
    names = sorted(hdrs)
    canon = OrderedDict((n, [" ".join(str(hdrs[n]).split())]) for n in names)
    cq = canonical_query_from_params(query) if isinstance(query, list) else normalize_query_string(query)
    inp = SigningInput(method.upper(), url_path, cq, canon, ";".join(names), payload)
    scope = f"{date}/{region}/s3/aws4_request"
    sig = calculate_signature(derive_signing_key(secret_key, date, region, "s3"),
                              string_to_sign(dt, scope, canonical_request(inp)))
    out = {k: v for k, v in hdrs.items() if k != "host"}
    out["Authorization"] = (f"{ALGORITHM} Credential={access_key}/{scope}, SignedHeaders={';'.join(names)}, "
                            f"Signature={sig}")
    return out


def encode_chunked(data: bytes, chunk_size: int, signing_key: bytes, timestamp: str, scope: str,
                   seed_signature: str) -> bytes:
    """Client-side aws-chunked encoder (test helper / SDK parity)."""
    v = ChunkVerifier(signing_key, timestamp, scope, seed_signature)
    out = bytearray()
    chunks = [data[i:i + chunk_size] for i in range(0, len(data), chunk_size)] + [b""]
    for c in chunks:
        sig = v.expected(c)
        v.prev = sig
        out += f"{len(c):x};chunk-signature={sig}\r\n".encode() + c + b"\r\n"
    return bytes(out)


def unquote_path(p: str) -> str:
    return unquote(p)
