"""Identity providers for the S3 gateway: static/env credentials, OIDC (JWT + JWKS),
STS session tokens and SSE envelope encryption.

* Credential providers (auth/credentials.rs): ``S3_ACCESS_KEY``/``S3_SECRET_KEY`` env pair,
  or a static pair (default ak/sk).
* ``OidcValidator`` (auth/oidc.rs:33-120): discovers ``jwks_uri`` from
  ``<issuer>/.well-known/openid-configuration``, caches the JWKS, refetches when a ``kid``
  is unknown, verifies RS256 signatures (OpenSSL via the native extension), ``aud`` ==
  client id, ``iss`` == issuer, ``exp`` (60 s leeway, like jsonwebtoken's default).
  HS256 ``oct`` keys are accepted only when ``allow_hs256`` is set (test fixtures, as the
  reference's ``#[cfg(test)]`` branch).
* ``StsTokenManager`` (auth/sts.rs): token = base64(kid_be32 || nonce12 || AES-256-GCM(
  JSON{role_arn, temp_secret_key, expiration, claims})), key ring by kid.
* ``SseManager`` (auth/sse.rs): per-object random DEK; object = nonce12 || GCM(DEK, data);
  DEK wrapped under the KEK as base64(nonce12 || GCM(KEK, DEK)).
"""
from __future__ import annotations

import base64
import hashlib
import hmac
import json
import os
import struct
import threading
import time
import urllib.request
from dataclasses import dataclass, field

from rust_hadoop_generated_by_llm_amd.native import lib
from rust_hadoop_generated_by_llm_amd.s3.auth.errors import AuthError
from tests.models.s3_policy import EvaluationContext


# ---------------------------------------------------------------------------- credentials
class EnvCredentialProvider:
    def __init__(self, env: dict | None = None):
        env = os.environ if env is None else env
        self.access_key = env.get("S3_ACCESS_KEY")
        self.secret_key = env.get("S3_SECRET_KEY")

    def get_secret_key(self, access_key: str) -> str | None:
        if self.access_key is not None and self.secret_key is not None and access_key == self.access_key:
            return self.secret_key
        return None


class StaticCredentialProvider:
    def __init__(self, access_key: str = "ak", secret_key: str = "sk"):
        self.access_key, self.secret_key = access_key, secret_key

    def get_secret_key(self, access_key: str) -> str | None:
        return self.secret_key if access_key == self.access_key else None


# ---------------------------------------------------------------------------- OIDC
def b64url_decode(s: str) -> bytes:
    return base64.urlsafe_b64decode(s + "=" * (-len(s) % 4))


def b64url_encode(b: bytes) -> str:
    return base64.urlsafe_b64encode(b).rstrip(b"=").decode()


@dataclass
class Claims:
    sub: str
    aud: str
    iss: str
    exp: int
    iat: int
    groups: list[str] = field(default_factory=list)
    extra: dict = field(default_factory=dict)

    @classmethod
    def from_json(cls, d: dict) -> "Claims":
        try:
            aud = d["aud"]
            if isinstance(aud, list):
                aud = aud[0] if aud else ""
            known = {"sub", "aud", "iss", "exp", "iat", "groups"}
            return cls(str(d["sub"]), str(aud), str(d["iss"]), int(d["exp"]), int(d["iat"]),
                       [str(g) for g in d.get("groups", [])], {k: v for k, v in d.items() if k not in known})
        except (KeyError, TypeError, ValueError) as e:
            raise AuthError("invalid_token", f"missing or invalid claim: {e}") from e

    def to_json(self) -> dict:
        d = dict(self.extra)
        d.update(sub=self.sub, aud=self.aud, iss=self.iss, exp=self.exp, iat=self.iat, groups=list(self.groups))
        return d

    def to_policy_context(self) -> EvaluationContext:
        return EvaluationContext(principal_id=self.sub, groups=list(self.groups),
                                 claims={"sub": self.sub, "iss": self.iss})


class OidcValidator:
    LEEWAY = 60

    def __init__(self, issuer_url: str, client_id: str, *, allow_hs256: bool = False, fetch_timeout: float = 5.0):
        self.issuer_url = issuer_url
        self.client_id = client_id
        self.allow_hs256 = allow_hs256
        self.fetch_timeout = fetch_timeout
        self._jwks: dict[str, dict] | None = None
        self._lock = threading.Lock()
        self.last_fetch = 0.0
        self.fetches = {"success": 0, "failure": 0}

    def _get_json(self, url: str) -> dict:
        with urllib.request.urlopen(url, timeout=self.fetch_timeout) as r:  # noqa: S310 (configured issuer)
            return json.loads(r.read())

    def fetch_jwks(self) -> None:
        try:
            conf = self._get_json(self.issuer_url.rstrip("/") + "/.well-known/openid-configuration")
            uri = conf.get("jwks_uri")
            if not uri:
                raise AuthError("internal", "missing jwks_uri in OIDC config")
            jwks = self._get_json(uri)
            keys = {k["kid"]: k for k in jwks.get("keys", []) if "kid" in k}
        except AuthError:
            self.fetches["failure"] += 1
            raise
        except Exception as e:  # noqa: BLE001
            self.fetches["failure"] += 1
            raise AuthError("internal", f"failed to fetch JWKS: {e}") from e
        with self._lock:
            self._jwks = keys
        self.fetches["success"] += 1
        self.last_fetch = time.time()

    def set_jwks(self, jwks: dict) -> None:
        with self._lock:
            self._jwks = {k["kid"]: k for k in jwks.get("keys", []) if "kid" in k}

    def _key(self, kid: str) -> dict:
        with self._lock:
            have = self._jwks is not None and kid in self._jwks
        if not have:
            try:
                self.fetch_jwks()
            except AuthError:
                pass
        with self._lock:
            if self._jwks is None:
                raise AuthError("internal", "JWKS is not available")
            k = self._jwks.get(kid)
        if k is None:
            raise AuthError("invalid_token", f"kid {kid} not found in JWKS")
        return k

    def validate_token(self, token: str, now: float | None = None) -> Claims:
        try:
            h64, p64, s64 = token.split(".")
            header = json.loads(b64url_decode(h64))
            payload = json.loads(b64url_decode(p64))
            sig = b64url_decode(s64)
        except (ValueError, json.JSONDecodeError) as e:
            raise AuthError("invalid_token", f"invalid JWT: {e}") from e
        kid = header.get("kid")
        if not kid:
            raise AuthError("invalid_token", "missing kid in JWT header")
        jwk = self._key(kid)
        alg = header.get("alg")
        msg = f"{h64}.{p64}".encode()
        if alg == "RS256" and jwk.get("kty") == "RSA":
            ok = lib.rsa_sha256_verify(b64url_decode(jwk["n"]), b64url_decode(jwk["e"]), msg, sig)
        elif alg == "HS256" and jwk.get("kty") == "oct" and self.allow_hs256:
            ok = hmac.compare_digest(hmac.new(b64url_decode(jwk["k"]), msg, hashlib.sha256).digest(), sig)
        else:
            raise AuthError("invalid_token", f"unsupported algorithm {alg}")
        if not ok:
            raise AuthError("invalid_token", "signature verification failed")
        now = time.time() if now is None else now
        aud = payload.get("aud")
        auds = aud if isinstance(aud, list) else [aud]
        if self.client_id not in auds:
            raise AuthError("invalid_token", "audience mismatch")
        if payload.get("iss") != self.issuer_url:
            raise AuthError("invalid_token", "issuer mismatch")
        if "exp" not in payload or float(payload["exp"]) + self.LEEWAY < now:
            raise AuthError("invalid_token", "token expired")
        if "nbf" in payload and float(payload["nbf"]) - self.LEEWAY > now:
            raise AuthError("invalid_token", "token not yet valid")
        return Claims.from_json(payload)


def make_hs256_jwt(claims: dict, secret: bytes, kid: str) -> str:
    """Mint an HS256 JWT (tests / local development issuers)."""
    h = b64url_encode(json.dumps({"alg": "HS256", "typ": "JWT", "kid": kid}).encode())
    p = b64url_encode(json.dumps(claims).encode())
    s = b64url_encode(hmac.new(secret, f"{h}.{p}".encode(), hashlib.sha256).digest())
    return f"{h}.{p}.{s}"


# ---------------------------------------------------------------------------- STS
@dataclass
class StsSessionData:
    role_arn: str
    temp_secret_key: str
    expiration: int
    claims: Claims

    def to_json(self) -> dict:
        return {"role_arn": self.role_arn, "temp_secret_key": self.temp_secret_key, "expiration": self.expiration,
                "claims": self.claims.to_json()}

    @classmethod
    def from_json(cls, d: dict) -> "StsSessionData":
        return cls(d["role_arn"], d["temp_secret_key"], int(d["expiration"]), Claims.from_json(d["claims"]))


def _key32(k: bytes | str) -> bytes:
    if isinstance(k, str):
        k = k.encode()
    return (k + b"\0" * 32)[:32]


class StsTokenManager:
    def __init__(self, keys: dict[int, bytes], active_kid: int):
        self.keys = {int(kid): _key32(k) for kid, k in keys.items()}
        self.active_kid = active_kid

    @classmethod
    def from_signing_key(cls, key: str) -> "StsTokenManager":
        return cls({1: key.encode()}, 1)

    def generate_token(self, data: StsSessionData) -> str:
        key = self.keys.get(self.active_kid)
        if key is None:
            raise AuthError("internal", f"active KID {self.active_kid} not found")
        nonce = lib.random_bytes(12)
        ct = lib.aes256gcm_encrypt(key, nonce, json.dumps(data.to_json()).encode(), b"")
        return base64.b64encode(struct.pack(">I", self.active_kid) + nonce + ct).decode()

    def decrypt_token(self, token: str) -> StsSessionData:
        try:
            raw = base64.b64decode(token, validate=True)
        except ValueError as e:
            raise AuthError("invalid_token", "invalid base64") from e
        if len(raw) < 16 + 16:
            raise AuthError("invalid_token", "token too short")
        (kid,) = struct.unpack(">I", raw[:4])
        key = self.keys.get(kid)
        if key is None:
            raise AuthError("invalid_token", f"unknown KID {kid}")
        try:
            pt = lib.aes256gcm_decrypt(key, raw[4:16], raw[16:], b"")
            return StsSessionData.from_json(json.loads(pt))
        except AuthError:
            raise
        except Exception as e:  # noqa: BLE001
            raise AuthError("invalid_token", f"decryption failed: {e}") from e


_ALNUM = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789"


def random_alnum(n: int) -> str:
    out = []
    while len(out) < n:
        for b in lib.random_bytes(2 * n):
            if b < 248:  # 248 = 4 * 62: unbiased
                out.append(_ALNUM[b % 62])
                if len(out) == n:
                    break
    return "".join(out)


# ---------------------------------------------------------------------------- SSE
def parse_sse_master_key(hex_str: str) -> bytes:
    b = bytes.fromhex(hex_str.strip())
    if len(b) != 32:
        raise ValueError("SSE_MASTER_KEY must be 32 bytes (64 hex chars)")
    return b


class SseManager:
    def __init__(self, kek: bytes):
        if len(kek) != 32:
            raise ValueError("KEK must be 32 bytes")
        self.kek = kek

    def encrypt_object(self, plaintext: bytes) -> tuple[bytes, str]:
        dek = lib.random_bytes(32)
        n1 = lib.random_bytes(12)
        ct = n1 + lib.aes256gcm_encrypt(dek, n1, plaintext, b"")
        n2 = lib.random_bytes(12)
        wrapped = n2 + lib.aes256gcm_encrypt(self.kek, n2, dek, b"")
        return ct, base64.b64encode(wrapped).decode()

    def decrypt_object(self, ciphertext: bytes, dek_b64: str) -> bytes:
        try:
            blob = base64.b64decode(dek_b64, validate=True)
        except ValueError as e:
            raise AuthError("invalid_token", "invalid base64 DEK") from e
        if len(blob) < 60:
            raise AuthError("invalid_token", "encrypted DEK too short")
        try:
            dek = lib.aes256gcm_decrypt(self.kek, blob[:12], blob[12:], b"")
        except Exception as e:  # noqa: BLE001
            raise AuthError("invalid_token", f"DEK decryption failed: {e}") from e
        if len(dek) != 32:
            raise AuthError("internal", "decrypted DEK has wrong length")
        if len(ciphertext) < 28:
            raise AuthError("invalid_token", "ciphertext too short")
        try:
            return lib.aes256gcm_decrypt(dek, ciphertext[:12], ciphertext[12:], b"")
        except Exception as e:  # noqa: BLE001
            raise AuthError("invalid_token", f"data decryption failed: {e}") from e
