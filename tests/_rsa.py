"""Tiny pure-Python RSA (keygen + PKCS#1 v1.5 SHA-256 signing) for OIDC test fixtures.

Stands in for the reference's mock OIDC issuer (test_scripts/mock_oidc.py) which uses the
``cryptography`` package — not installed here. Test-only; never use for real keys.
"""
from __future__ import annotations

import base64
import hashlib
import json
import random

_SHA256_PREFIX = bytes.fromhex("3031300d060960864801650304020105000420")


def _is_probable_prime(n: int, rnd: random.Random, rounds: int = 24) -> bool:
    if n < 2:
        return False
    for p in (2, 3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37):
        if n % p == 0:
            return n == p
    d, s = n - 1, 0
    while d % 2 == 0:
        d //= 2
        s += 1
    for _ in range(rounds):
        a = rnd.randrange(2, n - 2)
        x = pow(a, d, n)
        if x in (1, n - 1):
            continue
        for _ in range(s - 1):
            x = pow(x, 2, n)
            if x == n - 1:
                break
        else:
            return False
    return True


def _prime(bits: int, rnd: random.Random) -> int:
    while True:
        c = rnd.getrandbits(bits) | (1 << (bits - 1)) | (1 << (bits - 2)) | 1
        if _is_probable_prime(c, rnd):
            return c


def generate(bits: int = 2048, seed: int = 1234) -> tuple[int, int, int]:
    rnd = random.Random(seed)
    e = 65537
    while True:
        p, q = _prime(bits // 2, rnd), _prime(bits // 2, rnd)
        phi = (p - 1) * (q - 1)
        if p != q and phi % e != 0:
            n = p * q
            return n, e, pow(e, -1, phi)


def sign(msg: bytes, n: int, d: int) -> bytes:
    k = (n.bit_length() + 7) // 8
    t = _SHA256_PREFIX + hashlib.sha256(msg).digest()
    em = b"\x00\x01" + b"\xff" * (k - len(t) - 3) + b"\x00" + t
    return pow(int.from_bytes(em, "big"), d, n).to_bytes(k, "big")


def b64u(b: bytes) -> str:
    return base64.urlsafe_b64encode(b).rstrip(b"=").decode()


def int_b64u(i: int) -> str:
    return b64u(i.to_bytes((i.bit_length() + 7) // 8, "big"))


def jwk(n: int, e: int, kid: str) -> dict:
    return {"kty": "RSA", "kid": kid, "alg": "RS256", "use": "sig", "n": int_b64u(n), "e": int_b64u(e)}


def jwt_rs256(claims: dict, n: int, d: int, kid: str) -> str:
    h = b64u(json.dumps({"alg": "RS256", "typ": "JWT", "kid": kid}).encode())
    p = b64u(json.dumps(claims).encode())
    return f"{h}.{p}.{b64u(sign(f'{h}.{p}'.encode(), n, d))}"
