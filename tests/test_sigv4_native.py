"""Native SigV4 (csrc/sigv4.cpp) against a plain-Python model of the reference algorithm
(dfs/common/src/auth/{signing,encoding}.rs, auth_middleware.rs:676-716): URI encoding,
query normalisation, canonical request, signing-key chain, signature, constant-time verify —
plus the AWS documentation example (GET /test.txt, examplebucket, 20130524)."""
import hashlib
import hmac

from hypothesis import given, settings
from hypothesis import strategies as st

from rust_hadoop_generated_by_llm_amd.native import lib

UNRESERVED = frozenset(b"ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789_.-~")


def py_uri_encode(s: str, encode_slash: bool) -> str:
    return "".join(chr(b) if b in UNRESERVED or (b == 0x2F and not encode_slash) else f"%{b:02X}"
                   for b in s.encode())


def py_normalize(raw: str) -> str:
    pairs = []
    for p in raw.split("&"):
        if not p or p == "X-Amz-Signature" or p.startswith("X-Amz-Signature="):
            continue
        k, _, v = p.partition("=")
        pairs.append((k, v))
    return "&".join(f"{k}={v}" for k, v in sorted(pairs))


def py_creq(method, path, query, headers, signed, payload):
    lines = [method, path, query] + [f"{n}:{v}" for n, v in headers]
    return "\n".join(lines) + "\n\n" + signed + "\n" + payload


def py_key(secret, date, region, service):
    k = ("AWS4" + secret).encode()
    for m in (date, region, service, "aws4_request"):
        k = hmac.new(k, m.encode(), hashlib.sha256).digest()
    return k


def py_sig(key, method, path, query, headers, signed, payload, ts, scope):
    creq = py_creq(method, path, query, headers, signed, payload)
    sts = f"AWS4-HMAC-SHA256\n{ts}\n{scope}\n{hashlib.sha256(creq.encode()).hexdigest()}"
    return hmac.new(key, sts.encode(), hashlib.sha256).hexdigest()


text = st.text(alphabet=st.characters(min_codepoint=32, max_codepoint=0x2FF), max_size=40)
token = st.text(alphabet="abcdefghijklmnopqrstuvwxyzABC0123456789-_.~%", min_size=1, max_size=12)


@settings(max_examples=200, deadline=None)
@given(text, st.booleans())
def test_uri_encode_matches(s, slash):
    assert lib.sigv4_uri_encode(s, slash) == py_uri_encode(s, slash)


@settings(max_examples=200, deadline=None)
@given(st.lists(st.tuples(token, st.one_of(st.none(), token)), max_size=8), st.booleans())
def test_normalize_query_matches(pairs, with_sig):
    parts = [k if v is None else f"{k}={v}" for k, v in pairs]
    if with_sig:
        parts.insert(len(parts) // 2, "X-Amz-Signature=deadbeef")
    raw = "&".join(parts)
    assert lib.sigv4_normalize_query(raw) == py_normalize(raw)


@settings(max_examples=150, deadline=None)
@given(st.sampled_from(["GET", "PUT", "HEAD", "DELETE", "POST"]), text, st.lists(st.tuples(token, token), max_size=5),
       token, token, token)
def test_sign_and_verify_match_the_model(method, path, hdrs, secret, payload, region):
    path = "/" + py_uri_encode(path, False)
    headers = sorted({(n.lower(), v) for n, v in hdrs} | {("host", "h:9000")})
    signed = ";".join(n for n, _ in headers)
    ts, date = "20240102T030405Z", "20240102"
    scope = f"{date}/{region}/s3/aws4_request"
    key = py_key(secret, date, region, "s3")
    assert lib.sigv4_signing_key(secret, date, region, "s3") == key
    query = py_normalize("b=2&a=1")
    assert lib.sigv4_canonical_request(method, path, query, headers, signed, payload) == \
        py_creq(method, path, query, headers, signed, payload)
    sig = py_sig(key, method, path, query, headers, signed, payload, ts, scope)
    ok, creq = lib.sigv4_verify(method, path, query, headers, signed, payload, ts, scope, key, sig)
    assert ok and creq == py_creq(method, path, query, headers, signed, payload)
    bad = sig[:-1] + ("0" if sig[-1] != "0" else "1")
    assert not lib.sigv4_verify(method, path, query, headers, signed, payload, ts, scope, key, bad)[0]
    assert not lib.sigv4_verify(method, path + "x", query, headers, signed, payload, ts, scope, key, sig)[0]
    assert not lib.sigv4_verify(method, path, query, headers, signed, payload, ts, scope, key, sig[:10])[0]


def test_aws_documentation_example():
    # "GET Object" example of the SigV4 documentation (header-based auth, Range header)
    secret = "wJalrXUtnFEMI/K7MDENG/bPxRfiCYEXAMPLEKEY"
    key = lib.sigv4_signing_key(secret, "20130524", "us-east-1", "s3")
    headers = [("host", "examplebucket.s3.amazonaws.com"), ("range", "bytes=0-9"),
               ("x-amz-content-sha256", "e3b0c44298fc1c149afbf4c8996fb92427ae41e4649b934ca495991b7852b855"),
               ("x-amz-date", "20130524T000000Z")]
    signed = "host;range;x-amz-content-sha256;x-amz-date"
    ok, _ = lib.sigv4_verify("GET", "/test.txt", "", headers, signed,
                             "e3b0c44298fc1c149afbf4c8996fb92427ae41e4649b934ca495991b7852b855",
                             "20130524T000000Z", "20130524/us-east-1/s3/aws4_request", key,
                             "f0e8bdb87c964420e857bd35b5d6ed310bd44f0170aba48dd91039c6036bdb41")
    assert ok
