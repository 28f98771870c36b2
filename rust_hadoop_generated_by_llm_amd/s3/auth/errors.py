"""S3 authentication errors and their wire mapping.

Same code/message/HTTP-status table as the reference (dfs/common/src/auth/mod.rs:39-108,
s3_server/src/auth_middleware.rs:367-392 for the status codes, :806-819 for the metric
``error_type`` label).
"""
from __future__ import annotations

from xml.sax.saxutils import escape

_TABLE = {
    # kind: (S3 code, message, HTTP status, metric error_type)
    "missing_auth": ("AccessDenied", "Access Denied", 403, "missing_auth"),
    "invalid_access_key": ("InvalidAccessKeyId",
                           "The AWS Access Key Id you provided does not exist in our records.", 403,
                           "invalid_access_key"),
    "signature_mismatch": ("SignatureDoesNotMatch",
                           "The request signature we calculated does not match the signature you provided.",
                           403, "signature_mismatch"),
    "clock_skew": ("RequestTimeTooSkewed",
                   "The difference between the request time and the current time is too large.", 403,
                   "clock_skew"),
    "invalid_scope": ("AuthorizationHeaderMalformed",
                      "The authorization header is malformed; the region or service is wrong.", 400,
                      "invalid_credential_scope"),
    "insecure_transport": ("AccessDenied", "Access Denied (Insecure Transport)", 403, "insecure_transport"),
    "invalid_token": ("InvalidTokenId", "The security token included in the request is invalid.", 403,
                      "invalid_token"),
    "expired_token": ("ExpiredToken", "The provided token has expired.", 403, "expired_token"),
    "internal": ("InternalError", "An internal error occurred during authentication.", 500, "internal_error"),
}


class AuthError(Exception):
    def __init__(self, kind: str, detail: str = ""):
        if kind not in _TABLE:
            raise ValueError(f"unknown auth error kind {kind}")
        super().__init__(f"{kind}: {detail}" if detail else kind)
        self.kind = kind
        self.detail = detail

    @property
    def code(self) -> str:
        return _TABLE[self.kind][0]

    @property
    def message(self) -> str:
        return _TABLE[self.kind][1]

    @property
    def status(self) -> int:
        return _TABLE[self.kind][2]

    @property
    def error_type(self) -> str:
        return _TABLE[self.kind][3]

    def xml(self) -> str:
        return ('<?xml version="1.0" encoding="UTF-8"?>\n<Error>\n'
                f"  <Code>{escape(self.code)}</Code>\n  <Message>{escape(self.message)}</Message>\n"
                "  <Resource>/</Resource>\n</Error>")
