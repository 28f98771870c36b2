"""Logging setup. ``DFS_LOG`` (or the reference's ``RUST_LOG``) selects the level, e.g.
``DFS_LOG=debug`` or ``RUST_LOG=master=debug`` (reference: EnvFilter in every binary,
dfs/metaserver/src/bin/master.rs:101-107). Records carry the propagated request id."""
from __future__ import annotations

import logging
import os
import sys

from .rpc import current_request_id


class _RequestIdFilter(logging.Filter):
    def filter(self, record: logging.LogRecord) -> bool:
        record.request_id = current_request_id.get() or "-"
        return True


def _level_from_env(default: str) -> int:
    spec = os.environ.get("DFS_LOG") or os.environ.get("RUST_LOG") or default
    level = spec.split(",")[0].split("=")[-1].strip().upper()
    return getattr(logging, {"WARN": "WARNING", "TRACE": "DEBUG"}.get(level, level), logging.INFO)


def setup(name: str, default: str = "info") -> logging.Logger:
    root = logging.getLogger()
    if not getattr(root, "_dfs_configured", False):
        h = logging.StreamHandler(sys.stderr)
        h.setFormatter(logging.Formatter("%(asctime)s %(levelname)s %(name)s [req=%(request_id)s] %(message)s"))
        h.addFilter(_RequestIdFilter())
        root.addHandler(h)
        root.setLevel(_level_from_env(default))
        root._dfs_configured = True  # type: ignore[attr-defined]
    logging.getLogger("grpc").setLevel(logging.WARNING)
    logging.getLogger("aiohttp.access").setLevel(logging.WARNING)
    return logging.getLogger(name)
