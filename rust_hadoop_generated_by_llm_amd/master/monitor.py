"""Per-prefix request-rate monitor driving dynamic sharding (C31; reference
dfs/metaserver/src/master.rs:610-675). Requests are counted by first path component
("/x/"); every 5 s the counters fold into an EMA (0.3 old, 0.7 new)."""
from __future__ import annotations

import threading
import time
from dataclasses import dataclass


@dataclass
class PrefixMetrics:
    rps: float = 0.0
    bps: float = 0.0
    last_count: int = 0
    last_bytes: int = 0


def path_prefix(path: str) -> str:
    for part in path.split("/"):
        if part:
            return f"/{part}/"
    return "/"


class ThroughputMonitor:
    def __init__(self, split_threshold_rps: float = 100.0, merge_threshold_rps: float = 1.0,
                 split_cooldown_secs: int = 30, window_secs: float = 5.0):
        self.metrics: dict[str, PrefixMetrics] = {}
        self.split_threshold_rps = split_threshold_rps
        self.merge_threshold_rps = merge_threshold_rps
        self.split_cooldown_secs = split_cooldown_secs
        self.window = window_secs
        self.last_split_time = time.monotonic() - split_cooldown_secs
        self._lock = threading.Lock()
        self.source = None  # callable -> {prefix: count}: requests counted by the native handlers

    def record_request(self, path: str, nbytes: int = 0) -> None:
        p = path_prefix(path)
        with self._lock:
            m = self.metrics.get(p)
            if m is None:
                m = self.metrics[p] = PrefixMetrics()
            m.last_count += 1
            m.last_bytes += nbytes

    def decay_metrics(self) -> None:
        native_counts = self.source() if self.source is not None else {}
        with self._lock:
            for p, n in native_counts.items():
                m = self.metrics.get(p)
                if m is None:
                    m = self.metrics[p] = PrefixMetrics()
                m.last_count += n
            for m in self.metrics.values():
                m.rps = m.rps * 0.3 + (m.last_count / self.window) * 0.7
                m.bps = m.bps * 0.3 + (m.last_bytes / self.window) * 0.7
                m.last_count = 0
                m.last_bytes = 0

    def rps_per_prefix(self) -> dict[str, float]:
        with self._lock:
            return {p: m.rps for p, m in self.metrics.items()}

    def hot_prefix(self) -> tuple[str, float] | None:
        if time.monotonic() - self.last_split_time < self.split_cooldown_secs:
            return None
        with self._lock:
            for p, m in self.metrics.items():
                if m.rps > self.split_threshold_rps:
                    return p, m.rps
        return None

    def total_rps(self) -> float:
        with self._lock:
            return sum(m.rps for m in self.metrics.values())
