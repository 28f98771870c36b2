"""Minimal Prometheus text-exposition registry (counters, gauges, histograms) shared by
master, chunkserver and S3 gateway ``/metrics`` endpoints (reference: prometheus crate
registries in bin/master.rs:280-350, bin/chunkserver.rs:381-428, s3_server main.rs:30-36)."""
from __future__ import annotations

import bisect
import threading
from typing import Callable


def _labels(names: tuple[str, ...], values: tuple[str, ...]) -> str:
    if not names:
        return ""
    inner = ",".join(f'{n}="{str(v).replace(chr(92), chr(92) * 2).replace(chr(34), chr(92) + chr(34))}"'
                     for n, v in zip(names, values))
    return "{" + inner + "}"


class _Metric:
    kind = "untyped"

    def __init__(self, name: str, help_: str, labels: tuple[str, ...] = ()):
        self.name, self.help, self.label_names = name, help_, tuple(labels)
        self._lock = threading.Lock()
        self._values: dict[tuple[str, ...], float] = {}

    def _key(self, labels: dict | None) -> tuple[str, ...]:
        labels = labels or {}
        return tuple(str(labels.get(n, "")) for n in self.label_names)

    def render(self) -> list[str]:
        out = [f"# HELP {self.name} {self.help}", f"# TYPE {self.name} {self.kind}"]
        with self._lock:
            for k, v in sorted(self._values.items()):
                out.append(f"{self.name}{_labels(self.label_names, k)} {v:g}")
        return out


class Counter(_Metric):
    kind = "counter"

    def inc(self, amount: float = 1.0, labels: dict | None = None) -> None:
        k = self._key(labels)
        with self._lock:
            self._values[k] = self._values.get(k, 0.0) + amount

    def get(self, labels: dict | None = None) -> float:
        return self._values.get(self._key(labels), 0.0)


class Gauge(_Metric):
    kind = "gauge"

    def __init__(self, name, help_, labels=(), fn: Callable[[], float] | None = None):
        super().__init__(name, help_, labels)
        self._fn = fn

    def set(self, value: float, labels: dict | None = None) -> None:
        with self._lock:
            self._values[self._key(labels)] = float(value)

    def render(self) -> list[str]:
        if self._fn is not None:
            try:
                self.set(self._fn())
            except Exception:  # noqa: BLE001
                pass
        return super().render()


class Histogram(_Metric):
    kind = "histogram"
    DEFAULT = (0.0005, 0.001, 0.0025, 0.005, 0.01, 0.025, 0.05, 0.1, 0.25, 0.5, 1.0, 2.5, 5.0, 10.0)

    def __init__(self, name, help_, labels=(), buckets=DEFAULT):
        super().__init__(name, help_, labels)
        self.buckets = tuple(buckets)
        self._h: dict[tuple[str, ...], list] = {}

    def observe(self, v: float, labels: dict | None = None) -> None:
        k = self._key(labels)
        with self._lock:
            st = self._h.setdefault(k, [[0] * len(self.buckets), 0.0, 0])
            i = bisect.bisect_left(self.buckets, v)
            if i < len(self.buckets):
                st[0][i] += 1
            st[1] += v
            st[2] += 1

    def render(self) -> list[str]:
        out = [f"# HELP {self.name} {self.help}", f"# TYPE {self.name} histogram"]
        with self._lock:
            for k, (counts, total, n) in sorted(self._h.items()):
                cum = 0
                for b, c in zip(self.buckets, counts):
                    cum += c
                    lab = _labels(self.label_names + ("le",), k + (f"{b:g}",))
                    out.append(f"{self.name}_bucket{lab} {cum}")
                out.append(f"{self.name}_bucket{_labels(self.label_names + ('le',), k + ('+Inf',))} {n}")
                out.append(f"{self.name}_sum{_labels(self.label_names, k)} {total:g}")
                out.append(f"{self.name}_count{_labels(self.label_names, k)} {n}")
        return out


class Registry:
    def __init__(self):
        self._metrics: list[_Metric] = []

    def add(self, m: _Metric) -> _Metric:
        self._metrics.append(m)
        return m

    def counter(self, name, help_, labels=()):
        return self.add(Counter(name, help_, labels))

    def gauge(self, name, help_, labels=(), fn=None):
        return self.add(Gauge(name, help_, labels, fn))

    def histogram(self, name, help_, labels=(), buckets=Histogram.DEFAULT):
        return self.add(Histogram(name, help_, labels, buckets))

    def render(self) -> str:
        lines: list[str] = []
        for m in self._metrics:
            lines.extend(m.render())
        return "\n".join(lines) + "\n"
