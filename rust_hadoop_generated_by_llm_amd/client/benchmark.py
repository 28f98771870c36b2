"""``dfs_cli benchmark write|read|stress-write`` (reference dfs/client/src/bin/dfs_cli.rs:
581-807, print_stats :840-882). Same MB/s formula (count*size/2^20/secs) and latency
statistics, plus P50. Payloads are random bytes (the reference writes zeros)."""
from __future__ import annotations

import os
import threading
import time
from concurrent.futures import ThreadPoolExecutor
from dataclasses import dataclass, field


@dataclass
class Stats:
    name: str
    count: int
    avg_size: int
    total_s: float
    latencies: list[float] = field(default_factory=list)
    errors: int = 0

    def _pct(self, p: int) -> float:
        lat = sorted(self.latencies)
        if not lat:
            return 0.0
        return lat[min(len(lat) - 1, len(lat) * p // 100)]

    @property
    def mb_per_s(self) -> float:
        return (self.count * self.avg_size / (1024 * 1024)) / self.total_s if self.total_s > 0 else 0.0

    @property
    def ops_per_s(self) -> float:
        return self.count / self.total_s if self.total_s > 0 else 0.0

    def summary(self) -> dict:
        lat = sorted(self.latencies)
        return {
            "ops": self.count, "bytes": self.count * self.avg_size, "seconds": self.total_s,
            "mb_per_s": self.mb_per_s, "ops_per_s": self.ops_per_s, "errors": self.errors,
            "min_ms": 1e3 * (lat[0] if lat else 0), "avg_ms": 1e3 * (sum(lat) / len(lat) if lat else 0),
            "p50_ms": 1e3 * self._pct(50), "p95_ms": 1e3 * self._pct(95), "p99_ms": 1e3 * self._pct(99),
            "max_ms": 1e3 * (lat[-1] if lat else 0),
        }

    def format(self) -> str:
        s = self.summary()
        return "\n".join([
            f"\n📊 {self.name} Benchmark Results:",
            "----------------------------------------",
            f"Total Operations:  {self.count}",
            f"Total Time:        {self.total_s:.2f}s",
            f"Throughput:        {s['mb_per_s']:.2f} MB/s",
            f"Throughput (OPS):  {s['ops_per_s']:.2f} ops/s",
            "",
            "Latency Statistics:",
            f"  Min:  {s['min_ms']:.2f}ms",
            f"  Avg:  {s['avg_ms']:.2f}ms",
            f"  P50:  {s['p50_ms']:.2f}ms",
            f"  P95:  {s['p95_ms']:.2f}ms",
            f"  P99:  {s['p99_ms']:.2f}ms",
            f"  Max:  {s['max_ms']:.2f}ms",
            "----------------------------------------",
        ])


def make_payloads(n: int, size: int) -> list[bytes]:
    """Distinct random payloads, generated outside any timed region."""
    return [os.urandom(size) for _ in range(n)]


def bench_write(client, count: int = 100, size: int = 1 << 20, concurrency: int = 10, prefix: str = "bench_write",
                payloads: list[bytes] | None = None, run_id: str | None = None,
                pool: ThreadPoolExecutor | None = None) -> tuple[Stats, list[str]]:
    payloads = payloads or make_payloads(min(count, 64), size)
    run_id = run_id or str(int(time.time()))
    names = [f"{prefix}/{run_id}/bench_{i:010d}" for i in range(count)]
    lat: list[float] = []
    lock = threading.Lock()

    def one(i: int):
        t0 = time.perf_counter()
        client.create_file_from_buffer(payloads[i % len(payloads)], names[i])
        dt = time.perf_counter() - t0
        with lock:
            lat.append(dt)

    own = pool is None
    pool = pool or ThreadPoolExecutor(max_workers=concurrency, thread_name_prefix="bench")
    try:
        t0 = time.perf_counter()
        futs = [pool.submit(one, i) for i in range(count)]
        for f in futs:
            f.result()
        total = time.perf_counter() - t0
    finally:
        if own:
            pool.shutdown(wait=True)
    return Stats("Write", count, size, total, lat), names


def bench_read(client, prefix: str = "bench_write", concurrency: int = 10, files: list[str] | None = None,
               pool: ThreadPoolExecutor | None = None, verify: dict | None = None) -> Stats:
    if files is None:
        files = [f for f in client.list_all_files() if f.startswith(prefix)]
    if not files:
        return Stats("Read", 0, 0, 0.0)
    lat: list[float] = []
    total_bytes = [0]
    lock = threading.Lock()

    def one(name: str):
        t0 = time.perf_counter()
        data = client.get_file_content(name)
        dt = time.perf_counter() - t0
        if verify is not None and verify.get(name) is not None and verify[name] != data:
            raise RuntimeError(f"content mismatch reading {name}")
        with lock:
            lat.append(dt)
            total_bytes[0] += len(data)

    own = pool is None
    pool = pool or ThreadPoolExecutor(max_workers=concurrency, thread_name_prefix="bench")
    try:
        t0 = time.perf_counter()
        for f in [pool.submit(one, n) for n in files]:
            f.result()
        total = time.perf_counter() - t0
    finally:
        if own:
            pool.shutdown(wait=True)
    return Stats("Read", len(lat), total_bytes[0] // max(1, len(lat)), total, lat)


def bench_stress_write(client, duration: float = 30, size: int = 1 << 20, concurrency: int = 10,
                       prefix: str = "bench_stress") -> Stats:
    payloads = make_payloads(16, size)
    run_id = str(int(time.time()))
    deadline = time.perf_counter() + duration
    lat: list[float] = []
    errors = [0]
    lock = threading.Lock()
    counter = [0]
    first_error: list[str] = []

    def worker(w: int):
        while time.perf_counter() < deadline:
            with lock:
                i = counter[0]
                counter[0] += 1
            t0 = time.perf_counter()
            try:
                client.create_file_from_buffer(payloads[i % len(payloads)], f"{prefix}/{run_id}/stress_{w}_{i}")
                with lock:
                    lat.append(time.perf_counter() - t0)
            except Exception as e:  # noqa: BLE001
                with lock:
                    errors[0] += 1
                    if not first_error:
                        first_error.append(f"{type(e).__name__}: {e}"[:300])

    t0 = time.perf_counter()
    threads = [threading.Thread(target=worker, args=(w,)) for w in range(concurrency)]
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    st = Stats("Stress Write", len(lat), size, time.perf_counter() - t0, lat, errors[0])
    st.first_error = first_error[0] if first_error else ""
    return st
