"""``dfs_cli benchmark write|read|stress-write`` (reference dfs/client/src/bin/dfs_cli.rs:
581-807, print_stats :840-882). Same MB/s formula (count*size/2^20/secs) and latency
statistics, plus P50. Payloads are random bytes (the reference writes zeros)."""
from __future__ import annotations

import os
import threading
import time
from concurrent.futures import ThreadPoolExecutor
from dataclasses import dataclass, field

from .client import DfsError


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


_PHASES = {"write": ("crc", "create", "write", "md5_wait", "complete", "copy", "acquire"), "read": ("getinfo", "read")}


def _native_run(client, kind: str, names: list[str], bufs: list, concurrency: int) -> Stats | None:
    """The benchmark workers as native threads over the client's native data path
    (`bench_writes` / `bench_reads` in csrc/bindings_meta.cpp), like the reference CLI's
    tokio tasks (dfs_cli.rs:594-690). None when the client has no native path (TLS, hedged
    reads, no co-located chunkserver and no remote client) or DFS_BENCH_NATIVE=0. Ops the
    native client does not own come back as NotHandled and are redone on the Python path,
    so every name ends up written / read exactly as `create_file_from_buffer` /
    `get_file_content` would do it."""
    if os.environ.get("DFS_BENCH_NATIVE", "1") == "0":
        return None
    fc = (client._fast if client._fast is not None else client._remote) if kind == "write" else client._native_reader()
    if fc is None or not hasattr(fc, "bench_writes"):
        return None
    t0 = time.perf_counter()
    if kind == "write":
        status, lat, _, times, nbytes, err, _ = fc.bench_writes(names, bufs, concurrency)
    else:
        status, lat, _, times, nbytes, err, bad = fc.bench_reads(names, bufs, concurrency)
    lat = list(lat)
    for i, st in enumerate(status):
        if st == 2:
            raise DfsError(err or f"{kind} of {names[i]} failed")
        if st == 1:  # not handled natively: the Python client's path, timed the same way
            t = time.perf_counter()
            if kind == "write":
                client.create_file_from_buffer(bufs[i % len(bufs)], names[i])
            else:
                data = client.get_file_content(names[i])
                nbytes[i] = len(data)
                if bufs and bufs[i] is not None and bufs[i] != data:
                    raise RuntimeError(f"content mismatch reading {names[i]}")
            lat[i] = time.perf_counter() - t
    total = time.perf_counter() - t0
    if kind == "read" and bad:
        raise RuntimeError(f"content mismatch on {bad} native reads")
    done = sum(1 for st in status if st == 0)
    if fc is getattr(client, "_remote", None):
        client.remote_ops += done
    else:
        client.fp_ops += done
    if client.phase_times is not None:
        for st, tv in zip(status, times):
            if st == 0:
                for name, v in zip(_PHASES[kind], tv):
                    client.phase_times.setdefault(name, []).append(v)
    n = len(names)
    out = Stats("Write" if kind == "write" else "Read", n, sum(nbytes) // max(1, n), total, lat)
    # per-op phase times (seconds, _PHASES order; None for ops redone on the Python path)
    out.op_phases = [tuple(tv) if st == 0 else None for st, tv in zip(status, times)]
    return out


def bench_write(client, count: int = 100, size: int = 1 << 20, concurrency: int = 10, prefix: str = "bench_write",
                payloads: list[bytes] | None = None, run_id: str | None = None,
                pool: ThreadPoolExecutor | None = None) -> tuple[Stats, list[str]]:
    payloads = payloads or make_payloads(min(count, 64), size)
    run_id = run_id or str(int(time.time()))
    names = [f"{prefix}/{run_id}/bench_{i:010d}" for i in range(count)]
    nat = _native_run(client, "write", names, payloads, concurrency)
    if nat is not None:
        return nat, names
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
    nat = _native_run(client, "read", files, [verify.get(f) for f in files] if verify else [], concurrency)
    if nat is not None:
        return nat
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
