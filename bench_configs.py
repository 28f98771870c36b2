#!/usr/bin/env python3
"""Secondary BASELINE.json configurations (bench.py measures the headline, config 2/scaling).

    python bench_configs.py config1            # CPU plumbing: 1 master + 1 CS, put/get + benchmark
    python bench_configs.py config3 [--gpu 0]  # 3 chunkservers, RF 3: the benchmark, nvme-sync + hbm-ack
    python bench_configs.py config4 [--gpu 0]  # 2-shard Raft masters + 4 chunkservers (RF 3): stress-write 60 s
                                               # per shard prefix + cross-shard Rename
    python bench_configs.py config5 [--gpu 0]  # S3 gateway: PUT/GET/Range/MPU + Parquet over S3 (pyarrow)

Each prints one JSON line. The reference publishes no number for these configurations except
the stress-write throughput (470 ops/s, 10 KiB, conc 5: BASELINE.md); the harness follows the
reference's own flows:
  * config 4: `dfs_cli benchmark stress-write` (dfs/client/src/bin/dfs_cli.rs:697-807) against a
    two-shard namespace, then cross-shard renames through the coordinator's 2PC
    (dfs/metaserver/src/master.rs:2728-3021);
  * config 5: test_scripts/spark-s3-test/run_spark_test.sh writes and reads Parquet through
    S3A (path-style, SigV4). Spark is not in this image; pyarrow's S3 filesystem (AWS SDK,
    SigV4, multipart upload, ranged GETs for footer + column chunks) drives the same gateway
    calls, and the S3 object benchmarks use plain HTTP like s3_integration_test.py.
"""
from __future__ import annotations

import argparse
import hashlib
import json
import shutil
import os
import subprocess
import sys
import tempfile
import threading
import time
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

from rust_hadoop_generated_by_llm_amd.client.benchmark import (bench_read, bench_stress_write,  # noqa: E402
                                                               bench_write, make_payloads)
from rust_hadoop_generated_by_llm_amd.cluster.launcher import LocalCluster  # noqa: E402


def pct(v, p):
    v = sorted(v)
    return round(1e3 * v[min(len(v) - 1, len(v) * p // 100)], 3) if v else 0.0


def emit(d):
    print(json.dumps(d), flush=True)


def progress(msg: str):
    """One line per phase on stderr, so a long config run shows where it is (and a silent one
    where it stopped)."""
    print(f"[bench_configs {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


# ----------------------------------------------------------------------------- config 1
def config1(a):
    """single master + 1 chunkserver on CPU: put/get 1 MiB round trip + the benchmark."""
    with LocalCluster(n_chunkservers=1, gpus=None) as c:
        cl = c.client()
        data = os.urandom(1 << 20)
        t0 = time.perf_counter()
        cl.create_file_from_buffer(data, "/plumbing/one")
        t1 = time.perf_counter()
        got = cl.get_file_content("/plumbing/one")
        t2 = time.perf_counter()
        assert got == data
        ws, names = bench_write(cl, a.count, a.size, a.concurrency, prefix="/bench_write",
                                payloads=make_payloads(a.count, a.size))
        rs = bench_read(cl, files=names, concurrency=a.concurrency)
        emit({"config": 1, "topology": "1 master + 1 chunkserver, host store (no GPU), nvme-sync",
              "put_1mib_ms": round(1e3 * (t1 - t0), 3), "get_1mib_ms": round(1e3 * (t2 - t1), 3),
              "write_mb_per_s": round(ws.count * ws.avg_size / (1 << 20) / ws.total_s, 2),
              "read_mb_per_s": round(rs.count * rs.avg_size / (1 << 20) / rs.total_s, 2),
              "write_p50_ms": pct(ws.latencies, 50), "write_p99_ms": pct(ws.latencies, 99),
              "read_p50_ms": pct(rs.latencies, 50), "read_p99_ms": pct(rs.latencies, 99),
              "files": a.count, "size": a.size, "concurrency": a.concurrency})
        cl.close()


def _cs_gpus(a, n: int) -> tuple[list[int] | None, bool]:
    """GPU of each of n chunkservers: distinct GPUs while the box has them (from --gpu on),
    otherwise several chunkservers share one (a rehearsal of the multi-GPU topology: the
    replicas still cross between chunkserver processes, HBM to HBM over hipipc). Returns
    (gpus, shared)."""
    if a.gpu < 0:
        return None, False
    from rust_hadoop_generated_by_llm_amd.utils.gpu import visible_gpus

    ndev = max(1, visible_gpus())
    gpus = [(a.gpu + i) % ndev for i in range(n)]
    return gpus, len(set(gpus)) < n


def _topology(c, gpus, shared: bool) -> str:
    where = ("host store" if gpus is None else
             f"MI355X HBM store, {len(set(gpus))} GPU(s)" + (" shared by the chunkservers" if shared else ""))
    return f"{c.n_cs} chunkservers ({where}), RF {min(3, c.n_cs)}"


def _settle_journals(c, limit_s: float = 120.0) -> float:
    """Wait until no chunkserver's journal has a part a writer could be handed unwritten."""
    import urllib.request

    t0 = time.time()
    while time.time() - t0 < limit_s:
        unready = 0
        for u in c.cs_http:
            try:
                st = json.load(urllib.request.urlopen(f"{u}/stats", timeout=10))
            except OSError:
                unready += 1
                continue
            unready += int(st.get("journal_parts_unready", 0)) + int(st.get("journal_spares_missing", 0))
        if unready == 0:
            break
        time.sleep(0.2)
    return time.time() - t0


# ----------------------------------------------------------------------------- config 3
def config3(a):
    """BASELINE config 3: 3 chunkservers, replication factor 3 (the pipeline over the device
    transport), the benchmark's 1 MiB x 100 at concurrency 10 from one client, nvme-sync and
    hbm-ack. On a 1-GPU box the 3 chunkservers share the GPU (labelled)."""
    out = {"config": 3, "files": a.count, "size": a.size, "concurrency": a.concurrency, "steps": a.steps, "runs": []}
    # like bench.py: every chunkserver holds every block (RF 3 on 3), so each journal gets the
    # run's spare segments created and written out before the timed steps, not on demand
    # under the acked writes (which put 150 ms stalls into the write tail)
    need = (a.steps + 1) * a.count * (a.size + a.size // 128 + 4096)
    env = {"DFS_JOURNAL_SPARES": str(-(-need // int((256 << 20) * 0.96)) + 2)}
    for durability in ("nvme-sync", "hbm-ack"):
        gpus, shared = _cs_gpus(a, 3)
        progress(f"config 3: 3 chunkservers, {durability}")
        with LocalCluster(n_chunkservers=3, gpus=gpus, durability=durability, env=env,
                          hbm_capacity="16G" if gpus else "0", p2p="hipipc" if gpus else "socket") as c:
            _settle_journals(c)
            cl = c.client()
            payloads = make_payloads(a.count, a.size)
            ws, names = bench_write(cl, a.count, a.size, a.concurrency, prefix="/bench_write/w", payloads=payloads)
            bench_read(cl, files=names, concurrency=a.concurrency)  # warm-up step
            wl, rl, wt, rt, wb, rb = [], [], 0.0, 0.0, 0, 0
            for s in range(a.steps):
                ws, names = bench_write(cl, a.count, a.size, a.concurrency, prefix=f"/bench_write/s{s}", payloads=payloads)
                rs = bench_read(cl, files=names, concurrency=a.concurrency,
                                verify={n: payloads[i % len(payloads)] for i, n in enumerate(names)} if s == 0 else None)
                wl += ws.latencies
                rl += rs.latencies
                wt += ws.total_s
                rt += rs.total_s
                wb += ws.count * ws.avg_size
                rb += rs.count * rs.avg_size
            info = cl.get_file_info(names[0])
            replicas = len(info.blocks[0].locations) if info and info.blocks else 0
            out["runs"].append({"durability": durability, "topology": _topology(c, gpus, shared),
                                "replicas_per_block": replicas,
                                "mb_per_s": round((wb + rb) / (1 << 20) / (wt + rt), 1),
                                "write_mb_per_s": round(wb / (1 << 20) / wt, 1), "read_mb_per_s": round(rb / (1 << 20) / rt, 1),
                                "write_p50_ms": pct(wl, 50), "write_p99_ms": pct(wl, 99),
                                "read_p50_ms": pct(rl, 50), "read_p99_ms": pct(rl, 99)})
            cl.close()
    emit(out)


# ----------------------------------------------------------------------------- config 4
def config4(a):
    # the reference's compose topology: 4 chunkservers shared by both shards, so a write is
    # replicated 3 ways (docker-compose.yml:49,98,118,137; master.rs:2400-2402)
    gpus, shared = _cs_gpus(a, a.chunkservers)
    # a fixed two-shard map: with the default thresholds the shard whose prefix went idle
    # (/a during the /z phase) merges into its neighbour after a few seconds below 1 rps, and
    # the "cross-shard" renames then cross nothing (split/merge have their own cluster tests)
    with LocalCluster(shards=2, config_server=True, n_chunkservers=a.chunkservers, gpus=gpus,
                      hbm_capacity="16G" if gpus else "0", p2p=("hipipc" if gpus else "socket") if a.chunkservers > 1 else None,
                      master_args=["--split-threshold-rps", "1e12", "--merge-threshold-rps", "-1"]) as c:
        cl = c.client()
        from bench import cgroup_cpu, cgroup_cpu_delta

        # the two-shard range map: the second shard owns "< /m" (sharding.rs:99-106)
        cpu = []
        for pre in ("/a/stress", "/z/stress"):
            progress(f"config 4: stress-write {pre}, {a.stress_seconds:.0f} s")
            cg0, t0 = cgroup_cpu(), time.perf_counter()
            st = bench_stress_write(cl, a.stress_seconds, a.stress_size, a.stress_concurrency, prefix=pre)
            # the whole job's CPU in the phase: every process shares the box's quota
            cpu.append(cgroup_cpu_delta(cg0, cgroup_cpu(), time.perf_counter() - t0))
            if pre == "/a/stress":
                ss = st
            else:
                ss2 = st
        # cross-shard renames: /a/... (shard owning "< /m") -> /z/... (the other shard) via 2PC
        n = a.renames
        srcs = [f"/a/ren/src_{i:05d}" for i in range(n)]
        payload = os.urandom(a.stress_size)
        with ThreadPoolExecutor(a.stress_concurrency) as ex:
            list(ex.map(lambda p: cl.create_file_from_buffer(payload, p), srcs))
        lats, errors, first_error = [], 0, ""
        lock = threading.Lock()

        def ren(i):
            nonlocal errors, first_error
            t0 = time.perf_counter()
            try:
                cl.rename_file(srcs[i], f"/z/ren/dst_{i:05d}")
                with lock:
                    lats.append(time.perf_counter() - t0)
            except Exception as e:  # noqa: BLE001
                with lock:
                    errors += 1
                    first_error = first_error or f"{type(e).__name__}: {e}"[:300]

        t0 = time.perf_counter()
        with ThreadPoolExecutor(a.stress_concurrency) as ex:
            list(ex.map(ren, range(n)))
        el = time.perf_counter() - t0
        ok = all(cl.exists(f"/z/ren/dst_{i:05d}") and not cl.exists(srcs[i]) for i in range(0, n, max(1, n // 50)))
        shards = {sid: len(ms) for sid, ms in c.shard_masters.items()}
        probe = cl.get_file_info(srcs[0].replace("/a/ren/src", "/z/ren/dst"))
        replicas = len(probe.blocks[0].locations) if probe and probe.blocks else 0
        emit({"config": 4, "topology": f"config server + {len(shards)} Raft shards + {_topology(c, gpus, shared)}, nvme-sync",
              "replication_factor": min(3, c.n_cs), "replicas_per_block": replicas,
              "dynamic_sharding": "off (fixed two-shard map)",
              "durable_path": "per-file" if os.environ.get("DFS_JOURNAL") == "0" else "journal",
              "stress_write": [{"prefix": p, "seconds": s.total_s, "size": a.stress_size,
                                "concurrency": a.stress_concurrency, "ops": s.count, "errors": s.errors,
                                "ops_per_s": round(s.count / s.total_s, 1), "p50_ms": pct(s.latencies, 50),
                                "p99_ms": pct(s.latencies, 99),
                                # the published 470 ops/s ran at RF 3 (4 chunkservers): compare only
                                # a run at the same replication factor
                                "vs_published_470_ops_per_s": (round(s.count / s.total_s / 470.0, 1)
                                                               if min(3, c.n_cs) == 3 else None),
                                "host_cpu_job": cj}
                               for (p, s), cj in zip((("/a", ss), ("/z", ss2)), cpu)],
              "cross_shard_rename": {"ops": n, "errors": errors, "seconds": round(el, 3),
                                     "ops_per_s": round(len(lats) / el, 1), "p50_ms": pct(lats, 50),
                                     "p99_ms": pct(lats, 99), "verified": ok, "first_error": first_error}})
        cl.close()


# ----------------------------------------------------------------------------- config 5
def _s3_payload(i: int, size: int) -> bytes:
    import random

    return random.Random(i).randbytes(size)


def _s3_load(job):
    """One load-generator process (a GIL of its own, like one S3 client host): runs its share
    of the requests back to back over one keep-alive session; returns (start, end, latencies)."""
    import requests

    op, url, idxs, size, nobj = job[:5]
    pfx = job[5] if len(job) > 5 else "obj"
    s = requests.Session()
    bodies = {i: _s3_payload(i % nobj, size) for i in idxs} if op == "put" else {}
    lats = []
    t_start = time.time()
    for i in idxs:
        t0 = time.perf_counter()
        if op == "put":
            r = s.put(f"{url}/bench/{pfx}_{i:05d}", data=bodies[i])
            assert r.status_code == 200 and r.headers["ETag"] == f'"{hashlib.md5(bodies[i]).hexdigest()}"'
        elif op == "get":
            r = s.get(f"{url}/bench/{pfx}_{i:05d}")
            assert r.status_code == 200 and len(r.content) == size
        else:
            off = (i * 7919 * 4096) % (size - 65536)
            r = s.get(f"{url}/bench/obj_{i % nobj:05d}", headers={"Range": f"bytes={off}-{off + 65535}"})
            assert r.status_code == 206 and len(r.content) == 65536
        lats.append(time.perf_counter() - t0)
    return t_start, time.time(), lats


def config5(a):
    import requests

    gpus = [a.gpu] if a.gpu >= 0 else None
    with LocalCluster(n_chunkservers=1, gpus=gpus, hbm_capacity="16G" if gpus else "0") as c:
        # --remote-gateway: the gateway as if on another host (no co-located chunkserver): its
        # native front moves every body over gRPC (RemoteFrontStore) instead of shared memory
        env = {"AUDIT_LOG_ENABLED": "false"} if a.remote_gateway else \
            {"AUDIT_LOG_ENABLED": "false", "LOCAL_CHUNKSERVER": c.cs_addrs[0]}
        url = c.start_s3(env)
        out = {"config": 5, "topology": f"S3 gateway + 1 master + 1 chunkserver "
                                        f"({'MI355X HBM store' if gpus else 'host store'}), nvme-sync",
               "gateway": "remote: native front over gRPC" if a.remote_gateway else "co-located: native front over shm"}
        s = requests.Session()
        assert s.put(f"{url}/bench").status_code == 200
        n, size = a.count, a.size
        # concurrency = load-generator PROCESSES (Python threads in one process measured the
        # client's interpreter lock, not the gateway), spawned before anything is timed
        import multiprocessing as mp

        lg = mp.get_context("spawn").Pool(a.concurrency)

        def timed(op, count, pfx="obj"):
            jobs = [(op, url, list(range(k, count, a.concurrency)), size, n, pfx) for k in range(a.concurrency)]
            res = lg.map(_s3_load, jobs)
            return max(r[1] for r in res) - min(r[0] for r in res), [x for r in res for x in r[2]]

        lg.starmap(_s3_payload, [(0, 16)] * a.concurrency, chunksize=1)  # workers up before timing
        # untimed warm-up round (as bench.py's warmup steps): every gateway process and its
        # DFS client have served requests before the clock starts
        progress("config5: warm-up")
        timed("put", n, "warm")
        timed("get", n, "warm")
        progress("config5: put / get / range")
        el, lat = timed("put", n)
        out["put"] = {"objects": n, "size": size, "mb_per_s": round(n * size / (1 << 20) / el, 1),
                      "p50_ms": pct(lat, 50), "p99_ms": pct(lat, 99)}
        el, lat = timed("get", n)
        out["get"] = {"objects": n, "size": size, "mb_per_s": round(n * size / (1 << 20) / el, 1),
                      "p50_ms": pct(lat, 50), "p99_ms": pct(lat, 99)}
        m = 4 * n
        el, lat = timed("range", m)
        out["range_get_64k"] = {"requests": m, "req_per_s": round(m / el, 1), "p50_ms": pct(lat, 50),
                                "p99_ms": pct(lat, 99)}
        # multipart upload of one large object, parts in parallel (S3 MPU emulation, handlers.rs:234-432)
        import xml.etree.ElementTree as ET

        progress("config5: multipart")
        part = 8 << 20
        nparts = a.mpu_parts
        blob = os.urandom(part * nparts)
        t0 = time.perf_counter()
        r = s.post(f"{url}/bench/big.bin?uploads")
        upload_id = ET.fromstring(r.content).find("UploadId").text
        etags = {}

        def up(k):
            rr = requests.put(f"{url}/bench/big.bin?partNumber={k + 1}&uploadId={upload_id}",
                            data=blob[k * part:(k + 1) * part])
            assert rr.status_code == 200
            etags[k + 1] = rr.headers["ETag"]

        with ThreadPoolExecutor(min(8, nparts)) as ex:
            list(ex.map(up, range(nparts)))
        body = "<CompleteMultipartUpload>" + "".join(
            f"<Part><PartNumber>{k}</PartNumber><ETag>{etags[k]}</ETag></Part>" for k in sorted(etags)) + \
            "</CompleteMultipartUpload>"
        r = s.post(f"{url}/bench/big.bin?uploadId={upload_id}", data=body)
        assert r.status_code == 200, r.text
        mpu_s = time.perf_counter() - t0
        t0 = time.perf_counter()
        got = s.get(f"{url}/bench/big.bin").content
        mpu_get_s = time.perf_counter() - t0
        assert got == blob
        out["multipart"] = {"parts": nparts, "part_size": part, "upload_mb_per_s": round(len(blob) / (1 << 20) / mpu_s, 1),
                            "get_mb_per_s": round(len(blob) / (1 << 20) / mpu_get_s, 1)}
        lg.close()
        f0 = _front_counters(url)
        progress("config5: parquet")
        out["parquet_over_s3"] = parquet_phase(url, a)
        f1 = _front_counters(url)
        # what pyarrow's S3 client (the AWS C++ SDK, as S3A's) sent that the native front handed over
        pr = {k: v - f0["reasons"].get(k, 0) for k, v in f1["reasons"].items() if k != "metrics"}
        out["parquet_over_s3"]["front_requests"] = f1["requests"] - f0["requests"]
        out["parquet_over_s3"]["front_handoff_reasons"] = {k: v for k, v in pr.items() if v}
        out["native_load"] = native_load_phase(url, a, len(blob), cluster=c)
        out["load_generator"] = f"{a.concurrency} client processes (requests, keep-alive)"
        out["gateway"] += _gateway_kind(c)
        # what the native front end served itself vs handed to Python (none for the executable)
        nat = {}
        for ln in s.get(f"{url}/metrics").text.splitlines():
            if ln.startswith(("s3_native_requests_total", "s3_native_handoffs_total", "s3_native_bytes",
                              "s3_native_get_", "s3_native_fallback_answers_total")):
                k, v = ln.rsplit(" ", 1)
                nat[k] = round(float(v), 4) if "seconds" in k else int(float(v))
        out["native_front"] = nat
        emit(out)


def _gateway_kind(cluster, name: str = "s3") -> str:
    """Which S3 gateway process the launcher started: the native executable, or (an A/B run
    with S3_NATIVE_GATEWAY=0) the Python gateway model of tests/models with its worker count."""
    pr = next((p for p in cluster.procs if p.name == name), None)
    if pr is not None and pr.info.get("native_gateway"):
        return "; process: dfs_s3_gateway (native executable, no Python)"
    return f"; process: tests/models/s3_gateway.py (model), {int(os.environ.get('S3_WORKERS', '4'))} workers"


def _front_counters(url: str) -> dict:
    """The native front's request / hand-off counters from the gateway's /metrics: totals
    plus the hand-offs by reason."""
    import requests

    out = {"requests": 0, "handoffs": 0, "reasons": {}}
    try:
        text = requests.get(f"{url}/metrics", verify=False, timeout=10).text
    except Exception:  # noqa: BLE001
        return out
    for ln in text.splitlines():
        if ln.startswith("s3_native_requests_total{"):
            out["requests"] += int(float(ln.rsplit(" ", 1)[1]))
        elif ln.startswith("s3_native_handoffs_total{"):
            reason = ln.split('reason="', 1)[1].split('"', 1)[0]
            v = int(float(ln.rsplit(" ", 1)[1]))
            out["handoffs"] += v
            out["reasons"][reason] = v
    return out


def _proc_cpu(cluster) -> dict:
    """CPU seconds (user + system) of every cluster process and its children, by name, plus
    this process's finished children (the load generator)."""
    import resource

    import psutil

    out = {}
    for pr in (cluster.procs if cluster is not None else []):
        try:
            ps = psutil.Process(pr.popen.pid)
            kids = [ps] + ps.children(recursive=True)
            times = [k.cpu_times() for k in kids]
            out[pr.name] = sum(t.user + t.system for t in times)
            out[pr.name + "_sys"] = sum(t.system for t in times)  # kernel time (page cache, fs, flushes)
        except psutil.Error:
            pass
    ru = resource.getrusage(resource.RUSAGE_CHILDREN)
    out["load_generator"] = ru.ru_utime + ru.ru_stime
    return out


_CS_KEYS = ("journal_records", "journal_bypassed", "materialized_blocks", "materialize_batches",
            "journal_sync_rounds", "journal_full_waits", "direct_writes", "writes", "disk_gate_waits")


def _cs_counters(cluster) -> dict:
    """Durable-path counters of the first chunkserver (its /stats), for per-phase deltas."""
    if cluster is None or not cluster.cs_http:
        return {}
    try:
        import urllib.request

        st = json.loads(urllib.request.urlopen(cluster.cs_http[0] + "/stats", timeout=5).read())
    except (OSError, ValueError):
        return {}
    return {k: st.get(k, 0) for k in _CS_KEYS if isinstance(st.get(k, 0), (int, float))}


def _cs_gauges(cluster) -> dict:
    """Where the first chunkserver's journal stands after a phase: used / live bytes, blocks,
    reclaim work so far, whether it may still grow, and the volume's free bytes."""
    if cluster is None or not cluster.cs_http:
        return {}
    try:
        import urllib.request

        st = json.loads(urllib.request.urlopen(cluster.cs_http[0] + "/stats", timeout=5).read())
    except (OSError, ValueError):
        return {}
    keys = ("blocks", "journal_used_bytes", "journal_live_bytes", "journal_live_records", "journal_segs",
            "journal_grow_blocked", "compactions", "relocated_blocks", "journal_tombstones", "materialize_pending",
            "agent_deletes", "deletes")
    out = {k: st[k] for k in keys if k in st}
    try:
        out["volume_free_bytes"] = shutil.disk_usage(cluster.base if hasattr(cluster, "base") else "/tmp").free
    except OSError:
        pass
    return out


def native_load_phase(url: str, a, mpu_bytes: int, creds: dict | None = None, mpu_key: str = "big.bin",
                      cluster=None) -> dict:
    """PUT / GET / Range GET 64 KiB / ListObjectsV2 / the S3A operations (HEAD, CopyObject,
    DeleteObjects, rename, aws-chunked PUT) / multipart upload / multipart GET against
    the gateway from the native load generator (build/native/s3_load: C++ HTTP/1.1 clients,
    one keep-alive connection per thread), so the numbers describe the gateway, not Python's
    HTTP stack. Every phase runs for --phase-seconds (>= 10 s windows). With
    `creds` (secure mode) every request is HTTPS and SigV4-signed with an STS session, PUTs
    ask for SSE-S3; each phase reports the front's hand-offs to Python during it."""
    exe = ROOT / "build" / "native" / "s3_load"
    if not exe.exists():
        return {"skipped": "build/native/s3_load not built"}
    host, port = url.split("://")[1].rsplit(":", 1)
    base = [str(exe), "--host", host, "--port", port, "--bucket", "bench", "--conc", str(a.concurrency),
            "--seconds", str(a.phase_seconds)]
    sec = []
    if creds:
        sec = ["--tls", "--ak", creds["ak"], "--sk", creds["sk"], "--token", creds["token"]]
    out = {"client": f"s3_load, {a.concurrency} C++ threads, keep-alive, {a.phase_seconds:g} s per phase"
                     + (", HTTPS + SigV4 with an STS session token" if creds else "")}
    n = a.count * 10
    phases = (("put", ["--op", "put", "--keys", str(n), "--size", str(a.size), "--prefix", "nat"]
               + (["--sse"] if creds else [])),
              ("get", ["--op", "get", "--keys", str(n), "--size", str(a.size), "--prefix", "nat", "--verify"]),
              ("range_get_64k", ["--op", "range", "--keys", str(n), "--size", str(a.size), "--prefix", "nat",
                                 "--verify"]),
              ("list_v2", ["--op", "list", "--prefix", "nat_00"]),
              # the S3A shape (Hadoop S3AFileSystem): getFileStatus HEADs, rename = CopyObject +
              # DELETE, directory delete = DeleteObjects pages, SDK PUTs as aws-chunked bodies
              ("head", ["--op", "head", "--keys", str(n), "--prefix", "nat"]),
              ("copy", ["--op", "copy", "--keys", str(n), "--size", str(a.size), "--prefix", "nat",
                        "--count", str(n), "--seconds", "0"]),
              ("multi_delete_100", ["--op", "multidelete", "--keys", str(n), "--prefix", "nat", "--batch", "100",
                                    "--count", str(max(1, n // 100)), "--seconds", "0"]),
              ("rename", ["--op", "rename", "--keys", str(n), "--size", str(a.size), "--prefix", "nat"]),
              ("chunked_put", ["--op", "chunked", "--keys", str(n), "--size", str(a.size), "--prefix", "natc"]),
              ("multipart_upload", ["--op", "mpu", "--size", str(a.mpu_object_mb << 20), "--parts", str(a.mpu_parts),
                                    # 4 objects per thread, replaced in turn: a 10 s window at
                                    # 5 GB/s would otherwise keep ~50 GB of unique objects on a
                                    # 79 GB volume (r5w: the journal filled, uploads timed out)
                                    "--prefix", "natmpu", "--keys", "4"]),
              ("multipart_get", ["--op", "get", "--size", str(mpu_bytes), "--key", mpu_key, "--keys", "1"]))
    from bench import cgroup_cpu, cgroup_cpu_delta

    for name, extra in phases:
        progress(f"native load: {name}")
        before = _front_counters(url)
        cg0, pc0, cs0, t0 = cgroup_cpu(), _proc_cpu(cluster), _cs_counters(cluster), time.perf_counter()
        r = subprocess.run(base + sec + extra, capture_output=True, text=True, timeout=a.phase_seconds * 4 + 300)
        # the whole job's CPU during the phase (gateway, load generator, master, chunkserver
        # share the box's quota): cores used, quota, throttled time; and cores per process
        el = time.perf_counter() - t0
        job_cpu = cgroup_cpu_delta(cg0, cgroup_cpu(), el)
        pc1 = _proc_cpu(cluster)
        res = json.loads(r.stdout) if r.stdout.strip() else {"error": r.stderr[-500:]}
        res["job_cpu"] = job_cpu
        res["cores_by_process"] = {k: round((v - pc0.get(k, 0.0)) / el, 2) for k, v in pc1.items()}
        res["chunkserver"] = {k: v - cs0.get(k, 0) for k, v in _cs_counters(cluster).items()}
        res["chunkserver_after"] = _cs_gauges(cluster)
        after = _front_counters(url)
        res["front_requests"] = after["requests"] - before["requests"]
        # the /metrics scrapes around the phase are answered by the Python workers (their
        # registry plus the front's counters): reason "metrics", not counted as a hand-off
        reasons = {k: v - before["reasons"].get(k, 0) for k, v in after["reasons"].items() if k != "metrics"}
        res["front_handoffs"] = sum(reasons.values())
        res["front_handoff_reasons"] = {k: v for k, v in reasons.items() if v}
        out[name] = res
    return out


def _sts_session(url: str, role_arn: str) -> dict:
    """A mock OIDC identity provider (RS256 JWKS, as tests/test_s3_gateway.py's) and one
    AssumeRoleWithWebIdentity round trip: the STS session the secure load runs under."""
    import requests
    import xml.etree.ElementTree as ET

    sys.path.insert(0, str(ROOT / "tests"))
    import _rsa  # noqa: E402 - the tests' RSA / JWT helpers (no third-party JWT library here)

    st = _IDP
    claims = {"sub": "bench", "aud": "dfs-client", "iss": st["url"], "exp": int(time.time()) + 3600,
              "iat": int(time.time()), "groups": ["bench"]}
    tok = _rsa.jwt_rs256(claims, st["n"], st["d"], "kid-1")
    r = requests.get(url + "/", params={"Action": "AssumeRoleWithWebIdentity", "WebIdentityToken": tok,
                                        "RoleArn": role_arn, "DurationSeconds": "3600"}, verify=False, timeout=30)
    assert r.status_code == 200, r.text
    root = ET.fromstring(r.content)
    ns = {"s": root.tag.split("}")[0].strip("{")} if root.tag.startswith("{") else {}

    def text(tag):
        el = root.find(f".//s:{tag}", ns) if ns else root.find(f".//{tag}")
        return el.text

    return {"ak": text("AccessKeyId"), "sk": text("SecretAccessKey"), "token": text("SessionToken")}


_IDP: dict = {}


def _start_idp() -> None:
    from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer

    sys.path.insert(0, str(ROOT / "tests"))
    import _rsa  # noqa: E402

    from rust_hadoop_generated_by_llm_amd.cluster.launcher import free_port

    n, e, d = _rsa.generate(2048, seed=7)
    port = free_port()
    _IDP.update(url=f"http://127.0.0.1:{port}", jwk=_rsa.jwk(n, e, "kid-1"), n=n, d=d)

    class H(BaseHTTPRequestHandler):
        def do_GET(self):  # noqa: N802
            if self.path == "/.well-known/openid-configuration":
                body = json.dumps({"issuer": _IDP["url"], "jwks_uri": _IDP["url"] + "/jwks"})
            elif self.path == "/jwks":
                body = json.dumps({"keys": [_IDP["jwk"]]})
            else:
                self.send_response(404)
                self.end_headers()
                return
            self.send_response(200)
            self.send_header("Content-Type", "application/json")
            self.end_headers()
            self.wfile.write(body.encode())

        def log_message(self, *args):
            pass

    srv = ThreadingHTTPServer(("127.0.0.1", port), H)
    threading.Thread(target=srv.serve_forever, daemon=True).start()


def config5_secure(a):
    """Config 5 at the reference's production settings (main.rs:263-274 TLS, auth_middleware
    SigV4 + STS sessions + IAM role policy, sse.rs SSE-S3): the gateway terminates TLS in its
    native front, every request is signed with an STS session credential whose role policy
    the front evaluates, every PUT is SSE-S3 encrypted. Reports each phase's hand-offs to Python."""
    import requests
    import urllib3

    from rust_hadoop_generated_by_llm_amd.s3.auth import sigv4

    urllib3.disable_warnings()
    gpus = [a.gpu] if a.gpu >= 0 else None
    _start_idp()
    with LocalCluster(n_chunkservers=1, gpus=gpus, hbm_capacity="16G" if gpus else "0") as c:
        ca, crt, key = c.make_certs()
        iam = c.base / "iam.json"
        role = "arn:dfs:iam:::role/bench-role"
        iam.write_text(json.dumps({"Roles": [{
            "RoleName": "bench-role", "Arn": role,
            "AssumeRolePolicyDocument": {"Statement": [{
                "Effect": "Allow", "Action": "sts:AssumeRoleWithWebIdentity",
                "Condition": {"ForAnyValue:StringEquals": {"OIDC_ISSUER:groups": ["bench"]}}}]},
            "Policies": [{"PolicyName": "bench", "PolicyDocument": {"Statement": [
                {"Effect": "Allow", "Action": ["s3:GetObject", "s3:PutObject", "s3:ListBucket", "s3:HeadObject",
                                               "s3:DeleteObject"],
                 "Resource": ["arn:dfs:s3:::bench", "arn:dfs:s3:::bench/*"]}]}}]}]}))
        env = {"LOCAL_CHUNKSERVER": c.cs_addrs[0], "TLS_CERT": crt, "TLS_KEY": key, "S3_REQUIRE_TLS": "true",
               "S3_AUTH_ENABLED": "true", "S3_ACCESS_KEY": "admin", "S3_SECRET_KEY": "admin-secret",
               "OIDC_ISSUER_URL": _IDP["url"], "OIDC_CLIENT_ID": "dfs-client",
               "STS_SIGNING_KEY": "sts-signing-key-0123456789abcdef", "IAM_CONFIG_PATH": str(iam),
               "SSE_MASTER_KEY": "cd" * 32, "AUDIT_LOG_ENABLED": "true"}
        url = c.start_s3(env).replace("http://", "https://")
        host = url.split("://")[1]
        h = sigv4.sign_headers("PUT", "/bench", [], host, b"", "admin", "admin-secret")
        assert requests.put(url + "/bench", headers=h, verify=False).status_code == 200
        creds = _sts_session(url, role)
        out = {"config": "5-secure", "topology": f"S3 gateway (native front: TLS + SigV4 + STS session + IAM role + "
                                                 f"SSE-S3 + audit) + 1 master + 1 chunkserver "
                                                 f"({'MI355X HBM store' if gpus else 'host store'}), nvme-sync",
               "gateway": _gateway_kind(c).lstrip("; ")}
        # the multipart object the multipart_get phase reads (uploaded by the same session)
        exe = ROOT / "build" / "native" / "s3_load"
        hostn, port = host.rsplit(":", 1)
        subprocess.run([str(exe), "--host", hostn, "--port", port, "--bucket", "bench", "--conc", "1", "--op", "mpu",
                        "--count", "1", "--size", str(a.mpu_parts * (8 << 20)), "--parts", str(a.mpu_parts),
                        "--prefix", "seed", "--keys", "1", "--tls", "--ak", creds["ak"], "--sk", creds["sk"],
                        "--token", creds["token"]], check=True, capture_output=True, timeout=300)
        out["native_load"] = native_load_phase(url, a, a.mpu_parts * (8 << 20), creds, mpu_key="seed_mpu_0_0",
                                               cluster=c)
        emit(out)


def parquet_phase(url: str, a) -> dict:
    """The Spark S3A flow of run_spark_test.sh, driven by pyarrow's S3 filesystem: write a
    Parquet table (multipart upload), read it back whole and column-projected (ranged GETs
    of the footer and the column chunks), aggregate, compare with the source."""
    import numpy as np
    import pyarrow as pa
    import pyarrow.compute as pc
    import pyarrow.fs as pafs
    import pyarrow.parquet as pq

    rows = a.parquet_rows
    rng = np.random.default_rng(7)
    table = pa.table({"id": np.arange(rows, dtype=np.int64),
                      "grp": rng.integers(0, 100, rows, dtype=np.int32),
                      "value": rng.random(rows),
                      "payload": rng.integers(0, 1 << 62, rows, dtype=np.int64)})
    s3 = pafs.S3FileSystem(endpoint_override=url.split("://")[1], scheme="http", access_key="ak",
                           secret_key="sk", region="us-east-1", allow_bucket_creation=True)
    s3.create_dir("parquet")
    # where the write time goes: the same table encoded into memory (pyarrow's Parquet
    # encoder on this CPU, no S3), then those bytes uploaded on their own (the SDK's
    # multipart upload against the gateway), then the end-to-end write Spark would do
    t0 = time.perf_counter()
    buf = pa.BufferOutputStream()
    pq.write_table(table, buf, row_group_size=max(1, rows // 8))
    encoded = buf.getvalue()
    enc = time.perf_counter() - t0
    t0 = time.perf_counter()
    with s3.open_output_stream("parquet/encoded.parquet") as f:
        f.write(encoded)
    up = time.perf_counter() - t0
    t0 = time.perf_counter()
    pq.write_table(table, "parquet/events.parquet", filesystem=s3, row_group_size=max(1, rows // 8))
    w = time.perf_counter() - t0
    size = s3.get_file_info("parquet/events.parquet").size
    t0 = time.perf_counter()
    back = pq.read_table("parquet/events.parquet", filesystem=s3)
    r = time.perf_counter() - t0
    assert back.equals(table)
    t0 = time.perf_counter()
    cols = pq.read_table("parquet/events.parquet", filesystem=s3, columns=["grp", "value"])
    agg = pc.sum(cols["value"]).as_py()
    rc = time.perf_counter() - t0
    assert abs(agg - pc.sum(table["value"]).as_py()) < 1e-6 * rows
    return {"rows": rows, "file_bytes": size, "write_mb_per_s": round(size / (1 << 20) / w, 1),
            "encode_only_s": round(enc, 3), "upload_only_mb_per_s": round(encoded.size / (1 << 20) / up, 1),
            "write_s": round(w, 3),
            "read_mb_per_s": round(size / (1 << 20) / r, 1), "projected_read_sum_s": round(rc, 3),
            "verified": True}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("config", choices=["config1", "config3", "config4", "config5"])
    p.add_argument("--chunkservers", type=int, default=4,
                   help="config4: chunkservers (the reference's compose topology has 4: RF 3)")
    p.add_argument("--steps", type=int, default=10, help="config3: timed benchmark steps per durability mode")
    p.add_argument("--gpu", type=int, default=-1)
    p.add_argument("--count", type=int, default=100)
    p.add_argument("--size", type=int, default=1 << 20)
    p.add_argument("--concurrency", type=int, default=10)
    p.add_argument("--stress-seconds", type=float, default=60.0, help="config4: per shard prefix (BASELINE: 60 s)")
    p.add_argument("--stress-size", type=int, default=10240)
    p.add_argument("--stress-concurrency", type=int, default=10)
    p.add_argument("--renames", type=int, default=500)
    p.add_argument("--mpu-parts", type=int, default=8)
    p.add_argument("--parquet-rows", type=int, default=4_000_000)
    p.add_argument("--phase-seconds", type=float, default=10.0,
                   help="length of each native load phase (PUT / GET / Range / List / MPU upload / MPU GET)")
    p.add_argument("--mpu-object-mb", type=int, default=64, help="object size of the multipart-upload phase")
    p.add_argument("--remote-gateway", action="store_true",
                   help="config5: no LOCAL_CHUNKSERVER, the native front reaches the DFS over gRPC only")
    p.add_argument("--secure", action="store_true",
                   help="config5 with TLS + SigV4/STS session + IAM role + SSE-S3 (the reference's production settings)")
    a = p.parse_args()
    if a.config == "config5" and a.secure:
        a.config = "config5_secure"
    os.environ.setdefault("DFS_LOG", "warning")
    {"config1": config1, "config3": config3, "config4": config4, "config5": config5, "config5_secure": config5_secure}[a.config](a)


if __name__ == "__main__":
    main()
