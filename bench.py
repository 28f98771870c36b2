#!/usr/bin/env python3
"""Headline benchmark: ``dfs_cli benchmark write`` + ``read`` (1 MiB x 100 files, concurrency
10) on MI355X ChunkServers — the BASELINE.json metric.

One rank per GPU (``python -m torch.distributed.run --nproc-per-node N bench.py --gpus N``):
* every rank starts a ChunkServer process bound to its GPU (HBM chunk store + CDNA4
  CRC kernels + RCCL replication rank r of N) and a metadata master for namespace
  shard r (single-node Raft group, as in the reference's compose topology); the shard
  map routes ``/bench_r<r>/...`` to shard r, every chunkserver heartbeats to every master;
* every rank runs the reference benchmark client against its local ChunkServer:
  per step, 100 random 1 MiB files are written (CreateFile -> AllocateBlock ->
  WriteBlock chain with RF = min(3, N) -> CompleteFile) and then read back in full;
* W untimed warmup steps, then K timed steps bracketed by barrier + cuda synchronize;
  the reported value is aggregate (write+read) MiB/s over all ranks / max rank time.

Per-GPU work is fixed as N grows ("weak" scaling). Durability defaults to nvme-sync:
every replica's data and .meta are fdatasync'ed before the ack, like the reference.
"""
from __future__ import annotations

import argparse
import json
import os
import shutil
import signal
import subprocess
import sys
import tempfile
import threading
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

from rust_hadoop_generated_by_llm_amd.utils.gpu import visible_gpus  # noqa: E402

METRIC = "dfs_cli benchmark write+read MB/s & p50 lat, 1MB\u00d7100 conc=10, 1/2/4/8 GPUs"
PKG = "rust_hadoop_generated_by_llm_amd"


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--count", type=int, default=100)
    p.add_argument("--size", type=int, default=1 << 20)
    p.add_argument("--concurrency", type=int, default=10)
    p.add_argument("--durability", choices=["nvme-sync", "hbm-ack"], default="nvme-sync")
    p.add_argument("--hbm-capacity", default="32G")
    p.add_argument("--transport", choices=["hipipc", "hipipc-spin", "rccl", "grpc", "socket"], default="hipipc",
                   help="replica payload path between ranks: hipipc (HBM->HBM one-sided copies over xGMI, also "
                        "between ranks sharing one GPU), hipipc-spin (RCCL-like spinning p2p kernels), rccl, "
                        "grpc (reference), socket (host-memory P2P, CPU rehearsal)")
    p.add_argument("--transport-ab", choices=["auto", "on", "off"], default="auto",
                   help="after the run, a short second measurement with the other replica transport (hipipc <-> "
                        "rccl; socket -> grpc on CPU), reported under transport_ab; auto: on when every rank has "
                        "its own GPU")
    p.add_argument("--shards", choices=["per-gpu", "one"], default="per-gpu",
                   help="metadata shards: one per GPU rank (default) or a single master")
    p.add_argument("--cpu", action="store_true", help="CPU chunk store (plumbing config 1)")
    p.add_argument("--workdir", default=None)
    p.add_argument("--timeout", type=float, default=1500.0)
    p.add_argument("--keep", action="store_true")
    p.add_argument("--cleanup", choices=["auto", "always", "never"], default="auto",
                   help="delete the run's data at exit (auto: only when the disk is nearly full)")
    p.add_argument("--rehearse-rccl", action="store_true",
                   help="bring RCCL up even when ranks share a GPU (it must fail cleanly and every "
                        "rank must fall back together) - a 1-GPU rehearsal of the failure path")
    p.add_argument("--stress-seconds", type=float, default=0.0,
                   help="after the timed write+read steps, also run `dfs_cli benchmark stress-write` "
                        "for this long per rank (0 = skip); reported under stress_write")
    p.add_argument("--stress-size", type=int, default=10240)
    p.add_argument("--stress-concurrency", type=int, default=5)
    p.add_argument("--remote-steps", type=int, default=None,
                   help="after the timed steps, repeat write+read this many times with a REMOTE client "
                        "(no shared memory, no local sockets: every master and chunkserver RPC over gRPC/TCP, "
                        "as the reference's dfs_cli does); reported under remote_client (0 = skip; "
                        "default 2 on one GPU, 0 with several: their replicas would only add volume usage)")
    p.add_argument("--roofline-records", type=int, default=None,
                   help="after the timed region, every rank at once appends this many 1 MiB journal records "
                        "per writer thread to a fresh journal on its volume (io_bench --roofline): the "
                        "volume's rate each rank gets, recorded as volume.roofline_mb_s (0 = skip; "
                        "default 30, 4 with --cpu)")
    p.add_argument("--profile-dir", default=None,
                   help="run each ChunkServer under rocprofv3 --kernel-trace --stats, output here")
    return p.parse_args()


def free_port() -> int:
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _die_with_parent():
    """In the child between fork and exec: SIGKILL when the spawning rank exits (Linux
    PR_SET_PDEATHSIG; inherited across exec, cleared only by a setuid exec)."""
    import ctypes

    try:
        ctypes.CDLL("libc.so.6", use_errno=True).prctl(1, signal.SIGKILL, 0, 0, 0)  # PR_SET_PDEATHSIG
    except OSError:
        pass


class Procs:
    def __init__(self):
        self.items: list[subprocess.Popen] = []
        self.logs: list[str] = []

    def spawn(self, args: list[str], log: str, env: dict) -> subprocess.Popen:
        return self.spawn_raw([sys.executable, "-m", *args], log, env)

    def spawn_raw(self, cmd: list[str], log: str, env: dict) -> subprocess.Popen:
        f = open(log, "ab")
        # own session (stop() signals the whole group), and killed with this rank if the rank
        # itself dies before its stop() runs (a launcher or a timeout killing the ranks used to
        # leave masters and chunkservers running on the node)
        p = subprocess.Popen(cmd, stdout=f, stderr=subprocess.STDOUT, env=env, cwd=str(ROOT),
                             start_new_session=True, preexec_fn=_die_with_parent)
        f.close()
        self.items.append(p)
        self.logs.append(log)
        return p

    def stop(self):
        for p in self.items:
            if p.poll() is None:
                try:
                    os.killpg(p.pid, signal.SIGTERM)
                except ProcessLookupError:
                    pass
        deadline = time.time() + 30
        for p in self.items:
            try:
                p.wait(timeout=max(0.1, deadline - time.time()))
            except subprocess.TimeoutExpired:
                try:
                    os.killpg(p.pid, signal.SIGKILL)
                except ProcessLookupError:
                    pass

    def tails(self) -> str:
        out = []
        for log in self.logs:
            try:
                with open(log, errors="replace") as f:
                    out.append(f"==> {log}\n" + "".join(f.readlines()[-30:]))
            except OSError:
                pass
        return "\n".join(out)


def wait_file(path: str, proc: subprocess.Popen, timeout: float, procs: Procs) -> dict:
    deadline = time.time() + timeout
    while not os.path.exists(path):
        if proc.poll() is not None:
            raise RuntimeError(f"process exited ({proc.returncode}) before ready:\n{procs.tails()}")
        if time.time() > deadline:
            raise TimeoutError(f"not ready after {timeout}s:\n{procs.tails()}")
        time.sleep(0.05)
    time.sleep(0.02)
    with open(path) as f:
        return json.load(f)


def prefix_of(rank: int) -> str:
    return f"/bench_r{rank:03d}"


def launch_ranks(gpus: int) -> int:
    """`bench.py --gpus N` started without a launcher: run the N ranks under
    torch.distributed.run as a CHILD process (this process has not touched the GPU and never
    will; it is not replaced by exec) and return its exit code. The JSON line comes from the
    children's rank 0, on this process's stdout."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), str(Path(__file__).resolve()),
           *sys.argv[1:]]
    print(f"[bench] --gpus {gpus} without a launcher: starting {gpus} ranks under torch.distributed.run",
          file=sys.stderr, flush=True)
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
    return subprocess.call(cmd, env=env, cwd=str(ROOT))


def main():
    a = parse()
    if "WORLD_SIZE" not in os.environ and a.gpus > 1:
        sys.exit(launch_ranks(a.gpus))
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", str(rank)))
    if world != a.gpus:
        # the reported n_gpus must be what ran: refuse rather than mislabel the run
        print(f"bench: WORLD_SIZE={world} but --gpus {a.gpus}; start N ranks (or omit the launcher)",
              file=sys.stderr)
        sys.exit(2)
    n = max(world, 1)

    import torch
    import torch.distributed as dist

    if world > 1:
        # gloo prints its connection banner straight to fd 1; the driver reads exactly one
        # JSON line from rank 0's stdout, so keep the banner off it
        sys.stdout.flush()
        saved = os.dup(1)
        devnull = os.open(os.devnull, os.O_WRONLY)
        os.dup2(devnull, 1)
        try:
            dist.init_process_group("gloo")
            dist.barrier()
        finally:
            sys.stdout.flush()
            os.dup2(saved, 1)
            os.close(saved)
            os.close(devnull)

    def gather(obj):
        if world == 1:
            return [obj]
        out = [None] * world
        dist.all_gather_object(out, obj)
        return out

    def bcast(obj):
        if world == 1:
            return obj
        box = [obj]
        dist.broadcast_object_list(box, src=0)
        return box[0]

    def barrier():
        if world > 1:
            dist.barrier()

    if a.remote_steps is None:
        a.remote_steps = 2 if n == 1 else 0
    pending: dict = {}  # rank 0: the primary result while the transport A/B phase runs

    def measure(a, transport: str, alt: bool = False):
        """One cluster up, W warm-up + K timed steps, torn down; rank 0 returns the result.
        `alt`: the transport A/B phase, whose watchdog reports the primary result and exits
        cleanly instead of losing it."""
        procs = Procs()
        done = threading.Event()
        extra_dirs: list = []
        limit = min(a.timeout, 240.0) if alt else a.timeout  # the A/B phase: 10 steps, never the driver's budget

        def watchdog():
            if not done.wait(limit):
                print(f"bench watchdog: exceeded {limit}s ({'transport A/B' if alt else 'run'}), tearing down",
                      file=sys.stderr, flush=True)
                print(procs.tails(), file=sys.stderr, flush=True)
                procs.stop()
                if alt and rank == 0 and pending:
                    pending["transport_ab"] = {transport: {"error": f"timed out after {limit:.0f} s"}}
                    print(json.dumps(pending), flush=True)
                    os._exit(0)
                os._exit(3 if not alt else 0)

        threading.Thread(target=watchdog, daemon=True).start()

        tmp_parent = Path(os.environ.get("TMPDIR", "/tmp"))
        # ranks spread over the node's local volumes when it has several (one NVMe drive per
        # GPU is common on 8-GPU nodes): each rank's journal, blocks and master WAL live on
        # volume rank % V, so replicas of different ranks do not share one device's queue
        vols = bcast(_data_volumes(Path(a.workdir) if a.workdir else tmp_parent) if rank == 0 else None)
        vols = vols if (n > 1 and not a.workdir) else vols[:1]
        on_vol = [r for r in range(n) if r % len(vols) == rank % len(vols)]
        if rank == 0 and not a.workdir:
            _make_room(tmp_parent, _bytes_needed(a, n) * len([r for r in range(n) if r % len(vols) == 0]) // max(1, n))
        base = bcast((a.workdir or tempfile.mkdtemp(prefix="dfs_bench_", dir=str(tmp_parent))) if rank == 0 else None)
        base_p = Path(base)
        if rank == 0:
            base_p.mkdir(parents=True, exist_ok=True)
            (base_p / ".dfs_bench").touch()  # marks a directory _make_room may reclaim later
        my_vol = Path(vols[rank % len(vols)])
        if rank % len(vols) == 0:
            rank_dir = base_p / f"rank{rank}"
        else:
            rank_dir = my_vol / f"{base_p.name}_rank{rank}"
            extra_dirs.append(rank_dir)
        rank_dir.mkdir(parents=True, exist_ok=True)
        journal_segs = _journal_segments(base_p if rank % len(vols) == 0 else my_vol,
                                         _bytes_needed(a, n) * len(on_vol) // max(1, n), len(on_vol))
        # A run whose replicas do not fit its volumes (N ranks x RF copies of every step on one
        # shared device) deletes each step's files after reading them back, so the journals
        # reclaim them as the run goes: extra work inside the timed region (the number is
        # conservative, not inflated), reported as `reclaim_between_steps`. Without it the
        # journals would grow until the volume is full and the writers stall.
        my_room = _free_bytes(base_p if rank % len(vols) == 0 else my_vol) - (6 << 30)
        my_need = _bytes_needed(a, n) * len(on_vol) // max(1, n)
        reclaim_steps = os.environ.get("DFS_BENCH_RECLAIM", "auto") == "1" or (
            os.environ.get("DFS_BENCH_RECLAIM", "auto") == "auto" and any(gather(my_need > my_room)))
        env = dict(os.environ)
        env["PYTHONPATH"] = str(ROOT) + os.pathsep + env.get("PYTHONPATH", "")
        env.setdefault("DFS_LOG", "warning")
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        if _journal_store_mode():
            # the journal is the store of record and grows on demand: prepare (create and write
            # out once) as many segments as this run's replicas need up front, within the volume
            if journal_segs > 0:
                env.setdefault("DFS_JOURNAL_SPARES", str(journal_segs))
        elif journal_segs > 0:
            env.setdefault("DFS_JOURNAL_SEGS", str(journal_segs))
        elif journal_segs < 0:
            env["DFS_JOURNAL"] = "0"
        for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "LOCAL_WORLD_SIZE",
                  "GROUP_RANK", "ROLE_RANK", "ROLE_WORLD_SIZE", "TORCHELASTIC_RUN_ID"):
            env.pop(k, None)
        try:
            # ---------------- metadata shards: shard r owns /bench_r<r>/...
            per_gpu = a.shards == "per-gpu"
            runs_master = per_gpu or rank == 0
            gport, hport = (free_port(), free_port()) if runs_master else (0, 0)
            ports = gather(gport)
            if per_gpu:
                shards = {f"shard-{r:03d}": [f"http://127.0.0.1:{ports[r]}"] for r in range(n)}
                ranges = {prefix_of(r) + "/\U0010FFFF": f"shard-{r:03d}" for r in range(n - 1)}
                ranges["\U0010FFFF"] = f"shard-{n - 1:03d}"
            else:
                shards = {"shard-000": [f"http://127.0.0.1:{ports[0]}"]}
                ranges = {"\U0010FFFF": "shard-000"}
            shard_file = base_p / "shard_config.json"
            if rank == 0:
                shard_file.write_text(json.dumps({"shards": shards, "ranges": ranges}))
            barrier()
            if runs_master:
                ready = str(base_p / f"master{rank}.ready")
                from rust_hadoop_generated_by_llm_amd.cluster.launcher import role_command

                # the C++ dfs_master executable
                mp = procs.spawn_raw(role_command("master.server", [
                    "--addr", f"127.0.0.1:{gport}", "--http-port", str(hport),
                    "--storage-dir", str(rank_dir / "master"),
                    "--shard-id", f"shard-{rank:03d}", "--shard-config", str(shard_file)], env),
                    str(base_p / f"master{rank}.log"), dict(env, DFS_READY_FILE=ready))
                wait_file(ready, mp, 300, procs)
            barrier()
            my_master = f"http://127.0.0.1:{ports[rank if per_gpu else 0]}"
            # ---------------- chunkserver for this rank's GPU
            cport, chttp = free_port(), free_port()
            ready = str(base_p / f"cs{rank}.ready")
            # the benchmark ranks never open the GPU (no HIP / torch.cuda call in this process): the
            # chunkservers are the only GPU processes, so N ranks keep N processes on the cards.
            # The count comes from the KFD topology in sysfs, which opens no device.
            ndev = 0 if a.cpu else visible_gpus()
            gpu = -1 if a.cpu else local_rank % max(1, ndev)
            shared_gpu = (not a.cpu) and ndev < n  # rehearsal mode: several ranks on one GPU
            args = ["--addr", f"127.0.0.1:{cport}",
                    "--http-port", str(chttp), "--storage-dir", str(rank_dir / "data"),
                    "--gpu", str(gpu), "--durability", a.durability, "--hbm-capacity", a.hbm_capacity,
                    "--heartbeat-interval", "0.5", "--scrub-interval", "3600", "--rccl-timeout-ms", "90000"]
            if n > 1 and (transport == "socket" or (not a.cpu and transport in ("hipipc", "hipipc-spin"))):
                # hipipc works between processes that share a GPU too: a 1-GPU N-rank rehearsal
                # forwards replicas HBM -> HBM through the same code as the 8-GPU node
                args += ["--rccl-rank", str(rank), "--rccl-world", str(n), "--rccl-rendezvous",
                         str(base_p / "rccl_rdv"), "--replication-transport", transport]
            elif n > 1 and not a.cpu and transport == "rccl" and (not shared_gpu or a.rehearse_rccl):
                args += ["--rccl-rank", str(rank), "--rccl-world", str(n), "--rccl-rendezvous",
                         str(base_p / "rccl_rdv"), "--replication-transport", "rccl"]
            else:
                args += ["--replication-transport", "grpc"]
            cs_env = dict(env, DFS_READY_FILE=ready, SHARD_CONFIG=str(shard_file))
            from rust_hadoop_generated_by_llm_amd.cluster.launcher import role_command

            # the C++ dfs_chunkserver executable (the Python shell with DFS_NATIVE_CHUNKSERVER=0)
            cs_cmd = role_command("chunkserver.server", args, cs_env)
            if a.profile_dir:
                # profile only the ChunkServer (where the kernels run); rocprofv3 is started
                # before anything in this process touches the GPU
                pdir = os.path.abspath(os.path.join(a.profile_dir, f"cs{rank}"))
                os.makedirs(pdir, exist_ok=True)
                cs_env["TMPDIR"] = "/tmp"
                # DFS_PROF_EXTRA: more trace domains, e.g. "--memory-copy-trace" (never --pmc here)
                extra = [x for x in os.environ.get("DFS_PROF_EXTRA", "").split() if not x.startswith("--pmc")]
                cp = procs.spawn_raw(["rocprofv3", "--kernel-trace", "--marker-trace", *extra, "--stats", "--output-format",
                                      "csv", "-d", pdir, "-o", "cs", "--", *cs_cmd],
                                     str(base_p / f"cs{rank}.log"), cs_env)
            else:
                cp = procs.spawn_raw(cs_cmd, str(base_p / f"cs{rank}.log"), cs_env)
            cs_info = wait_file(ready, cp, 900, procs)
            my_cs = f"127.0.0.1:{cport}"
            t_start = time.time()

            def note(msg: str) -> None:
                # progress on stderr outside the timed region (the JSON line stays alone on stdout)
                print(f"[bench r{rank} +{time.time() - t_start:.1f}s] {msg}", file=sys.stderr, flush=True)

            note("chunkserver up")

            from rust_hadoop_generated_by_llm_amd.client.benchmark import bench_read, bench_write, make_payloads
            from rust_hadoop_generated_by_llm_amd.client.client import Client
            from rust_hadoop_generated_by_llm_amd.models import proto as pb
            from rust_hadoop_generated_by_llm_amd.parallel.sharding import ShardMap
            from rust_hadoop_generated_by_llm_amd.utils.rpc import ChannelPool

            # wait until our shard's master has registered every chunkserver and left safe mode
            pool = ChannelPool()
            deadline = time.time() + 300
            while True:
                try:
                    st = pool.call(my_master, "MasterService", "GetSafeModeStatus", pb.GetSafeModeStatusRequest(),
                                   timeout=2)
                    if st.chunk_server_count >= n and not st.is_safe_mode:
                        break
                except Exception:  # noqa: BLE001
                    pass
                if time.time() > deadline:
                    raise TimeoutError("master never registered all chunkservers")
                time.sleep(0.1)
            pool.close()
            note("master has every chunkserver")
            # the journal creates its segment files, and writes each out once, in the background
            # after start (journal.h); let that finish first, so the first-cycle zero fill and its
            # flushes do not share the volume with the timed writes (a startup transient, not the
            # steady state); bounded, and reported
            import urllib.request

            def settle_journal(limit_s: float):
                t_fill = time.perf_counter()
                fill_deadline = time.time() + limit_s
                unready = None
                while time.time() < fill_deadline:
                    try:
                        st = json.loads(urllib.request.urlopen(f"http://127.0.0.1:{chttp}/stats", timeout=5).read())
                    except OSError:
                        st = {}
                    # every spare this run's replicas need created and written out once (the journal
                    # then neither creates nor fills a segment while the timed writes run)
                    unready = (st.get("journal_parts_unready", 0) + st.get("journal_spares_missing", 0) * 8
                               if st.get("journal") else 0)
                    if unready == 0:
                        break
                    time.sleep(0.05)
                return round(time.perf_counter() - t_fill, 2), unready

            journal_settle_s, unready = settle_journal(180)
            note(f"journal settled in {journal_settle_s} s ({unready} parts still unready)")
            barrier()

            client = Client([my_master], local_chunkserver=my_cs)
            client.set_shard_map(ShardMap.load_config_file(str(shard_file)))
            payloads = make_payloads(a.count, a.size)
            from concurrent.futures import ThreadPoolExecutor

            tpool = ThreadPoolExecutor(max_workers=a.concurrency, thread_name_prefix="bench")

            def step(tag: str):
                ws, names = bench_write(client, a.count, a.size, a.concurrency, prefix=prefix_of(rank),
                                        payloads=payloads, run_id=tag, pool=tpool)
                verify = {nm: payloads[i % len(payloads)] for i, nm in enumerate(names)} if tag == "w0" else None
                rs = bench_read(client, files=names, pool=tpool, verify=verify)
                if reclaim_steps:
                    list(tpool.map(client.delete_file, names))
                return ws, rs

            for w in range(a.warmup):
                ws, rs = step(f"w{w}")
                note(f"warm-up step {w}: write p50 {1e3 * ws._pct(50):.2f} ms, read p50 {1e3 * rs._pct(50):.2f} ms")
            # the warm-up's pauses let the journal top its spares up; let those be written out too,
            # so the timed region starts (and, with two spares to spare, ends) with none unready
            resettle_s, unready = settle_journal(60) if os.environ.get("DFS_BENCH_RESETTLE", "1") != "0" else (0.0, 0)
            journal_settle_s = round(journal_settle_s + resettle_s, 2)
            if resettle_s > 0.05 or unready:
                note(f"journal re-settled after the warm-up in {resettle_s} s ({unready} parts still unready)")
            # the timed region is bracketed by barrier + device synchronize on both sides; the
            # synchronize runs in the process that owns the GPU and queued all of its work (the
            # chunkserver's /sync: hipDeviceSynchronize), not in this client process
            sync_log: list = []  # (request ms, hipDeviceSynchronize ms) of each device sync

            # one keep-alive connection to the chunkserver's native /sync listener, opened here, so
            # a sync inside the bracket is one request on an established connection (no connect,
            # accept or server thread start in the timed region)
            import http.client

            sync_conn = http.client.HTTPConnection("127.0.0.1", cs_info.get("sync_port") or chttp, timeout=60)

            def device_sync():
                if a.cpu:
                    return
                t_req = time.perf_counter()
                sync_conn.request("GET", "/sync")
                r = json.loads(sync_conn.getresponse().read())
                if not r.get("synchronized"):
                    raise RuntimeError(f"chunkserver device sync failed: {r}")
                sync_log.append((round(1e3 * (time.perf_counter() - t_req), 3), r.get("sync_ms")))

            # no cyclic-GC pass inside the timed region: a full collection over this process's
            # imports (torch, grpc, numpy) is tens of ms, and one landing in the closing bracket
            # showed up as a 100 ms device sync whose server side took 0.02 ms (profiles/r4_journal)
            import gc

            gc.collect()
            gc.freeze()
            gc.disable()
            device_sync()
            barrier()
            device_sync()
            import psutil

            def cpu_snapshot():
                snap = {"client": sum(psutil.Process().cpu_times()[:2])}
                for i, p in enumerate(procs.items):
                    try:
                        kids = [psutil.Process(p.pid)] + psutil.Process(p.pid).children(recursive=True)
                        name = os.path.basename(procs.logs[i]).split(".")[0]
                        times = [k.cpu_times() for k in kids]
                        snap[name] = sum(t.user + t.system for t in times)
                        snap[name + "_sys"] = sum(t.system for t in times)  # page cache / reclaim / flush
                    except psutil.Error:
                        pass
                return snap

            def cs_stats() -> dict:
                try:
                    import urllib.request

                    return json.loads(urllib.request.urlopen(f"http://127.0.0.1:{chttp}/stats", timeout=5).read())
                except Exception:  # noqa: BLE001
                    return {}

            st0 = cs_stats()
            thr0 = st0.get("thread_cpu_ms", {})  # per-thread CPU of the chunkserver, before
            vm0 = _vmstat()
            # journal readiness at the start of the timed region (reported with its end)
            jr0 = {k: st0.get("journal_" + k, 0) for k in JOURNAL_READY_KEYS}
            client.phase_times = {}
            cpu0 = cpu_snapshot()
            cg0 = cgroup_cpu()
            t0 = time.perf_counter()
            wl, rl, wbytes, rbytes = [], [], 0, 0
            wt = rt = 0.0
            slow: list = []  # the write tail: (ms, step, op, phase ms)
            for s in range(a.steps):
                ws, rs = step(f"s{s}")
                ph = getattr(ws, "op_phases", None) or []
                slow += [(x, s, i, ph[i] if i < len(ph) else None) for i, x in enumerate(ws.latencies)]
                slow = sorted(slow, key=lambda e: -e[0])[:20]
                wl += ws.latencies
                rl += rs.latencies
                wbytes += ws.count * ws.avg_size
                rbytes += rs.count * rs.avg_size
                wt += ws.total_s
                rt += rs.total_s
            t_loop = time.perf_counter() - t0
            device_sync()
            barrier()
            device_sync()
            elapsed = time.perf_counter() - t0
            end_sync_s = elapsed - t_loop
            gc.enable()
            note(f"{a.steps} timed steps in {elapsed:.3f} s")
            cpu1 = cpu_snapshot()
            host_cpu = {k: round((cpu1[k] - cpu0.get(k, 0.0)) / elapsed, 2) for k in cpu1}
            job_cpu = cgroup_cpu_delta(cg0, cgroup_cpu(), elapsed)
            # counters of the timed phase only (the stress / remote phases below add their own hops)
            stats = cs_stats()
            jr1 = {k: stats.get("journal_" + k, 0) for k in JOURNAL_READY_KEYS}
            vm1 = _vmstat()
            vm_delta = {k: vm1[k] - vm0.get(k, 0) for k in vm1 if vm1[k] - vm0.get(k, 0)}
            thr1 = stats.get("thread_cpu_ms", {})
            # cores each named chunkserver thread group used over the timed region (HIP runtime
            # threads keep the executable's name)
            thread_cores = {k: round((v - thr0.get(k, 0)) / 1e3 / elapsed, 2) for k, v in thr1.items()
                            if (v - thr0.get(k, 0)) / 1e3 / elapsed >= 0.01}
            vol = {"rank_dir_bytes": _allocated_bytes(rank_dir), "volume": str(my_vol), "volumes_in_job": len(vols),
                   "journal_used_bytes": stats.get("journal_used_bytes", 0),
                   "journal_live_bytes": stats.get("journal_live_bytes", 0),
                   "exported_blocks": stats.get("materialized_blocks", 0),
                   "durable_path": "per-file" if env.get("DFS_JOURNAL") == "0" else (
                       stats.get("journal_mode", "journal") if stats.get("journal") else "per-file")}
            stress = None
            if a.stress_seconds > 0:
                # the reference's only published throughput (stress-write 30 s, 10240 B,
                # conc 5 -> 470 ops/s); run outside the timed region, same cluster, every rank at once
                from rust_hadoop_generated_by_llm_amd.client.benchmark import bench_stress_write

                barrier()
                ss = bench_stress_write(client, a.stress_seconds, a.stress_size, a.stress_concurrency,
                                        prefix=prefix_of(rank) + "/stress")
                stress = {"ops": ss.count, "seconds": ss.total_s, "errors": ss.errors, "lat": ss.latencies,
                          "first_error": getattr(ss, "first_error", "")}
            remote = None
            if a.remote_steps > 0:
                # the reference's wire path (dfs/client/src/mod.rs:415-451,921-944): a client that
                # is not co-located, so every WriteBlock/ReadBlock carries the payload over gRPC
                rc = Client([my_master], local_chunkserver=None, local_rpc=False)
                rc.set_shard_map(ShardMap.load_config_file(str(shard_file)))
                rc.phase_times = {}
                barrier()
                rwl, rrl, rwb, rrb, rwt, rrt = [], [], 0, 0, 0.0, 0.0
                for s in range(a.remote_steps):
                    ws, names = bench_write(rc, a.count, a.size, a.concurrency, prefix=prefix_of(rank) + "/remote",
                                            payloads=payloads, run_id=f"rem{s}", pool=tpool)
                    rs = bench_read(rc, files=names, pool=tpool,
                                    verify={nm: payloads[i % len(payloads)] for i, nm in enumerate(names)} if s == 0 else None)
                    rwl += ws.latencies
                    rrl += rs.latencies
                    rwb += ws.count * ws.avg_size
                    rrb += rs.count * rs.avg_size
                    rwt += ws.total_s
                    rrt += rs.total_s
                remote = {"wl": rwl, "rl": rrl, "wbytes": rwb, "rbytes": rrb, "wt": rwt, "rt": rrt,
                          "native_ops": rc.remote_ops, "ops": 2 * a.remote_steps * a.count,
                          "phases": {k: round(1e3 * sorted(v)[len(v) // 2], 3) for k, v in rc.phase_times.items() if v}}
                rc.close()
            roof = None
            nroof = a.roofline_records if a.roofline_records is not None else (4 if a.cpu else 30)
            if nroof > 0 and a.durability == "nvme-sync":
                # the volume's journal write rate with every rank appending at once (outside the
                # timed region, after it): the bound the nvme-sync write of this N is read against
                barrier()
                try:
                    r = subprocess.run([str(ROOT / "build" / "native" / "io_bench"), "--roofline", "--dir",
                                        str(rank_dir / "roofline"), "--threads", str(a.concurrency),
                                        "--per", str(nroof)], capture_output=True, text=True, timeout=180)
                    roof = json.loads(r.stdout.strip().splitlines()[-1]) if r.returncode == 0 else {"error": r.stderr[-300:]}
                except (OSError, ValueError, IndexError, subprocess.TimeoutExpired) as e:
                    roof = {"error": str(e)[:300]}
            slow_w = [{"ms": round(1e3 * x, 3), "step": st, "op": i,
                       **({k: round(1e3 * v, 3) for k, v in zip(("crc", "create", "write", "md5_wait", "complete", "copy", "acquire"), ph)}
                          if ph else {})} for x, st, i, ph in slow]
            allr = gather({"md5": getattr(client._fast, "md5_mode", None), "vm": vm_delta, "slow_w": slow_w, "roof": roof, "elapsed": elapsed, "end_sync": end_sync_s, "loop": t_loop, "syncs": sync_log, "wl": wl, "rl": rl, "wbytes": wbytes,
                           "rbytes": rbytes, "wt": wt,
                           "rt": rt, "cs": stats, "stress": stress, "remote": remote, "vol": vol,
                           "p2p": bool(cs_info.get("rccl", False)), "p2p_transport": cs_info.get("transport", "grpc"),
                           "cpu": host_cpu, "job_cpu": job_cpu, "thread_cores": thread_cores, "settle": journal_settle_s,
                           "jready": {"start": jr0, "end": jr1}, "phases": {k: round(1e3 * sorted(v)[len(v) // 2], 3)
                                                       for k, v in (client.phase_times or {}).items() if v}})
            if rank == 0:
                tmax = max(r["elapsed"] for r in allr)
                tot = sum(r["wbytes"] + r["rbytes"] for r in allr)
                wlat = sorted(x for r in allr for x in r["wl"])
                rlat = sorted(x for r in allr for x in r["rl"])

                def pct(v, p):
                    return 1e3 * v[min(len(v) - 1, len(v) * p // 100)] if v else 0.0

                wmax = max(r["wt"] for r in allr)
                rmax = max(r["rt"] for r in allr)
                result = {
                    "metric": METRIC, "value": round(tot / (1 << 20) / tmax, 2), "unit": "MB/s", "n_gpus": n,
                    "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(1e3 * tmax / a.steps, 3),
                    "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "uint8",
                    "data": "synthetic random bytes",
                    "config": {"model": "dfs_cli benchmark write+read (1 MiB files)", "global_batch": a.count * n,
                               "seq_len": a.size, "parallelism": f"cs{n}-shards{n if per_gpu else 1}",
                               "files_per_gpu_per_step": a.count, "file_size": a.size, "concurrency": a.concurrency,
                               "replication_factor": min(3, n), "durability": a.durability,
                               "store": "cpu" if a.cpu else "hbm",
                               "durable_path": "per-file" if env.get("DFS_JOURNAL") == "0" else (
                                   "journal (store of record)" if _journal_store_mode() else "journal (round-4 ring)"),
                               "transport": observed_transport(allr, n)},
                    "write_mb_per_s": round(sum(r["wbytes"] for r in allr) / (1 << 20) / wmax, 2),
                    "read_mb_per_s": round(sum(r["rbytes"] for r in allr) / (1 << 20) / rmax, 2),
                    "write_p50_ms": round(pct(wlat, 50), 3), "write_p95_ms": round(pct(wlat, 95), 3),
                    "write_p99_ms": round(pct(wlat, 99), 3), "read_p50_ms": round(pct(rlat, 50), 3),
                    "read_p95_ms": round(pct(rlat, 95), 3), "read_p99_ms": round(pct(rlat, 99), 3),
                    "write_ops_per_s": round(len(wlat) / wmax, 1),
                    # where the timed region went besides the write and read phases (rank 0): the
                    # closing barrier + device synchronize, and the loop's own bookkeeping
                    "closing_sync_ms_rank0": round(1e3 * allr[0]["end_sync"], 3),
                    "device_syncs_rank0": allr[0]["syncs"],
                    "between_phases_ms_per_step_rank0": round(1e3 * (allr[0]["loop"] - allr[0]["wt"] - allr[0]["rt"]) / a.steps, 3),
                    # replica hops between same-node chunkservers: which device transport carried
                    # them (hipipc / rccl / socket), on how many ranks, and how often it fell back
                    "p2p_transport": ",".join(sorted({r["p2p_transport"] for r in allr if r["p2p"]})) or "none",
                    "p2p_ranks": sum(1 for r in allr if r["p2p"]),
                    "repl_pairs_up": sum(r["cs"].get("repl_pairs_up", 0) for r in allr),
                    **forward_counts(allr),
                    "p2p_fallbacks": sum(r["cs"].get("rccl_fallbacks", 0) + r["cs"].get("fp_p2p_fallbacks", 0)
                                         for r in allr),
                    "replica_failures": sum(r["cs"].get("fp_replica_failures", 0) for r in allr),
                    "repl_pair_failures": sum(r["cs"].get("repl_pair_failures", 0) for r in allr),
                    "gpu_kernel_launches": sum(r["cs"].get("gpu_kernel_launches", 0) for r in allr),
                    "fused_reads": sum(r["cs"].get("fused_reads", 0) for r in allr),
                    "direct_writes": sum(r["cs"].get("direct_writes", 0) for r in allr),
                    "disk_gate_waits": sum(r["cs"].get("disk_gate_waits", 0) for r in allr),
                    # store calls that found all of a chunkserver's GPU stream contexts busy
                    "lane_waits": sum(r["cs"].get("lane_waits", 0) for r in allr),
                    "lane_wait_ms": round(sum(r["cs"].get("lane_wait_ns", 0) for r in allr) / 1e6, 3),
                    # block journal (group commit): records appended, flush rounds that covered them,
                    # and blocks already written out as <id> + <id>.meta by the materializer
                    "journal": {k: sum(r["cs"].get(f, 0) for r in allr) for k, f in (
                        ("records", "journal_records"), ("sync_rounds", "journal_sync_rounds"),
                        ("materialized_blocks", "materialized_blocks"), ("materialize_pending", "materialize_pending"),
                        ("full_waits", "journal_full_waits"), ("segments", "journal_segs"),
                        ("segments_retired", "journal_segs_retired"), ("parts_filled", "journal_segs_filled"),
                        ("prepare_errors", "journal_prepare_errors"),
                        ("materialize_errors", "materialize_errors"), ("sync_ns", "journal_sync_ns"),
                        ("commit_ns", "journal_commit_ns"), ("bypassed", "journal_bypassed"),
                        ("parts_unready", "journal_parts_unready"), ("live_records", "journal_live_records"),
                        ("segments_in_use", "journal_segs_in_use"), ("segments_marked", "journal_segs_marked"),
                        ("relocated_blocks", "relocated_blocks"), ("supersedes", "journal_supersedes"),
                        ("export_deferred_headroom", "export_deferred_headroom"))} | {
                        "mode": ",".join(sorted({r["cs"].get("journal_mode", "?") for r in allr})),
                        "settle_s_before_warmup": max(r["settle"] for r in allr),
                        # readiness at both ends of the timed region, summed over ranks: parts a
                        # writer could be handed unwritten, spares owed (topped up when idle),
                        # top-ups deferred so far, segments created so far
                        "timed_region": {end: {k: sum(r["jready"][end][k] for r in allr) for k in JOURNAL_READY_KEYS}
                                         for end in ("start", "end")}} if any(r["cs"].get("journal") for r in allr) else None,
                    # where each rank's replicas live and how much of the volume they take
                    "volume": {"per_rank": [r["vol"] for r in allr], "free_bytes_after": _free_bytes(base_p),
                               "reclaim_between_steps": reclaim_steps,
                               # every rank appending 1 MiB journal records at once after the timed
                               # region (io_bench --roofline, conc threads each): per-rank MB/s, sum
                               "roofline_mb_s": [(r["roof"] or {}).get("roofline_mb_s") for r in allr],
                               "roofline_total_mb_s": round(sum((r["roof"] or {}).get("roofline_mb_s") or 0
                                                                for r in allr), 1),
                               "roofline_p50_ms": [(r["roof"] or {}).get("p50_ms") for r in allr]},
                    "host_cpu_util_rank0": allr[0]["cpu"],
                    # the whole job's CPU over the timed region, from the cgroup every rank shares
                    # (cores used, the quota, and time the quota throttled it); null without cgroup
                    "host_cpu_job": allr[0]["job_cpu"],
                    # host cores the whole job kept busy per GB/s of client writes (timed region,
                    # reads included): what an 8-rank node's CPU quota is read against
                    # how each rank's client hashed its ETags: OpenSSL per message, or the AVX-512
                    # multi-buffer engine when the rank's CPU budget is small (md5_mb.h)
                    "etag_md5": sorted({str(r["md5"]) for r in allr}),
                    "cores_per_gb_written": (round(allr[0]["job_cpu"]["cores_used"] / (
                        sum(r["wbytes"] for r in allr) / 1e9 / max(r["wt"] for r in allr)), 3)
                        if allr[0]["job_cpu"] and allr[0]["job_cpu"].get("cores_used") else None),
                    "cs_thread_cores_rank0": dict(sorted(allr[0]["thread_cores"].items(), key=lambda kv: -kv[1])),
                    "client_phase_p50_ms_rank0": allr[0]["phases"],
                    # rank 0's 20 slowest timed writes: step, op index and where the time went
                    "write_tail_rank0": allr[0]["slow_w"],
                    # node-wide /proc/vmstat deltas over rank 0's timed region (NUMA hinting faults /
                    # migrations, THP and compaction stalls that show up as a stalled copy)
                    "vmstat_timed_rank0": allr[0]["vm"],
                    **repl_phases(allr),
                }
                if a.remote_steps > 0:
                    rwl = sorted(x for r in allr for x in r["remote"]["wl"])
                    rrl = sorted(x for r in allr for x in r["remote"]["rl"])
                    rw = sum(r["remote"]["wbytes"] for r in allr) / (1 << 20) / max(r["remote"]["wt"] for r in allr)
                    rr = sum(r["remote"]["rbytes"] for r in allr) / (1 << 20) / max(r["remote"]["rt"] for r in allr)
                    result["remote_client"] = {
                        "steps": a.remote_steps,
                        "path": "gRPC/TCP for every master and chunkserver RPC (no shm, no UNIX sockets), " + (
                            "native C++ client (HTTP/2 on nghttp2)" if all(
                                r["remote"]["native_ops"] == r["remote"]["ops"] for r in allr) else
                            "Python grpcio client" if all(r["remote"]["native_ops"] == 0 for r in allr) else
                            "native C++ client with Python fallbacks"),
                        "native_client_ops": sum(r["remote"]["native_ops"] for r in allr),
                        "write_mb_per_s": round(rw, 2), "read_mb_per_s": round(rr, 2),
                        "mb_per_s": round((sum(r["remote"]["wbytes"] + r["remote"]["rbytes"] for r in allr) / (1 << 20))
                                          / max(r["remote"]["wt"] + r["remote"]["rt"] for r in allr), 2),
                        "write_p50_ms": round(pct(rwl, 50), 3), "write_p99_ms": round(pct(rwl, 99), 3),
                        "read_p50_ms": round(pct(rrl, 50), 3), "read_p99_ms": round(pct(rrl, 99), 3),
                        "client_phase_p50_ms_rank0": allr[0]["remote"].get("phases", {})}
                if a.stress_seconds > 0:
                    slat = sorted(x for r in allr for x in r["stress"]["lat"])
                    ops = sum(r["stress"]["ops"] for r in allr) / max(r["stress"]["seconds"] for r in allr)
                    result["stress_write"] = {
                        "seconds": a.stress_seconds, "size": a.stress_size, "concurrency_per_rank": a.stress_concurrency,
                        "ops_per_s": round(ops, 1), "mb_per_s": round(ops * a.stress_size / (1 << 20), 2),
                        "errors": sum(r["stress"]["errors"] for r in allr),
                        "first_error": next((r["stress"]["first_error"] for r in allr if r["stress"]["first_error"]), ""),
                        "avg_ms": round(1e3 * sum(slat) / max(1, len(slat)), 3), "p50_ms": round(pct(slat, 50), 3),
                        "p95_ms": round(pct(slat, 95), 3), "p99_ms": round(pct(slat, 99), 3),
                        "vs_published_470_ops_per_s": round(ops / 470.0, 1)}
            barrier()
            tpool.shutdown(wait=False)
            client.close()
            return result if rank == 0 else None
        finally:
            done.set()
            procs.stop()
            if rank == 0 and _should_clean(a, base):
                shutil.rmtree(base, ignore_errors=True)
            for d in extra_dirs:  # a rank's directory on another volume: always removed
                shutil.rmtree(d, ignore_errors=True)

    result = measure(a, a.transport)
    # transport A/B: on distinct GPUs, the other device transport runs a short
    # second measurement in the same job, so one JSON carries hipipc and RCCL side by side
    other = {"hipipc": "rccl", "rccl": "hipipc", "socket": "grpc"}.get(a.transport)
    ab = a.transport_ab == "on" or (a.transport_ab == "auto" and n > 1 and not a.cpu and visible_gpus() >= n)
    if ab and other:
        import copy

        b = copy.copy(a)
        b.steps, b.warmup, b.remote_steps, b.stress_seconds = min(a.steps, 10), 1, 0, 0.0
        b.profile_dir = None
        if rank == 0:
            pending.update(result)
        try:
            alt = measure(b, other, alt=True)
            if rank == 0:
                result["transport_ab"] = {other: {k: alt.get(k) for k in (
                    "value", "steps", "ms_per_step", "write_mb_per_s", "read_mb_per_s", "write_p50_ms", "write_p99_ms",
                    "read_p50_ms", "p2p_transport", "repl_pairs_up", "p2p_forwards", "rccl_forwards",
                    "p2p_fallbacks", "replica_failures")} | {"transport": alt["config"]["transport"]}}
        except Exception as e:  # noqa: BLE001 - the primary result stands either way
            if rank == 0:
                result["transport_ab"] = {other: {"error": f"{type(e).__name__}: {e}"[:500]}}
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        try:
            dist.barrier()
            dist.destroy_process_group()
        except Exception:  # noqa: BLE001
            pass


def repl_phases(allr) -> dict:
    """Mean microseconds per replica hop by phase, over every rank's chunkserver (empty when no
    hop went over the replication engine). Head: staging + checksum of a chained write, then
    its persist + fan-out; per device forward the descriptor round trip. Engine send side:
    channel turn, slice posts, the copies landing; receive side: turn + posts, landing (with
    the per-slice checksums), verify + index/persist."""
    def tot(k):
        return sum(r["cs"].get(k, 0) for r in allr)

    out = {}
    if tot("fp_chain_writes"):
        out["head_stage"] = tot("fp_chain_stage_ns") / tot("fp_chain_writes")
        out["head_forward"] = tot("fp_chain_forward_ns") / tot("fp_chain_writes")
    if tot("fp_desc_calls"):
        out["descriptor_rtt"] = tot("fp_desc_ns") / tot("fp_desc_calls")
    if tot("repl_send_calls"):
        for k in ("send_stage", "send_turn", "send_post"):
            out[k] = tot(f"repl_{k}_ns") / tot("repl_send_calls")
    if tot("repl_blocks_sent"):
        out["wait_send"] = tot("repl_wait_send_ns") / tot("repl_blocks_sent")
    if tot("repl_recv_calls"):
        for k in ("recv_turn", "recv_land", "recv_finish"):
            out[k] = tot(f"repl_{k}_ns") / tot("repl_recv_calls")
    return {"repl_phase_us": {k: round(v / 1e3, 1) for k, v in out.items()}} if out else {}


def forward_counts(allr) -> dict:
    """Replica hops as the chunkservers counted them (native fast path + gRPC service).
    p2p_forwards: hops over the replication engine, whatever its transport; rccl_forwards:
    the subset carried by RCCL itself (0 unless the engine's transport is rccl)."""
    def p2p(r):
        return r["cs"].get("fp_rccl_forwards", 0) + r["cs"].get("rccl_forwards", 0)

    return {
        "p2p_forwards": sum(p2p(r) for r in allr),
        "rccl_forwards": sum(p2p(r) for r in allr if r["p2p"] and r["p2p_transport"] == "rccl"),
        "shm_forwards": sum(r["cs"].get("fp_shm_forwards", 0) for r in allr),
        "grpc_forwards": sum(r["cs"].get("grpc_forwards", 0) for r in allr),
    }


def cgroup_cpu() -> dict | None:
    """CPU counters of this process's cgroup (v2 `cpu.stat` / `cpu.max`, else v1 cpuacct + cpu):
    usage and throttling cover every process of the job, chunkservers and masters included."""
    snap = {"t": time.perf_counter(), "cpus": len(os.sched_getaffinity(0))}

    def read(path):
        with open(path) as f:
            return f.read()

    try:  # cgroup v2
        rel = next((ln.split(":", 2)[2].strip() for ln in read("/proc/self/cgroup").splitlines()
                    if ln.startswith("0::")), "/")
        for base in ("/sys/fs/cgroup" + rel.rstrip("/"), "/sys/fs/cgroup"):
            if os.path.exists(base + "/cpu.stat") and os.path.exists(base + "/cpu.max"):
                st = dict(ln.split() for ln in read(base + "/cpu.stat").splitlines() if len(ln.split()) == 2)
                q, per = read(base + "/cpu.max").split()
                snap.update(usage_s=int(st["usage_usec"]) / 1e6, throttled_s=int(st.get("throttled_usec", 0)) / 1e6,
                            nr_throttled=int(st.get("nr_throttled", 0)),
                            quota_cores=None if q == "max" else round(int(q) / int(per), 2))
                return snap
        # cgroup v1: cpuacct usage (ns), cpu.stat throttled_time (ns), cfs quota
        snap["usage_s"] = int(read("/sys/fs/cgroup/cpuacct/cpuacct.usage")) / 1e9
        st = dict(ln.split() for ln in read("/sys/fs/cgroup/cpu/cpu.stat").splitlines() if len(ln.split()) == 2)
        snap.update(throttled_s=int(st.get("throttled_time", 0)) / 1e9, nr_throttled=int(st.get("nr_throttled", 0)))
        q = int(read("/sys/fs/cgroup/cpu/cpu.cfs_quota_us"))
        snap["quota_cores"] = None if q < 0 else round(q / int(read("/sys/fs/cgroup/cpu/cpu.cfs_period_us")), 2)
        return snap
    except (OSError, ValueError, KeyError):
        return snap if "usage_s" in snap else None


def cgroup_cpu_delta(c0: dict | None, c1: dict | None, elapsed: float) -> dict | None:
    if not c0 or not c1 or "usage_s" not in c0:
        return None
    out = {"cores_used": round((c1["usage_s"] - c0["usage_s"]) / elapsed, 2), "cpus_visible": c1["cpus"]}
    if "quota_cores" in c1:
        out["quota_cores"] = c1["quota_cores"]
    if "throttled_s" in c1:
        out["throttled_ms"] = round(1e3 * (c1["throttled_s"] - c0["throttled_s"]), 1)
        out["nr_throttled"] = c1["nr_throttled"] - c0["nr_throttled"]
    return out


def observed_transport(allr, n: int) -> str:
    """config.transport from what the replicas actually travelled over, not from flags: "local"
    (RF 1), "rccl" / "shm" / "grpc" when one path carried every hop, else "mixed(...)"."""
    if n <= 1:
        return "local"
    c = forward_counts(allr)
    c.pop("rccl_forwards")  # a subset of p2p_forwards
    p2p = {r["cs"].get("repl_transport") for r in allr} - {None}
    p2p_name = p2p.pop() if len(p2p) == 1 else "p2p"  # "socket" in CPU rehearsals
    used = {(p2p_name if k.startswith("p2p") else k.split("_")[0]): v for k, v in c.items() if v}
    if not used:
        return "none"
    if len(used) == 1:
        return next(iter(used))
    return "mixed(" + ",".join(f"{k}={v}" for k, v in sorted(used.items())) + ")"


def _bytes_needed(a, n: int) -> int:
    """Block bytes this run leaves on the node's volume (every replica of every file)."""
    rf = min(3, n)
    steps = a.steps + a.warmup + (a.remote_steps or 0)
    return n * rf * steps * a.count * (a.size + a.size // 128 + 4096)


_VMSTAT_KEYS = ("numa_hint_faults", "numa_hint_faults_local", "numa_pages_migrated", "pgmigrate_success",
                "pgmigrate_fail", "thp_fault_alloc", "compact_stall", "pgmajfault", "pgfault", "allocstall_normal",
                "pgscan_direct", "nr_dirty")


def _vmstat() -> dict:
    try:
        with open("/proc/vmstat") as f:
            return {k: int(v) for k, v in (ln.split() for ln in f) if k in _VMSTAT_KEYS}
    except (OSError, ValueError):
        return {}


JOURNAL_SEG_BYTES = 256 << 20
JOURNAL_READY_KEYS = ("parts_unready", "spares_missing", "grow_deferred", "segs", "segs_in_use", "full_waits")
# a 256 MiB segment = 8 parts of 32 MiB; a 1 MiB block's record is 1 MiB + 12 KiB (header and
# .meta page), 31 to a part: 96.8 % of a segment is block bytes
JOURNAL_SEG_DATA = int(JOURNAL_SEG_BYTES * 0.96)


def _journal_store_mode() -> bool:
    return os.environ.get("DFS_JOURNAL_EXPORT", "store") != "idle"


def _journal_segments(parent: Path, need: int, n: int) -> int:
    """Journal segments per chunkserver for this run.

    Store of record (default): the journal holds the run's replicas in about one copy's
    space and grows on demand; the returned count is how many segments each chunkserver
    prepares (creates and writes out once) before the timed region, so the timed appends
    overwrite written extents. Bounded by the volume (what does not fit is created on
    demand, never a per-file fallback). 0 = the chunkservers' default.

    Round-4 mode (DFS_JOURNAL_EXPORT=idle): a ring of segments recycled by the materializer,
    sized to hold the run below the 70 % mark; -1 = the ring cannot hold this run on this
    volume: the per-file path instead."""
    if os.environ.get("DFS_JOURNAL_SEGS") or os.environ.get("DFS_JOURNAL") or os.environ.get("DFS_JOURNAL_SPARES"):
        return 0
    try:
        free = shutil.disk_usage(parent).free
    except OSError:
        return 0
    per_cs = need // max(1, n)
    if _journal_store_mode():
        # + 2: the journal tops its spares up only in idle windows unless fewer than 2 are
        # free (DFS_JOURNAL_SPARES_LOW), so with two to spare no segment is created mid-run
        want = -(-per_cs // JOURNAL_SEG_DATA) + 2
        budget = (free - (4 << 30)) // max(1, n) // JOURNAL_SEG_BYTES
        return int(max(4, min(want, budget)))
    budget = (free - int(need * 1.15) - (2 << 30)) // max(1, n)
    # enough segments to hold the run below the materializer's 70 % mark, two spare
    want = -(-int(per_cs / 0.7) // JOURNAL_SEG_BYTES) + 2
    segs = int(max(3, min(64, want, budget // JOURNAL_SEG_BYTES)))
    if segs * JOURNAL_SEG_BYTES * 0.7 < per_cs:
        return -1
    return segs


_LOCAL_FS = {"ext4", "ext3", "xfs", "btrfs", "f2fs"}


def _data_volumes(default: Path) -> list[str]:
    """Writable directories on distinct local block devices, `default` (TMPDIR) first.

    DFS_BENCH_DIRS (comma-separated) names them explicitly; DFS_BENCH_SPREAD=0 keeps every rank
    on `default`. Otherwise every mounted local filesystem on another device that this user can
    write to (the mount point, or its tmp/ or $USER/ subdirectory) with at least 64 GiB free is
    added, one directory per device."""
    if os.environ.get("DFS_BENCH_DIRS"):
        return [p.strip() for p in os.environ["DFS_BENCH_DIRS"].split(",") if p.strip()]
    out = [str(default)]
    if os.environ.get("DFS_BENCH_SPREAD", "1") == "0":
        return out
    try:
        devs = {os.stat(default).st_dev}
        mounts = Path("/proc/mounts").read_text().splitlines()
    except OSError:
        return out
    skip = ("/proc", "/sys", "/dev", "/run", "/boot", "/etc", "/usr", "/snap", "/var/lib", "/root", "/home")
    for ln in mounts:
        f = ln.split()
        if len(f) < 3 or f[2] not in _LOCAL_FS or not f[0].startswith("/dev/"):
            continue
        mnt = f[1].replace("\\040", " ")
        if mnt == "/" or mnt.startswith(skip) or "sandbox" in mnt or "graft" in mnt:
            continue
        try:
            st = os.stat(mnt)
        except OSError:
            continue
        if st.st_dev in devs or not Path(mnt).is_dir():
            continue
        for c in (Path(mnt), Path(mnt) / "tmp", Path(mnt) / os.environ.get("USER", "-")):
            try:
                if c.is_dir() and os.access(c, os.W_OK | os.X_OK) and shutil.disk_usage(c).free >= (64 << 30):
                    devs.add(st.st_dev)
                    out.append(str(c))
                    break
            except OSError:
                continue
    return out


def _allocated_bytes(d: Path) -> int:
    tot = 0
    for root, _dirs, files in os.walk(d):
        for f in files:
            try:
                tot += os.lstat(os.path.join(root, f)).st_blocks * 512
            except OSError:
                pass
    return tot


def _free_bytes(d: Path) -> int:
    try:
        return shutil.disk_usage(d).free
    except OSError:
        return -1


def _make_room(parent: Path, need: int) -> None:
    """Reclaim earlier runs' data (oldest first) only when this run would not fit otherwise."""
    try:
        free = shutil.disk_usage(parent).free
    except OSError:
        return
    want = int(need * 1.15) + (2 << 30)
    if free >= want:
        return
    olds = sorted((d for d in parent.glob("dfs_bench_*") if (d / ".dfs_bench").exists()),
                  key=lambda d: d.stat().st_mtime)
    for d in olds:
        print(f"[bench] reclaiming {d} for {need >> 20} MiB of new data", file=sys.stderr, flush=True)
        shutil.rmtree(d, ignore_errors=True)
        if shutil.disk_usage(parent).free >= want:
            return


def _should_clean(a, base: str) -> bool:
    """Whether to delete this run's data directory at exit.

    Like `dfs_cli benchmark` (which never deletes what it wrote), the written blocks stay
    on disk by default while the volume keeps plenty of room: measured on the MI355X boxes
    (profiles/archive/r1_disk/keep_vs_delete.md), deleting a run's ~1 GB of fsynced 1 MiB files makes
    the NEXT durable-write run on the same overlay volume 1.4-2.4x slower for minutes, which
    would leak one run's cleanup into the next run's timed region. `--cleanup always` deletes
    anyway; `auto` deletes only when the disk is getting full (free < max(10 GiB, 10 %)), and
    a later run reclaims kept data itself if it would not fit (`_make_room`)."""
    if a.keep or a.cleanup == "never":
        return False
    if a.cleanup == "always":
        return True
    try:
        du = shutil.disk_usage(base)
    except OSError:
        return True
    return du.free < max(10 << 30, du.total // 10)


if __name__ == "__main__":
    main()
