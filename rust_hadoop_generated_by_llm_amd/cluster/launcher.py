"""Single-host multi-process cluster launcher — the replacement for the reference's
docker-compose topologies (C60; docker-compose.yml, docker-compose.auto-scaling.yml).

One process per role: config server(s), one master per shard (or a Raft group per shard),
and one ChunkServer per GPU (``gpus=[0..7]``) or CPU ChunkServers (``gpus=None``). All
ports are picked free at start; readiness is signalled through ``DFS_READY_FILE``.
Used by the tests, ``bench.py`` and ``dfs_cli cluster up``.
"""
from __future__ import annotations

import json
import os
import shutil
import signal
import random
import socket
import subprocess
import sys
import tempfile
import time
from dataclasses import dataclass, field
from pathlib import Path

PKG = "rust_hadoop_generated_by_llm_amd"
ROOT = Path(__file__).resolve().parents[2]


_handed_out: set[int] = set()

# Roles that run as native executables (csrc/tools/dfs_master.cpp, dfs_config_server.cpp,
# dfs_chunkserver.cpp, dfs_s3_gateway.cpp): no Python interpreter lives in a master,
# config-server, chunkserver or gateway process. The Python chunkserver shell and S3 gateway
# are test models under tests/models/ (the interop and A/B tests ask for them with the knobs
# below); the product has no Python form of these roles.
NATIVE_BINARIES = {"master.server": "dfs_master", "config_server.server": "dfs_config_server",
                   "chunkserver.server": "dfs_chunkserver", "s3.server": "dfs_s3_gateway"}
TEST_MODELS = {"chunkserver.server": "tests.models.chunkserver_shell", "s3.server": "tests.models.s3_gateway"}


def _model_gateway(env) -> bool:
    """Tests asking for the Python gateway model (S3_NATIVE_GATEWAY=0)."""
    return env.get("S3_NATIVE_GATEWAY", "1") == "0"


def _model_chunkserver(args: list[str], env) -> bool:
    """Tests asking for the Python chunkserver model (its grpcio server stack, its own paths)."""
    return (env.get("DFS_NATIVE_CHUNKSERVER", "1") == "0" or env.get("DFS_CS_GRPC", "native") != "native"
            or env.get("DFS_CS_AGENT", "native") != "native" or "--no-fastpath" in args
            or any(a.startswith("--grpc-impl") and (a.endswith("grpcio") or a == "--grpc-impl") for a in args))


def role_command(module: str, args: list[str], environ: dict | None = None) -> list[str]:
    """argv for a role: its native executable, or (tests only) the Python model under tests/models."""
    env = os.environ if environ is None else environ
    exe = ROOT / "build" / "native" / NATIVE_BINARIES.get(module, "-")
    model = (module == "chunkserver.server" and _model_chunkserver(args, env)) or \
            (module == "s3.server" and _model_gateway(env))
    if model:
        if not (ROOT / "tests" / "models").is_dir():
            raise RuntimeError(f"{module}: the Python model is a test fixture (tests/models), not installed")
        return [sys.executable, "-m", TEST_MODELS[module], *args]
    if module in NATIVE_BINARIES:
        if not exe.exists():
            raise FileNotFoundError(f"{exe} is not built (python build_native.py)")
        return [str(exe), *args]
    return [sys.executable, "-m", f"{PKG}.{module}", *args]


def free_port() -> int:
    """A port nothing listens on, below the kernel's ephemeral range (32768+) so that no
    outgoing connection takes it before its server binds, and never the same one twice in a
    process (a port closed here is otherwise free to come back on the next call)."""
    for _ in range(200):
        p = random.randint(15000, 32000)
        if p in _handed_out:
            continue
        with socket.socket() as s:
            try:
                s.bind(("127.0.0.1", p))
            except OSError:
                continue
        _handed_out.add(p)
        return p
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@dataclass
class Proc:
    name: str
    popen: subprocess.Popen
    ready_file: str
    info: dict = field(default_factory=dict)
    log_path: str = ""
    module: str = ""
    args: list = field(default_factory=list)
    extra_env: dict | None = None


class LocalCluster:
    def __init__(self, base_dir: str | None = None, *, n_chunkservers: int = 1, gpus: list[int] | None = None,
                 shards: int = 1, masters_per_shard: int = 1, config_server: bool = False,
                 durability: str = "nvme-sync", fsync: bool = True, rccl: bool = True,
                 hbm_capacity: str = "0", heartbeat_interval: float = 0.5, scrub_interval: float = 60.0,
                 rack_ids: list[str] | None = None, fast_intervals: bool = False, cold_dir: bool = False,
                 env: dict | None = None, master_args: list[str] | None = None, cs_args: list[str] | None = None,
                 tls: bool = False, standby_masters: int = 0, p2p: str | None = None):
        self.owns_dir = base_dir is None
        self.base = Path(base_dir or tempfile.mkdtemp(prefix="dfs_cluster_"))
        self.base.mkdir(parents=True, exist_ok=True)
        self.gpus = gpus
        self.n_cs = len(gpus) if gpus is not None else n_chunkservers
        self.shards = shards
        self.masters_per_shard = masters_per_shard
        self.use_config = config_server or shards > 1
        self.durability = durability
        self.fsync = fsync
        self.rccl = rccl
        # "socket": native replication engine over the host-memory P2P transport (CPU tests of
        # the same protocol the device transports run); "hipipc" / "hipipc-spin": the device
        # transport between chunkserver processes (works with several of them on one GPU);
        # None: RCCL with GPUs, reference gRPC without
        self.p2p = p2p
        self.hbm_capacity = hbm_capacity
        self.heartbeat_interval = heartbeat_interval
        self.scrub_interval = scrub_interval
        self.rack_ids = rack_ids
        self.fast_intervals = fast_intervals
        self.standby_masters = standby_masters
        self.standby_addrs: list[str] = []
        self.cold_dir = cold_dir
        self.env = dict(os.environ)
        self.env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        self.env["PYTHONPATH"] = str(ROOT) + os.pathsep + self.env.get("PYTHONPATH", "")
        self.env.setdefault("DFS_LOG", "warning")
        if env:
            self.env.update(env)
        self.master_args = master_args or []
        self.cs_args = cs_args or []
        self.tls = tls
        self.ca_cert: str | None = None
        self.procs: list[Proc] = []
        self.config_addrs: list[str] = []
        self.shard_masters: dict[str, list[str]] = {}
        self.master_http: dict[str, str] = {}
        self.cs_addrs: list[str] = []
        self.cs_http: list[str] = []

    # ------------------------------------------------------------------ process helpers
    def _spawn(self, name: str, module: str, args: list[str], extra_env: dict | None = None) -> Proc:
        ready = str(self.base / f"{name}.ready")
        if os.path.exists(ready):
            os.unlink(ready)
        env = dict(self.env)
        env["DFS_READY_FILE"] = ready
        if extra_env:
            env.update(extra_env)
        log_path = str(self.base / f"{name}.log")
        logf = open(log_path, "ab")
        p = subprocess.Popen(role_command(module, args, env), env=env, stdout=logf,
                             stderr=subprocess.STDOUT, cwd=str(ROOT), start_new_session=True)
        logf.close()
        proc = Proc(name, p, ready, log_path=log_path, module=module, args=list(args), extra_env=extra_env)
        self.procs.append(proc)
        return proc

    def _wait_ready(self, procs: list[Proc], timeout: float = 180.0) -> None:
        deadline = time.time() + timeout
        for pr in procs:
            while not os.path.exists(pr.ready_file):
                if pr.popen.poll() is not None:
                    raise RuntimeError(f"{pr.name} exited with {pr.popen.returncode}:\n{self.tail(pr)}")
                if time.time() > deadline:
                    raise TimeoutError(f"{pr.name} not ready after {timeout}s:\n{self.tail(pr)}")
                time.sleep(0.05)
            with open(pr.ready_file) as f:
                try:
                    pr.info = json.load(f)
                except ValueError:
                    pr.info = {}

    @staticmethod
    def tail(pr: Proc, n: int = 40) -> str:
        try:
            with open(pr.log_path, errors="replace") as f:
                return "".join(f.readlines()[-n:])
        except OSError:
            return ""

    # ------------------------------------------------------------------ lifecycle
    def start(self) -> "LocalCluster":
        try:
            self._start()
        except Exception:
            self.stop()
            raise
        return self

    def make_certs(self) -> tuple[str, str, str]:
        """Self-signed CA + a server certificate for 127.0.0.1/localhost (openssl CLI)."""
        d = self.base / "tls"
        d.mkdir(exist_ok=True)
        ca_key, ca, key, csr, crt = (str(d / n) for n in ("ca.key", "ca.pem", "server.key", "server.csr", "server.pem"))
        ext = d / "san.cnf"
        ext.write_text("subjectAltName=IP:127.0.0.1,DNS:localhost\nbasicConstraints=CA:FALSE\n")
        run = lambda *a: subprocess.run(["openssl", *a], check=True, capture_output=True)  # noqa: E731
        run("req", "-x509", "-newkey", "rsa:2048", "-nodes", "-keyout", ca_key, "-out", ca, "-days", "2",
            "-subj", "/CN=dfs-test-ca")
        run("req", "-newkey", "rsa:2048", "-nodes", "-keyout", key, "-out", csr, "-subj", "/CN=localhost")
        run("x509", "-req", "-in", csr, "-CA", ca, "-CAkey", ca_key, "-CAcreateserial", "-out", crt, "-days", "2",
            "-extfile", str(ext))
        return ca, crt, key

    def _start(self) -> None:
        fs = [] if self.fsync else ["--no-fsync"]
        tls_args: list[str] = []
        if self.tls:
            ca, crt, key = self.make_certs()
            self.ca_cert = ca
            tls_args = ["--tls-cert", crt, "--tls-key", key, "--ca-cert", ca]
        if self.use_config:
            port, http = free_port(), free_port()
            pr = self._spawn("config", "config_server.server", [
                "--addr", f"127.0.0.1:{port}", "--http-port", str(http), "--storage-dir",
                str(self.base / "config"), *fs])
            self._wait_ready([pr])
            self.config_addrs = [f"http://127.0.0.1:{port}"]
            self.config_http = f"http://127.0.0.1:{http}"
        # masters
        shard_cfg: dict[str, list[str]] = {}
        plans = []
        for s in range(self.shards):
            sid = f"shard-{s}"
            ids = list(range(1, self.masters_per_shard + 1))
            ports = {i: (free_port(), free_port()) for i in ids}
            shard_cfg[sid] = [f"http://127.0.0.1:{ports[i][0]}" for i in ids]
            plans.append((sid, ids, ports))
        shard_file = self.base / "shard_config.json"
        shard_file.write_text(json.dumps({"shards": shard_cfg}))
        mprocs = []
        for sid, ids, ports in plans:
            for i in ids:
                gport, hport = ports[i]
                peers = ",".join(f"{j}@http://127.0.0.1:{ports[j][1]}" for j in ids if j != i)
                args = ["--addr", f"127.0.0.1:{gport}", "--id", str(i), "--http-port", str(hport),
                        "--storage-dir", str(self.base / f"master_{sid}"), "--shard-id", sid, *fs, *tls_args,
                        *self.master_args]
                if peers:
                    args += ["--peers", peers]
                if self.use_config:
                    args += ["--config-servers", ",".join(self.config_addrs)]
                else:
                    args += ["--shard-config", str(shard_file)]
                if self.fast_intervals:
                    args.append("--fast-intervals")
                mprocs.append(self._spawn(f"master_{sid}_{i}", "master.server", args))
                self.master_http[f"http://127.0.0.1:{gport}"] = f"http://127.0.0.1:{hport}"
        for i in range(self.standby_masters if self.use_config else 0):
            gport, hport = free_port(), free_port()
            args = ["--addr", f"127.0.0.1:{gport}", "--id", "1", "--http-port", str(hport), "--storage-dir",
                    str(self.base / f"master_standby{i}"), "--standby", "--config-servers", ",".join(self.config_addrs),
                    *fs, *tls_args, *self.master_args]
            if self.fast_intervals:
                args.append("--fast-intervals")
            mprocs.append(self._spawn(f"master_standby{i}", "master.server", args))
            self.standby_addrs.append(f"http://127.0.0.1:{gport}")
            self.master_http[f"http://127.0.0.1:{gport}"] = f"http://127.0.0.1:{hport}"
        self._wait_ready(mprocs)
        self.shard_masters = shard_cfg
        # chunkservers
        rdv = self.base / "rccl_rendezvous"
        if rdv.exists():
            shutil.rmtree(rdv)
        cprocs = []
        for i in range(self.n_cs):
            port, http = free_port(), free_port()
            gpu = self.gpus[i] if self.gpus is not None else -1
            args = ["--addr", f"127.0.0.1:{port}", "--http-port", str(http),
                    "--storage-dir", str(self.base / f"cs{i}"), "--gpu", str(gpu),
                    "--durability", self.durability, "--hbm-capacity", self.hbm_capacity,
                    "--heartbeat-interval", str(self.heartbeat_interval),
                    "--scrub-interval", str(self.scrub_interval), *fs, *tls_args, *self.cs_args]
            if self.cold_dir:
                args += ["--cold-storage-dir", str(self.base / f"cs{i}_cold")]
            if self.rack_ids:
                args += ["--rack-id", self.rack_ids[i % len(self.rack_ids)]]
            if self.use_config:
                args += ["--config-servers", ",".join(self.config_addrs)]
            else:
                args += ["--masters", ",".join(m for ms in shard_cfg.values() for m in ms)]
            if self.p2p in ("socket", "hipipc", "hipipc-spin") and self.n_cs > 1:
                args += ["--rccl-rank", str(i), "--rccl-world", str(self.n_cs), "--rccl-rendezvous", str(rdv),
                         "--replication-transport", self.p2p, "--rccl-timeout-ms", "10000",
                         "--repl-turn-timeout-ms", "1500"]
            elif self.gpus is not None and self.n_cs > 1 and self.rccl:
                args += ["--rccl-rank", str(i), "--rccl-world", str(self.n_cs), "--rccl-rendezvous", str(rdv),
                         "--replication-transport", "rccl"]
            else:
                args += ["--replication-transport", "grpc"]
            cprocs.append(self._spawn(f"cs{i}", "chunkserver.server", args))
            self.cs_addrs.append(f"127.0.0.1:{port}")
            self.cs_http.append(f"http://127.0.0.1:{http}")
        self._wait_ready(cprocs)
        self.wait_registered()
        if self.n_cs > 1 and (self.p2p in ("socket", "hipipc", "hipipc-spin") or (self.gpus is not None and self.rccl)):
            self.wait_replication_mesh()
        if self.shards > 1:
            self.wait_shard_maps()

    def wait_replication_mesh(self, timeout: float = 60.0) -> None:
        """Block until every chunkserver reports every peer pair up. A chunkserver writes its
        ready file once ITS side of each pair is connected; the peer's side of the last pair can
        still be finishing then, so /stats may briefly show one pair short."""
        import urllib.request

        want = self.n_cs - 1
        deadline = time.time() + timeout
        seen: list = []
        while time.time() < deadline:
            seen = []
            for http in self.cs_http:
                try:
                    with urllib.request.urlopen(http + "/stats", timeout=2.0) as r:
                        seen.append(json.loads(r.read()).get("repl_pairs_up"))
                except OSError:
                    seen.append(None)
            if all(v == want for v in seen):
                return
            time.sleep(0.2)
        raise TimeoutError(f"replication mesh not up after {timeout}s: pairs per chunkserver {seen}")

    def wait_shard_maps(self, timeout: float = 30.0) -> None:
        """Block until every master's shard map lists every shard (maps propagate from the
        config server by polling; a master with a stale map would misroute renames)."""
        import urllib.request

        want = set(self.shard_masters)
        deadline = time.time() + timeout
        for http in self.master_http.values():
            while True:
                try:
                    with urllib.request.urlopen(f"{http}/shard_map", timeout=2) as r:
                        have = set(json.load(r)["map"].get("shards", []))
                    if have >= want:
                        break
                except OSError:
                    pass
                if time.time() > deadline:
                    raise TimeoutError(f"master {http} never learned all shards {sorted(want)}")
                time.sleep(0.05)

    def start_s3(self, env: dict | None = None, name: str = "s3") -> str:
        """Start an S3 gateway process against this cluster; returns its endpoint URL."""
        port = free_port()
        e = {"PORT": str(port), "MASTER_ADDR": self.master_addrs[0],
             "AUDIT_LOG_DIR": str(self.base / f"{name}_audit")}
        if self.use_config:
            e["CONFIG_SERVERS"] = ",".join(self.config_addrs)
        else:
            e["SHARD_CONFIG"] = str(self.base / "shard_config.json")
        e.update(env or {})
        pr = self._spawn(name, "s3.server", [], e)
        self._wait_ready([pr])
        return f"http://127.0.0.1:{port}"

    @property
    def master_addrs(self) -> list[str]:
        return [m for ms in self.shard_masters.values() for m in ms]

    def client(self, **kw):
        from ..client.client import Client

        if self.tls:
            kw.setdefault("ca_cert", self.ca_cert)
        c = Client(self.master_addrs, self.config_addrs, **kw)
        if not self.use_config:
            from ..parallel.sharding import ShardMap

            c.set_shard_map(ShardMap.from_config(self.shard_masters))
        else:
            c.refresh_shard_map()
        return c

    def wait_registered(self, timeout: float = 60.0) -> None:
        """Block until every master leader has seen every chunkserver and left safe mode."""
        import grpc

        from ..models import proto as pb
        from ..utils.rpc import ChannelPool

        pool = ChannelPool(self.ca_cert)
        deadline = time.time() + timeout
        try:
            for sid, masters in self.shard_masters.items():
                while True:
                    ok = False
                    for m in masters:
                        try:
                            st = pool.call(m, "MasterService", "GetSafeModeStatus", pb.GetSafeModeStatusRequest(),
                                           timeout=2.0)
                            if st.chunk_server_count >= self.n_cs and not st.is_safe_mode:
                                ok = True
                                break
                        except grpc.RpcError:
                            pass
                    if ok:
                        break
                    if time.time() > deadline:
                        raise TimeoutError(f"shard {sid} never saw {self.n_cs} chunkservers")
                    time.sleep(0.1)
        finally:
            pool.close()

    def kill(self, name: str, sig: int = signal.SIGKILL) -> None:
        for pr in self.procs:
            if pr.name == name and pr.popen.poll() is None:
                try:
                    os.killpg(pr.popen.pid, sig)
                except ProcessLookupError:
                    pass
                pr.popen.wait(timeout=30)

    def restart(self, name: str, sig: int = signal.SIGKILL, before_start=None) -> Proc:
        """Kill process `name` (SIGKILL by default: a crash, nothing flushed) and start it again
        with the same arguments and storage; returns once it signalled ready again.
        `before_start` runs while it is down (e.g. to damage its files)."""
        old = next(pr for pr in self.procs if pr.name == name)
        self.kill(name, sig)
        self.procs.remove(old)
        if before_start is not None:
            before_start()
        pr = self._spawn(name, old.module, old.args, old.extra_env)
        self._wait_ready([pr])
        return pr

    def stop(self) -> None:
        # DFS_KEEP_LOGS=<dir>: every process's log (and the exit status of any that died before
        # the stop) survives the cluster's scratch directory, for post-mortems of benchmark runs
        keep = os.environ.get("DFS_KEEP_LOGS")
        died = {pr.name: pr.popen.returncode for pr in self.procs if pr.popen.poll() is not None}
        for pr in reversed(self.procs):
            if pr.popen.poll() is None:
                try:
                    os.killpg(pr.popen.pid, signal.SIGTERM)
                except ProcessLookupError:
                    pass
        deadline = time.time() + 20
        for pr in self.procs:
            try:
                pr.popen.wait(timeout=max(0.1, deadline - time.time()))
            except subprocess.TimeoutExpired:
                try:
                    os.killpg(pr.popen.pid, signal.SIGKILL)
                except ProcessLookupError:
                    pass
                pr.popen.wait(timeout=10)
        if keep:
            os.makedirs(keep, exist_ok=True)
            for pr in self.procs:
                if pr.log_path and os.path.exists(pr.log_path):
                    shutil.copy(pr.log_path, os.path.join(keep, os.path.basename(pr.log_path)))
            with open(os.path.join(keep, "exited_before_stop.json"), "w") as f:
                json.dump(died, f)
        self.procs = []
        if self.owns_dir:
            shutil.rmtree(self.base, ignore_errors=True)

    def __enter__(self):
        return self.start()

    def __exit__(self, *exc):
        self.stop()
