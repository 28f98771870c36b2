"""TEST MODEL (not part of the product): the Python chunkserver shell (grpcio server + Python
control loop over the native store), kept for the interop tests against a grpcio server
stack. The product's chunkserver process is dfs_chunkserver (csrc/tools/dfs_chunkserver.cpp).

``dfs_chunkserver --gpu <i>`` — one ChunkServer process per MI355X (C43; reference
dfs/chunkserver/src/bin/chunkserver.rs).

Startup: HBM ChunkStore on GPU i (or the CPU store with ``--gpu -1``), optional RCCL
replication rank (``--rccl-rank/--rccl-world/--rccl-rendezvous``), gRPC server, HTTP
/health + /metrics, a 5 s heartbeat loop to every master of every shard (stats, bad
blocks, commands, master term) and the 60 s scrubber."""
from __future__ import annotations

import argparse
import json
import logging
import os
import shutil
import signal
import threading
import time
import uuid
import zlib
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from pathlib import Path

from rust_hadoop_generated_by_llm_amd.models import proto as pb
from rust_hadoop_generated_by_llm_amd.native import lib as native
from rust_hadoop_generated_by_llm_amd.native import require_gpu
from rust_hadoop_generated_by_llm_amd.parallel.sharding import ShardMap
from rust_hadoop_generated_by_llm_amd.utils import log as logsetup
from rust_hadoop_generated_by_llm_amd.utils.metrics import Registry
from rust_hadoop_generated_by_llm_amd.utils.rpc import (ChannelPool, RpcStatus, current_request_id, make_sync_server, rpc_details,
                         server_credentials, snake, strip_scheme, with_scheme)
from tests.models.chunkserver_service import ChunkServer

log = logging.getLogger("dfs.chunkserver")


def build_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser("dfs_chunkserver", description="DFS ChunkServer (one per GPU)")
    p.add_argument("--addr", default="127.0.0.1:50052")
    p.add_argument("--config-servers", default="")
    p.add_argument("--storage-dir", default="/tmp/chunkserver_data")
    p.add_argument("--cold-storage-dir", default="")
    p.add_argument("--advertise-addr", default=None)
    p.add_argument("--http-port", type=int, default=8082)
    p.add_argument("--tls-cert")
    p.add_argument("--tls-key")
    p.add_argument("--ca-cert")
    p.add_argument("--domain-name")
    p.add_argument("--rack-id", default="")
    # MI355X-native build additions
    p.add_argument("--masters", default="", help="static master list when no shard map/config server")
    p.add_argument("--gpu", type=int, default=-1, help="HIP device for the HBM store (-1 = CPU store)")
    p.add_argument("--hbm-capacity", default="0", help="arena bytes (suffix K/M/G ok); 0 = auto")
    p.add_argument("--durability", choices=["nvme-sync", "hbm-ack"], default="nvme-sync")
    p.add_argument("--lanes", type=int, default=16)
    p.add_argument("--rccl-rank", type=int, default=-1)
    p.add_argument("--rccl-world", type=int, default=0)
    p.add_argument("--rccl-rendezvous", default="")
    p.add_argument("--rccl-timeout-ms", type=int, default=60000)
    p.add_argument("--replication-transport", choices=["hipipc", "hipipc-spin", "rccl", "grpc", "socket"],
                   default="hipipc",
                   help="payload path between same-node chunkservers: hipipc (HIP IPC one-sided copies into the "
                        "peer's HBM over xGMI; no kernel ever waits on a peer), hipipc-spin (the same with RCCL-like "
                        "spinning p2p kernels, for tests), rccl (ncclSend/ncclRecv), grpc (reference), socket "
                        "(host-memory P2P transport used by the CPU tests)")
    p.add_argument("--repl-turn-timeout-ms", type=int, default=3000,
                   help="how long a replica waits for an earlier sequence number before failing the pair")
    p.add_argument("--heartbeat-interval", type=float, default=5.0)
    p.add_argument("--scrub-interval", type=float, default=60.0)
    p.add_argument("--no-fsync", action="store_true", help="skip fdatasync (tests only)")
    p.add_argument("--workers", type=int, default=64)
    p.add_argument("--no-fastpath", action="store_true", help="disable the native local UNIX-socket data path")
    p.add_argument("--grpc-impl", choices=["native", "grpcio"], default=os.environ.get("DFS_CS_GRPC", "native"),
                   help="ChunkServerService transport: native HTTP/2 gRPC (nghttp2, C++ data RPCs, Python "
                        "handlers for the rest) or Python grpcio for everything")
    return p


def parse_size(s: str) -> int:
    s = str(s).strip().upper()
    mult = {"K": 1 << 10, "M": 1 << 20, "G": 1 << 30, "T": 1 << 40}
    if s and s[-1] in mult:
        return int(float(s[:-1]) * mult[s[-1]])
    return int(s)


def rendezvous_ranks(d: str, rank: int, world: int, addr: str, timeout: float = 120.0,
                     fastpath: str = "") -> tuple[dict[str, int], dict[str, str]]:
    """Publish our advertise address (and native fast-path socket) for our rank and wait
    for every rank's. Returns ({addr: rank}, {addr: fast-path socket name})."""
    Path(d).mkdir(parents=True, exist_ok=True)
    tmp = Path(d) / f".addr_{rank}.tmp"
    tmp.write_text(addr + ("\n" + fastpath if fastpath else ""))
    os.replace(tmp, Path(d) / f"addr_{rank}")
    deadline = time.time() + timeout
    out: dict[str, int] = {}
    names: dict[str, str] = {}
    while time.time() < deadline:
        out, names = {}, {}
        for r in range(world):
            f = Path(d) / f"addr_{r}"
            if f.exists():
                lines = f.read_text().split("\n")
                a = strip_scheme(lines[0].strip())
                out[a] = r
                if len(lines) > 1 and lines[1].strip():
                    names[a] = lines[1].strip()
        if len(out) == world:
            return out, names
        time.sleep(0.05)
    raise TimeoutError(f"rendezvous: only {len(out)}/{world} chunkservers published in {d}")


class ChunkServerProcess:
    def __init__(self, args):
        self.args = args
        # chunkserver addresses travel scheme-less, as in the reference (clients prepend http://)
        self.advertise = strip_scheme(args.advertise_addr or args.addr)
        if args.gpu >= 0:
            require_gpu(args.gpu)
        self.store = native.ChunkStore(
            args.storage_dir, args.cold_storage_dir, args.gpu, parse_size(args.hbm_capacity),
            0 if args.durability == "nvme-sync" else 1, int(os.environ.get("BLOCK_CACHE_SIZE", "100")),
            args.lanes, 4, not args.no_fsync)
        self.pool = ChannelPool(args.ca_cert, args.domain_name)
        self.config_servers = [with_scheme(c) for c in args.config_servers.split(",") if c.strip()]
        self.static_masters = [with_scheme(m) for m in args.masters.split(",") if m.strip()]
        shard_cfg = os.environ.get("SHARD_CONFIG")
        self.shard_map = ShardMap.load_config_file(shard_cfg) if shard_cfg else ShardMap.new_range()
        self.fastpath = None
        if not args.no_fastpath:
            port = strip_scheme(args.addr).rsplit(":", 1)[-1]
            # deterministic name: same-host peers find each other from the advertised port
            fp = native.FastPathServer(self.store, f"dfs_fp_{port}")
            ok, err = fp.start()
            if ok:
                fp.set_self_host(self.advertise.rsplit(":", 1)[0])
                fp.set_self_addr(self.advertise)
                self.fastpath = fp
            else:
                log.warning("native fast path disabled: %s", err)
        self.rccl = None  # the replication engine (RCCL over xGMI, or sockets in CPU tests)
        self.repl_pairs_up = 0
        rank_map: dict[str, int] = {}
        transport = args.replication_transport
        if (transport in ("hipipc", "hipipc-spin", "rccl", "socket") and args.rccl_world > 1 and args.rccl_rank >= 0
                and args.rccl_rendezvous and (args.gpu >= 0 or transport == "socket")):
            if self.fastpath is None:
                log.error("replication engine needs the native fast path (pair control); using gRPC replication")
            else:
                rank_map, fp_names = rendezvous_ranks(args.rccl_rendezvous, args.rccl_rank, args.rccl_world,
                                                      self.advertise, fastpath=self.fastpath.name)
                ns = "%08x" % (zlib.crc32(os.path.abspath(args.rccl_rendezvous).encode()) & 0xFFFFFFFF)
                try:
                    eng = native.ReplicationEngine(self.store, transport, args.rccl_rank, args.rccl_world, ns=ns,
                                                   open_timeout_ms=args.rccl_timeout_ms,
                                                   turn_timeout_ms=args.repl_turn_timeout_ms,
                                                   xfer_timeout_ms=min(args.rccl_timeout_ms, 20000))
                except RuntimeError as e:
                    log.error("replication engine unavailable (%s); using gRPC replication", e)
                else:
                    self.rccl = eng
                    for a, r in rank_map.items():
                        if r != args.rccl_rank:
                            self.fastpath.set_peer(a, r, fp_names.get(a, ""))
                    self.fastpath.set_replication(eng)
                    eng.start()
                    # pairs come up in the background; wait a bounded time so a benchmark starts
                    # with its channels ready (a pair that is not up just falls back per block)
                    self.repl_pairs_up = eng.wait_ready(args.rccl_timeout_ms)
                    log.info("%s replication: rank %d/%d, %d/%d pairs up", transport, args.rccl_rank,
                             args.rccl_world, self.repl_pairs_up, args.rccl_world - 1)
        self.native_grpc = None
        self.metrics = Registry()
        self.cs = ChunkServer(self.store, self.advertise, self.pool, self.masters, self.rccl, rank_map,
                              args.rccl_rank, self.metrics, fastpath=self.fastpath)
        self.agent = None
        if self.fastpath is not None and os.environ.get("DFS_CS_AGENT", "native") == "native":
            # heartbeat, the masters' commands, recovery and the scrubber run natively
            # (csrc/cs_agent.cpp); the Python loops below stay as the DFS_CS_AGENT=python A/B
            self.agent = native.CsAgent(
                self.store, self.fastpath, self.advertise, rack_id=args.rack_id, storage_dir=args.storage_dir,
                gpu_rank=args.rccl_rank, masters=[strip_scheme(m) for m in self.masters()],
                config_servers=[strip_scheme(c) for c in self.config_servers],
                heartbeat_interval=args.heartbeat_interval, scrub_interval=args.scrub_interval,
                ca_cert=args.ca_cert or "", domain_name=args.domain_name or "", tls=bool(args.tls_cert))
            self.cs.agent = self.agent
        self._setup_metrics()
        self._stop = threading.Event()

    # ------------------------------------------------------------------ helpers
    def masters(self) -> list[str]:
        if getattr(self, "agent", None) is not None:  # the native loop keeps the shard map fresh
            ms = self.agent.masters()
            if ms:
                return [with_scheme(m) for m in ms]
        ms = self.shard_map.get_all_masters()
        return [with_scheme(m) for m in ms] if ms else self.static_masters

    def disk_stats(self) -> tuple[int, int]:
        du = shutil.disk_usage(self.args.storage_dir)
        return du.total - du.free, du.free

    def _setup_metrics(self) -> None:
        m = self.metrics
        m.gauge("dfs_chunkserver_available_space_bytes", "free bytes on the storage fs", fn=lambda: self.disk_stats()[1])
        m.gauge("dfs_chunkserver_used_space_bytes", "used bytes on the storage fs", fn=lambda: self.disk_stats()[0])
        m.gauge("dfs_chunkserver_total_chunks", "blocks held", fn=lambda: self.store.stats()["blocks"])
        for k in ("hbm_capacity", "hbm_used", "hbm_resident_blocks", "dirty_blocks", "spill_queue", "evictions",
                  "promotions", "crc_mismatches", "gpu_kernel_launches", "disk_gate_waits"):
            m.gauge(f"dfs_chunkserver_{k}", f"chunk store {k}", fn=lambda k=k: self.store.stats()[k])
        m.gauge("dfs_chunkserver_rccl_bytes_sent", "bytes replicated over RCCL",
                fn=lambda: self.rccl.bytes_sent if self.rccl else 0)
        m.gauge("dfs_chunkserver_rccl_bytes_recv", "bytes received over RCCL",
                fn=lambda: self.rccl.bytes_recv if self.rccl else 0)
        for k in self.cs.stats:
            m.gauge(f"dfs_chunkserver_{k}_total", k, fn=lambda k=k: self.cs.stats[k])

    def refresh_shard_map(self) -> bool:
        for c in self.config_servers:
            try:
                r = self.pool.call(c, "ConfigService", "FetchShardMap", pb.FetchShardMapRequest(), timeout=5.0)
                new = ShardMap.from_fetch(r)
                sm = self.shard_map
                sm.strategy, sm.ranges, sm.ring, sm.shards, sm.shard_peers = (
                    new.strategy, new.ranges, new.ring, new.shards, new.shard_peers)
                sm._dirty()
                return True
            except Exception as e:  # noqa: BLE001
                log.debug("FetchShardMap from %s failed: %s", c, rpc_details(e))
        return False

    def heartbeat_once(self) -> None:
        if self.config_servers:
            self.refresh_shard_map()
        used, avail = self.disk_stats()
        st = self.store.stats()
        if self.fastpath is not None:
            for bid in self.fastpath.drain_suspects():  # partial-read corruption seen natively
                self.cs.queue_recovery(bid)
        bad, new, enc, fail, rebuilt = self.cs.drain_reports()
        req = pb.HeartbeatRequest(chunk_server_address=self.advertise, used_space=used, available_space=avail,
                                  chunk_count=st["blocks"], bad_blocks=bad, rack_id=self.args.rack_id,
                                  gpu_rank=self.args.rccl_rank, hbm_capacity=st["hbm_capacity"],
                                  hbm_used=st["hbm_used"], new_blocks=new, ec_encoded=enc,
                                  ec_failed=fail, ec_rebuilt=rebuilt)
        for m in self.masters():
            try:
                r = self.pool.call(m, "MasterService", "Heartbeat", req, timeout=5.0)
            except Exception as e:  # noqa: BLE001
                log.debug("heartbeat to %s failed: %s", m, rpc_details(e))
                continue
            self.cs.adopt_term(r.master_term)
            for cmd in r.commands:
                self.cs.handle_command(cmd)

    def _heartbeat_loop(self) -> None:
        if self.config_servers:
            while not self._stop.is_set() and not self.refresh_shard_map():
                self._stop.wait(2.0)
        while not self._stop.is_set():
            try:
                self.heartbeat_once()
            except Exception:  # noqa: BLE001
                log.exception("heartbeat failed")
            self._stop.wait(self.args.heartbeat_interval)

    def _scrub_loop(self) -> None:
        while not self._stop.wait(self.args.scrub_interval):
            try:
                bad = self.cs.scrub_once()
                if bad:
                    log.warning("scrubber found %d corrupt block(s)", len(bad))
            except Exception:  # noqa: BLE001
                log.exception("scrub failed")

    def _http(self) -> ThreadingHTTPServer:
        proc = self

        class H(BaseHTTPRequestHandler):
            def log_message(self, *a):  # noqa: D401
                pass

            def do_GET(self):
                if self.path == "/health":
                    body, ctype = b"OK", "text/plain"
                elif self.path == "/metrics":
                    body, ctype = proc.metrics.render().encode(), "text/plain"
                elif self.path == "/sync":
                    # device-side completion of everything this process queued on its GPU
                    t_sync = time.perf_counter()
                    ok = native.device_synchronize(proc.args.gpu)
                    body, ctype = json.dumps({"synchronized": bool(ok), "gpu": proc.args.gpu,
                                              "sync_ms": round(1e3 * (time.perf_counter() - t_sync), 3)}).encode(), \
                        "application/json"
                elif self.path == "/stats":
                    d = dict(proc.store.stats())
                    d.update(proc.cs.stats)
                    if proc.fastpath is not None:
                        d.update(proc.fastpath.stats())
                    if proc.native_grpc is not None:
                        d.update(proc.native_grpc.stats())
                    if proc.agent is not None:
                        d.update(proc.agent.stats())
                    if proc.rccl is not None:
                        d.update({f"repl_{k}": v for k, v in proc.rccl.stats().items()})
                        d["repl_transport"] = proc.rccl.transport
                        d["repl_pairs_up"] = sum(1 for r in range(proc.rccl.world)
                                                 if r != proc.rccl.rank and proc.rccl.pair_ok(r))
                    body, ctype = json.dumps(d).encode(), "application/json"
                elif self.path.startswith("/debug/") and os.environ.get("DFS_DEBUG_ENDPOINTS") == "1":
                    # fault injection for tests (off unless DFS_DEBUG_ENDPOINTS=1):
                    # /debug/corrupt?block=<id>&offset=<n>  flips one byte everywhere it lives
                    # /debug/scrub                           runs one scrub pass now
                    from urllib.parse import parse_qs, urlsplit

                    u = urlsplit(self.path)
                    q = {k: v[0] for k, v in parse_qs(u.query).items()}
                    if u.path == "/debug/corrupt":
                        ok = proc.store.debug_corrupt(q["block"], int(q.get("offset", "0")))
                        body = json.dumps({"corrupted": bool(ok)}).encode()
                    elif u.path == "/debug/scrub":
                        body = json.dumps({"bad": proc.cs.scrub_once()}).encode()
                    elif u.path == "/debug/pause_spill":
                        proc.store.debug_pause_spill(q.get("on", "1") == "1")
                        body = b"{}"
                    elif u.path == "/debug/remove":  # lose a block (EC degraded-read tests)
                        body = json.dumps({"removed": bool(proc.store.remove(q["block"]))}).encode()
                    elif u.path == "/debug/command" and proc.agent is not None:
                        # a master command, serialized ChunkServerCommand as hex, run as if heartbeated
                        proc.agent.submit_command(bytes.fromhex(q["hex"]))
                        body = b"{}"
                    elif u.path == "/debug/drop_resident":
                        proc.store.drop_resident(q["block"])
                        body = b"{}"
                    elif u.path == "/debug/drop_descriptors" and proc.fastpath is not None:
                        proc.fastpath.debug_drop_descriptors(int(q.get("n", "1")))
                        body = b"{}"
                    elif u.path == "/debug/drop_sends" and proc.rccl is not None:
                        proc.rccl.debug_drop_sends(int(q["peer"]), int(q.get("n", "1")))
                        body = b"{}"
                    elif u.path == "/debug/fail_pair" and proc.rccl is not None:
                        proc.rccl.fail_pair(int(q["peer"]), "debug")
                        body = b"{}"
                    else:
                        self.send_response(404)
                        self.end_headers()
                        return
                    ctype = "application/json"
                else:
                    self.send_response(404)
                    self.end_headers()
                    return
                self.send_response(200)
                self.send_header("Content-Type", ctype)
                self.send_header("Content-Length", str(len(body)))
                self.end_headers()
                self.wfile.write(body)

        host = strip_scheme(self.args.addr).rsplit(":", 1)[0] or "0.0.0.0"
        srv = ThreadingHTTPServer((host, self.args.http_port), H)
        srv.daemon_threads = True
        return srv

    def _grpc_fallback(self, path: str, rid: str, payload: bytes):
        """Python side of the native gRPC server: the RPCs (or cases) it does not run in C++."""
        method = path.rsplit("/", 1)[-1]
        entry = self._py_methods.get(method)
        if entry is None:
            return 12, f"unknown method {path}"
        fn, req_cls = entry
        token = current_request_id.set(rid or uuid.uuid4().hex)
        try:
            return 0, fn(req_cls.FromString(payload), None).SerializeToString()
        except RpcStatus as e:
            return e.code.value[0], e.message
        except Exception as e:  # noqa: BLE001 - reported as INTERNAL like grpcio would
            log.exception("%s failed", method)
            return 13, f"{type(e).__name__}: {e}"
        finally:
            current_request_id.reset(token)

    def _start_grpc(self, a, creds):
        host, port = strip_scheme(a.addr).rsplit(":", 1)
        if a.grpc_impl == "native" and self.fastpath is not None:
            self._py_methods = {name: (getattr(self.cs, snake(name)), req)
                                for name, req, _resp in pb.SERVICES["ChunkServerService"]}
            # TLS (--tls-cert/--tls-key) is served natively: OpenSSL + ALPN h2 (csrc/tls.cpp)
            srv = native.NativeGrpcChunkServer(self.store, self.fastpath, host, int(port), self._grpc_fallback,
                                               workers=a.workers, tls_cert=a.tls_cert or "" if creds else "",
                                               tls_key=a.tls_key or "" if creds else "")
            ok, err = srv.start()
            if ok:
                self.native_grpc = srv
                return None
            log.error("native gRPC server failed (%s); serving ChunkServerService on grpcio", err)
        server = make_sync_server({"ChunkServerService": self.cs}, a.addr, workers=a.workers, creds=creds)
        server.start()
        return server

    def run(self) -> None:
        a = self.args
        creds = server_credentials(a.tls_cert, a.tls_key)
        server = self._start_grpc(a, creds)
        http = self._http()
        threading.Thread(target=http.serve_forever, daemon=True, name="cs-http").start()
        sync_port = 0
        try:  # GET /sync served natively (the benchmark's device-sync bracket, no Python on the path)
            self._sync_srv = native.DeviceSyncServer("127.0.0.1", 0, a.gpu)
            ok, _err = self._sync_srv.start()
            sync_port = self._sync_srv.port if ok else 0
        except AttributeError:
            self._sync_srv = None
        if self.agent is not None:
            self.agent.start()
        else:
            threading.Thread(target=self._heartbeat_loop, daemon=True, name="cs-heartbeat").start()
            threading.Thread(target=self._scrub_loop, daemon=True, name="cs-scrub").start()
        ready = os.environ.get("DFS_READY_FILE")
        if ready:
            with open(ready, "w") as f:
                json.dump({"addr": a.addr, "gpu": a.gpu, "rccl": self.rccl is not None,
                           "transport": self.rccl.transport if self.rccl is not None else "grpc",
                           "pairs_up": self.repl_pairs_up, "sync_port": sync_port}, f)
        for sig in (signal.SIGTERM, signal.SIGINT):
            signal.signal(sig, lambda *_: self._stop.set())
        log.info("chunkserver %s serving (gpu=%d, durability=%s)", self.advertise, a.gpu, a.durability)
        while not self._stop.wait(0.5):
            pass
        if self.agent is not None:
            self.agent.stop()
        if server is not None:
            server.stop(1.0).wait()
        if self.native_grpc is not None:
            self.native_grpc.stop()
        http.shutdown()
        if getattr(self, "_sync_srv", None) is not None:
            self._sync_srv.stop()
        if self.rccl is not None:
            self.rccl.stop()
        if self.fastpath is not None:
            self.fastpath.stop()
        self.store.flush()


def main(argv=None) -> None:
    args = build_parser().parse_args(argv)
    logsetup.setup("chunkserver")
    ChunkServerProcess(args).run()


if __name__ == "__main__":
    main()
