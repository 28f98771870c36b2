"""``dfs_master`` — one metadata-shard Raft member (C35; reference
dfs/metaserver/src/bin/master.rs). Flags and defaults follow the reference so its
compose/helm command lines translate 1:1; HTTP serves /health, /metrics, /raft/state and
the Raft peer endpoints /raft/{vote,append,snapshot,timeout_now}."""
from __future__ import annotations

import argparse
import asyncio
import json
import logging
import os
import signal
import ssl

from aiohttp import web

from ..parallel.sharding import ShardMap
from ..raft.membership import initial_members
from ..raft.node import RaftNode, resolve_native_peers
from ..raft.transport import HttpTransport
from ..utils import log as logsetup
from ..utils.metrics import Registry
from ..native import lib as native
from ..utils.localrpc import build_dispatch, socket_name
from ..utils.rpc import AioChannelPool, make_aio_server, server_credentials, with_scheme
from .background import Intervals, MasterBackground
from .monitor import ThroughputMonitor
from .service import MasterService
from .state import MasterState

log = logging.getLogger("dfs.master.server")


def build_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser("dfs_master", description="DFS metadata master (one Raft member of a shard)")
    p.add_argument("-a", "--addr", default="127.0.0.1:50051")
    p.add_argument("--id", type=int, default=1)
    p.add_argument("--peers", default="", help="comma-separated Raft peer HTTP addresses ([id@]url)")
    p.add_argument("--http-port", type=int, default=8080)
    p.add_argument("--advertise-addr", default=None)
    p.add_argument("--storage-dir", default="/tmp/raft-logs")
    p.add_argument("--shard-id", default="shard-0")
    p.add_argument("--standby", action="store_true",
                   help="start without a shard: registered with the config server until a split allocates one")
    p.add_argument("--shard-config", default=None)
    p.add_argument("--config-servers", default="")
    p.add_argument("--split-threshold-rps", type=float, default=100.0)
    p.add_argument("--split-cooldown-secs", type=int, default=30)
    p.add_argument("--merge-threshold-rps", type=float, default=1.0)
    p.add_argument("--tls-cert")
    p.add_argument("--tls-key")
    p.add_argument("--ca-cert")
    p.add_argument("--domain-name")
    p.add_argument("--backup-s3-endpoint")
    p.add_argument("--backup-bucket", default="dfs-backups")
    # MI355X-native build additions
    p.add_argument("--snapshot-threshold", type=int, default=10000,
                   help="log entries between snapshots (reference: 100)")
    p.add_argument("--no-fsync", action="store_true", help="skip WAL fdatasync (tests only)")
    p.add_argument("--fast-intervals", action="store_true", help="short background intervals (tests)")
    p.add_argument("--http-host", default=None)
    return p


class MasterProcess:
    def __init__(self, args):
        self.args = args
        host = args.addr.split(":")[0] if ":" in args.addr else "127.0.0.1"
        self.http_host = args.http_host or host
        self.self_http = f"http://{self.http_host}:{args.http_port}"
        self.client_addr = with_scheme(args.advertise_addr or args.addr)
        self.state = MasterState()  # facade over the native MasterCore
        peers = [p for p in args.peers.split(",") if p.strip()]
        members = initial_members(args.id, self.self_http, peers)
        ssl_ctx = None
        if args.ca_cert:
            ssl_ctx = ssl.create_default_context(cafile=args.ca_cert)
        self.transport = HttpTransport(ssl_ctx=ssl_ctx)
        self.raft = RaftNode(args.id, members, self.client_addr, os.path.join(args.storage_dir, f"raft_node_{args.id}"),
                             self.state, self.transport, snapshot_threshold=args.snapshot_threshold,
                             sync=not args.no_fsync, backup_s3_endpoint=args.backup_s3_endpoint,
                             backup_bucket=args.backup_bucket, native_sm=self.state.core,
                             peer_tls=(args.ca_cert or "", args.domain_name or "") if args.tls_cert else None)
        self.state.core.attach(self.raft._core)
        if os.environ.get("DFS_NATIVE_2PC", "1") == "1":
            # cross-shard Rename coordinated in C++ (MasterCore::rename_2pc) over the native
            # gRPC client; DFS_NATIVE_2PC=0 keeps the Python coordinator (master/service.py)
            self.state.core.enable_native_2pc(bool(args.ca_cert), args.ca_cert or "",
                                              args.domain_name or "")
        self.state.enter_safe_mode()
        self.config_servers = [with_scheme(c) for c in args.config_servers.split(",") if c.strip()]
        if self.config_servers:
            self.shard_map = ShardMap.new_range()
        else:
            self.shard_map = ShardMap.load_config_file(args.shard_config)
        self.monitor = ThroughputMonitor(args.split_threshold_rps, args.merge_threshold_rps, args.split_cooldown_secs)
        self.monitor.source = self.state.core.take_request_counts
        self.pool = AioChannelPool(args.ca_cert, args.domain_name)
        self.svc = MasterService(self.state, self.raft, self.shard_map, "" if args.standby else args.shard_id,
                                 self.monitor, self.pool,
                                 advertise_addr=self.client_addr)
        iv = Intervals()
        if args.fast_intervals:
            iv = Intervals(liveness=1, healer_first=2, healer=5, balancer=2, tx_cleanup=1, tx_recovery=2,
                           shuffler=1, decay=1, shard_refresh=0.5, split=1, tiering=2)
        cold = int(os.environ.get("COLD_THRESHOLD_SECS", "604800"))
        ecs = int(os.environ.get("EC_THRESHOLD_SECS", "2592000"))
        self.bg = MasterBackground(self.svc, self.config_servers, iv, cold, ecs)
        self.metrics = Registry()
        r = self.raft
        self.metrics.gauge("raft_role", "0=follower 1=candidate 2=leader",
                           fn=lambda: {"Follower": 0, "Candidate": 1, "Leader": 2}[r.role])
        self.metrics.gauge("raft_current_term", "current term", fn=lambda: r.current_term)
        self.metrics.gauge("raft_commit_index", "commit index", fn=lambda: r.commit_index)
        self.metrics.gauge("raft_last_applied", "last applied", fn=lambda: r.last_applied)
        self.metrics.gauge("raft_log_len", "log length", fn=lambda: r.last_index())
        self.metrics.gauge("raft_votes_received", "votes", fn=lambda: r.votes_received)
        self.metrics.gauge("raft_wal_fsyncs", "WAL group-commit fsyncs", fn=lambda: r.wal.syncs)
        self.metrics.gauge("dfs_master_safe_mode_status", "1 if in safe mode", fn=lambda: int(self.state.safe_mode))
        self.metrics.gauge("dfs_master_files", "files in this shard", fn=lambda: len(self.state.files))
        self.metrics.gauge("dfs_master_chunkservers", "live chunkservers", fn=lambda: len(self.state.chunk_servers))
        self.metrics.gauge("dfs_master_native_requests", "requests served by the native handlers",
                           fn=lambda: self.state.core.requests)
        self.metrics.gauge("dfs_master_native_heartbeats", "chunkserver heartbeats served by the native handler",
                           fn=lambda: self.state.core.heartbeats)
        for key, help_ in (("native_started", "cross-shard renames coordinated natively"),
                           ("native_committed", "native 2PC renames committed"),
                           ("native_aborted", "native 2PC renames aborted"),
                           ("native_pending", "native 2PC renames left to tx recovery"),
                           ("declined", "cross-shard renames handed to the Python coordinator")):
            self.metrics.gauge(f"dfs_master_tx_{key}", help_,
                               fn=lambda k=key: json.loads(self.state.core.txn_stats())[k])
        self._native_grpc = None
        for key, help_ in (("native_grpc_calls", "gRPC calls served by the native HTTP/2 server"),
                           ("native_grpc_fallback", "native gRPC calls handed to the Python handlers"),
                           ("native_raft_rpcs", "Raft peer RPCs received over the native server")):
            self.metrics.gauge(f"dfs_master_{key}", help_,
                               fn=lambda k=key: self._native_grpc.stats()[k] if self._native_grpc else 0)

    def http_app(self) -> web.Application:
        app = web.Application(client_max_size=1 << 30)

        async def health(_):
            return web.Response(text="OK")

        async def metrics(_):
            return web.Response(text=self.metrics.render(), content_type="text/plain")

        async def raft_state(_):
            return web.json_response(self.raft.cluster_info())

        def raft_route(kind):
            async def h(req):
                try:
                    return web.Response(text=await self.raft.handle_raw(kind, await req.text()),
                                        content_type="application/json")
                except Exception:  # noqa: BLE001
                    return web.Response(status=500, text="Internal server error")

            return h

        async def raft_endpoint(_):
            # where this node takes Raft peer RPCs natively (/dfs.RaftPeer/* on its gRPC port)
            return web.json_response({"grpc": self.client_addr if self._native_grpc is not None else ""})

        app.router.add_get("/health", health)
        app.router.add_get("/metrics", metrics)
        app.router.add_get("/raft/state", raft_state)
        app.router.add_get("/raft/endpoint", raft_endpoint)

        async def shard_map(_):
            return web.json_response({"shard_id": self.svc.shard_id, "map": self.svc.shard_map.to_json()})
        app.router.add_get("/shard_map", shard_map)
        for k in ("vote", "append", "snapshot", "timeout_now"):
            app.router.add_post(f"/raft/{k}", raft_route(k))
        if os.environ.get("DFS_DEBUG_ENDPOINTS") == "1":
            # fault injection for process-level chaos tests (the reference uses Toxiproxy):
            # {"block": [raft peer http addresses]} drops this node's traffic to them
            async def partition(req):
                body = await req.json()
                self.transport.blocked = {HttpTransport._base(a) for a in body.get("block", [])}
                self.raft._core.set_blocked(sorted(self.transport.blocked))
                return web.json_response({"blocked": sorted(self.transport.blocked)})

            app.router.add_post("/debug/partition", partition)
        return app

    async def _resolve_native_peers(self) -> None:
        await resolve_native_peers(self.raft)

    async def run(self, ready_file: str | None = None) -> None:
        a = self.args
        runner = web.AppRunner(self.http_app(), access_log=None)
        await runner.setup()
        site = web.TCPSite(runner, self.http_host if self.http_host != "localhost" else "127.0.0.1", a.http_port,
                           reuse_address=True)
        await site.start()
        creds = server_credentials(a.tls_cert, a.tls_key)
        bind = a.addr if ":" in a.addr else f"0.0.0.0:{a.addr}"
        loop = asyncio.get_running_loop()
        dispatch = build_dispatch({"MasterService": self.svc})

        def fallback(path, rid, payload):
            return asyncio.run_coroutine_threadsafe(dispatch(path, rid, bytes(payload)), loop).result(120)

        server = self._native_grpc = None
        if os.environ.get("DFS_MASTER_GRPC", "native") == "native":
            # MasterService on the native HTTP/2 server: MasterCore's methods (the whole
            # write/read metadata path) are answered in C++, the rest by the handlers below
            host, port = bind.rsplit(":", 1)
            srv = native.NativeGrpcMasterServer(self.state.core, host, int(port), fallback,
                                                tls_cert=a.tls_cert or "" if creds else "",
                                                tls_key=a.tls_key or "" if creds else "")
            ok, err = srv.start()
            if ok:
                self._native_grpc = srv
            else:
                log.warning("native gRPC server unavailable (%s); serving with grpcio", err)
        if self._native_grpc is None:
            server = make_aio_server({"MasterService": self.svc}, bind, creds)
            await server.start()
        self._local_srv = None
        if os.environ.get("DFS_NO_LOCALRPC") != "1":
            # same-host clients skip HTTP/2: a native listener serves the hot methods from
            # MasterCore and hands the rest to the Python handlers on this loop

            srv = native.MasterLocalServer(socket_name(a.addr.rsplit(":", 1)[-1]), self.state.core, fallback)
            ok, err = srv.start()
            if ok:
                self._local_srv = srv
            else:
                log.warning("local RPC listener unavailable: %s", err)
        await self.raft.start()
        resolver = None
        if self._native_grpc is not None:
            resolver = asyncio.get_running_loop().create_task(self._resolve_native_peers())
        if self.config_servers:
            await self.bg.register()
            await self.bg.refresh_shard_map()
        self.bg.start()
        stop = asyncio.Event()
        loop = asyncio.get_running_loop()
        for sig in (signal.SIGTERM, signal.SIGINT):
            try:
                loop.add_signal_handler(sig, stop.set)
            except (NotImplementedError, RuntimeError):
                pass
        if ready_file:
            with open(ready_file, "w") as f:
                json.dump({"addr": a.addr, "http": self.self_http}, f)
        await stop.wait()
        if resolver is not None:
            resolver.cancel()
        await self.bg.stop()
        if self._local_srv is not None:
            await asyncio.get_running_loop().run_in_executor(None, self._local_srv.stop)
        if server is not None:
            await server.stop(0.5)
        if self._native_grpc is not None:
            await asyncio.get_running_loop().run_in_executor(None, self._native_grpc.stop)
        await self.raft.stop()
        self.state.core.detach()
        await self.transport.close()
        await self.pool.close()
        await runner.cleanup()


def main(argv=None) -> None:
    args = build_parser().parse_args(argv)
    logsetup.setup("master")
    prof_path = os.environ.get("DFS_CPROFILE")  # perf investigations: dump cProfile stats on exit
    if prof_path:
        import cProfile

        prof = cProfile.Profile()
        prof.enable()
        try:
            asyncio.run(MasterProcess(args).run(os.environ.get("DFS_READY_FILE")))
        finally:
            prof.disable()
            prof.dump_stats(f"{prof_path}.{os.getpid()}")
        return
    asyncio.run(MasterProcess(args).run(os.environ.get("DFS_READY_FILE")))


if __name__ == "__main__":
    main()
