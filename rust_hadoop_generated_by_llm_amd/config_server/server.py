"""``dfs_config_server`` — Raft-replicated shard map + master registry (C36; reference
dfs/metaserver/src/config_server.rs and bin/config_server.rs).

State ``{"Config": {"shard_map": ShardMap(Range), "masters": {addr: MasterInfo}}}``, held and
applied natively (csrc/config_core.cpp) on the native Raft node's applier thread, which also
answers every ConfigService RPC and the Raft peer RPC (``NativeGrpcConfigServer`` over HTTP/2,
``ConfigLocalServer`` on the same-host socket): no request runs Python. The grpcio service
below stays as the ``DFS_CONFIG_GRPC=grpcio`` A/B and for tests.
FetchShardMap is linearizable (ReadIndex) and, like the reference, returns only
shard -> peers (no range boundaries). SplitShard without peers allocates standby masters (registered
with an empty shard id) first, else the three most recently heartbeated masters; the
``ranges`` extension of FetchShardMap carries the split keys. HTTP: /raft/{vote,append,snapshot}, /shards, plus
/health and /metrics (the reference has neither)."""
from __future__ import annotations

import argparse
import asyncio
import json
import logging
import os
import signal

from aiohttp import web

from ..models import proto as pb
from ..native import lib as _native
from ..parallel.sharding import ShardMap
from ..raft.membership import initial_members
from ..raft.node import NotLeader, RaftNode, resolve_native_peers
from ..raft.transport import HttpTransport
from ..utils import log as logsetup
from ..utils.metrics import Registry
from ..utils.localrpc import serve_local, socket_name
from ..utils.rpc import RpcStatus, StatusCode, make_aio_server, server_credentials, with_scheme

log = logging.getLogger("dfs.config_server")


class ConfigState:
    """Facade over the native state machine (csrc/config_core.cpp), which the native Raft
    node applies on its own thread; views are re-parsed only when the state changed."""

    def __init__(self):
        self.core = _native.ConfigCore()
        self._map: tuple[int, ShardMap | None] = (-1, None)

    @property
    def shard_map(self) -> ShardMap:
        v = self.core.version
        if self._map[0] != v or self._map[1] is None:
            self._map = (v, ShardMap.from_json(json.loads(self.core.shard_map_json())))
        return self._map[1]

    @property
    def masters(self) -> dict[str, dict]:
        return json.loads(self.core.masters_json())

    def apply(self, command, index: int = 0):
        r = self.core.apply(index, json.dumps(command))
        if r.startswith("!"):
            raise ValueError(r[1:])
        return json.loads(r)

    def snapshot(self) -> dict:
        return json.loads(self.core.snapshot())

    def restore(self, state: dict) -> None:
        self.core.restore(json.dumps(state))


class ConfigService:
    def __init__(self, state: ConfigState, raft: RaftNode):
        self.state = state
        self.raft = raft

    async def _propose(self, name, args):
        return await self.raft.propose({"Config": {name: args}})

    async def _simple(self, resp_cls, name, args):
        try:
            await self._propose(name, args)
        except NotLeader as e:
            return resp_cls(success=False, error_message="Not Leader", leader_hint=e.hint)
        return resp_cls(success=True)

    async def fetch_shard_map(self, req, ctx):
        try:
            await self.raft.read_index()
        except NotLeader as e:
            raise RpcStatus(StatusCode.FAILED_PRECONDITION, f"Not Leader|{e.hint}")
        resp = pb.FetchShardMapResponse()
        sm = self.state.shard_map
        for sid in sm.get_all_shards():
            resp.shards[sid].peers.extend(sm.get_shard_peers(sid) or [])
        if sm.strategy == "range":
            for end, sid in sm.ranges.items():
                resp.ranges[end] = sid
        return resp

    async def add_shard(self, req, ctx):
        return await self._simple(pb.AddShardResponse, "AddShard", {"shard_id": req.shard_id, "peers": list(req.peers)})

    async def remove_shard(self, req, ctx):
        return await self._simple(pb.RemoveShardResponse, "RemoveShard", {"shard_id": req.shard_id})

    async def split_shard(self, req, ctx):
        peers = list(req.new_shard_peers)
        if not peers:
            # prefer standby masters (registered without a shard); the reference takes the
            # three most recently heartbeated masters even if they serve another shard
            peers = self.state.core.split_candidates(3)
        if not peers:
            return pb.SplitShardResponse(success=False, error_message="No available master nodes for new shard")
        try:
            ok = await self._propose("SplitShard", {"shard_id": req.shard_id, "split_key": req.split_key,
                                                    "new_shard_id": req.new_shard_id, "new_shard_peers": peers})
        except NotLeader as e:
            return pb.SplitShardResponse(success=False, error_message="Not Leader", leader_hint=e.hint)
        if not ok:
            return pb.SplitShardResponse(success=False, error_message="split rejected by the shard map")
        return pb.SplitShardResponse(success=True, new_shard_peers=peers)

    async def merge_shard(self, req, ctx):
        # the apply result decides: two idle neighbours may try to merge into each other,
        # and only the first may win (the reference reports success either way)
        try:
            ok = await self._propose("MergeShard", {"victim_shard_id": req.victim_shard_id,
                                                    "retained_shard_id": req.retained_shard_id})
        except NotLeader as e:
            return pb.MergeShardResponse(success=False, error_message="Not Leader", leader_hint=e.hint)
        if not ok:
            return pb.MergeShardResponse(success=False, error_message="merge rejected: unknown shard")
        return pb.MergeShardResponse(success=True)

    async def rebalance_shard(self, req, ctx):
        return await self._simple(pb.RebalanceShardResponse, "RebalanceShard",
                                  {"old_key": req.old_key, "new_key": req.new_key})

    async def register_master(self, req, ctx):
        try:
            await self._propose("RegisterMaster", {"address": req.address, "shard_id": req.shard_id})
        except NotLeader:
            return pb.RegisterMasterResponse(success=False)
        return pb.RegisterMasterResponse(success=True)

    async def shard_heartbeat(self, req, ctx):
        if not self.raft.is_leader():
            return pb.ShardHeartbeatResponse(success=False)
        self.raft.propose_nowait({"Config": {"ShardHeartbeat": {"address": req.address,
                                                                "rps_per_prefix": dict(req.rps_per_prefix)}}})
        return pb.ShardHeartbeatResponse(success=True)


def build_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser("dfs_config_server")
    p.add_argument("--addr", default="127.0.0.1:50052")
    p.add_argument("--id", type=int, default=1)
    p.add_argument("--peers", default="")
    p.add_argument("--http-port", type=int, default=8081)
    p.add_argument("--advertise-addr", default=None)
    p.add_argument("--storage-dir", default="/tmp/config-raft-logs")
    p.add_argument("--tls-cert")
    p.add_argument("--tls-key")
    p.add_argument("--ca-cert")
    p.add_argument("--no-fsync", action="store_true")
    p.add_argument("--snapshot-threshold", type=int, default=10000)
    return p


async def run(args) -> None:
    host = args.addr.split(":")[0] if ":" in args.addr else "127.0.0.1"
    self_http = f"http://{host}:{args.http_port}"
    state = ConfigState()
    members = initial_members(args.id, self_http, [p for p in args.peers.split(",") if p.strip()])
    transport = HttpTransport()
    raft = RaftNode(args.id, members, with_scheme(args.advertise_addr or args.addr),
                    os.path.join(args.storage_dir, f"raft_node_{args.id}"), state, transport,
                    snapshot_threshold=args.snapshot_threshold, sync=not args.no_fsync,
                    native_sm=state.core)
    state.core.attach(raft._core)
    svc = ConfigService(state, raft)
    metrics = Registry()
    metrics.gauge("raft_role", "0=follower 1=candidate 2=leader",
                  fn=lambda: {"Follower": 0, "Candidate": 1, "Leader": 2}[raft.role])
    metrics.gauge("config_shards", "shards in the map", fn=lambda: len(state.shard_map.shards))
    metrics.gauge("config_native_requests", "ConfigService RPCs answered by the native core",
                  fn=lambda: state.core.requests)
    native_srv = None
    app = web.Application(client_max_size=1 << 30)

    def raft_route(kind):
        async def h(req):
            try:
                return web.Response(text=await raft.handle_raw(kind, await req.text()),
                                    content_type="application/json")
            except Exception:  # noqa: BLE001
                return web.Response(status=500, text="Internal server error")

        return h

    for k in ("vote", "append", "snapshot", "timeout_now"):
        app.router.add_post(f"/raft/{k}", raft_route(k))

    async def shards(_):
        return web.json_response({"shards": state.shard_map.get_all_shards()})

    async def health(_):
        return web.Response(text="OK")

    async def metrics_h(_):
        return web.Response(text=metrics.render(), content_type="text/plain")

    async def raft_state(_):
        return web.json_response(raft.cluster_info())

    async def raft_endpoint(_):
        # where this node takes Raft peer RPCs natively (/dfs.RaftPeer/* on its gRPC port)
        return web.json_response({"grpc": with_scheme(args.advertise_addr or args.addr) if native_srv else ""})

    app.router.add_get("/shards", shards)
    app.router.add_get("/health", health)
    app.router.add_get("/metrics", metrics_h)
    app.router.add_get("/raft/state", raft_state)
    app.router.add_get("/raft/endpoint", raft_endpoint)
    runner = web.AppRunner(app, access_log=None)
    await runner.setup()
    await web.TCPSite(runner, host, args.http_port, reuse_address=True).start()
    creds = server_credentials(args.tls_cert, args.tls_key)
    server = None
    if os.environ.get("DFS_CONFIG_GRPC", "native") == "native":
        bind = args.addr if ":" in args.addr else f"0.0.0.0:{args.addr}"
        h, port = bind.rsplit(":", 1)
        srv = _native.NativeGrpcConfigServer(state.core, h, int(port), tls_cert=args.tls_cert or "" if creds else "",
                                             tls_key=args.tls_key or "" if creds else "")
        ok, err = srv.start()
        if ok:
            native_srv = srv
        else:
            log.warning("native gRPC server unavailable (%s); serving with grpcio", err)
    if native_srv is None:
        server = make_aio_server({"ConfigService": svc}, args.addr, creds)
        await server.start()
    local_srv = native_local = None
    if creds is None and os.environ.get("DFS_NO_LOCALRPC") != "1":
        if native_srv is not None:
            srv = _native.ConfigLocalServer(socket_name(args.addr.rsplit(":", 1)[-1]), state.core)
            ok, err = srv.start()
            if ok:
                native_local = srv
            else:
                log.warning("local RPC listener unavailable: %s", err)
        else:
            try:
                local_srv = await serve_local({"ConfigService": svc}, args.addr.rsplit(":", 1)[-1])
            except OSError as e:
                log.warning("local RPC listener unavailable: %s", e)
    await raft.start()
    resolver = asyncio.get_running_loop().create_task(resolve_native_peers(raft)) if native_srv else None
    stop = asyncio.Event()
    loop = asyncio.get_running_loop()
    for sig in (signal.SIGTERM, signal.SIGINT):
        try:
            loop.add_signal_handler(sig, stop.set)
        except (NotImplementedError, RuntimeError):
            pass
    ready = os.environ.get("DFS_READY_FILE")
    if ready:
        with open(ready, "w") as f:
            json.dump({"addr": args.addr}, f)
    await stop.wait()
    if resolver is not None:
        resolver.cancel()
    if native_local is not None:
        await loop.run_in_executor(None, native_local.stop)
    if server is not None:
        await server.stop(0.5)
    if native_srv is not None:
        await loop.run_in_executor(None, native_srv.stop)
    await raft.stop()
    state.core.detach()
    await transport.close()
    await runner.cleanup()


def main(argv=None) -> None:
    args = build_parser().parse_args(argv)
    logsetup.setup("config_server")
    asyncio.run(run(args))


if __name__ == "__main__":
    main()
