"""Raft consensus node for the metadata plane (C20-C25) — asyncio face of the native node.

The algorithm runs in C++ (``csrc/raft.cpp``: election, log replication, commit-wait,
ReadIndex, snapshots + InstallSnapshot, joint consensus, TimeoutNow, WAL group commit;
reference dfs/metaserver/src/simple_raft.rs). This module only adapts it to the asyncio
services:

* proposals / ReadIndex return asyncio futures completed from native threads;
* the state machine is either native (``native_sm``: the master's MasterCore or the config
  server's ConfigCore, applied on the Raft applier thread without the GIL) or a Python
  object (tests),
  whose ``apply``/``snapshot``/``restore`` always run on the event loop thread (the
  native applier hands a committed batch over and waits), so service code never races
  the state machine;
* peer RPCs go out through the asyncio transport (HTTP/JSON or the in-process fault
  injector of the tests), incoming ones run the native handler on a worker thread.
"""
from __future__ import annotations

import asyncio
import concurrent.futures as cf
import json
import logging
import os
import threading
import time
from concurrent.futures import ThreadPoolExecutor
from typing import Any, Protocol

from rust_hadoop_generated_by_llm_amd.native import lib as native
from .raft_membership import ClusterConfiguration

log = logging.getLogger("dfs.raft")

FOLLOWER, CANDIDATE, LEADER = "Follower", "Candidate", "Leader"
_COMPACT = (",", ":")


class NotLeader(Exception):
    def __init__(self, hint: str | None):
        super().__init__(f"Not Leader|{hint or ''}")
        self.hint = hint or ""


class StateMachine(Protocol):
    def apply(self, command: Any, index: int) -> Any: ...
    def snapshot(self) -> dict: ...
    def restore(self, state: dict) -> None: ...


class _Host:
    """Callbacks of the native node (invoked on native threads, GIL held)."""

    def __init__(self, sm: StateMachine, transport):
        self.sm = sm
        self.transport = transport
        self.loop: asyncio.AbstractEventLoop | None = None
        self.loop_tid: int | None = None

    def bind(self, loop: asyncio.AbstractEventLoop) -> None:
        self.loop = loop
        self.loop_tid = threading.get_ident()

    def _on_loop(self, fn, *args):
        loop = self.loop
        if loop is None or threading.get_ident() == self.loop_tid or not loop.is_running():
            return fn(*args)
        fut: cf.Future = cf.Future()

        def run():
            try:
                fut.set_result(fn(*args))
            except BaseException as e:  # noqa: BLE001
                fut.set_exception(e)

        loop.call_soon_threadsafe(run)
        while True:
            try:
                return fut.result(timeout=1.0)
            except cf.TimeoutError:
                if not loop.is_running():  # loop gone (shutdown): nothing else touches the state
                    return fn(*args)

    # -- state machine
    def _apply_batch(self, items):
        out = []
        for idx, text in items:
            try:
                out.append(json.dumps(self.sm.apply(json.loads(text), idx), separators=_COMPACT))
            except Exception as e:  # noqa: BLE001
                log.exception("apply failed at %d", idx)
                out.append("!" + str(e))
        return out

    def apply_batch(self, items):
        return self._on_loop(self._apply_batch, items)

    def snapshot(self) -> str:
        return self._on_loop(lambda: json.dumps(self.sm.snapshot(), separators=_COMPACT))

    def restore(self, text: str) -> None:
        self._on_loop(self.sm.restore, json.loads(text))

    # -- transport
    def send(self, addr: str, kind: str, body: str):
        loop = self.loop
        if loop is None or loop.is_closed():
            return None
        if hasattr(self.transport, "send_raw"):
            coro = self.transport.send_raw(addr, kind, body)
        else:
            coro = self._send_json(addr, kind, body)
        try:
            return asyncio.run_coroutine_threadsafe(coro, loop).result(timeout=5.0)
        except Exception:  # noqa: BLE001 - transport failure: the node retries on its own
            return None

    async def _send_json(self, addr, kind, body):
        return json.dumps(await self.transport.send(addr, kind, json.loads(body)))

    def backup(self, url: str, data: bytes) -> None:
        loop = self.loop
        if loop is not None and not loop.is_closed():
            async def put():
                try:
                    await self.transport.put_bytes(url, data)
                except Exception as e:  # noqa: BLE001
                    log.warning("snapshot backup to %s failed: %s", url, e)

            asyncio.run_coroutine_threadsafe(put(), loop)


def _settle(fut: asyncio.Future, code: int, payload: str, parse) -> None:
    if fut.done():
        return
    if code == 0:
        fut.set_result(parse(payload))
    elif code == 1:
        fut.set_exception(NotLeader(payload or None))
    else:
        fut.set_exception(RuntimeError(payload))


class _Wal:
    def __init__(self, core):
        self._core = core

    @property
    def syncs(self) -> int:
        return self._core.wal_syncs

    @property
    def size_bytes(self) -> int:
        return self._core.wal_bytes


class RaftNode:
    def __init__(self, node_id: int, members: dict[int, str], client_address: str, storage_dir: str,
                 state_machine: StateMachine, transport, *, snapshot_threshold: int = 10000,
                 election_timeout: tuple[float, float] = (1.5, 3.0), heartbeat_interval: float = 0.1,
                 sync: bool = True, backup_s3_endpoint: str | None = None, backup_bucket: str = "dfs-backups",
                 max_append_batch: int = 512, native_sm=None, peer_tls: tuple[str, str] | None = None):
        self.id = node_id
        self.client_address = client_address
        self.dir = storage_dir
        os.makedirs(storage_dir, exist_ok=True)
        self.sm = state_machine
        self.transport = transport
        self.heartbeat_interval = heartbeat_interval
        self._host = _Host(state_machine, transport)
        try:  # a node created inside a running loop restores its snapshot on that loop
            self._host.bind(asyncio.get_running_loop())
        except RuntimeError:
            pass
        self._core = native.RaftNode(
            node_id, {int(k): v for k, v in members.items()}, client_address, storage_dir, self._host,
            election_timeout[0], election_timeout[1], heartbeat_interval, sync, snapshot_threshold,
            max_append_batch, backup_s3_endpoint or "", backup_bucket, native_sm,
            peer_tls=peer_tls is not None, peer_ca=(peer_tls or ("", ""))[0], peer_domain=(peer_tls or ("", ""))[1])
        self.wal = _Wal(self._core)
        self._rpc = ThreadPoolExecutor(max_workers=4, thread_name_prefix=f"raft-rpc-{node_id}")
        self._running = False

    # ------------------------------------------------------------------ lifecycle
    async def start(self) -> None:
        self._host.bind(asyncio.get_running_loop())
        self._running = True
        await asyncio.get_running_loop().run_in_executor(self._rpc, self._core.start)

    async def stop(self) -> None:
        if not self._running:
            return
        self._running = False
        await asyncio.get_running_loop().run_in_executor(None, self._core.stop)
        self._rpc.shutdown(wait=False)

    # ------------------------------------------------------------------ proposals / reads
    def _future(self, parse):
        loop = asyncio.get_running_loop()
        fut = loop.create_future()

        def done(code, payload):
            try:
                loop.call_soon_threadsafe(_settle, fut, code, payload, parse)
            except RuntimeError:  # loop closed
                pass

        return fut, done

    async def propose(self, command: Any) -> Any:
        """Append ``command`` and wait until it is committed and applied (commit-wait)."""
        fut, done = self._future(json.loads)
        self._core.propose(json.dumps(command, separators=_COMPACT), done)
        return await fut

    def propose_nowait(self, command: Any) -> bool:
        """Fire-and-forget proposal (reference: UpdateAccessStats on every GetFileInfo)."""
        return self._core.propose_nowait(json.dumps(command, separators=_COMPACT))

    async def read_index(self) -> int:
        """ReadIndex: return once a read at the current commit point is linearizable."""
        fut, done = self._future(int)
        self._core.read_index(done)
        return await fut

    # ------------------------------------------------------------------ RPC handlers
    async def handle_raw(self, kind: str, body: str) -> str:
        return await asyncio.get_running_loop().run_in_executor(self._rpc, self._core.handle, kind, body)

    async def handle(self, kind: str, args: dict) -> dict:
        return json.loads(await self.handle_raw(kind, json.dumps(args, separators=_COMPACT)))

    async def transfer_leadership(self, target: int) -> bool:
        return await asyncio.get_running_loop().run_in_executor(self._rpc, self._core.transfer_leadership, target)

    async def snapshot_now(self) -> None:
        await asyncio.get_running_loop().run_in_executor(None, self._core.snapshot_now)

    # ------------------------------------------------------------------ membership
    async def add_server(self, server_id: int, address: str) -> Any:
        return await self.propose({"Membership": {"AddServer": {"server_id": server_id, "server_address": address}}})

    async def remove_server(self, server_id: int) -> Any:
        return await self.propose({"Membership": {"RemoveServer": {"server_id": server_id}}})

    async def change_membership(self, new_members: dict[int, str], catch_up_timeout: float = 10.0) -> Any:
        """Joint consensus: new servers catch up as non-voters (10 rounds at commit), then
        C_old,new is committed, then C_new (reference simple_raft.rs:2458-2737)."""
        if not self.is_leader():
            raise NotLeader(self.leader_address)
        cfg = self.config
        added = {i: a for i, a in new_members.items() if i not in cfg.voters()}
        for i, a in added.items():
            self._core.add_non_voter(i, a)
        deadline = time.monotonic() + catch_up_timeout
        while added and time.monotonic() < deadline:
            if all(self._core.caught_up(i) for i in added):
                break
            await asyncio.sleep(self.heartbeat_interval)
        v = cfg.version + 1
        await self.propose({"Membership": {"BeginJointConsensus": {
            "old_members": {str(k): x for k, x in cfg.members.items()},
            "new_members": {str(k): x for k, x in new_members.items()}, "version": v}}})
        res = await self.propose({"Membership": {"FinalizeConfiguration": {
            "new_members": {str(k): x for k, x in new_members.items()}, "version": v + 1}}})
        for i in added:
            self._core.drop_non_voter(i)
        return res

    # ------------------------------------------------------------------ introspection
    @property
    def role(self) -> str:
        return self._core.role

    @property
    def current_term(self) -> int:
        return self._core.term

    @property
    def leader_id(self) -> int | None:
        i = self._core.leader_id
        return None if i < 0 else i

    @property
    def leader_address(self) -> str | None:
        return self._core.leader_address or None

    @property
    def commit_index(self) -> int:
        return self._core.commit_index

    @property
    def last_applied(self) -> int:
        return self._core.last_applied

    @property
    def last_included_index(self) -> int:
        return self._core.last_included_index

    @property
    def votes_received(self) -> int:
        return self._core.votes

    @property
    def config(self) -> ClusterConfiguration:
        return ClusterConfiguration.from_json(json.loads(self._core.config_json))

    def last_index(self) -> int:
        return self._core.last_index

    def is_leader(self) -> bool:
        return self._core.role == LEADER

    def cluster_info(self) -> dict:
        return json.loads(self._core.info_json())


async def resolve_native_peers(raft: "RaftNode") -> None:
    """Learn each Raft peer's native endpoint (GET /raft/endpoint) and hand it to the native
    node: from then on AppendEntries / RequestVote travel node-to-node over the native HTTP/2
    servers without touching Python on either side. Peers without one (grpcio, older builds)
    stay on the HTTP/JSON transport. Runs until cancelled; only unresolved members are asked."""
    import aiohttp

    known: dict[str, str] = {}
    async with aiohttp.ClientSession(timeout=aiohttp.ClientTimeout(total=2)) as sess:
        while True:
            members = dict(raft.config.all_members())
            for mid, addr in members.items():
                if mid == raft.id or addr in known:
                    continue
                try:
                    async with sess.get(addr.rstrip("/") + "/raft/endpoint") as r:
                        ep = (await r.json(content_type=None)).get("grpc", "") if r.status == 200 else ""
                except Exception:  # noqa: BLE001 - peer not up yet: ask again later
                    continue
                known[addr] = ep
                if ep:
                    raft._core.set_peer_endpoint(addr, ep)
            await asyncio.sleep(1.0)
