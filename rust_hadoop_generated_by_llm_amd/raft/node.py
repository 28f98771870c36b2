"""Raft consensus node for the metadata plane (C20-C25).

Semantics follow the reference's ``simple_raft`` (dfs/metaserver/src/simple_raft.rs):
randomised 1.5-3 s election timeout, 100 ms heartbeats, a NoOp on becoming leader,
commit only of current-term entries by (joint) majority, replies answered after apply
("commit-wait"), ReadIndex for linearizable reads, snapshots + InstallSnapshot, legacy
AddServer/RemoveServer and joint-consensus membership, TimeoutNow leader transfer and an
optional snapshot backup PUT to an S3 endpoint.

MI355X-native build notes:
* Persistence is the native CRC-framed WAL (csrc/wal.cpp) plus an atomically replaced
  JSON snapshot — no RocksDB. One fdatasync per batch of proposals (group commit): while a
  WAL write is in flight new proposals accumulate and go out in the next write, which is
  the reference's "leader batching" (P8) without a fixed 256-event window.
* ReadIndex requests are coalesced onto heartbeat rounds: one majority round trip
  confirms leadership for every read that arrived before it was sent.
* The algorithm is re-derived from the Raft paper rather than transcribed; the
  reference's index-mapping fragilities are avoided by keeping
  ``log[i - first_index]`` arithmetic in one place.
"""
from __future__ import annotations

import asyncio
import json
import logging
import os
import random
import time
from concurrent.futures import ThreadPoolExecutor
from typing import Any, Protocol

from ..native import lib as native
from .membership import CatchUpProgress, ClusterConfiguration

log = logging.getLogger("dfs.raft")

FOLLOWER, CANDIDATE, LEADER = "Follower", "Candidate", "Leader"


class NotLeader(Exception):
    def __init__(self, hint: str | None):
        super().__init__(f"Not Leader|{hint or ''}")
        self.hint = hint or ""


class StateMachine(Protocol):
    def apply(self, command: Any, index: int) -> Any: ...
    def snapshot(self) -> dict: ...
    def restore(self, state: dict) -> None: ...


class RaftNode:
    def __init__(self, node_id: int, members: dict[int, str], client_address: str, storage_dir: str,
                 state_machine: StateMachine, transport, *, snapshot_threshold: int = 10000,
                 election_timeout: tuple[float, float] = (1.5, 3.0), heartbeat_interval: float = 0.1,
                 sync: bool = True, backup_s3_endpoint: str | None = None, backup_bucket: str = "dfs-backups",
                 max_append_batch: int = 512):
        self.id = node_id
        self.client_address = client_address
        self.dir = storage_dir
        os.makedirs(storage_dir, exist_ok=True)
        self.sm = state_machine
        self.transport = transport
        self.snapshot_threshold = snapshot_threshold
        self.election_timeout_range = election_timeout
        self.heartbeat_interval = heartbeat_interval
        self.sync = sync
        self.backup_s3_endpoint = backup_s3_endpoint
        self.backup_bucket = backup_bucket
        self.max_append_batch = max_append_batch

        # persistent
        self.current_term = 0
        self.voted_for: int | None = None
        self.log: list[tuple[int, Any]] = []  # (term, command); index = first_index + pos
        self.last_included_index = 0
        self.last_included_term = 0
        self.config = ClusterConfiguration(dict(members))
        # volatile
        self.role = FOLLOWER
        self.leader_id: int | None = None
        self.leader_address: str | None = None
        self.commit_index = 0
        self.last_applied = 0
        self.next_index: dict[int, int] = {}
        self.match_index: dict[int, int] = {}
        self.votes: set[int] = set()
        self.non_voting: dict[int, str] = {}
        self.catch_up: dict[int, CatchUpProgress] = {}
        self._pending: dict[int, tuple[int, asyncio.Future]] = {}
        self._unsynced_from: int | None = None
        self._durable_index = 0
        self._inflight: dict[int, bool] = {}
        self._again: dict[int, bool] = {}
        self._hb_round = 0
        self._acked_round: dict[int, int] = {}
        self._read_waiters: list[tuple[int, int, asyncio.Future]] = []  # (read_index, need_round, fut)
        self._leader_noop_index = 0
        self._election_deadline = 0.0
        self._flush_evt: asyncio.Event | None = None
        self._append_lock: asyncio.Lock | None = None
        self._tasks: list[asyncio.Task] = []
        self._io = ThreadPoolExecutor(max_workers=1, thread_name_prefix=f"raft-wal-{node_id}")
        self._running = False
        self._apply_listeners: list = []
        self.wal = native.Wal(os.path.join(storage_dir, "raft.wal"), sync)
        self._load()

    # ------------------------------------------------------------------ persistence
    @property
    def first_index(self) -> int:
        return self.last_included_index + 1

    def last_index(self) -> int:
        return self.last_included_index + len(self.log)

    def term_at(self, idx: int) -> int:
        if idx == self.last_included_index:
            return self.last_included_term
        if idx < self.last_included_index or idx > self.last_index():
            return -1
        return self.log[idx - self.first_index][0]

    def _snap_path(self) -> str:
        return os.path.join(self.dir, "snapshot.json")

    def _load(self) -> None:
        sp = self._snap_path()
        if os.path.exists(sp):
            with open(sp) as f:
                snap = json.load(f)
            self.last_included_index, self.last_included_term = snap["meta"]
            if snap.get("config"):
                self.config = ClusterConfiguration.from_json(snap["config"])
            self.sm.restore(snap["state"])
            self.commit_index = self.last_applied = self.last_included_index
        for raw in self.wal.replay():
            rec = json.loads(raw)
            k = rec["k"]
            if k == "H":
                self.current_term, self.voted_for = rec["term"], rec["vote"]
            elif k == "E":
                idx = rec["i"]
                if idx <= self.last_included_index:
                    continue
                pos = idx - self.first_index
                if pos < len(self.log):
                    del self.log[pos:]
                if pos == len(self.log):
                    self.log.append((rec["t"], rec["c"]))
            elif k == "T":
                pos = rec["from"] - self.first_index
                if pos >= 0:
                    del self.log[pos:]
            elif k == "C":
                self.config = ClusterConfiguration.from_json(rec["config"])
        self._durable_index = self.last_index()
        log.info("raft node %d loaded: term=%d snapshot=%d last=%d", self.id, self.current_term,
                 self.last_included_index, self.last_index())

    def _hs_record(self) -> bytes:
        return json.dumps({"k": "H", "term": self.current_term, "vote": self.voted_for}).encode()

    def _entry_record(self, idx: int) -> bytes:
        t, c = self.log[idx - self.first_index]
        return json.dumps({"k": "E", "i": idx, "t": t, "c": c}, separators=(",", ":")).encode()

    def _config_record(self) -> bytes:
        return json.dumps({"k": "C", "config": self.config.to_json()}).encode()

    async def _wal(self, records: list[bytes]) -> None:
        if records:
            await asyncio.get_running_loop().run_in_executor(self._io, self.wal.append, records)

    async def _persist_hard_state(self) -> None:
        await self._wal([self._hs_record()])

    # ------------------------------------------------------------------ lifecycle
    async def start(self) -> None:
        self._flush_evt = asyncio.Event()
        self._append_lock = asyncio.Lock()
        self._running = True
        self._reset_election_timer()
        loop = asyncio.get_running_loop()
        self._tasks = [loop.create_task(self._ticker()), loop.create_task(self._flusher())]
        if self._peers() == [] and self.id in self.config.voters():
            await self._start_election()  # single-node group: lead immediately

    async def stop(self) -> None:
        self._running = False
        for t in self._tasks:
            t.cancel()
        for t in self._tasks:
            try:
                await t
            except (asyncio.CancelledError, Exception):  # noqa: BLE001
                pass
        self._fail_pending(NotLeader(None))
        self._io.shutdown(wait=True)

    def _peers(self) -> list[int]:
        ids = set(self.config.all_members()) | set(self.non_voting)
        ids.discard(self.id)
        return sorted(ids)

    def _addr(self, peer: int) -> str:
        return self.config.all_members().get(peer) or self.non_voting.get(peer, "")

    def _reset_election_timer(self) -> None:
        lo, hi = self.election_timeout_range
        self._election_deadline = time.monotonic() + random.uniform(lo, hi)

    async def _ticker(self) -> None:
        while self._running:
            await asyncio.sleep(self.heartbeat_interval)
            try:
                if self.role == LEADER:
                    self._broadcast()
                elif time.monotonic() >= self._election_deadline and self.id in self.config.voters():
                    await self._start_election()
                self._maybe_snapshot()  # every member compacts its own log
            except Exception:  # noqa: BLE001
                log.exception("raft tick failed")

    # ------------------------------------------------------------------ elections
    async def _start_election(self) -> None:
        self.role = CANDIDATE
        self.current_term += 1
        self.voted_for = self.id
        self.leader_id = None
        self.votes = {self.id}
        term = self.current_term
        self._reset_election_timer()
        await self._persist_hard_state()
        log.info("node %d starting election for term %d", self.id, term)
        if self.config.has_joint_majority(self.votes):
            await self._become_leader()
            return
        args = {"term": term, "candidate_id": self.id, "last_log_index": self.last_index(),
                "last_log_term": self.term_at(self.last_index())}
        for p in self._peers():
            if p in self.config.voters():
                asyncio.get_running_loop().create_task(self._request_vote(p, args))

    async def _request_vote(self, peer: int, args: dict) -> None:
        try:
            reply = await self.transport.send(self._addr(peer), "vote", args)
        except Exception:  # noqa: BLE001
            return
        if reply["term"] > self.current_term:
            await self._step_down(reply["term"], None)
            return
        if self.role != CANDIDATE or self.current_term != args["term"] or not reply.get("vote_granted"):
            return
        self.votes.add(reply.get("peer_id", peer))
        if self.config.has_joint_majority(self.votes):
            await self._become_leader()

    async def _become_leader(self) -> None:
        if self.role == LEADER:
            return
        self.role = LEADER
        self.leader_id = self.id
        self.leader_address = self.client_address
        nxt = self.last_index() + 1
        self.next_index = {p: nxt for p in self._peers()}
        self.match_index = {p: 0 for p in self._peers()}
        self._acked_round = {}
        log.info("node %d became leader for term %d", self.id, self.current_term)
        self._leader_noop_index = self._append_local("NoOp")
        self._broadcast()

    async def _step_down(self, term: int, leader_address: str | None, leader_id: int | None = None) -> None:
        # The role must change in the same step as the term: persisting the hard state
        # yields, and a concurrent _replicate() of this node that still saw LEADER would
        # otherwise send AppendEntries stamped with the *new* term it never won.
        was_leader = self.role == LEADER
        self.role = FOLLOWER
        self.leader_id = leader_id
        self.leader_address = leader_address
        if term > self.current_term:
            self.current_term = term
            self.voted_for = None
            await self._persist_hard_state()
        self._reset_election_timer()
        if was_leader:
            self._fail_pending(NotLeader(leader_address))

    def _fail_pending(self, exc: Exception) -> None:
        for _, (_, fut) in list(self._pending.items()):
            if not fut.done():
                fut.set_exception(exc)
        self._pending.clear()
        for _, _, fut in self._read_waiters:
            if not fut.done():
                fut.set_exception(exc)
        self._read_waiters.clear()

    # ------------------------------------------------------------------ proposals
    def _append_local(self, command: Any) -> int:
        self.log.append((self.current_term, command))
        idx = self.last_index()
        if self._unsynced_from is None:
            self._unsynced_from = idx
        self._flush_evt.set()
        return idx

    async def propose(self, command: Any) -> Any:
        """Append ``command`` and wait until it is committed and applied (commit-wait)."""
        if self.role != LEADER:
            raise NotLeader(self.leader_address)
        idx = self._append_local(command)
        fut = asyncio.get_running_loop().create_future()
        self._pending[idx] = (self.current_term, fut)
        return await fut

    def propose_nowait(self, command: Any) -> bool:
        """Fire-and-forget proposal (reference: UpdateAccessStats on every GetFileInfo)."""
        if self.role != LEADER:
            return False
        self._append_local(command)
        return True

    async def _flusher(self) -> None:
        while self._running:
            await self._flush_evt.wait()
            self._flush_evt.clear()
            if self._unsynced_from is None:
                continue
            start, end = self._unsynced_from, self.last_index()
            self._unsynced_from = None
            if start > end or start < self.first_index:
                continue
            recs = [self._entry_record(i) for i in range(start, end + 1)]
            try:
                await self._wal(recs)
            except Exception:  # noqa: BLE001
                log.exception("WAL append failed")
                continue
            self._durable_index = max(self._durable_index, end)
            if self.role == LEADER:
                self._advance_commit()
                self._broadcast()

    # ------------------------------------------------------------------ replication
    def _broadcast(self) -> None:
        if self.role != LEADER:
            return
        self._hb_round += 1
        for p in self._peers():
            if self._inflight.get(p):
                self._again[p] = True
                continue
            self._inflight[p] = True
            asyncio.get_running_loop().create_task(self._replicate(p, self._hb_round))
        self._check_reads()

    async def _replicate(self, peer: int, rnd: int) -> None:
        try:
            while True:
                self._again[peer] = False
                if self.role != LEADER:
                    return
                term = self.current_term
                nxt = self.next_index.get(peer, self.last_index() + 1)
                if nxt <= self.last_included_index:
                    await self._send_snapshot(peer)
                else:
                    prev = nxt - 1
                    last = min(self.last_index(), prev + self.max_append_batch)
                    entries = [{"term": self.log[i - self.first_index][0], "command": self.log[i - self.first_index][1]}
                               for i in range(nxt, last + 1)]
                    args = {"term": term, "leader_id": self.id, "prev_log_index": prev,
                            "prev_log_term": self.term_at(prev), "entries": entries,
                            "leader_commit": self.commit_index, "leader_address": self.client_address,
                            "round": rnd}
                    try:
                        reply = await self.transport.send(self._addr(peer), "append", args)
                    except Exception:  # noqa: BLE001
                        return
                    if reply["term"] > self.current_term:
                        await self._step_down(reply["term"], None)
                        return
                    if self.role != LEADER or self.current_term != term:
                        return
                    if reply.get("success"):
                        m = reply.get("match_index", prev + len(entries))
                        self.match_index[peer] = max(self.match_index.get(peer, 0), m)
                        self.next_index[peer] = self.match_index[peer] + 1
                        self._acked_round[peer] = max(self._acked_round.get(peer, 0), rnd)
                        if peer in self.catch_up:
                            self.catch_up[peer].update(m)
                        self._advance_commit()
                        self._check_reads()
                    else:
                        hint = reply.get("match_index", prev - 1)
                        self.next_index[peer] = max(1, min(nxt - 1, hint + 1))
                        self._again[peer] = True
                if not self._again.get(peer) and self.next_index.get(peer, 0) > self.last_index():
                    return
                rnd = self._hb_round
        finally:
            self._inflight[peer] = False

    async def _send_snapshot(self, peer: int) -> None:
        sp = self._snap_path()
        if not os.path.exists(sp):
            self._take_snapshot()
        with open(sp) as f:
            data = f.read()
        args = {"term": self.current_term, "leader_id": self.id,
                "last_included_index": self.last_included_index, "last_included_term": self.last_included_term,
                "data": data, "leader_address": self.client_address}
        try:
            reply = await self.transport.send(self._addr(peer), "snapshot", args)
        except Exception:  # noqa: BLE001
            return
        if reply["term"] > self.current_term:
            await self._step_down(reply["term"], None)
            return
        self.match_index[peer] = max(self.match_index.get(peer, 0), reply["last_included_index"])
        self.next_index[peer] = self.match_index[peer] + 1

    def _advance_commit(self) -> None:
        if self.role != LEADER:
            return
        new_commit = self.commit_index
        for n in range(self.last_index(), self.commit_index, -1):
            if self.term_at(n) != self.current_term:
                break
            acks = {p for p, m in self.match_index.items() if m >= n}
            if self._durable_index >= n:
                acks.add(self.id)
            if self.config.has_joint_majority(acks):
                new_commit = n
                break
        if new_commit > self.commit_index:
            self.commit_index = new_commit
            self._apply()

    def _apply(self) -> None:
        while self.last_applied < self.commit_index:
            idx = self.last_applied + 1
            term, cmd = self.log[idx - self.first_index]
            result: Any = None
            err: Exception | None = None
            try:
                if isinstance(cmd, dict) and "Membership" in cmd:
                    result = self._apply_membership(cmd["Membership"], idx)
                elif cmd != "NoOp":
                    result = self.sm.apply(cmd, idx)
            except Exception as e:  # noqa: BLE001
                log.exception("apply failed at %d", idx)
                err = e
            self.last_applied = idx
            p = self._pending.pop(idx, None)
            if p is not None and not p[1].done():
                if p[0] != term:
                    p[1].set_exception(NotLeader(self.leader_address))
                elif err is not None:
                    p[1].set_exception(err)
                else:
                    p[1].set_result(result)
            for cb in self._apply_listeners:
                cb(idx, cmd)
        self._check_reads()

    # ------------------------------------------------------------------ linearizable reads
    async def read_index(self) -> int:
        """ReadIndex: return once a read at the current commit point is linearizable."""
        if self.role != LEADER:
            raise NotLeader(self.leader_address)
        if self.commit_index < self._leader_noop_index:
            # leader must have committed an entry of its term first
            for _ in range(200):
                await asyncio.sleep(0.005)
                if self.role != LEADER:
                    raise NotLeader(self.leader_address)
                if self.commit_index >= self._leader_noop_index:
                    break
        idx = self.commit_index
        if not self._peers() or self.config.voters() == {self.id}:
            return idx
        fut = asyncio.get_running_loop().create_future()
        self._read_waiters.append((idx, self._hb_round + 1, fut))
        self._broadcast()
        return await fut

    def _check_reads(self) -> None:
        if not self._read_waiters or self.role != LEADER:
            return
        keep = []
        for idx, need, fut in self._read_waiters:
            if fut.done():
                continue
            acks = {p for p, r in self._acked_round.items() if r >= need} | {self.id}
            if self.config.has_joint_majority(acks) and self.last_applied >= idx:
                fut.set_result(idx)
            else:
                keep.append((idx, need, fut))
        self._read_waiters = keep

    # ------------------------------------------------------------------ RPC handlers
    async def handle(self, kind: str, args: dict) -> dict:
        if kind == "vote":
            return await self.handle_request_vote(args)
        if kind == "append":
            return await self.handle_append_entries(args)
        if kind == "snapshot":
            return await self.handle_install_snapshot(args)
        if kind == "timeout_now":
            return await self.handle_timeout_now(args)
        raise ValueError(kind)

    async def handle_request_vote(self, a: dict) -> dict:
        if a["term"] > self.current_term:
            await self._step_down(a["term"], None)
        granted = False
        if a["term"] == self.current_term and self.voted_for in (None, a["candidate_id"]):
            my_last = self.last_index()
            my_term = self.term_at(my_last)
            if a["last_log_term"] > my_term or (a["last_log_term"] == my_term and a["last_log_index"] >= my_last):
                granted = True
                self.voted_for = a["candidate_id"]
                await self._persist_hard_state()
                self._reset_election_timer()
        return {"term": self.current_term, "vote_granted": granted, "peer_id": self.id}

    async def handle_append_entries(self, a: dict) -> dict:
        async with self._append_lock:
            if a["term"] < self.current_term:
                return {"term": self.current_term, "success": False, "match_index": self.last_index(),
                        "peer_id": self.id}
            if a["term"] > self.current_term or self.role != FOLLOWER:
                await self._step_down(a["term"], a.get("leader_address"), a.get("leader_id"))
            self.leader_id = a.get("leader_id")
            self.leader_address = a.get("leader_address")
            self._reset_election_timer()
            prev = a["prev_log_index"]
            if prev > self.last_index():
                return {"term": self.current_term, "success": False, "match_index": self.last_index(),
                        "peer_id": self.id}
            if prev >= self.last_included_index and self.term_at(prev) != a["prev_log_term"]:
                return {"term": self.current_term, "success": False,
                        "match_index": min(prev - 1, self.commit_index), "peer_id": self.id}
            recs: list[bytes] = []
            idx = prev
            for e in a["entries"]:
                idx += 1
                if idx <= self.last_included_index:
                    continue
                if idx <= self.last_index():
                    if self.term_at(idx) == e["term"]:
                        continue
                    log.debug("node %d truncating from %d (term %d, role %s) on append term %d from %s prev %d",
                              self.id, idx, self.current_term, self.role, a["term"], a.get("leader_id"), prev)
                    del self.log[idx - self.first_index:]
                    recs.append(json.dumps({"k": "T", "from": idx}).encode())
                self.log.append((e["term"], e["command"]))
                recs.append(self._entry_record(idx))
            await self._wal(recs)
            self._durable_index = self.last_index()
            last_new = prev + len(a["entries"])
            if a["leader_commit"] > self.commit_index:
                self.commit_index = min(a["leader_commit"], last_new)
                self._apply()
            return {"term": self.current_term, "success": True, "match_index": last_new, "peer_id": self.id}

    async def handle_install_snapshot(self, a: dict) -> dict:
        async with self._append_lock:
            if a["term"] < self.current_term:
                return {"term": self.current_term, "last_included_index": self.last_included_index,
                        "peer_id": self.id}
            if a["term"] > self.current_term or self.role != FOLLOWER:
                await self._step_down(a["term"], a.get("leader_address"), a.get("leader_id"))
            self.leader_address = a.get("leader_address")
            self._reset_election_timer()
            lii, lit = a["last_included_index"], a["last_included_term"]
            if lii <= self.last_included_index:
                return {"term": self.current_term, "last_included_index": self.last_included_index,
                        "peer_id": self.id}
            snap = json.loads(a["data"])
            native.atomic_write(self._snap_path(), a["data"].encode(), self.sync)
            if lii <= self.last_index() and self.term_at(lii) == lit:
                self.log = self.log[lii - self.first_index + 1:]
            else:
                self.log = []
            self.last_included_index, self.last_included_term = lii, lit
            if snap.get("config"):
                self.config = ClusterConfiguration.from_json(snap["config"])
            self.sm.restore(snap["state"])
            self.commit_index = max(self.commit_index, lii)
            self.last_applied = lii
            self._compact_wal()
            self._durable_index = self.last_index()
            return {"term": self.current_term, "last_included_index": lii, "peer_id": self.id}

    async def handle_timeout_now(self, a: dict) -> dict:
        if a["term"] >= self.current_term and self.role != LEADER:
            asyncio.get_running_loop().create_task(self._start_election())
            return {"term": self.current_term, "success": True}
        return {"term": self.current_term, "success": False}

    async def transfer_leadership(self, target: int) -> bool:
        if self.role != LEADER or target not in self.config.voters():
            return False
        try:
            r = await self.transport.send(self._addr(target), "timeout_now",
                                          {"term": self.current_term, "sender_id": self.id})
            return bool(r.get("success"))
        except Exception:  # noqa: BLE001
            return False

    # ------------------------------------------------------------------ snapshots
    def _maybe_snapshot(self) -> None:
        if self.last_applied - self.last_included_index > self.snapshot_threshold:
            self._take_snapshot()

    def _take_snapshot(self) -> None:
        idx = self.last_applied
        if idx < self.last_included_index:
            return
        term = self.term_at(idx)
        snap = {"meta": [idx, term], "state": self.sm.snapshot(), "config": self.config.to_json()}
        data = json.dumps(snap, separators=(",", ":"))
        native.atomic_write(self._snap_path(), data.encode(), self.sync)
        self.log = self.log[idx - self.first_index + 1:]
        self.last_included_index, self.last_included_term = idx, term
        self._compact_wal()
        log.info("node %d snapshot at %d (log now %d entries)", self.id, idx, len(self.log))
        if self.backup_s3_endpoint and self.role == LEADER:
            url = (f"{self.backup_s3_endpoint.rstrip('/')}/{self.backup_bucket}/master-snapshots/"
                   f"node-{self.id}/{int(time.time())}--idx{idx}.bin")
            asyncio.get_running_loop().create_task(self._backup(url, data.encode()))

    async def _backup(self, url: str, data: bytes) -> None:
        try:
            await self.transport.put_bytes(url, data)
        except Exception as e:  # noqa: BLE001
            log.warning("snapshot backup to %s failed: %s", url, e)

    def _compact_wal(self) -> None:
        recs = [self._hs_record(), self._config_record()]
        recs += [self._entry_record(i) for i in range(self.first_index, self.last_index() + 1)]
        self.wal.reset(recs)

    # ------------------------------------------------------------------ membership
    def _apply_membership(self, m: dict, idx: int) -> Any:
        members = dict(self.config.members)
        if "AddServer" in m:
            a = m["AddServer"]
            members[int(a["server_id"])] = a["server_address"]
            self.config = ClusterConfiguration(members, None, self.config.version + 1)
        elif "RemoveServer" in m:
            members.pop(int(m["RemoveServer"]["server_id"]), None)
            self.config = ClusterConfiguration(members, None, self.config.version + 1)
        elif "BeginJointConsensus" in m:
            b = m["BeginJointConsensus"]
            self.config = ClusterConfiguration({int(k): v for k, v in b["new_members"].items()},
                                               {int(k): v for k, v in b["old_members"].items()}, int(b["version"]))
        elif "FinalizeConfiguration" in m:
            f = m["FinalizeConfiguration"]
            self.config = ClusterConfiguration({int(k): v for k, v in f["new_members"].items()}, None,
                                               int(f["version"]))
        for p in self._peers():
            if p in self.config.voters():
                self.non_voting.pop(p, None)
            if self.role == LEADER and p not in self.next_index:
                self.next_index[p] = self.last_index() + 1
                self.match_index[p] = 0
        asyncio.get_running_loop().create_task(self._wal([self._config_record()]))
        if self.role == LEADER and self.id not in self.config.voters():
            asyncio.get_running_loop().create_task(self._step_down(self.current_term, None))
        return self.config.to_json()

    async def add_server(self, server_id: int, address: str) -> Any:
        return await self.propose({"Membership": {"AddServer": {"server_id": server_id, "server_address": address}}})

    async def remove_server(self, server_id: int) -> Any:
        return await self.propose({"Membership": {"RemoveServer": {"server_id": server_id}}})

    async def change_membership(self, new_members: dict[int, str], catch_up_timeout: float = 10.0) -> Any:
        """Joint consensus: new servers catch up as non-voters (10 rounds at commit), then
        C_old,new is committed, then C_new (reference simple_raft.rs:2458-2737)."""
        if self.role != LEADER:
            raise NotLeader(self.leader_address)
        added = {i: a for i, a in new_members.items() if i not in self.config.voters()}
        for i, a in added.items():
            self.non_voting[i] = a
            self.catch_up[i] = CatchUpProgress(added_at=time.time())
            self.next_index[i] = self.last_index() + 1
            self.match_index[i] = 0
        deadline = time.monotonic() + catch_up_timeout
        while added and time.monotonic() < deadline:
            self._broadcast()
            if all(self.catch_up[i].is_caught_up(self.commit_index) for i in added):
                break
            await asyncio.sleep(self.heartbeat_interval)
        v = self.config.version + 1
        await self.propose({"Membership": {"BeginJointConsensus": {
            "old_members": {str(k): x for k, x in self.config.members.items()},
            "new_members": {str(k): x for k, x in new_members.items()}, "version": v}}})
        res = await self.propose({"Membership": {"FinalizeConfiguration": {
            "new_members": {str(k): x for k, x in new_members.items()}, "version": v + 1}}})
        for i in added:
            self.catch_up.pop(i, None)
        return res

    # ------------------------------------------------------------------ introspection
    def is_leader(self) -> bool:
        return self.role == LEADER

    def cluster_info(self) -> dict:
        return {
            "node_id": self.id, "role": self.role, "current_term": self.current_term,
            "leader_id": self.leader_id, "leader_address": self.leader_address,
            "peers": [self._addr(p) for p in self._peers()], "commit_index": self.commit_index,
            "last_applied": self.last_applied, "log_len": self.last_index(),
            "votes_received": len(self.votes), "cluster_config": self.config.to_json(),
            "wal_bytes": self.wal.size_bytes, "wal_syncs": self.wal.syncs,
        }
