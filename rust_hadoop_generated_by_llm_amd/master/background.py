"""Master background tasks (reference: dfs/metaserver/src/master.rs:729-2138, spawned by
MyMaster::new at :1856-1896 and the tiering loop in bin/master.rs:229-238):

liveness (5 s, 15 s timeout) · healer (60 s, then 300 s) · balancer (30 s) ·
tx cleanup (5 s) · tx recovery (30 s) · data shuffler (10 s) · metrics decay (5 s) ·
shard-map refresh (5 s) · split/merge detector (5 s) · tiering + EC conversion (60 s).

Intervals are constructor arguments so tests can run them fast.
"""
from __future__ import annotations

import asyncio
import logging
import os
import uuid
from dataclasses import dataclass

from ..models import meta as M
from ..models import proto as pb
from ..parallel.sharding import ShardMap
from ..raft.node import NotLeader
from ..utils.rpc import rpc_details
from .service import MasterService
from .state import TX_STALE_MS, TX_TIMEOUT_MS, now_ms

log = logging.getLogger("dfs.master.bg")

MAX_INQUIRY_RETRIES = 60
CS_DEAD_MS = int(os.environ.get("DFS_CS_DEAD_MS", "15000"))  # reference: 15 s
BALANCE_GAP = 100 * 1024 * 1024
EC_JOB_TIMEOUT_MS = 120_000


@dataclass
class Intervals:
    liveness: float = 5.0
    healer_first: float = 60.0
    healer: float = 300.0
    balancer: float = 30.0
    tx_cleanup: float = 5.0
    tx_recovery: float = 30.0
    shuffler: float = 10.0
    decay: float = 5.0
    shard_refresh: float = 1.0  # reference: 5 s; a stale map misroutes renames
    split: float = 5.0
    tiering: float = 60.0


def _timed_out(rec: dict) -> bool:
    return now_ms() - rec.get("timestamp", 0) > TX_TIMEOUT_MS


def _stale(rec: dict) -> bool:
    return now_ms() - rec.get("timestamp", 0) > TX_STALE_MS


class MasterBackground:
    def __init__(self, svc: MasterService, config_servers: list[str], intervals: Intervals | None = None,
                 cold_threshold_secs: int = 604800, ec_threshold_secs: int = 2592000,
                 ec_conversion: bool | None = None):
        self.svc = svc
        self.state = svc.state
        self.raft = svc.raft
        self.config_servers = config_servers
        self.iv = intervals or Intervals()
        self.cold_threshold_ms = cold_threshold_secs * 1000
        self.ec_threshold_ms = ec_threshold_secs * 1000
        self.ec_conversion = (os.environ.get("EC_CONVERSION_ENABLED", "0") == "1") if ec_conversion is None \
            else ec_conversion
        # reference converts to RS(6,3); smaller codes for small clusters / tests
        self.ec_k = int(os.environ.get("EC_CONVERSION_DATA_SHARDS", "6"))
        self.ec_m = int(os.environ.get("EC_CONVERSION_PARITY_SHARDS", "3"))
        self.registered = False
        self._tasks: list[asyncio.Task] = []
        if config_servers:
            svc.shard_map_refresher = self.refresh_shard_map
            # the native Rename trusts the map only while it is this young (else: Python refreshes)
            svc.core.set_shard_map_max_age(svc.shard_map_max_age_ms)

    def start(self) -> None:
        loop = asyncio.get_running_loop()
        jobs = [
            (self.iv.liveness, self.liveness_check, self.iv.liveness),
            (self.iv.healer_first, self.periodic_heal, self.iv.healer),
            (self.iv.balancer, self.balance, self.iv.balancer),
            (self.iv.tx_cleanup, self.tx_cleanup, self.iv.tx_cleanup),
            (self.iv.tx_recovery, self.tx_recovery, self.iv.tx_recovery),
            (self.iv.shuffler, self.shuffle, self.iv.shuffler),
            (self.iv.decay, self.decay, self.iv.decay),
            (self.iv.shard_refresh, self.refresh_shard_map, self.iv.shard_refresh),
            (self.iv.split, self.split_detector, self.iv.split),
            (self.iv.tiering, self.tiering, self.iv.tiering),
            (0.25, self.heartbeat_reports, 0.25),
        ]
        for first, fn, every in jobs:
            self._tasks.append(loop.create_task(self._every(first, fn, every)))

    async def stop(self) -> None:
        for t in self._tasks:
            t.cancel()
        for t in self._tasks:
            try:
                await t
            except (asyncio.CancelledError, Exception):  # noqa: BLE001
                pass

    async def _every(self, first: float, fn, every: float) -> None:
        await asyncio.sleep(first)
        while True:
            try:
                await fn()
            except asyncio.CancelledError:
                raise
            except Exception:  # noqa: BLE001
                log.exception("background task %s failed", fn.__name__)
            await asyncio.sleep(every)

    async def _propose(self, name: str, args: dict) -> bool:
        try:
            await self.raft.propose({"Master": {name: args}})
            return True
        except NotLeader:
            return False

    # ---------------------------------------------------------------- liveness + healing
    async def liveness_check(self) -> None:
        now = now_ms()
        dead = [a for a, s in self.state.chunk_servers.items() if now - s.last_heartbeat > CS_DEAD_MS]
        for a in dead:
            log.warning("chunkserver %s missed heartbeats; removing", a)
            del self.state.chunk_servers[a]
            self.state.pending_commands.pop(a, None)
        if dead:
            self.state.heal_under_replicated_blocks()

    async def heartbeat_reports(self) -> None:
        """What the native Heartbeat handler recorded: a bad block report triggers a heal pass
        right away (as the reference's heartbeat handler does), EC conversion results update
        tiering's jobs."""
        self.svc.drain_heartbeat_reports()
        if self.state.core.take_heal_request():
            n = self.state.heal_under_replicated_blocks()
            if n:
                log.info("healer queued %d commands after a bad-block report", n)

    async def periodic_heal(self) -> None:
        n = self.state.heal_under_replicated_blocks()
        if n:
            log.info("healer queued %d commands", n)

    # ---------------------------------------------------------------- balancer / shuffler
    def _pick_block(self, src: str, dst: str, prefix: str | None = None) -> str | None:
        # one native pass under the state lock (no per-file decode in Python)
        return self.state.core.pick_block(src, dst, prefix) or None

    async def balance(self) -> None:
        servers = sorted(self.state.chunk_servers.items(), key=lambda kv: kv[1].available_space)
        if len(servers) < 2:
            return
        (fullest, lo), (emptiest, hi) = servers[0], servers[-1]
        if hi.available_space - lo.available_space <= BALANCE_GAP:
            return
        bid = self._pick_block(fullest, emptiest)
        if bid:
            T = pb.ChunkServerCommand
            self.state.pending_commands.setdefault(fullest, []).append(
                T(type=T.REPLICATE, block_id=bid, target_chunk_server_address=emptiest))
            log.info("balancer: replicate %s %s -> %s", bid, fullest, emptiest)

    async def shuffle(self) -> None:
        prefixes = sorted(self.state.shuffling_prefixes)
        servers = sorted(self.state.chunk_servers.items(), key=lambda kv: -kv[1].available_space)
        if not prefixes or len(servers) < 2:
            return
        coolest, hottest = servers[0][0], servers[-1][0]
        T = pb.ChunkServerCommand
        for p in prefixes:
            bid = self._pick_block(hottest, coolest, p)
            if bid:
                self.state.pending_commands.setdefault(hottest, []).append(
                    T(type=T.REPLICATE, block_id=bid, target_chunk_server_address=coolest))
            elif self.raft.is_leader():
                await self._propose("StopShuffle", {"prefix": p})

    # ---------------------------------------------------------------- 2PC maintenance
    async def _inquire(self, rec: dict) -> str | None:
        peers = self.svc.shard_map.get_shard_peers(rec.get("coordinator_shard", "")) or \
            rec.get("coordinator_peers", [])
        for addr in peers:
            try:
                r = await self.svc.pool.call(addr, "MasterService", "InquireTransaction",
                                             pb.InquireTransactionRequest(tx_id=rec["tx_id"]), timeout=3.0)
                return r.status
            except Exception as e:  # noqa: BLE001
                log.debug("inquire %s at %s failed: %s", rec["tx_id"], addr, rpc_details(e))
        return None

    async def tx_cleanup(self) -> None:
        if not self.raft.is_leader():
            return
        shard = self.svc.shard_id
        for tx_id, rec in list(self.state.transaction_records.items()):
            if not (_timed_out(rec) or _stale(rec)):
                continue
            st = rec["state"]
            coord = rec.get("coordinator_shard", "")
            if not coord:
                if st in ("Pending", "Prepared") and _timed_out(rec):
                    await self._propose("UpdateTransactionState", {"tx_id": tx_id, "new_state": "Aborted"})
                elif _stale(rec):
                    await self._propose("DeleteTransactionRecord", {"tx_id": tx_id})
                continue
            is_coord = coord == shard
            if st == "Pending":
                await self._propose("UpdateTransactionState", {"tx_id": tx_id, "new_state": "Aborted"})
            elif st == "Prepared" and not is_coord:
                status = await self._inquire(rec)
                if status == "COMMITTED":
                    if rec.get("operations"):
                        await self._propose("ApplyTransactionOperation",
                                            {"tx_id": tx_id, "operation": rec["operations"][0]})
                    await self._propose("UpdateTransactionState", {"tx_id": tx_id, "new_state": "Committed"})
                elif status == "ABORTED":
                    await self._propose("UpdateTransactionState", {"tx_id": tx_id, "new_state": "Aborted"})
                elif status == "UNKNOWN":
                    await self._propose("IncrementInquiryCount", {"tx_id": tx_id})
                    if rec.get("inquiry_count", 0) + 1 > MAX_INQUIRY_RETRIES:
                        log.warning("tx %s: presuming abort after %d inquiries", tx_id, MAX_INQUIRY_RETRIES)
                        await self._propose("UpdateTransactionState", {"tx_id": tx_id, "new_state": "Aborted"})
            elif st in ("Committed", "Aborted") and _stale(rec):
                if st == "Committed" and is_coord and not rec.get("participant_acked"):
                    continue
                await self._propose("DeleteTransactionRecord", {"tx_id": tx_id})

    async def tx_recovery(self) -> None:
        if not self.raft.is_leader():
            return
        shard = self.svc.shard_id
        for tx_id, rec in list(self.state.transaction_records.items()):
            if rec.get("coordinator_shard") != shard:
                continue
            st = rec["state"]
            if not ((st == "Committed" and not rec.get("participant_acked")) or (st == "Prepared" and _timed_out(rec))):
                continue
            dest = next((p for p in rec.get("participants", []) if p != shard), "")
            peers = self.svc.shard_map.get_shard_peers(dest) or []
            if not peers:
                continue
            if not await self.svc.send_commit(tx_id, peers):
                continue
            src_op = next((op for op in rec.get("operations", []) if "Delete" in op["op_type"]), None)
            if st == "Prepared" and src_op is not None:
                await self._propose("ApplyTransactionOperation", {"tx_id": tx_id, "operation": src_op})
                await self._propose("UpdateTransactionState", {"tx_id": tx_id, "new_state": "Committed"})
            await self._propose("SetParticipantAcked", {"tx_id": tx_id})
            log.info("tx %s recovered (participant committed)", tx_id)

    # ---------------------------------------------------------------- sharding
    async def decay(self) -> None:
        self.svc.monitor.decay_metrics()

    async def _config_call(self, method: str, request):
        last = None
        for addr in self.config_servers:
            try:
                return await self.svc.pool.call(addr, "ConfigService", method, request, timeout=5.0)
            except Exception as e:  # noqa: BLE001
                last = e
        if last is not None:
            log.debug("config %s failed: %s", method, rpc_details(last))
        return None

    async def refresh_shard_map(self) -> None:
        if not self.config_servers:
            return
        resp = await self._config_call("FetchShardMap", pb.FetchShardMapRequest())
        if resp is None or not resp.shards:
            return
        new = ShardMap.from_fetch(resp)
        self.svc.shard_map_fetched_ms = now_ms()
        m = self.svc.shard_map
        m.strategy, m.ranges, m.ring, m.shards, m.shard_peers = new.strategy, new.ranges, new.ring, new.shards, \
            new.shard_peers
        m._dirty()
        self.svc.sync_routing()
        self.svc.core.note_shard_map_fresh()
        if not self.svc.shard_id:  # standby master: a SplitShard allocated us a shard
            me = self.svc.advertise_addr
            for sid in m.get_all_shards():
                if me in (m.get_shard_peers(sid) or []):
                    self.svc.shard_id = sid
                    log.info("standby master %s now serves shard %s", me, sid)
                    break

    async def register(self) -> None:
        if self.registered or not self.config_servers:
            return
        r = await self._config_call("RegisterMaster", pb.RegisterMasterRequest(address=self.svc.advertise_addr,
                                                                              shard_id=self.svc.shard_id))
        self.registered = bool(r and r.success)

    async def split_detector(self) -> None:
        if not self.config_servers:
            return
        mon = self.svc.monitor
        addr = self.svc.advertise_addr
        await self.register()
        hb = pb.ShardHeartbeatRequest(address=addr)
        for p, v in mon.rps_per_prefix().items():
            hb.rps_per_prefix[p] = v
        await self._config_call("ShardHeartbeat", hb)
        if not self.raft.is_leader():
            return
        hot = mon.hot_prefix()
        if hot is not None and self.svc.shard_id:
            prefix, rps = hot
            await self._split(prefix, rps)
            return
        total = mon.total_rps()
        if 0 <= mon.merge_threshold_rps and total < mon.merge_threshold_rps and self.state.files \
                and self.svc.shard_id:
            prev, nxt = self.svc.shard_map.get_neighbors(self.svc.shard_id)
            neighbor = prev or nxt
            if neighbor is None:
                return
            await self._merge_into(neighbor)

    async def _merge_into(self, neighbor: str) -> None:
        """Hand this idle shard's range and files to ``neighbor`` (C31 merge). The config
        server's MergeShard goes first because it arbitrates: two idle neighbours may try
        to merge into each other and only one MergeShard can apply. The winner then pushes
        its files (IngestMetadata, retried until the retained shard takes them), drops its
        namespace in one Raft entry and re-registers as a standby master that a later split
        can reuse. The reference reports success to both and keeps serving stale copies."""
        victim = self.svc.shard_id
        r = await self._config_call("MergeShard", pb.MergeShardRequest(victim_shard_id=victim,
                                                                       retained_shard_id=neighbor))
        if r is None or not r.success:
            return
        peers = self.svc.shard_map.get_shard_peers(neighbor) or []
        self.svc.shard_id = ""  # stop accepting our old range (requests now redirect)
        paths = list(self.state.files)
        for attempt in range(30):
            req = pb.IngestMetadataRequest(files=[self.state.files[p] for p in paths if p in self.state.files])
            if not req.files or await self.svc._call_peers(peers, "IngestMetadata", req, lambda x: x.success):
                break
            await asyncio.sleep(min(0.1 * (attempt + 1), 1.0))
        else:
            log.error("merge of %s into %s: ingest kept failing; files stay here", victim, neighbor)
            return
        await self._propose("SplitShard", {"split_key": "", "new_shard_id": neighbor, "new_shard_peers": [],
                                           "paths": paths})
        log.info("merged shard %s into %s; now standby", victim, neighbor)
        self.registered = False
        await self.refresh_shard_map()

    async def _split(self, prefix: str, rps: float) -> None:
        """Split this shard at ``prefix`` (C31). The files that move are exactly the ones the
        post-split map routes to the new shard (reference ShardMap semantics: the new id takes
        the keys below the split key), so routing and data agree — the reference deletes
        ``p >= key`` while routing the other side there, and ships the batch after the
        delete (master.rs:1600-1615). Order: config SplitShard (allocates standby masters),
        IngestMetadata at the new shard, then one Raft entry dropping the moved files here."""
        import time as _t

        mon = self.svc.monitor
        new_id = f"{self.svc.shard_id}-split-{uuid.uuid4().hex[:8]}"
        after = self.svc.shard_map.copy()
        if not after.split_shard(prefix, new_id, []):
            mon.last_split_time = _t.monotonic()
            return
        log.info("hot prefix %s (%.1f rps): splitting shard %s -> %s", prefix, rps, self.svc.shard_id, new_id)
        mon.last_split_time = _t.monotonic()
        moving = [p for p in self.state.files if after.get_shard(p) == new_id]
        r = await self._config_call("SplitShard", pb.SplitShardRequest(
            shard_id=self.svc.shard_id, split_key=prefix, new_shard_id=new_id))
        if r is None or not r.success:
            log.warning("config server refused split of %s at %s", self.svc.shard_id, prefix)
            return
        if moving:
            req = pb.IngestMetadataRequest(files=[self.state.files[p] for p in moving if p in self.state.files])
            await self.svc._call_peers(list(r.new_shard_peers), "IngestMetadata", req, lambda x: x.success)
        await self._propose("SplitShard", {"split_key": prefix, "new_shard_id": new_id,
                                           "new_shard_peers": list(r.new_shard_peers), "paths": moving})
        await self.refresh_shard_map()

    # ---------------------------------------------------------------- tiering (C32)
    async def tiering(self) -> None:
        if not self.raft.is_leader():
            return
        now = now_ms()
        T = pb.ChunkServerCommand
        # the namespace scan is native (MasterCore::tiering_scan): only idle files come back
        for path, blocks in self.state.core.tiering_scan(now, self.cold_threshold_ms):
            for bid, locs in blocks:
                for loc in locs:
                    self.state.pending_commands.setdefault(loc, []).append(T(type=T.MOVE_TO_COLD, block_id=bid))
            await self._propose("MoveToCold", {"path": path, "moved_at_ms": now})
        if not self.ec_conversion:
            return
        await self._ec_convert(now)

    async def _ec_convert(self, now: int) -> None:
        """Cold files older than EC_THRESHOLD_SECS become RS(k,m): each block is re-encoded
        by a chunkserver holding a replica (ENCODE_EC, GPU RS kernel) into shards under a new
        block id; once every block of the file reported success one Raft ConvertToEc swaps
        the metadata and the old replicas get DELETE. Jobs are leader-local; a failed or
        lost job is simply retried on a later pass."""
        k, m = self.ec_k, self.ec_m
        T = pb.ChunkServerCommand
        jobs = self.svc.ec_jobs
        for bid, job in list(jobs.items()):
            if not job["done"] and now - job["started_ms"] > EC_JOB_TIMEOUT_MS:
                log.warning("EC job for %s timed out; will retry", bid)
                jobs.pop(bid, None)
        live = {a for a, s in self.state.chunk_servers.items() if s.available_space > 0}
        for raw in self.state.core.ec_candidates(now, self.ec_threshold_ms):
            f = pb.FileMetadata.FromString(raw)
            if all(b.block_id in jobs and jobs[b.block_id]["done"] for b in f.blocks):
                new_blocks = []
                for b in f.blocks:
                    job = jobs[b.block_id]
                    d = M.block_to_dict(b)
                    d.update(block_id=job["new_id"], locations=job["targets"], ec_data_shards=job["k"],
                             ec_parity_shards=job["m"], original_size=b.original_size or b.size)
                    new_blocks.append(d)
                old = [(b.block_id, list(b.locations)) for b in f.blocks]
                jk, jm = jobs[f.blocks[0].block_id]["k"], jobs[f.blocks[0].block_id]["m"]
                ok = await self._propose("ConvertToEc", {"path": f.path, "ec_data_shards": jk,
                                                         "ec_parity_shards": jm, "new_blocks": new_blocks})
                for bid, locs in old:
                    jobs.pop(bid, None)
                    if ok:
                        for loc in locs:
                            self.state.pending_commands.setdefault(loc, []).append(T(type=T.DELETE, block_id=bid))
                if ok:
                    log.info("converted %s to RS(%d,%d)", f.path, jk, jm)
                continue
            servers = sorted(live)[: k + m]
            if len(servers) < k + m:
                continue
            for b in f.blocks:
                if b.block_id in jobs:
                    continue
                src = next((loc for loc in b.locations if loc in live), None)
                if src is None:
                    continue
                new_id = f"{b.block_id}-rs{k}.{m}"
                jobs[b.block_id] = {"path": f.path, "new_id": new_id, "targets": servers, "k": k, "m": m,
                                    "started_ms": now, "done": False}
                self.state.pending_commands.setdefault(src, []).append(
                    T(type=T.ENCODE_EC, block_id=b.block_id, new_block_id=new_id, ec_data_shards=k,
                      ec_parity_shards=m, ec_shard_sources=servers, original_block_size=b.size,
                      master_term=self.raft.current_term))
