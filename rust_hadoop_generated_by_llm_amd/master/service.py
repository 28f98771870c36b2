"""MasterService gRPC handlers (C27, C33) on grpc.aio + the Raft node.

Status codes and message strings match the reference so unmodified clients behave the
same (reference: dfs/metaserver/src/master.rs:2141-3660):
* wrong shard            -> OUT_OF_RANGE ``REDIRECT:<first peer of owning shard>``
* not leader (reads)     -> FAILED_PRECONDITION ``Not Leader|<leader>``
* not leader (writes)    -> success=false, error_message ``Not Leader``, leader_hint
* safe mode (writes)     -> UNAVAILABLE ``Cluster is in Safe Mode. Write operations are blocked.``
"""
from __future__ import annotations

import asyncio
import json
import logging
import os
import uuid
from concurrent.futures import ThreadPoolExecutor

from ..models import meta as M
from ..models import proto as pb
from ..parallel.sharding import ShardMap
from ..raft.node import NotLeader, RaftNode
from ..utils.rpc import AioChannelPool, RpcStatus, StatusCode, rpc_details
from .monitor import ThroughputMonitor
from .state import ChunkServerStatus, MasterState, now_ms

log = logging.getLogger("dfs.master")

SAFE_MODE_MSG = "Cluster is in Safe Mode. Write operations are blocked."
_CODES = {c.value[0]: c for c in StatusCode}


def new_rename_record(tx_id, source_path, dest_path, source_shard, dest_shard, dest_meta) -> dict:
    return {
        "tx_id": tx_id,
        "tx_type": {"Rename": {"source_path": source_path, "dest_path": dest_path}},
        "state": "Pending",
        "timestamp": now_ms(),
        "participants": [source_shard, dest_shard],
        "operations": [
            {"shard_id": source_shard, "op_type": {"Delete": {"path": source_path}}},
            {"shard_id": dest_shard, "op_type": {"Create": {"path": dest_path, "metadata": M.file_to_dict(dest_meta)}}},
        ],
        "coordinator_shard": source_shard,
        "participant_acked": False,
        "inquiry_count": 0,
    }


class MasterService:
    def __init__(self, state: MasterState, raft: RaftNode, shard_map: ShardMap, shard_id: str,
                 monitor: ThroughputMonitor, pool: AioChannelPool, *, advertise_addr: str = "",
                 access_stats: bool = True, access_stats_flush_ms: int = 1000):
        self.state = state
        self.core = state.core
        self.raft = raft
        self.shard_map = shard_map
        self._shard_id = shard_id
        self._exec = ThreadPoolExecutor(max_workers=16, thread_name_prefix="master-native")
        self.monitor = monitor
        self.pool = pool
        self.advertise_addr = advertise_addr
        self.core.set_access_stats(access_stats, access_stats_flush_ms)
        self.sync_routing()
        # set by MasterBackground when config servers exist: a rename decides same-shard
        # vs 2PC from the shard map, so it refreshes a map older than this first
        self.shard_map_refresher = None
        self.shard_map_fetched_ms = 0
        self.shard_map_max_age_ms = 1000
        # leader-local EC conversion jobs (tiering, C32): source block id ->
        # {"path", "new_id", "targets", "k", "m", "started_ms", "done"}
        self.ec_jobs: dict[str, dict] = {}

    @property
    def shard_id(self) -> str:
        return self._shard_id

    @shard_id.setter
    def shard_id(self, value: str) -> None:
        self._shard_id = value
        self.sync_routing()

    def sync_routing(self) -> None:
        """Push the shard map + our shard id into the native handlers (ownership checks)."""
        self.core.set_shard_map(json.dumps(self.shard_map.to_json()), self._shard_id)

    async def fresh_shard_map(self, force: bool = False) -> None:
        if self.shard_map_refresher is None:
            return
        if not force and now_ms() - self.shard_map_fetched_ms < self.shard_map_max_age_ms:
            return
        try:
            await asyncio.wait_for(self.shard_map_refresher(), 2.0)
        except Exception as e:  # noqa: BLE001 - fall back to the cached map
            log.debug("shard map refresh before rename failed: %s", e)

    # ------------------------------------------------------------------ guards
    def check_shard_ownership(self, path: str) -> None:
        target = self.shard_map.get_shard(path)
        if target is not None and target != self.shard_id:
            # our map may be the stale one (e.g. a shard registered moments ago): refresh it
            # in the background so a client bounced between two masters converges
            if self.shard_map_refresher is not None and \
                    now_ms() - self.shard_map_fetched_ms >= self.shard_map_max_age_ms:
                self.shard_map_fetched_ms = now_ms()
                asyncio.get_running_loop().create_task(self.fresh_shard_map(force=True))
            peers = self.shard_map.get_shard_peers(target) or []
            raise RpcStatus(StatusCode.OUT_OF_RANGE, f"REDIRECT:{peers[0] if peers else ''}")

    async def wait_unlocked(self, path: str, timeout: float = 5.0) -> None:
        """Block while ``path`` is pinned by an unresolved cross-shard rename."""
        if path not in self.state.tx_locks:
            return
        loop = asyncio.get_running_loop()
        end = loop.time() + timeout
        delay = 0.002
        while path in self.state.tx_locks:
            if loop.time() > end:
                raise RpcStatus(StatusCode.UNAVAILABLE, f"{path} is locked by transaction "
                                                        f"{self.state.tx_locks.get(path)}")
            await asyncio.sleep(delay)
            delay = min(delay * 2, 0.05)

    def check_safe_mode(self) -> None:
        if self.state.safe_mode:
            raise RpcStatus(StatusCode.UNAVAILABLE, SAFE_MODE_MSG)

    async def ensure_linearizable_read(self) -> None:
        try:
            await self.raft.read_index()
        except NotLeader as e:
            raise RpcStatus(StatusCode.FAILED_PRECONDITION, f"Not Leader|{e.hint}" if e.hint else "Not Leader")

    async def _propose(self, name: str, args: dict):
        return await self.raft.propose({"Master": {name: args}})

    async def _propose_unlocked(self, name: str, args: dict, attempts: int = 50):
        """Propose a namespace mutation whose apply refuses paths pinned by an in-flight
        cross-shard rename ({"locked": path}); wait for the pin to clear and retry."""
        for _ in range(attempts):
            res = await self._propose(name, args)
            if not (isinstance(res, dict) and res.get("locked")):
                return res
            await self.wait_unlocked(res["locked"])
        raise RpcStatus(StatusCode.UNAVAILABLE, f"{name}: path stays locked by cross-shard renames")

    # ------------------------------------------------------------------ native hot path
    async def _native(self, method: str, req, resp_cls):
        """GetFileInfo / CreateFile / AllocateBlock / CompleteFile / ListFiles / DeleteFile /
        GetBlockLocations run in the native MasterCore (the same-host RPC listener calls it
        directly; gRPC requests come through here on a worker thread)."""
        code, out = await asyncio.get_running_loop().run_in_executor(
            self._exec, self.core.handle, method, req.SerializeToString())
        if code != 0:
            raise RpcStatus(_CODES.get(code, StatusCode.UNKNOWN), out.decode("utf-8", "replace"))
        return resp_cls.FromString(out)

    async def get_file_info(self, req, ctx):
        return await self._native("GetFileInfo", req, pb.GetFileInfoResponse)

    async def create_file(self, req, ctx):
        return await self._native("CreateFile", req, pb.CreateFileResponse)

    async def delete_file(self, req, ctx):
        return await self._native("DeleteFile", req, pb.DeleteFileResponse)

    async def allocate_block(self, req, ctx):
        return await self._native("AllocateBlock", req, pb.AllocateBlockResponse)

    async def complete_file(self, req, ctx):
        return await self._native("CompleteFile", req, pb.CompleteFileResponse)

    async def list_files(self, req, ctx):
        return await self._native("ListFiles", req, pb.ListFilesResponse)

    async def get_block_locations(self, req, ctx):
        return await self._native("GetBlockLocations", req, pb.GetBlockLocationsResponse)

    async def register_chunk_server(self, req, ctx):
        self.state.chunk_servers[req.address] = ChunkServerStatus(
            last_heartbeat=now_ms(), available_space=req.capacity, rack_id=req.rack_id)
        return pb.RegisterChunkServerResponse(success=True)

    async def heartbeat(self, req, ctx):
        """Served natively (MasterCore::heartbeat) on the native gRPC server and the local
        socket; this is the grpcio path (no native server), the same native handler."""
        return await self._native("Heartbeat", req, pb.HeartbeatResponse)

    def drain_heartbeat_reports(self) -> None:
        """EC conversion reports the native Heartbeat recorded (tiering's jobs live here)."""
        encoded, failed = self.core.take_ec_reports()
        for bid in encoded:
            job = self.ec_jobs.get(bid)
            if job is not None:
                job["done"] = True
        for bid in failed:
            if self.ec_jobs.pop(bid, None) is not None:
                log.warning("EC conversion of block %s failed; will retry", bid)

    # ------------------------------------------------------------------ rename / 2PC
    async def rename(self, req, ctx):
        src, dst = req.source_path, req.dest_path
        self.monitor.record_request(src)
        await self.fresh_shard_map()
        self.check_shard_ownership(src)
        self.check_safe_mode()
        src_shard = self.shard_map.get_shard(src) or self.shard_id
        dst_shard = self.shard_map.get_shard(dst) or self.shard_id
        dst_peers = self.shard_map.get_shard_peers(dst_shard) or []
        await self.wait_unlocked(src)
        if src_shard == dst_shard:
            await self.wait_unlocked(dst)
        meta = self.state.visible(src)
        if meta is None:
            return pb.RenameResponse(success=False, error_message=f"Source file not found: {src}")
        if src_shard == dst_shard:
            try:
                res = await self._propose_unlocked("RenameFile", {"source_path": src, "dest_path": dst})
            except NotLeader as e:
                return pb.RenameResponse(success=False, error_message="Not Leader", leader_hint=e.hint)
            if isinstance(res, dict) and res.get("error"):
                return pb.RenameResponse(success=False, error_message=res["error"])
            return pb.RenameResponse(success=True)
        tx_id = str(uuid.uuid4())
        dmeta = pb.FileMetadata()
        dmeta.CopyFrom(meta)
        dmeta.path = dst
        rec = new_rename_record(tx_id, src, dst, src_shard, dst_shard, dmeta)
        try:
            res = await self._propose("CreateTransactionRecord", {"record": rec})
        except NotLeader as e:
            return pb.RenameResponse(success=False, error_message="Not Leader", leader_hint=e.hint)
        if isinstance(res, dict) and res.get("conflict"):
            return pb.RenameResponse(success=False, error_message=res["conflict"])
        try:
            await self._propose("UpdateTransactionState", {"tx_id": tx_id, "new_state": "Prepared"})
        except Exception:  # noqa: BLE001
            await self.send_abort(tx_id, dst_peers)
            return pb.RenameResponse(success=False, error_message="Internal error: Raft commit failed")
        ok = await self.send_prepare(tx_id, dst, dmeta, dst_peers)
        if not ok:
            await self.send_abort(tx_id, dst_peers)
            try:
                await self._propose("UpdateTransactionState", {"tx_id": tx_id, "new_state": "Aborted"})
            except Exception:  # noqa: BLE001
                pass
            return pb.RenameResponse(success=False, error_message="Cross-shard prepare failed")
        if os.environ.get("DFS_DEBUG_2PC_DROP_COMMIT") == "1":
            # fault injection (tests): behave as if the coordinator died right after the
            # participant prepared; tx_recovery must finish the rename
            log.warning("tx %s: debug hook dropped the commit RPC", tx_id)
            return pb.RenameResponse(success=False, error_message="Cross-shard commit pending, will be retried")
        if not await self.send_commit(tx_id, dst_peers):
            log.warning("commit RPC failed for tx %s; recovery task will retry", tx_id)
            return pb.RenameResponse(success=False, error_message="Cross-shard commit pending, will be retried")
        await self._finish_coordinator_commit(tx_id, src_shard, src)
        return pb.RenameResponse(success=True)

    async def _finish_coordinator_commit(self, tx_id: str, src_shard: str, src: str) -> None:
        try:
            await self._propose("ApplyTransactionOperation", {
                "tx_id": tx_id, "operation": {"shard_id": src_shard, "op_type": {"Delete": {"path": src}}}})
            await self._propose("UpdateTransactionState", {"tx_id": tx_id, "new_state": "Committed"})
            await self._propose("SetParticipantAcked", {"tx_id": tx_id})
        except Exception as e:  # noqa: BLE001
            log.error("tx %s: coordinator finish failed: %s", tx_id, e)

    async def _call_peers(self, peers: list[str], method: str, request, ok) -> bool:
        """Try each peer of the shard, following ``leader_hint`` on Not Leader."""
        tried: set[str] = set()
        queue = list(peers)
        while queue:
            addr = queue.pop(0)
            if addr in tried or not addr:
                continue
            tried.add(addr)
            try:
                resp = await self.pool.call(addr, "MasterService", method, request, timeout=5.0)
            except Exception as e:  # noqa: BLE001
                log.debug("%s to %s failed: %s", method, addr, rpc_details(e))
                continue
            if ok(resp):
                return True
            hint = getattr(resp, "leader_hint", "")
            if hint and hint not in tried:
                queue.insert(0, hint)
            elif getattr(resp, "error_message", "") not in ("Not Leader", ""):
                return False
        return False

    async def send_prepare(self, tx_id, path, meta, peers) -> bool:
        req = pb.PrepareTransactionRequest(tx_id=tx_id, operation_type="CREATE", path=path, metadata=meta,
                                           coordinator_shard=self.shard_id,
                                           coordinator_peers=self.shard_map.get_shard_peers(self.shard_id) or [])
        return await self._call_peers(peers, "PrepareTransaction", req, lambda r: r.success)

    async def send_commit(self, tx_id, peers) -> bool:
        return await self._call_peers(peers, "CommitTransaction", pb.CommitTransactionRequest(tx_id=tx_id),
                                      lambda r: r.success)

    async def send_abort(self, tx_id, peers) -> bool:
        return await self._call_peers(peers, "AbortTransaction", pb.AbortTransactionRequest(tx_id=tx_id),
                                      lambda r: r.success)

    async def prepare_transaction(self, req, ctx):
        if req.tx_id in self.state.transaction_records:
            return pb.PrepareTransactionResponse(success=True)
        await self.fresh_shard_map()
        self.check_shard_ownership(req.path)
        try:
            await self.wait_unlocked(req.path, timeout=1.0)
        except RpcStatus:
            return pb.PrepareTransactionResponse(success=False,
                                                 error_message=f"Destination is locked by another transaction: {req.path}")
        if req.path in self.state.files:
            return pb.PrepareTransactionResponse(success=False,
                                                 error_message=f"Destination file already exists: {req.path}")
        meta = req.metadata if req.HasField("metadata") else pb.FileMetadata()
        rec = {
            "tx_id": req.tx_id, "tx_type": {"Rename": {"source_path": "", "dest_path": req.path}},
            "state": "Prepared", "timestamp": now_ms(), "participants": [req.coordinator_shard, self.shard_id],
            "operations": [{"shard_id": self.shard_id,
                            "op_type": {"Create": {"path": req.path, "metadata": M.file_to_dict(meta)}}}],
            "coordinator_shard": req.coordinator_shard, "participant_acked": False, "inquiry_count": 0,
            "coordinator_peers": list(req.coordinator_peers),
        }
        try:
            res = await self._propose("CreateTransactionRecord", {"record": rec})
        except NotLeader as e:
            return pb.PrepareTransactionResponse(success=False, error_message="Not Leader", leader_hint=e.hint)
        if isinstance(res, dict) and res.get("conflict"):
            return pb.PrepareTransactionResponse(success=False, error_message=res["conflict"])
        return pb.PrepareTransactionResponse(success=True)

    async def commit_transaction(self, req, ctx):
        rec = self.state.transaction_records.get(req.tx_id)
        if rec is not None and rec["state"] == "Committed":
            return pb.CommitTransactionResponse(success=True)
        if rec is None or not rec.get("operations"):
            return pb.CommitTransactionResponse(success=False, error_message=f"Transaction not found: {req.tx_id}")
        try:
            await self._propose("ApplyTransactionOperation", {"tx_id": req.tx_id, "operation": rec["operations"][0]})
        except NotLeader as e:
            return pb.CommitTransactionResponse(success=False, error_message="Not Leader", leader_hint=e.hint)
        try:
            await self._propose("UpdateTransactionState", {"tx_id": req.tx_id, "new_state": "Committed"})
        except Exception:  # noqa: BLE001
            pass
        return pb.CommitTransactionResponse(success=True)

    async def abort_transaction(self, req, ctx):
        try:
            await self._propose("UpdateTransactionState", {"tx_id": req.tx_id, "new_state": "Aborted"})
        except NotLeader as e:
            return pb.AbortTransactionResponse(success=False, error_message="Not Leader", leader_hint=e.hint)
        return pb.AbortTransactionResponse(success=True)

    async def inquire_transaction(self, req, ctx):
        await self.ensure_linearizable_read()
        rec = self.state.transaction_records.get(req.tx_id)
        status = "UNKNOWN"
        if rec is not None:
            status = {"Committed": "COMMITTED", "Aborted": "ABORTED"}.get(rec["state"], "UNKNOWN")
        return pb.InquireTransactionResponse(status=status)

    # ------------------------------------------------------------------ safe mode
    async def get_safe_mode_status(self, req, ctx):
        await self.ensure_linearizable_read()
        st = self.state
        return pb.GetSafeModeStatusResponse(
            is_safe_mode=st.safe_mode, is_manual=st.safe_mode_manual, chunk_server_count=len(st.chunk_servers),
            expected_blocks=st.expected_block_count, reported_blocks=st.reported_block_count,
            threshold=st.safe_mode_threshold, entered_at=st.safe_mode_entered_at)

    async def set_safe_mode(self, req, ctx):
        if req.enter:
            self.state.force_enter_safe_mode()
        else:
            self.state.force_exit_safe_mode()
        return pb.SetSafeModeResponse(success=True, is_safe_mode=self.state.safe_mode)

    # ------------------------------------------------------------------ membership
    async def add_raft_server(self, req, ctx):
        try:
            await self.raft.add_server(req.server_id, req.server_address)
        except NotLeader as e:
            return pb.AddRaftServerResponse(success=False, error_message="Not Leader", leader_hint=e.hint)
        return pb.AddRaftServerResponse(success=True)

    async def remove_raft_server(self, req, ctx):
        if not self.raft.is_leader():
            return pb.RemoveRaftServerResponse(success=False, error_message="Not Leader",
                                               leader_hint=self.raft.leader_address or "")
        if len(self.raft.config.voters()) <= 1:
            return pb.RemoveRaftServerResponse(success=False,
                                               error_message="Cannot remove server: would leave cluster empty")
        try:
            await self.raft.remove_server(req.server_id)
        except NotLeader as e:
            return pb.RemoveRaftServerResponse(success=False, error_message="Not Leader", leader_hint=e.hint)
        return pb.RemoveRaftServerResponse(success=True)

    async def get_cluster_info(self, req, ctx):
        info = self.raft.cluster_info()
        members = [pb.ClusterMember(server_id=i, address=a, is_self=(i == self.raft.id))
                   for i, a in sorted(self.raft.config.all_members().items())]
        return pb.GetClusterInfoResponse(
            node_id=info["node_id"], role=info["role"], current_term=info["current_term"],
            leader_id=info["leader_id"] or 0, leader_address=info["leader_address"] or "", members=members,
            commit_index=info["commit_index"], last_applied=info["last_applied"])

    # ------------------------------------------------------------------ sharding
    async def ingest_metadata(self, req, ctx):
        prefix = None
        if req.files:
            p = req.files[0].path
            if "/" in p:
                prefix = p[: p.rfind("/") + 1]
        try:
            await self._propose("IngestBatch", {"files": [M.file_to_dict(f) for f in req.files]})
        except NotLeader as e:
            return pb.IngestMetadataResponse(success=False, error_message="Not Leader", leader_hint=e.hint)
        if prefix:
            self.raft.propose_nowait({"Master": {"TriggerShuffle": {"prefix": prefix}}})
        return pb.IngestMetadataResponse(success=True)

    async def initiate_shuffle(self, req, ctx):
        self.check_shard_ownership(req.prefix)
        self.check_safe_mode()
        try:
            await self._propose("TriggerShuffle", {"prefix": req.prefix})
        except NotLeader as e:
            return pb.InitiateShuffleResponse(success=False, error_message="Not Leader", leader_hint=e.hint)
        return pb.InitiateShuffleResponse(success=True)
