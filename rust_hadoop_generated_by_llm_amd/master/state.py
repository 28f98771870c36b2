"""Master replicated state machine (C24, C26, C28, C29).

Raft-persisted: ``files`` (path -> FileMetadata), ``transaction_records`` (2PC),
``shuffling_prefixes``. Local only (rebuilt from heartbeats): chunk-server registry,
pending commands, safe-mode counters, bad-block reports
(reference: dfs/metaserver/src/master.rs:195-367, simple_raft.rs:2995-3398).

Differences from the reference, all behaviour-preserving for clients:
* a ``block_id -> path`` index makes GetBlockLocations O(1) (the reference scans every
  file, master.rs:2699-2719);
* ``AddBlockLocation`` records replicas created by healer/balancer REPLICATE commands once
  the target chunkserver reports them, so the healer stops re-issuing the same copy
  (the reference never learns about new replicas);
* placement can put a writer-local chunkserver first (``preferred``) and treats each GPU
  ChunkServer of a node as its own failure domain inside the node's rack;
* files are invisible to GetFileInfo/ListFiles until CompleteFile (the reference shows a
  half-written file as an empty one, which a concurrent reader can observe — a
  linearizability violation), and CreateFile decides existence at apply time.
"""
from __future__ import annotations

import logging
import os
import time
from dataclasses import dataclass, field
from typing import Any

from ..models import meta as M
from ..models import proto as pb

log = logging.getLogger("dfs.master.state")

REPLICATION_FACTOR = 3
SAFE_MODE_THRESHOLD = 0.99
SAFE_MODE_TIMEOUT_MS = 60_000
TX_TIMEOUT_MS = int(os.environ.get("DFS_TX_TIMEOUT_MS", "10000"))  # reference: 10 s
TX_STALE_MS = 3_600_000
# a file left under construction this long (writer died) may be re-created by CreateFile
CREATE_LEASE_MS = int(os.environ.get("DFS_CREATE_LEASE_MS", "60000"))


def now_ms() -> int:
    return int(time.time() * 1000)


@dataclass
class ChunkServerStatus:
    last_heartbeat: int
    used_space: int = 0
    available_space: int = 0
    chunk_count: int = 0
    rack_id: str = ""
    gpu_rank: int = -1
    hbm_capacity: int = 0
    hbm_used: int = 0
    scheduled: int = 0  # bytes of blocks placed here since the last heartbeat (local only)


SCHEDULE_QUANTUM = 64 << 20

def select_servers_rack_aware(servers: list[tuple[str, ChunkServerStatus]], n: int,
                              preferred: str | None = None) -> list[str]:
    """Sort by available space, bucket by rack (an empty rack is its own bucket), then
    round-robin across racks (reference master.rs:378-432). ``preferred`` (writer-local
    chunkserver) is pinned to position 0 when it is live."""
    if n <= 0 or not servers:
        return []
    # free space net of blocks scheduled since the last heartbeat (HDFS-style), so a burst
    # of allocations between two heartbeats rotates over equally-free servers instead of
    # piling onto the same two (all GPU chunkservers of a node share one filesystem)
    cands = sorted(servers, key=lambda s: (-(s[1].available_space - s[1].scheduled), s[0]))
    selected: list[str] = []
    if preferred and any(a == preferred for a, _ in cands):
        selected.append(preferred)
        cands = [c for c in cands if c[0] != preferred]
    buckets: dict[str, list] = {}
    order: list[str] = []
    for addr, st in cands:
        key = st.rack_id if st.rack_id else f"__addr__{addr}"
        if key not in buckets:
            buckets[key] = []
            order.append(key)
        buckets[key].append((addr, st))
    # racks ordered by their best server (already sorted), preferred's rack goes last so
    # the next replicas spread to other racks first
    if selected:
        pref_rack = next((st.rack_id for a, st in servers if a == preferred), "")
        if pref_rack and pref_rack in buckets:
            order.remove(pref_rack)
            order.append(pref_rack)
    racks = [buckets[k] for k in order]
    pos = [0] * len(racks)
    while len(selected) < n:
        picked = False
        for i, rack in enumerate(racks):
            if len(selected) >= n:
                break
            if pos[i] < len(rack):
                selected.append(rack[pos[i]][0])
                pos[i] += 1
                picked = True
        if not picked:
            break
    return selected[:n]


class MasterState:
    def __init__(self):
        self.files: dict[str, Any] = {}
        self.transaction_records: dict[str, dict] = {}
        self.shuffling_prefixes: set[str] = set()
        self.block_index: dict[str, str] = {}
        # files between CreateFile and CompleteFile -> creation time (ms, from the command):
        # invisible to GetFileInfo/ListFiles so a concurrent reader never observes a
        # half-written (empty) file; an expired lease lets CreateFile take the path over
        self.under_construction: dict[str, int] = {}
        # paths pinned by an unresolved cross-shard rename (derived from
        # transaction_records): the source on the coordinator shard, the reserved
        # destination on the participant. Readers and writers of a pinned path wait for
        # the outcome, which makes the 2PC rename atomic to observers.
        self.tx_locks: dict[str, str] = {}
        # local (not replicated)
        self.chunk_servers: dict[str, ChunkServerStatus] = {}
        self.pending_commands: dict[str, list] = {}
        self.safe_mode = False
        self.safe_mode_entered_at = 0
        self.safe_mode_min_chunkservers = 1
        self.expected_block_count = 0
        self.reported_block_count = 0
        self.safe_mode_threshold = SAFE_MODE_THRESHOLD
        self.safe_mode_manual = False
        self.bad_block_locations: dict[str, set[str]] = {}
        self.applied_index = 0

    # ------------------------------------------------------------------ file index helpers
    def _put(self, path: str, m) -> None:
        old = self.files.get(path)
        if old is not None:
            for b in old.blocks:
                if self.block_index.get(b.block_id) == path:
                    del self.block_index[b.block_id]
        self.files[path] = m
        for b in m.blocks:
            self.block_index[b.block_id] = path

    def _del(self, path: str):
        self.under_construction.pop(path, None)
        m = self.files.pop(path, None)
        if m is not None:
            for b in m.blocks:
                if self.block_index.get(b.block_id) == path:
                    del self.block_index[b.block_id]
        return m

    def find_block(self, block_id: str):
        path = self.block_index.get(block_id)
        if path is None:
            return None, None
        m = self.files.get(path)
        if m is None:
            return None, None
        for b in m.blocks:
            if b.block_id == block_id:
                return m, b
        return None, None

    def count_total_blocks(self) -> int:
        return sum(len(f.blocks) for f in self.files.values())

    # ------------------------------------------------------------------ safe mode
    def enter_safe_mode(self) -> None:
        self.safe_mode = True
        self.safe_mode_entered_at = now_ms()
        self.safe_mode_min_chunkservers = 1
        self.safe_mode_threshold = SAFE_MODE_THRESHOLD
        self.expected_block_count = self.count_total_blocks()
        self.reported_block_count = 0
        self.safe_mode_manual = False
        log.info("entering safe mode: expecting %d blocks", self.expected_block_count)

    def should_exit_safe_mode(self) -> bool:
        if self.safe_mode_manual or not self.safe_mode:
            return False
        if len(self.chunk_servers) < self.safe_mode_min_chunkservers:
            return False
        if self.expected_block_count == 0:
            return True
        if self.reported_block_count / self.expected_block_count >= self.safe_mode_threshold:
            return True
        return now_ms() - self.safe_mode_entered_at > SAFE_MODE_TIMEOUT_MS

    def exit_safe_mode(self) -> None:
        if self.safe_mode:
            log.info("leaving safe mode (%d/%d blocks reported)", self.reported_block_count,
                     self.expected_block_count)
            self.safe_mode = False
            self.safe_mode_manual = False

    def force_enter_safe_mode(self) -> None:
        self.enter_safe_mode()
        self.safe_mode_manual = True

    def force_exit_safe_mode(self) -> None:
        self.safe_mode_manual = False
        self.exit_safe_mode()

    def update_reported_blocks(self, n: int) -> None:
        self.reported_block_count += n
        if self.should_exit_safe_mode():
            self.exit_safe_mode()

    # ------------------------------------------------------------------ replicated apply
    def apply(self, command: Any, index: int = 0) -> Any:
        self.applied_index = index
        if not isinstance(command, dict) or "Master" not in command:
            return None
        (name, a), = command["Master"].items()
        fn = getattr(self, "_cmd_" + name, None)
        if fn is None:
            log.warning("unknown master command %s", name)
            return None
        return fn(a)

    def _cmd_CreateFile(self, a):
        """Existence is decided here, in log order, so two racing creates of one path
        cannot both succeed. Returns the replaced (expired) metadata's blocks for GC."""
        path, ts = a["path"], int(a.get("ts", 0))
        if path in self.tx_locks:
            return {"locked": path}
        old = self.files.get(path)
        if old is not None:
            started = self.under_construction.get(path)
            if started is None or ts - started < CREATE_LEASE_MS:
                return {"exists": True}
        m = pb.FileMetadata(path=path, ec_data_shards=a.get("ec_data_shards", 0),
                            ec_parity_shards=a.get("ec_parity_shards", 0))
        if a.get("block_id"):
            b = m.blocks.add(block_id=a["block_id"], ec_data_shards=m.ec_data_shards,
                             ec_parity_shards=m.ec_parity_shards)
            b.locations.extend(a.get("locations", []))
        self._put(path, m)
        self.under_construction[path] = ts
        return {"exists": False, "orphans": [(b.block_id, list(b.locations)) for b in old.blocks] if old else []}

    def _cmd_CreateComplete(self, a):
        """Deferred create: the file appears, complete, in one entry (after its data)."""
        path, ts = a["path"], int(a.get("ts", 0))
        if path in self.tx_locks:
            return {"locked": path}
        old = self.files.get(path)
        if old is not None:
            started = self.under_construction.get(path)
            if started is None or ts - started < CREATE_LEASE_MS:
                return {"exists": True}
        m = pb.FileMetadata(path=path, ec_data_shards=a.get("ec_data_shards", 0),
                            ec_parity_shards=a.get("ec_parity_shards", 0))
        for bd in a.get("blocks", []):
            m.blocks.append(M.block_from_dict(bd))
        self._put(path, m)
        self.under_construction.pop(path, None)
        self._cmd_CompleteFile(a)
        return {"exists": False, "orphans": [(b.block_id, list(b.locations)) for b in old.blocks] if old else []}

    def visible(self, path: str):
        """Metadata of a completed file, else None."""
        if path in self.under_construction:
            return None
        return self.files.get(path)

    def _cmd_DeleteFile(self, a):
        if a["path"] in self.tx_locks:
            return {"locked": a["path"]}
        if self.visible(a["path"]) is None:
            return {"found": False}
        m = self._del(a["path"])
        return {"found": True, "blocks": [(b.block_id, list(b.locations)) for b in m.blocks]}

    def _cmd_AllocateBlock(self, a):
        m = self.files.get(a["path"])
        if m is None:
            return None
        b = m.blocks.add(block_id=a["block_id"], ec_data_shards=m.ec_data_shards,
                         ec_parity_shards=m.ec_parity_shards)
        b.locations.extend(a.get("locations", []))
        self.block_index[a["block_id"]] = a["path"]
        return None

    def _cmd_RegisterChunkServer(self, a):
        return None

    def _cmd_RenameFile(self, a):
        """Same-shard rename, decided in log order: the source must be a completed file and
        the destination must not exist (the reference silently overwrote it, so two racing
        renames onto one name could both "succeed")."""
        src, dst = a["source_path"], a["dest_path"]
        for p in (src, dst):
            if p in self.tx_locks:
                return {"locked": p}
        if self.visible(src) is None:
            return {"error": f"Source file not found: {src}"}
        if dst in self.files:
            return {"error": f"Destination file already exists: {dst}"}
        m = self._del(src)
        m.path = dst
        self._put(dst, m)
        return {"error": None}

    @staticmethod
    def _locked_path(rec: dict) -> str | None:
        ren = rec.get("tx_type", {}).get("Rename")
        if not ren or rec.get("state") in ("Committed", "Aborted"):
            return None
        return ren.get("source_path") or ren.get("dest_path") or None

    def _relock(self, rec: dict) -> None:
        for p, t in list(self.tx_locks.items()):
            if t == rec["tx_id"]:
                del self.tx_locks[p]
        p = self._locked_path(rec)
        if p:
            self.tx_locks[p] = rec["tx_id"]

    def _cmd_CreateTransactionRecord(self, a):
        """Admission happens here, in log order: a rename may only pin a path nobody else
        has pinned; the coordinator's source must be a completed file and the
        participant's destination must not exist. Returns {"conflict": reason} if not."""
        rec = a["record"]
        if rec["tx_id"] in self.transaction_records:
            return {"conflict": None}
        ren = rec.get("tx_type", {}).get("Rename")
        p = self._locked_path(rec)
        if ren and p:
            if self.tx_locks.get(p, rec["tx_id"]) != rec["tx_id"]:
                return {"conflict": f"{p} is locked by another transaction"}
            if ren.get("source_path"):
                if self.visible(p) is None:
                    return {"conflict": f"Source file not found: {p}"}
            elif p in self.files:
                return {"conflict": f"Destination file already exists: {p}"}
        self.transaction_records[rec["tx_id"]] = rec
        self._relock(rec)
        return {"conflict": None}

    def _cmd_UpdateTransactionState(self, a):
        rec = self.transaction_records.get(a["tx_id"])
        if rec is not None:
            rec["state"] = a["new_state"]
            self._relock(rec)

    def _cmd_ApplyTransactionOperation(self, a):
        op = a["operation"]["op_type"]
        if "Delete" in op:
            self._del(op["Delete"]["path"])
        elif "Create" in op:
            c = op["Create"]
            if c["path"] not in self.files:
                m = M.file_from_dict(c["metadata"])
                m.path = c["path"]
                self._put(c["path"], m)

    def _cmd_DeleteTransactionRecord(self, a):
        rec = self.transaction_records.pop(a["tx_id"], None)
        if rec is not None:
            rec = dict(rec, state="Aborted")
            self._relock(rec)

    def _cmd_SplitShard(self, a):
        if "paths" in a:  # explicit list: the files the post-split map routes away
            for p in a["paths"]:
                if p in self.files:
                    self._del(p)
            return
        key = a["split_key"]
        for p in [p for p in self.files if p >= key]:
            self._del(p)

    def _cmd_MergeShard(self, a):
        return None

    def _cmd_IngestBatch(self, a):
        for f in a["files"]:
            m = M.file_from_dict(f)
            self._put(m.path, m)

    def _cmd_TriggerShuffle(self, a):
        self.shuffling_prefixes.add(a["prefix"])

    def _cmd_StopShuffle(self, a):
        self.shuffling_prefixes.discard(a["prefix"])

    def _cmd_CompleteFile(self, a):
        m = self.files.get(a["path"])
        if m is None:
            return {"found": False}
        self.under_construction.pop(a["path"], None)
        m.size = a["size"]
        if a.get("etag_md5"):
            m.etag_md5 = a["etag_md5"]
        if a.get("created_at_ms"):
            m.created_at_ms = a["created_at_ms"]
        sums = a.get("block_checksums") or []
        if sums:
            by_id = {b.block_id: b for b in m.blocks}
            for s in sums:
                b = by_id.get(s["block_id"])
                if b is not None:
                    b.checksum_crc32c = s.get("checksum_crc32c", 0)
                    b.size = s.get("actual_size", 0)
                    b.original_size = s.get("actual_size", 0)
        elif m.blocks:
            n = len(m.blocks)
            per = m.size // n
            for b in m.blocks[:-1]:
                b.size = per
            m.blocks[-1].size = m.size - per * (n - 1)
        return {"found": True}

    def _cmd_UpdateAccessStats(self, a):
        m = self.files.get(a["path"])
        if m is not None:
            m.last_access_ms = a["accessed_at_ms"]
            m.access_count += 1

    def _cmd_UpdateAccessStatsBatch(self, a):
        t = a["accessed_at_ms"]
        for path, count in a["paths"].items():
            m = self.files.get(path)
            if m is not None:
                m.last_access_ms = t
                m.access_count += int(count)

    def _cmd_MoveToCold(self, a):
        m = self.files.get(a["path"])
        if m is not None:
            m.moved_to_cold_at_ms = a["moved_at_ms"]

    def _cmd_ConvertToEc(self, a):
        m = self.files.get(a["path"])
        if m is None:
            return None
        for b in m.blocks:
            self.block_index.pop(b.block_id, None)
        m.ec_data_shards = a["ec_data_shards"]
        m.ec_parity_shards = a["ec_parity_shards"]
        del m.blocks[:]
        for bd in a["new_blocks"]:
            m.blocks.append(M.block_from_dict(bd))
        for b in m.blocks:
            self.block_index[b.block_id] = m.path

    def _cmd_SetParticipantAcked(self, a):
        rec = self.transaction_records.get(a["tx_id"])
        if rec is not None:
            rec["participant_acked"] = True

    def _cmd_IncrementInquiryCount(self, a):
        rec = self.transaction_records.get(a["tx_id"])
        if rec is not None:
            rec["inquiry_count"] = rec.get("inquiry_count", 0) + 1

    def _cmd_AddBlockLocation(self, a):
        _, b = self.find_block(a["block_id"])
        if b is None:
            return
        idx = a.get("shard_index")
        if idx is not None and b.ec_data_shards > 0:
            # EC locations are positional (shard i lives at locations[i]): a rebuilt shard
            # replaces its dead holder instead of being appended
            if 0 <= idx < len(b.locations):
                b.locations[idx] = a["address"]
            return
        if a["address"] not in b.locations:
            b.locations.append(a["address"])

    def _cmd_UpdateBlockLocations(self, a):
        _, b = self.find_block(a["block_id"])
        if b is not None:
            del b.locations[:]
            b.locations.extend(a["locations"])

    # ------------------------------------------------------------------ snapshot serde
    def snapshot(self) -> dict:
        return {"Master": {
            "files": {p: M.file_to_dict(m) for p, m in self.files.items()},
            "transaction_records": self.transaction_records,
            "shuffling_prefixes": sorted(self.shuffling_prefixes),
            "under_construction": self.under_construction,
        }}

    def restore(self, state: dict) -> None:
        st = state.get("Master", state)  # legacy raw MasterState accepted too
        self.files = {}
        self.block_index = {}
        for p, d in st.get("files", {}).items():
            self._put(p, M.file_from_dict(d))
        self.transaction_records = dict(st.get("transaction_records", {}))
        self.tx_locks = {}
        for rec in self.transaction_records.values():
            self._relock(rec)
        self.shuffling_prefixes = set(st.get("shuffling_prefixes", []))
        self.under_construction = {p: int(t) for p, t in st.get("under_construction", {}).items()
                                   if p in self.files}

    # ------------------------------------------------------------------ healer (C29)
    def heal_under_replicated_blocks(self, rf: int = REPLICATION_FACTOR) -> int:
        """Queue REPLICATE / RECONSTRUCT_EC_SHARD commands (reference master.rs:436-602)."""
        live = sorted(self.chunk_servers)
        if not live:
            return 0
        issued = 0
        T = pb.ChunkServerCommand
        for f in self.files.values():
            for b in f.blocks:
                if b.ec_data_shards > 0:
                    k = b.ec_data_shards
                    total = b.ec_data_shards + b.ec_parity_shards
                    if len(b.locations) != total:
                        continue
                    live_count = sum(1 for loc in b.locations if loc in self.chunk_servers)
                    for idx, loc in enumerate(b.locations):
                        if loc in self.chunk_servers:
                            continue
                        if live_count < k:
                            break
                        target = next((s for s in live if s not in b.locations), None)
                        if target is None:
                            continue
                        srcs = [l if l in self.chunk_servers else "" for l in b.locations]
                        self.pending_commands.setdefault(target, []).append(T(
                            type=T.RECONSTRUCT_EC_SHARD, block_id=b.block_id, target_chunk_server_address=target,
                            shard_index=idx, ec_data_shards=b.ec_data_shards, ec_parity_shards=b.ec_parity_shards,
                            ec_shard_sources=srcs, original_block_size=b.original_size))
                        issued += 1
                else:
                    bad_on = self.bad_block_locations.get(b.block_id, set())
                    live_locs = [l for l in b.locations if l in self.chunk_servers and l not in bad_on]
                    needed = max(0, min(rf, len(live)) - len(live_locs))
                    if needed == 0 or not live_locs:
                        continue
                    src = live_locs[0]
                    queued = {c.target_chunk_server_address for c in self.pending_commands.get(src, [])
                              if c.block_id == b.block_id}
                    targets = [s for s in live if s not in b.locations and s not in queued][:needed]
                    for t in targets:
                        self.pending_commands.setdefault(src, []).append(T(
                            type=T.REPLICATE, block_id=b.block_id, target_chunk_server_address=t, shard_index=-1))
                        issued += 1
        return issued
