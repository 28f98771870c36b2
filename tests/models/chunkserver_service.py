"""ChunkServerService (C37-C42) on top of the native HBM ChunkStore.

WriteBlock / ReplicateBlock / ReadBlock keep the reference's wire semantics
(dfs/chunkserver/src/chunkserver.rs:721-1088): epoch fencing, CRC verification, local
durable write, store-and-forward chain replication with ``replicas_written`` counting,
downstream errors logged-not-returned, full-read verification with synchronous recovery,
partial-read verification with background recovery.

The forwarding hop is where the MI355X design departs: when the next chunkserver is a
GPU rank of the same node, the block goes ``ncclSend`` -> ``ncclRecv`` straight from
this GPU's HBM into the peer's HBM over xGMI (csrc/replication.cpp, sliced and checksummed
as it lands) and the gRPC ReplicateBlock carries only a descriptor (rccl_src_rank,
rccl_gen, rccl_seq, rccl_size, rccl_slice). Any failure aborts that pair (it is rebuilt
under a new generation in the background) and this block falls back to the reference
gRPC data path.
"""
from __future__ import annotations

import logging
import threading
from concurrent.futures import ThreadPoolExecutor

from rust_hadoop_generated_by_llm_amd.models import proto as pb
from rust_hadoop_generated_by_llm_amd.native import lib as _native
from rust_hadoop_generated_by_llm_amd.ops import erasure
from rust_hadoop_generated_by_llm_amd.utils.rpc import ChannelPool, RpcStatus, StatusCode, rpc_details, strip_scheme
from rust_hadoop_generated_by_llm_amd.utils.shm import ShmMapper

log = logging.getLogger("dfs.chunkserver")

ST_OK, ST_NOT_FOUND, ST_OUT_OF_RANGE, ST_CORRUPT, ST_IO = 0, 1, 2, 3, 4


class ChunkServer:
    def __init__(self, store, advertise_addr: str, pool: ChannelPool, masters_fn, rccl=None,
                 rank_map: dict[str, int] | None = None, my_rank: int = -1, metrics=None, fastpath=None):
        self.store = store
        # native local data path (csrc/fastpath.cpp); when present it owns the fencing term
        self.fastpath = fastpath
        self.fastpath_socket = fastpath.name if fastpath is not None else ""
        self.addr = advertise_addr
        self.pool = pool
        self.masters_fn = masters_fn  # () -> list of master addresses
        self.rccl = rccl
        self.rank_map = {strip_scheme(k): v for k, v in (rank_map or {}).items()}
        self.my_rank = my_rank
        self.known_term = 0
        self._term_lock = threading.Lock()
        self.pending_bad_blocks: list[str] = []
        self.new_blocks: list[str] = []
        self.ec_encoded: list[str] = []
        self.ec_failed: list[str] = []
        self.ec_rebuilt: list[str] = []
        self._lists_lock = threading.Lock()
        self._bg = ThreadPoolExecutor(max_workers=4, thread_name_prefix="cs-bg")
        self._fwd = ThreadPoolExecutor(max_workers=64, thread_name_prefix="cs-fwd")
        self.metrics = metrics
        self.stats = {"writes": 0, "reads": 0, "replicas_in": 0, "rccl_forwards": 0, "grpc_forwards": 0,
                      "rccl_fallbacks": 0, "recoveries": 0, "shm_writes": 0, "shm_reads": 0}
        self.shm = ShmMapper()
        # native control loop (csrc/cs_agent.cpp): when set, it owns the heartbeat, the master's
        # commands, recovery and the scrubber; the paths below delegate to it
        self.agent = None

    # ------------------------------------------------------------------ fencing
    def fence(self, term: int) -> None:
        if self.fastpath is not None:
            ok, known = self.fastpath.fence(term)
            self.known_term = known
            if not ok:
                raise RpcStatus(StatusCode.FAILED_PRECONDITION,
                                f"Stale master term: request has {term} but known term is {known}")
            return
        with self._term_lock:
            known = self.known_term
            if 0 < term < known:
                raise RpcStatus(StatusCode.FAILED_PRECONDITION,
                                f"Stale master term: request has {term} but known term is {known}")
            if term > known:
                self.known_term = term

    def adopt_term(self, term: int) -> None:
        if self.fastpath is not None:
            self.fastpath.adopt_term(term)
            self.known_term = self.fastpath.term
            return
        with self._term_lock:
            if term > self.known_term:
                self.known_term = term

    def queue_recovery(self, block_id: str) -> None:
        if self.agent is not None:
            self.agent.queue_recovery(block_id)
            return
        self._bg.submit(self.recover_block, block_id)

    # ------------------------------------------------------------------ forwarding
    def _rank_of(self, addr: str) -> int | None:
        return self.rank_map.get(strip_scheme(addr))

    def forward(self, block_id: str, data: bytes | None, next_servers: list[str], crc: int, term: int,
                heal: bool = False) -> int:
        """Send the block to next_servers[0] with the rest of the chain; returns the
        downstream replicas_written (0 on failure, which is logged, not raised)."""
        nxt, rest = next_servers[0], list(next_servers[1:])
        peer = self._rank_of(nxt)
        if self.rccl is not None and peer is not None and self.rccl.pair_ok(peer):
            tk, err = self.rccl.send(peer, block_id, None if self.store.gpu else data)
            if tk is not None:
                req = pb.ReplicateBlockRequest(block_id=block_id, next_servers=rest, expected_checksum_crc32c=crc,
                                               master_term=term, rccl=True, rccl_src_rank=self.my_rank,
                                               rccl_seq=tk.seq, rccl_size=tk.size, rccl_gen=tk.gen,
                                               rccl_slice=tk.slice, rccl_channel=tk.ch, heal=heal)
                resp = None
                try:
                    resp = self.pool.call(nxt, "ChunkServerService", "ReplicateBlock", req, timeout=120.0)
                except Exception as e:  # noqa: BLE001
                    log.error("P2P descriptor to %s failed: %s", nxt, rpc_details(e))
                if resp is None:
                    # the posted send can never be matched: the engine aborts and rebuilds the pair
                    self.rccl.cancel_send(tk, "descriptor failed")
                else:
                    ok, werr = self.rccl.wait_send(tk)
                    if resp.success or ok:
                        self.stats["rccl_forwards"] += 1
                        if resp.success:
                            return resp.replicas_written
                        log.error("downstream replication failed at %s: %s", nxt, resp.error_message)
                        return 0
                self.stats["rccl_fallbacks"] += 1
                log.warning("P2P path %d->%d failed; falling back to gRPC", self.my_rank, peer)
            else:
                log.warning("P2P send to rank %d unavailable: %s", peer, err)
        if data is None:
            st, _total, data, _p, _b, err = self.store.read(block_id, 0, 0)
            if st != ST_OK:
                log.error("cannot forward %s: %s", block_id, err)
                return 0
        elif not isinstance(data, bytes):
            data = bytes(data)  # short-circuit shm view -> owned payload for the gRPC hop
        req = pb.ReplicateBlockRequest(block_id=block_id, data=data, next_servers=rest,
                                       expected_checksum_crc32c=crc, master_term=term, heal=heal)
        try:
            resp = self.pool.call(nxt, "ChunkServerService", "ReplicateBlock", req, timeout=120.0)
        except Exception as e:  # noqa: BLE001
            log.error("failed to replicate to %s: %s", nxt, rpc_details(e))
            return 0
        self.stats["grpc_forwards"] += 1
        if not resp.success:
            log.error("downstream replication failed at %s: %s", nxt, resp.error_message)
            return 0
        return resp.replicas_written

    # ------------------------------------------------------------------ RPCs
    def _store_and_forward(self, block_id: str, data: bytes | None, next_servers: list[str], crc: int, term: int,
                           heal: bool, rccl_src: int = -1, rccl_seq: int = -1, rccl_size: int = 0,
                           rccl_gen: int = 0, rccl_slice: int = 0, rccl_channel: int = 0):
        """Local write + downstream forwarding, pipelined.

        The reference writes+fsyncs locally and only then forwards (serial chain,
        chunkserver.rs:777-819). Here the block is first *staged* (landed in HBM and
        CRC-verified), then the forward to the next replica (RCCL send from HBM, or gRPC)
        runs concurrently with the local fdatasync. The ack still waits for both, so the
        durability contract (every counted replica is on NVMe) is unchanged while the
        chain latency drops from sum(hops x (copy + 2 fsync)) to roughly one fsync.
        Returns (ok, error, replicas_written)."""
        if rccl_src >= 0:
            ok, _crc, err = self.rccl.recv(rccl_src, rccl_gen, rccl_seq, block_id, rccl_size, rccl_slice, crc,
                                           persist=not next_servers, ch=rccl_channel)
            staged_in_hbm = True
        elif next_servers and self.store.gpu:
            ok, _crc, err = self.store.stage(block_id, data, crc)
            staged_in_hbm = True
        elif next_servers:
            # CPU store: forward and write at the same time (downstream re-verifies the CRC)
            fut = self._fwd.submit(self.forward, block_id, data, next_servers, crc, term, heal)
            ok, _crc, err = self.store.write(block_id, data, crc)
            down = fut.result()
            return ok, err, (1 + down) if ok else 0
        else:
            ok, _crc, err = self.store.write(block_id, data, crc)
            return ok, err, 1 if ok else 0
        if not ok:
            return False, err, 0
        if not next_servers:
            return True, "", 1
        fut = self._fwd.submit(self.forward, block_id, data, next_servers, crc, term, heal)
        pok, perr = self.store.persist(block_id, data if rccl_src < 0 else None)
        down = fut.result()
        if not pok:
            return False, perr, 0
        _ = staged_in_hbm
        return True, "", 1 + down

    def write_block(self, req, ctx):
        self.fence(req.master_term)
        data = req.data
        if req.shm_path:
            try:
                data = self.shm.view(req.shm_path, req.shm_offset, req.shm_length)
            except (OSError, ValueError) as e:
                raise RpcStatus(StatusCode.FAILED_PRECONDITION, f"short-circuit unavailable: {e}")
            self.stats["shm_writes"] += 1
        ok, err, replicas = self._store_and_forward(req.block_id, data, list(req.next_servers),
                                                    req.expected_checksum_crc32c, req.master_term, False)
        if not ok:
            return pb.WriteBlockResponse(success=False, error_message=err)
        self.stats["writes"] += 1
        return pb.WriteBlockResponse(success=True, replicas_written=replicas,
                                     fastpath_socket=self.fastpath_socket if req.shm_path else "")

    def replicate_block(self, req, ctx):
        self.fence(req.master_term)
        if req.rccl and self.rccl is None:
            return pb.ReplicateBlockResponse(success=False, error_message="RCCL transport not enabled")
        if req.rccl:
            ok, err, replicas = self._store_and_forward(req.block_id, None, list(req.next_servers),
                                                        req.expected_checksum_crc32c, req.master_term, req.heal,
                                                        req.rccl_src_rank, req.rccl_seq, req.rccl_size,
                                                        req.rccl_gen, req.rccl_slice, req.rccl_channel)
        else:
            ok, err, replicas = self._store_and_forward(req.block_id, req.data, list(req.next_servers),
                                                        req.expected_checksum_crc32c, req.master_term, req.heal)
        if not ok:
            if err.startswith("Checksum mismatch"):
                err = "Replication c" + err[1:]
            return pb.ReplicateBlockResponse(success=False, error_message=err)
        self.stats["replicas_in"] += 1
        if req.heal:
            if self.agent is not None:
                self.agent.report_new_block(req.block_id)
            else:
                with self._lists_lock:
                    self.new_blocks.append(req.block_id)
        return pb.ReplicateBlockResponse(success=True, replicas_written=replicas)

    def _read_shm(self, req):
        try:
            out = self.shm.view(req.shm_path, req.shm_offset, req.shm_capacity)
        except (OSError, ValueError) as e:
            raise RpcStatus(StatusCode.FAILED_PRECONDITION, f"short-circuit unavailable: {e}")
        st, total, n, partial_bad, bad_slice, err = self.store.read_into(req.block_id, req.offset, req.length, out)
        if st == ST_CORRUPT:
            log.error("CRITICAL: data corruption detected for block %s: %s", req.block_id, err)
            rec_err = self.recover_block(req.block_id)
            if rec_err is not None:
                raise RpcStatus(StatusCode.DATA_LOSS, f"Data corruption detected: {err}. Recovery failed: {rec_err}")
            st, total, n, partial_bad, bad_slice, err = self.store.read_into(req.block_id, req.offset, req.length,
                                                                             out)
            if st != ST_OK:
                raise RpcStatus(StatusCode.DATA_LOSS, f"Recovered block is still corrupted: {err}")
        elif st == ST_NOT_FOUND:
            raise RpcStatus(StatusCode.NOT_FOUND, "Block not found")
        elif st == ST_OUT_OF_RANGE:
            raise RpcStatus(StatusCode.OUT_OF_RANGE, err)
        elif st != ST_OK:
            raise RpcStatus(StatusCode.INTERNAL, f"Failed to read block: {err}")
        if partial_bad:
            self._bg.submit(self.recover_block, req.block_id)
        self.stats["reads"] += 1
        self.stats["shm_reads"] += 1
        return pb.ReadBlockResponse(bytes_read=n, total_size=total, shm_filled=True,
                                    fastpath_socket=self.fastpath_socket)

    def read_block(self, req, ctx):
        if req.shm_path:
            return self._read_shm(req)
        st, total, data, partial_bad, bad_slice, err = self.store.read(req.block_id, req.offset, req.length)
        if st == ST_NOT_FOUND:
            raise RpcStatus(StatusCode.NOT_FOUND, "Block not found")
        if st == ST_OUT_OF_RANGE:
            raise RpcStatus(StatusCode.OUT_OF_RANGE, err)
        if st == ST_IO:
            raise RpcStatus(StatusCode.INTERNAL, f"Failed to read block: {err}")
        if st == ST_CORRUPT:
            log.error("CRITICAL: data corruption detected for block %s: %s", req.block_id, err)
            rec_err = self.recover_block(req.block_id)
            if rec_err is not None:
                raise RpcStatus(StatusCode.DATA_LOSS, f"Data corruption detected: {err}. Recovery failed: {rec_err}")
            st, total, data, _p, _b, err2 = self.store.read(req.block_id, req.offset, req.length)
            if st != ST_OK:
                raise RpcStatus(StatusCode.DATA_LOSS, f"Recovered block is still corrupted: {err2}")
        elif partial_bad:
            log.warning("partial read verification failed for %s (offset=%d): %s", req.block_id, req.offset, err)
            self._bg.submit(self.recover_block, req.block_id)
        self.stats["reads"] += 1
        return pb.ReadBlockResponse(data=data, bytes_read=len(data), total_size=total)

    # ------------------------------------------------------------------ recovery
    def block_locations(self, block_id: str) -> list[str]:
        for m in self.masters_fn():
            try:
                r = self.pool.call(m, "MasterService", "GetBlockLocations",
                                   pb.GetBlockLocationsRequest(block_id=block_id), timeout=5.0)
                if r.found:
                    return list(r.locations)
            except Exception as e:  # noqa: BLE001
                log.debug("GetBlockLocations via %s failed: %s", m, rpc_details(e))
        return []

    def recover_block(self, block_id: str) -> str | None:
        """Fetch a healthy replica, verify it against OUR .meta, rewrite locally
        (reference recover_block, chunkserver.rs:353-460; the self-skip uses the
        advertise address instead of the CHUNK_SERVER_ADDR env quirk)."""
        self.stats["recoveries"] += 1
        if self.agent is not None:
            err = self.agent.recover(block_id)
            return err or None
        locs = self.block_locations(block_id)
        if not locs:
            return "No replica locations found for block"
        local_meta = self.store.meta(block_id)
        me = strip_scheme(self.addr)
        for loc in locs:
            if strip_scheme(loc) == me:
                continue
            try:
                r = self.pool.call(loc, "ChunkServerService", "ReadBlock",
                                   pb.ReadBlockRequest(block_id=block_id), timeout=60.0)
            except Exception as e:  # noqa: BLE001
                log.debug("recovery read from %s failed: %s", loc, rpc_details(e))
                continue
            if local_meta and _native.crc32_meta(r.data) != local_meta:
                log.warning("fetched block %s from %s is also corrupted", block_id, loc)
                continue
            ok, _c, err = self.store.write(block_id, r.data, 0)
            if ok:
                log.info("recovered block %s from %s", block_id, loc)
                return None
        return "Failed to recover block from any replica"

    def initiate_replication(self, block_id: str, target: str) -> bool:
        if not self.store.exists(block_id):
            log.error("REPLICATE: block %s not held here", block_id)
            return False
        if self.fastpath is not None and self.rccl is not None:
            # same-node target with a P2P pair: the copy runs on the replication engine (HBM ->
            # HBM over xGMI on GPUs), the descriptor on the target's fast-path socket, no Python
            # on the receiving side (VERDICT r2 item 6 / SURVEY M7)
            n, _done = self.fastpath.replicate_block(block_id, [strip_scheme(target)], self.known_term)
            if n > 0:
                self.stats["rccl_forwards"] += 1
                return True
        n = self.forward(block_id, None, [target], 0, self.known_term, heal=True)
        return n > 0

    def reconstruct_ec_shard(self, cmd) -> bool:
        """Rebuild one EC shard from >= k survivors (reference chunkserver.rs:503-640);
        the GF(2^8) decode runs on the GPU when the store has one."""
        k, m = cmd.ec_data_shards, cmd.ec_parity_shards
        srcs = list(cmd.ec_shard_sources)
        if len(srcs) != k + m:
            log.error("ec_shard_sources length %d != %d", len(srcs), k + m)
            return False
        shards: list[bytes | None] = [None] * (k + m)
        futs = {}
        for i, a in enumerate(srcs):
            if a and i != cmd.shard_index:
                futs[i] = self._bg.submit(
                    self.pool.call, a, "ChunkServerService", "ReadBlock", pb.ReadBlockRequest(block_id=cmd.block_id),
                    60.0)
        for i, f in futs.items():
            try:
                shards[i] = f.result().data
            except Exception as e:  # noqa: BLE001
                log.warning("EC shard %d fetch failed: %s", i, rpc_details(e))
        if sum(1 for s in shards if s is not None) < k:
            log.error("EC reconstruct of %s: fewer than %d shards available", cmd.block_id, k)
            return False
        full = erasure.reconstruct(shards, k, m, self.store)
        ok, _c, err = self.store.write(cmd.block_id, full[cmd.shard_index], 0)
        if ok:
            with self._lists_lock:  # the master puts us at the shard's index, not at the end
                self.ec_rebuilt.append(f"{cmd.block_id}/{cmd.shard_index}")
        return ok

    def encode_ec(self, cmd) -> bool:
        """Tiering's EC conversion (C32) done for real: read the verified local replica,
        RS(k,m)-encode it (GF(2^8) kernel on the GPU when the store has one) and write shard
        i as block ``new_block_id`` to ec_shard_sources[i]. The master swaps the file to the
        new shards only after every block reported success, then deletes the replicas —
        the reference converts metadata only and never re-encodes (master.rs:2108-2118)."""
        k, m = cmd.ec_data_shards, cmd.ec_parity_shards
        targets = list(cmd.ec_shard_sources)
        new_id = cmd.new_block_id
        ok = False
        try:
            if k <= 0 or m <= 0 or len(targets) != k + m or not new_id:
                raise ValueError(f"bad ENCODE_EC command for {cmd.block_id}")
            st, _total, data, _p, _b, err = self.store.read(cmd.block_id, 0, 0)
            if st != ST_OK:
                raise ValueError(f"source replica unreadable: {err}")
            shards = erasure.encode(data, k, m, self.store)
            me = strip_scheme(self.addr)

            def put(i: int) -> None:
                crc = _native.crc32(shards[i])
                if strip_scheme(targets[i]) == me:
                    w_ok, _c, w_err = self.store.write(new_id, shards[i], crc)
                    if not w_ok:
                        raise ValueError(f"local shard {i}: {w_err}")
                    return
                r = self.pool.call(targets[i], "ChunkServerService", "WriteBlock",
                                   pb.WriteBlockRequest(block_id=new_id, data=shards[i], expected_checksum_crc32c=crc,
                                                        shard_index=i, master_term=cmd.master_term), timeout=60.0)
                if not r.success:
                    raise ValueError(f"shard {i} at {targets[i]}: {r.error_message}")

            with ThreadPoolExecutor(max_workers=min(16, k + m), thread_name_prefix="cs-ec") as ex:
                for f in [ex.submit(put, i) for i in range(k + m)]:
                    f.result()
            ok = True
            log.info("encoded %s as RS(%d,%d) -> %s", cmd.block_id, k, m, new_id)
        except Exception as e:  # noqa: BLE001
            log.error("ENCODE_EC %s failed: %s", cmd.block_id, rpc_details(e) if hasattr(e, "code") else e)
        with self._lists_lock:
            (self.ec_encoded if ok else self.ec_failed).append(cmd.block_id)
        return ok

    def handle_command(self, cmd) -> None:
        if self.agent is not None:
            self.agent.submit_command(cmd.SerializeToString())
            return
        T = pb.ChunkServerCommand
        if cmd.master_term:
            self.adopt_term(cmd.master_term)
        if cmd.type == T.REPLICATE:
            self._bg.submit(self.initiate_replication, cmd.block_id, cmd.target_chunk_server_address)
        elif cmd.type == T.RECONSTRUCT_EC_SHARD:
            self._bg.submit(self.reconstruct_ec_shard, cmd)
        elif cmd.type == T.MOVE_TO_COLD:
            self._bg.submit(self.store.move_to_cold, cmd.block_id)
        elif cmd.type == T.DELETE:
            self._bg.submit(self.store.remove, cmd.block_id)
        elif cmd.type == T.ENCODE_EC:
            self._bg.submit(self.encode_ec, cmd)

    def drain_reports(self) -> tuple[list[str], list[str], list[str], list[str], list[str]]:
        """(bad blocks, new blocks, EC jobs finished, EC jobs failed, EC shards rebuilt) for
        the next heartbeat."""
        healed = self.fastpath.drain_healed() if self.fastpath is not None else []
        with self._lists_lock:
            bad, self.pending_bad_blocks = self.pending_bad_blocks, []
            new, self.new_blocks = self.new_blocks + healed, []
            enc, self.ec_encoded = self.ec_encoded, []
            fail, self.ec_failed = self.ec_failed, []
            rebuilt, self.ec_rebuilt = self.ec_rebuilt, []
        return bad, new, enc, fail, rebuilt

    def scrub_once(self) -> list[str]:
        """K1b batched scrub: verify every block; queue bad ones for the next heartbeat
        and try to recover them (reference run_background_scrubber, chunkserver.rs:642-718)."""
        if self.agent is not None:
            return self.agent.scrub_once()
        bad = self.store.scrub()
        if bad:
            with self._lists_lock:
                self.pending_bad_blocks.extend(b for b in bad if b not in self.pending_bad_blocks)
            for b in bad:
                self._bg.submit(self.recover_block, b)
        return bad
