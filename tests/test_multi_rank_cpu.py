"""CPU analogues of the multi-GPU kit (tests/test_gpu_multi.py) at 8 ranks: the same
replication engine and pair protocol over the host-memory socket transport, so what the first
8-GPU node runs is rehearsed here on every CPU run.

* a full mesh of 8 ranks (56 directed pairs, K channels each) under crossing RF 3 fan-out
  traffic: every write lands 3 verified copies and every link's byte counters balance exactly
  against the traffic the test generated (sender's sent_to == receiver's recv_from);
* a rank killed while transfers to it are in flight: writes naming it finish with fewer
  replicas inside a bound (reference chunkserver.rs:777-829,1039-1077: a downstream failure is
  success with a smaller replicas_written), and no other pair is disturbed;
* RS(6,3) across 9 chunkserver processes: every shard on its own server, a degraded read with
  3 shards lost decodes, checked against the CPU codec.

Each assertion carries the per-link byte report, so a failure names the link.
"""
import os
import random
import threading
import time
import zlib
from concurrent.futures import ThreadPoolExecutor

import pytest

from rust_hadoop_generated_by_llm_amd.utils import fastpath as fp
from rust_hadoop_generated_by_llm_amd.utils.shm import ShmArena

from .test_replication import Node, put, read_block, write_via

pytestmark = pytest.mark.slow

WORLD = 8


def link_report(nodes) -> str:
    rows = []
    for nd in nodes:
        try:
            s = nd.eng.stats()
        except Exception as e:  # noqa: BLE001
            rows.append(f"rank {nd.rank}: stats unavailable ({e})")
            continue
        sent = {k.rsplit("_", 1)[1]: v for k, v in s.items() if k.startswith("link_sent_to_")}
        recv = {k.rsplit("_", 1)[1]: v for k, v in s.items() if k.startswith("link_recv_from_")}
        rows.append(f"rank {nd.rank}: pair_failures={s['pair_failures']} turn_timeouts={s['turn_timeouts']} "
                    f"sent_to={sent} recv_from={recv}")
    return "\n".join(rows)


@pytest.fixture()
def mesh(native, tmp_path):
    ns = "%x" % (zlib.crc32(str(tmp_path).encode()) & 0xFFFFFF)
    nodes = [Node(native, tmp_path, r, WORLD, ns) for r in range(WORLD)]
    for nd in nodes:
        nd.connect(nodes)
    for nd in nodes:
        assert nd.eng.wait_ready(20000) == WORLD - 1, link_report(nodes)
    yield nodes
    for nd in nodes:
        nd.down()


def test_eight_rank_full_mesh_crossing_rf3(mesh):
    nodes = mesh
    arena = ShmArena(size=128 << 20, slot=1 << 20)
    rng = random.Random(8)
    jobs = []
    for i in range(160):
        head, *rest = rng.sample(nodes, 3)
        jobs.append((head, rest, os.urandom(rng.choice([1, 4097, 300_000, 1 << 20])), f"mesh-{i}"))
    expect = {}  # (sender, receiver) -> bytes the fan-out must move over that link
    for head, rest, data, _ in jobs:
        for r in rest:
            expect[(head.rank, r.rank)] = expect.get((head.rank, r.rank), 0) + len(data)
    lock = threading.Lock()

    def one(job):
        head, rest, data, bid = job
        with lock:
            slot = put(arena, data)
        try:
            return write_via(head, arena, slot, data, bid, rest)
        finally:
            with lock:
                arena.release(slot)

    t0 = time.time()
    with ThreadPoolExecutor(10) as ex:
        results = list(ex.map(one, jobs))
    assert time.time() - t0 < 120, link_report(nodes)
    for (head, rest, data, bid), (st, replicas, msg) in zip(jobs, results):
        assert st == fp.OK and replicas == 3, (bid, st, replicas, msg, link_report(nodes))
        for nd in (head, *rest):
            assert read_block(nd, bid) == data, (bid, nd.rank)
    stats = {nd.rank: nd.eng.stats() for nd in nodes}
    for (a, b), n in expect.items():
        assert stats[a].get(f"link_sent_to_{b}") == n, (a, b, n, link_report(nodes))
        assert stats[b].get(f"link_recv_from_{a}") == n, (a, b, n, link_report(nodes))
    assert len(expect) >= 48, len(expect)  # the traffic really crossed (nearly) the whole mesh
    assert all(s["pair_failures"] == 0 for s in stats.values()), link_report(nodes)
    assert sum(nd.fp.stats()["fp_shm_forwards"] for nd in nodes) == 0
    arena.close()


def test_eight_ranks_a_rank_killed_mid_transfer(mesh):
    nodes = mesh
    victim = nodes[5]
    arena = ShmArena(size=96 << 20, slot=4 << 20)
    data = os.urandom(4 << 20)
    lock = threading.Lock()
    heads = [nd for nd in nodes if nd is not victim]

    def one(i):
        head = heads[i % len(heads)]
        other = heads[(i + 1) % len(heads)]
        with lock:
            slot = put(arena, data)
        try:
            t0 = time.time()
            st, replicas, msg = write_via(head, arena, slot, data, f"kill-{i}", [victim, other])
            return st, replicas, msg, time.time() - t0
        finally:
            with lock:
                arena.release(slot)

    with ThreadPoolExecutor(10) as ex:
        futs = [ex.submit(one, i) for i in range(20)]
        time.sleep(0.05)
        victim.down()  # engine and fast path gone while its transfers are in flight
        res = [f.result(timeout=120) for f in futs]
    for st, replicas, msg, secs in res:
        assert st == fp.OK and replicas in (2, 3), (st, replicas, msg, link_report(nodes))
        assert secs < 30, (secs, link_report(nodes))
    assert any(r[1] == 2 for r in res), "no write lost its replica: the kill came too late"
    # every surviving pair is untouched
    for a in heads:
        for b in heads:
            if a is not b:
                assert a.eng.pair_ok(b.rank), (a.rank, b.rank, link_report(nodes))
    # the survivors still replicate among themselves at full RF
    with lock:
        slot = put(arena, data)
    st, replicas, msg = write_via(nodes[0], arena, slot, data, "after", [nodes[1], nodes[7]])
    assert st == fp.OK and replicas == 3, msg
    arena.close()
    victim.up()  # the fixture's teardown stops every node


def test_rs63_across_nine_chunkservers():
    from rust_hadoop_generated_by_llm_amd.cluster.launcher import LocalCluster
    from rust_hadoop_generated_by_llm_amd.models import proto as pb
    from rust_hadoop_generated_by_llm_amd.ops import erasure
    from rust_hadoop_generated_by_llm_amd.utils.rpc import ChannelPool
    import urllib.request

    with LocalCluster(n_chunkservers=9, fsync=False, env={"DFS_DEBUG_ENDPOINTS": "1"}) as c:
        cl = c.client(local_chunkserver=c.cs_addrs[0])
        d = os.urandom((6 << 20) + 4321)
        cl.create_file_from_buffer_ec(d, "/ec63/f", 6, 3)
        blk = cl.get_file_info("/ec63/f").blocks[0]
        assert len(blk.locations) == 9 and len(set(blk.locations)) == 9, blk.locations
        want = erasure.encode(d, 6, 3, None)
        pool = ChannelPool(local=False)
        try:
            for i, loc in enumerate(blk.locations):
                r = pool.call(f"http://{loc}", "ChunkServerService", "ReadBlock",
                              pb.ReadBlockRequest(block_id=blk.block_id), timeout=60)
                assert r.data == want[i], i
        finally:
            pool.close()
        # lose three shards (two data, one parity) on their holders: the read decodes
        for i in (1, 4, 7):
            h = c.cs_http[c.cs_addrs.index(blk.locations[i])]
            urllib.request.urlopen(f"{h}/debug/remove?block={blk.block_id}", timeout=10).read()
        assert cl.get_file_content("/ec63/f") == d
        assert cl.read_file_range("/ec63/f", 999_999, 2 << 20) == d[999_999:999_999 + (2 << 20)]
        cl.close()
