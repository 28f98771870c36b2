"""Crash-restart of a GPU-tier ChunkServer with real fsync (nvme-sync durability on an HBM
store, MI355X): blocks acknowledged before a SIGKILL are read back after the restart
(promoted disk -> HBM with their .meta image, every read checked by the fused range-verify
CRC kernel), and a block whose file was damaged while the process was down is refused,
not served.
CPU twin of the restart/rescan rules: tests/test_wal_store_cpu.py::test_restart_rescans_directories."""
import json
import os
import time
import urllib.request

import pytest

from rust_hadoop_generated_by_llm_amd.client.client import DfsError
from rust_hadoop_generated_by_llm_amd.cluster.launcher import LocalCluster



def stats(cl):
    return json.load(urllib.request.urlopen(f"{cl.cs_http[0]}/stats"))


def block_file(cl, block_id):
    for root, _, files in os.walk(cl.base / "cs0"):
        if block_id in files:
            return os.path.join(root, block_id)
    raise AssertionError(f"no file for block {block_id}")


def crash_restart(cl, gpu):
    c = cl.client(initial_backoff_ms=100, max_retries=20)
    files = {f"/rs/f{i}": os.urandom((1 << 20) * (1 + i % 3) + 4097 * i) for i in range(8)}
    for p, d in files.items():
        c.create_file_from_buffer(d, p)
    if gpu:
        st = stats(cl)
        assert st["hbm_resident_blocks"] >= len(files) and st["gpu_kernel_launches"] > 0
    c.close()

    # SIGKILL: nothing gets a chance to flush; acknowledged writes must already be durable
    cl.restart("cs0")
    cl.wait_registered()
    if gpu:
        assert stats(cl)["hbm_resident_blocks"] == 0  # HBM is volatile: everything comes back from disk
    c = cl.client(initial_backoff_ms=100, max_retries=20)
    for p, d in files.items():
        assert c.get_file_content(p) == d, p
    assert c.read_file_range("/rs/f5", 777_777, 100_000) == files["/rs/f5"][777_777:877_777]
    st = stats(cl)
    assert st["crc_mismatches"] == 0 and (st["promotions"] >= 1 or not gpu)
    victim = c.get_file_info("/rs/f2").blocks[0].block_id
    c.close()

    # damage one block's file while the server is down: the verified load must refuse it
    def flip():
        path = block_file(cl, victim)
        with open(path, "r+b") as f:
            f.seek(123_456)
            b = f.read(1)
            f.seek(123_456)
            f.write(bytes([b[0] ^ 0x5A]))

    cl.restart("cs0", before_start=flip)
    cl.wait_registered()
    c = cl.client(initial_backoff_ms=50, max_retries=2)
    with pytest.raises(DfsError):
        c.get_file_content("/rs/f2")  # RF=1: no healthy replica to fall back to
    assert stats(cl)["crc_mismatches"] >= 1
    for p in ("/rs/f0", "/rs/f7"):  # the others are untouched
        assert c.get_file_content(p) == files[p]
    c.close()


@pytest.mark.gpu
def test_gpu_chunkserver_crash_restart_fsync():
    from rust_hadoop_generated_by_llm_amd import native

    if native.gpu_count() < 1:
        pytest.fail("GPU test selected but no HIP device is visible")
    with LocalCluster(gpus=[0], fsync=True, durability="nvme-sync", hbm_capacity="2G") as cl:
        crash_restart(cl, gpu=True)


@pytest.mark.slow
def test_host_chunkserver_crash_restart_fsync():
    with LocalCluster(n_chunkservers=1, fsync=True, durability="nvme-sync") as cl:
        crash_restart(cl, gpu=False)


@pytest.mark.gpu
def test_gpu_hbm_ack_crash_semantics():
    """hbm-ack acknowledges once the block is checksummed in HBM and spills to NVMe behind
    the ack. Pinned here: blocks whose spill finished survive a SIGKILL;
    blocks acked but not yet spilled are gone after it — reported missing, never served
    torn — and the spill leaves no partial file under a block's real name."""
    from rust_hadoop_generated_by_llm_amd import native

    if native.gpu_count() < 1:
        pytest.fail("GPU test selected but no HIP device is visible")
    with LocalCluster(gpus=[0], fsync=True, durability="hbm-ack", hbm_capacity="2G",
                      env={"DFS_DEBUG_ENDPOINTS": "1"}) as cl:
        c = cl.client(initial_backoff_ms=50, max_retries=2)
        spilled = {f"/ack/s{i}": os.urandom((1 << 20) + 3 * i) for i in range(4)}
        for p, d in spilled.items():
            c.create_file_from_buffer(d, p)
        deadline = time.time() + 30
        while stats(cl)["dirty_blocks"] > 0:  # spill drained: these are durable now
            assert time.time() < deadline, "spill never drained"
            time.sleep(0.05)
        urllib.request.urlopen(f"{cl.cs_http[0]}/debug/pause_spill?on=1").read()
        held = {f"/ack/h{i}": os.urandom((1 << 20) + 5 * i) for i in range(4)}
        for p, d in held.items():
            c.create_file_from_buffer(d, p)  # acked from HBM
            assert c.get_file_content(p) == d
        assert stats(cl)["dirty_blocks"] >= len(held)
        held_ids = [c.get_file_info(p).blocks[0].block_id for p in held]
        c.close()

        cl.restart("cs0")
        cl.wait_registered()
        names = {n for _, _, fs in os.walk(cl.base / "cs0") for n in fs}
        assert not any(n.endswith(".tmp") for n in names)
        assert not any(b in names for b in held_ids)
        c = cl.client(initial_backoff_ms=50, max_retries=2)
        for p, d in spilled.items():
            assert c.get_file_content(p) == d
        for p in held:
            with pytest.raises(DfsError):
                c.get_file_content(p)
        assert stats(cl)["crc_mismatches"] == 0
        c.close()
