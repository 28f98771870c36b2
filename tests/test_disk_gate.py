"""Node-wide disk admission gate (csrc/disk_gate.h): at most `slots` durable writes in
flight per filesystem across processes, slots freed when their holder dies."""
import multiprocessing as mp
import os
import signal
import time

import pytest

from rust_hadoop_generated_by_llm_amd.native import lib as native

pytestmark = pytest.mark.skipif(not hasattr(native, "DiskGate"), reason="native extension without DiskGate")


def _slots(tmp_path):
    # the /dev/shm key is (st_dev, slots): stay clear of the chunk store's default (12)
    return 2 if "across" in str(tmp_path) else 5


def _hold(d, slots, q):
    g = native.DiskGate(d, slots)
    s = g.acquire()
    q.put(s.held)
    time.sleep(60)


def test_slots_are_exclusive_within_a_process(tmp_path):
    n = _slots(tmp_path)
    g = native.DiskGate(str(tmp_path), n)
    assert g.enabled and g.slots == n
    held = [g.try_acquire() for _ in range(n)]
    assert all(h is not None and h.held for h in held)
    assert g.try_acquire() is None
    held[0].release()
    again = g.try_acquire()
    assert again is not None
    again.release()
    for h in held[1:]:
        h.release()


def test_slots_are_shared_across_processes_and_freed_on_death(tmp_path):
    n = _slots(tmp_path)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_hold, args=(str(tmp_path), n, q)) for _ in range(n)]
    for p in procs:
        p.start()
    try:
        assert all(q.get(timeout=60) for _ in procs)
        g = native.DiskGate(str(tmp_path), n)
        assert g.try_acquire() is None  # every slot held by another process
        os.kill(procs[0].pid, signal.SIGKILL)
        procs[0].join(10)
        deadline = time.time() + 10
        s = None
        while s is None and time.time() < deadline:
            s = g.try_acquire()
            time.sleep(0.05)
        assert s is not None, "a dead holder's slot must come back"
        s.release()
    finally:
        for p in procs:
            if p.is_alive():
                p.kill()
            p.join(10)


def test_disabled_gate_never_blocks(tmp_path):
    g = native.DiskGate(str(tmp_path), 0)
    assert not g.enabled
    s = g.acquire()
    assert not s.held


def test_admission_is_fifo(tmp_path):
    """Waiters are admitted strictly in arrival order (ticket semaphore): no late arrival
    barges past a queued writer, which is what bounds the RF=3 write tail under load."""
    import threading

    g = native.DiskGate(str(tmp_path), 1)
    hold = [g.acquire()]  # node saturated
    order, threads = [], []

    def writer(i):
        s = g.acquire()
        order.append(i)
        time.sleep(0.01)
        s.release()

    for i in range(8):
        t = threading.Thread(target=writer, args=(i,))
        t.start()
        threads.append(t)
        time.sleep(0.05)  # arrival order = i
    for s in hold:
        s.release()
    for t in threads:
        t.join(10)
    assert order == list(range(8))
    assert g.waits >= 8
