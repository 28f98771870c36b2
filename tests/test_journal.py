"""Block journal of the chunk store (csrc/journal.{h,cpp}): group-committed durable writes,
crash replay with checksum verification, tombstones, segment reuse.

Two modes. The default since round 5 is the store of record (tests/test_journal_store.py):
records stay the blocks' durable home and the reference's `<id>` + `<id>.meta` files
(chunkserver.rs:192-209) are exported at a bounded rate. The tests here pin the round-4
mode (`DFS_JOURNAL_EXPORT=idle`: everything materialized once the writers pause, replay
writes the files out and retires the journal), kept as the A/B.
Host-mode store (CPU); the GPU tier runs the same protocol from HBM (test_gpu_kernels.py)."""
import os
import struct
import subprocess
import sys
import textwrap
import zlib
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]


@pytest.fixture(autouse=True)
def _idle_mode(monkeypatch):
    monkeypatch.setenv("DFS_JOURNAL_EXPORT", "idle")


def meta_of(d: bytes) -> bytes:
    return b"".join(struct.pack(">I", zlib.crc32(d[i:i + 512])) for i in range(0, len(d), 512))


def blob(i: int) -> bytes:
    return bytes([(i * 7 + j) & 0xFF for j in range(256)]) * (1 + i * 9)


def run_child(code: str, env: dict | None = None) -> subprocess.CompletedProcess:
    """Runs `code` in a fresh interpreter that ends with os._exit (no destructors: a crash)."""
    e = dict(os.environ, PYTHONPATH=str(ROOT), DFS_JOURNAL_EXPORT="idle")
    e.update(env or {})
    return subprocess.run([sys.executable, "-c", textwrap.dedent(code)], env=e, capture_output=True, text=True,
                          timeout=120)


def open_store(native, d, **kw):
    return native.ChunkStore(str(d / "hot"), str(d / "cold"), -1, 0, 0, 100, 1, 1, True, journal=1, **kw)


def test_journaled_until_materialized(native, tmp_path):
    s = open_store(native, tmp_path)
    s.debug_pause_materializer(True)
    data = {f"j{i}": blob(i) for i in range(12)}
    for k, v in data.items():
        assert s.write(k, v, zlib.crc32(v))[0]
    st = s.stats()
    assert st["journal"] and st["journal_records"] == 12 and st["materialize_pending"] == 12
    assert st["journal_sync_rounds"] >= 1 and st["journal_sync_rounds"] <= st["journal_commits"]
    # durable and readable from the journal before any file exists
    assert all(s.journaled(k) for k in data)
    assert not (tmp_path / "hot" / "j3").exists()
    for k, v in data.items():
        assert s.read(k, 0, 0)[2] == v
        assert s.read(k, 100, 300)[2] == v[100:400]
        assert s.meta(k) == meta_of(v)
        assert s.verify_on_disk(k) == ""
    assert s.scrub() == []
    s.debug_pause_materializer(False)
    s.materialize()
    st = s.stats()
    assert st["materialized_blocks"] == 12 and st["materialize_pending"] == 0
    for k, v in data.items():
        assert not s.journaled(k)
        assert (tmp_path / "hot" / k).read_bytes() == v
        assert (tmp_path / "hot" / f"{k}.meta").read_bytes() == meta_of(v)


def test_crash_replay_restores_acked_writes_and_deletes(native, tmp_path):
    r = run_child(f"""
        import os, zlib
        from rust_hadoop_generated_by_llm_amd import native
        s = native.lib.ChunkStore({str(tmp_path / 'hot')!r}, {str(tmp_path / 'cold')!r}, -1, 0, 0, 100, 1, 1, True,
                                  journal=1)
        s.debug_pause_materializer(True)
        for i in range(20):
            v = bytes([i]) * (3000 + 4096 * i)
            assert s.write(f"c{{i}}", v, zlib.crc32(v))[0]
        s.remove("c4")                                  # tombstone
        v = b"second version" * 300
        assert s.write("c5", v, zlib.crc32(v))[0]       # rewrite: the later record wins
        os._exit(0)
    """)
    assert r.returncode == 0, r.stderr
    assert not (tmp_path / "hot" / "c1").exists()
    s = open_store(native, tmp_path)
    st = s.stats()
    assert st["journal_replayed"] == 19 and st["journal_replay_skipped"] == 0
    assert st["journal_mode"] == "idle"
    assert st["journal_segs_free"] >= 1 and st["journal_records"] == 0
    assert not s.exists("c4") and not (tmp_path / "hot" / "c4").exists()
    assert s.read("c5", 0, 0)[2] == b"second version" * 300
    for i in range(20):
        if i in (4, 5):
            continue
        v = bytes([i]) * (3000 + 4096 * i)
        assert s.read(f"c{i}", 0, 0)[2] == v
        assert (tmp_path / "hot" / f"c{i}.meta").read_bytes() == meta_of(v)
    # replayed segments were retired: a second restart has nothing to replay
    del s
    assert open_store(native, tmp_path).stats()["journal_replayed"] == 0


def test_torn_record_is_dropped_on_replay(native, tmp_path):
    r = run_child(f"""
        import os, zlib
        from rust_hadoop_generated_by_llm_amd import native
        s = native.lib.ChunkStore({str(tmp_path / 'hot')!r}, "", -1, 0, 0, 100, 1, 1, True, journal=1)
        s.debug_pause_materializer(True)
        for i in range(3):
            v = bytes([65 + i]) * 10000
            assert s.write(f"t{{i}}", v, zlib.crc32(v))[0]
        os._exit(0)
    """)
    assert r.returncode == 0, r.stderr
    # the segment holding the records (spare segments are zero-filled)
    seg = next(p for p in (tmp_path / "hot" / ".journal").glob("seg-*.log")
               if bytes([67]) * 10000 in p.read_bytes()[: 1 << 20])
    raw = bytearray(seg.read_bytes()[: 1 << 20])
    # the last record's data: flip a byte as a torn write would leave it
    pos = raw.rfind(bytes([67]) * 10000)
    assert pos > 0
    raw[pos + 5000] ^= 0xFF
    with open(seg, "r+b") as f:
        f.write(raw)
    s = native.ChunkStore(str(tmp_path / "hot"), "", -1, 0, 0, 100, 1, 1, True, journal=1)
    st = s.stats()
    assert st["journal_replayed"] == 2 and st["journal_replay_skipped"] == 1
    assert s.read("t0", 0, 0)[2] == b"A" * 10000 and s.read("t1", 0, 0)[2] == b"B" * 10000
    assert not s.exists("t2")


def test_corrupt_journal_copy_is_detected(native, tmp_path):
    s = open_store(native, tmp_path)
    s.debug_pause_materializer(True)
    v = os.urandom(5000)
    assert s.write("bad", v, zlib.crc32(v))[0]
    assert s.debug_corrupt("bad", 1030)
    st, total, out, partial, bad, err = s.read("bad", 0, 0)
    assert st == 3 and bad == 2
    assert s.read("bad", 0, 100)[3] is False  # untouched slice reads fine
    assert s.read("bad", 1024, 100)[3] is True
    assert s.verify_on_disk("bad") == "Checksum mismatch at chunk 2"
    assert s.scrub() == ["bad"]


def test_small_journal_recycles_segments_under_pressure(native, tmp_path, monkeypatch):
    # 8 MiB segments of two 4 MiB parts, 3 of them: 30 x 1 MiB writes only fit if the
    # materializer retires segments while the writers run (backpressure, then reuse with a
    # new sequence number)
    monkeypatch.setenv("DFS_JOURNAL_SEG_MB", "8")
    monkeypatch.setenv("DFS_JOURNAL_PARTS", "2")
    monkeypatch.setenv("DFS_JOURNAL_SEGS", "3")
    monkeypatch.setenv("DFS_JOURNAL_BYPASS", "0")  # writers wait for recycled segments
    s = open_store(native, tmp_path)
    vals = {}
    for i in range(30):
        v = os.urandom((1 << 20) - 17 * i)
        vals[f"p{i}"] = v
        assert s.write(f"p{i}", v, zlib.crc32(v))[0]
    s.materialize()
    st = s.stats()
    assert 2 <= st["journal_segs"] <= 3 and st["journal_segs_retired"] >= 3
    assert st["materialized_blocks"] == 30
    for k, v in vals.items():
        assert s.read(k, 0, 0)[2] == v and (tmp_path / "hot" / k).read_bytes() == v
    del s
    s = open_store(native, tmp_path)
    assert s.stats()["journal_replayed"] == 0 and sorted(s.list_blocks()) == sorted(vals)


def test_concurrent_writers_recycle_a_small_journal(native, tmp_path, monkeypatch):
    """Many writers at once on a journal of 3 small segments: whenever the active segment
    fills, several writers wait for a free one at the same time. Exactly one activation may
    win (the others append to it), or a segment left unsealed behind a newer one would block
    retirement for good and every writer would end on 'journal full'."""
    from concurrent.futures import ThreadPoolExecutor

    monkeypatch.setenv("DFS_JOURNAL_SEG_MB", "8")
    monkeypatch.setenv("DFS_JOURNAL_PARTS", "2")
    monkeypatch.setenv("DFS_JOURNAL_SEGS", "3")
    monkeypatch.setenv("DFS_JOURNAL_SPARES", "2")
    monkeypatch.setenv("DFS_JOURNAL_FULL_TIMEOUT_S", "20")
    monkeypatch.setenv("DFS_JOURNAL_BYPASS", "0")
    s = open_store(native, tmp_path)
    vals = {f"c{i}": os.urandom((1 << 20) - 4096 * (i % 7)) for i in range(120)}
    with ThreadPoolExecutor(12) as ex:
        res = list(ex.map(lambda kv: s.write(kv[0], kv[1], zlib.crc32(kv[1])), vals.items()))
    assert all(r[0] for r in res), next(r for r in res if not r[0])
    s.materialize()
    st = s.stats()
    assert st["journal_segs"] <= 3 and st["journal_segs_retired"] >= 15 and st["materialized_blocks"] == 120
    for k, v in vals.items():
        assert s.read(k, 0, 0)[2] == v


def test_writes_past_the_materialize_mark_take_the_per_file_path(native, tmp_path):
    """Once the journal is at the materializer's mark, every journaled block will be written a
    second time; new durable writes then go straight to `<id>` + `<id>.meta` (written once)
    until the materializer has caught up."""
    import subprocess as sp

    code = f"""
import os, zlib
from rust_hadoop_generated_by_llm_amd import native
s = native.lib.ChunkStore({str(tmp_path / 'hot')!r}, "", -1, 0, 0, 100, 1, 1, True, journal=1)
s.debug_pause_materializer(True)
vals = {{f"b{{i}}": os.urandom((1 << 20) - 512 * i) for i in range(24)}}
for k, v in vals.items():
    assert s.write(k, v, zlib.crc32(v))[0]
st = s.stats()
assert st["journal_bypassed"] > 0, st
assert st["journal_records"] + st["journal_bypassed"] == 24, st
# bypassed writes are files already; journaled ones are not until materialized
on_disk = [k for k in vals if os.path.exists({str(tmp_path / 'hot')!r} + "/" + k)]
assert len(on_disk) == st["journal_bypassed"], (on_disk, st)
for k, v in vals.items():
    assert s.read(k, 0, 0)[2] == v
s.debug_pause_materializer(False)
s.materialize()
assert all(os.path.exists({str(tmp_path / 'hot')!r} + "/" + k) for k in vals)
print("ok")
"""
    env = dict(os.environ, PYTHONPATH=str(ROOT), DFS_JOURNAL_SEG_MB="8", DFS_JOURNAL_PARTS="2", DFS_JOURNAL_SEGS="4")
    r = sp.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "ok" in r.stdout, r.stderr[-2000:]


def test_concurrent_writers_share_group_commits(native, tmp_path, monkeypatch):
    from concurrent.futures import ThreadPoolExecutor

    # a slow flush (as on a real device) lets the writers that arrive meanwhile join the round
    monkeypatch.setenv("DFS_JOURNAL_SYNC_DELAY_US", "3000")
    s = open_store(native, tmp_path)
    vals = {f"g{i}": os.urandom(200_000 + i) for i in range(64)}
    with ThreadPoolExecutor(16) as ex:
        res = list(ex.map(lambda kv: s.write(kv[0], kv[1], zlib.crc32(kv[1]))[0], vals.items()))
    assert all(res)
    st = s.stats()
    assert st["journal_commits"] == 64
    assert st["journal_sync_rounds"] < 64  # flushes were shared between writers
    for k, v in vals.items():
        assert s.read(k, 0, 0)[2] == v


def test_torn_data_file_without_meta_is_quarantined(native, tmp_path):
    hot = tmp_path / "hot"
    hot.mkdir()
    (hot / "torn").write_bytes(b"x" * 5000)  # a data file whose .meta never made it
    (hot / "short").write_bytes(b"y" * 5000)
    (hot / "short.meta").write_bytes(b"\0" * 4)  # wrong length for 5000 bytes
    d = b"z" * 700
    (hot / "good").write_bytes(d)
    (hot / "good.meta").write_bytes(meta_of(d))
    s = native.ChunkStore(str(hot), "", -1, 0, 0, 100, 1, 1, True, journal=0)
    assert s.list_blocks() == ["good"]
    assert (hot / ".quarantine-torn").exists() and (hot / ".quarantine-short.meta").exists()
    assert s.read("good", 0, 0)[2] == d


@pytest.mark.parametrize("journal", [0, 1])
def test_journal_flag_off_keeps_per_file_path(native, tmp_path, journal):
    s = open_store(native, tmp_path) if journal else native.ChunkStore(
        str(tmp_path / "hot"), "", -1, 0, 0, 100, 1, 1, True, journal=0)
    v = os.urandom(3000)
    assert s.write("f", v, zlib.crc32(v))[0]
    assert s.stats()["journal"] == bool(journal)
    assert (tmp_path / "hot" / "f").exists() == (not journal) or s.journaled("f") == bool(journal)
