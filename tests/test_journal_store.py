"""The block journal as the store of record (round 5, `DFS_JOURNAL_EXPORT=store|never`).

Records stay the blocks' durable home: segments grow on demand while the volume keeps a
reserve, replay indexes records in place (no files written), a clean stop marks segments
sealed so the next start trusts them, deletes commit a tombstone, per-file rewrites commit a
supersede marker, compaction relocates live records out of the oldest segment, and the
exporter writes the reference's `<id>` + `<id>.meta` (chunkserver.rs:182-209: raw bytes, and
big-endian CRC-32/IEEE per 512 bytes) at a bounded rate, byte-checked against zlib here.
Host-mode store (CPU); the GPU tier covers the K1b scrub of journal-resident copies.
"""
import json
import os
import struct
import subprocess
import sys
import textwrap
import zlib
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
SMALL = {"DFS_JOURNAL_SEG_MB": "8", "DFS_JOURNAL_PARTS": "2", "DFS_JOURNAL_SPARES": "2"}


def meta_of(d: bytes) -> bytes:
    return b"".join(struct.pack(">I", zlib.crc32(d[i:i + 512])) for i in range(0, len(d), 512))


def run_child(code: str, env: dict) -> subprocess.CompletedProcess:
    """`code` in a fresh interpreter that ends with os._exit (no destructors: a crash)."""
    e = dict(os.environ, PYTHONPATH=str(ROOT))
    e.update(env)
    return subprocess.run([sys.executable, "-c", textwrap.dedent(code)], env=e, capture_output=True, text=True,
                          timeout=180)


def open_store(native, d):
    return native.ChunkStore(str(d / "hot"), str(d / "cold"), -1, 0, 0, 100, 1, 1, True, journal=1)


@pytest.fixture
def never(monkeypatch):
    """Store of record with the exporter off: the journal is the only durable copy."""
    monkeypatch.setenv("DFS_JOURNAL_EXPORT", "never")
    for k, v in SMALL.items():
        monkeypatch.setenv(k, v)


def data_files(d: Path) -> list:
    hot = d / "hot"
    return sorted(p.name for p in hot.iterdir() if not p.name.startswith(".")) if hot.exists() else []


def test_journal_is_the_only_copy_across_a_crash(native, tmp_path, never):
    r = run_child(f"""
        import os, zlib
        from rust_hadoop_generated_by_llm_amd import native
        s = native.lib.ChunkStore({str(tmp_path / 'hot')!r}, {str(tmp_path / 'cold')!r}, -1, 0, 0, 100, 1, 1, True,
                                  journal=1)
        for i in range(40):
            v = bytes([i]) * (300_000 + 40_960 * i)
            assert s.write(f"c{{i}}", v, zlib.crc32(v))[0]
        assert s.remove("c4")                           # tombstone, committed before it returns
        v = b"second version" * 300
        assert s.write("c5", v, zlib.crc32(v))[0]       # rewrite: the later record wins
        st = s.stats()
        assert st["journal_mode"] == "store-noexport" and st["journal_segs"] > 4, st
        os._exit(0)
    """, dict(SMALL, DFS_JOURNAL_EXPORT="never"))
    assert r.returncode == 0, r.stderr
    assert data_files(tmp_path) == []  # no <id> files: the segments are the only copy
    s = open_store(native, tmp_path)
    st = s.stats()
    # crashed: the records of segments not yet marked sealed (at least the active one) were
    # re-verified against their checksums; the marked ones were trusted
    assert st["journal_replayed"] == 39 and st["journal_replay_skipped"] == 0
    assert 1 <= st["journal_replay_verified"] <= 39
    assert data_files(tmp_path) == []
    assert not s.exists("c4")
    assert s.read("c5", 0, 0)[2] == b"second version" * 300
    for i in range(40):
        if i in (4, 5):
            continue
        v = bytes([i]) * (300_000 + 40_960 * i)
        assert s.journaled(f"c{i}")
        assert s.read(f"c{i}", 0, 0)[2] == v
        assert s.read(f"c{i}", 1000, 5000)[2] == v[1000:6000]
        assert s.meta(f"c{i}") == meta_of(v)
        assert s.verify_on_disk(f"c{i}") == ""
    assert s.scrub() == []
    # a clean stop marks the segments sealed: the next start trusts the records
    del s
    s = open_store(native, tmp_path)
    st = s.stats()
    assert st["journal_replayed"] == 39 and st["journal_replay_verified"] == 0, st
    assert sorted(s.list_blocks()) == sorted(f"c{i}" for i in range(40) if i != 4)


def test_journal_grows_on_demand(native, tmp_path, never, monkeypatch):
    monkeypatch.setenv("DFS_JOURNAL_SPARES", "1")
    s = open_store(native, tmp_path)
    vals = {f"g{i}": os.urandom((1 << 20) - 333 * i) for i in range(48)}
    for k, v in vals.items():
        assert s.write(k, v, zlib.crc32(v))[0]
    st = s.stats()
    # 8 MiB segments hold ~7 blocks: the journal grew well past one spare, with no bypass
    assert st["journal_segs"] >= 7 and st["journal_bypassed"] == 0 and st["journal_full_waits"] == 0
    assert st["journal_live_records"] == 48 and st["materialized_blocks"] == 0
    assert data_files(tmp_path) == []
    for k, v in vals.items():
        assert s.read(k, 0, 0)[2] == v


def test_export_writes_reference_format_files(native, tmp_path, monkeypatch):
    for k, v in SMALL.items():
        monkeypatch.setenv(k, v)
    monkeypatch.setenv("DFS_JOURNAL_EXPORT", "store")
    monkeypatch.setenv("DFS_EXPORT_HEADROOM_MB", "1")
    s = open_store(native, tmp_path)
    s.debug_pause_materializer(True)
    vals = {f"e{i}": os.urandom(5000 + 70_001 * i) for i in range(24)}
    for k, v in vals.items():
        assert s.write(k, v, zlib.crc32(v))[0]
    assert data_files(tmp_path) == []
    s.debug_pause_materializer(False)
    s.materialize()  # on request: everything, whatever the token bucket
    st = s.stats()
    assert st["materialized_blocks"] == 24 and st["journal_live_records"] == 0, st
    assert st["journal_segs_retired"] >= 1  # exported records are released, their segments recycle
    for k, v in vals.items():
        assert not s.journaled(k)
        # F3: <id> raw bytes, <id>.meta big-endian CRC-32/IEEE per 512 B slice (zlib)
        assert (tmp_path / "hot" / k).read_bytes() == v
        assert (tmp_path / "hot" / f"{k}.meta").read_bytes() == meta_of(v)
        assert s.read(k, 0, 0)[2] == v
    assert not [p for p in (tmp_path / "hot").iterdir() if p.name.endswith(".tmp")]
    del s
    s = open_store(native, tmp_path)  # the files are the home now
    assert s.stats()["journal_replayed"] == 0 and sorted(s.list_blocks()) == sorted(vals)


def test_exporter_runs_at_its_rate_without_a_pause(native, tmp_path, monkeypatch):
    """No idle gate: the exporter drains while writers keep writing, bounded by its bucket."""
    import time

    for k, v in SMALL.items():
        monkeypatch.setenv(k, v)
    monkeypatch.setenv("DFS_JOURNAL_EXPORT", "store")
    monkeypatch.setenv("DFS_EXPORT_HEADROOM_MB", "1")
    monkeypatch.setenv("DFS_EXPORT_MBPS", "40")
    s = open_store(native, tmp_path)
    t0 = time.time()
    n = 0
    while time.time() - t0 < 1.5:  # writers never pause for 500 ms
        v = os.urandom(256 << 10)
        assert s.write(f"w{n}", v, zlib.crc32(v))[0]
        n += 1
        time.sleep(0.002)
    st = s.stats()
    exported = st["materialized_bytes"]
    assert exported > 0, st
    assert exported <= (40e6 * 2.0 + (64 << 20)), st  # bucket: rate x time + one burst


def test_overwrites_reclaim_the_journal_while_the_exporter_runs(native, tmp_path, monkeypatch):
    """Sustained overwrites of a few keys with the exporter busy and the journal capped at
    6 segments: the dead records of overwritten blocks, and the records of blocks already
    exported, are reclaimed while the writers keep writing (exports and compaction share the
    token bucket, compaction first), so no writer ever finds the journal full."""
    import time

    for k, v in SMALL.items():
        monkeypatch.setenv(k, v)
    monkeypatch.setenv("DFS_JOURNAL_EXPORT", "store")
    monkeypatch.setenv("DFS_EXPORT_HEADROOM_MB", "1")
    monkeypatch.setenv("DFS_EXPORT_MBPS", "40")
    monkeypatch.setenv("DFS_JOURNAL_SEGS", "6")  # 6 x 8 MiB: no growth past 48 MiB
    monkeypatch.setenv("DFS_JOURNAL_FULL_TIMEOUT_S", "10")
    s = open_store(native, tmp_path)
    keep = os.urandom(100_000)
    assert s.write("keep", keep, zlib.crc32(keep))[0]
    t0 = time.time()
    n = 0
    while time.time() - t0 < 2.0:  # ~4x the journal's capacity, well above the export rate
        v = os.urandom(256 << 10)
        ok, _crc, err = s.write(f"k{n % 16}", v, zlib.crc32(v))[:3]
        assert ok, (n, err, s.stats())
        n += 1
    st = s.stats()
    assert n * (256 << 10) > 2 * 6 * (8 << 20), (n, st)  # the journal wrapped at least twice
    assert st["journal_full_waits"] == 0, st
    assert st["materialized_blocks"] > 0, st  # the exporter kept running beside compaction
    assert s.read("keep", 0, 0)[2] == keep


def test_busy_writers_still_get_segments_compacted(native, tmp_path, monkeypatch):
    """Writers that never pause, with a long-lived record landing in every segment: segments
    only come back through compaction (no headroom for exports here). The exporter's slow
    busy-writer rate must not starve compaction: with it gating compaction too, config 5's
    multipart phase found the journal full and timed out (profiles/r6/config5.json, r6 first
    run: 6,371 writer waits, 10 uploads failed)."""
    import time

    for k, v in SMALL.items():
        monkeypatch.setenv(k, v)
    monkeypatch.setenv("DFS_JOURNAL_EXPORT", "store")
    monkeypatch.setenv("DFS_EXPORT_HEADROOM_MB", str(1 << 30))  # never headroom: no exports
    monkeypatch.setenv("DFS_EXPORT_BUSY_MBPS", "1")
    monkeypatch.setenv("DFS_JOURNAL_SEGS", "6")
    monkeypatch.setenv("DFS_JOURNAL_FULL_TIMEOUT_S", "10")
    s = open_store(native, tmp_path)
    kept = {}
    t0 = time.time()
    n = 0
    # until the journal wrapped twice (a slow host just takes longer); ~100 MB/s at most, and
    # never idle for 50 ms
    while n * (256 << 10) <= 2 * 6 * (8 << 20) and time.time() - t0 < 30:
        v = os.urandom(256 << 10)
        key = f"live{n}" if n % 16 == 0 and len(kept) < 40 else f"k{n % 8}"
        ok, _crc, err = s.write(key, v, zlib.crc32(v))[:3]
        assert ok, (n, err, s.stats())
        if key.startswith("live"):
            kept[key] = v
        n += 1
        time.sleep(0.002)
    st = s.stats()
    assert n * (256 << 10) > 2 * 6 * (8 << 20), (n, st)  # wrapped the journal twice
    assert st["journal_full_waits"] == 0, st
    assert st["relocated_blocks"] > 0, st
    for key, v in list(kept.items())[:8]:
        assert s.read(key, 0, 0)[2] == v


def test_a_mostly_live_oldest_segment_does_not_pin_the_journal(native, tmp_path, monkeypatch):
    """The oldest segment is full of blocks nobody overwrites (and no headroom to export
    them); everything written after it dies quickly. Segments retire oldest first, so unless
    that live segment is relocated, every dead segment behind it stays in use and the writers
    find the journal full (config 5's multipart phase after the PUT phases: 80 GB of journal
    for 2.35 GB live, r6c5)."""
    import time

    for k, v in SMALL.items():
        monkeypatch.setenv(k, v)
    monkeypatch.setenv("DFS_JOURNAL_EXPORT", "store")
    monkeypatch.setenv("DFS_EXPORT_HEADROOM_MB", str(1 << 30))  # never headroom: no exports
    monkeypatch.setenv("DFS_JOURNAL_SEGS", "6")
    monkeypatch.setenv("DFS_JOURNAL_FULL_TIMEOUT_S", "10")
    s = open_store(native, tmp_path)
    old = {f"old{i}": os.urandom(256 << 10) for i in range(28)}  # ~7 MiB: most of segment 1
    for k, v in old.items():
        assert s.write(k, v, zlib.crc32(v))[0]
    t0 = time.time()
    n = 0
    while n * (256 << 10) <= 2 * 6 * (8 << 20) and time.time() - t0 < 30:
        v = os.urandom(256 << 10)
        ok, _crc, err = s.write(f"k{n % 8}", v, zlib.crc32(v))[:3]
        assert ok, (n, err, s.stats())
        n += 1
        time.sleep(0.002)
    st = s.stats()
    assert n * (256 << 10) > 2 * 6 * (8 << 20), (n, st)  # wrapped the journal twice
    assert st["journal_full_waits"] == 0, st
    assert st["relocated_blocks"] >= len(old), st
    for k, v in old.items():
        assert s.read(k, 0, 0)[2] == v


def test_supersede_marker_keeps_a_per_file_rewrite(native, tmp_path, never):
    """A rewrite too large for a segment part goes to its own files; the committed supersede
    marker stops replay from bringing back the older journal version."""
    r = run_child(f"""
        import os, zlib
        from rust_hadoop_generated_by_llm_amd import native
        s = native.lib.ChunkStore({str(tmp_path / 'hot')!r}, "", -1, 0, 0, 100, 1, 1, True, journal=1)
        v1 = b"a" * 10000
        assert s.write("x", v1, zlib.crc32(v1))[0] and s.journaled("x")
        v2 = b"b" * (5 << 20)                            # > a 4 MiB part: per-file
        assert s.write("x", v2, zlib.crc32(v2))[0] and not s.journaled("x")
        assert s.stats()["journal_supersedes"] == 1
        os._exit(0)
    """, dict(SMALL, DFS_JOURNAL_EXPORT="never"))
    assert r.returncode == 0, r.stderr
    s = native.ChunkStore(str(tmp_path / "hot"), "", -1, 0, 0, 100, 1, 1, True, journal=1)
    assert s.read("x", 0, 0)[2] == b"b" * (5 << 20)
    assert not s.journaled("x")


def test_compaction_relocates_live_records(native, tmp_path, never):
    # the writes, deletes and the compaction run in a process that then crashes: relocated
    # copies (which keep their LSN) and the tombstones must replay consistently
    r = run_child(f"""
        import os, zlib, json
        from rust_hadoop_generated_by_llm_amd import native
        s = native.lib.ChunkStore({str(tmp_path / 'hot')!r}, {str(tmp_path / 'cold')!r}, -1, 0, 0, 100, 1, 1, True,
                                  journal=1)
        keep = []
        for i in range(40):
            v = bytes([i + 1]) * ((900 << 10) + i)
            assert s.write(f"k{{i}}", v, zlib.crc32(v))[0]
        for i in range(40):
            if i % 4:
                assert s.remove(f"k{{i}}")
            else:
                keep.append(f"k{{i}}")
        st0 = s.stats()
        moved = s.compact(0.5)
        st = s.stats()
        # the background compactor may already have relocated some (the deletes trigger it):
        # the explicit pass moves what is left
        assert moved >= 0 and st["relocated_blocks"] >= st0["relocated_blocks"] + moved, (st0, st)
        assert st["relocated_blocks"] > 0, st
        assert st["journal_segs_retired"] > st0["journal_segs_retired"], (st0, st)
        assert st["journal_live_records"] == len(keep), st
        for k in keep:
            i = int(k[1:])
            assert s.read(k, 0, 0)[2] == bytes([i + 1]) * ((900 << 10) + i)
        print(json.dumps(sorted(keep)), flush=True)
        os._exit(0)
    """, dict(SMALL, DFS_JOURNAL_EXPORT="never"))
    assert r.returncode == 0, r.stderr
    keep = json.loads(r.stdout.strip())
    s = open_store(native, tmp_path)
    assert sorted(s.list_blocks()) == keep
    for k in keep:
        i = int(k[1:])
        assert s.read(k, 0, 0)[2] == bytes([i + 1]) * ((900 << 10) + i)


def test_no_stale_records_after_clean_restart(native, tmp_path):
    """sequence numbers restarted at 1 after a clean stop, so a reused segment's old
    records (not zero-filled) could match again and replay past the real tail. Now retired
    headers keep their sequence number and every run's numbers are larger."""
    env = dict(SMALL, DFS_JOURNAL_EXPORT="idle", DFS_JOURNAL_ZERO_FILL="0", DFS_JOURNAL_SEGS="3")
    r = run_child(f"""
        import os, zlib
        from rust_hadoop_generated_by_llm_amd import native
        s = native.lib.ChunkStore({str(tmp_path / 'hot')!r}, "", -1, 0, 0, 100, 1, 1, True, journal=1)
        for i in range(12):
            v = bytes([i + 1]) * 300_000
            assert s.write(f"old{{i}}", v, zlib.crc32(v))[0]
        s.materialize()
        for i in range(12):
            assert s.remove(f"old{{i}}")
        s.materialize()
        del s                                            # clean stop: every segment retired
        s = native.lib.ChunkStore({str(tmp_path / 'hot')!r}, "", -1, 0, 0, 100, 1, 1, True, journal=1)
        s.debug_pause_materializer(True)
        v = b"new" * 1000
        assert s.write("fresh", v, zlib.crc32(v))[0]     # reuses a segment holding old records
        os._exit(0)
    """, env)
    assert r.returncode == 0, r.stderr
    for k, v in env.items():
        os.environ[k] = v
    try:
        s = native.ChunkStore(str(tmp_path / "hot"), "", -1, 0, 0, 100, 1, 1, True, journal=1)
        st = s.stats()
        assert st["journal_replayed"] == 1, st
        assert s.list_blocks() == ["fresh"]
    finally:
        for k in env:
            os.environ.pop(k, None)


def test_delete_commits_its_tombstone(native, tmp_path, never):
    s = open_store(native, tmp_path)
    v = os.urandom(10000)
    assert s.write("d", v, zlib.crc32(v))[0]
    c0 = s.stats()["journal_commits"]
    assert s.remove("d")
    st = s.stats()
    assert st["journal_tombstones"] == 1 and st["journal_commits"] == c0 + 1
