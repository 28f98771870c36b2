"""Native WAL and the CPU (host-mode) chunk store: on-disk format, verification,
partial reads, cold tier (reference chunkserver.rs tests :1091+)."""
import os
import struct
import zlib

import pytest


def test_wal_append_replay_and_torn_tail(native, tmp_path):
    p = str(tmp_path / "w.log")
    w = native.Wal(p, True)
    assert w.replay() == []
    w.append([b"a", b"bb"])
    w.append([b"ccc"])
    del w
    with open(p, "ab") as f:
        f.write(b"\x10\x00\x00\x00garbage")  # torn frame
    w = native.Wal(p, True)
    assert w.replay() == [b"a", b"bb", b"ccc"]
    w.append([b"d"])
    assert native.Wal(p, True).replay() == [b"a", b"bb", b"ccc", b"d"]
    w.reset([b"x"])
    assert native.Wal(p, True).replay() == [b"x"]


def test_wal_corrupt_record_stops_replay(native, tmp_path):
    p = str(tmp_path / "w.log")
    w = native.Wal(p, False)
    w.append([b"one", b"two", b"three"])
    raw = bytearray(open(p, "rb").read())
    raw[8 + 3 + 8] ^= 0xFF  # first byte of "two"
    open(p, "wb").write(bytes(raw))
    assert native.Wal(p, False).replay() == [b"one"]


def test_atomic_write(native, tmp_path):
    p = str(tmp_path / "snap.json")
    native.atomic_write(p, b"{}", True)
    native.atomic_write(p, b'{"a":1}', True)
    assert open(p, "rb").read() == b'{"a":1}'


@pytest.fixture(params=[1, 0], ids=["journal", "per-file"])
def store(native, tmp_path, request):
    # journal=1: durable writes go through the group-committed block journal and the files
    # appear once materialized; journal=0: the per-file fdatasync path
    return native.ChunkStore(str(tmp_path / "hot"), str(tmp_path / "cold"), -1, 0, 0, 100, 1, 1, True,
                             journal=request.param)


def test_write_creates_data_and_meta(store, tmp_path):
    d = os.urandom(2000)
    ok, crc, err = store.write("blk", d, zlib.crc32(d))
    assert ok and crc == zlib.crc32(d)
    store.materialize()
    assert not store.journaled("blk")
    assert (tmp_path / "hot" / "blk").read_bytes() == d
    meta = (tmp_path / "hot" / "blk.meta").read_bytes()
    assert meta == b"".join(struct.pack(">I", zlib.crc32(d[i:i + 512])) for i in range(0, 2000, 512))
    assert store.verify_on_disk("blk") == ""


def test_checksum_mismatch_rejected(store):
    d = b"hello world"
    ok, crc, err = store.write("x", d, 12345)
    assert not ok and err == f"Checksum mismatch: expected 12345, actual {zlib.crc32(d)}"
    assert not store.exists("x")


def test_full_and_partial_reads(store):
    d = os.urandom(5000)
    store.write("b", d, 0)
    st, total, out, partial, bad, err = store.read("b", 0, 0)
    assert (st, total, out) == (0, 5000, d)
    st, total, out, partial, bad, err = store.read("b", 1000, 100)
    assert out == d[1000:1100] and not partial
    st, total, out, *_ = store.read("b", 4990, 0)
    assert out == d[4990:]
    st, total, out, partial, bad, err = store.read("b", 5000, 0)
    assert st == 2 and err == "Offset 5000 exceeds block size 5000"
    assert store.read("nope", 0, 0)[0] == 1


def test_corruption_detection(store, tmp_path):
    d = os.urandom(4096)
    store.write("c", d, 0)
    store.materialize()
    p = tmp_path / "hot" / "c"
    raw = bytearray(p.read_bytes())
    raw[0] ^= 0xFF
    p.write_bytes(bytes(raw))
    assert store.verify_on_disk("c") == "Checksum mismatch at chunk 0"
    st, *_r, err = store.read("c", 0, 0)
    assert st == 3 and "chunk 0" in err
    st, total, out, partial, bad, err = store.read("c", 0, 10)
    assert partial and bad == 0
    st, total, out, partial, bad, err = store.read("c", 1024, 10)
    assert not partial
    assert store.scrub() == ["c"]


def test_cold_tier_move_and_read(store, tmp_path):
    d = os.urandom(3000)
    store.write("k", d, 0)
    assert store.move_to_cold("k")
    assert not (tmp_path / "hot" / "k").exists() and (tmp_path / "cold" / "k").exists()
    assert (tmp_path / "cold" / "k.meta").exists()
    assert store.read("k", 0, 0)[2] == d
    assert store.read("k", 100, 50)[2] == d[100:150]
    assert store.verify_on_disk("k") == ""


def test_restart_rescans_directories(native, tmp_path):
    s = native.ChunkStore(str(tmp_path / "hot"), str(tmp_path / "cold"), -1, 0, 0, 100, 1, 1, True)
    d = os.urandom(777)
    s.write("r", d, 0)
    s.write("q", b"x" * 10, 0)
    s.move_to_cold("q")
    del s
    s2 = native.ChunkStore(str(tmp_path / "hot"), str(tmp_path / "cold"), -1, 0, 0, 100, 1, 1, True)
    assert sorted(s2.list_blocks()) == ["q", "r"]
    assert s2.read("r", 0, 0)[2] == d and s2.crc("r") == zlib.crc32(d)
    assert s2.read("q", 0, 0)[2] == b"x" * 10
    assert s2.stats()["blocks"] == 2


def test_remove(store, tmp_path):
    store.write("z", b"abc", 0)
    store.materialize()
    assert store.remove("z")
    assert not (tmp_path / "hot" / "z").exists() and not store.exists("z")


def test_aes_gcm_and_rsa_helpers(native):
    key, nonce = os.urandom(32), os.urandom(12)
    ct = native.aes256gcm_encrypt(key, nonce, b"secret data")
    assert native.aes256gcm_decrypt(key, nonce, ct) == b"secret data"
    bad = bytearray(ct)
    bad[0] ^= 1
    with pytest.raises(RuntimeError):
        native.aes256gcm_decrypt(key, nonce, bytes(bad))
