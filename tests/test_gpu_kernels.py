"""GPU numerics: every CDNA4 kernel against the CPU reference (zlib CRC, table RS).
Marked gpu; the HIP path must be the one exercised (no silent CPU fallback)."""
import os
import struct
import zlib

import pytest

pytestmark = pytest.mark.gpu

SIZES = [1, 7, 511, 512, 513, 4096, 16384, 16385, 65536 + 3, (1 << 20), (1 << 20) + 777, 3 * (1 << 20) + 1,
         (16 << 20) + 512 * 3 + 5]


@pytest.fixture(scope="module")
def gstore(native, tmp_path_factory):
    from rust_hadoop_generated_by_llm_amd import native as n

    assert n.gpu_count() > 0, "GPU tests need a HIP device"
    s = native.ChunkStore(str(tmp_path_factory.mktemp("gstore")), "", 0, 1 << 30, 0, 100, 4, 2, False)
    assert s.gpu
    yield s
    del s


def ref_meta(d: bytes) -> bytes:
    return b"".join(struct.pack(">I", zlib.crc32(d[i:i + 512])) for i in range(0, len(d), 512))


@pytest.mark.parametrize("n", SIZES)
def test_gpu_crc_matches_zlib(gstore, n):
    d = os.urandom(n)
    crc, meta = gstore.gpu_crc(d)
    assert crc == zlib.crc32(d)
    assert meta == ref_meta(d)


@pytest.mark.parametrize("n", [511, 4096, (1 << 20) + 13, 8 << 20])
def test_gpu_crc_matrix_core_kernel_below_the_dispatch_threshold(gstore, native, n):
    """Blocks under 16 MiB run the LDS-table kernel by default (size-based dispatch); the
    matrix-core kernel stays correct there too when forced (DFS_CRC_LDS_MAX_MIB=0)."""
    native.set_crc_lds_max_mib(0)
    try:
        d = os.urandom(n)
        crc, meta = gstore.gpu_crc(d)
        assert crc == zlib.crc32(d) and meta == ref_meta(d)
    finally:
        native.set_crc_lds_max_mib(16)


@pytest.mark.parametrize("mode", [0, 1, 2])
@pytest.mark.parametrize("n", [511, (1 << 20) + 13, (8 << 20) - 4096 + 7, (64 << 20) + 513, 300 << 20])
def test_gpu_crc_wide_workgroups(gstore, native, mode, n):
    """K1/K2 with one workgroup per CU (three (mode 1) or two (mode 2) 4-wave groups sharing
    the LDS image and the MFMA basis, two-lookup combine) against zlib: whole-block CRC and
    every slice word, with tails."""
    saved = native.crc_wide_mode()
    native.set_crc_lds_max_mib(0)
    native.set_crc_wide(mode)
    try:
        d = os.urandom(n)
        crc, meta = gstore.gpu_crc(d)
        assert crc == zlib.crc32(d) and meta == ref_meta(d)
        if n < (100 << 20):
            ok, _, err = gstore.write(f"wide{mode}_{n}", d, zlib.crc32(d))
            assert ok, err
            st, total, out, partial, bad, err = gstore.read(f"wide{mode}_{n}", 0, 0)
            assert (st, total, out) == (0, n, d)
    finally:
        native.set_crc_wide(saved)
        native.set_crc_lds_max_mib(16)


@pytest.mark.parametrize("mode", [1, 2])
@pytest.mark.parametrize("n", [511, 4096 + 5, (1 << 20) + 13, (8 << 20) - 4096 + 7, (64 << 20) + 513, 300 << 20])
def test_gpu_crc_wide_fp4_matrix_cores(gstore, native, mode, n):
    """The wide K1/K2 kernel with its chunk CRCs on the FP4 matrix cores
    (v_mfma_scale_f32_32x32x64_f8f6f4, e2m1 operands, parity in bit 7 of an f32 biased by 2^16)
    against zlib: whole-block CRC, every slice word, tails; plus a patterned block whose bytes
    set every nibble bit (0xFF) and the sign bit of every nibble (0x88)."""
    saved_w, saved_f = native.crc_wide_mode(), native.crc_fp4_enabled()
    native.set_crc_lds_max_mib(0)
    native.set_crc_wide(mode)
    native.set_crc_fp4(True)
    try:
        for d in (os.urandom(n), (b"\xff\x88\x00\x11" * (n // 4 + 1))[:n]):
            crc, meta = gstore.gpu_crc(d)
            assert crc == zlib.crc32(d) and meta == ref_meta(d)
        if n < (100 << 20):
            ok, _, err = gstore.write(f"fp4_{mode}_{n}", d, zlib.crc32(d))
            assert ok, err
            st, total, out, partial, bad, err = gstore.read(f"fp4_{mode}_{n}", 0, 0)
            assert (st, total, out) == (0, n, d)
    finally:
        native.set_crc_fp4(saved_f)
        native.set_crc_wide(saved_w)
        native.set_crc_lds_max_mib(16)


def test_gpu_crc_zero_and_pattern(gstore):
    for d in (b"\0" * (1 << 20), bytes(range(256)) * 4099):
        crc, meta = gstore.gpu_crc(d)
        assert crc == zlib.crc32(d) and meta == ref_meta(d)


@pytest.mark.parametrize("n", [1000, (1 << 20) + 13])
def test_gpu_write_read_verify(gstore, n):
    d = os.urandom(n)
    ok, crc, err = gstore.write(f"b{n}", d, zlib.crc32(d))
    assert ok, err
    st, total, out, partial, bad, err = gstore.read(f"b{n}", 0, 0)
    assert (st, total, out, partial) == (0, n, d, False)
    for off, ln in [(0, 1), (511, 2), (1000 % n, 0), (n - 1, 5), (n // 3, n // 4 + 1)]:
        st, total, out, partial, bad, err = gstore.read(f"b{n}", off, ln)
        exp = d[off:] if ln == 0 else d[off:off + ln]
        assert st == 0 and out == exp and not partial


@pytest.mark.parametrize("rings", [(2, 2), (3, 3), (4, 4)])
def test_gpu_ring_depths(gstore, native, rings):
    """The register-ring variants of the MFMA kernels (scrub, and K1/K2/K3 on blocks of at
    least kCrcRingMinTiles tiles = 32 MiB) against zlib, including the verify path and a
    corruption the scrub must find."""
    saved = native.crc_kernels()
    native.set_crc_kernels(True, *rings)
    try:
        n = (40 << 20) + 512 * 5 + 77
        d = os.urandom(n)
        crc, meta = gstore.gpu_crc(d)
        assert crc == zlib.crc32(d) and meta == ref_meta(d)
        ok, crc, err = gstore.write("ring", d, zlib.crc32(d))
        assert ok, err
        st, total, out, partial, bad, err = gstore.read("ring", 0, 0)
        assert (st, total, partial) == (0, n, False) and out == d
        st, total, out, partial, bad, err = gstore.read("ring", 5 << 20, 33 << 20)
        assert st == 0 and out == d[5 << 20:38 << 20] and not partial
        assert gstore.scrub_resident(["ring"]) == []
        assert gstore.debug_corrupt("ring", (33 << 20) + 100)
        assert gstore.scrub_resident(["ring"]) == ["ring"]
        st, *_rest, err = gstore.read("ring", 0, 0)
        assert st == 3 and f"chunk {((33 << 20) + 100) // 512}" in err
    finally:
        native.set_crc_kernels(*saved)
        gstore.remove("ring")


def test_gpu_write_rejects_bad_crc(gstore):
    d = os.urandom(5000)
    ok, crc, err = gstore.write("badcrc", d, zlib.crc32(d) ^ 1)
    assert not ok and err.startswith("Checksum mismatch: expected")
    assert not gstore.exists("badcrc")


def test_gpu_durable_write_names(native, tmp_path):
    """nvme-sync writes of fresh ids go straight to their final names (directory flush beside
    the data flushes); a rejected fresh write leaves no file; a re-write of a known id takes
    the tmp+rename path and a rejected re-write keeps the durable copy."""
    s = native.ChunkStore(str(tmp_path), "", 0, 64 << 20, 0, 100, 2, 1, True, journal=0)
    base = s.stats()["final_name_writes"]
    d = os.urandom((1 << 20) + 5)
    assert s.write("fresh", d, zlib.crc32(d))[0]
    assert (tmp_path / "fresh").read_bytes() == d and (tmp_path / "fresh.meta").read_bytes() == ref_meta(d)
    assert s.stats()["final_name_writes"] == base + 1
    ok, _crc, err = s.write("fresh_bad", d, zlib.crc32(d) ^ 1)
    assert not ok and err.startswith("Checksum mismatch")
    assert not (tmp_path / "fresh_bad").exists() and not (tmp_path / "fresh_bad.meta").exists()
    d2 = os.urandom(70000)
    assert not s.write("fresh", d2, zlib.crc32(d2) ^ 1)[0]  # known id: the old copy survives
    assert (tmp_path / "fresh").read_bytes() == d
    assert s.write("fresh", d2, zlib.crc32(d2))[0]
    assert (tmp_path / "fresh").read_bytes() == d2 and (tmp_path / "fresh.meta").read_bytes() == ref_meta(d2)
    assert s.stats()["final_name_writes"] == base + 1
    assert not [p for p in os.listdir(tmp_path) if p.endswith(".tmp")]
    assert s.read("fresh", 0, 0)[2] == d2


def test_gpu_journal_write_evict_promote_materialize(native, tmp_path):
    """nvme-sync through the block journal on the GPU store: the fused staging kernel runs
    while the bytes are appended, one group commit acks; blocks evicted from a small arena
    are promoted back from their journal records (checksummed), then materialized into the
    reference files."""
    s = native.ChunkStore(str(tmp_path), "", 0, 8 << 20, 0, 100, 2, 1, True, journal=1)
    s.debug_pause_materializer(True)
    blobs = {f"j{i}": os.urandom((1 << 20) + 977 * i) for i in range(12)}
    blobs["small"] = os.urandom(4000)
    for k, v in blobs.items():
        ok, crc, err = s.write(k, v, zlib.crc32(v))
        assert ok and crc == zlib.crc32(v), err
    st = s.stats()
    assert st["journal_records"] == 13 and st["evictions"] > 0 and not (tmp_path / "j0").exists()
    for k, v in blobs.items():
        assert s.read(k, 0, 0)[2] == v
        assert s.read(k, 1000, 3000)[2] == v[1000:4000]
    assert s.stats()["promotions"] > 0
    assert s.scrub() == []
    s.debug_pause_materializer(False)
    s.materialize()
    for k, v in blobs.items():
        assert (tmp_path / k).read_bytes() == v and (tmp_path / f"{k}.meta").read_bytes() == ref_meta(v)
    bad = os.urandom(70000)
    assert not s.write("rej", bad, zlib.crc32(bad) ^ 1)[0] and not s.exists("rej")
    assert s.stats()["journal_failed"] is False


def test_gpu_journal_crash_replay_verifies_on_device(native, tmp_path):
    import subprocess
    import sys
    import textwrap

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = textwrap.dedent(f"""
        import os, zlib
        from rust_hadoop_generated_by_llm_amd import native
        s = native.lib.ChunkStore({str(tmp_path)!r}, "", 0, 64 << 20, 0, 100, 2, 1, True, journal=1)
        s.debug_pause_materializer(True)
        for i in range(6):
            v = bytes([i + 1]) * ((2 << 20) + i)
            assert s.write(f"r{{i}}", v, zlib.crc32(v))[0]
        s.remove("r2")
        os._exit(0)
    """)
    r = subprocess.run([sys.executable, "-c", code], env=dict(os.environ, PYTHONPATH=root), capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    s = native.ChunkStore(str(tmp_path), "", 0, 64 << 20, 0, 100, 2, 1, True, journal=1)
    st = s.stats()
    assert st["journal_replayed"] == 5 and st["journal_replay_skipped"] == 0
    assert st["gpu_kernel_launches"] >= 5  # K1/K2 verified every replayed record
    assert not s.exists("r2")
    for i in (0, 1, 3, 4, 5):
        v = bytes([i + 1]) * ((2 << 20) + i)
        assert s.read(f"r{i}", 0, 0)[2] == v


def test_gpu_scrub_runs_k1b_over_journal_resident_copies(native, tmp_path, monkeypatch):
    """Store of record: blocks whose only durable copy is their journal record (evicted from
    HBM) are scrubbed by the K1b kernel from staged batches; a flipped byte in one record is
    found, and resident blocks' journal copies are checked the same way."""
    monkeypatch.setenv("DFS_JOURNAL_EXPORT", "never")
    s = native.ChunkStore(str(tmp_path), "", 0, 16 << 20, 0, 100, 2, 1, True, journal=1)
    blobs = {f"k{i}": os.urandom((1 << 20) + 4099 * i) for i in range(24)}
    for k, v in blobs.items():
        assert s.write(k, v, zlib.crc32(v))[0]
    assert all(s.journaled(k) for k in blobs) and not (tmp_path / "k0").exists()
    s.drop_resident()
    assert s.scrub() == []
    st = s.stats()
    assert st["scrub_device_blocks"] >= len(blobs) and st["journal_live_records"] == len(blobs)
    assert s.debug_corrupt("k7", 5000)
    assert s.scrub() == ["k7"]
    for k, v in blobs.items():
        if k != "k7":
            assert s.read(k, 0, 0)[2] == v


def test_gpu_corruption_detected_full_and_partial(gstore):
    d = os.urandom(300000)
    assert gstore.write("corrupt", d, 0)[0]
    assert gstore.debug_corrupt("corrupt", 70000)
    st, *_rest, err = gstore.read("corrupt", 0, 0)
    assert st == 3 and "chunk 136" in err
    st, total, out, partial, bad, err = gstore.read("corrupt", 69000, 2000)
    assert st == 0 and partial and bad == 136
    st, total, out, partial, bad, err = gstore.read("corrupt", 0, 4096)
    assert st == 0 and not partial
    assert "corrupt" in gstore.scrub()
    gstore.remove("corrupt")


@pytest.mark.parametrize("fp4", [False, True])
def test_gpu_batched_scrub_finds_exactly_the_corrupt_blocks(gstore, native, fp4):
    # K1b: one launch over blocks of every shape (tiny, exact slices, tails, multi-tile);
    # corrupt a middle slice, a last full slice and a tail byte in different blocks; with the
    # chunk CRCs on the i8 and on the FP4 matrix cores
    saved = native.crc_fp4_enabled()
    native.set_crc_fp4(fp4)
    try:
        _batched_scrub(gstore)
    finally:
        native.set_crc_fp4(saved)


def _batched_scrub(gstore):
    sizes = [1, 100, 511, 512, 513, 4096, 16384 + 1, 65536, (1 << 20), (1 << 20) + 300, 3 * (1 << 20) + 7]
    ids = []
    for i, n in enumerate(sizes * 3):
        bid = f"scrub{i}"
        d = os.urandom(n)
        assert gstore.write(bid, d, zlib.crc32(d))[0]
        ids.append((bid, n))
    assert gstore.scrub_resident([b for b, _ in ids]) == []
    targets = {ids[9][0]: 600000, ids[10 + 11][0]: 3 * (1 << 20) + 3, ids[2 * 11 + 7][0]: 65535,
               ids[4][0]: 512}
    for bid, off in targets.items():
        assert gstore.debug_corrupt(bid, off), bid
    found = gstore.scrub_resident([b for b, _ in ids])
    assert sorted(found) == sorted(targets)
    for bid, _ in ids:
        gstore.remove(bid)


def test_gpu_eviction_and_promotion(native, tmp_path):
    s = native.ChunkStore(str(tmp_path), "", 0, 8 << 20, 0, 100, 2, 1, False)
    blobs = {f"e{i}": os.urandom(1 << 20) for i in range(20)}
    for k, v in blobs.items():
        assert s.write(k, v, zlib.crc32(v))[0]
    st = s.stats()
    assert st["evictions"] > 0 and st["hbm_used"] <= 8 << 20
    for k, v in blobs.items():
        r = s.read(k, 0, 0)
        assert r[0] == 0 and r[2] == v
    assert s.stats()["promotions"] > 0


def test_gpu_hbm_ack_spill(native, tmp_path):
    s = native.ChunkStore(str(tmp_path), "", 0, 64 << 20, 1, 100, 2, 2, False)
    d = os.urandom(777777)
    assert s.write("spill", d, 0)[0]
    s.flush()
    assert (tmp_path / "spill").read_bytes() == d
    assert (tmp_path / "spill.meta").read_bytes() == ref_meta(d)
    assert s.verify_on_disk("spill") == ""


def test_gpu_reed_solomon(gstore):
    from rust_hadoop_generated_by_llm_amd.ops import erasure

    for k, m, n in [(2, 2, 10000), (4, 2, 1 << 20), (6, 3, (1 << 20) + 5)]:
        d = os.urandom(n)
        g = erasure.encode(d, k, m, gstore)
        c = erasure.encode(d, k, m, None)
        assert g == c
        lost = list(range(m))
        shards = [None if i in lost else s for i, s in enumerate(g)]
        assert erasure.decode(shards, k, m, n, gstore) == d
    assert gstore.stats()["gpu_kernel_launches"] > 0


def test_gpu_small_block_mirror(gstore):
    """Blocks <= 64 KiB keep a host copy: reads are a CPU-verified memcpy (no GPU round trip);
    a corrupted slice is still caught (the mirror is dropped and the device path reports it)."""
    d = os.urandom(40_000)
    assert gstore.write("mir", d, zlib.crc32(d))[0]
    h0 = gstore.stats()["mirror_hits"]
    st, total, out, partial, bad, err = gstore.read("mir", 0, 0)
    assert st == 0 and out == d and total == len(d)
    st, total, out, partial, bad, err = gstore.read("mir", 1234, 4096)
    assert st == 0 and out == d[1234:1234 + 4096] and not partial
    assert gstore.stats()["mirror_hits"] == h0 + 2
    assert gstore.debug_corrupt("mir", 30_000)
    st, *_rest, err = gstore.read("mir", 0, 0)
    assert st == 3 and "chunk 58" in err  # 30000 // 512
    st, total, out, partial, bad, err = gstore.read("mir", 29_900, 200)
    assert st == 0 and partial and bad == 58
    assert gstore.stats()["mirror_hits"] == h0 + 2  # the damaged mirror served nothing
    gstore.remove("mir")


def test_gpu_fused_write_copy(gstore):
    """K1/K2 fused with the host-to-device copy (crc_write_copy_kernel): a write whose bytes sit
    in registered host memory is one kernel that stores the block into HBM, checksums it and
    leaves the .meta image in host memory — against zlib, with tails and a multi-tile block,
    and a wrong expected CRC still rejected. Blocks <= 64 KiB keep the host-CRC path."""
    import numpy as np

    buf = np.zeros((40 << 20) + 4096, dtype=np.uint8)
    assert gstore.register_host(buf)
    try:
        f0 = gstore.stats()["fused_writes"]
        sizes = [65537, 300000, (1 << 20), (1 << 20) + 13, 3 * (1 << 20) + 1, (40 << 20) + 512 * 3 + 77]
        for i, n in enumerate(sizes):
            d = np.frombuffer(os.urandom(n), dtype=np.uint8)
            buf[:n] = d
            ok, crc, err = gstore.write(f"fw{i}", buf[:n], zlib.crc32(d.tobytes()))
            assert ok and crc == zlib.crc32(d.tobytes()), (n, err)
            buf[:n] = 0  # the store must hold its own copy
            st, total, out, partial, bad, err = gstore.read(f"fw{i}", 0, 0)
            assert (st, total, partial) == (0, n, False) and out == d.tobytes(), n
            assert gstore.scrub_resident([f"fw{i}"]) == []  # the HBM .meta image matches too
        assert gstore.stats()["fused_writes"] - f0 == len(sizes)
        d = os.urandom(500000)
        buf[:len(d)] = np.frombuffer(d, dtype=np.uint8)
        ok, _crc, err = gstore.write("fw_bad", buf[:len(d)], zlib.crc32(d) ^ 1)
        assert not ok and err.startswith("Checksum mismatch") and not gstore.exists("fw_bad")
        small = os.urandom(4000)
        buf[:4000] = np.frombuffer(small, dtype=np.uint8)
        f1 = gstore.stats()["fused_writes"]
        assert gstore.write("fw_small", buf[:4000], zlib.crc32(small))[0]
        assert gstore.stats()["fused_writes"] == f1 and gstore.read("fw_small", 0, 0)[2] == small
    finally:
        gstore.unregister_host(buf)
        for i in range(6):
            gstore.remove(f"fw{i}")
        gstore.remove("fw_small")


def test_gpu_fused_read_copy(gstore):
    """K3 fused verify + copy (crc_read_copy_kernel): reads into a registered buffer are one
    kernel that checks every touched slice and stores the range straight into host memory.
    Whole blocks, slice-unaligned ranges (byte-wise edges), tails, and a corruption that
    must still be reported; bytes outside the range are never written."""
    import numpy as np

    buf = np.zeros((40 << 20) + 4096, dtype=np.uint8)
    assert gstore.register_host(buf)
    try:
        sizes = [(1 << 20), (1 << 20) + 777, 300000, 3 * (1 << 20) + 1, (33 << 20) + 512 * 3 + 5]
        datas = {}
        for i, n in enumerate(sizes):
            d = os.urandom(n)
            assert gstore.write(f"fz{i}", d, zlib.crc32(d))[0]
            datas[f"fz{i}"] = d
        f0 = gstore.stats()["fused_reads"]
        expect_fused = 0
        cases = [(0, 0), (0, 4096), (512 * 7, 512 * 9), (100, 70001), (1000, 1), (511, 2)]
        for bid, d in datas.items():
            n = len(d)
            for off, ln in cases + [(n - 600, 600), (n - 1, 1), (n // 2 + 3, n // 2 - 3)]:
                ln = n if ln == 0 else ln
                if off + ln > n:
                    continue
                k = off % 16  # (out - off) % 16 == 0 keeps the 16 B stores aligned
                buf[:] = 0xA5
                st, total, got, partial, bad, err = gstore.read_into(bid, off, ln, buf[k:])
                assert st == 0 and not partial, (bid, off, ln, err)
                assert got == ln and buf[k:k + ln].tobytes() == d[off:off + ln], (bid, off, ln)
                assert (buf[:k] == 0xA5).all() and (buf[k + ln:k + ln + 4096] == 0xA5).all(), (bid, off, ln)
                expect_fused += 1
        assert gstore.stats()["fused_reads"] - f0 == expect_fused  # every read took the fused kernel
        # corruption: the whole-block read fails, a range around it reports the slice
        assert gstore.debug_corrupt("fz1", 700000)
        st, *_rest, err = gstore.read_into("fz1", 0, len(datas["fz1"]), buf)
        assert st == 3 and f"chunk {700000 // 512}" in err
        st, total, got, partial, bad, err = gstore.read_into("fz1", 699000, 4000, buf[699000 % 16:])
        assert st == 0 and partial and bad == 700000 // 512
        st, total, got, partial, bad, err = gstore.read_into("fz1", 0, 65536, buf)
        assert st == 0 and not partial and buf[:65536].tobytes() == datas["fz1"][:65536]
    finally:
        gstore.unregister_host(buf)
        for i in range(5):
            gstore.remove(f"fz{i}")
