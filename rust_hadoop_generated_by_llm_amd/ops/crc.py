"""CRC-32/IEEE helpers (what the reference stores in every ``*_crc32c`` field and in
``.meta`` files; dfs/chunkserver/src/chunkserver.rs:182-190)."""
from __future__ import annotations

import struct

from ..native import lib

SLICE = 512


def crc32(data, crc: int = 0) -> int:
    return lib.crc32(data, crc)


def meta_image(data) -> bytes:
    """Big-endian CRC per 512-byte slice (the on-disk ``<block>.meta`` format)."""
    return lib.crc32_meta(data)


def parse_meta(meta: bytes) -> list[int]:
    return list(struct.unpack(f">{len(meta) // 4}I", meta))


def crc32_from_meta(meta: bytes, n: int) -> int:
    return lib.crc32_from_meta(meta, n)


def combine(crc_a: int, crc_b: int, len_b: int) -> int:
    return lib.crc32_combine(crc_a, crc_b, len_b)


def gpu_crc32(store, data) -> tuple[int, bytes]:
    """K1+K2 on the device of an HBM ChunkStore: (block crc, .meta image)."""
    return store.gpu_crc(data)
