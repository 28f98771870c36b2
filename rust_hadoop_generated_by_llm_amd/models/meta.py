"""JSON (serde-layout) codecs for metadata messages.

Raft log entries and snapshots carry ``FileMetadata``/``BlockInfo`` as JSON objects with
snake_case proto field names and integers as JSON numbers, the layout the reference gets
from ``#[derive(Serialize)]`` on its prost structs (dfs/metaserver/build.rs:2-4; SURVEY
Appendix C). ``json_format`` would render uint64 as strings, so these are hand-written.
"""
from __future__ import annotations

from . import proto as pb

_BLOCK_FIELDS = ("block_id", "size", "checksum_crc32c", "ec_data_shards", "ec_parity_shards", "original_size")
_FILE_FIELDS = ("path", "size", "etag_md5", "created_at_ms", "ec_data_shards", "ec_parity_shards",
                "last_access_ms", "access_count", "moved_to_cold_at_ms")


def block_to_dict(b) -> dict:
    d = {f: getattr(b, f) for f in _BLOCK_FIELDS}
    d["locations"] = list(b.locations)
    return d


def block_from_dict(d: dict):
    b = pb.BlockInfo(**{f: d[f] for f in _BLOCK_FIELDS if f in d and d[f] is not None})
    b.locations.extend(d.get("locations", []))
    return b


def file_to_dict(m) -> dict:
    d = {f: getattr(m, f) for f in _FILE_FIELDS}
    d["blocks"] = [block_to_dict(b) for b in m.blocks]
    if m.attributes:  # extension; absent keeps the reference layout
        d["attributes"] = dict(m.attributes)
    return d


def file_from_dict(d: dict):
    m = pb.FileMetadata(**{f: d[f] for f in _FILE_FIELDS if f in d and d[f] is not None})
    for b in d.get("blocks", []):
        m.blocks.append(block_from_dict(b))
    m.attributes.update(d.get("attributes") or {})
    return m


def checksum_to_dict(c) -> dict:
    return {"block_id": c.block_id, "checksum_crc32c": c.checksum_crc32c, "actual_size": c.actual_size}


def checksum_from_dict(d: dict):
    return pb.BlockChecksumInfo(block_id=d["block_id"], checksum_crc32c=d.get("checksum_crc32c", 0),
                                actual_size=d.get("actual_size", 0))


def command_to_dict(c) -> dict:
    d = {"type": int(c.type), "block_id": c.block_id, "target_chunk_server_address": c.target_chunk_server_address,
         "shard_index": c.shard_index, "ec_data_shards": c.ec_data_shards, "ec_parity_shards": c.ec_parity_shards,
         "ec_shard_sources": list(c.ec_shard_sources), "original_block_size": c.original_block_size,
         "master_term": c.master_term}
    return d
