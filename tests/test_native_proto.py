"""Golden tests of the generated native proto3 codec (csrc/dfs_pb.h, scripts/gen_proto.py)
against Python protobuf built from the same proto/dfs.proto: random messages of every
type are decoded and re-encoded natively and must come back identical."""
import random

import pytest
from google.protobuf.descriptor import FieldDescriptor as FD

from rust_hadoop_generated_by_llm_amd.models import proto as pb
from rust_hadoop_generated_by_llm_amd.native import lib as native

MESSAGES = sorted(pb.FILE_DESCRIPTOR.message_types_by_name)


def _scalar(f, rng):
    t = f.type
    if t == FD.TYPE_STRING:
        return rng.choice(["", "a", "/bench_r000/w0/bench_0000000001", "ünï/☃", "x" * rng.randint(0, 300)])
    if t == FD.TYPE_BYTES:
        return rng.randbytes(rng.choice([0, 1, 17, 1000]))
    if t == FD.TYPE_BOOL:
        return rng.random() < 0.5
    if t == FD.TYPE_UINT32:
        return rng.choice([0, 1, 127, 128, 2**32 - 1, rng.randrange(2**32)])
    if t == FD.TYPE_UINT64:
        return rng.choice([0, 1, 300, 2**63, 2**64 - 1, rng.randrange(2**64)])
    if t in (FD.TYPE_INT32, FD.TYPE_ENUM):
        if t == FD.TYPE_ENUM:
            return rng.choice([v.number for v in f.enum_type.values])
        return rng.choice([0, -1, 1, -(2**31), 2**31 - 1, rng.randrange(-(2**31), 2**31)])
    if t == FD.TYPE_INT64:
        return rng.choice([0, -1, rng.randrange(-(2**63), 2**63)])
    if t == FD.TYPE_DOUBLE:
        return rng.choice([0.0, 1.5, -2.25, 1e300, rng.random()])
    raise AssertionError(f"unhandled type {t}")


def _fill(msg, rng, depth=0):
    for f in msg.DESCRIPTOR.fields:
        if rng.random() < 0.3:
            continue
        if f.message_type is not None and f.message_type.GetOptions().map_entry:
            kf, vf = f.message_type.fields_by_name["key"], f.message_type.fields_by_name["value"]
            m = getattr(msg, f.name)
            for _ in range(rng.randint(0, 3)):
                k = _scalar(kf, rng)
                if vf.message_type is not None:
                    _fill(m[k], rng, depth + 1)
                else:
                    m[k] = _scalar(vf, rng)
        elif f.is_repeated:
            if f.message_type is not None:
                for _ in range(rng.randint(0, 3 if depth < 2 else 0)):
                    _fill(getattr(msg, f.name).add(), rng, depth + 1)
            else:
                getattr(msg, f.name).extend(_scalar(f, rng) for _ in range(rng.randint(0, 4)))
        elif f.message_type is not None:
            if depth < 3:
                _fill(getattr(msg, f.name), rng, depth + 1)
                getattr(msg, f.name).SetInParent()
        else:
            setattr(msg, f.name, _scalar(f, rng))


@pytest.mark.parametrize("name", MESSAGES)
def test_native_codec_roundtrip(name):
    rng = random.Random(hash(name) & 0xFFFF)
    cls = getattr(pb, name)
    for _ in range(40):
        m = cls()
        _fill(m, rng)
        wire = m.SerializeToString()
        out = native.pb_roundtrip(name, wire)
        assert out is not None, f"native decode of {name} failed"
        assert cls.FromString(out) == m
        if not _has_map(m.DESCRIPTOR):  # canonical encoding: identical bytes (map order is free)
            assert out == wire


def _has_map(desc, seen=None) -> bool:
    seen = set() if seen is None else seen
    if desc.full_name in seen:
        return False
    seen.add(desc.full_name)
    for f in desc.fields:
        if f.message_type is not None:
            if f.message_type.GetOptions().map_entry or _has_map(f.message_type, seen):
                return True
    return False


def test_native_codec_rejects_truncated_input():
    m = pb.FileMetadata(path="/a/b", size=5, blocks=[pb.BlockInfo(block_id="x", locations=["h:1", "h:2"])])
    wire = m.SerializeToString()
    assert native.pb_roundtrip("FileMetadata", wire[:-3]) is None
    # unknown fields are skipped (forward compatibility with newer peers)
    extra = wire + b"\xa8\x1f\x05"  # field 501, varint 5
    assert pb.FileMetadata.FromString(native.pb_roundtrip("FileMetadata", extra)) == m
