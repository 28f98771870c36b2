"""Routing parity between the two ShardMap implementations: the native one the masters and the
config server route with (csrc/shard_map.cpp) and the Python one clients, chunkservers and the
S3 gateway use (parallel/sharding.py). Clients and servers compute routing independently
(reference dfs/common/src/sharding.rs:17-341), so they must agree on every key, after every
split / merge / boundary move, and on the serialised map itself."""
import json
import random

from hypothesis import given, settings
from hypothesis import strategies as st

from rust_hadoop_generated_by_llm_amd.native import lib as native
from rust_hadoop_generated_by_llm_amd.parallel.sharding import MAX_KEY, ShardMap

# keys as paths look, plus arbitrary text (no lone surrogates: keys are UTF-8 on the wire)
_chars = st.characters(blacklist_categories=("Cs",))
keys = st.one_of(
    st.text(_chars, max_size=24),
    st.builds(lambda parts: "/" + "/".join(parts), st.lists(st.text(_chars, min_size=1, max_size=8), max_size=4)),
    st.sampled_from(["", "/", "/m", "/m/", "/l", "/n", "z-", "z-shard-1", "zz", MAX_KEY, "\x00", "/a/b"]),
)
shard_ids = st.text("abcdefghijklmnopqrstuvwxyz-0123456789", min_size=1, max_size=10)


def _native_of(m: ShardMap):
    return native.NativeShardMap.from_json(json.dumps(m.to_json()))


def _agree(py: ShardMap, nat, ks):
    got = nat.get_shards(list(ks))
    for k, g in zip(ks, got):
        assert (g or None) == py.get_shard(k), (k, g, py.get_shard(k))


@settings(max_examples=60, deadline=None)
@given(st.lists(shard_ids, min_size=1, max_size=6, unique=True), st.integers(1, 160), st.lists(keys, max_size=60))
def test_consistent_hash_routing_agrees(ids, vnodes, ks):
    py = ShardMap.new_consistent_hash(vnodes)
    nat = native.NativeShardMap.new_consistent_hash(vnodes)
    for sid in ids:
        py.add_shard(sid, [f"http://{sid}:1"])
        nat.add_shard(sid, [f"http://{sid}:1"])
    assert json.loads(nat.to_json()) == py.to_json()  # identical ring, hashes included
    _agree(py, nat, ks)
    # removing a shard moves only that shard's keys, identically on both sides
    py.remove_shard(ids[0])
    nat.remove_shard(ids[0])
    _agree(py, nat, ks)
    assert json.loads(nat.to_json()) == py.to_json()


ops = st.lists(st.tuples(st.sampled_from(["add", "remove", "split", "merge", "rebalance"]), shard_ids, keys, keys),
               max_size=25)


@settings(max_examples=80, deadline=None)
@given(st.lists(shard_ids, min_size=1, max_size=4, unique=True), ops, st.lists(keys, max_size=40))
def test_range_map_operations_agree(ids, seq, ks):
    """Random sequences of the config server's map mutations applied to both maps: same
    results, same serialised map, same owner for every key after every step."""
    py, nat = ShardMap.new_range(), native.NativeShardMap.new_range()
    for sid in ids:
        py.add_shard(sid, [sid])
        nat.add_shard(sid, [sid])
    for op, sid, k1, k2 in seq:
        shards = sorted(py.shards)
        if op == "add":
            py.add_shard(sid, [sid])
            nat.add_shard(sid, [sid])
        elif op == "remove" and shards:
            victim = shards[len(sid) % len(shards)]
            py.remove_shard(victim)
            nat.remove_shard(victim)
        elif op == "split":
            assert py.split_shard(k1, sid, [sid]) == nat.split_shard(k1, sid, [sid])
        elif op == "merge" and len(shards) >= 2:
            v, r = shards[len(sid) % len(shards)], shards[(len(sid) + 1) % len(shards)]
            assert py.merge_shards(v, r) == nat.merge_shards(v, r)
        elif op == "rebalance":
            ends = sorted(py.ranges)
            old = ends[len(k1) % len(ends)] if ends and k1 else k1
            assert py.rebalance_boundary(old, k2) == nat.rebalance_boundary(old, k2)
        assert json.loads(nat.to_json()) == py.to_json(), (op, sid, k1, k2)
        _agree(py, nat, ks + sorted(py.ranges))


def test_bulk_random_paths_agree():
    """100k random paths against a 16-shard range map with dynamic split keys and a
    16-shard hash ring: one native batch call, compared key by key."""
    rng = random.Random(20260)
    py = ShardMap.from_config({f"shard-{i}": [f"m{i}"] for i in range(4)})
    for i in range(4, 16):
        key = "/" + "".join(rng.choice("abcdefghijklmnopqrstuvwxyz") for _ in range(rng.randint(1, 6)))
        py.split_shard(key, f"shard-{i}", [f"m{i}"])
    ring = ShardMap.new_consistent_hash(100)
    for i in range(16):
        ring.add_shard(f"shard-{i}", [f"m{i}"])
    alphabet = "abcdefghijklmnopqrstuvwxyz/-_.0123456789éü中"
    paths = ["/" + "".join(rng.choice(alphabet) for _ in range(rng.randint(0, 40))) for _ in range(100_000)]
    for m in (py, ring):
        nat = _native_of(m)
        got = nat.get_shards(paths)
        want = [m.get_shard(p) for p in paths]
        assert got == want
        assert len(set(want)) > 4  # the keys really spread over the shards
