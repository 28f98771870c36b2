"""Client library and CLI unit tests (reference dfs/client/src/mod.rs:1538 — EC shard sizes,
dead-port errors, hedge config, degraded EC decode — and dfs_cli.rs:810 parse_s3_url)."""
import os
import time
from types import SimpleNamespace

import pytest

from rust_hadoop_generated_by_llm_amd.cli.dfs_cli import build_parser, parse_s3_url
from rust_hadoop_generated_by_llm_amd.client.client import Client, DfsError
from rust_hadoop_generated_by_llm_amd.ops import erasure


# ----------------------------------------------------------------------------- CLI
def test_parse_s3_url_simple():
    assert parse_s3_url("s3://bucket/key") == ("bucket", "key")


def test_parse_s3_url_nested_key():
    assert parse_s3_url("s3://my-bucket/a/b/c.txt") == ("my-bucket", "a/b/c.txt")


@pytest.mark.parametrize("url,msg", [
    ("http://bucket/key", "s3://"),
    ("s3://bucket", "key"),
    ("s3:///key", "empty"),
    ("s3://bucket/", "empty"),
])
def test_parse_s3_url_errors(url, msg):
    with pytest.raises(ValueError, match=msg):
        parse_s3_url(url)


def test_cli_has_every_reference_subcommand():
    p = build_parser()
    sub = next(a for a in p._actions if a.__class__.__name__ == "_SubParsersAction")
    for cmd in ("ls", "put", "get", "inspect", "rename", "safe-mode", "cluster", "shuffle", "benchmark",
                "workload", "check-history", "presign"):
        assert cmd in sub.choices, cmd


# ----------------------------------------------------------------------------- EC sizing
@pytest.mark.parametrize("n,k,expect", [(10, 4, 3), (12, 4, 3), (1, 6, 1), (0, 2, 0), (1 << 20, 6, 174763)])
def test_ec_shard_sizes(n, k, expect):
    assert erasure.shard_len(n, k) == expect
    if n:
        shards = erasure.encode(bytes(range(256)) * (n // 256) + bytes(n % 256), k, 2)
        assert len(shards) == k + 2 and all(len(s) == expect for s in shards)


# ----------------------------------------------------------------------------- dead ports
def test_unreachable_masters_fail_after_bounded_retries():
    c = Client(["127.0.0.1:19997", "127.0.0.1:19998"], max_retries=2, initial_backoff_ms=10, rpc_timeout=0.5)
    try:
        t0 = time.time()
        with pytest.raises(DfsError, match="No available leader"):
            c.list_files("/")
        assert time.time() - t0 < 10
    finally:
        c.close()


def test_retry_and_hedge_config_builders():
    c = Client(["127.0.0.1:19999"]).with_retry_config(7, 25).with_hedge_delay(15)
    try:
        assert (c.max_retries, c.initial_backoff_ms, c.hedge_delay_ms) == (7, 25, 15)
        assert c.master_addrs == ["http://127.0.0.1:19999"]
    finally:
        c.close()


# ----------------------------------------------------------------------------- hedged reads
def _client_with_fake_replicas(behaviour):
    """behaviour: addr -> (delay_s, bytes | Exception)"""
    c = Client(["127.0.0.1:19999"], hedge_delay_ms=50)
    calls = []

    def read(loc, block_id, offset=0, length=0, *a, **kw):
        calls.append(loc)
        delay, out = behaviour[loc]
        time.sleep(delay)
        if isinstance(out, Exception):
            raise out
        return out

    c.read_block_from_location = read
    return c, calls


def test_hedged_read_races_a_slow_primary():
    c, calls = _client_with_fake_replicas({"p": (1.0, b"slow"), "s": (0.0, b"fast")})
    try:
        t0 = time.time()
        assert c._hedged_read(["p", "s"], "b1", 0, 0) == b"fast"
        assert time.time() - t0 < 0.8 and calls[:2] == ["p", "s"]
    finally:
        c.close()


def test_hedged_read_fast_primary_never_hedges():
    c, calls = _client_with_fake_replicas({"p": (0.0, b"primary"), "s": (0.0, b"second")})
    try:
        assert c._hedged_read(["p", "s"], "b1", 0, 0) == b"primary"
        assert calls == ["p"]
    finally:
        c.close()


def test_hedged_read_all_replicas_fail():
    import grpc

    class Dead(grpc.RpcError):
        pass

    c, _ = _client_with_fake_replicas({"p": (0.0, Dead()), "s": (0.0, Dead()), "t": (0.0, Dead())})
    try:
        with pytest.raises(DfsError, match="every replica"):
            c._hedged_read(["p", "s", "t"], "b1", 0, 0)
    finally:
        c.close()


# ----------------------------------------------------------------------------- degraded EC
@pytest.mark.parametrize("lost", [(), (0,), (1, 4), (0, 2)])
def test_degraded_ec_read_decodes(lost):
    data = os.urandom(10_000)
    k, m = 4, 2
    shards = erasure.encode(data, k, m)
    addrs = [f"cs{i}" for i in range(k + m)]
    behaviour = {a: (0.0, RuntimeError("down") if i in lost else shards[i]) for i, a in enumerate(addrs)}
    c, _ = _client_with_fake_replicas(behaviour)
    try:
        block = SimpleNamespace(ec_data_shards=k, ec_parity_shards=m, locations=addrs, block_id="b",
                                original_size=len(data), size=len(data))
        assert c.read_ec_block(block) == data
    finally:
        c.close()


def test_ec_read_with_too_many_losses_fails():
    data = os.urandom(5000)
    shards = erasure.encode(data, 2, 1)
    addrs = ["a", "b", "c"]
    behaviour = {"a": (0.0, RuntimeError("x")), "b": (0.0, RuntimeError("y")), "c": (0.0, shards[2])}
    c, _ = _client_with_fake_replicas(behaviour)
    try:
        block = SimpleNamespace(ec_data_shards=2, ec_parity_shards=1, locations=addrs, block_id="b",
                                original_size=len(data), size=len(data))
        with pytest.raises(Exception):
            c.read_ec_block(block)
    finally:
        c.close()
