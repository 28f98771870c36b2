"""Linearizability checker (C49) and workload generator (C50).

Mirrors the reference's checker unit tests (dfs/client/src/checker.rs:850: hand-written
JSONL histories — linearizable, stale read, lost value, duplicated value, renames, crashed
ops, self-tests) and drives the workload generator against in-memory stores: a correct
(locked) one must always check clean, a store with a stale read cache must be caught."""
import hashlib
import json
import threading
import time

import pytest

from rust_hadoop_generated_by_llm_amd.client import checker
from rust_hadoop_generated_by_llm_amd.client.checker import (HistoryError, _h, _inv, _ret, check_linearizability,
                                                              parse_history)
from rust_hadoop_generated_by_llm_amd.client.workload import key_path, run_workload


def _ok(lines) -> bool:
    return not check_linearizability(parse_history(lines))


@pytest.mark.parametrize("name", sorted(checker.SELF_TESTS))
def test_self_test_histories(name):
    expect_ok, lines = checker.SELF_TESTS[name]
    assert _ok(lines) == expect_ok


def test_run_self_tests_is_clean():
    assert checker.run_self_tests() == []


def test_real_time_order_is_enforced():
    # the put returned before the get was invoked: the get must see it
    assert not _ok(_h(_inv(1, "put", 1, path="/a", data_hash="h"), _ret(1, "put_ok:h", 2),
                      _inv(2, "get", 3, path="/a", client="c2"), _ret(2, "not_found", 4, "c2")))
    # overlapping: either order is allowed
    assert _ok(_h(_inv(1, "put", 1, path="/a", data_hash="h"),
                  _inv(2, "get", 2, path="/a", client="c2"), _ret(2, "not_found", 3, "c2"),
                  _ret(1, "put_ok:h", 4)))


def test_put_over_existing_file_must_fail():
    lines = _h(_inv(1, "put", 1, path="/a", data_hash="h1"), _ret(1, "put_ok:h1", 2),
               _inv(2, "put", 3, path="/a", data_hash="h2"), _ret(2, "error", 4),
               _inv(3, "get", 5, path="/a"), _ret(3, "get_ok:h1", 6))
    assert _ok(lines)


def test_rename_onto_existing_destination_fails():
    base = [_inv(1, "put", 1, path="/a", data_hash="h1"), _ret(1, "put_ok:h1", 2),
            _inv(2, "put", 3, path="/z", data_hash="h2"), _ret(2, "put_ok:h2", 4),
            _inv(3, "rename", 5, src="/a", dst="/z")]
    assert not _ok(_h(*base, _ret(3, "ok", 6)))
    assert _ok(_h(*base, _ret(3, "error", 6)))
    # the reference reports a missing source as not_found: same as a failed rename
    assert _ok(_h(_inv(1, "rename", 1, src="/a", dst="/z"), _ret(1, "not_found", 2)))


def test_half_done_rename_is_a_violation():
    # both names visible after a completed rename = the cross-shard anomaly 2PC prevents
    lines = _h(_inv(1, "put", 1, path="/a", data_hash="h1"), _ret(1, "put_ok:h1", 2),
               _inv(2, "rename", 3, src="/a", dst="/z"), _ret(2, "ok", 4),
               _inv(3, "get", 5, path="/a"), _ret(3, "get_ok:h1", 6),
               _inv(4, "get", 7, path="/z"), _ret(4, "get_ok:h1", 8))
    assert not _ok(lines)


def test_crashed_delete_can_linearize_late():
    lines = _h(_inv(1, "put", 1, path="/a", data_hash="h1"), _ret(1, "put_ok:h1", 2),
               _inv(2, "delete", 3, path="/a"),  # never returns
               _inv(3, "get", 4, path="/a", client="c2"), _ret(3, "get_ok:h1", 5, "c2"),
               _inv(4, "get", 6, path="/a", client="c2"), _ret(4, "not_found", 7, "c2"))
    assert _ok(lines)
    # ...but a value cannot come back after it was observed gone with no put in between
    lines2 = lines[:-2] + _h(_inv(4, "get", 6, path="/a", client="c2"), _ret(4, "not_found", 7, "c2"),
                             _inv(5, "get", 8, path="/a", client="c2"), _ret(5, "get_ok:h1", 9, "c2"))
    assert not _ok(lines2)


def test_independent_keys_are_checked_separately():
    good = [_inv(1, "put", 1, path="/a", data_hash="x"), _ret(1, "put_ok:x", 2)]
    bad = [_inv(2, "put", 3, path="/b", data_hash="y"), _ret(2, "put_ok:y", 4),
           _inv(3, "get", 5, path="/b"), _ret(3, "not_found", 6)]
    v = check_linearizability(parse_history(_h(*good, *bad)))
    assert len(v) == 1 and "/b" in v[0] and "/a" not in v[0]


def test_rename_links_keys_into_one_component():
    ops = parse_history(_h(_inv(1, "rename", 1, src="/a", dst="/b"), _ret(1, "error", 2),
                           _inv(2, "rename", 3, src="/b", dst="/c"), _ret(2, "error", 4),
                           _inv(3, "get", 5, path="/d"), _ret(3, "not_found", 6)))
    comps = checker._components(ops)
    assert sorted(len(c) for c in comps) == [1, 2]


def test_budget_exhaustion_is_reported_not_passed():
    # many concurrent ambiguous ops on one key, then a read no order can explain: the
    # search must explore (and exhaust) the space before it could say "violation"
    recs = []
    for i in range(40):
        recs.append(_inv(i, "put", 1, path="/a", data_hash=f"h{i}", client=f"c{i}"))
    for i in range(40):
        recs.append(_ret(i, "error", 100, f"c{i}"))
    recs += [_inv(99, "get", 200, path="/a"), _ret(99, "get_ok:never-written", 201)]
    v = check_linearizability(parse_history(_h(*recs)), budget=500)
    assert v and "budget" in v[0]


@pytest.mark.parametrize("bad,err", [
    ('{"id": 1, "type": "return", "result": "ok", "ts_ns": 1}', "without matching invoke"),
    ('{"id": 1, "type": "bogus"}', "unknown entry type"),
    ('{"id": 1, "type": "invoke", "op": "chmod", "ts_ns": 1}', "unknown op"),
    ('not json', "line 1"),
])
def test_malformed_histories_are_rejected(bad, err):
    with pytest.raises(HistoryError, match=err):
        parse_history([bad])


def test_check_file_and_blank_lines(tmp_path):
    p = tmp_path / "h.jsonl"
    _, lines = checker.SELF_TESTS["rename_moves_value"]
    p.write_text("\n".join(lines[:2]) + "\n\n" + "\n".join(lines[2:]) + "\n")
    assert checker.check_file(str(p)) == []


# ----------------------------------------------------------------------------- workload
class _MemClient:
    """Linearizable in-memory stand-in for Client: one lock around the map."""

    def __init__(self):
        self.files: dict[str, bytes] = {}
        self.lock = threading.Lock()

    def create_file_from_buffer(self, data: bytes, path: str) -> int:
        with self.lock:
            if path in self.files:
                raise RuntimeError("File already exists")
            self.files[path] = bytes(data)
        return len(data)

    def get_file_content(self, path: str) -> bytes:
        with self.lock:
            if path not in self.files:
                raise RuntimeError("File not found")
            return self.files[path]

    def delete_file(self, path: str) -> None:
        with self.lock:
            if self.files.pop(path, None) is None:
                raise RuntimeError("File not found")

    def rename_file(self, src: str, dst: str) -> None:
        with self.lock:
            if src not in self.files:
                raise RuntimeError("Source file not found")
            if dst in self.files:
                raise RuntimeError("Destination exists")
            self.files[dst] = self.files.pop(src)


class _StaleCacheClient(_MemClient):
    """Serves reads from a per-thread cache that deletes do not invalidate (a stale read)."""

    def __init__(self):
        super().__init__()
        self.cache = threading.local()

    def get_file_content(self, path: str) -> bytes:
        c = self.cache.__dict__.setdefault("m", {})
        if path in c:
            return c[path]
        data = super().get_file_content(path)
        c[path] = data
        time.sleep(0.0005)
        return data


def test_workload_history_shape(tmp_path):
    h = tmp_path / "h.jsonl"
    run_workload(_MemClient(), str(h), ops=20, clients=3, key_space=4, rename_ratio=0.3, seed=7)
    recs = [json.loads(x) for x in h.read_text().splitlines()]
    assert len(recs) == 2 * 20 * 3
    inv = [r for r in recs if r["type"] == "invoke"]
    assert {r["op"] for r in inv} <= {"put", "get", "delete", "rename"}
    assert any(r["op"] == "rename" for r in inv)
    for r in inv:
        for k in ("path", "src", "dst"):
            if k in r:
                assert r[k] in {key_path(i) for i in range(4)}
    puts = [r for r in inv if r["op"] == "put"]
    assert all(len(r["data_hash"]) == 32 for r in puts)
    assert key_path(0).startswith("/a/") and key_path(1).startswith("/z/")


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_workload_on_linearizable_store_checks_clean(tmp_path, seed):
    h = tmp_path / "h.jsonl"
    run_workload(_MemClient(), str(h), ops=40, clients=5, key_space=4, rename_ratio=0.3, seed=seed)
    assert checker.check_file(str(h)) == []


def test_workload_on_stale_cache_store_is_caught(tmp_path):
    found = False
    for seed in range(10):
        h = tmp_path / f"h{seed}.jsonl"
        run_workload(_StaleCacheClient(), str(h), ops=60, clients=4, key_space=2, rename_ratio=0.2, seed=seed)
        if checker.check_file(str(h)):
            found = True
            break
    assert found, "a store serving stale reads must produce a non-linearizable history"


def test_put_hash_matches_payload(tmp_path):
    c = _MemClient()
    h = tmp_path / "h.jsonl"
    run_workload(c, str(h), ops=30, clients=1, key_space=3, rename_ratio=0.0, seed=5)
    recs = [json.loads(x) for x in h.read_text().splitlines()]
    hashes = {r["data_hash"] for r in recs if r.get("op") == "put" and r["type"] == "invoke"}
    for data in c.files.values():
        assert hashlib.md5(data).hexdigest() in hashes
