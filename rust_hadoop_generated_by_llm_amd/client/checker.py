"""Linearizability checker for DFS histories (C49; reference dfs/client/src/checker.rs).

Input: JSONL ``invoke``/``return`` records (``id, client, type, op, path, src, dst,
data_hash, result, ts_ns``); an invoke without a return is a crashed op. The sequential
specification is a map path -> content hash:

* ``put(p, h)``   p absent -> store h, ``put_ok:h``; p present -> fails (CreateFile refuses)
* ``get(p)``      ``get_ok:h`` / ``not_found``
* ``delete(p)``   ``ok`` (p removed) / ``not_found``
* ``rename(s,d)`` s present and d absent -> moved, ``ok``; otherwise it fails

Operations whose outcome is unknown (``error`` results, crashed ops) may or may not have
taken effect. The check is Wing-Gong-Leung search with memoisation, run independently
per connected component of keys (keys linked by renames form one component — the
P-compositionality the reference exploits with its per-key / rename-linked split). A
search budget bounds pathological histories; exceeding it is reported, not silently passed.
"""
from __future__ import annotations

import json
from dataclasses import dataclass

INF = float("inf")


@dataclass
class Operation:
    id: int
    client: str
    op: str
    path: str
    src: str
    dst: str
    data_hash: str
    invoke_ts: int
    return_ts: float  # INF when crashed
    result: str       # "" when crashed

    @property
    def ambiguous(self) -> bool:
        return self.return_ts == INF or self.result in ("error", "")

    def keys(self) -> tuple[str, ...]:
        return (self.src, self.dst) if self.op == "rename" else (self.path,)


class HistoryError(ValueError):
    pass


def parse_history(lines) -> list[Operation]:
    invokes: dict[int, dict] = {}
    ops: dict[int, Operation] = {}
    for no, line in enumerate(lines, 1):
        line = line.strip()
        if not line:
            continue
        try:
            e = json.loads(line)
        except ValueError as ex:
            raise HistoryError(f"line {no}: {ex}") from ex
        t = e.get("type")
        if t == "invoke":
            invokes[e["id"]] = e
        elif t == "return":
            inv = invokes.pop(e["id"], None)
            if inv is None:
                raise HistoryError(f"return without matching invoke for id {e['id']}")
            ops[inv["id"]] = _mk(inv, e.get("ts_ns", 0), e.get("result", ""))
        else:
            raise HistoryError(f"unknown entry type '{t}' at line {no}")
    for i, inv in invokes.items():
        ops[i] = _mk(inv, INF, "")
    return [ops[k] for k in sorted(ops)]


def _mk(inv: dict, ret_ts, result: str) -> Operation:
    op = inv.get("op", "")
    if op not in ("put", "get", "delete", "rename"):
        raise HistoryError(f"unknown op '{op}'")
    return Operation(inv["id"], inv.get("client", ""), op, inv.get("path", ""), inv.get("src", ""),
                     inv.get("dst", ""), inv.get("data_hash", ""), inv.get("ts_ns", 0), ret_ts, result)


def _apply(state: dict, op: Operation):
    """Sequential spec: returns (new_state, expected_result)."""
    if op.op == "put":
        if op.path in state:
            return state, "error"
        s = dict(state)
        s[op.path] = op.data_hash
        return s, f"put_ok:{op.data_hash}"
    if op.op == "get":
        return state, (f"get_ok:{state[op.path]}" if op.path in state else "not_found")
    if op.op == "delete":
        if op.path not in state:
            return state, "not_found"
        s = dict(state)
        del s[op.path]
        return s, "ok"
    # rename
    if op.src not in state or op.dst in state:
        return state, "error"
    s = dict(state)
    s[op.dst] = s.pop(op.src)
    return s, "ok"


def _matches(expected: str, op: Operation) -> bool:
    if op.ambiguous:
        return True
    if op.op == "rename" and op.result == "not_found":
        return expected == "error"
    return expected == op.result


class _Search:
    def __init__(self, ops: list[Operation], budget: int):
        self.ops = ops
        self.budget = budget
        self.steps = 0
        self.seen: set = set()
        self.max_depth = 0
        self.best_prefix: list[int] = []

    def run(self) -> bool:
        return self._go(frozenset(), {}, [])

    def _go(self, done: frozenset, state: dict, order: list[int]) -> bool:
        if len(done) == len(self.ops):
            return True
        self.steps += 1
        if self.steps > self.budget:
            raise TimeoutError
        key = (done, tuple(sorted(state.items())))
        if key in self.seen:
            return False
        self.seen.add(key)
        if len(order) > self.max_depth:
            self.max_depth, self.best_prefix = len(order), list(order)
        pending = [i for i in range(len(self.ops)) if i not in done]
        # an op may be linearized next only if no other pending op returned before it was invoked
        min_ret = min(self.ops[i].return_ts for i in pending)
        for i in pending:
            op = self.ops[i]
            if op.invoke_ts > min_ret:
                continue
            new_state, exp = _apply(state, op)
            if _matches(exp, op) and self._go(done | {i}, new_state, order + [i]):
                return True
            # an op with unknown outcome may also have never taken effect
            if op.ambiguous and self._go(done | {i}, state, order + [i]):
                return True
        return False


def _components(ops: list[Operation]) -> list[list[Operation]]:
    parent: dict[str, str] = {}

    def find(x):
        while parent.setdefault(x, x) != x:
            parent[x] = parent[parent[x]]
            x = parent[x]
        return x

    for op in ops:
        ks = op.keys()
        for k in ks[1:]:
            parent[find(k)] = find(ks[0])
        find(ks[0])
    groups: dict[str, list[Operation]] = {}
    for op in ops:
        groups.setdefault(find(op.keys()[0]), []).append(op)
    return list(groups.values())


def check_linearizability(ops: list[Operation], budget: int = 2_000_000) -> list[str]:
    """Returns a list of violations (empty = linearizable)."""
    violations = []
    for comp in _components(ops):
        comp = sorted(comp, key=lambda o: o.invoke_ts)
        s = _Search(comp, budget)
        try:
            ok = s.run()
        except TimeoutError:
            violations.append(f"search budget exhausted on {len(comp)} ops over keys "
                              f"{sorted({k for o in comp for k in o.keys()})}")
            continue
        if not ok:
            stuck = [comp[i] for i in range(len(comp)) if i not in set(s.best_prefix)]
            first = min(stuck, key=lambda o: o.invoke_ts) if stuck else None
            detail = f"; first unlinearizable op: id={first.id} {first.op} {first.keys()} -> {first.result!r}" \
                if first else ""
            violations.append(f"non-linearizable history over keys {sorted({k for o in comp for k in o.keys()})}"
                              f" ({len(s.best_prefix)}/{len(comp)} ops placed){detail}")
    return violations


def check_file(path: str) -> list[str]:
    with open(path) as f:
        return check_linearizability(parse_history(f))


# ----------------------------------------------------------------------------- self tests
def _h(*recs) -> list[str]:
    return [json.dumps(r) for r in recs]


def _inv(i, op, ts, client="c1", **kw):
    return {"id": i, "client": client, "type": "invoke", "op": op, "ts_ns": ts, **kw}


def _ret(i, result, ts, client="c1"):
    return {"id": i, "client": client, "type": "return", "result": result, "ts_ns": ts}


SELF_TESTS = {
    "sequential_put_get": (True, _h(_inv(1, "put", 1, path="/a", data_hash="h1"), _ret(1, "put_ok:h1", 2),
                                    _inv(2, "get", 3, path="/a"), _ret(2, "get_ok:h1", 4))),
    "stale_read": (False, _h(_inv(1, "put", 1, path="/a", data_hash="h1"), _ret(1, "put_ok:h1", 2),
                             _inv(2, "delete", 3, path="/a"), _ret(2, "ok", 4),
                             _inv(3, "get", 5, path="/a"), _ret(3, "get_ok:h1", 6))),
    "lost_write": (False, _h(_inv(1, "put", 1, path="/a", data_hash="h1"), _ret(1, "put_ok:h1", 2),
                             _inv(2, "get", 3, path="/a"), _ret(2, "not_found", 4))),
    "duplicated_value": (False, _h(_inv(1, "put", 1, path="/a", data_hash="h1"), _ret(1, "put_ok:h1", 2),
                                   _inv(2, "put", 3, path="/a", data_hash="h2"), _ret(2, "put_ok:h2", 4))),
    "concurrent_put_get": (True, _h(_inv(1, "put", 1, path="/a", data_hash="h1"),
                                    _inv(2, "get", 2, path="/a", client="c2"), _ret(2, "get_ok:h1", 3, "c2"),
                                    _ret(1, "put_ok:h1", 4))),
    "rename_moves_value": (True, _h(_inv(1, "put", 1, path="/a", data_hash="h1"), _ret(1, "put_ok:h1", 2),
                                    _inv(2, "rename", 3, src="/a", dst="/z"), _ret(2, "ok", 4),
                                    _inv(3, "get", 5, path="/z"), _ret(3, "get_ok:h1", 6),
                                    _inv(4, "get", 7, path="/a"), _ret(4, "not_found", 8))),
    "rename_lost": (False, _h(_inv(1, "put", 1, path="/a", data_hash="h1"), _ret(1, "put_ok:h1", 2),
                              _inv(2, "rename", 3, src="/a", dst="/z"), _ret(2, "ok", 4),
                              _inv(3, "get", 5, path="/z"), _ret(3, "not_found", 6))),
    "crashed_put_may_apply": (True, _h(_inv(1, "put", 1, path="/a", data_hash="h1"),
                                       _inv(2, "get", 5, path="/a", client="c2"), _ret(2, "get_ok:h1", 6, "c2"))),
    "crashed_put_may_not_apply": (True, _h(_inv(1, "put", 1, path="/a", data_hash="h1"),
                                           _inv(2, "get", 5, path="/a", client="c2"),
                                           _ret(2, "not_found", 6, "c2"))),
    "error_is_ambiguous": (True, _h(_inv(1, "delete", 1, path="/a"), _ret(1, "error", 2),
                                    _inv(2, "get", 3, path="/a"), _ret(2, "not_found", 4))),
}


def run_self_tests() -> list[str]:
    failures = []
    for name, (expect_ok, lines) in SELF_TESTS.items():
        got_ok = not check_linearizability(parse_history(lines))
        if got_ok != expect_ok:
            failures.append(f"{name}: expected {'linearizable' if expect_ok else 'violation'}")
    return failures
