"""Concurrent workload generator recording a JSONL history for the linearizability checker
(C50; reference dfs/client/src/workload.rs). N clients x M ops over a key space of K paths
(``/a/lin_i`` for even i, ``/z/lin_i`` for odd i so renames cross shards); a
``rename_ratio`` share are renames, the rest split evenly over put/get/delete."""
from __future__ import annotations

import hashlib
import itertools
import json
import random
import threading
import time

from .client import Client


def key_path(i: int) -> str:
    return f"/a/lin_{i}" if i % 2 == 0 else f"/z/lin_{i}"


class _Recorder:
    def __init__(self, path: str):
        self.f = open(path, "w")
        self.lock = threading.Lock()
        self.ids = itertools.count()

    def write(self, rec: dict) -> None:
        with self.lock:
            self.f.write(json.dumps(rec) + "\n")
            self.f.flush()

    def close(self) -> None:
        self.f.close()


def _classify(err: Exception) -> str:
    msg = str(err)
    return "not_found" if ("not found" in msg or "Not found" in msg) else "error"


def run_workload(client: Client, history_path: str, ops: int = 50, clients: int = 5, key_space: int = 4,
                 rename_ratio: float = 0.3, seed: int | None = None) -> None:
    rec = _Recorder(history_path)
    rng_master = random.Random(seed)

    def worker(cid: int):
        rng = random.Random(rng_master.random())
        name = f"client_{cid}"
        for _ in range(ops):
            op_id = next(rec.ids)
            r = rng.random()
            base = {"id": op_id, "client": name}
            if r < rename_ratio:
                s, d = rng.sample(range(key_space), 2) if key_space > 1 else (0, 0)
                src, dst = key_path(s), key_path(d)
                rec.write({**base, "type": "invoke", "op": "rename", "src": src, "dst": dst, "ts_ns": time.time_ns()})
                try:
                    client.rename_file(src, dst)
                    res = "ok"
                except Exception as e:  # noqa: BLE001
                    res = _classify(e)
                rec.write({**base, "type": "return", "op": "rename", "result": res, "ts_ns": time.time_ns()})
                continue
            kind = ("put", "get", "delete")[min(2, int((r - rename_ratio) / ((1 - rename_ratio) / 3)))]
            path = key_path(rng.randrange(key_space))
            if kind == "put":
                data = f"data_{op_id}_{time.time_ns()}".encode()
                h = hashlib.md5(data).hexdigest()
                rec.write({**base, "type": "invoke", "op": "put", "path": path, "data_hash": h,
                           "ts_ns": time.time_ns()})
                try:
                    client.create_file_from_buffer(data, path)
                    res = f"put_ok:{h}"
                except Exception:  # noqa: BLE001
                    res = "error"
            elif kind == "get":
                rec.write({**base, "type": "invoke", "op": "get", "path": path, "ts_ns": time.time_ns()})
                try:
                    res = "get_ok:" + hashlib.md5(client.get_file_content(path)).hexdigest()
                except Exception as e:  # noqa: BLE001
                    res = _classify(e)
            else:
                rec.write({**base, "type": "invoke", "op": "delete", "path": path, "ts_ns": time.time_ns()})
                try:
                    client.delete_file(path)
                    res = "ok"
                except Exception as e:  # noqa: BLE001
                    res = _classify(e)
            rec.write({**base, "type": "return", "op": kind, "path": path, "result": res, "ts_ns": time.time_ns()})

    threads = [threading.Thread(target=worker, args=(c,)) for c in range(clients)]
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    rec.close()
