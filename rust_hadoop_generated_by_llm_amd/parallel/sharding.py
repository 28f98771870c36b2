"""Namespace sharding (P1/P2): the ShardMap shared by clients, masters, chunkservers and the
config server. Routing must agree bit-for-bit with the reference because clients and
servers compute it independently (reference: dfs/common/src/sharding.rs:17-341).

Two strategies:
* ConsistentHash — CRC32("{shard}:{i}") for ``virtual_nodes`` vnodes on a ring; a key maps
  to the first vnode >= CRC32(key), wrapping around.
* Range — ``ranges`` maps an inclusive range END key to a shard; a key maps to the first
  end >= key (the reference's ``BTreeMap::range(key..)``). Bootstrap is order dependent:
  first shard ends at U+10FFFF; the second takes everything <= "/m"; later ones get
  ``"z-{id}"`` (sharding.rs:70-112).
"""
from __future__ import annotations

import bisect
import json
import zlib
from typing import Iterable

MAX_KEY = "\U0010FFFF"


def _hash_key(key: str) -> int:
    return zlib.crc32(key.encode())


class ShardMap:
    def __init__(self, strategy: str = "consistent_hash", virtual_nodes: int = 100):
        if strategy not in ("consistent_hash", "range"):
            raise ValueError(strategy)
        self.strategy = strategy
        self.virtual_nodes = virtual_nodes
        self.ring: dict[int, str] = {}
        self.ranges: dict[str, str] = {}
        self.shards: set[str] = set()
        self.shard_peers: dict[str, list[str]] = {}
        self._sorted: list | None = None

    # ------------------------------------------------------------------ constructors
    @classmethod
    def new_consistent_hash(cls, virtual_nodes: int = 100) -> "ShardMap":
        return cls("consistent_hash", virtual_nodes)

    @classmethod
    def new_range(cls) -> "ShardMap":
        return cls("range")

    @classmethod
    def from_config(cls, shards: dict[str, list[str]], ranges: dict[str, str] | None = None) -> "ShardMap":
        """Shard JSON config ``{"shards": {id: [peers]}}``: sorted ids added to a Range map
        (reference ShardConfig::to_shard_map, sharding.rs:288-296). Extension: an optional
        ``"ranges": {end_key: shard_id}`` gives explicit boundaries instead of the
        order-dependent bootstrap (used to give each writer prefix its own shard)."""
        m = cls.new_range()
        for sid in sorted(shards):
            m.add_shard(sid, list(shards[sid]))
        if ranges:
            m.ranges = {k: v for k, v in ranges.items() if v in m.shards}
            m._dirty()
        return m

    @classmethod
    def load_config_file(cls, path: str | None, virtual_nodes: int = 100) -> "ShardMap":
        if path:
            try:
                with open(path) as f:
                    cfg = json.load(f)
                return cls.from_config(cfg["shards"], cfg.get("ranges"))
            except (OSError, ValueError, KeyError):
                pass
        return cls.new_consistent_hash(virtual_nodes)

    # ------------------------------------------------------------------ mutation
    def _dirty(self) -> None:
        self._sorted = None

    def add_shard(self, shard_id: str, peers: list[str]) -> None:
        if shard_id in self.shards:
            self.shard_peers[shard_id] = list(peers)
            return
        self.shards.add(shard_id)
        self.shard_peers[shard_id] = list(peers)
        if self.strategy == "consistent_hash":
            for i in range(self.virtual_nodes):
                self.ring[_hash_key(f"{shard_id}:{i}")] = shard_id
        else:
            if not self.ranges:
                self.ranges[MAX_KEY] = shard_id
            elif len(self.ranges) == 1:
                old = next(iter(self.ranges.values()))
                self.ranges.clear()
                self.ranges["/m"] = shard_id
                self.ranges[MAX_KEY] = old
            else:
                self.ranges[f"z-{shard_id}"] = shard_id
        self._dirty()

    def remove_shard(self, shard_id: str) -> None:
        if shard_id not in self.shards:
            return
        self.shards.discard(shard_id)
        self.shard_peers.pop(shard_id, None)
        if self.strategy == "consistent_hash":
            self.ring = {h: s for h, s in self.ring.items() if s != shard_id}
        else:
            self.ranges = {k: s for k, s in self.ranges.items() if s != shard_id}
        self._dirty()

    def split_shard(self, split_key: str, new_shard_id: str, peers: list[str]) -> bool:
        if self.strategy != "range" or new_shard_id in self.shards or split_key in self.ranges:
            return False
        ends = sorted(self.ranges)
        i = bisect.bisect_left(ends, split_key)
        if i >= len(ends):
            return False
        self.ranges[split_key] = new_shard_id
        self.shards.add(new_shard_id)
        self.shard_peers[new_shard_id] = list(peers)
        self._dirty()
        return True

    def merge_shards(self, victim: str, retained: str) -> bool:
        if self.strategy != "range" or victim not in self.shards or retained not in self.shards:
            return False
        vk = next((k for k in sorted(self.ranges) if self.ranges[k] == victim), None)
        if vk is None:
            return False
        del self.ranges[vk]
        if vk == MAX_KEY:
            rk = next((k for k in sorted(self.ranges) if self.ranges[k] == retained), None)
            if rk is not None:
                del self.ranges[rk]
            self.ranges[MAX_KEY] = retained
        self.shards.discard(victim)
        self.shard_peers.pop(victim, None)
        self._dirty()
        return True

    def rebalance_boundary(self, old_key: str, new_key: str) -> bool:
        if self.strategy != "range" or old_key not in self.ranges:
            return False
        self.ranges[new_key] = self.ranges.pop(old_key)
        self._dirty()
        return True

    # ------------------------------------------------------------------ queries
    def get_shard(self, key: str) -> str | None:
        if self._sorted is None:
            self._sorted = sorted(self.ring) if self.strategy == "consistent_hash" else sorted(self.ranges)
        keys = self._sorted
        if not keys:
            return None
        if self.strategy == "consistent_hash":
            i = bisect.bisect_left(keys, _hash_key(key))
            return self.ring[keys[i if i < len(keys) else 0]]
        i = bisect.bisect_left(keys, key)
        return self.ranges[keys[i]] if i < len(keys) else None

    def has_shard(self, shard_id: str) -> bool:
        return shard_id in self.shards

    def get_shard_peers(self, shard_id: str) -> list[str] | None:
        p = self.shard_peers.get(shard_id)
        return list(p) if p is not None else None

    get_peers = get_shard_peers

    def get_all_shards(self) -> list[str]:
        return sorted(self.shards)

    def get_all_masters(self) -> list[str]:
        out: set[str] = set()
        for peers in self.shard_peers.values():
            out.update(peers)
        return sorted(out)

    def get_neighbors(self, shard_id: str) -> tuple[str | None, str | None]:
        if self.strategy != "range":
            return None, None
        order = [self.ranges[k] for k in sorted(self.ranges)]
        for i, s in enumerate(order):
            if s == shard_id:
                return (order[i - 1] if i > 0 else None, order[i + 1] if i + 1 < len(order) else None)
        return None, None

    def range_end_of(self, shard_id: str) -> str | None:
        for k in sorted(self.ranges):
            if self.ranges[k] == shard_id:
                return k
        return None

    # ------------------------------------------------------------------ serde
    def to_json(self) -> dict:
        """serde layout of the reference (snapshot compatibility)."""
        if self.strategy == "consistent_hash":
            strat = {"ConsistentHash": {"ring": {str(k): v for k, v in sorted(self.ring.items())},
                                        "virtual_nodes": self.virtual_nodes}}
        else:
            strat = {"Range": {"ranges": dict(sorted(self.ranges.items()))}}
        return {"strategy": strat, "shards": sorted(self.shards), "shard_peers": self.shard_peers}

    @classmethod
    def from_json(cls, d: dict) -> "ShardMap":
        strat = d.get("strategy", {})
        if "Range" in strat:
            m = cls.new_range()
            m.ranges = dict(strat["Range"].get("ranges", {}))
        else:
            ch = strat.get("ConsistentHash", {})
            m = cls.new_consistent_hash(int(ch.get("virtual_nodes", 100)))
            m.ring = {int(k): v for k, v in ch.get("ring", {}).items()}
        m.shards = set(d.get("shards", []))
        m.shard_peers = {k: list(v) for k, v in d.get("shard_peers", {}).items()}
        return m

    @classmethod
    def from_peers(cls, shards: dict[str, Iterable[str]]) -> "ShardMap":
        """Range map rebuilt from a FetchShardMap response (ids sorted; the reference does
        the same because split keys are not transported, config_server.rs:43-61)."""
        return cls.from_config({k: list(v) for k, v in shards.items()})

    @classmethod
    def from_fetch(cls, resp) -> "ShardMap":
        """FetchShardMapResponse -> map. With the ``ranges`` extension the boundaries are
        exact (dynamic split keys included); without it, the reference's id-sorted rebuild."""
        return cls.from_config({k: list(v.peers) for k, v in resp.shards.items()}, dict(resp.ranges) or None)

    def copy(self) -> "ShardMap":
        return ShardMap.from_json(json.loads(json.dumps(self.to_json())))

    def __repr__(self) -> str:
        return f"ShardMap({self.strategy}, shards={sorted(self.shards)})"
