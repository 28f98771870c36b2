"""The config server's state machine as tests drive it: a facade over the native
csrc/config_core.cpp (the state the native `dfs_config_server` executable applies on its Raft
node; reference dfs/metaserver/src/config_server.rs)."""
from __future__ import annotations

import json

from rust_hadoop_generated_by_llm_amd.native import lib as _native
from rust_hadoop_generated_by_llm_amd.parallel.sharding import ShardMap


class ConfigState:
    """Facade over the native state machine (csrc/config_core.cpp), which the native Raft
    node applies on its own thread; views are re-parsed only when the state changed."""

    def __init__(self):
        self.core = _native.ConfigCore()
        self._map: tuple[int, ShardMap | None] = (-1, None)

    @property
    def shard_map(self) -> ShardMap:
        v = self.core.version
        if self._map[0] != v or self._map[1] is None:
            self._map = (v, ShardMap.from_json(json.loads(self.core.shard_map_json())))
        return self._map[1]

    @property
    def masters(self) -> dict[str, dict]:
        return json.loads(self.core.masters_json())

    def apply(self, command, index: int = 0):
        r = self.core.apply(index, json.dumps(command))
        if r.startswith("!"):
            raise ValueError(r[1:])
        return json.loads(r)

    def snapshot(self) -> dict:
        return json.loads(self.core.snapshot())

    def restore(self, state: dict) -> None:
        self.core.restore(json.dumps(state))
