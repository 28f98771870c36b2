"""Raft cluster configuration: simple and joint (C_old,new) configurations, plus the
non-voting catch-up tracker used before a server becomes a voter
(reference: dfs/metaserver/src/simple_raft.rs:70-252)."""
from __future__ import annotations

import re
from dataclasses import dataclass, field


@dataclass
class ClusterConfiguration:
    members: dict[int, str] = field(default_factory=dict)        # Simple, or C_new when joint
    old_members: dict[int, str] | None = None                     # set only in a joint config
    version: int = 0

    @property
    def joint(self) -> bool:
        return self.old_members is not None

    def all_members(self) -> dict[int, str]:
        out = dict(self.old_members or {})
        out.update(self.members)
        return out

    def voters(self) -> set[int]:
        return set(self.all_members())

    def has_joint_majority(self, acks: set[int]) -> bool:
        def maj(group: dict[int, str]) -> bool:
            return sum(1 for i in acks if i in group) > len(group) // 2

        if self.old_members is not None:
            return maj(self.old_members) and maj(self.members)
        return maj(self.members)

    def to_json(self) -> dict:
        if self.old_members is not None:
            return {"Joint": {"old_members": {str(k): v for k, v in self.old_members.items()},
                              "new_members": {str(k): v for k, v in self.members.items()},
                              "version": self.version}}
        return {"Simple": {"members": {str(k): v for k, v in self.members.items()}, "version": self.version}}

    @classmethod
    def from_json(cls, d: dict) -> "ClusterConfiguration":
        if "Joint" in d:
            j = d["Joint"]
            return cls({int(k): v for k, v in j["new_members"].items()},
                       {int(k): v for k, v in j["old_members"].items()}, int(j.get("version", 0)))
        s = d.get("Simple", {})
        return cls({int(k): v for k, v in s.get("members", {}).items()}, None, int(s.get("version", 0)))


@dataclass
class CatchUpProgress:
    match_index: int = 0
    rounds_caught_up: int = 0
    added_at: float = 0.0

    def update(self, new_match: int) -> None:
        if new_match > self.match_index:
            self.match_index = new_match
            self.rounds_caught_up += 1

    def is_caught_up(self, leader_commit: int) -> bool:
        return self.match_index >= leader_commit and self.rounds_caught_up >= 10


_POD = re.compile(r"(?:configserver|metaserver)-(\d+)")


def parse_peer(spec: str) -> tuple[int | None, str]:
    """``"3@http://host:8080"`` -> (3, url); ``...metaserver-N...`` -> (N+1, url) like the
    reference (simple_raft.rs:791-807); otherwise (None, url)."""
    if "@" in spec and spec.split("@", 1)[0].isdigit():
        i, addr = spec.split("@", 1)
        return int(i), addr
    m = _POD.search(spec)
    if m:
        return int(m.group(1)) + 1, spec
    return None, spec


def initial_members(node_id: int, self_addr: str, peers: list[str]) -> dict[int, str]:
    members = {node_id: self_addr}
    unnamed = []
    for p in peers:
        pid, addr = parse_peer(p)
        if pid is None:
            unnamed.append(addr)
        else:
            members[pid] = addr
    # peers without an id: deterministic ids from the sorted address list of the whole group
    if unnamed:
        everyone = sorted(set(unnamed) | {self_addr})
        for addr in unnamed:
            members[everyone.index(addr) + 1] = addr
    return members
