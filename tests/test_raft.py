"""Raft on the in-process transport with a fault injector (reference tier-2 tests:
network_partition_tests.rs, raft_logic_tests.rs, membership_change_unit_tests.rs —
here the REAL node runs, not a simulation)."""
import asyncio

import pytest

from .harness.raft_membership import CatchUpProgress, ClusterConfiguration, initial_members
from .harness.raft_node import LEADER, NotLeader, RaftNode
from .harness.raft_transport import FaultInjector, LocalTransport


class KV:
    def __init__(self):
        self.d = {}
        self.applied = []

    def apply(self, cmd, idx):
        self.applied.append(idx)
        k, v = cmd["set"]
        self.d[k] = v
        return v

    def snapshot(self):
        return {"d": self.d}

    def restore(self, s):
        self.d = dict(s["d"])


class Cluster:
    def __init__(self, tmp, n=3, threshold=10000):
        self.tmp = tmp
        self.registry = {}
        self.faults = FaultInjector()
        self.addrs = {i: f"node{i}" for i in range(1, n + 1)}
        self.nodes = {}
        self.threshold = threshold
        for i in self.addrs:
            self.make(i)

    def make(self, i, members=None):
        sm = KV()
        node = RaftNode(i, members or dict(self.addrs), f"client{i}", str(self.tmp / f"n{i}"), sm,
                        LocalTransport(self.addrs.get(i, f"node{i}"), self.registry, self.faults),
                        election_timeout=(0.15, 0.3), heartbeat_interval=0.03, sync=False,
                        snapshot_threshold=self.threshold)
        self.registry[f"node{i}"] = node.handle
        self.nodes[i] = node
        return node

    async def start(self):
        for n in self.nodes.values():
            await n.start()

    async def stop(self):
        for n in self.nodes.values():
            await n.stop()

    async def leader(self, timeout=5.0, exclude=()):
        loop = asyncio.get_running_loop()
        end = loop.time() + timeout
        while loop.time() < end:
            ls = [n for i, n in self.nodes.items() if n.role == LEADER and i not in exclude and n._running]
            if len(ls) == 1:
                return ls[0]
            await asyncio.sleep(0.02)
        raise AssertionError("no unique leader")


def run(coro):
    return asyncio.run(asyncio.wait_for(coro, 60))


def test_membership_math():
    c = ClusterConfiguration({1: "a", 2: "b", 3: "c"})
    assert c.has_joint_majority({1, 2}) and not c.has_joint_majority({1})
    j = ClusterConfiguration({3: "c", 4: "d", 5: "e"}, {1: "a", 2: "b", 3: "c"}, 2)
    assert not j.has_joint_majority({1, 2})          # old majority only
    assert j.has_joint_majority({1, 3, 4})
    assert ClusterConfiguration.from_json(j.to_json()) == j
    p = CatchUpProgress()
    for i in range(10):
        p.update(i + 1)
    assert p.is_caught_up(10) and not p.is_caught_up(11)
    assert initial_members(1, "h1", ["2@h2", "http://x-metaserver-2:80"]) == {1: "h1", 2: "h2", 3: "http://x-metaserver-2:80"}


def test_single_node_commits_immediately(tmp_path):
    async def go():
        sm = KV()
        n = RaftNode(1, {1: "solo"}, "c", str(tmp_path), sm, LocalTransport("solo", {}), sync=False)
        await n.start()
        assert n.role == LEADER
        assert await n.propose({"set": ["a", 1]}) == 1
        await n.read_index()
        await n.stop()
        # restart: state rebuilt from the WAL
        sm2 = KV()
        n2 = RaftNode(1, {1: "solo"}, "c", str(tmp_path), sm2, LocalTransport("solo", {}), sync=False)
        await n2.start()
        await n2.propose({"set": ["b", 2]})
        assert sm2.d == {"a": 1, "b": 2}
        await n2.stop()

    run(go())


def test_election_replication_and_failover(tmp_path):
    async def go():
        c = Cluster(tmp_path)
        await c.start()
        l1 = await c.leader()
        for i in range(20):
            await l1.propose({"set": [f"k{i}", i]})
        await asyncio.sleep(0.3)
        for n in c.nodes.values():
            assert n.sm.d == {f"k{i}": i for i in range(20)}
        follower = next(n for n in c.nodes.values() if n is not l1)
        with pytest.raises(NotLeader):
            await follower.propose({"set": ["x", 0]})
        # isolate the leader: the majority elects a new one with a higher term
        c.faults.isolate(f"node{l1.id}", list(c.registry))
        l2 = await c.leader(exclude=(l1.id,))
        assert l2.current_term > l1.current_term or l2.id != l1.id
        await l2.propose({"set": ["after", 1]})
        # the old leader cannot commit in the minority
        with pytest.raises((NotLeader, asyncio.TimeoutError)):
            await asyncio.wait_for(l1.propose({"set": ["lost", 1]}), 0.5)
        c.faults.heal()
        await asyncio.sleep(1.0)
        for n in c.nodes.values():
            assert n.sm.d.get("after") == 1 and "lost" not in n.sm.d
        await c.stop()

    run(go())


def test_read_index_requires_majority(tmp_path):
    async def go():
        c = Cluster(tmp_path)
        await c.start()
        l = await c.leader()
        await l.propose({"set": ["a", 1]})
        await asyncio.wait_for(l.read_index(), 2)
        c.faults.isolate(f"node{l.id}", list(c.registry))
        with pytest.raises((NotLeader, asyncio.TimeoutError)):
            await asyncio.wait_for(l.read_index(), 0.5)
        c.faults.heal()
        await c.stop()

    run(go())


def test_snapshot_and_install_snapshot(tmp_path):
    async def go():
        c = Cluster(tmp_path, threshold=20)
        await c.start()
        l = await c.leader()
        lag = next(n for n in c.nodes.values() if n is not l)
        c.faults.isolate(f"node{lag.id}", list(c.registry))
        for i in range(60):
            await l.propose({"set": [f"k{i}", i]})
        await asyncio.sleep(0.3)
        # every member that could lead after the heal has compacted past the laggard's log,
        # so whoever leads must catch it up with InstallSnapshot
        for n in c.nodes.values():
            if n is not lag:
                await n.snapshot_now()
                assert n.last_included_index > 0
        c.faults.heal()
        for _ in range(100):
            if lag.sm.d.get("k59") == 59:
                break
            await asyncio.sleep(0.05)
        assert lag.sm.d == l.sm.d
        assert lag.last_included_index > 0  # caught up through InstallSnapshot
        await c.stop()

    run(go())


def test_add_and_remove_server(tmp_path):
    async def go():
        c = Cluster(tmp_path, n=3)
        await c.start()
        l = await c.leader()
        await l.propose({"set": ["a", 1]})
        c.addrs[4] = "node4"
        new = c.make(4, members={4: "node4"})
        await new.start()
        await l.add_server(4, "node4")
        for _ in range(100):
            if new.sm.d.get("a") == 1:
                break
            await asyncio.sleep(0.05)
        assert new.sm.d.get("a") == 1 and 4 in l.config.voters()
        await l.remove_server(4)
        assert 4 not in l.config.voters()
        await c.stop()

    run(go())


def test_joint_consensus_change(tmp_path):
    async def go():
        c = Cluster(tmp_path, n=3)
        await c.start()
        l = await c.leader()
        await l.propose({"set": ["a", 1]})
        c.addrs[4] = "node4"
        n4 = c.make(4, members={4: "node4"})
        await n4.start()
        target = {i: a for i, a in c.addrs.items()}
        await l.change_membership(target, catch_up_timeout=3)
        assert not l.config.joint and set(l.config.voters()) == {1, 2, 3, 4}
        await c.stop()

    run(go())
