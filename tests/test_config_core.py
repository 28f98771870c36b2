"""Native config-server state machine (csrc/config_core.cpp, C36) against an executable
model of the reference's ConfigCommand apply (dfs/metaserver/src/config_server.rs,
simple_raft.rs): random command sequences must give the same results and snapshots."""
import json
import time

from hypothesis import given, settings
from hypothesis import strategies as st

from .harness.config_state import ConfigState
from rust_hadoop_generated_by_llm_amd.native import lib
from rust_hadoop_generated_by_llm_amd.parallel.sharding import ShardMap


class Model:
    """The reference semantics, in plain Python over the Python ShardMap."""

    def __init__(self):
        self.sm = ShardMap.new_range()
        self.masters = {}

    def apply(self, cmd):
        (name, a), = cmd["Config"].items()
        sm = self.sm
        if name == "AddShard":
            sm.add_shard(a["shard_id"], a["peers"])
        elif name == "RemoveShard":
            sm.remove_shard(a["shard_id"])
        elif name == "SplitShard":
            ok = sm.split_shard(a["split_key"], a["new_shard_id"], a["new_shard_peers"])
            if ok:
                for p in a["new_shard_peers"]:
                    if p in self.masters:
                        self.masters[p]["shard_id"] = a["new_shard_id"]
            return ok
        elif name == "MergeShard":
            return sm.merge_shards(a["victim_shard_id"], a["retained_shard_id"])
        elif name == "RebalanceShard":
            return sm.rebalance_boundary(a["old_key"], a["new_key"])
        elif name == "RegisterMaster":
            addr, sid = a["address"], a["shard_id"]
            if not sid:
                owned = next((s for s in sm.get_all_shards() if addr in (sm.get_shard_peers(s) or [])), "")
                self.masters[addr] = {"address": addr, "shard_id": owned, "last_heartbeat": 0, "rps_per_prefix": {}}
                return None
            if not sm.has_shard(sid):
                sm.add_shard(sid, [addr])
            elif addr not in (sm.get_shard_peers(sid) or []):
                sm.add_shard(sid, (sm.get_shard_peers(sid) or []) + [addr])
            self.masters[addr] = {"address": addr, "shard_id": sid, "last_heartbeat": 0, "rps_per_prefix": {}}
        elif name == "ShardHeartbeat":
            if a["address"] in self.masters:
                self.masters[a["address"]]["rps_per_prefix"] = dict(a.get("rps_per_prefix", {}))
        return None

    def snapshot(self):
        return {"Config": {"shard_map": self.sm.to_json(), "masters": self.masters}}


addrs = st.sampled_from(["m1:1", "m2:1", "m3:1", "m4:1"])
sids = st.sampled_from(["shard-0", "shard-1", "shard-2", "shard-3"])
keys = st.sampled_from(["/b", "/f", "/m", "/q", "/t", "/x"])
commands = st.one_of(
    st.builds(lambda s, p: {"AddShard": {"shard_id": s, "peers": p}}, sids, st.lists(addrs, max_size=2)),
    st.builds(lambda s: {"RemoveShard": {"shard_id": s}}, sids),
    st.builds(lambda s, k, n, p: {"SplitShard": {"shard_id": s, "split_key": k, "new_shard_id": n,
                                                 "new_shard_peers": p}}, sids, keys, sids,
              st.lists(addrs, min_size=1, max_size=2)),
    st.builds(lambda v, r: {"MergeShard": {"victim_shard_id": v, "retained_shard_id": r}}, sids, sids),
    st.builds(lambda o, n: {"RebalanceShard": {"old_key": o, "new_key": n}}, keys, keys),
    st.builds(lambda a, s: {"RegisterMaster": {"address": a, "shard_id": s}}, addrs, st.one_of(st.just(""), sids)),
    st.builds(lambda a, r: {"ShardHeartbeat": {"address": a, "rps_per_prefix": {"/x/": r}}}, addrs,
              st.floats(0, 100, allow_nan=False)),
)


def _norm(snap):
    snap = json.loads(json.dumps(snap))
    for m in snap["Config"]["masters"].values():
        m["last_heartbeat"] = 0
    return snap


@settings(max_examples=150, deadline=None)
@given(st.lists(commands, max_size=25))
def test_native_config_core_matches_model(cmds):
    core, model = lib.ConfigCore(), Model()
    for i, c in enumerate(cmds, 1):
        cmd = {"Config": c}
        assert json.loads(core.apply(i, json.dumps(cmd))) == model.apply(cmd), cmd
    assert _norm(json.loads(core.snapshot())) == _norm(model.snapshot())
    again = lib.ConfigCore()
    again.restore(core.snapshot())
    assert again.snapshot() == core.snapshot()


def test_facade_views_follow_the_native_state():
    s = ConfigState()
    v0 = s.core.version
    s.apply({"Config": {"RegisterMaster": {"address": "a:1", "shard_id": "shard-0"}}}, 1)
    s.apply({"Config": {"RegisterMaster": {"address": "b:1", "shard_id": ""}}}, 2)
    assert s.core.version > v0
    assert s.shard_map.get_all_shards() == ["shard-0"]
    assert s.core.split_candidates(3) == ["b:1"]  # standby masters first
    assert s.apply({"Config": {"SplitShard": {"shard_id": "shard-0", "split_key": "/m", "new_shard_id": "shard-1",
                                              "new_shard_peers": ["b:1"]}}}, 3) is True
    assert s.shard_map.get_shard("/apple") == "shard-1" and s.masters["b:1"]["shard_id"] == "shard-1"
    assert abs(s.masters["a:1"]["last_heartbeat"] - time.time()) < 5
    t = ConfigState()
    t.restore(s.snapshot())
    assert t.snapshot() == s.snapshot()


def test_unknown_command_is_an_apply_error():
    s = ConfigState()
    try:
        s.apply({"Config": {"Bogus": {}}}, 1)
    except ValueError as e:
        assert "Bogus" in str(e)
    else:
        raise AssertionError("expected an error")
    assert s.apply("NoOp", 2) is None


def test_native_config_service_over_grpc_and_local_socket(tmp_path):
    """Every ConfigService method answered by ConfigCore on the native HTTP/2 server (a grpcio
    client interoperates) and on the same-host socket; a core without a Raft node answers like
    a follower (success=false + "Not Leader", FetchShardMap FAILED_PRECONDITION)."""
    import asyncio
    import socket

    import grpc
    import pytest

    from rust_hadoop_generated_by_llm_amd.models import proto as pb
    from .harness.raft_node import RaftNode
    from .harness.raft_transport import LocalTransport
    from rust_hadoop_generated_by_llm_amd.utils.localrpc import socket_name
    from rust_hadoop_generated_by_llm_amd.utils.rpc import ChannelPool

    loop = asyncio.new_event_loop()
    s = ConfigState()
    node = RaftNode(1, {1: "solo"}, "http://127.0.0.1:1", str(tmp_path / "raft"), s, LocalTransport("solo", {}),
                    sync=False, native_sm=s.core)
    s.core.attach(node._core)
    loop.run_until_complete(node.start())
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    srv = lib.NativeGrpcConfigServer(s.core, "127.0.0.1", port)
    assert srv.start()[0]
    local = lib.ConfigLocalServer(socket_name(port), s.core)
    assert local.start()[0]
    addr = f"http://127.0.0.1:{port}"
    remote, near = ChannelPool(local=False), ChannelPool()
    try:
        deadline = time.time() + 10
        while not node.is_leader() and time.time() < deadline:
            time.sleep(0.05)
        call = lambda m, r, p=remote: p.call(addr, "ConfigService", m, r)  # noqa: E731
        assert call("RegisterMaster", pb.RegisterMasterRequest(address="m1:1", shard_id="shard-0")).success
        assert call("RegisterMaster", pb.RegisterMasterRequest(address="m2:1", shard_id="")).success
        assert call("AddShard", pb.AddShardRequest(shard_id="shard-9", peers=["m9:1"])).success
        assert call("RemoveShard", pb.RemoveShardRequest(shard_id="shard-9")).success
        sp = call("SplitShard", pb.SplitShardRequest(shard_id="shard-0", split_key="/m", new_shard_id="shard-1"))
        assert sp.success and list(sp.new_shard_peers) == ["m2:1"]  # the standby master
        bad = call("SplitShard", pb.SplitShardRequest(shard_id="shard-0", split_key="/m", new_shard_id="shard-1",
                                                      new_shard_peers=["x:1"]))
        assert not bad.success and bad.error_message == "split rejected by the shard map"
        fm = call("FetchShardMap", pb.FetchShardMapRequest(), near)  # same-host socket
        assert {k: list(v.peers) for k, v in fm.shards.items()} == {"shard-0": ["m1:1"], "shard-1": ["m2:1"]}
        assert fm.ranges["/m"] == "shard-1" and "shard-0" in fm.ranges.values()
        assert call("RebalanceShard", pb.RebalanceShardRequest(old_key="/m", new_key="/n")).success
        assert call("ShardHeartbeat", pb.ShardHeartbeatRequest(address="m1:1", rps_per_prefix={"/a/": 2.5})).success
        deadline = time.time() + 5
        while s.masters["m1:1"]["rps_per_prefix"] != {"/a/": 2.5} and time.time() < deadline:
            time.sleep(0.05)
        assert s.masters["m1:1"]["rps_per_prefix"] == {"/a/": 2.5}
        mg = call("MergeShard", pb.MergeShardRequest(victim_shard_id="shard-1", retained_shard_id="shard-0"))
        assert mg.success and s.shard_map.get_all_shards() == ["shard-0"]
        mg = call("MergeShard", pb.MergeShardRequest(victim_shard_id="shard-7", retained_shard_id="shard-0"))
        assert not mg.success and mg.error_message == "merge rejected: unknown shard"
        assert s.core.requests == 11 and srv.stats()["native_grpc_calls"] == 10 and local.requests == 1
        # follower behaviour: no node attached
        s.core.detach()
        r = call("AddShard", pb.AddShardRequest(shard_id="s", peers=["p:1"]))
        assert not r.success and r.error_message == "Not Leader"
        assert not call("RegisterMaster", pb.RegisterMasterRequest(address="m3:1", shard_id="s")).success
        assert not call("ShardHeartbeat", pb.ShardHeartbeatRequest(address="m1:1")).success
        with pytest.raises(grpc.RpcError) as ei:
            call("FetchShardMap", pb.FetchShardMapRequest())
        assert ei.value.code() == grpc.StatusCode.FAILED_PRECONDITION and "Not Leader" in ei.value.details()
    finally:
        remote.close()
        near.close()
        local.stop()
        srv.stop()
        loop.run_until_complete(node.stop())
        s.core.detach()
        loop.close()
