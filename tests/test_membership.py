"""Process-level Raft membership change on a live metadata shard, driven through dfs_cli the
way an operator does it (reference: dynamic_membership_test.sh — start a node with --peers of
the running group, `cluster add-server`, verify it catches up and votes, `remove-server`).

Three master processes form shard-0; a fourth is started pointing at them, added, made part of
the quorum (two originals are removed, so every later commit needs its ack), then removed again,
and the last voter refuses its own removal. The removed processes keep running: pre-vote and
leader stickiness (csrc/raft.cpp on_vote / run_pre_vote) keep them from bumping the term."""
import time
import urllib.request

import pytest

from rust_hadoop_generated_by_llm_amd.cluster.launcher import LocalCluster, free_port
from rust_hadoop_generated_by_llm_amd.models import proto as pb
from rust_hadoop_generated_by_llm_amd.utils.rpc import ChannelPool

pytestmark = pytest.mark.slow


def cli(capsys, *args):
    """The native dfs_cli executable, as an operator runs it (cluster admin is native)."""
    import subprocess
    from pathlib import Path

    exe = Path(__file__).resolve().parents[1] / "build" / "native" / "dfs_cli"
    p = subprocess.run([str(exe), *args], capture_output=True, text=True, timeout=60,
                       env={"PATH": "/nonexistent"})  # no python3 on PATH: nothing is handed over
    return p.returncode, p.stdout + p.stderr


def info(pool, addr):
    return pool.call(addr, "MasterService", "GetClusterInfo", pb.GetClusterInfoRequest(), timeout=5.0)


def find_leader(pool, addrs, timeout=30.0):
    deadline = time.time() + timeout
    while time.time() < deadline:
        for a in addrs:
            try:
                r = info(pool, a)
            except Exception:  # noqa: BLE001 - a node may be down or starting
                continue
            if r.role == "Leader":
                return a, r
        time.sleep(0.1)
    raise AssertionError("no leader")


def wait_for(pred, timeout=30.0, what="condition"):
    deadline = time.time() + timeout
    while time.time() < deadline:
        v = pred()
        if v:
            return v
        time.sleep(0.1)
    raise AssertionError(f"timed out waiting for {what}")


def test_add_and_remove_master_via_cli(capsys):
    with LocalCluster(n_chunkservers=1, masters_per_shard=3, fsync=False) as cl:
        pool = ChannelPool()
        c = cl.client(initial_backoff_ms=100, max_retries=20)
        try:
            c.create_file_from_buffer(b"before", "/m/before")
            originals = list(cl.master_addrs)  # ids 1, 2, 3 in order
            https = [cl.master_http[a] for a in originals]
            leader, linfo = find_leader(pool, originals)
            term0 = linfo.current_term

            # start node 4 with the running group as its peers (it knows them; they do not know it)
            g4, h4 = free_port(), free_port()
            addr4, http4 = f"http://127.0.0.1:{g4}", f"http://127.0.0.1:{h4}"
            peers = ",".join(f"{i + 1}@{h}" for i, h in enumerate(https))
            pr = cl._spawn("master_shard-0_4", "master.server", [
                "--addr", f"127.0.0.1:{g4}", "--id", "4", "--http-port", str(h4), "--storage-dir",
                str(cl.base / "master_shard-0"), "--shard-id", "shard-0", "--no-fsync", "--peers", peers,
                "--shard-config", str(cl.base / "shard_config.json")])
            cl._wait_ready([pr])

            # a follower refuses membership changes and points at the leader
            follower = next(a for a in originals if a != leader)
            rc, out = cli(capsys, "-m", follower, "cluster", "add-server", "4", http4)
            assert rc == 1 and "Not Leader" in out

            rc, out = cli(capsys, "-m", leader, "cluster", "add-server", "4", http4)
            assert rc == 0 and "Added server 4" in out, out
            committed = info(pool, leader).commit_index
            r4 = wait_for(lambda: (lambda r: r if len(r.members) == 4 and r.last_applied >= committed else None)(
                info(pool, addr4)), what="node 4 to catch up")
            assert r4.role == "Follower" and r4.leader_address == leader
            rc, out = cli(capsys, "-m", addr4, "cluster", "info")
            assert rc == 0 and "Members (4)" in out and "[4]" in out and "(self)" in out

            # shrink to {leader, 4}: from here on every commit needs node 4's vote
            removed = [a for a in originals if a != leader]
            for a in removed:
                sid = originals.index(a) + 1
                rc, out = cli(capsys, "-m", leader, "cluster", "remove-server", str(sid))
                assert rc == 0 and f"Removed server {sid}" in out, out
            wait_for(lambda: sorted(m.server_id for m in info(pool, leader).members) ==
                     sorted([originals.index(leader) + 1, 4]), what="two-member config")
            c.create_file_from_buffer(b"after", "/m/after")
            before_apply = info(pool, leader).commit_index
            wait_for(lambda: info(pool, addr4).last_applied >= before_apply, what="node 4 apply")

            # the removed nodes still run; past their election timeouts (1.5-3 s) they have
            # not unseated the leader or raised the term
            time.sleep(4.0)
            li = info(pool, leader)
            assert li.role == "Leader" and li.current_term == term0
            assert c.get_file_content("/m/before") == b"before"
            assert c.get_file_content("/m/after") == b"after"

            # remove node 4 again; the last voter refuses its own removal
            rc, out = cli(capsys, "-m", leader, "cluster", "remove-server", "4")
            assert rc == 0, out
            wait_for(lambda: len(info(pool, leader).members) == 1, what="single-member config")
            rc, out = cli(capsys, "-m", leader, "cluster", "remove-server", str(originals.index(leader) + 1))
            assert rc == 1 and "would leave cluster empty" in out
            # Raft peer RPCs reached node 4 natively (/dfs.RaftPeer/* on its gRPC port)
            text = urllib.request.urlopen(f"{http4}/metrics").read().decode()
            vals = {ln.split()[0]: float(ln.split()[1]) for ln in text.splitlines() if ln and not ln.startswith("#")}
            assert vals["dfs_master_native_raft_rpcs"] > 0
            c.create_file_from_buffer(b"solo", "/m/solo")
            assert c.get_file_content("/m/solo") == b"solo"
        finally:
            c.close()
            pool.close()
