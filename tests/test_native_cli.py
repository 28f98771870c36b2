"""The native dfs_cli (csrc/tools/dfs_cli.cpp, built to build/native/dfs_cli) against live CPU
clusters: the same commands and output as the Python CLI's test (test_cluster.py::
test_cli_commands, reference dfs/client/src/bin/dfs_cli.rs), run as a separate process over
gRPC/TCP, plus a two-shard cluster reached through the config server (shard map fetch, routing,
cross-shard rename, a linearizability workload across both shards) and the tooling commands
(shuffle, presign, workload, check-history, cluster add/remove-server in test_membership.py)."""
import json
import os
import subprocess
from pathlib import Path

import pytest

from rust_hadoop_generated_by_llm_amd.cluster.launcher import LocalCluster

pytestmark = pytest.mark.slow

ROOT = Path(__file__).resolve().parents[1]
CLI = ROOT / "build" / "native" / "dfs_cli"

if not CLI.exists():
    pytest.skip("build/native/dfs_cli not built (python3 build_native.py)", allow_module_level=True)


def run(*args, env=None, timeout=120):
    e = dict(os.environ)
    e.update(env or {})
    p = subprocess.run([str(CLI), *args], capture_output=True, text=True, timeout=timeout, env=e)
    return p.returncode, p.stdout, p.stderr


@pytest.fixture(scope="module")
def cluster3():
    with LocalCluster(n_chunkservers=3, fsync=False) as c:
        yield c


def test_native_cli_commands(cluster3, tmp_path):
    m = ["-m", cluster3.master_addrs[0]]
    src = tmp_path / "in.bin"
    data = os.urandom(200_000)
    src.write_bytes(data)
    rc, out, err = run(*m, "put", str(src), "/ncli/file.bin")
    assert rc == 0 and "uploaded successfully with replication" in out, err
    rc, out, _ = run(*m, "ls")
    assert rc == 0 and "/ncli/file.bin" in out.split()
    rc, out, _ = run(*m, "inspect", "/ncli/file.bin")
    assert rc == 0 and "Size: 200000 bytes" in out and "Storage: Replicated" in out and "Locations=" in out
    dst = tmp_path / "out.bin"
    rc, out, err = run(*m, "get", "/ncli/file.bin", str(dst))
    assert rc == 0 and "downloaded successfully" in out, err
    assert dst.read_bytes() == data
    rc, out, _ = run(*m, "rename", "/ncli/file.bin", "/ncli/renamed.bin")
    assert rc == 0 and "renamed successfully" in out
    rc, out, _ = run(*m, "inspect", "/ncli/file.bin")
    assert "File not found" in out
    rc, out, _ = run(*m, "delete", "/ncli/renamed.bin")
    assert rc == 0 and "File deleted" in out
    rc, _, err = run(*m, "delete", "/ncli/renamed.bin")
    assert rc == 1 and "Failed to delete file" in err
    # EC upload: RS encode on this host's CPU, k + m shard writes in parallel
    rc, out, err = run(*m, "put", str(src), "/ncli/ec.bin", "--ec-data", "2", "--ec-parity", "1")
    assert rc == 0 and "EC RS(2,1)" in out, err
    rc, out, _ = run(*m, "inspect", "/ncli/ec.bin")
    assert "Storage: EC RS(2,1)" in out and "Shards=" in out
    assert run(*m, "get", "/ncli/ec.bin", str(dst))[0] == 0 and dst.read_bytes() == data
    # admin
    rc, out, _ = run(*m, "safe-mode", "get")
    assert rc == 0 and "Active: false" in out and "ChunkServers: 3" in out
    rc, out, _ = run(*m, "cluster", "info")
    assert rc == 0 and "Role: Leader" in out and "Members (1)" in out
    # benchmarks
    rc, out, err = run(*m, "benchmark", "write", "-c", "12", "-s", "65536", "-n", "4", "-p", "/nbw", "--json")
    w = json.loads(out.strip().splitlines()[-1])
    assert rc == 0 and w["name"] == "Write" and w["ops"] == 12 and w["errors"] == 0 and w["p50_ms"] > 0, err
    rc, out, _ = run(*m, "benchmark", "read", "-p", "/nbw", "-n", "4", "--json")
    r = json.loads(out.strip().splitlines()[-1])
    assert rc == 0 and r["ops"] == 12 and r["bytes"] == 12 * 65536
    rc, out, _ = run(*m, "benchmark", "write", "-c", "3", "-s", "4096", "-n", "2", "-p", "/nbt")
    assert rc == 0 and "Write Benchmark Results" in out and "P50:" in out and "Throughput:" in out
    rc, out, _ = run(*m, "benchmark", "stress-write", "-d", "1", "-s", "4096", "-n", "2", "-p", "/nbs", "--json")
    s = json.loads(out.strip().splitlines()[-1])
    assert rc == 0 and s["ops"] > 0 and s["errors"] == 0
    rc, out, _ = run(*m, "benchmark", "read", "-p", "/nothing-here")
    assert rc == 0 and "No files found" in out


NO_PYTHON = {"PATH": "/nonexistent"}  # no python3 to hand anything to: the command ran natively


def test_native_cli_tooling_commands(cluster3, tmp_path):
    """shuffle, presign, check-history and workload run in the executable (reference
    dfs_cli.rs:45-199,471-522), with no Python CLI to fall back to."""
    from rust_hadoop_generated_by_llm_amd.s3.auth import sigv4

    m = ["-m", cluster3.master_addrs[0]]
    rc, out, err = run(*m, "shuffle", "/ncli", env=NO_PYTHON)
    assert rc == 0 and "Triggered background shuffling" in out, err
    rc, out, err = run("check-history", "--self-test", env=NO_PYTHON)
    assert rc == 0 and "self-tests passed" in out, err
    # presign: byte-identical to the Python generator at the same timestamp
    env = dict(NO_PYTHON, AWS_ACCESS_KEY_ID="AK", AWS_SECRET_ACCESS_KEY="SK", AWS_REGION="us-east-1")
    rc, out, err = run("presign", "s3://bucket/dir/obj.txt", "--method", "put", "--expires", "120",
                       "--endpoint", "http://127.0.0.1:9000", env=env)
    assert rc == 0, err
    url = out.strip()
    dt = url.split("X-Amz-Date=")[1].split("&")[0]
    assert url == sigv4.generate_presigned_url("http://127.0.0.1:9000", "bucket", "dir/obj.txt", "PUT", "AK", "SK",
                                               "us-east-1", 120, now=(dt[:8], dt))
    assert run("presign", "s3://bucket/k", "--method", "POST", env=env)[0] == 1
    assert run("presign", "s3://bucket/k", "--expires", "604801", env=env)[0] == 1
    assert run("presign", "s3://b/k", env=NO_PYTHON)[0] == 1  # no credentials
    # workload -> history -> checker, all native; the Python checker agrees
    hist = tmp_path / "hist.jsonl"
    rc, out, err = run(*m, "workload", "--ops", "15", "--clients", "3", "--key-space", "3", "--rename-ratio", "0.3",
                       "--history", str(hist), env=NO_PYTHON)
    assert rc == 0 and "Workload completed" in out, err
    rc, out, err = run("check-history", str(hist), env=NO_PYTHON)
    assert rc == 0 and "Parsed 45 operations" in out and "PASSED" in out, (out, err)
    from rust_hadoop_generated_by_llm_amd.client import checker

    with open(hist) as f:
        assert checker.check_linearizability(checker.parse_history(f)) == []
    # a history with a stale read fails, naming the operation
    bad = tmp_path / "bad.jsonl"
    bad.write_text("\n".join(json.dumps(r) for r in [
        {"id": 1, "client": "c", "type": "invoke", "op": "put", "path": "/a", "data_hash": "h1", "ts_ns": 1},
        {"id": 1, "client": "c", "type": "return", "result": "put_ok:h1", "ts_ns": 2},
        {"id": 2, "client": "c", "type": "invoke", "op": "delete", "path": "/a", "ts_ns": 3},
        {"id": 2, "client": "c", "type": "return", "result": "ok", "ts_ns": 4},
        {"id": 3, "client": "c", "type": "invoke", "op": "get", "path": "/a", "ts_ns": 5},
        {"id": 3, "client": "c", "type": "return", "result": "get_ok:h1", "ts_ns": 6}]) + "\n")
    rc, out, err = run("check-history", str(bad), env=NO_PYTHON)
    assert rc == 1 and "non-linearizable history over keys ['/a']" in err and "id=3 get" in err, err
    # DFS_CLI_PYTHON forces the Python implementation of a native command (same output)
    rc, out, _ = run(*m, "ls", env={"DFS_CLI_PYTHON": "1"})
    assert rc == 0


def test_native_cli_routes_through_the_config_server(tmp_path):
    with LocalCluster(n_chunkservers=3, shards=2, fsync=False) as cl:
        g = ["-m", cl.master_addrs[0], "--config-servers", ",".join(cl.config_addrs)]
        src = tmp_path / "x.bin"
        src.write_bytes(b"moving")
        for p in ("/a/src", "/z/taken"):
            rc, out, err = run(*g, "put", str(src), p)
            assert rc == 0, err
        c = cl.client()
        assert c.shard_map.get_shard("/a/src") != c.shard_map.get_shard("/z/taken")
        assert c.get_file_content("/a/src") == b"moving"
        rc, out, err = run(*g, "rename", "/a/src", "/z/dst")
        assert rc == 0 and "renamed successfully" in out, err
        assert c.get_file_content("/z/dst") == b"moving" and not c.exists("/a/src")
        rc, out, _ = run(*g, "ls")
        assert rc == 0 and {"/z/dst", "/z/taken"} <= set(out.split())
        dst = tmp_path / "y.bin"
        assert run(*g, "get", "/z/dst", str(dst))[0] == 0 and dst.read_bytes() == b"moving"
        rc, _, err = run(*g, "rename", "/z/dst", "/z/taken")
        assert rc == 1 and "Rename failed" in err
        # a workload whose renames cross the shards, checked natively
        hist = tmp_path / "x.jsonl"
        rc, out, err = run(*g, "workload", "--ops", "20", "--clients", "3", "--key-space", "4", "--rename-ratio", "0.4",
                           "--history", str(hist), env=NO_PYTHON)
        assert rc == 0, err
        rc, out, err = run("check-history", str(hist), env=NO_PYTHON)
        assert rc == 0 and "PASSED" in out, (out, err)
        c.close()
