"""Disaster recovery from an off-box snapshot backup (the reference's
backup is upload-only, simple_raft.rs:1214-1271; the recommended fix is a restore path).

A leader with `--backup-s3-endpoint` PUTs each snapshot to
`{endpoint}/{bucket}/master-snapshots/node-{id}/...`; `dfs_master --restore-snapshot FILE|URL`
seeds an empty storage directory with such an object and starts with the members of its
own command line (csrc/raft.cpp restore_snapshot_dir)."""
import json
import os
import subprocess
import threading
import time
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from pathlib import Path

import pytest

from rust_hadoop_generated_by_llm_amd.cluster.launcher import free_port
from rust_hadoop_generated_by_llm_amd.models import proto as pb
from rust_hadoop_generated_by_llm_amd.native import lib as native
from rust_hadoop_generated_by_llm_amd.utils.rpc import ChannelPool

ROOT = Path(__file__).resolve().parents[1]
MASTER = ROOT / "build" / "native" / "dfs_master"


class Host:
    restored = None

    def apply_batch(self, items):
        return ["null"] * len(items)

    def snapshot(self):
        return "{}"

    def restore(self, text):
        self.restored = text

    def send(self, addr, kind, body):
        return None

    def backup(self, url, data):
        pass


def test_restore_seeds_an_empty_node_with_the_backup(tmp_path):
    state = {"files": {"/a": {"size": 3}}, "n": 1}
    payload = json.dumps({"meta": [42, 7], "state": state, "config": {"members": {"9": "elsewhere"}}})
    ok, err = native.raft_restore_snapshot_dir(str(tmp_path / "n1"), payload)
    assert ok, err
    host = Host()
    node = native.RaftNode(1, {1: "here"}, "client-a", str(tmp_path / "n1"), host, sync=False)
    assert json.loads(host.restored) == state
    assert node.last_included_index == 42 and node.commit_index == 42
    assert node.term == 7  # entries appended after the snapshot keep non-decreasing terms
    members = json.loads(node.config_json)
    assert "elsewhere" not in json.dumps(members) and "here" in json.dumps(members)  # our --peers, not the backup's
    del node
    # a directory that already holds state is never overwritten
    ok, err = native.raft_restore_snapshot_dir(str(tmp_path / "n1"), payload)
    assert not ok and "already holds" in err
    # what is not a snapshot backup is refused
    for bad in ("not json", json.dumps({"meta": [1], "state": {}}), json.dumps({"meta": [1, 2], "state": 3})):
        ok, err = native.raft_restore_snapshot_dir(str(tmp_path / "fresh"), bad)
        assert not ok and err


class _Backups(BaseHTTPRequestHandler):
    got: list = []

    def do_PUT(self):  # noqa: N802 (http.server API)
        body = self.rfile.read(int(self.headers.get("Content-Length", 0)))
        _Backups.got.append((self.path, body))
        self.send_response(200)
        self.send_header("Content-Length", "0")
        self.end_headers()

    def do_GET(self):  # noqa: N802
        for path, body in reversed(_Backups.got):
            if path == self.path:
                self.send_response(200)
                self.send_header("Content-Length", str(len(body)))
                self.end_headers()
                self.wfile.write(body)
                return
        self.send_response(404)
        self.send_header("Content-Length", "0")
        self.end_headers()

    def log_message(self, *a):
        pass


def _start_master(tmp_path, name, extra):
    port, http = free_port(), free_port()
    log = open(tmp_path / f"{name}.log", "w")
    p = subprocess.Popen([str(MASTER), "--addr", f"127.0.0.1:{port}", "--id", "1", "--http-port", str(http),
                          "--storage-dir", str(tmp_path / name), "--no-fsync", "--fast-intervals", *extra],
                         stdout=log, stderr=subprocess.STDOUT)
    return p, f"127.0.0.1:{port}"


def _wait_leader(pool, addr, deadline=30):
    t0 = time.time()
    while time.time() - t0 < deadline:
        try:
            info = pool.call(addr, "MasterService", "GetClusterInfo", pb.GetClusterInfoRequest(), timeout=2)
            if info.role == "Leader":
                # no chunkservers here: leave safe mode by hand (the admin command)
                r = pool.call(addr, "MasterService", "SetSafeMode", pb.SetSafeModeRequest(enter=False), timeout=5)
                assert r.success, r
                return
        except Exception:  # noqa: BLE001 (starting up)
            pass
        time.sleep(0.2)
    raise AssertionError(f"{addr} never led")


@pytest.mark.skipif(not MASTER.exists(), reason="native executables not built")
def test_master_restores_from_its_snapshot_backup(tmp_path):
    _Backups.got = []
    srv = ThreadingHTTPServer(("127.0.0.1", 0), _Backups)
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    endpoint = f"http://127.0.0.1:{srv.server_address[1]}"
    pool = ChannelPool(local=False)
    procs = []
    try:
        p, addr = _start_master(tmp_path, "old", ["--backup-s3-endpoint", endpoint, "--backup-bucket", "bk",
                                                  "--snapshot-threshold", "5"])
        procs.append(p)
        _wait_leader(pool, addr)
        names = [f"/restore/f{i}" for i in range(12)]
        for nm in names:  # empty files, created and completed (pending files are not listed)
            r = pool.call(addr, "MasterService", "CreateFile", pb.CreateFileRequest(path=nm), timeout=5)
            assert r.success, r
            r = pool.call(addr, "MasterService", "CompleteFile", pb.CompleteFileRequest(path=nm, size=0), timeout=5)
            assert r.success, r
        # snapshots (and their backups) follow the log every few entries; take the newest
        deadline = time.time() + 30
        while time.time() < deadline and not any(b"/restore/f5\"" in body for _p, body in _Backups.got):
            time.sleep(0.2)
        path, body = _Backups.got[-1]
        assert path.startswith("/bk/master-snapshots/node-1/") and "--idx" in path, path
        master_state = json.loads(body)["state"]["Master"]
        backed_up = set(master_state["files"]) - set(master_state.get("under_construction") or {})
        assert len(backed_up & set(names)) >= 5, (path, body[:300])
        p.terminate()
        p.wait(timeout=30)
        # a new master, a new empty directory: seeded from the backup object by URL
        p2, addr2 = _start_master(tmp_path, "new", ["--restore-snapshot", endpoint + path])
        procs.append(p2)
        _wait_leader(pool, addr2)
        listed = pool.call(addr2, "MasterService", "ListFiles", pb.ListFilesRequest(path="/restore"), timeout=5)
        assert backed_up <= set(listed.files), (sorted(backed_up), list(listed.files))
        # and it keeps working: new entries on top of the restored state
        r = pool.call(addr2, "MasterService", "CreateFile", pb.CreateFileRequest(path="/restore/after"), timeout=5)
        assert r.success, r
        # restoring over a directory that now holds state is refused
        p2.terminate()
        p2.wait(timeout=30)
        file_copy = tmp_path / "backup.bin"
        file_copy.write_bytes(body)
        r = subprocess.run([str(MASTER), "--addr", f"127.0.0.1:{free_port()}", "--http-port", str(free_port()),
                            "--storage-dir", str(tmp_path / "new"), "--no-fsync", "--restore-snapshot",
                            str(file_copy)], capture_output=True, text=True, timeout=30)
        assert r.returncode == 2 and "already holds" in r.stderr, r.stderr
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait(timeout=10)
        pool.close()
        srv.shutdown()
    assert not os.environ.get("DFS_TEST_KEEP")
