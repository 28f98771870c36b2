"""build/native/audit_reader (csrc/tools/audit_reader.cpp) against the Python reader
(tests/models/s3_audit.py::reader_main, reference dfs/s3_server/src/bin/audit_reader.rs) on the same
segment store: identical output for every filter combination, index lookups with a lagging
index, chain verification with the right and a wrong secret, and tamper detection."""
import json
import subprocess
from datetime import datetime, timedelta, timezone
from pathlib import Path

import pytest

from tests.models.s3_audit import AuditLogger, SegmentStore, make_record, reader_main

ROOT = Path(__file__).resolve().parents[1]
READER = ROOT / "build" / "native" / "audit_reader"

if not READER.exists():
    pytest.skip("build/native/audit_reader not built (python3 build_native.py)", allow_module_level=True)

SECRET = "0123456789abcdef-secret"


def native(*args):
    p = subprocess.run([str(READER), *args], capture_output=True, text=True, timeout=60)
    return p.returncode, p.stdout


def python(capsys, *args):
    rc = reader_main(list(args))
    return rc, capsys.readouterr().out


@pytest.fixture(scope="module")
def logdir(tmp_path_factory):
    d = tmp_path_factory.mktemp("audit")
    lg = AuditLogger(str(d), batch_size=23, hmac_secret=SECRET, flush_interval=0.1)
    base = datetime(2026, 3, 1, 10, 0, tzinfo=timezone.utc)
    users = ["alice", "bob", "Zoë", None, "tab\tuser"]
    for i in range(240):
        now = base + timedelta(minutes=i)  # four hourly segments
        lg.log(make_record(request_id=f"req-{i:04d}", remote_ip="10.0.0.1", user_id=users[i % 5],
                           role_arn=None if i % 3 else "arn:aws:iam::1:role/r", action=["s3:GetObject", "s3:PutObject"][i % 2],
                           resource=f"arn:dfs:s3:::b{i % 3}/k{i}" if i % 7 else f"b{i % 3}",
                           status_code=[200, 403, 404][i % 3], error_code=None if i % 3 == 0 else "AccessDenied",
                           user_agent="agent \"q\" \\ é 𝄞 \x01" if i % 11 == 0 else "aws-cli/2",
                           duration_ms=i, now=now))
    assert lg.flush(10)
    lg.close()
    # a lagging index: drop the last index lines of the last segment (crash between appends)
    seg = SegmentStore(str(d)).segments()[-1][0]
    for ext in (".uidx", ".ridx"):
        p = d / f"seg-{seg}{ext}"
        lines = p.read_text().splitlines(keepends=True)
        p.write_text("".join(lines[:-7]))
    return d


CASES = [
    [],
    ["--json"],
    ["-l", "5"],
    ["--json", "-u", "alice"],
    ["-u", "Zoë"],
    ["--json", "-u", "tab user"],
    ["--json", "-r", "b1"],
    ["--json", "-r", "b2", "-s", "403"],
    ["-r", "arn:dfs:s3:::b0/k5"],
    ["--json", "-a", "s3:PutObject", "-l", "1000"],
    ["--json", "-s", "404", "-l", "7"],
    ["--json", "--start", "2026-03-01T11:30:00Z", "--end", "2026-03-01T12:10:00+00:00", "-l", "1000"],
    ["--json", "-u", "bob", "--start", "2026-03-01T12:00:00Z"],
    ["-u", "nobody"],
]


@pytest.mark.parametrize("args", CASES, ids=[" ".join(c) or "all" for c in CASES])
def test_native_reader_matches_python(logdir, capsys, args):
    assert native(str(logdir), *args) == python(capsys, str(logdir), *args)


def test_native_verify_chain_and_tamper(logdir, capsys, tmp_path):
    rc, out = native(str(logdir), "--verify-chain", SECRET)
    assert rc == 0 and out.strip() == "verified 240 records: OK"
    assert (rc, out) == python(capsys, str(logdir), "--verify-chain", SECRET)
    rc, out = native(str(logdir), "--verify-chain", "wrong-secret-123456")
    assert rc == 1 and "record_hash mismatch" in out
    assert (rc, out) == python(capsys, str(logdir), "--verify-chain", "wrong-secret-123456")
    # tamper one record in a copy of the store
    import shutil
    t = tmp_path / "t"
    shutil.copytree(logdir, t)
    seg = SegmentStore(str(t)).segments()[1][1]
    lines = open(seg, encoding="utf-8").read().splitlines()
    ts, js = lines[4].split("\t", 1)
    r = json.loads(js)
    r["status_code"] = 500
    lines[4] = ts + "\t" + json.dumps(r, separators=(",", ":"))
    open(seg, "w", encoding="utf-8").write("\n".join(lines) + "\n")
    rc, out = native(str(t), "--verify-chain", SECRET)
    assert rc == 1 and "record_hash mismatch" in out and "1 errors" in out
    assert (rc, out) == python(capsys, str(t), "--verify-chain", SECRET)


def test_native_writer_matches_python_writer(tmp_path):
    """csrc/audit_log.cpp (the default writer) and the Python writer produce byte-identical
    segments and index files for the same records and batch boundaries: same sort, same
    monotonic keys, same canonical JSON (non-ASCII, control characters, nulls), same HMAC
    chain, continued across a restart."""
    from tests.models.s3_audit import NativeAuditLogger, PyAuditLogger, verify_chain

    base = datetime(2026, 5, 2, 23, 58, tzinfo=timezone.utc)
    users = ["alice", "Zoë", None, "tab\tuser", "nl\nuser"]

    def records(lo, hi):
        for i in range(lo, hi):
            # same-millisecond pairs logged in reverse request-id order, one stale timestamp
            now = base + timedelta(seconds=(i // 2) * 7 if i != 57 else -3600)
            yield make_record(request_id=f"req-{(i ^ 1):04d}", remote_ip="10.0.0.2", user_id=users[i % 5],
                              role_arn=None if i % 4 else "arn:aws:iam::1:role/r", action="s3:PutObject",
                              resource=f"arn:dfs:s3:::bk{i % 3}:x/k{i}" if i % 6 else f"bk{i % 3}/k",
                              status_code=200 + i % 3, error_code=None if i % 2 else "Eé",
                              user_agent="ua \"q\" \\ \x7f \x1f 𝄞", duration_ms=i, now=now)

    dirs = {}
    for kind, cls in (("py", PyAuditLogger), ("native", NativeAuditLogger)):
        d = tmp_path / kind
        for lo, hi in ((0, 90), (90, 130)):  # a restart between the two groups
            lg = cls(str(d), batch_size=17, hmac_secret=SECRET, flush_interval=30)
            for rec in records(lo, hi):
                lg.log(rec)
                if rec["duration_ms"] % 17 == 16:
                    assert lg.flush(10)  # batch boundaries at the same records in both writers
            assert lg.flush(10)
            lg.close()
        dirs[kind] = d
    names = sorted(p.name for p in dirs["py"].iterdir())
    assert names == sorted(p.name for p in dirs["native"].iterdir()) and len(names) >= 3
    for n in names:
        assert (dirs["py"] / n).read_bytes() == (dirs["native"] / n).read_bytes(), n
    n, errs = verify_chain(SegmentStore(str(dirs["native"])), SECRET)
    assert n == 130 and errs == []
    assert native(str(dirs["native"]), "--verify-chain", SECRET)[0] == 0


def test_native_writer_ingest_and_drops(tmp_path):
    """Datagrams on the ingest socket are logged by the native thread; a full queue drops
    (never blocks) and counts it."""
    import socket

    from tests.models.s3_audit import NativeAuditLogger

    lg = NativeAuditLogger(str(tmp_path / "a"), batch_size=1000, hmac_secret=SECRET, flush_interval=60,
                           capacity=8)
    for i in range(20):
        lg.log(make_record(request_id=f"r{i}", remote_ip="", user_id="u", role_arn=None, action="a",
                           resource="r", status_code=200, error_code=None, user_agent=None, duration_ms=0))
    assert lg.m_dropped.get() == 12 and lg.m_total.get() == 20
    assert lg.flush(10)
    path = str(tmp_path / "ingest.sock")
    srv = socket.socket(socket.AF_UNIX, socket.SOCK_DGRAM)
    srv.bind(path)
    lg.start_ingest(srv)
    cli = socket.socket(socket.AF_UNIX, socket.SOCK_DGRAM)
    for i in range(5):
        rec = make_record(request_id=f"d{i}", remote_ip="", user_id="dg", role_arn=None, action="a",
                          resource="r", status_code=200, error_code=None, user_agent=None, duration_ms=0)
        cli.sendto(json.dumps(rec).encode(), path)
    cli.sendto(b"not json", path)
    import time

    deadline = time.time() + 10
    while lg.stats()["ingested"] < 6 and time.time() < deadline:
        time.sleep(0.02)
    assert lg.flush(10)
    lg.close()
    recs = [r for _, r in SegmentStore(str(tmp_path / "a")).scan()]
    assert [r["user_id"] for r in recs].count("dg") == 5 and len(recs) == 13
