"""Flag names and defaults of every binary match the reference (SURVEY §5.6 table:
bin/master.rs:21-80, bin/config_server.rs:19-48, bin/chunkserver.rs:33-72,
dfs_cli.rs:16-43,131-171), so the reference's scripts and compose command lines translate 1:1."""
from tests.models.chunkserver_shell import build_parser as cs_parser
from rust_hadoop_generated_by_llm_amd.cli.dfs_cli import build_parser as cli_parser


def _native_help(exe: str) -> tuple[set[str], dict[str, str]]:
    """Flag names and the defaults table of a native executable's --help."""
    import re
    import subprocess
    from pathlib import Path

    path = Path(__file__).resolve().parents[1] / "build" / "native" / exe
    out = subprocess.run([str(path), "--help"], capture_output=True, text=True, timeout=30).stdout
    usage, _, defaults = out.partition("defaults:\n")
    table = dict(ln.strip()[2:].split(" ", 1) for ln in defaults.splitlines() if ln.strip())
    return set(re.findall(r"--[a-z0-9-]+", usage)), table


MASTER_FLAGS = {"--addr", "--id", "--peers", "--http-port", "--advertise-addr", "--storage-dir", "--shard-id",
                "--standby", "--shard-config", "--config-servers", "--split-threshold-rps",
                "--split-cooldown-secs", "--merge-threshold-rps", "--tls-cert", "--tls-key", "--ca-cert",
                "--domain-name", "--backup-s3-endpoint", "--backup-bucket"}
CONFIG_FLAGS = {"--addr", "--id", "--peers", "--http-port", "--advertise-addr", "--storage-dir", "--tls-cert",
                "--tls-key", "--ca-cert"}


def test_master_flags_and_defaults():
    """dfs_master takes every flag of bin/master.rs with its default (plus the launcher's
    --no-fsync / --fast-intervals / --http-host / --snapshot-threshold knobs)."""
    flags, d = _native_help("dfs_master")
    assert MASTER_FLAGS <= flags, MASTER_FLAGS - flags
    assert d["addr"] == "127.0.0.1:50051" and d["id"] == "1" and d["http-port"] == "8080"
    assert d["storage-dir"] == "/tmp/raft-logs" and d["shard-id"] == "shard-0"
    assert (float(d["split-threshold-rps"]), int(d["split-cooldown-secs"]), float(d["merge-threshold-rps"])) == \
        (100.0, 30, 1.0)
    assert d["backup-bucket"] == "dfs-backups"


def test_config_server_flags_and_defaults():
    flags, d = _native_help("dfs_config_server")
    assert CONFIG_FLAGS <= flags, CONFIG_FLAGS - flags
    assert (d["addr"], d["id"], d["http-port"], d["storage-dir"]) == \
        ("127.0.0.1:50052", "1", "8081", "/tmp/config-raft-logs")


def test_chunkserver_flags_and_defaults():
    a = cs_parser().parse_args([])
    assert a.addr == "127.0.0.1:50052" and a.storage_dir == "/tmp/chunkserver_data" and a.http_port == 8082
    assert a.rack_id == ""
    a = cs_parser().parse_args(["--config-servers", "c", "--cold-storage-dir", "/c", "--advertise-addr", "h",
                                "--tls-cert", "t", "--tls-key", "k", "--ca-cert", "ca", "--domain-name", "d",
                                "--gpu", "3", "--hbm-capacity", "64G", "--durability", "hbm-ack",
                                "--rccl-rank", "1", "--rccl-world", "8", "--replication-transport", "grpc"])
    assert a.gpu == 3 and a.durability == "hbm-ack" and a.replication_transport == "grpc"


def test_dfs_cli_flags_and_benchmark_defaults():
    p = cli_parser()
    a = p.parse_args(["ls"])
    assert a.master == "http://127.0.0.1:50051" and a.max_retries == 5 and a.initial_backoff_ms == 500
    a = p.parse_args(["benchmark", "write"])
    assert (a.count, a.size, a.concurrency, a.prefix) == (100, 1048576, 10, "bench_write")
    a = p.parse_args(["benchmark", "stress-write"])
    assert (a.duration, a.prefix) == (30, "bench_stress")
    a = p.parse_args(["--host-alias", "a=b", "--host-alias", "c=d", "--ca-cert", "x", "--domain-name", "y",
                      "--config-servers", "c1", "ls"])
    assert a.host_alias == ["a=b", "c=d"]


def test_native_chunkserver_takes_the_shell_flags():
    """dfs_chunkserver accepts every flag of the chunkserver command line except the two that
    select the Python shell's own paths (--grpc-impl, --no-fastpath: the launcher starts the
    shell for those)."""
    py = {s for a in cs_parser()._actions for s in a.option_strings if s.startswith("--") and s != "--help"}
    flags, _ = _native_help("dfs_chunkserver")
    assert py - flags == {"--grpc-impl", "--no-fastpath"}, py - flags
