"""The driver's bench.py contract, rehearsed on the CPU.

The round-end driver runs `bench.py` at N=1 directly and at N=2/4/8 under
`torch.distributed.run` (one rank per GPU, MAX over ranks, ONE JSON line from rank 0).
Here the same multi-process path runs with the host chunk store (`--cpu`) and the
host-memory socket replication transport, which speaks the same pair/sequence/descriptor
protocol as the RCCL transport (`csrc/replication.cpp`), so the rendezvous, the fan-out to
RF-1 replicas, the observed-transport label and the JSON shape are all exercised without
a GPU. Reference workload: `dfs/client/src/bin/dfs_cli.rs:594-628` (write then read).
"""
import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent

REQUIRED = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
            "scaling", "vs_baseline", "dtype", "data", "config"}


def _run(cmd, tmp_path, timeout=300):
    env = dict(os.environ, TMPDIR=str(tmp_path), MASTER_ADDR="127.0.0.1")
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)
    assert p.returncode == 0, p.stderr[-4000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, p.stdout  # exactly one JSON line on rank 0's stdout
    return json.loads(lines[0])


def _check_common(d, n, steps, warmup):
    assert REQUIRED <= set(d)
    base = json.loads((ROOT / "BASELINE.json").read_text())
    assert d["metric"] == base["metric"]
    assert d["n_gpus"] == n and d["steps"] == steps and d["warmup"] == warmup
    assert d["value"] > 0 and d["higher_is_better"] is True and d["scaling"] == "weak"
    assert d["config"]["replication_factor"] == min(3, n)
    assert d["config"]["store"] == "cpu"


def test_bench_single_rank_cpu(tmp_path):
    d = _run([sys.executable, "bench.py", "--cpu", "--steps", "1", "--warmup", "1", "--count", "10",
              "--remote-steps", "1"], tmp_path)
    _check_common(d, 1, 1, 1)
    assert d["config"]["transport"] == "local"
    assert d["remote_client"]["native_client_ops"] == d["remote_client"]["steps"] * 2 * 10


@pytest.mark.parametrize("n", [4, 8])
def test_bench_multi_rank_socket_transport(tmp_path, n):
    d = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
              "--master-addr", "127.0.0.1", "--master-port", str(29671 + n), "bench.py", "--gpus", str(n),
              "--steps", "1", "--warmup", "1", "--cpu", "--count", "10", "--transport", "socket",
              "--remote-steps", "0"], tmp_path)
    _check_common(d, n, 1, 1)
    assert d["config"]["global_batch"] == 10 * n
    # every rank's engine came up, every directed pair is up, and every write reached
    # RF-1 replicas over the peer transport (nothing fell back, nothing failed)
    assert d["p2p_ranks"] == n and d["p2p_transport"] == "socket"
    assert d["repl_pairs_up"] == n * (n - 1)
    writes = (1 + 1) * 10 * n  # warmup + timed step
    assert d["p2p_forwards"] == writes * (min(3, n) - 1)
    assert d["rccl_forwards"] == 0  # the socket transport carried them, not RCCL
    assert d["p2p_fallbacks"] == 0 and d["replica_failures"] == 0 and d["repl_pair_failures"] == 0
    assert d["config"]["transport"] == "socket"


def test_bench_reclaims_steps_when_the_volume_is_short(tmp_path, monkeypatch):
    """A run whose replicas would not fit the volume deletes each step's files after reading
    them (inside the timed region, reported), so the journals reclaim them as it goes."""
    monkeypatch.setenv("DFS_BENCH_RECLAIM", "1")
    d = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
              "--master-addr", "127.0.0.1", "--master-port", "29699", "bench.py", "--gpus", "2",
              "--steps", "2", "--warmup", "1", "--cpu", "--count", "10", "--transport", "socket",
              "--remote-steps", "0"], tmp_path)
    _check_common(d, 2, 2, 1)
    assert d["volume"]["reclaim_between_steps"] is True
    assert d["p2p_fallbacks"] == 0 and d["replica_failures"] == 0


def test_bench_never_opens_the_gpu():
    """The ranks leave the device to their chunkservers: no torch.cuda / HIP call in bench.py
    (an N-rank node then has N GPU processes, not 2N), and the timed region is bracketed by
    the chunkservers' device synchronize."""
    src = (ROOT / "bench.py").read_text()
    assert "torch.cuda" not in src.replace("(no HIP / torch.cuda call", "")
    assert "native" not in src.split("def main")[1].split("client.benchmark")[0]
    assert src.count("device_sync()") >= 4


def test_bench_sizes_the_journal_to_the_volume(monkeypatch):
    """Store of record (default): every N keeps the journal (never the per-file fallback); each
    chunkserver prepares the segments its replicas need, within the volume. Round-4 ring
    (DFS_JOURNAL_EXPORT=idle): sized below the materializer's mark, per-file where the volume
    cannot hold the ring next to the materialized replicas (N=4/8 x RF 3 on a 79 GB volume)."""
    import shutil
    import types

    sys.path.insert(0, str(ROOT))
    import bench

    a = types.SimpleNamespace(steps=20, warmup=5, remote_steps=0, count=100, size=1 << 20)
    for k in ("DFS_JOURNAL", "DFS_JOURNAL_SEGS", "DFS_JOURNAL_SPARES", "DFS_JOURNAL_EXPORT"):
        monkeypatch.delenv(k, raising=False)
    monkeypatch.setattr(shutil, "disk_usage", lambda p: types.SimpleNamespace(free=79 << 30))
    got = {n: bench._journal_segments(Path("/tmp"), bench._bytes_needed(a, n), n) for n in (1, 2, 4, 8)}
    assert all(v >= 4 for v in got.values()), got
    for n in (1, 2, 4):
        per_cs = bench._bytes_needed(a, n) // n
        assert got[n] * bench.JOURNAL_SEG_DATA >= per_cs  # the run's replicas fit the prepared segments
    assert got[8] * 8 * bench.JOURNAL_SEG_BYTES <= (79 << 30)  # within the volume (the rest on demand)
    monkeypatch.setenv("DFS_JOURNAL_EXPORT", "idle")
    got = {n: bench._journal_segments(Path("/tmp"), bench._bytes_needed(a, n), n) for n in (1, 2, 4, 8)}
    assert got[1] >= 3 and got[2] >= 3 and got[4] == -1 and got[8] == -1, got
    for n in (1, 2):
        per_cs = bench._bytes_needed(a, n) // n
        assert got[n] * bench.JOURNAL_SEG_BYTES * 0.7 >= per_cs
    monkeypatch.setenv("DFS_JOURNAL", "0")  # an explicit choice is left alone
    assert bench._journal_segments(Path("/tmp"), bench._bytes_needed(a, 8), 8) == 0


def test_bench_gpus_without_a_launcher_runs_every_rank(tmp_path):
    """`bench.py --gpus 4` with no WORLD_SIZE starts the 4 ranks itself (torch.distributed.run
    as a child process) and reports n_gpus 4, never a silent 1-rank run."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(TMPDIR=str(tmp_path))
    p = subprocess.run([sys.executable, "bench.py", "--gpus", "4", "--cpu", "--steps", "1", "--warmup", "1",
                        "--count", "8", "--remote-steps", "0"], cwd=ROOT, env=env, capture_output=True, text=True,
                       timeout=400)
    assert p.returncode == 0, p.stderr[-4000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, p.stdout
    d = json.loads(lines[0])
    _check_common(d, 4, 1, 1)
    assert d["config"]["global_batch"] == 8 * 4
    assert len(d["volume"]["per_rank"]) == 4


def test_bench_refuses_a_mismatched_world(tmp_path):
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0", TMPDIR=str(tmp_path))
    p = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--cpu", "--steps", "1"], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=120)
    assert p.returncode != 0 and not p.stdout.strip()


def test_bench_transport_ab_block(tmp_path):
    """--transport-ab: after the primary run, a short second measurement over the other replica
    transport in the same job; the one JSON line carries both (the first multi-GPU run records
    hipipc and RCCL side by side). On CPU the pair is socket -> grpc."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(TMPDIR=str(tmp_path))
    p = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--cpu", "--steps", "2", "--warmup", "1",
                        "--count", "8", "--remote-steps", "0", "--transport", "socket", "--transport-ab", "on"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, p.stderr[-4000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, p.stdout
    d = json.loads(lines[0])
    _check_common(d, 2, 2, 1)
    assert d["config"]["transport"] == "socket" and d["p2p_forwards"] > 0
    ab = d["transport_ab"]["grpc"]
    assert "error" not in ab, ab
    # without a P2P pair the next server stages from the writer's slot (same host): "shm"
    assert ab["value"] > 0 and ab["transport"] in ("grpc", "shm") and ab["p2p_forwards"] == 0


def test_bench_spreads_ranks_over_volumes(tmp_path):
    """DFS_BENCH_DIRS: rank r keeps its journal, blocks and master WAL on volume r % V (the
    8-GPU node's one-NVMe-per-GPU layout); each rank reports its volume, and a rank's
    directory on another volume is removed at exit."""
    v2 = tmp_path / "vol2"
    v2.mkdir()
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(TMPDIR=str(tmp_path), DFS_BENCH_DIRS=f"{tmp_path},{v2}")
    p = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--cpu", "--steps", "1", "--warmup", "1",
                        "--count", "8", "--remote-steps", "0", "--transport", "socket"], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=400)
    assert p.returncode == 0, p.stderr[-4000:]
    d = json.loads([ln for ln in p.stdout.splitlines() if ln.strip()][0])
    per = d["volume"]["per_rank"]
    assert [r["volume"] for r in per] == [str(tmp_path), str(v2)] and per[1]["rank_dir_bytes"] > 0, per
    assert all(r["volumes_in_job"] == 2 for r in per)
    assert d["p2p_forwards"] > 0
    assert list(v2.iterdir()) == []  # the second volume's rank directory is gone
