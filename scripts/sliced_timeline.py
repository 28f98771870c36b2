"""Pipelined head write on one MI355X (fast path -> replication engine, hiploop transport in
one process, three HBM stores): 64 MiB blocks written with RF=3. Run under
`rocprofv3 --kernel-trace` and summarise with `--summary DIR`: per block, the first replica
copy (copyBuffer on the engine's streams) against the last fused copy+checksum kernel of the
head's staging — the sends start before the staging ends."""
import csv
import glob
import os
import sys
import tempfile
import time
from pathlib import Path


def run() -> None:
    sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
    sys.path.insert(0, str(Path(__file__).resolve().parent.parent / "tests"))
    from rust_hadoop_generated_by_llm_amd import native as nat
    from rust_hadoop_generated_by_llm_amd.utils import fastpath as fp
    from rust_hadoop_generated_by_llm_amd.utils.shm import ShmArena
    from test_gpu_replication import GNode, wait_registered, write

    native = nat.lib
    root = Path(tempfile.mkdtemp(prefix="sliced_"))
    ns = "st%x" % (os.getpid() & 0xFFFFFF)
    nodes = [GNode(native, root, r, 3, ns) for r in range(3)]
    for n in nodes:
        n.connect(nodes)
    for n in nodes:
        assert n.eng.wait_ready(10000) == 2
    a, b, c = nodes
    arena = ShmArena(size=160 << 20, slot=80 << 20)
    try:
        assert write(a, arena, b"warm", "warm", [b, c])[0] == fp.OK
        wait_registered(a.store, 160 << 20)
        for i in range(4):
            data = os.urandom(64 << 20)
            t0 = time.perf_counter()
            st, replicas, msg = write(a, arena, data, f"big{i}", [b, c])
            dt = time.perf_counter() - t0
            assert st == fp.OK and replicas == 3, msg
            for n in (b, c):
                assert n.store.read(f"big{i}", 0, 0)[2] == data
            print(f"block {i}: 64 MiB RF=3 in {dt * 1e3:.2f} ms", flush=True)
        print({k: v for k, v in a.fp.stats().items() if k in ("fp_sliced_writes", "fp_rccl_forwards", "fp_writes")})
        print({k: v for k, v in a.store.stats().items() if k in ("sliced_stages", "fused_writes", "direct_dma")})
    finally:
        arena.close()
        for n in nodes:
            n.down()


def summary(d: str) -> None:
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        with open(f, newline="") as fh:
            for r in csv.DictReader(fh):
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    stage = [r for r in rows if "crc_write_copy_kernel" in r[2]]
    copies = [r for r in rows if "copyBuffer" in r[2]]
    # the 64 MiB blocks: runs of 16 write-copy kernels (4 MiB engine slices)
    i = 0
    while i + 16 <= len(stage):
        run_ = stage[i:i + 16]
        first_k, last_k = run_[0][0], run_[-1][1]
        if last_k - first_k > 50_000_000:  # not one block
            i += 1
            continue
        sends = [c for c in copies if c[0] >= first_k and c[0] < last_k + 50_000_000]
        if sends:
            s0 = sends[0][0]
            print(f"block staged {first_k / 1e3:.1f}..{last_k / 1e3:.1f} us: first replica copy starts "
                  f"{(s0 - first_k) / 1e3:.1f} us after staging began, {(last_k - s0) / 1e3:.1f} us before it ended "
                  f"({len([c for c in sends if c[0] < last_k])} copies started while staging)")
        i += 16


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--summary":
        summary(sys.argv[2])
    else:
        run()
