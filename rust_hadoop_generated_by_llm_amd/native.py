"""Loader for the in-tree native extension ``_dfs_native`` (csrc/, built by build_native.py).

The extension is required: the chunk store, checksum kernels, RCCL replication engine,
Raft WAL and AES-GCM all live there. If the .so is missing it is built in place (hipcc
cross-compiles gfx950 without a GPU) under a file lock so concurrent processes do not race.
"""
from __future__ import annotations

import fcntl
import importlib.util
import os
import sys
import sysconfig
from pathlib import Path

_PKG = Path(__file__).resolve().parent
_ROOT = _PKG.parent
_SO = _PKG / ("_dfs_native" + sysconfig.get_config_var("EXT_SUFFIX"))


def _sources_newer() -> bool:
    if not _SO.exists():
        return True
    t = _SO.stat().st_mtime
    csrc = _ROOT / "csrc"
    return any(p.stat().st_mtime > t for p in csrc.glob("*") if p.suffix in (".cpp", ".hip", ".h"))


def _ensure_built() -> None:
    if _SO.exists() and os.environ.get("DFS_NATIVE_AUTOBUILD", "1") == "0":
        return
    if not _sources_newer():
        return
    lock_path = _ROOT / "build" / ".native.lock"
    lock_path.parent.mkdir(parents=True, exist_ok=True)
    with open(lock_path, "w") as lf:
        fcntl.flock(lf, fcntl.LOCK_EX)
        if _sources_newer():
            sys.path.insert(0, str(_ROOT))
            try:
                import build_native  # noqa: PLC0415

                # the extension and tools only: the sanitizer builds are the native unit
                # tests' business (tests/test_native_unit.py builds them on demand)
                saved = os.environ.get("DFS_BUILD_SANITIZERS")
                os.environ["DFS_BUILD_SANITIZERS"] = "0"
                # the build's output goes to stderr, whoever prints it (this process or the
                # compilers it starts): stdout may be a contract, e.g. bench.py's one JSON line
                sys.stdout.flush()
                out_fd = os.dup(1)
                os.dup2(2, 1)
                try:
                    build_native.build()
                finally:
                    sys.stdout.flush()
                    os.dup2(out_fd, 1)
                    os.close(out_fd)
                    if saved is None:
                        os.environ.pop("DFS_BUILD_SANITIZERS", None)
                    else:
                        os.environ["DFS_BUILD_SANITIZERS"] = saved
            finally:
                sys.path.pop(0)


def _load():
    _ensure_built()
    spec = importlib.util.spec_from_file_location(f"{__package__}._dfs_native", _SO)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    sys.modules[f"{__package__}._dfs_native"] = mod
    return mod


lib = _load()
SO_PATH = str(_SO)


def gpu_count() -> int:
    """Number of visible HIP devices (0 on a CPU-only host)."""
    return lib.device_count()


def require_gpu(device: int) -> None:
    n = gpu_count()
    if device >= n:
        raise RuntimeError(
            f"GPU {device} requested but only {n} HIP device(s) visible; the HBM chunk store and "
            "CDNA4 kernels need an MI355X (use --gpu -1 for the CPU store)"
        )
