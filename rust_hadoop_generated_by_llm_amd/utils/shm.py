"""Short-circuit local I/O (HDFS "short-circuit reads", extended to writes).

A client co-located with a ChunkServer owns a shared-memory arena under /dev/shm, cut
into fixed slots. For a local WriteBlock it copies the payload into a slot and sends only
(path, offset, length); the ChunkServer maps the same file and stages the block straight
from it into HBM (H2D DMA), persists from it, and forwards it over RCCL — the 1 MiB
payload never crosses the gRPC socket. For a local ReadBlock the ChunkServer DMAs the
range out of HBM directly into the client's slot. Off-host or on any error the client
falls back to the regular gRPC payload path, so wire compatibility is unchanged.
"""
from __future__ import annotations

import mmap
import os
import threading
import uuid

SHM_DIR = "/dev/shm"
SHM_PREFIX = "dfs_sc_"


class ShmArena:
    def __init__(self, size: int = 256 << 20, slot: int = 16 << 20):
        self.slot = slot
        self.size = max(slot, size // slot * slot)
        self.path = os.path.join(SHM_DIR, f"{SHM_PREFIX}{os.getpid()}_{uuid.uuid4().hex[:8]}")
        fd = os.open(self.path, os.O_RDWR | os.O_CREAT | os.O_EXCL, 0o600)
        try:
            os.ftruncate(fd, self.size)
            self.mm = mmap.mmap(fd, self.size)
        finally:
            os.close(fd)
        self.view = memoryview(self.mm)
        self._free = list(range(0, self.size, slot))
        self._cv = threading.Condition()
        self.closed = False

    def acquire(self, n: int, timeout: float = 5.0) -> int | None:
        if n > self.slot or self.closed:
            return None
        with self._cv:
            if not self._free and not self._cv.wait_for(lambda: bool(self._free), timeout):
                return None
            return self._free.pop()

    def release(self, off: int) -> None:
        with self._cv:
            self._free.append(off)
            self._cv.notify()

    def close(self) -> None:
        if self.closed:
            return
        self.closed = True
        try:
            os.unlink(self.path)
        except OSError:
            pass
        try:
            self.view.release()
            self.mm.close()
        except (BufferError, ValueError):
            pass

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass


class ShmMapper:
    """Server side: maps client arenas on first use (validated to live under /dev/shm)."""

    def __init__(self):
        self._maps: dict[str, tuple[mmap.mmap, memoryview]] = {}
        self._lock = threading.Lock()

    def view(self, path: str, offset: int, length: int) -> memoryview:
        real = os.path.realpath(path)
        if os.path.dirname(real) != SHM_DIR or not os.path.basename(real).startswith(SHM_PREFIX):
            raise PermissionError(f"refusing shared-memory path {path}")
        ent = self._maps.get(real)
        if ent is None:
            with self._lock:
                ent = self._maps.get(real)
                if ent is None:
                    fd = os.open(real, os.O_RDWR)
                    try:
                        size = os.fstat(fd).st_size
                        mm = mmap.mmap(fd, size)
                    finally:
                        os.close(fd)
                    ent = (mm, memoryview(mm))
                    self._maps[real] = ent
        mm, mv = ent
        if offset + length > len(mm):
            # the client may have grown/recreated the arena: remap once
            with self._lock:
                self._maps.pop(real, None)
            return self.view(path, offset, length) if os.path.exists(real) and \
                os.path.getsize(real) >= offset + length else _raise(offset, length, len(mm))
        return mv[offset:offset + length]

    def forget(self, path: str) -> None:
        with self._lock:
            ent = self._maps.pop(os.path.realpath(path), None)
        if ent is not None:
            try:
                ent[1].release()
                ent[0].close()
            except (BufferError, ValueError):
                pass


def _raise(offset, length, size):
    raise ValueError(f"shm range [{offset}, {offset + length}) outside mapping of {size} bytes")
