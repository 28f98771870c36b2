"""Client side of the ChunkServer's native local data path (csrc/fastpath.h).

One persistent abstract-namespace UNIX socket per client thread; requests carry only
(block id, shared-memory slot, length, CRC, master term) — the payload moves through the
client's /dev/shm arena (utils/shm.py). Any status other than OK tells the caller to
use the regular gRPC call instead, so the fast path never changes semantics.
"""
from __future__ import annotations

import socket
import struct
import threading
import uuid

OK, NOT_FOUND, OUT_OF_RANGE, CORRUPT, IO_ERROR, FENCED, UNSUPPORTED, BAD_REQUEST, PARTIAL_CORRUPT = range(9)

_HDR = struct.Struct("<IB")
_RESP = struct.Struct("<BQQH")
_WRITE = struct.Struct("<QIQQ")
_READ = struct.Struct("<QQQQ")


def _s(b: bytes) -> bytes:
    return struct.pack("<H", len(b)) + b


class FastPathError(Exception):
    pass


class FastPathClient:
    def __init__(self, name: str, timeout: float = 120.0):
        self.name = name
        self.timeout = timeout
        self._tls = threading.local()
        self.broken = False

    def _conn(self) -> socket.socket:
        s = getattr(self._tls, "sock", None)
        if s is None:
            s = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
            s.settimeout(self.timeout)
            s.connect("\0" + self.name)
            self._tls.sock = s
        return s

    def _drop(self) -> None:
        s = getattr(self._tls, "sock", None)
        self._tls.sock = None
        if s is not None:
            try:
                s.close()
            except OSError:
                pass

    def _recv_exact(self, s: socket.socket, n: int) -> bytes:
        buf = bytearray(n)
        view = memoryview(buf)
        got = 0
        while got < n:
            r = s.recv_into(view[got:])
            if r == 0:
                raise FastPathError("connection closed")
            got += r
        return bytes(buf)

    def _call(self, op: int, body: bytes) -> tuple[int, int, int, str]:
        try:
            s = self._conn()
            s.sendall(_HDR.pack(len(body) + 1, op) + body)
            (n,) = struct.unpack("<I", self._recv_exact(s, 4))
            resp = self._recv_exact(s, n)
        except OSError as e:
            self._drop()
            raise FastPathError(str(e)) from e
        except FastPathError:
            self._drop()
            raise
        st, total, nbytes, ml = _RESP.unpack_from(resp)
        msg = resp[_RESP.size:_RESP.size + ml].decode("utf-8", "replace")
        return st, total, nbytes, msg

    def write(self, block_id: str, shm_path: str, shm_off: int, length: int, crc: int, term: int,
              next_servers: list[str] | tuple = (), request_id: str | None = None):
        """Returns (status, replicas_written, message). With ``next_servers`` the server
        fans the block out to those replicas natively (P2P / shm) or answers UNSUPPORTED.
        The request id travels to every replica (defaults to the current one)."""
        body = _WRITE.pack(term, crc & 0xFFFFFFFF, shm_off, length) + _s(block_id.encode()) + _s(shm_path.encode())
        body += struct.pack("<H", len(next_servers)) + b"".join(_s(a.encode()) for a in next_servers)
        body += _s(self._rid(request_id))
        st, _total, replicas, msg = self._call(1, body)
        return st, replicas, msg

    def read(self, block_id: str, offset: int, length: int, shm_path: str, shm_off: int, cap: int,
             request_id: str | None = None):
        body = _READ.pack(offset, length, shm_off, cap) + _s(block_id.encode()) + _s(shm_path.encode())
        body += _s(self._rid(request_id))
        return self._call(2, body)  # (status, total, bytes, msg)

    def ec_matmul(self, matrix, k: int, length: int, shm_path: str, in_off: int, out_off: int,
                  request_id: str | None = None):
        """GF(2^8) ``matrix`` (rows x k) times the k shards at ``in_off`` of the client's
        arena (each ``length`` bytes at a 16-byte-aligned stride); the rows land at ``out_off``.
        Runs on the chunkserver's GPU (csrc/fastpath.cpp op 6). Returns the status."""
        rows = len(matrix)
        mat = bytes(v for row in matrix for v in row)
        body = struct.pack("<HHQQQ", k, rows, length, in_off, out_off) + _s(mat) + _s(shm_path.encode())
        body += _s(self._rid(request_id))
        st, _total, _n, msg = self._call(6, body)
        self.last_ec_message = msg
        return st

    @staticmethod
    def _rid(request_id: str | None) -> bytes:
        from .rpc import current_request_id

        return (request_id or current_request_id.get() or uuid.uuid4().hex).encode()

    def close(self) -> None:
        self._drop()


class FastPathEc:
    """Erasure-coding provider for ``ops/erasure.py`` backed by the co-located chunkserver's
    GPU: shards are staged in the client's shared-memory slot (registered for direct DMA on
    the server side) and the RS matrix product runs there. ``gf_matmul`` returns None when
    the job does not fit a slot or the server cannot run it (the caller then counts a CPU
    fallback)."""

    def __init__(self, client: FastPathClient, arena_fn):
        self.client = client
        self.arena_fn = arena_fn  # () -> ShmArena | None
        self.gpu = True  # False once the server said it has no GPU (host-store chunkserver)

    def gf_matmul(self, matrix, inputs, length: int):
        arena = self.arena_fn()
        if arena is None or not matrix:
            return None
        k, rows = len(inputs), len(matrix)
        stride = -(-max(length, 1) // 16) * 16
        need = stride * (k + rows)
        slot = arena.acquire(need)
        if slot is None:
            return None
        try:
            view = arena.view
            for c, shard in enumerate(inputs):
                off = slot + c * stride
                view[off:off + length] = shard
            try:
                st = self.client.ec_matmul(matrix, k, length, arena.path, slot, slot + k * stride)
            except FastPathError:
                return None
            if st == UNSUPPORTED and "no GPU" in getattr(self.client, "last_ec_message", ""):
                self.gpu = False
            if st != OK:
                return None
            base = slot + k * stride
            return [bytes(view[base + r * stride:base + r * stride + length]) for r in range(rows)]
        finally:
            arena.release(slot)
