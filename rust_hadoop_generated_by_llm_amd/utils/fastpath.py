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

    @staticmethod
    def _rid(request_id: str | None) -> bytes:
        from .rpc import current_request_id

        return (request_id or current_request_id.get() or uuid.uuid4().hex).encode()

    def close(self) -> None:
        self._drop()
