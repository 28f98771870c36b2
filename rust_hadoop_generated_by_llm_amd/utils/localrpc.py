"""Same-host transport for the unary gRPC services (master, config server).

A Python gRPC round trip costs ~350 µs of HTTP/2 + grpc-core work on each side, which
dominates metadata latency when the client and the master share a node (every GPU
rank of the benchmark has its own co-located metadata shard). Servers therefore also
listen on an abstract UNIX socket named after their TCP port (``dfs_rpc_<port>``) and
speak a minimal framing of the *same* protobuf messages and handlers:

    request  = u32 body_len | u16 len path "/dfs.Service/Method" | u16 len request_id | payload
    response = u32 body_len | u8 grpc status code | payload (OK) or utf-8 details

``ChannelPool.call`` uses it automatically for loopback targets and falls back to gRPC
when nothing listens, so behaviour (status codes, redirects, Not-Leader hints) is
identical — only the envelope is cheaper. TLS deployments (``https://``) never use it.
"""
from __future__ import annotations

import asyncio
import inspect
import logging
import socket
import struct
import threading
import time

import grpc

from ..models import proto as pb

log = logging.getLogger("dfs.localrpc")

_LOOPBACK = ("127.0.0.1", "localhost", "::1", "[::1]")


def socket_name(port: int | str) -> str:
    return f"dfs_rpc_{port}"


def local_name_for(addr: str) -> str | None:
    """Abstract socket name for a loopback ``host:port`` target, else None."""
    if addr.startswith("https://"):
        return None
    a = addr.split("://", 1)[-1].rstrip("/")
    host, _, port = a.rpartition(":")
    if host not in _LOOPBACK or not port.isdigit():
        return None
    return socket_name(port)


class LocalRpcError(grpc.RpcError):
    def __init__(self, code: grpc.StatusCode, details: str):
        super().__init__(f"{code.name}: {details}")
        self._code = code
        self._details = details

    def code(self):
        return self._code

    def details(self):
        return self._details


_CODES = {c.value[0]: c for c in grpc.StatusCode}


# ---------------------------------------------------------------------------- server
class _AbortCtx:
    """Minimal stand-in for grpc's ServicerContext (handlers only call abort())."""

    def invocation_metadata(self):
        return ()

    async def abort(self, code, details):
        raise _Abort(code, details)


class _Abort(Exception):
    def __init__(self, code, details):
        super().__init__(details)
        self.code, self.details = code, details


def build_dispatch(services: dict):
    """``async dispatch(path, request_id, payload) -> (grpc code, response or message bytes)``
    over the service handlers ({service name: impl}); shared by the Python listener below
    and the native one (csrc/localrpc.cpp), which forwards the methods it does not serve
    itself."""
    from .rpc import RpcStatus, current_request_id, snake

    table = {}
    for sname, impl in services.items():
        for mname, req_cls, _resp_cls in pb.SERVICES[sname]:
            fn = getattr(impl, snake(mname), None)
            if fn is not None:
                table[pb.method_path(sname, mname)] = (fn, req_cls, inspect.iscoroutinefunction(fn))
    ctx = _AbortCtx()

    async def dispatch(path: str, rid: str, payload: bytes) -> tuple[int, bytes]:
        ent = table.get(path)
        if ent is None:
            return grpc.StatusCode.UNIMPLEMENTED.value[0], f"unknown method {path}".encode()
        fn, req_cls, is_async = ent
        token = current_request_id.set(rid)
        try:
            req = req_cls.FromString(payload)
            resp = (await fn(req, ctx)) if is_async else fn(req, ctx)
            return 0, resp.SerializeToString()
        except RpcStatus as e:
            return e.code.value[0], e.message.encode()
        except _Abort as e:
            return e.code.value[0], str(e.details).encode()
        except Exception as e:  # noqa: BLE001
            log.exception("local rpc %s failed", path)
            return grpc.StatusCode.INTERNAL.value[0], str(e).encode()
        finally:
            current_request_id.reset(token)

    return dispatch


async def serve_local(services: dict, port: int | str):
    """Start the UNIX-socket listener for ``services`` ({service name: impl})."""
    dispatch = build_dispatch(services)

    async def handle(reader: asyncio.StreamReader, writer: asyncio.StreamWriter):
        try:
            while True:
                hdr = await reader.readexactly(4)
                (n,) = struct.unpack("<I", hdr)
                body = await reader.readexactly(n)
                (pl,) = struct.unpack_from("<H", body, 0)
                path = body[2:2 + pl].decode()
                (rl,) = struct.unpack_from("<H", body, 2 + pl)
                rid = body[4 + pl:4 + pl + rl].decode()
                code, data = await dispatch(path, rid, body[4 + pl + rl:])
                out = bytes([code]) + data
                writer.write(struct.pack("<I", len(out)) + out)
                await writer.drain()
        except (asyncio.IncompleteReadError, ConnectionError):
            pass
        finally:
            writer.close()

    return await asyncio.start_unix_server(handle, path="\0" + socket_name(port))


# ---------------------------------------------------------------------------- client
class LocalRpcClient:
    """Thread-local persistent connections to one abstract socket."""

    def __init__(self, name: str):
        self.name = name
        self._tls = threading.local()

    def _sock(self, timeout):
        s = getattr(self._tls, "s", None)
        if s is None:
            s = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
            s.connect("\0" + self.name)
            self._tls.s = s
        s.settimeout(timeout)
        return s

    def _drop(self):
        s = getattr(self._tls, "s", None)
        self._tls.s = None
        if s is not None:
            try:
                s.close()
            except OSError:
                pass

    @staticmethod
    def _recv(s, n):
        buf = bytearray(n)
        v = memoryview(buf)
        got = 0
        while got < n:
            r = s.recv_into(v[got:])
            if r == 0:
                raise ConnectionError("local rpc connection closed")
            got += r
        return buf

    def call(self, path: str, request, resp_cls, timeout: float | None, rid: str):
        p = path.encode()
        r = rid.encode()
        payload = request.SerializeToString()
        msg = struct.pack("<IH", 2 + len(p) + 2 + len(r) + len(payload), len(p)) + p + struct.pack("<H", len(r)) + r
        s = self._sock(timeout)
        try:
            s.sendall(msg + payload)
            (n,) = struct.unpack("<I", self._recv(s, 4))
            body = self._recv(s, n)
        except socket.timeout as e:
            self._drop()
            raise LocalRpcError(grpc.StatusCode.DEADLINE_EXCEEDED, "Deadline Exceeded") from e
        except OSError:
            self._drop()
            raise
        code = body[0]
        if code == 0:
            return resp_cls.FromString(bytes(body[1:]))
        raise LocalRpcError(_CODES.get(code, grpc.StatusCode.UNKNOWN), bytes(body[1:]).decode("utf-8", "replace"))


class LocalRegistry:
    """Per-process cache of which loopback targets have a local listener."""

    def __init__(self):
        self._clients: dict[str, LocalRpcClient] = {}
        self._absent: dict[str, float] = {}
        self._lock = threading.Lock()

    def client_for(self, addr: str) -> LocalRpcClient | None:
        name = local_name_for(addr)
        if name is None:
            return None
        c = self._clients.get(name)
        if c is not None:
            return c
        if self._absent.get(name, 0.0) > time.monotonic():
            return None
        s = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
        try:
            s.connect("\0" + name)
        except OSError:
            self._absent[name] = time.monotonic() + 5.0
            return None
        finally:
            s.close()
        with self._lock:
            c = self._clients.setdefault(name, LocalRpcClient(name))
        return c

    def forget(self, addr: str) -> None:
        name = local_name_for(addr)
        if name is not None:
            with self._lock:
                self._clients.pop(name, None)
            self._absent[name] = time.monotonic() + 5.0
