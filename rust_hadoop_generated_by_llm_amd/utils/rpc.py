"""gRPC plumbing shared by every service.

* Servers: generic method handlers built from the proto service table, so a service is a
  plain Python object with snake_case methods (sync or ``async def``). Handlers raise
  :class:`RpcStatus` to return a gRPC status (reference conventions: ``REDIRECT:<peer>``
  in OUT_OF_RANGE, ``Not Leader|<hint>`` in FAILED_PRECONDITION/UNAVAILABLE,
  dfs/metaserver/src/master.rs:2141-2173).
* Clients: a process-wide pool of persistent channels keyed by target. The reference
  opens a fresh TCP/HTTP2 connection for every RPC (dfs/client/src/mod.rs:1412,
  chunkserver.rs:785); pooling removes a connect+TLS handshake from every hop.
* ``x-request-id`` metadata is propagated end to end (reference dfs/common/src/lib.rs:8-50).
"""
from __future__ import annotations

import contextvars
import inspect
import os
import re
import threading
import uuid
from typing import Any, Callable

import grpc

from ..models import proto as pb

MAX_MESSAGE = 100 * 1024 * 1024 + 64 * 1024  # reference caps gRPC messages at 100 MiB
REQUEST_ID_HEADER = "x-request-id"
_OPTIONS = [
    ("grpc.max_send_message_length", MAX_MESSAGE),
    ("grpc.max_receive_message_length", MAX_MESSAGE),
    ("grpc.so_reuseport", 0),
    ("grpc.http2.write_buffer_size", 1 << 20),
    ("grpc.max_concurrent_streams", 1024),
]
_CLIENT_OPTIONS = [
    ("grpc.max_send_message_length", MAX_MESSAGE),
    ("grpc.max_receive_message_length", MAX_MESSAGE),
    ("grpc.enable_retries", 0),
    ("grpc.http2.write_buffer_size", 1 << 20),
]

current_request_id: contextvars.ContextVar[str] = contextvars.ContextVar("request_id", default="")

StatusCode = grpc.StatusCode


class RpcStatus(Exception):
    """Raised by handlers to end an RPC with a non-OK status."""

    def __init__(self, code: grpc.StatusCode, message: str = ""):
        super().__init__(f"{code.name}: {message}")
        self.code = code
        self.message = message


def snake(name: str) -> str:
    return re.sub(r"(?<!^)(?=[A-Z])", "_", name).lower()


def _request_id(context) -> str:
    for k, v in context.invocation_metadata() or ():
        if k == REQUEST_ID_HEADER:
            return v
    return ""


def _wrap_sync(fn: Callable):
    def handler(request, context):
        rid = _request_id(context) or uuid.uuid4().hex
        token = current_request_id.set(rid)
        try:
            return fn(request, context)
        except RpcStatus as e:
            context.abort(e.code, e.message)
        finally:
            current_request_id.reset(token)

    return handler


def _wrap_async(fn: Callable):
    async def handler(request, context):
        rid = _request_id(context) or uuid.uuid4().hex
        token = current_request_id.set(rid)
        try:
            return await fn(request, context)
        except RpcStatus as e:
            await context.abort(e.code, e.message)
        finally:
            current_request_id.reset(token)

    return handler


def generic_handler(service: str, impl: Any) -> grpc.GenericRpcHandler:
    handlers = {}
    for name, req_cls, resp_cls in pb.SERVICES[service]:
        fn = getattr(impl, snake(name), None)
        if fn is None:
            continue
        wrapped = _wrap_async(fn) if inspect.iscoroutinefunction(fn) else _wrap_sync(fn)
        handlers[name] = grpc.unary_unary_rpc_method_handler(
            wrapped, request_deserializer=req_cls.FromString, response_serializer=resp_cls.SerializeToString
        )
    return grpc.method_handlers_generic_handler(f"{pb.PACKAGE}.{service}", handlers)


def server_credentials(tls_cert: str | None, tls_key: str | None, ca_cert: str | None = None):
    if not tls_cert or not tls_key:
        return None
    with open(tls_cert, "rb") as f:
        cert = f.read()
    with open(tls_key, "rb") as f:
        key = f.read()
    root = None
    if ca_cert:
        with open(ca_cert, "rb") as f:
            root = f.read()
    return grpc.ssl_server_credentials([(key, cert)], root_certificates=root, require_client_auth=False)


def make_sync_server(services: dict[str, Any], addr: str, workers: int = 32, creds=None) -> grpc.Server:
    from concurrent.futures import ThreadPoolExecutor

    server = grpc.server(ThreadPoolExecutor(max_workers=workers, thread_name_prefix="grpc"), options=_OPTIONS)
    for name, impl in services.items():
        server.add_generic_rpc_handlers((generic_handler(name, impl),))
    bind = strip_scheme(addr)
    if creds is not None:
        server.add_secure_port(bind, creds)
    else:
        server.add_insecure_port(bind)
    return server


def make_aio_server(services: dict[str, Any], addr: str, creds=None):
    server = grpc.aio.server(options=_OPTIONS)
    for name, impl in services.items():
        server.add_generic_rpc_handlers((generic_handler(name, impl),))
    bind = strip_scheme(addr)
    if creds is not None:
        server.add_secure_port(bind, creds)
    else:
        server.add_insecure_port(bind)
    return server


def strip_scheme(addr: str) -> str:
    for p in ("http://", "https://", "grpc://"):
        if addr.startswith(p):
            addr = addr[len(p):]
    return addr.rstrip("/")


def with_scheme(addr: str, tls: bool = False) -> str:
    if addr.startswith("http://") or addr.startswith("https://"):
        return addr
    return ("https://" if tls else "http://") + addr


LOCAL_SERVICES = frozenset({"MasterService", "ConfigService"})


class ChannelPool:
    """Persistent channels keyed by (target, tls). Thread-safe; shared per process."""

    def __init__(self, ca_cert: str | None = None, domain_name: str | None = None, local: bool = True):
        self._lock = threading.Lock()
        self._chans: dict[str, grpc.Channel] = {}
        self._ca = None
        if ca_cert:
            with open(ca_cert, "rb") as f:
                self._ca = f.read()
        self._domain = domain_name
        self._callables: dict[tuple[str, str, str], Callable] = {}
        # same-host fast transport for metadata services (utils/localrpc.py)
        self._local = None
        if local and os.environ.get("DFS_NO_LOCALRPC") != "1" and ca_cert is None:
            from .localrpc import LocalRegistry

            self._local = LocalRegistry()
        self._resp_cls: dict[tuple[str, str], Any] = {}

    def channel(self, addr: str) -> grpc.Channel:
        key = addr
        ch = self._chans.get(key)
        if ch is not None:
            return ch
        with self._lock:
            ch = self._chans.get(key)
            if ch is None:
                target = strip_scheme(addr)
                tls = addr.startswith("https://") or self._ca is not None
                if tls:
                    opts = list(_CLIENT_OPTIONS)
                    if self._domain:
                        opts.append(("grpc.ssl_target_name_override", self._domain))
                    ch = grpc.secure_channel(target, grpc.ssl_channel_credentials(self._ca), options=opts)
                else:
                    ch = grpc.insecure_channel(target, options=_CLIENT_OPTIONS)
                self._chans[key] = ch
        return ch

    def callable(self, addr: str, service: str, method: str):
        key = (addr, service, method)
        fn = self._callables.get(key)
        if fn is None:
            req_cls = resp_cls = None
            for name, rq, rs in pb.SERVICES[service]:
                if name == method:
                    req_cls, resp_cls = rq, rs
            fn = self.channel(addr).unary_unary(
                pb.method_path(service, method),
                request_serializer=req_cls.SerializeToString,
                response_deserializer=resp_cls.FromString,
            )
            self._callables[key] = fn
        return fn

    def call(self, addr: str, service: str, method: str, request, timeout: float | None = 30.0,
             request_id: str | None = None):
        rid = request_id or current_request_id.get() or uuid.uuid4().hex
        if self._local is not None and service in LOCAL_SERVICES:
            lc = self._local.client_for(addr)
            if lc is not None:
                key = (service, method)
                rc = self._resp_cls.get(key)
                if rc is None:
                    rc = next(rs for name, _rq, rs in pb.SERVICES[service] if name == method)
                    self._resp_cls[key] = rc
                try:
                    return lc.call(pb.method_path(service, method), request, rc, timeout, rid)
                except grpc.RpcError:
                    raise
                except OSError:
                    self._local.forget(addr)  # listener gone: plain gRPC from now on
        return self.callable(addr, service, method)(request, timeout=timeout, metadata=((REQUEST_ID_HEADER, rid),))

    def drop(self, addr: str) -> None:
        with self._lock:
            ch = self._chans.pop(addr, None)
            for k in [k for k in self._callables if k[0] == addr]:
                del self._callables[k]
        if ch is not None:
            ch.close()

    def close(self) -> None:
        with self._lock:
            chans = list(self._chans.values())
            self._chans.clear()
            self._callables.clear()
        for ch in chans:
            ch.close()


class AioChannelPool:
    """asyncio flavour of :class:`ChannelPool` for services running on grpc.aio."""

    def __init__(self, ca_cert: str | None = None, domain_name: str | None = None):
        self._chans: dict[str, grpc.aio.Channel] = {}
        self._ca = None
        if ca_cert:
            with open(ca_cert, "rb") as f:
                self._ca = f.read()
        self._domain = domain_name
        self._callables: dict[tuple[str, str, str], Any] = {}

    def channel(self, addr: str):
        ch = self._chans.get(addr)
        if ch is None:
            target = strip_scheme(addr)
            if addr.startswith("https://") or self._ca is not None:
                opts = list(_CLIENT_OPTIONS)
                if self._domain:
                    opts.append(("grpc.ssl_target_name_override", self._domain))
                ch = grpc.aio.secure_channel(target, grpc.ssl_channel_credentials(self._ca), options=opts)
            else:
                ch = grpc.aio.insecure_channel(target, options=_CLIENT_OPTIONS)
            self._chans[addr] = ch
        return ch

    async def call(self, addr: str, service: str, method: str, request, timeout: float | None = 10.0,
                   request_id: str | None = None):
        key = (addr, service, method)
        fn = self._callables.get(key)
        if fn is None:
            req_cls = resp_cls = None
            for name, rq, rs in pb.SERVICES[service]:
                if name == method:
                    req_cls, resp_cls = rq, rs
            fn = self.channel(addr).unary_unary(
                pb.method_path(service, method),
                request_serializer=req_cls.SerializeToString,
                response_deserializer=resp_cls.FromString,
            )
            self._callables[key] = fn
        rid = request_id or current_request_id.get() or uuid.uuid4().hex
        return await fn(request, timeout=timeout, metadata=((REQUEST_ID_HEADER, rid),))

    async def close(self) -> None:
        chans = list(self._chans.values())
        self._chans.clear()
        self._callables.clear()
        for ch in chans:
            await ch.close()


def rpc_code(err: Exception) -> grpc.StatusCode | None:
    if isinstance(err, grpc.RpcError):
        try:
            return err.code()
        except Exception:  # noqa: BLE001
            return None
    if isinstance(err, RpcStatus):
        return err.code
    return None


def rpc_details(err: Exception) -> str:
    if isinstance(err, grpc.RpcError):
        try:
            return err.details() or ""
        except Exception:  # noqa: BLE001
            return str(err)
    if isinstance(err, RpcStatus):
        return err.message
    return str(err)
