"""Raft peer transports.

* :class:`HttpTransport` — POST JSON to ``/raft/{vote,append,snapshot,timeout_now}`` with a
  1.5 s timeout and the reference's retry policy (3 tries / 50 ms x2 backoff for vote and
  snapshot, 2 tries / 20 ms for append; simple_raft.rs:1313-1363,1485-1532,1587-1651).
* :class:`LocalTransport` — in-process delivery for tests, with a fault injector
  (partitions, isolation, drops, delay) standing in for Toxiproxy / docker kill
  (reference tests: dfs/metaserver/tests/network_partition_tests.rs MockNetwork).
"""
from __future__ import annotations

import asyncio
import json
import random
from typing import Any, Awaitable, Callable

_RETRY = {"vote": (3, 0.05), "snapshot": (3, 0.05), "append": (2, 0.02), "timeout_now": (1, 0.0)}


class TransportError(Exception):
    pass


class HttpTransport:
    def __init__(self, timeout: float = 1.5, ssl_ctx=None):
        self.timeout = timeout
        self.ssl_ctx = ssl_ctx
        self._session = None
        # peers this process may not reach (network-partition injection for process-level
        # chaos tests; set through the master's /debug/partition when DFS_DEBUG_ENDPOINTS=1)
        self.blocked: set[str] = set()

    @staticmethod
    def _base(addr: str) -> str:
        a = addr.rstrip("/")
        return a if a.startswith("http") else "http://" + a

    def _check(self, addr: str) -> None:
        if self.blocked and self._base(addr) in self.blocked:
            raise TransportError(f"{addr}: partitioned")

    async def _sess(self):
        if self._session is None:
            import aiohttp

            self._session = aiohttp.ClientSession(
                timeout=aiohttp.ClientTimeout(total=self.timeout),
                connector=aiohttp.TCPConnector(limit=64, ssl=self.ssl_ctx if self.ssl_ctx else False),
                json_serialize=json.dumps,
            )
        return self._session

    async def send(self, addr: str, kind: str, payload: dict) -> dict:
        self._check(addr)
        tries, backoff = _RETRY.get(kind, (1, 0.0))
        sess = await self._sess()
        url = addr.rstrip("/") + f"/raft/{kind}"
        if not url.startswith("http"):
            url = "http://" + url
        last: Exception | None = None
        for attempt in range(tries):
            try:
                async with sess.post(url, json=payload) as r:
                    if r.status != 200:
                        raise TransportError(f"{url}: HTTP {r.status}")
                    return await r.json(content_type=None)
            except Exception as e:  # noqa: BLE001
                last = e
                if attempt + 1 < tries:
                    await asyncio.sleep(backoff * (2 ** attempt))
        raise TransportError(str(last))

    async def send_raw(self, addr: str, kind: str, body: str) -> str:
        """Same as :meth:`send` with the JSON body already encoded (the native node builds
        AppendEntries text directly from its log)."""
        self._check(addr)
        tries, backoff = _RETRY.get(kind, (1, 0.0))
        sess = await self._sess()
        url = addr.rstrip("/") + f"/raft/{kind}"
        if not url.startswith("http"):
            url = "http://" + url
        last: Exception | None = None
        for attempt in range(tries):
            try:
                async with sess.post(url, data=body, headers={"Content-Type": "application/json"}) as r:
                    if r.status != 200:
                        raise TransportError(f"{url}: HTTP {r.status}")
                    return await r.text()
            except Exception as e:  # noqa: BLE001
                last = e
                if attempt + 1 < tries:
                    await asyncio.sleep(backoff * (2 ** attempt))
        raise TransportError(str(last))

    async def put_bytes(self, url: str, data: bytes) -> int:
        sess = await self._sess()
        async with sess.put(url, data=data) as r:
            return r.status

    async def close(self) -> None:
        if self._session is not None:
            await self._session.close()
            self._session = None


class FaultInjector:
    """Partition matrix + per-node crash/slow toggles shared by LocalTransports."""

    def __init__(self):
        self.blocked: set[tuple[str, str]] = set()
        self.down: set[str] = set()
        self.delay_s: dict[str, float] = {}
        self.drop_rate = 0.0

    def partition(self, group_a: list[str], group_b: list[str]) -> None:
        for a in group_a:
            for b in group_b:
                self.blocked.add((a, b))
                self.blocked.add((b, a))

    def isolate(self, node: str, everyone: list[str]) -> None:
        self.partition([node], [n for n in everyone if n != node])

    def heal(self) -> None:
        self.blocked.clear()
        self.down.clear()
        self.delay_s.clear()
        self.drop_rate = 0.0

    def can_communicate(self, a: str, b: str) -> bool:
        return a not in self.down and b not in self.down and (a, b) not in self.blocked


class LocalTransport:
    """Delivers to handlers registered in a shared ``registry`` dict (addr -> handler)."""

    def __init__(self, self_addr: str, registry: dict[str, Callable[[str, dict], Awaitable[dict]]],
                 faults: FaultInjector | None = None):
        self.self_addr = self_addr
        self.registry = registry
        self.faults = faults or FaultInjector()

    async def send(self, addr: str, kind: str, payload: dict) -> dict:
        f = self.faults
        if not f.can_communicate(self.self_addr, addr) or addr not in self.registry:
            await asyncio.sleep(0.01)
            raise TransportError(f"{self.self_addr} -> {addr} unreachable")
        if f.drop_rate and random.random() < f.drop_rate:
            raise TransportError("dropped")
        d = f.delay_s.get(addr, 0.0) + f.delay_s.get(self.self_addr, 0.0)
        if d:
            await asyncio.sleep(d)
        # round-trip through JSON like the wire would
        reply = await self.registry[addr](kind, json.loads(json.dumps(payload)))
        if not f.can_communicate(addr, self.self_addr):
            raise TransportError("reply lost")
        return json.loads(json.dumps(reply))

    async def put_bytes(self, url: str, data: bytes) -> int:
        return 200

    async def close(self) -> None:
        return None


Handler = Callable[[str, dict], Awaitable[Any]]
