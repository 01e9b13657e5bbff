"""Hyperswarm-style swarm over the native encrypted transport.

API mirror of what the reference uses (``global.d.ts:4-36``,
``src/provider.ts:38-58, 84-91``): ``Swarm(...)``, ``join(topic, server=,
client=)`` returning a discovery handle with ``flushed()``, ``flush()``,
``on('connection' | 'error')``, ``leave(topic)``, ``destroy()``, ``peers``,
``connecting``.  Each connection is an authenticated, encrypted, message-framed
stream (one ``write`` == one ``data`` event on the other side), exposing the
fields the provider reads: ``public_key`` (local), ``remote_public_key``,
``handshake_hash``, ``raw_stream.remote_host`` and Node-stream semantics for
back-pressure (``write()`` returns False above the high-water mark, then
``'drain'``).

The data plane (sockets, Noise XX, secretstream AEAD, framing, keep-alives)
is C++ (``csrc/net``, the udx-native/sodium-native equivalent); this module is
the control plane: announce/lookup through :mod:`.discovery`, connection
dedup, reconnect with backoff, firewall and connection limits.
"""
from __future__ import annotations

import asyncio
import collections
import inspect
import logging
import random

from . import _native
from .discovery import DiscoveryClient
from .identity import KeyPair
from .identity import key_pair as make_key_pair

log = logging.getLogger("symmetry_amd.net")


class EventEmitter:
    def __init__(self):
        self._handlers: dict[str, list] = collections.defaultdict(list)

    def on(self, event: str, cb):
        self._handlers[event].append(cb)
        return self

    def once(self, event: str, cb):
        def wrapper(*a):
            self.off(event, wrapper)
            return cb(*a)

        return self.on(event, wrapper)

    def off(self, event: str, cb):
        try:
            self._handlers[event].remove(cb)
        except ValueError:
            pass
        return self

    def emit(self, event: str, *args) -> bool:
        hs = list(self._handlers.get(event, ()))
        for cb in hs:
            try:
                r = cb(*args)
                if inspect.isawaitable(r):
                    asyncio.ensure_future(r)
            except Exception:  # a listener bug must not kill the transport pump
                log.exception("listener for %r failed", event)
        return bool(hs)

    def listener_count(self, event: str) -> int:
        return len(self._handlers.get(event, ()))


class RawStream:
    def __init__(self, host: str, port: int):
        self.remote_host = host
        self.remote_port = port
        self.remoteHost = host  # REF spelling (src/types.ts:91-100)


class Connection(EventEmitter):
    """One encrypted peer stream (the reference's ``peer`` / secret-stream object)."""

    def __init__(self, swarm: "Swarm", conn_id: int, info: dict):
        super().__init__()
        self.swarm = swarm
        self.id = conn_id
        self.public_key: bytes = swarm.key_pair.public_key
        self.remote_public_key: bytes = info["remote_public_key"]
        self.handshake_hash: bytes = info["handshake_hash"]
        self.is_initiator: bool = info["initiator"]
        self.raw_stream = RawStream(info["host"], info["port"])
        self.rawStream = self.raw_stream
        self.topics: set[bytes] = set()
        self._open = True
        self._drain_waiters: list[asyncio.Future] = []
        self.bytes_written = 0
        self.bytes_read = 0

    @property
    def writable(self) -> bool:
        return self._open

    @property
    def destroyed(self) -> bool:
        return not self._open

    def write(self, data) -> bool:
        if not self._open:
            return False
        if isinstance(data, str):
            data = data.encode("utf-8")
        self.bytes_written += len(data)
        return self.swarm._transport.write(self.id, bytes(data))

    async def drain(self) -> None:
        """Await the 'drain' event (only meaningful after write() returned False)."""
        if not self._open:
            return
        fut = asyncio.get_running_loop().create_future()
        self._drain_waiters.append(fut)
        await fut

    def inject_fault(self, kind: str, data: bytes = b"\x00" * 16) -> None:
        """Fault injection for tests: ``"raw"`` writes unframed bytes into the encrypted
        stream, ``"corrupt"`` sends a message whose ciphertext fails authentication at the peer."""
        self.swarm._transport.inject_fault(self.id, {"raw": 0, "corrupt": 1}[kind], bytes(data))

    def end(self) -> None:
        if self._open:
            self.swarm._transport.end(self.id)

    def destroy(self) -> None:
        if self._open:
            self.swarm._transport.destroy(self.id)

    # transport callbacks
    def _on_data(self, data: bytes) -> None:
        self.bytes_read += len(data)
        self.emit("data", data)

    def _on_drain(self) -> None:
        for f in self._drain_waiters:
            if not f.done():
                f.set_result(None)
        self._drain_waiters.clear()
        self.emit("drain")

    def _on_close(self, error: str) -> None:
        self._open = False
        for f in self._drain_waiters:
            if not f.done():
                f.set_result(None)
        self._drain_waiters.clear()
        if error:
            self.emit("error", ConnectionError(error))
        self.emit("close")


class PeerDiscovery:
    """Handle returned by :meth:`Swarm.join` (REF ``discovery.flushed()``)."""

    def __init__(self, swarm: "Swarm", topic: bytes, server: bool, client: bool):
        self.swarm, self.topic, self.server, self.client = swarm, topic, server, client
        self._flushed = asyncio.get_running_loop().create_future()
        self._task: asyncio.Task | None = None
        self.destroyed = False

    async def flushed(self) -> None:
        await asyncio.shield(self._flushed)

    def _done_first_round(self) -> None:
        if not self._flushed.done():
            self._flushed.set_result(None)

    async def refresh(self) -> None:
        await self.swarm._round(self)

    def destroy(self) -> None:
        self.destroyed = True
        if self._task is not None:
            self._task.cancel()


class Swarm(EventEmitter):
    def __init__(self, key_pair: KeyPair | None = None, seed: bytes | None = None, *, bootstrap=None,
                 static_peers: dict | None = None, host: str = "127.0.0.1", port: int = 0, max_peers: int = 64,
                 max_connections: int | None = None, firewall=None, keepalive_ms: int = 5000,
                 timeout_ms: int = 20000, high_watermark: int = 1 << 20, announce_ttl: float = 30.0,
                 refresh_interval: float = 2.0):
        super().__init__()
        self.key_pair = key_pair or make_key_pair(seed)
        self.host, self.port = host, port
        self.max_peers = max_peers if max_connections is None else max(1, int(max_connections))
        self.firewall = firewall
        self.announce_ttl = announce_ttl
        self.refresh_interval = refresh_interval
        self.discovery = DiscoveryClient(bootstrap) if bootstrap else None
        self.static_peers = static_peers or {}
        self._transport = _native.Transport(self.key_pair.public_key, self.key_pair.secret_key, keepalive_ms,
                                            timeout_ms, high_watermark)
        self._loop = asyncio.get_running_loop()
        self._loop.add_reader(self._transport.fileno(), self._pump)
        self._listening_port: int | None = None
        self._topics: dict[bytes, PeerDiscovery] = {}
        self._conns: dict[int, Connection] = {}
        self.peers: dict[str, Connection] = {}       # remote pk hex -> connection
        self._dialing: dict[int, str] = {}           # conn id -> expected remote pk hex
        self._dial_waiters: dict[int, asyncio.Future] = {}
        self._backoff: dict[str, float] = {}
        self.destroyed = False

    # ------------------------------------------------------------------------------------------
    @property
    def connecting(self) -> int:
        return len(self._dialing)

    @property
    def connections(self) -> set:
        return set(self._conns.values())

    def listen(self) -> int:
        if self._listening_port is None:
            self._listening_port = self._transport.listen(self.host, self.port)
        return self._listening_port

    def join(self, topic: bytes, server: bool = True, client: bool = True) -> PeerDiscovery:
        if len(topic) != 32:
            raise ValueError("topic must be 32 bytes")
        d = self._topics.get(topic)
        if d is None:
            d = PeerDiscovery(self, topic, server, client)
            self._topics[topic] = d
        else:
            d.server, d.client = d.server or server, d.client or client
        if server:
            self.listen()
        if d._task is None:
            d._task = asyncio.ensure_future(self._topic_loop(d))
        return d

    async def leave(self, topic: bytes) -> None:
        d = self._topics.pop(topic, None)
        if d is None:
            return
        d.destroy()
        if d.server and self.discovery is not None:
            try:
                await self.discovery.unannounce(topic, self.key_pair.public_key)
            except Exception:
                pass

    async def flush(self) -> None:
        """Wait until every joined topic finished its first announce/lookup/connect round."""
        await asyncio.gather(*(d.flushed() for d in list(self._topics.values())))

    async def destroy(self) -> None:
        if self.destroyed:
            return
        self.destroyed = True
        for t in list(self._topics):
            await self.leave(t)
        for c in list(self._conns.values()):
            c.destroy()
        await asyncio.sleep(0.05)
        self._loop.remove_reader(self._transport.fileno())
        self._transport.close()
        if self.discovery is not None:
            await self.discovery.close()

    # ------------------------------------------------------------------------------------------
    async def _topic_loop(self, d: PeerDiscovery) -> None:
        delay = 0.0
        while not d.destroyed and not self.destroyed:
            try:
                await self._round(d)
            except asyncio.CancelledError:
                raise
            except Exception as exc:
                self.emit("error", exc)
            d._done_first_round()
            await asyncio.sleep(self.refresh_interval if delay == 0 else delay)
            delay = min(self.announce_ttl / 3, self.refresh_interval * 2)

    async def _round(self, d: PeerDiscovery) -> None:
        if d.server and self.discovery is not None:
            await self.discovery.announce(d.topic, self.key_pair.public_key, self.host, self.listen(),
                                          self.announce_ttl)
        if not d.client:
            return
        peers = list(self.static_peers.get(d.topic.hex(), []))
        if self.discovery is not None:
            peers += await self.discovery.lookup(d.topic)
        dials = []
        me = self.key_pair.public_key.hex()
        for p in peers:
            pk = p.get("publicKey")
            if pk == me or (pk and pk in self.peers) or pk in self._dialing.values():
                continue
            if pk and self._loop.time() < self._backoff.get(pk, 0):
                continue
            if len(self.peers) + len(self._dialing) >= self.max_peers:
                break
            dials.append(self._dial(p["host"], int(p["port"]), pk, d.topic))
        if dials:
            await asyncio.gather(*dials, return_exceptions=True)

    async def _dial(self, host: str, port: int, pk_hex: str | None, topic: bytes) -> None:
        cid = self._transport.connect(host, port)
        self._dialing[cid] = pk_hex or ""
        fut = self._loop.create_future()
        self._dial_waiters[cid] = fut
        try:
            await asyncio.wait_for(fut, 10.0)
        except asyncio.TimeoutError:
            self._transport.destroy(cid)
        finally:
            self._dial_waiters.pop(cid, None)
        c = self._conns.get(cid)
        if c is not None:
            c.topics.add(topic)

    def _pump(self) -> None:
        for ev in self._transport.poll():
            kind, cid = ev["kind"], ev["conn"]
            if kind == "open":
                self._on_open(cid, ev)
            elif kind == "data":
                c = self._conns.get(cid)
                if c is not None:
                    c._on_data(ev["data"])
            elif kind == "drain":
                c = self._conns.get(cid)
                if c is not None:
                    c._on_drain()
            elif kind == "close":
                self._on_close(cid, ev.get("error") or "", ev)

    def _resolve_dial(self, cid: int) -> None:
        self._dialing.pop(cid, None)
        f = self._dial_waiters.get(cid)
        if f is not None and not f.done():
            f.set_result(None)

    def _on_open(self, cid: int, ev: dict) -> None:
        rpk = ev["remote_public_key"]
        expected = self._dialing.get(cid)
        self._resolve_dial(cid)
        reason = None
        if expected and expected != rpk.hex():
            reason = "remote key does not match the announced key"
        elif rpk.hex() in self.peers:
            reason = "duplicate connection"
        elif len(self.peers) >= self.max_peers:
            reason = "max connections reached"
        elif self.firewall is not None:
            try:
                if self.firewall(rpk):
                    reason = "firewalled"
            except Exception:
                reason = "firewall error"
        if reason is not None:
            log.debug("dropping connection %s: %s", rpk.hex()[:8], reason)
            self._transport.destroy(cid)
            return
        conn = Connection(self, cid, ev)
        self._conns[cid] = conn
        self.peers[rpk.hex()] = conn
        self._backoff.pop(rpk.hex(), None)
        self.emit("connection", conn, {"public_key": rpk, "client": conn.is_initiator})

    def _on_close(self, cid: int, error: str, ev: dict) -> None:
        expected = self._dialing.get(cid)
        self._resolve_dial(cid)
        if expected:
            self._backoff[expected] = self._loop.time() + min(30.0, 0.5 + random.random())
        conn = self._conns.pop(cid, None)
        if conn is None:
            return
        key = conn.remote_public_key.hex()
        if self.peers.get(key) is conn:
            del self.peers[key]
            self._backoff[key] = self._loop.time() + 0.25
        conn._on_close(error)
