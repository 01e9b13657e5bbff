"""SymmetryProvider: the provider node (REF ``src/provider.ts:21-322``, C3a-C3h).

Lifecycle:

* ``init()`` -- identity keypair from ``Buffer.alloc(32).fill(name)``, topic =
  ``discoveryKey(publicKey)``, join it as server+client and wait for the
  announce; register the connection listener; log the discovery key; if
  ``public``, ``join_server()``.
* ``join_server()`` -- a second swarm joins ``discoveryKey(utf8(serverKey))``
  client-only; on each server connection write ``challenge`` (32 random bytes
  in Node Buffer-JSON form) then ``join`` (the whole config + discoveryKey hex);
  answer ``ping`` with ``pong``; verify the server's signed ``challenge`` reply
  against the hex-decoded ``serverKey`` (ed25519).  A failed verification only
  logs, as in the reference, unless ``strictServerAuth`` is set.
* ``listeners(peer)`` -- ``newConversation`` bumps the global conversation
  index; ``inference`` streams a completion: the raw header
  ``{"symmetryEmitterKey": key}``, one swarm message per chunk (awaiting
  ``drain`` on back-pressure), then ``{"key":"inferenceEnded","data":key}``;
  data collection when enabled and the key is ``"inference"``.

Deliberate deviations (each additive):
  (5)  ``strictServerAuth: true`` drops the server link on a bad signature;
  (9)  backend errors send an OpenAI-style error event AND ``inferenceEnded``;
  (10) a peer that goes away aborts generation (frees its KV blocks);
  (12) ``maxConnections`` is enforced (swarm connection limit + engine admission);
  (Q5) ``apiKey`` is redacted from the ``join`` payload unless ``shareApiKey``;
  requests on one peer are served one at a time (no interleaved streams).
"""
from __future__ import annotations

import asyncio
import base64
import signal
import time

from ..backends.base import Backend, BackendError
from ..config import ConfigManager
from ..log import logger
from ..net import identity
from ..net.swarm import Swarm
from ..protocol import sse
from ..protocol.codec import buffer_json, create_message, emitter_header, safe_parse_json
from ..protocol.keys import NATIVE_PROVIDER, Keys
from ..utils.metrics import MetricsReporter
from .datacollect import save_completion

DEFAULT_BOOTSTRAP = "127.0.0.1:49737"


def parse_bootstrap(value) -> list[tuple[str, int]]:
    if value is None:
        value = DEFAULT_BOOTSTRAP
    if isinstance(value, str):
        value = [v for v in value.replace(",", " ").split() if v]
    out = []
    for v in value:
        if isinstance(v, (list, tuple)):
            out.append((str(v[0]), int(v[1])))
        else:
            host, _, port = str(v).rpartition(":")
            out.append((host or "127.0.0.1", int(port)))
    return out


def make_backend(config: dict) -> Backend:
    if str(config.get("apiProvider", "")).lower() == NATIVE_PROVIDER:
        from ..backends.native import NativeBackend

        return NativeBackend(config)
    from ..backends.proxy import ProxyBackend

    return ProxyBackend(config)


class SymmetryProvider:
    def __init__(self, config_path: str | ConfigManager, backend: Backend | None = None, bootstrap=None,
                 install_signal_handlers: bool = False):
        path = config_path if isinstance(config_path, str) else config_path.path
        logger.info(f"🔗 Initializing client using config file: {path}")
        self._config = config_path if isinstance(config_path, ConfigManager) else ConfigManager(config_path)
        cfg = self._config
        self._is_public = cfg.get("public")
        self._challenge: bytes | None = None
        self._conversation_index = 0
        self._discovery_key: bytes | None = None
        self._provider_swarm: Swarm | None = None
        self._server_swarm: Swarm | None = None
        self._server_peer = None
        self._server_verified: bool | None = None
        self.backend = backend or make_backend(cfg.get_all())
        self.bootstrap = parse_bootstrap(bootstrap if bootstrap is not None else cfg.get("bootstrap"))
        self.install_signal_handlers = install_signal_handlers
        self._peer_locks: dict[int, asyncio.Lock] = {}
        self._tasks: set[asyncio.Task] = set()
        self.active_peers = 0
        self.completed = 0
        self.saved_files: list[str] = []
        self._stopped = asyncio.Event()
        # fault containment: 0 = healthy / orderly shutdown; 1 = the backend lost its engine (e.g. a tensor-
        # parallel rank died): the provider left the server and the CLI exits with this code
        self.exit_code = 0
        self.fatal: str | None = None
        self._closing = False

    # ------------------------------------------------------------------------------------------
    @property
    def discovery_key(self) -> bytes | None:
        return self._discovery_key

    @property
    def key_pair(self) -> identity.KeyPair:
        return identity.key_pair(identity.seed_from_name(self._config.get("name")))

    async def init(self) -> None:
        cfg = self._config
        await self.backend.start()
        max_conn = cfg.get("maxConnections")
        kp = self.key_pair
        self._provider_swarm = Swarm(kp, bootstrap=self.bootstrap, host=str(cfg.get("listenHost", "127.0.0.1")),
                                     port=int(cfg.get("listenPort", 0)),
                                     max_connections=int(max_conn) if max_conn else None)
        self._discovery_key = identity.discovery_key(kp.public_key)
        discovery = self._provider_swarm.join(self._discovery_key, server=True, client=True)
        await discovery.flushed()
        self._provider_swarm.on("error", lambda err: logger.error("🚨 Swarm Error:", err))
        self._provider_swarm.on("connection", self._on_connection)
        logger.info("📁 Symmetry client initialized.")
        logger.info(f"🔑 Discovery key: {self._discovery_key.hex()}")
        if self._is_public:
            logger.info(f"🔑 Server key: {cfg.get('serverKey')}")
            logger.info("🔗 Joining server, please wait.")
            await self.join_server()
        self.http = None
        if cfg.get("serveHttp") and getattr(self.backend, "name", "") == "native":
            from ..serve.http import LocalAPIServer

            self.http = LocalAPIServer(self.backend, str(cfg.get("modelName")), host=str(cfg.get("apiHostname")),
                                       port=int(cfg.get("apiPort") or 0), path=str(cfg.get("apiPath")),
                                       api_key=cfg.get("apiKey"), stats=self.stats)
            port = await self.http.start()
            logger.info(f"🌐 OpenAI-compatible API on http://{self.http.host}:{port}{self.http.path}")
        self.metrics_reporter = MetricsReporter(
            self.stats, interval_s=float(cfg.get("metricsInterval", 60) or 0),
            path=cfg.get("metricsFile"), log=lambda line: logger.info(f"📊 {line}"))
        self.metrics_reporter.start()
        add_fatal = getattr(self.backend, "add_fatal_listener", None)
        if add_fatal is not None:
            add_fatal(self._on_backend_fatal)
        if self.install_signal_handlers:
            loop = asyncio.get_running_loop()
            for sig in (signal.SIGINT, signal.SIGTERM):
                try:
                    loop.add_signal_handler(sig, lambda: asyncio.ensure_future(self.shutdown("provider shutting down")))
                except (NotImplementedError, RuntimeError):
                    pass

    def _on_connection(self, peer, info=None) -> None:
        logger.info(f"⚡️ New connection from peer: {peer.raw_stream.remote_host}")
        self.active_peers += 1
        peer.on("close", self._on_peer_close)
        self.listeners(peer)

    def _on_peer_close(self) -> None:
        self.active_peers = max(0, self.active_peers - 1)

    # ------------------------------------------------------------------------------------------
    async def join_server(self) -> None:
        self._server_swarm = Swarm(bootstrap=self.bootstrap)
        topic = identity.server_topic(str(self._config.get("serverKey")))
        self._server_swarm.join(topic, server=False, client=True)
        asyncio.ensure_future(self._server_swarm.flush())  # REF: flush() not awaited
        self._server_swarm.on("connection", self._on_server_connection)

    def _join_payload(self) -> dict:
        data = dict(self._config.get_all())
        if not data.get("shareApiKey") and "apiKey" in data:
            data["apiKey"] = None
        data["discoveryKey"] = self._discovery_key.hex() if self._discovery_key else None
        return data

    def _on_server_connection(self, peer, info=None) -> None:
        self._server_peer = peer
        logger.info("🔗 Connected to server.")
        self._challenge = identity.random_bytes(32)
        peer.write(create_message(Keys.CHALLENGE, {"challenge": buffer_json(self._challenge)}))
        peer.write(create_message(Keys.JOIN, self._join_payload()))

        def on_data(buf: bytes) -> None:
            if not buf:
                return
            data = safe_parse_json(buf)
            if not isinstance(data, dict) or not data.get("key"):
                return
            key = data["key"]
            if key == Keys.CHALLENGE:
                self.handle_server_verification(data.get("data") or {})
            elif key == Keys.PING:
                peer.write(create_message(Keys.PONG))

        peer.on("data", on_data)

    def get_server_public_key(self, server_key_hex: str) -> bytes:
        return identity.server_public_key(server_key_hex)

    def handle_server_verification(self, data: dict) -> bool | None:
        if not self._challenge:
            print("No challenge set. Cannot verify.")
            return None
        try:
            public_key = self.get_server_public_key(str(self._config.get("serverKey")))
            signature = base64.b64decode(str((data.get("signature") or {}).get("data", "")))
            verified = identity.verify(self._challenge, signature, public_key)
        except Exception as exc:
            print("Error during verification:", exc)
            return None
        self._server_verified = verified
        if verified:
            logger.info("✅ Verification successful.")
        else:
            logger.error("❌ Verification failed!")
            if self._config.get("strictServerAuth") and self._server_peer is not None:
                self._server_peer.destroy()
        return verified

    # ------------------------------------------------------------------------------------------
    def listeners(self, peer) -> None:
        lock = self._peer_locks.setdefault(id(peer), asyncio.Lock())

        def on_data(buf: bytes) -> None:
            if not buf:
                return
            data = safe_parse_json(buf)
            if not isinstance(data, dict) or not data.get("key"):
                return
            key = data["key"]
            if key == Keys.NEW_CONVERSATION:
                self._conversation_index += 1
            elif key == Keys.INFERENCE:
                if isinstance(data.get("data"), dict):  # request-path timing (NativeBackend.timings)
                    data["data"]["_t_recv"] = time.perf_counter()
                logger.info(f"📦 Inference message received from {peer.raw_stream.remote_host}")
                t = asyncio.ensure_future(self._serialized(lock, data, peer))
                self._tasks.add(t)
                t.add_done_callback(self._tasks.discard)

        peer.on("data", on_data)
        peer.on("close", lambda: self._peer_locks.pop(id(peer), None))

    async def _serialized(self, lock: asyncio.Lock, data: dict, peer) -> None:
        async with lock:
            await self.handle_inference_request(data, peer)

    async def handle_inference_request(self, data: dict, peer) -> None:
        req = data.get("data") or {}
        emitter_key = req.get("key")
        completion = ""
        # prefix-cache scope: a client's multi-turn prompts reuse its own cached KV only (no cross-client
        # aliasing, no cross-client TTFT side channel on a public provider)
        scope = bytes(getattr(peer, "remotePublicKey", b"") or b"")
        direct = getattr(self.backend, "stream_direct", None)
        gen = None if direct is not None else self.backend.stream(req, scope=scope)
        try:
            header_sent = False
            if direct is not None:
                # native engine: each token's event is written by the engine's per-step output callback on
                # this loop (no per-token task switch); a congested peer is bounded by maxBacklog outputs
                parts: list = []

                def write(raw: bytes, delta: str):
                    nonlocal header_sent
                    if not header_sent:
                        peer.write(emitter_header(emitter_key))
                        header_sent = True
                    if not peer.writable:
                        return None
                    parts.append(delta)
                    return bool(peer.write(raw))

                try:
                    await direct(req, write, scope=scope)
                finally:
                    completion = "".join(parts)
            else:
                async for chunk in gen:
                    if not header_sent:
                        peer.write(emitter_header(emitter_key))
                        header_sent = True
                    if not peer.writable:
                        break
                    completion += chunk.delta
                    if not peer.write(chunk.raw):
                        await peer.drain()
            if not peer.writable:
                return
            if not header_sent:
                peer.write(emitter_header(emitter_key))
            peer.write(create_message(Keys.INFERENCE_ENDED, emitter_key))
            self.completed += 1
            if self._config.get("dataCollectionEnabled") and emitter_key == Keys.INFERENCE:
                t = asyncio.ensure_future(save_completion(str(self._config.get("path")), peer.public_key,
                                                          self._conversation_index, req.get("messages"),
                                                          completion))
                t.add_done_callback(lambda f: self.saved_files.append(f.result()) if not f.exception() else None)
        except (BackendError, OSError, asyncio.TimeoutError, Exception) as exc:  # noqa: B014
            message = str(exc) or "An error occurred during inference"
            logger.error(f"🚨 {message}")
            if peer.writable:
                peer.write(sse.error_event(message))
                peer.write(create_message(Keys.INFERENCE_ENDED, emitter_key))
        finally:
            if gen is not None:
                await gen.aclose()

    # ------------------------------------------------------------------------------------------
    def _on_backend_fatal(self, message: str) -> None:
        """The backend can no longer serve (a tensor-parallel peer died): every open stream has already been
        ended with the error event + ``inferenceEnded`` (deviation 9); leave the server so no client is assigned
        here any more, and stop with a non-zero exit code for the supervisor (the reference would keep answering
        pings, ``src/provider.ts:124-126``, while every request failed)."""
        logger.error(f"🚨 {message}")
        self.fatal = message
        self.exit_code = 1
        asyncio.ensure_future(self.shutdown(None))

    def _send_leave(self) -> None:
        peer = self._server_peer
        if peer is not None and getattr(peer, "writable", False):
            peer.write(create_message(Keys.LEAVE, {"discoveryKey": self._discovery_key.hex()
                                                   if self._discovery_key else None, "reason": self.fatal}))

    async def shutdown(self, message: str | None) -> None:
        """Orderly stop (signal or fault): end open streams with an error event + ``inferenceEnded`` (``message``;
        None: already ended by the backend), send ``leave`` to the server, let those writes drain, destroy."""
        if self._closing:
            return
        self._closing = True
        probe = getattr(self.backend, "health_fault", None)
        fault = probe() if (probe is not None and self.fatal is None) else None
        if fault:  # e.g. SIGTERM from torchrun after a worker rank died: that is a fault, not a clean stop
            logger.error(f"🚨 {fault}")
            self.fatal, self.exit_code = fault, 1
            message = f"provider unavailable: {fault}"
        fail = getattr(self.backend, "fail_active", None)
        n = fail(message) if (fail is not None and message) else 0
        self._send_leave()
        if n or self._tasks or self.fatal:
            # the streams' error events + inferenceEnded are written by their own tasks: give them the loop
            deadline = asyncio.get_running_loop().time() + 2.0
            while self._tasks and asyncio.get_running_loop().time() < deadline:
                await asyncio.sleep(0.02)
            await asyncio.sleep(0.1)  # the encrypted writes (and leave) leave the socket buffers
        await self.destroy()

    def stats(self) -> dict:
        """Backend (engine) metrics merged with the provider's own counters."""
        d = dict(self.backend.stats())
        d.update(active_peers=self.active_peers, completed=self.completed,
                 conversations=self._conversation_index, server_verified=self._server_verified)
        return d

    async def destroy(self) -> None:
        if getattr(self, "metrics_reporter", None) is not None:
            self.metrics_reporter.stop()
        if getattr(self, "http", None) is not None:
            await self.http.stop()
        for t in list(self._tasks):
            t.cancel()
        if self._provider_swarm is not None:
            await self._provider_swarm.destroy()
        if self._server_swarm is not None:
            await self._server_swarm.destroy()
        await self.backend.stop()
        self._stopped.set()

    async def wait_closed(self) -> None:
        await self._stopped.wait()
