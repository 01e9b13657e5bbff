"""A Symmetry client (the twinny side): server assignment, then a streamed chat over the swarm.

Flow (inferred from the reference's message keys and
README): connect to the server topic, ``requestProvider{modelName}`` ->
``providerDetails{discoveryKey}``, join the provider's topic, send
``newConversation`` and ``inference{key, messages}``, then read the
``{"symmetryEmitterKey"}`` header, the SSE chunks and ``inferenceEnded``.
Measures TTFT (request write -> first content delta) and tokens/s.
Fault injection: ``disconnect_after`` chunks, ``slow_reader_s``.
"""
from __future__ import annotations

import asyncio
import time
from dataclasses import dataclass, field

from ..net import identity
from ..net.swarm import Swarm
from ..protocol.codec import create_message, safe_parse_json
from ..protocol.keys import Keys
from ..protocol.sse import SSEParser, delta_of


@dataclass
class ChatResult:
    header: dict | None = None
    chunks: list = field(default_factory=list)
    text: str = ""
    ended: bool = False
    ended_key: str | None = None
    error: str | None = None
    ttft_s: float | None = None
    t_start: float = 0.0
    t_end: float = 0.0
    content_events: int = 0

    @property
    def tokens_per_s(self) -> float:
        if self.ttft_s is None or self.content_events < 2:
            return 0.0
        dt = self.t_end - (self.t_start + self.ttft_s)
        return (self.content_events - 1) / dt if dt > 0 else 0.0


class SymmetryClient:
    def __init__(self, bootstrap, server_key: str | None = None):
        self.bootstrap = bootstrap
        self.server_key = server_key
        self.swarm: Swarm | None = None

    async def start(self) -> None:
        self.swarm = Swarm(bootstrap=self.bootstrap)

    async def stop(self) -> None:
        if self.swarm is not None:
            await self.swarm.destroy()

    async def _connect(self, topic: bytes, timeout: float = 15.0):
        fut = asyncio.get_running_loop().create_future()

        def on_conn(conn, info=None):
            if not fut.done():
                fut.set_result(conn)

        self.swarm.on("connection", on_conn)
        self.swarm.join(topic, server=False, client=True)
        try:
            return await asyncio.wait_for(fut, timeout)
        finally:
            self.swarm.off("connection", on_conn)

    async def request_provider(self, model: str, timeout: float = 15.0) -> dict:
        conn = await self._connect(identity.server_topic(self.server_key), timeout)
        q: asyncio.Queue = asyncio.Queue()
        conn.on("data", lambda b: q.put_nowait(safe_parse_json(b)))
        conn.write(create_message(Keys.REQUEST_PROVIDER, {"modelName": model}))
        while True:
            msg = await asyncio.wait_for(q.get(), timeout)
            if isinstance(msg, dict) and msg.get("key") == Keys.PROVIDER_DETAILS:
                conn.destroy()
                await self.swarm.leave(identity.server_topic(self.server_key))
                return msg.get("data") or {}

    async def connect_provider(self, discovery_key_hex: str, timeout: float = 15.0):
        return await self._connect(bytes.fromhex(discovery_key_hex), timeout)

    async def chat(self, conn, messages, emitter_key: str = "inference", timeout: float = 120.0,
                   extra: dict | None = None, new_conversation: bool = True, disconnect_after: int | None = None,
                   slow_reader_s: float = 0.0, on_chunk=None) -> ChatResult:
        """``on_chunk(result)``: called after every streamed message (fault-injection tests act mid-stream)."""
        res = ChatResult()
        q: asyncio.Queue = asyncio.Queue()
        handler = q.put_nowait
        conn.on("data", handler)
        parser = SSEParser()
        try:
            if new_conversation:
                conn.write(create_message(Keys.NEW_CONVERSATION))
            payload = {"key": emitter_key, "messages": messages}
            if extra:
                payload.update(extra)
            res.t_start = time.perf_counter()
            conn.write(create_message(Keys.INFERENCE, payload))
            while True:
                buf = await asyncio.wait_for(q.get(), timeout)
                if slow_reader_s:
                    await asyncio.sleep(slow_reader_s)
                obj = safe_parse_json(buf)
                if isinstance(obj, dict) and "symmetryEmitterKey" in obj and res.header is None:
                    res.header = obj
                    continue
                if isinstance(obj, dict) and obj.get("key") == Keys.INFERENCE_ENDED:
                    res.ended, res.ended_key = True, obj.get("data")
                    break
                res.chunks.append(buf)
                for ev in parser.feed(buf):
                    if ev.strip().startswith("{") and '"error"' in ev[:20]:
                        res.error = ev
                    d = delta_of(ev)
                    if d:
                        if res.ttft_s is None:
                            res.ttft_s = time.perf_counter() - res.t_start
                        res.content_events += 1
                        res.text += d
                if on_chunk is not None:
                    on_chunk(res)
                if disconnect_after is not None and len(res.chunks) >= disconnect_after:
                    conn.destroy()
                    break
        finally:
            conn.off("data", handler)
            res.t_end = time.perf_counter()
        return res
