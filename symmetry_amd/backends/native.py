"""NativeBackend: the in-process MI355X engine replaces the upstream server.

Every generated token becomes exactly one OpenAI ``chat.completion.chunk``
SSE event, written to the peer as one swarm message:
the first event carries ``role: assistant``, the last carries
``finish_reason`` and is followed by ``data: [DONE]``.  Per-request sampling
fields (``max_tokens``, ``temperature``, ``top_p``, ``seed``, ``stop``) are
honoured when the inference request carries them; the reference sends none
(``src/provider.ts:312-316``), so the default is greedy with a
``maxTokens`` cap.  Closing the stream (peer gone) aborts the sequence and
frees its KV blocks (item 10).
"""
from __future__ import annotations

import asyncio
import collections
import hashlib
import itertools
import os
import time

from ..engine.llm_engine import AsyncEngine, EngineConfig, LLMEngine
from ..engine.sequence import SamplingParams
from ..protocol import sse
from .base import Backend, BackendError, Chunk

_ids = itertools.count()
_TIMING_SALT = os.urandom(16)


def timing_key(content) -> str | None:
    """Request-timing key of a prompt's last message: a salted digest, so the (opt-in) timing records of a
    provider never hold its clients' prompt text."""
    if content is None:
        return None
    return hashlib.blake2b(str(content).encode(), digest_size=8, key=_TIMING_SALT).hexdigest()


class NativeBackend(Backend):
    name = "native"

    def __init__(self, config: dict, engine: LLMEngine | None = None, record_timings: bool | None = None,
                 **engine_overrides):
        self.cfg = config
        self._engine = engine
        self._overrides = engine_overrides
        self.aengine: AsyncEngine | None = None
        self.model_name = str(config.get("modelName", "llama3:8b"))
        # request-path timing of the direct stream (perf_counter = CLOCK_MONOTONIC, comparable with the
        # clients' clocks on the same host): receive -> submit -> first token on the engine thread -> first
        # output callback on the event loop -> first SSE event written; keyed by timing_key(last message).
        # Opt-in (bench / e2e runs, or SYMMETRY_REQUEST_TIMINGS=1): a serving provider records nothing.
        if record_timings is None:
            record_timings = os.environ.get("SYMMETRY_REQUEST_TIMINGS", "0") == "1"
        self.record_timings = bool(record_timings)
        self.timings: collections.deque = collections.deque(maxlen=4096)
        # fault containment: open direct streams (rid -> finish) and the listeners of a fatal engine fault
        self.fatal: str | None = None
        self._active: dict = {}
        self._fatal_listeners: list = []
        self._loop = None

    def add_fatal_listener(self, fn) -> None:
        """``fn(message)`` on the backend's event loop, once, when the engine becomes unusable."""
        if self.fatal is not None:
            fn(self.fatal)
        else:
            self._fatal_listeners.append(fn)

    def _engine_fatal(self, message: str) -> None:  # any thread
        loop = self._loop
        if loop is not None and not loop.is_closed():
            loop.call_soon_threadsafe(self._on_fatal, message)

    def _on_fatal(self, message: str) -> None:  # event loop
        if self.fatal is not None:
            return
        self.fatal = message
        # end every open stream now (the engine thread may still be blocked on the lost step)
        for finish in list(self._active.values()):
            finish(BackendError(f"provider unavailable: {message}"))
        listeners, self._fatal_listeners = self._fatal_listeners, []
        for fn in listeners:
            fn(message)

    def health_fault(self) -> str | None:
        """A lost tensor-parallel peer, if the engine's health monitor sees one right now (else None)."""
        eng = self._engine
        h = getattr(eng, "health", None) if eng is not None else None
        return (h.check() if h is not None else None) or getattr(eng, "fatal", None)

    def fail_active(self, message: str) -> int:
        """End every open stream with an error (provider shutdown); returns how many were open."""
        n = len(self._active)
        for finish in list(self._active.values()):
            finish(BackendError(message))
        return n

    @property
    def engine(self) -> LLMEngine:
        assert self.aengine is not None, "backend not started"
        return self.aengine.engine

    async def start(self) -> None:
        if self.aengine is not None:
            return
        if self._engine is None:
            ecfg = EngineConfig.from_provider(self.cfg, **self._overrides)
            self._engine = await asyncio.to_thread(LLMEngine, ecfg)
            if self._engine.device.type != "cpu":
                # start-up warmup (prefill size classes + decode hipGraphs) before the first client
                await asyncio.to_thread(self._engine.warmup)
        self.aengine = AsyncEngine(self._engine, queue_limit=int(self.cfg.get("maxBacklog") or 4096))
        self._loop = asyncio.get_running_loop()
        self._engine.add_fatal_listener(self._engine_fatal)
        self.aengine.start()

    async def stop(self) -> None:
        if self.aengine is not None:
            await asyncio.to_thread(self.aengine.stop)
            self.aengine = None

    async def stream(self, request: dict, scope: bytes = b""):
        await self.start()
        if self.fatal is not None:
            raise BackendError(f"provider unavailable: {self.fatal}")
        messages = request.get("messages") or []
        if not isinstance(messages, list):
            raise BackendError("messages must be a list")
        params = SamplingParams.from_request(request, default_max_tokens=self.engine.cfg.default_max_tokens)
        rid = f"chatcmpl-{next(_ids)}-{int(time.time() * 1000)}"
        created = int(time.time())
        first = True
        async for out in self.aengine.generate(rid, messages=messages, params=params, cache_scope=scope):
            if out.error:
                raise BackendError(out.error)
            if out.text or first or out.finished:
                ev = sse.chunk_event(rid, self.model_name, out.text, role="assistant" if first else None,
                                     finish_reason=out.finish_reason if out.finished else None, created=created)
                first = False
                yield Chunk(ev.encode("utf-8"), out.text)
            if out.finished:
                yield Chunk(sse.done_event().encode("utf-8"), "")

    async def stream_direct(self, request: dict, write, scope: bytes = b"", backlog: int | None = None) -> None:
        """The stream of :meth:`stream`, written by the engine's per-step output callback itself: each
        output becomes its SSE event and ``write(raw, delta)`` runs right there on the event loop -- no task
        wake-up and no async-generator hops per token (at 100+ concurrent clients those cost more event-loop
        time than the encoding and the encrypted send).  ``write`` returns True (accepted), False (accepted,
        but the peer is congested) or None (the peer is gone: the request is aborted).  A peer that stays
        congested for ``backlog`` outputs is a stalled reader: its request is aborted and BackendError
        raised, as the queue-based path does.  Returns when the request has finished."""
        await self.start()
        if self.fatal is not None:
            raise BackendError(f"provider unavailable: {self.fatal}")
        messages = request.get("messages") or []
        if not isinstance(messages, list):
            raise BackendError("messages must be a list")
        params = SamplingParams.from_request(request, default_max_tokens=self.engine.cfg.default_max_tokens)
        rid = f"chatcmpl-{next(_ids)}-{int(time.time() * 1000)}"
        created = int(time.time())
        limit = int(backlog or self.aengine.queue_limit)
        done = asyncio.get_running_loop().create_future()
        st = {"first": True, "congested": 0}
        tm = {}
        if self.record_timings:
            content = messages[-1].get("content") if messages and isinstance(messages[-1], dict) else None
            tm.update(key=timing_key(content), recv=request.get("_t_recv"), enter=time.perf_counter())
            self.timings.append(tm)

        def finish(exc: BaseException | None = None) -> None:
            if not done.done():
                done.set_exception(exc) if exc is not None else done.set_result(None)

        def on_output(out) -> None:
            if done.done():
                return
            if out.error:
                return finish(BackendError(out.error))
            if out.text or st["first"] or out.finished:
                first = st["first"]
                if first:
                    tm["engine_first"] = getattr(out, "t_engine", None)
                    tm["callback_first"] = time.perf_counter()
                ev = sse.chunk_event(rid, self.model_name, out.text, role="assistant" if st["first"] else None,
                                     finish_reason=out.finish_reason if out.finished else None, created=created)
                st["first"] = False
                ok = write(ev.encode("utf-8"), out.text)
                if first:
                    tm["written_first"] = time.perf_counter()
                if ok is None:  # peer gone
                    self.aengine.abort(rid)
                    return finish()
                st["congested"] = 0 if ok else st["congested"] + 1
                if st["congested"] > limit and not out.finished:
                    self.aengine.abort(rid)
                    return finish(BackendError(f"client too slow: more than {limit} outputs behind"))
            if out.finished:
                write(sse.done_event().encode("utf-8"), "")
                finish()

        self._active[rid] = finish
        try:
            self.aengine.submit(rid, on_output, messages=messages, params=params, cache_scope=scope)
        except RuntimeError as exc:  # the engine became unusable in between
            self._active.pop(rid, None)
            raise BackendError(str(exc)) from exc
        tm["submitted"] = time.perf_counter()
        try:
            await done
        finally:
            self._active.pop(rid, None)
            if not done.done() or done.cancelled():
                self.aengine.abort(rid)

    def stats(self) -> dict:
        return self.engine.metrics.summary() if self.aengine is not None else {}
