"""A local OpenAI-compatible streaming server standing in for Ollama (BASELINE config 1).

``POST {path}`` with ``{"model", "messages", "stream": true}`` streams
``chat.completion.chunk`` SSE events (one per word of a deterministic reply)
and ``data: [DONE]`` -- the shape Ollama's ``/v1/chat/completions`` emits.
Knobs for fault injection: ``status`` (non-2xx), ``delay_s`` between chunks,
``coalesce`` (several events per HTTP chunk, the case the reference's
first-``data:`` parser drops), ``fail_after`` (drop the connection mid-stream).
"""
from __future__ import annotations

import asyncio
import json
import time

from aiohttp import web


def reply_for(messages) -> str:
    last = ""
    for m in messages or []:
        if m.get("role") == "user":
            last = str(m.get("content", ""))
    return f"Echo from mock ollama: {last}".strip()


class MockOllama:
    def __init__(self, host: str = "127.0.0.1", port: int = 0, path: str = "/v1/chat/completions",
                 delay_s: float = 0.0, status: int = 200, coalesce: int = 1, fail_after: int | None = None,
                 api_key: str | None = None):
        self.host, self.port, self.path = host, port, path
        self.delay_s, self.status, self.coalesce, self.fail_after = delay_s, status, coalesce, fail_after
        self.api_key = api_key
        self.requests: list[dict] = []
        self.headers: list[dict] = []
        self.cancelled = 0
        self._runner: web.AppRunner | None = None

    async def start(self) -> int:
        app = web.Application()
        app.router.add_post(self.path, self._chat)
        self._runner = web.AppRunner(app)
        await self._runner.setup()
        site = web.TCPSite(self._runner, self.host, self.port)
        await site.start()
        self.port = site._server.sockets[0].getsockname()[1]
        return self.port

    async def stop(self) -> None:
        if self._runner is not None:
            await self._runner.cleanup()

    @staticmethod
    def event(content: str, model: str, finish=None) -> str:
        obj = {"id": "chatcmpl-mock", "object": "chat.completion.chunk", "created": int(time.time()), "model": model,
               "system_fingerprint": "fp_ollama",
               "choices": [{"index": 0, "delta": {"role": "assistant", "content": content},
                            "finish_reason": finish}]}
        return "data: " + json.dumps(obj) + "\n\n"

    async def _chat(self, request: web.Request) -> web.StreamResponse:
        body = await request.json()
        self.requests.append(body)
        self.headers.append(dict(request.headers))
        if self.status != 200:
            return web.Response(status=self.status, text="mock failure")
        model = body.get("model", "mock")
        words = reply_for(body.get("messages")).split(" ")
        events = [self.event(w if i == 0 else " " + w, model) for i, w in enumerate(words)]
        events.append(self.event("", model, finish="stop"))
        events.append("data: [DONE]\n\n")
        resp = web.StreamResponse(headers={"Content-Type": "text/event-stream"})
        await resp.prepare(request)
        sent = 0
        try:
            for i in range(0, len(events), self.coalesce):
                if self.fail_after is not None and sent >= self.fail_after:
                    request.transport.close()
                    return resp
                await resp.write("".join(events[i:i + self.coalesce]).encode())
                sent += 1
                if self.delay_s:
                    await asyncio.sleep(self.delay_s)
            await resp.write_eof()
        except (ConnectionResetError, asyncio.CancelledError):
            self.cancelled += 1
            raise
        return resp
