"""Local OpenAI-compatible HTTP endpoint of the native engine (with ``apiProvider:
native`` the ``apiHostname`` / ``apiPort`` / ``apiPath`` fields become the address of the API the engine
emulates, so local tools that spoke to Ollama keep working against the MI355X engine).

Enabled by ``serveHttp: true`` in provider.yaml (or ``symmetry-cli`` with ``SYMMETRY_SERVEHTTP=true``).
Routes:
  POST <apiPath> (default /v1/chat/completions)  stream=true -> SSE chunk per token + [DONE];
                                                 stream=false -> one chat.completion object
  GET  /v1/models                                the served model
  GET  /metrics                                  engine + provider counters (JSON)
Requests share the engine (and its continuous batching) with swarm peers.  ``apiKey``, when set, is
required as ``Authorization: Bearer <apiKey>``.
"""
from __future__ import annotations

import json
import time

from aiohttp import web

from ..backends.base import Backend, BackendError
from ..protocol import sse


class LocalAPIServer:
    def __init__(self, backend: Backend, model_name: str, host: str = "127.0.0.1", port: int = 0,
                 path: str = "/v1/chat/completions", api_key: str | None = None, stats=None):
        self.backend, self.model_name = backend, model_name
        self.host, self.port, self.path = host, int(port), path
        self.api_key = api_key or None
        self.stats = stats or backend.stats
        self._runner: web.AppRunner | None = None

    async def start(self) -> int:
        app = web.Application()
        app.router.add_post(self.path, self._chat)
        app.router.add_get("/v1/models", self._models)
        app.router.add_get("/metrics", self._metrics)
        self._runner = web.AppRunner(app)
        await self._runner.setup()
        site = web.TCPSite(self._runner, self.host, self.port)
        await site.start()
        self.port = site._server.sockets[0].getsockname()[1]  # actual port when 0 was requested
        return self.port

    async def stop(self) -> None:
        if self._runner is not None:
            await self._runner.cleanup()
            self._runner = None

    def _authorized(self, request: web.Request) -> bool:
        return self.api_key is None or request.headers.get("Authorization") == f"Bearer {self.api_key}"

    async def _models(self, request: web.Request) -> web.Response:
        return web.json_response({"object": "list", "data": [
            {"id": self.model_name, "object": "model", "created": 0, "owned_by": "symmetry"}]})

    async def _metrics(self, request: web.Request) -> web.Response:
        return web.json_response(self.stats())

    async def _chat(self, request: web.Request) -> web.StreamResponse:
        if not self._authorized(request):
            return web.json_response({"error": {"message": "invalid api key", "type": "auth"}}, status=401)
        try:
            body = await request.json()
        except (json.JSONDecodeError, ValueError):
            return web.json_response({"error": {"message": "invalid JSON body", "type": "invalid_request"}},
                                     status=400)
        if not isinstance(body, dict) or not isinstance(body.get("messages"), list):
            return web.json_response({"error": {"message": "messages must be a list", "type": "invalid_request"}},
                                     status=400)
        if body.get("stream"):
            resp = web.StreamResponse(headers={"Content-Type": "text/event-stream", "Cache-Control": "no-cache"})
            await resp.prepare(request)
            try:
                async for chunk in self.backend.stream(body):
                    await resp.write(chunk.raw)
            except BackendError as exc:
                await resp.write(sse.error_event(str(exc)).encode("utf-8"))
            except ConnectionResetError:  # client went away: the backend generator aborts the sequence
                pass
            return resp
        text, finish = [], "stop"
        try:
            async for chunk in self.backend.stream(body):
                text.append(chunk.delta)
                for ev in sse.SSEParser().feed(chunk.raw):
                    if ev.strip().startswith("{"):
                        fr = (json.loads(ev).get("choices") or [{}])[0].get("finish_reason")
                        finish = fr or finish
        except BackendError as exc:
            return web.json_response({"error": {"message": str(exc), "type": "server_error"}}, status=500)
        content = "".join(text)
        return web.json_response({
            "id": f"chatcmpl-{int(time.time() * 1000)}", "object": "chat.completion", "created": int(time.time()),
            "model": self.model_name,
            "choices": [{"index": 0, "message": {"role": "assistant", "content": content}, "finish_reason": finish}],
        })
