"""ProxyBackend: the reference's behaviour -- relay an upstream OpenAI-compatible server.

REF ``src/provider.ts:195-257, 299-319``: POST
``{apiProtocol}://{apiHostname}:{apiPort}{apiPath}`` with
``Authorization: Bearer <apiKey>`` and body ``{model: modelName, messages,
stream: true}``; throw on non-2xx; relay every upstream body chunk verbatim;
accumulate the completion with ``safeParseStreamResponse`` +
``getChatDataFromProvider`` (so a chunk carrying several SSE events
contributes only its first, exactly like the reference).

Deviations (documented): closing the async generator (client
gone) cancels the upstream request (REF keeps reading, item 10); the saved
completion is assembled by a real SSE parser (every event of every chunk)
because the reference's first-``data:`` parse silently truncates transcripts
whenever the upstream coalesces events into one HTTP chunk (item 8).  The
bytes relayed to the peer are untouched.  ``completionParser: ref`` in
provider.yaml restores the reference's parse.
"""
from __future__ import annotations

import aiohttp

from ..protocol.sse import SSEParser, delta_of, get_chat_data_from_provider, safe_parse_stream_response
from .base import Backend, BackendError, Chunk


class ProxyBackend(Backend):
    name = "proxy"

    def __init__(self, config: dict, completion_parser: str | None = None, timeout_s: float = 600.0):
        self.cfg = config
        self.completion_parser = completion_parser or str(config.get("completionParser", "sse"))
        self.timeout = aiohttp.ClientTimeout(total=timeout_s, sock_read=timeout_s)
        self._session: aiohttp.ClientSession | None = None

    async def start(self) -> None:
        if self._session is None:
            self._session = aiohttp.ClientSession(timeout=self.timeout)

    async def stop(self) -> None:
        if self._session is not None:
            await self._session.close()
            self._session = None

    def build_stream_request(self, messages) -> tuple[str, dict, dict]:
        c = self.cfg
        url = f"{c['apiProtocol']}://{c['apiHostname']}:{int(c['apiPort'])}{c['apiPath']}"
        headers = {"Content-Type": "application/json", "Authorization": f"Bearer {c.get('apiKey')}"}
        body = {"model": c.get("modelName"), "messages": messages, "stream": True}
        if messages is None:
            body.pop("messages")
        return url, headers, body

    async def stream(self, request: dict, scope: bytes = b""):
        await self.start()
        url, headers, body = self.build_stream_request(request.get("messages"))
        provider = str(self.cfg.get("apiProvider"))
        parser = SSEParser() if self.completion_parser == "sse" else None
        async with self._session.post(url, json=body, headers=headers) as resp:
            if resp.status < 200 or resp.status >= 300:
                raise BackendError(f"Server responded with status code: {resp.status}")
            async for chunk in resp.content.iter_any():
                if parser is not None:
                    delta = "".join(d for d in (delta_of(e) for e in parser.feed(chunk)) if d)
                else:
                    d = get_chat_data_from_provider(provider, safe_parse_stream_response(chunk))
                    delta = "" if d is None else d
                yield Chunk(bytes(chunk), delta)
