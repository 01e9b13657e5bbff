"""OpenAI-style Server-Sent-Events: the encoder used by the native backend and
the REF-compatible parsers used by the proxy backend.

REF parsing (``src/utils.ts:16-52``):

* :func:`safe_parse_stream_response` parses only the text between the first
  two ``data:`` markers of a chunk -- a chunk carrying several events
  contributes only its first event to the completion (the reference's quirk;
  SURVEY.md §2.7 item 8).
* :func:`get_chat_data_from_provider` extracts the content delta per upstream
  flavour: ollama/openwebui ``choices[0].delta.content or ''``; llamacpp
  ``content`` (None when absent); everything else ``choices[0].delta.content``.

NEW: :class:`SSEParser` is a correct incremental parser (multi-event chunks,
events split across chunks), and :func:`chunk_event` / :func:`done_event`
emit exactly one SSE event per swarm message -- one per generated token.
"""
from __future__ import annotations

import json
import time
from typing import Any

from .codec import safe_parse_json
from .keys import API_PROVIDERS


def is_stream_with_data_prefix(s: str) -> bool:
    return s.startswith("data:")


def safe_parse_stream_response(s) -> Any | None:
    if isinstance(s, (bytes, bytearray)):
        s = bytes(s).decode("utf-8", errors="replace")
    try:
        if is_stream_with_data_prefix(s):
            return json.loads(s.split("data:")[1])
        return json.loads(s)
    except Exception:
        return None


def get_chat_data_from_provider(provider: str, data: Any) -> str | None:
    if provider in (API_PROVIDERS["Ollama"], API_PROVIDERS["OpenWebUI"]):
        try:
            c = data["choices"][0].get("delta", {}).get("content") if data else None
        except (KeyError, IndexError, TypeError, AttributeError):
            c = None
        return c if c else ""
    if provider == API_PROVIDERS["LlamaCpp"]:
        return data.get("content") if isinstance(data, dict) else None
    try:
        c = data["choices"][0]["delta"].get("content") if data else None
    except (KeyError, IndexError, TypeError, AttributeError):
        return ""
    if c == "undefined":
        return ""
    return c if c else ""


class SSEParser:
    """Incremental SSE decoder: feed raw bytes, get complete ``data:`` payloads."""

    def __init__(self):
        self.buf = ""

    def feed(self, chunk) -> list[str]:
        if isinstance(chunk, (bytes, bytearray, memoryview)):
            chunk = bytes(chunk).decode("utf-8", errors="replace")
        self.buf += chunk.replace("\r\n", "\n")
        events = []
        while "\n\n" in self.buf:
            raw, self.buf = self.buf.split("\n\n", 1)
            data = [ln[5:].lstrip(" ") for ln in raw.split("\n") if ln.startswith("data:")]
            if data:
                events.append("\n".join(data))
        return events


def delta_of(payload: str) -> str | None:
    """Content delta of one parsed ``data:`` payload (None for [DONE] / non-JSON)."""
    if payload.strip() == "[DONE]":
        return None
    obj = safe_parse_json(payload)
    if not isinstance(obj, dict):
        return None
    try:
        return obj["choices"][0]["delta"].get("content") or ""
    except (KeyError, IndexError, TypeError, AttributeError):
        return obj.get("content") if isinstance(obj.get("content"), str) else ""


def _dump(obj) -> str:
    return json.dumps(obj, separators=(",", ":"), ensure_ascii=False)


_esc = json.encoder.encode_basestring  # the C string encoder json.dumps(..., ensure_ascii=False) uses


def chunk_event(completion_id: str, model: str, content: str | None = None, *, role: str | None = None,
                finish_reason: str | None = None, created: int | None = None, usage: dict | None = None) -> str:
    if role is None and usage is None and content is not None:
        # per-token fast path (one event per token per client on the serving hot path): the same bytes as
        # the generic encoding below, assembled from C-escaped strings instead of a json.dumps of a dict
        return ('data: {"id":' + _esc(completion_id) + ',"object":"chat.completion.chunk","created":'
                + str(int(created if created is not None else time.time())) + ',"model":' + _esc(model)
                + ',"system_fingerprint":"symmetry_amd","choices":[{"index":0,"delta":{"content":' + _esc(content)
                + '},"finish_reason":' + ("null" if finish_reason is None else _esc(finish_reason)) + "}]}\n\n")
    delta: dict = {}
    if role is not None:
        delta["role"] = role
    if content is not None:
        delta["content"] = content
    obj = {
        "id": completion_id,
        "object": "chat.completion.chunk",
        "created": int(created if created is not None else time.time()),
        "model": model,
        "system_fingerprint": "symmetry_amd",
        "choices": [{"index": 0, "delta": delta, "finish_reason": finish_reason}],
    }
    if usage is not None:
        obj["usage"] = usage
    return "data: " + _dump(obj) + "\n\n"


def error_event(message: str, code: str = "inference_error") -> str:
    return "data: " + _dump({"error": {"message": message, "type": code}}) + "\n\n"


def done_event() -> str:
    return "data: [DONE]\n\n"
