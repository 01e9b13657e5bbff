"""Message codec (REF ``src/utils.ts:4-14``).

Every swarm message is one JSON document ``{"key": ..., "data": ...}``
(``createMessage``).  ``data`` is omitted when undefined, exactly as
``JSON.stringify`` drops ``undefined`` (so ``pong`` is ``{"key":"pong"}``,
SURVEY.md §2.2).  Node ``Buffer`` values serialise as
``{"type":"Buffer","data":[...]}``; :func:`buffer_json` / :func:`from_buffer_json`
reproduce that form for the provider's challenge (``src/provider.ts:97-101``).
"""
from __future__ import annotations

import json
from typing import Any

_UNDEFINED = object()


def _compact(obj) -> str:
    # JSON.stringify: no spaces, non-ASCII kept verbatim
    return json.dumps(obj, separators=(",", ":"), ensure_ascii=False)


def create_message(key: str, data: Any = _UNDEFINED) -> str:
    """``createMessage(key, data?)``; pass nothing for JS ``undefined``, ``None`` for ``null``."""
    if data is _UNDEFINED:
        return _compact({"key": key})
    return _compact({"key": key, "data": data})


def safe_parse_json(data) -> Any | None:
    """``safeParseJson``: parse or return None (never raises)."""
    try:
        if isinstance(data, (bytes, bytearray, memoryview)):
            data = bytes(data).decode("utf-8")
        return json.loads(data)
    except Exception:
        return None


def buffer_json(b: bytes) -> dict:
    """Node's ``Buffer.toJSON()`` form."""
    return {"type": "Buffer", "data": list(bytes(b))}


def from_buffer_json(obj) -> bytes | None:
    if isinstance(obj, dict) and obj.get("type") == "Buffer" and isinstance(obj.get("data"), list):
        try:
            return bytes(obj["data"])
        except (ValueError, TypeError):
            return None
    return None


def emitter_header(emitter_key: str) -> str:
    """Raw (not {key,data}) stream header, ``src/provider.ts:234-238``."""
    return _compact({"symmetryEmitterKey": emitter_key})
