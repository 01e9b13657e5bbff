"""Inference backend interface used by the provider node.

A backend turns one ``inference`` request (``{"key": emitterKey, "messages":
[...] , ...}``, REF ``src/types.ts:28-31``) into a stream of :class:`Chunk`
objects.  Each chunk carries the exact bytes to relay to the peer and the
assistant-text delta it contributes to the completion (for data collection).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import AsyncIterator


@dataclass
class Chunk:
    raw: bytes          # bytes written to the peer as one swarm message
    delta: str = ""     # assistant text carried by this chunk


class BackendError(Exception):
    pass


class Backend:
    name = "base"

    async def start(self) -> None:
        pass

    async def stop(self) -> None:
        pass

    def stream(self, request: dict, scope: bytes = b"") -> AsyncIterator[Chunk]:  # pragma: no cover - interface
        """Stream one chat request.  ``scope``: identity of the requesting client (the peer's public key);
        backends that cache per-client state (the native engine's KV prefix cache) keep it per scope."""
        raise NotImplementedError

    def stats(self) -> dict:
        return {}
