"""Optional data collection (REF ``src/provider.ts:264-297``).

When ``dataCollectionEnabled`` is true and the request's emitter key is
``"inference"``, the transcript (request messages + the assistant
completion) is written as a JSON array to
``{path}/{peer.publicKey hex}-{conversationIndex}.json``.  ``peer.publicKey``
is the provider's own (local) stream key and the index is the global
``newConversation`` counter, exactly as in the reference (SURVEY.md §2.7
item 7).  The write is asynchronous and does not delay the stream.
"""
from __future__ import annotations

import asyncio
import json
import os

from ..log import logger


def transcript_path(directory: str, local_public_key: bytes, conversation_index: int) -> str:
    return f"{directory}/{local_public_key.hex()}-{conversation_index}.json"


def transcript(messages, completion: str) -> str:
    msgs = list(messages or [])
    return json.dumps(msgs + [{"role": "assistant", "content": completion}], separators=(",", ":"),
                      ensure_ascii=False)


def _write(path: str, text: str) -> None:
    os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
    with open(path, "w", encoding="utf-8") as f:
        f.write(text)


async def save_completion(directory: str, local_public_key: bytes, conversation_index: int, messages,
                          completion: str) -> str:
    path = transcript_path(directory, local_public_key, conversation_index)
    try:
        await asyncio.to_thread(_write, path, transcript(messages, completion))
        logger.info("📝 Completion saved to file")
    except OSError as exc:
        logger.error(f"🚨 failed to save completion: {exc}")
    return path
