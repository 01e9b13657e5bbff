"""Tokenizers, chat templates and incremental (streaming) detokenization.

The reference forwards ``messages`` to an upstream server that owns the
tokenizer (``src/provider.ts:312-316``).  The native provider applies the
model's chat template itself:

* :class:`HFTokenizer` wraps a HuggingFace ``tokenizer.json`` (``tokenizers``
  library) when a checkpoint directory provides one;
* :class:`ByteTokenizer` is the deterministic offline fallback used with
  random-init weights: ids 0..255 are UTF-8 bytes, the model's special tokens
  keep their ids, and every other id decodes to one printable ASCII character
  so random-weight generations stream visible text.
"""
from __future__ import annotations

import codecs
import json
import os

from ..models.config import ModelConfig

LLAMA3_SPECIALS = {
    "<|begin_of_text|>": 128000,
    "<|end_of_text|>": 128001,
    "<|start_header_id|>": 128006,
    "<|end_header_id|>": 128007,
    "<|eot_id|>": 128009,
}


class Tokenizer:
    bos_id: int
    eos_ids: tuple
    vocab_size: int
    chat_format: str = "llama3"
    specials: dict

    def encode(self, text: str) -> list[int]:
        raise NotImplementedError

    def decode_bytes(self, ids) -> bytes:
        raise NotImplementedError

    def decode(self, ids) -> str:
        return self.decode_bytes(ids).decode("utf-8", errors="replace")

    def special(self, name: str) -> int:
        return self.specials[name]

    def apply_chat_template(self, messages: list, add_generation_prompt: bool = True) -> list[int]:
        ids: list[int] = []
        if self.chat_format == "mistral":
            ids.append(self.bos_id)
            sys_prefix = ""
            for m in messages:
                role, content = m.get("role", "user"), str(m.get("content", ""))
                if role == "system":
                    sys_prefix += content + "\n\n"
                elif role == "user":
                    ids += self.encode(f"[INST] {sys_prefix}{content} [/INST]")
                    sys_prefix = ""
                else:
                    ids += self.encode(content)
                    ids += list(self.eos_ids[:1])
            return ids
        ids.append(self.special("<|begin_of_text|>"))
        for m in messages:
            ids.append(self.special("<|start_header_id|>"))
            ids += self.encode(str(m.get("role", "user")))
            ids.append(self.special("<|end_header_id|>"))
            ids += self.encode("\n\n" + str(m.get("content", "")))
            ids.append(self.special("<|eot_id|>"))
        if add_generation_prompt:
            ids.append(self.special("<|start_header_id|>"))
            ids += self.encode("assistant")
            ids.append(self.special("<|end_header_id|>"))
            ids += self.encode("\n\n")
        return ids


class ByteTokenizer(Tokenizer):
    def __init__(self, cfg: ModelConfig):
        self.vocab_size = cfg.vocab_size
        self.chat_format = cfg.chat_format
        self.bos_id = cfg.bos_token_id
        self.eos_ids = tuple(cfg.eos_token_ids)
        if cfg.vocab_size > max(LLAMA3_SPECIALS.values()) and cfg.chat_format == "llama3":
            self.specials = dict(LLAMA3_SPECIALS)
        else:
            top = cfg.vocab_size
            names = ["<|begin_of_text|>", "<|end_of_text|>", "<|start_header_id|>", "<|end_header_id|>",
                     "<|eot_id|>"]
            self.specials = {n: top - 1 - i for i, n in enumerate(names)}
            self.specials["<|begin_of_text|>"] = cfg.bos_token_id
            if cfg.eos_token_ids:
                self.specials["<|eot_id|>"] = cfg.eos_token_ids[-1]
                self.specials["<|end_of_text|>"] = cfg.eos_token_ids[0]
        self._special_ids = set(self.specials.values()) | set(self.eos_ids) | {self.bos_id}

    def encode(self, text: str) -> list[int]:
        return list(text.encode("utf-8"))

    def decode_bytes(self, ids) -> bytes:
        out = bytearray()
        for t in ids:
            t = int(t)
            if t < 256:
                out.append(t)
            elif t in self._special_ids:
                continue
            else:
                out.append(0x21 + (t % 94))
        return bytes(out)


class HFTokenizer(Tokenizer):
    def __init__(self, path: str, cfg: ModelConfig):
        from tokenizers import Tokenizer as _Tok

        tj = path if path.endswith(".json") else os.path.join(path, "tokenizer.json")
        self.tok = _Tok.from_file(tj)
        self.vocab_size = self.tok.get_vocab_size(with_added_tokens=True)
        self.chat_format = cfg.chat_format
        self.bos_id = cfg.bos_token_id
        self.eos_ids = tuple(cfg.eos_token_ids)
        self.specials = {}
        for name in LLAMA3_SPECIALS:
            i = self.tok.token_to_id(name)
            if i is not None:
                self.specials[name] = i
        cfgf = os.path.join(os.path.dirname(tj), "tokenizer_config.json")
        if os.path.exists(cfgf):
            with open(cfgf) as f:
                tc = json.load(f)
            b = tc.get("bos_token")
            if isinstance(b, str) and self.tok.token_to_id(b) is not None:
                self.bos_id = self.tok.token_to_id(b)

    def encode(self, text: str) -> list[int]:
        return self.tok.encode(text, add_special_tokens=False).ids

    def decode_bytes(self, ids) -> bytes:
        return self.tok.decode([int(i) for i in ids], skip_special_tokens=True).encode("utf-8")


def load_tokenizer(cfg: ModelConfig, path: str | None = None) -> Tokenizer:
    if path and (os.path.exists(path) if path.endswith(".json") else os.path.exists(os.path.join(path, "tokenizer.json"))):
        return HFTokenizer(path, cfg)
    return ByteTokenizer(cfg)


class IncrementalDetokenizer:
    """Turns a growing token list into UTF-8-complete text deltas.

    Trailing bytes of an incomplete UTF-8 sequence are held back, so every
    streamed SSE event carries valid text.  Cost per
    token is O(1) for byte-level vocabularies and O(window) for BPE ones
    (decode of a short suffix window, the "prefix offset" method).
    """

    WINDOW = 6

    def __init__(self, tok: Tokenizer):
        self.tok = tok
        self.ids: list[int] = []
        self._utf8 = codecs.getincrementaldecoder("utf-8")(errors="replace")
        self.text = ""
        self._byte_level = isinstance(tok, ByteTokenizer)
        self._prefix = 0      # start of the decode window
        self._read = 0        # tokens already turned into emitted text

    def add(self, token: int) -> str:
        self.ids.append(int(token))
        if self._byte_level:
            delta = self._utf8.decode(self.tok.decode_bytes((token,)))
            self.text += delta
            return delta
        prefix_text = self.tok.decode(self.ids[self._prefix:self._read])
        new_text = self.tok.decode(self.ids[self._prefix:])
        if new_text.endswith("\ufffd") or len(new_text) <= len(prefix_text):
            return ""
        delta = new_text[len(prefix_text):]
        self._read = len(self.ids)
        self._prefix = max(0, self._read - self.WINDOW)
        self.text += delta
        return delta

    def flush(self) -> str:
        if self._byte_level:
            rest = self._utf8.decode(b"", final=True)
        else:
            prefix_text = self.tok.decode(self.ids[self._prefix:self._read])
            full = self.tok.decode(self.ids[self._prefix:])
            rest = full[len(prefix_text):] if len(full) > len(prefix_text) else ""
            self._read = len(self.ids)
        self.text += rest
        return rest
