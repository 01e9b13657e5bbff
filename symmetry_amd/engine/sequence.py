"""Request / sequence state for the continuous-batching engine.

REF equivalence: one ``inference`` message (``src/types.ts:28-31``,
handled at ``src/provider.ts:184-189``) becomes one :class:`Sequence`.  The
reference sends no sampling parameters upstream (``src/provider.ts:312-316``),
so the defaults here are greedy with a max-new-tokens cap;
OpenAI-style fields in the request override them.
"""
from __future__ import annotations

import enum
import itertools
import time
from dataclasses import dataclass, field


@dataclass
class SamplingParams:
    max_tokens: int = 256
    temperature: float = 0.0
    top_p: float = 1.0
    top_k: int = 0
    seed: int | None = None
    ignore_eos: bool = False
    stop: tuple = ()
    stop_token_ids: tuple = ()

    @classmethod
    def from_request(cls, body: dict | None, default_max_tokens: int = 256) -> "SamplingParams":
        body = body or {}
        p = cls(max_tokens=int(body.get("max_tokens") or body.get("max_completion_tokens") or default_max_tokens))
        if body.get("temperature") is not None:
            p.temperature = max(0.0, float(body["temperature"]))
        if body.get("top_p") is not None:
            p.top_p = float(body["top_p"])
        if body.get("top_k") is not None:
            p.top_k = int(body["top_k"])
        if body.get("seed") is not None:
            p.seed = int(body["seed"])
        if body.get("ignore_eos") is not None:
            p.ignore_eos = bool(body["ignore_eos"])
        stop = body.get("stop")
        if isinstance(stop, str):
            p.stop = (stop,)
        elif isinstance(stop, (list, tuple)):
            p.stop = tuple(str(s) for s in stop)
        return p


class SeqStatus(enum.Enum):
    WAITING = "waiting"
    RUNNING = "running"
    FINISHED_STOPPED = "stop"
    FINISHED_LENGTH = "length"
    FINISHED_ABORTED = "abort"
    FINISHED_ERROR = "error"

    @property
    def finished(self) -> bool:
        return self.value in ("stop", "length", "abort", "error")


_ids = itertools.count()


@dataclass
class Sequence:
    request_id: str
    prompt_ids: list
    params: SamplingParams
    eos_ids: tuple = ()
    seq_id: int = field(default_factory=lambda: next(_ids))
    output_ids: list = field(default_factory=list)
    status: SeqStatus = SeqStatus.WAITING
    block_table: list = field(default_factory=list)
    num_computed: int = 0          # tokens whose KV is in the cache (or enqueued to be written)
    num_pending: int = 0           # sampled tokens launched on the GPU but not yet seen by the host
    arrival_time: float = field(default_factory=time.perf_counter)
    first_token_time: float | None = None
    last_token_time: float | None = None
    finish_time: float | None = None
    num_preemptions: int = 0
    sampling_seed: int = 0
    output_text: str = ""
    cache_scope: bytes = b""       # prefix-cache namespace (client identity)
    prefix_checked: bool = False   # the prefix cache was consulted for the current (fresh) KV state
    prefix_epoch: int = -1         # the prefix cache's size at that look (a grown cache is re-queried)

    @property
    def token_ids(self) -> list:
        return self.prompt_ids + self.output_ids

    def token_slice(self, start: int, n: int) -> list:
        """token_ids[start:start + n] without concatenating the whole prompt + output list."""
        npr = len(self.prompt_ids)
        if start + n <= npr:
            return self.prompt_ids[start:start + n]
        if start >= npr:
            return self.output_ids[start - npr:start - npr + n]
        return self.prompt_ids[start:] + self.output_ids[:start + n - npr]

    @property
    def num_tokens(self) -> int:
        return len(self.prompt_ids) + len(self.output_ids)

    @property
    def prefill_target(self) -> int:
        """Tokens whose KV must be cached before decoding: the whole prompt for a fresh
        sequence; everything but the newest sampled token after a preemption (recompute)."""
        return self.num_tokens - 1 if self.output_ids else self.num_tokens

    @property
    def in_prefill(self) -> bool:
        return self.num_computed < self.prefill_target

    def append(self, token: int, now: float) -> None:
        self.output_ids.append(int(token))
        if self.first_token_time is None:
            self.first_token_time = now
        self.last_token_time = now

    def check_stop(self) -> SeqStatus | None:
        if self.output_ids and not self.params.ignore_eos:
            t = self.output_ids[-1]
            if t in self.eos_ids or t in self.params.stop_token_ids:
                return SeqStatus.FINISHED_STOPPED
        if len(self.output_ids) >= self.params.max_tokens:
            return SeqStatus.FINISHED_LENGTH
        return None

    @property
    def ttft(self) -> float | None:
        return None if self.first_token_time is None else self.first_token_time - self.arrival_time
