"""Paged KV block manager and continuous-batching scheduler.

REF: the reference has no scheduler -- every peer's ``data`` handler is an
independent async task that fetches from Ollama (``src/provider.ts:174-192``)
and ``maxConnections`` is passed to Hyperswarm and never enforced
(``src/provider.ts:38-40``).  Here all active requests
share one engine: each step is either a *prefill* batch (new prompts, chunked
to a token budget, prefill-first for TTFT) or a *decode* batch (one token for
every running sequence).  ``max_num_seqs`` is the admission limit (fed by
``maxConnections``); KV blocks are allocated on demand and a sequence is
preempted (recomputed later) when the cache runs out.
"""
from __future__ import annotations

import array
import collections
import hashlib
import itertools
import os
from dataclasses import dataclass, field

from .sequence import Sequence, SeqStatus


class BlockManager:
    """Paged KV block pool with optional automatic prefix caching.

    Prefix caching (vLLM-style, block granular): a FULL block whose KV has been computed is registered
    under the hash chain of the token ids it holds (``hash(parent_hash, tokens)``), so the identity of
    a block covers its whole prefix.  A new sequence adopts the longest run of cached blocks matching
    its prompt (reference counts: shared blocks are read-only, a sequence only ever writes positions
    >= its ``num_computed``, i.e. past the adopted blocks), and skips their prefill.  A released block
    that holds registered content goes to an LRU list instead of the free list: it stays adoptable
    until the allocator runs out of never-used blocks and evicts it.  This is what makes a chat
    provider fast on multi-turn conversations: the reference's clients resend the whole message list
    every turn (``src/provider.ts:312-316``), so each turn's prompt starts with the previous turn's
    prompt + answer.  KV writes and reads are ordered on the engine's stream, so a block released with
    a write still in flight is reused only by later launches.
    """

    def __init__(self, num_blocks: int, block_size: int, reserved: int = 1, prefix_caching: bool = False):
        # block 0 is reserved as the scratch block of padded (graph) batch rows
        self.block_size = block_size
        self.num_blocks = num_blocks
        self.free = collections.deque(range(reserved, num_blocks))
        self.reserved = reserved
        self.prefix_caching = prefix_caching
        self.ref = [0] * num_blocks
        self.block_hash: dict[int, bytes] = {}      # block -> content key (registered blocks)
        self.cached: dict[bytes, int] = {}          # content key -> block
        self.cache_gen = 0                          # blocks ever registered
        self.scope_gen: dict[bytes, int] = {}       # blocks ever registered per scope (queued misses re-look when
                                                    # their own scope's count grows: no other scope can match them)
        self.evictable: collections.OrderedDict[int, None] = collections.OrderedDict()  # ref 0, LRU order
        self.hit_tokens = 0
        self.query_tokens = 0
        self._key = os.urandom(32)

    @property
    def num_free(self) -> int:
        return len(self.free) + len(self.evictable)

    def utilization(self) -> float:
        usable = self.num_blocks - self.reserved
        return 1.0 - self.num_free / max(1, usable)

    def blocks_needed(self, seq: Sequence, num_tokens: int) -> int:
        need = (num_tokens + self.block_size - 1) // self.block_size
        return max(0, need - len(seq.block_table))

    def can_grow(self, seq: Sequence, num_tokens: int) -> bool:
        return self.blocks_needed(seq, num_tokens) <= self.num_free

    def _alloc(self) -> int:
        if self.free:
            b = self.free.popleft()
        else:  # evict the least recently released cached block
            b, _ = self.evictable.popitem(last=False)
            del self.cached[self.block_hash.pop(b)]
        self.ref[b] = 1
        return b

    def grow(self, seq: Sequence, num_tokens: int) -> None:
        n = self.blocks_needed(seq, num_tokens)
        if n > self.num_free:
            raise MemoryError("out of KV blocks")
        for _ in range(n):
            seq.block_table.append(self._alloc())

    # ---- prefix caching ------------------------------------------------------------------------
    def _chain(self, tokens: list, nblocks: int, scope: bytes = b""):
        """Content keys of the first ``nblocks`` full blocks: a keyed BLAKE2b chain over the token ids.
        Keyed with a per-process secret and collision resistant, so clients of a public provider cannot
        craft a prompt whose blocks alias another client's cached prefix (Python's ``hash`` is neither);
        rooted in the sequence's ``cache_scope`` (the client's public key), so clients never share blocks
        (no cross-client TTFT side channel either)."""
        bs, h = self.block_size, hashlib.blake2b(scope, digest_size=16, key=self._key).digest()
        for i in range(nblocks):
            blk = tokens[i * bs:(i + 1) * bs]
            h = hashlib.blake2b(h + array.array("q", blk).tobytes(), digest_size=16, key=self._key).digest()
            yield i, h

    def match_prefix(self, seq: Sequence) -> int:
        """Adopt the cached blocks of the longest matching full-block prefix of a sequence that has no
        KV yet; returns the number of tokens whose prefill is skipped.  At least one prompt token is
        always left to compute (its logits give the first output token)."""
        if not self.prefix_caching or seq.block_table or seq.num_computed:
            return 0
        # a miss is not re-queried on every schedule() (which kept the hit-rate denominator growing while a
        # prompt waited) unless blocks were cached since the last look: a queued prompt that missed while a
        # same-scope prefix was still being prefilled finds it once that prefill registered its blocks
        gen = self.scope_gen.get(seq.cache_scope, 0)
        if seq.prefix_checked and seq.prefix_epoch == gen:
            return 0
        first = not seq.prefix_checked
        seq.prefix_checked, seq.prefix_epoch = True, gen
        tokens = seq.token_ids
        target = seq.prefill_target
        nfull = max(0, target - 1) // self.block_size  # >= 1 token left to prefill
        if first:  # a re-look after new blocks were cached is the same query: its tokens count once
            self.query_tokens += target
        for _, h in self._chain(tokens, nfull, seq.cache_scope):
            b = self.cached.get(h)
            if b is None:
                break
            if self.ref[b] == 0:
                self.evictable.pop(b, None)
            self.ref[b] += 1
            seq.block_table.append(b)
        n = len(seq.block_table) * self.block_size
        seq.num_computed = n
        self.hit_tokens += n
        return n

    def register(self, seq: Sequence) -> None:
        """Register the sequence's full blocks whose KV is computed and whose token ids are known."""
        if not self.prefix_caching:
            return
        tokens = seq.token_ids
        nfull = min(seq.num_computed, len(tokens)) // self.block_size
        nfull = min(nfull, len(seq.block_table))
        for i, h in self._chain(tokens, nfull, seq.cache_scope):
            b = seq.block_table[i]
            if b in self.block_hash:       # already registered (adopted, or registered earlier)
                continue
            if h in self.cached:           # same content computed elsewhere: keep the first copy
                continue
            self.block_hash[b] = h
            self.cached[h] = b
            self.cache_gen += 1
            if seq.cache_scope not in self.scope_gen and len(self.scope_gen) >= 1 << 16:
                self.scope_gen.clear()  # bounded (one entry per client ever seen); a reset costs a re-look each
            self.scope_gen[seq.cache_scope] = self.scope_gen.get(seq.cache_scope, 0) + 1

    def release(self, seq: Sequence) -> None:
        self.register(seq)
        for b in seq.block_table:
            self.ref[b] -= 1
            if self.ref[b] > 0:
                continue
            if b in self.block_hash:
                self.evictable[b] = None
            else:
                self.free.append(b)
        seq.block_table = []


@dataclass
class SchedulerConfig:
    max_num_seqs: int = 64
    max_num_batched_tokens: int = 8192
    max_model_len: int = 8192
    enable_chunked_prefill: bool = True
    # prompt tokens per step while other sequences are decoding: mixed steps keep every running
    # sequence streaming (one token per step) while long prompts prefill in chunks
    mixed_prefill_tokens: int = 512
    # burst split (0 = off): see Scheduler._burst_budget
    burst_split_tokens: int = 1024


@dataclass
class ScheduledBatch:
    kind: str                       # "prefill" | "decode"
    seqs: list                      # sequences in batch order
    num_new_tokens: list            # tokens computed this step per sequence
    sample: list = field(default_factory=list)  # whether this step's sample is kept per sequence
    preempted: list = field(default_factory=list)

    @property
    def num_tokens(self) -> int:
        return sum(self.num_new_tokens)


class Scheduler:
    def __init__(self, cfg: SchedulerConfig, blocks: BlockManager):
        self.cfg = cfg
        self.blocks = blocks
        self.waiting: collections.deque[Sequence] = collections.deque()
        self.running: list[Sequence] = []
        self._burst_rest = 0  # prompt tokens of a split burst left for the next step

    # ------------------------------------------------------------------------------------------
    def add(self, seq: Sequence) -> None:
        if seq.num_tokens + seq.params.max_tokens > self.cfg.max_model_len:
            seq.params.max_tokens = max(1, self.cfg.max_model_len - seq.num_tokens)
        if seq.num_tokens >= self.cfg.max_model_len:
            raise ValueError(f"prompt of {seq.num_tokens} tokens exceeds max_model_len {self.cfg.max_model_len}")
        seq.status = SeqStatus.WAITING
        self.waiting.append(seq)

    def finish(self, seq: Sequence, status: SeqStatus) -> None:
        seq.status = status
        self.blocks.release(seq)
        if seq in self.running:
            self.running.remove(seq)
        else:
            try:
                self.waiting.remove(seq)
            except ValueError:
                pass

    def abort(self, request_id: str) -> Sequence | None:
        for seq in list(self.running) + list(self.waiting):
            if seq.request_id == request_id:
                self.finish(seq, SeqStatus.FINISHED_ABORTED)
                return seq
        return None

    def has_work(self) -> bool:
        return bool(self.waiting or self.running)

    @property
    def num_active(self) -> int:
        return len(self.waiting) + len(self.running)

    # ------------------------------------------------------------------------------------------
    def schedule(self) -> ScheduledBatch | None:
        """Pure prefill when nothing is decoding (best TTFT for simultaneous arrivals), pure decode when
        no prompt work is pending, otherwise a mixed step: one token for every decoding sequence plus
        prompt chunks up to ``mixed_prefill_tokens`` (decodes never stall behind a long prompt)."""
        prompt_work = bool(self.waiting) or any(s.in_prefill for s in self.running)
        decoding = any(not s.in_prefill for s in self.running)
        if not prompt_work:
            return self._schedule_decode()
        if not decoding:
            return self._schedule_prefill(self._burst_budget())
        d = self._schedule_decode()
        nd = len(d.seqs) if d is not None else 0
        budget = max(self.cfg.mixed_prefill_tokens - nd, 1)
        if self._burst_rest:  # the rest of a split burst goes in ONE step, not in mixed-step chunks
            budget = max(budget, min(self._burst_rest, self.cfg.max_num_batched_tokens - nd))
            self._burst_rest = 0
        p = self._schedule_prefill(budget)
        if d is None or not d.seqs:
            return p if p is not None else d
        if p is None:
            return d
        return ScheduledBatch("prefill", d.seqs + p.seqs, d.num_new_tokens + p.num_new_tokens, d.sample + p.sample,
                              d.preempted)

    def _burst_budget(self) -> int | None:
        """Token budget of the first step of a prompt burst (None: the configured budget).

        n prompts arriving together while nothing decodes would all get their first token after ONE
        prefill step of every prompt.  A step costs roughly a + b * tokens (Llama-3-8B, one MI355X:
        a ~3.5 ms, b ~13 us per token, profiles/prefill_len_sweep_r2.jsonl), so prefilling the first
        n // 2 + 1 prompts first and the rest in the next (mixed, whole-remainder) step moves the median request's first
        token to the smaller step and lowers the mean as well: 10 x 128 tokens, p50 TTFT 21.3 -> 14.7 ms
        (profiles/ttft_burst_split_r2.jsonl); the last requests pay one step overhead more.  Only for
        bursts that would otherwise fit one step and are large enough for the overhead to be small."""
        self._burst_rest = 0
        min_tokens = self.cfg.burst_split_tokens
        if min_tokens <= 0 or any(s.in_prefill for s in self.running):
            return None
        fresh = list(itertools.islice(self.waiting, max(0, self.cfg.max_num_seqs - len(self.running))))
        if len(fresh) < 4:
            return None
        for s in fresh:  # prefix-cache hits first (take() would adopt them anyway): split uncached work
            if not s.block_table and not s.num_computed:
                self.blocks.match_prefix(s)
        lens = [s.prefill_target - s.num_computed for s in fresh]
        total = sum(lens)
        if total < min_tokens or total > self.cfg.max_num_batched_tokens:
            return None
        first = sum(lens[: len(fresh) // 2 + 1])
        self._burst_rest = total - first
        return first

    def _schedule_prefill(self, budget: int | None = None) -> ScheduledBatch | None:
        budget = self.cfg.max_num_batched_tokens if budget is None else budget
        seqs, counts, sample = [], [], []

        def take(seq: Sequence) -> bool:
            nonlocal budget
            if not seq.block_table and not seq.num_computed:
                self.blocks.match_prefix(seq)  # adopt cached KV of a known prefix (no-op when disabled)
            remaining = seq.prefill_target - seq.num_computed
            n = min(remaining, budget) if self.cfg.enable_chunked_prefill else remaining
            if n <= 0 or n > budget:
                return False
            if not self.blocks.can_grow(seq, seq.num_computed + n):
                return False
            self.blocks.grow(seq, seq.num_computed + n)
            seqs.append(seq)
            counts.append(n)
            # the final chunk of a fresh prompt samples the first output token
            sample.append(seq.num_computed + n == seq.num_tokens and not seq.output_ids)
            budget -= n
            return True

        # 1) continue partially prefilled running sequences
        for seq in self.running:
            if seq.in_prefill and budget > 0:
                take(seq)
        # 2) admit waiting sequences
        while self.waiting and budget > 0 and len(self.running) < self.cfg.max_num_seqs:
            seq = self.waiting[0]
            if not take(seq):
                break
            self.waiting.popleft()
            seq.status = SeqStatus.RUNNING
            self.running.append(seq)
        if not seqs:
            return None
        return ScheduledBatch("prefill", seqs, counts, sample)

    def _schedule_decode(self) -> ScheduledBatch | None:
        preempted = []
        # a sequence whose in-flight tokens already reach max_tokens needs no further step
        ready = [s for s in self.running if not s.in_prefill and len(s.output_ids) + s.num_pending < s.params.max_tokens]
        # ensure a cache slot for each decoding sequence; preempt the newest on exhaustion
        ready.sort(key=lambda s: s.arrival_time)
        bs = self.blocks.block_size
        growing = [s for s in ready if s.num_computed + 1 > len(s.block_table) * bs]
        if len(growing) <= self.blocks.num_free:  # common case: every sequence gets its slot, no preemption
            for s in growing:
                self.blocks.grow(s, s.num_computed + 1)
            return ScheduledBatch("decode", ready, [1] * len(ready), [True] * len(ready), []) if ready else None
        out = []
        while ready:
            seq = ready.pop(0)
            if self.blocks.can_grow(seq, seq.num_computed + 1):
                self.blocks.grow(seq, seq.num_computed + 1)
                out.append(seq)
                continue
            victim = ready.pop() if ready else seq
            if victim is not seq:
                ready.insert(0, seq)
            self._preempt(victim)
            preempted.append(victim)
        if not out:
            return ScheduledBatch("decode", [], [], [], preempted) if preempted else None
        return ScheduledBatch("decode", out, [1] * len(out), [True] * len(out), preempted)

    def schedule_lookahead(self) -> ScheduledBatch | None:
        """Next decode step while the previous one is still in flight (pipelined decode).  Only a pure
        decode continuation qualifies: new arrivals and prefill chunks wait until the pipeline drains."""
        if self.waiting or any(s.in_prefill for s in self.running):
            return None
        b = self._schedule_decode()
        return b if b is not None and b.seqs else None

    def _preempt(self, seq: Sequence) -> None:
        self.blocks.release(seq)
        seq.num_computed = 0
        seq.prefix_checked = False
        seq.num_preemptions += 1
        seq.status = SeqStatus.WAITING
        if seq in self.running:
            self.running.remove(seq)
        self.waiting.appendleft(seq)
