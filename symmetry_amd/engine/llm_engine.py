"""The native inference engine: model + paged KV cache + scheduler + streaming outputs.

This replaces the external Ollama process that the reference proxies to
(``src/provider.ts:206-214``): the provider submits chat requests here and
receives one :class:`RequestOutput` per generated token.

:class:`LLMEngine` is synchronous (``step()``); :class:`AsyncEngine` runs it
on a dedicated thread and bridges outputs into asyncio with bounded
per-request queues, so slow peers never stall the GPU loop (SURVEY.md §7.4
item 6).
"""
from __future__ import annotations

import asyncio
import collections
import hashlib
import os
import queue
import sys
import threading
import time
import traceback
from dataclasses import dataclass, field

import torch

from ..models.config import ModelConfig, resolve
from ..models.transformer import KVCache, TransformerLM
from ..models.weights import ModelWeights, ShardSpec, load_hf_weights, random_weights
from ..utils.metrics import EngineMetrics
from .model_runner import MAX_DECODE_ROWS, ModelRunner
from .scheduler import BlockManager, Scheduler, SchedulerConfig
from .sequence import SamplingParams, Sequence, SeqStatus
from .tokenizer import IncrementalDetokenizer, load_tokenizer


@dataclass
class EngineConfig:
    model: str = "llama3:8b"
    weights: str = "random"              # "random" or a HF safetensors directory
    tokenizer: str | None = None
    device: str = "auto"                 # "auto" | "cuda" | "cuda:N" | "cpu"
    seed: int = 0
    max_num_seqs: int = 64               # admission limit (maxConnections)
    max_num_batched_tokens: int = 8192
    max_model_len: int = 8192
    block_size: int = 64
    kv_cache_fraction: float = 0.85      # of the HBM left after weights + workspace
    num_kv_blocks: int | None = None
    use_graphs: bool = True
    default_max_tokens: int = 256
    tp_size: int = 1
    tp_rank: int = 0
    ep_size: int = 1
    ep_rank: int = 0
    weight_init: str = "auto"            # "full" | "shard" | "auto"
    pipeline: bool = True                # enqueue decode step N+1 before step N's tokens reach the host
    mixed_prefill_tokens: int = 512      # prompt-chunk budget of steps that also carry decodes
    decode_weights: str = "auto"         # "preshuffled" | "replace" | "shared" | "auto": MFMA-ordered decode weights
    enable_prefix_caching: bool = True   # adopt cached KV blocks of a known prompt prefix (multi-turn chats)
    # a burst of >= 4 prompts totalling >= this many tokens, arriving while nothing decodes, prefills its
    # first n // 2 + 1 prompts in one step and the rest in the next (0 = one step for the whole burst)
    burst_split_tokens: int = int(os.environ.get("SYMMETRY_BURST_SPLIT", "1024"))
    # an idle engine that receives a request waits until no further request has arrived for
    # arrival_quiet_us (at most arrival_window_us) before its first step, so requests sent together by many
    # clients -- spread over a millisecond or two by the network and the per-peer decryption -- prefill as one
    # burst instead of one lone prompt followed by the rest (0 = off)
    arrival_quiet_us: int = int(os.environ.get("SYMMETRY_ARRIVAL_QUIET_US", "300"))
    arrival_window_us: int = int(os.environ.get("SYMMETRY_ARRIVAL_WINDOW_US", "2000"))
    model_config: ModelConfig | None = None

    @classmethod
    def from_provider(cls, cfg: dict, **overrides) -> "EngineConfig":
        """Map provider.yaml fields (REF schema + optional engine fields)."""
        ec = cls(model=str(cfg.get("modelName", "llama3:8b")))
        mc = cfg.get("maxConnections")
        if mc:
            ec.max_num_seqs = int(mc)
        m = {"weights": "weights", "tokenizer": "tokenizer", "seed": "seed", "maxBatchTokens": "max_num_batched_tokens",
             "maxModelLen": "max_model_len", "kvCacheFraction": "kv_cache_fraction", "blockSize": "block_size",
             "maxTokens": "default_max_tokens", "tensorParallelSize": "tp_size", "expertParallelSize": "ep_size",
             "device": "device",
             "useGraphs": "use_graphs", "numKvBlocks": "num_kv_blocks", "decodeWeights": "decode_weights",
             "prefillChunk": "mixed_prefill_tokens",
             "enablePrefixCaching": "enable_prefix_caching", "burstSplitTokens": "burst_split_tokens",
             "arrivalQuietUs": "arrival_quiet_us", "arrivalWindowUs": "arrival_window_us"}
        for k, attr in m.items():
            if cfg.get(k) is not None:
                cur, val = getattr(ec, attr), cfg[k]
                if isinstance(cur, bool) and isinstance(val, str):  # env overrides arrive as strings
                    val = val.strip().lower() in ("1", "true", "yes", "on")
                setattr(ec, attr, type(cur)(val) if cur is not None else val)
        for k, v in overrides.items():
            setattr(ec, k, v)
        return ec


@dataclass
class RequestOutput:
    request_id: str
    token_ids: list
    text: str
    finished: bool = False
    finish_reason: str | None = None
    error: str | None = None
    seq: Sequence | None = field(default=None, repr=False)


def _pick_device(spec: str) -> torch.device:
    if spec == "auto":
        return torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")
    return torch.device(spec)


_PROFILE_DIR = os.environ.get("SYMMETRY_PROFILE")


class LLMEngine:
    def __init__(self, cfg: EngineConfig, tp_comm=None, ep_comm=None, cpu_group=None):
        self.cfg = cfg
        if cfg.tp_size > 1 and tp_comm is None:
            raise ValueError(f"tp_size {cfg.tp_size} needs a TP communicator: build TP engines with "
                             "parallel.launch.init_tp_engine under torchrun (symmetry-cli starts it)")
        self.device = _pick_device(cfg.device)
        self.model_cfg = cfg.model_config or self._model_config(cfg)
        mcfg = self.model_cfg
        max_model_len = min(cfg.max_model_len, mcfg.max_position)
        self.metrics = EngineMetrics()
        shard = ShardSpec(cfg.tp_rank, cfg.tp_size, cfg.ep_rank, cfg.ep_size)
        t0 = time.perf_counter()
        if cfg.weights == "random":
            mode = cfg.weight_init
            if mode == "auto":
                mode = "full" if mcfg.num_params() < 2e9 else "shard"
            weights = random_weights(mcfg, shard, device=self.device, seed=cfg.seed, mode=mode)
        else:
            weights = load_hf_weights(cfg.weights, mcfg, shard, device=self.device)
        self.weights: ModelWeights = weights
        self.load_time = time.perf_counter() - t0
        # what the KV cache needs for the admission limit at full context: the optional weight copies (preshuffled decode
        # / expert streams) are sized from the HBM left after it, never from the KV cache's share
        per_block = mcfg.kv_bytes_per_token() // cfg.tp_size * cfg.block_size
        kv_need = (cfg.num_kv_blocks or -(-cfg.max_num_seqs * max_model_len // cfg.block_size)) * per_block
        self.model = TransformerLM(weights, self.device, tp_comm=tp_comm, ep_comm=ep_comm,
                                   max_decode_ctx=max_model_len, decode_weights=cfg.decode_weights,
                                   kv_reserve_bytes=kv_need)
        self.tokenizer = load_tokenizer(mcfg, cfg.tokenizer or (cfg.weights if cfg.weights != "random" else None))
        nb = cfg.num_kv_blocks or self._auto_blocks(max_model_len)
        self.kv = KVCache(mcfg.num_layers, nb, mcfg.num_kv_heads // cfg.tp_size, mcfg.head_dim, cfg.block_size,
                          self.device)
        self.blocks = BlockManager(nb, cfg.block_size, prefix_caching=cfg.enable_prefix_caching)
        if self.device.type != "cpu":
            extra = self.model.extra_weight_bytes()
            print(f"symmetry: {mcfg.name} weights {weights.nbytes() / 1e9:.1f} GB + layout copies {extra / 1e9:.1f} GB; "
                  f"KV cache {nb} blocks x {cfg.block_size} = {nb * cfg.block_size} tokens ({self.kv.nbytes() / 1e9:.1f} GB; "
                  f"{cfg.max_num_seqs} seqs x {max_model_len} need {kv_need / 1e9:.1f} GB)", file=sys.stderr, flush=True)
        self.scheduler = Scheduler(
            SchedulerConfig(max_num_seqs=min(cfg.max_num_seqs, self._max_decode_rows(mcfg)),
                            max_num_batched_tokens=cfg.max_num_batched_tokens, max_model_len=max_model_len,
                            mixed_prefill_tokens=cfg.mixed_prefill_tokens,
                            burst_split_tokens=cfg.burst_split_tokens),
            self.blocks)
        self.runner = ModelRunner(self.model, self.kv, self.scheduler.cfg.max_num_seqs, max_model_len,
                                  use_graphs=cfg.use_graphs and self._graph_safe(tp_comm, ep_comm),
                                  tp_rank=cfg.tp_rank, tp_size=cfg.tp_size, cpu_group=cpu_group,
                                  max_num_tokens=max(cfg.max_num_batched_tokens, 8192))
        self.requests: dict[str, tuple] = {}
        self.last_arrival = 0.0  # perf_counter of the latest add_request (arrival coalescing)
        self.lock = threading.Lock()
        self._inflight: dict | None = None
        self._last_done = 0.0
        # (launch, done, kind, seqs, tokens, enqueued) of recent steps, perf_counter clock (TTFT breakdowns, e2e.py)
        self.step_trace: collections.deque = collections.deque(maxlen=2048)
        # pipelined decode on one GPU and under TP (the workers poll the shared-memory metadata ring and
        # never synchronise: parallel/metaplane.py)
        self.pipeline = cfg.pipeline
        self._profiler = None
        self._profile_left = int(os.environ.get("SYMMETRY_PROFILE_STEPS", "20"))
        self.profile_trace: str | None = None
        # fault containment (tensor parallel): once a peer rank is lost the engine cannot compute any step; it
        # fails every request and refuses new ones, and its listeners (the backend -> the provider) take the
        # provider offline (parallel/health.py)
        self.host_phase = {"schedule": 0.0}  # host seconds in scheduling (pipelined decode; bench breakdowns)
        self.fatal: str | None = None
        self.health = None  # rank 0's TPHealthMonitor (parallel/launch.py), if any
        self._fatal_listeners: list = []

    # ------------------------------------------------------------------------------------------
    @staticmethod
    def _model_config(cfg: "EngineConfig") -> ModelConfig:
        """A HF checkpoint directory's config.json wins over the registry (any Llama / Mixtral size)."""
        if cfg.weights != "random":
            path = os.path.join(cfg.weights, "config.json")
            if os.path.exists(path):
                import json

                from ..models.config import from_hf_config

                with open(path) as f:
                    return from_hf_config(json.load(f), name=cfg.model)
        return resolve(cfg.model)

    def _max_decode_rows(self, mcfg: ModelConfig) -> int:
        """Concurrent sequences per decode step: up to MAX_DECODE_ROWS (rows past the fused decode kernels run
        the general path -- medium-M GEMMs with fused epilogues on one GPU; under TP the slab path whose
        all-reduces are capturable; for MoE the grouped GEMMs whose segment bounds stay on the device -- one
        hipGraph per bucket)."""
        return MAX_DECODE_ROWS

    def _graph_safe(self, tp_comm, ep_comm) -> bool:
        """Decode hipGraphs need every collective to be capturable (our RCCL communicator, or the xGMI
        kernels over it).  The MoE block reads nothing on the host (device-side segment offsets, fixed-
        capacity expert all-to-all), whichever EP mode it runs."""
        from .. import ops

        if ops.torch_mode():  # eager torch baseline: host-synchronising reference ops
            return False
        for c in (tp_comm, ep_comm):
            if c is not None and getattr(c, "world", 1) > 1 and not getattr(c, "capturable", False):
                return False
        return True

    def _auto_blocks(self, max_model_len: int) -> int:
        per_block = self.model_cfg.kv_bytes_per_token() // self.cfg.tp_size * self.cfg.block_size
        if self.device.type == "cpu":
            want = (self.cfg.max_num_seqs * max_model_len) // self.cfg.block_size + 8
            return max(16, min(want, (1 << 30) // per_block))
        free, total = torch.cuda.mem_get_info(self.device)
        reserve = 6 << 30  # workspace, graphs, library GEMM scratch
        # ranks sharing one GPU (the one-GPU TP/EP rehearsal) each read the same free memory at about the same time:
        # each takes its share of it, or the later allocation runs out of HBM
        local = int(os.environ.get("LOCAL_WORLD_SIZE", max(self.cfg.tp_size, self.cfg.ep_size)))
        sharing = max(1, -(-local // max(1, torch.cuda.device_count())))
        budget = max(0, int((free - reserve) * self.cfg.kv_cache_fraction) // sharing)
        return max(16, budget // per_block)

    # ---- fault containment ----------------------------------------------------------------------
    def add_fatal_listener(self, fn) -> None:
        """``fn(message)`` once, when the engine becomes unusable (a TP peer was lost)."""
        if self.fatal is not None:
            fn(self.fatal)
        else:
            self._fatal_listeners.append(fn)

    def declare_fatal(self, message: str) -> None:
        """Any thread: the engine can no longer compute steps.  The engine thread fails every request at its next
        step; the listeners run here, once."""
        with self.lock:
            if self.fatal is not None:
                return
            self.fatal = message
            listeners, self._fatal_listeners = self._fatal_listeners, []
        if self.health is not None:
            self.health.declare(message)  # stops the device collectives if the monitor has not yet
        for fn in listeners:
            try:
                fn(message)
            except Exception:  # noqa: BLE001
                traceback.print_exc()

    def _fail_all(self, message: str) -> list[RequestOutput]:
        """Fail every known request (running, waiting, in flight) with an error output."""
        outs = []
        with self.lock:
            self._inflight = None
            for rid, (seq, _, cb) in list(self.requests.items()):
                if not seq.status.finished:
                    self.metrics.on_abort(error=True)
                    self.scheduler.finish(seq, SeqStatus.FINISHED_ERROR)
                out = RequestOutput(rid, [], "", True, "error", error=message, seq=seq)
                outs.append(out)
                self._emit(cb, out)
            self.requests.clear()
            for seq in list(self.scheduler.running) + list(self.scheduler.waiting):
                self.scheduler.finish(seq, SeqStatus.FINISHED_ERROR)
        return outs

    def add_request(self, request_id: str, prompt_ids: list, params: SamplingParams | None = None,
                    callback=None, cache_scope: bytes = b"") -> Sequence:
        """``cache_scope``: prefix-cache namespace (the provider passes the client's public key, so one
        client's conversation reuses only its own cached KV blocks)."""
        if self.fatal is not None:
            raise RuntimeError(f"engine unavailable: {self.fatal}")
        params = params or SamplingParams(max_tokens=self.cfg.default_max_tokens)
        seq = Sequence(request_id, list(prompt_ids), params, eos_ids=tuple(self.model_cfg.eos_token_ids),
                       cache_scope=bytes(cache_scope))
        if params.seed is not None:
            seq.sampling_seed = int(params.seed)
        else:
            seq.sampling_seed = int.from_bytes(hashlib.blake2b(request_id.encode(), digest_size=8).digest(), "little")
        with self.lock:
            self.scheduler.add(seq)
            self.requests[request_id] = (seq, IncrementalDetokenizer(self.tokenizer), callback)
            self.metrics.on_arrival()
            self.last_arrival = time.perf_counter()
        return seq

    def add_chat_request(self, request_id: str, messages: list, params: SamplingParams | None = None,
                         callback=None) -> Sequence:
        return self.add_request(request_id, self.tokenizer.apply_chat_template(messages), params, callback)

    def abort(self, request_id: str) -> None:
        with self.lock:
            seq = self.scheduler.abort(request_id)
            entry = self.requests.pop(request_id, None)
        if seq is not None:
            self.metrics.on_abort()
        if seq is not None and entry is not None:
            self._emit(entry[2], RequestOutput(request_id, [], "", True, "abort", seq=seq))

    def has_unfinished(self) -> bool:
        fl = self._inflight
        live = fl is not None and any(not s.status.finished for s in fl["batch"].seqs)
        return self.scheduler.has_work() or live

    @staticmethod
    def _emit(cb, out: RequestOutput) -> None:
        if cb is not None:
            cb(out)

    # ------------------------------------------------------------------------------------------
    def step(self) -> list[RequestOutput]:
        """One engine iteration; returns the outputs that completed in it.

        Pipelined decode (single-GPU and TP engines): step N+1 is scheduled and enqueued on the GPU before
        step N's sampled ids are copied back -- its pending input tokens are gathered on the device
        from step N's output buffer -- and only then does the host wait for, detokenize and stream
        step N.  Host scheduling, detokenization and the provider's socket writes thus overlap the GPU,
        which never idles between decode steps.  A sequence that stops at step N has already been
        given one extra step; that token is discarded (its KV blocks are released in stream order)."""
        if self.fatal is not None:
            return self._fail_all(self.fatal) if self.requests or self.scheduler.has_work() else []
        t_sched = time.perf_counter()
        prev = self._inflight
        if prev is not None:
            with self.lock:
                nxt = self.scheduler.schedule_lookahead()
            self.host_phase["schedule"] += time.perf_counter() - t_sched
            self._inflight = None
            if nxt is not None:
                fl = self._launch(nxt, prev)
                if "failed" not in fl:
                    self._inflight = fl
            return self._complete(prev, time.perf_counter() - t_sched)
        with self.lock:
            batch = self.scheduler.schedule()
        if batch is None or not batch.seqs:
            return []
        fl = self._launch(batch, None)
        if "failed" in fl:
            return fl["failed"]
        if self.pipeline and batch.kind == "decode":
            self._inflight = fl
            return []
        return self._complete(fl, time.perf_counter() - t_sched)

    def has_in_flight(self) -> bool:
        return self._inflight is not None

    def _fail(self, batch, exc) -> list[RequestOutput]:
        """Engine watchdog: fail the requests of a step that raised, keep serving the others -- unless the step
        lost a tensor-parallel peer: then no later step can succeed either (fault containment)."""
        from ..parallel.health import TPFaultError

        msg = f"{type(exc).__name__}: {exc}"
        traceback.print_exc()
        if self.health is not None and self.fatal is None:
            self.health.check()  # a collective that raised (gloo: peer socket closed) -- is a peer gone?
        if isinstance(exc, TPFaultError) or self.fatal is not None:
            self.declare_fatal(self.fatal or str(exc))
            return self._fail_all(self.fatal)
        outs = []
        with self.lock:
            for seq in batch.seqs:
                if seq.status.finished:
                    continue
                self.metrics.on_abort(error=True)
                self.scheduler.finish(seq, SeqStatus.FINISHED_ERROR)
                entry = self.requests.pop(seq.request_id, None)
                out = RequestOutput(seq.request_id, [], "", True, "error", error=msg, seq=seq)
                outs.append(out)
                if entry:
                    self._emit(entry[2], out)
        return outs

    def _launch(self, batch, prev) -> dict:
        if self._profiler is None and _PROFILE_DIR and self._profile_left > 0:
            self._start_profiler()
        t0 = time.perf_counter()
        prev_rows = None
        if prev is not None:
            prev_rows = {s.seq_id: i for i, s in enumerate(prev["batch"].seqs)}
        try:
            handle = self.runner.launch(batch, prev_rows)
        except Exception as exc:
            return {"failed": self._fail(batch, exc)}
        with self.lock:
            for seq, n, keep in zip(batch.seqs, batch.num_new_tokens, batch.sample):
                seq.num_computed += n
                seq.num_pending += int(keep)
                if batch.kind == "prefill" and n > 1:
                    # prompt blocks completed by this (enqueued) step become adoptable by later arrivals
                    self.blocks.register(seq)
        return {"batch": batch, "handle": handle, "t0": t0, "t_enq": time.perf_counter()}

    def _complete(self, fl: dict, t_launch: float) -> list[RequestOutput]:
        """Wait for a launched step and stream its tokens.  ``t_launch``: host seconds this iteration spent
        scheduling + enqueueing (metrics phases: launch / wait on the GPU / postprocess)."""
        batch, t0 = fl["batch"], fl["t0"]
        t_wait = time.perf_counter()
        try:
            ids = self.runner.wait(fl["handle"])
        except Exception as exc:
            return self._fail(batch, exc)
        now = time.perf_counter()
        self.step_trace.append((t0, now, batch.kind, len(batch.seqs), batch.num_tokens, fl.get("t_enq", t0)))
        # step latency: completion-to-completion while the pipeline is full, launch-to-completion otherwise
        dt = now - max(t0, self._last_done)
        self._last_done = now
        self.metrics.on_step(batch.kind, len(batch.seqs), batch.num_tokens, dt, self.blocks.utilization(),
                             len(self.scheduler.waiting))
        self.metrics.prefix_hits, self.metrics.prefix_queries = self.blocks.hit_tokens, self.blocks.query_tokens
        outs = []
        with self.lock:
            for seq, keep, tok in zip(batch.seqs, batch.sample, ids):
                if keep:
                    seq.num_pending -= 1
                if seq.status.finished or not keep:
                    continue
                first = seq.first_token_time is None
                seq.append(tok, now)
                entry = self.requests.get(seq.request_id)
                if entry is None:
                    continue
                _, detok, cb = entry
                stop = seq.check_stop()
                text = detok.add(tok)  # special / EOS ids decode to ''
                if seq.params.stop and text:
                    hit = min((i for i in (detok.text.find(s) for s in seq.params.stop) if i >= 0), default=-1)
                    if hit >= 0:
                        cut = len(detok.text) - hit
                        text = text[:-cut] if cut <= len(text) else ""
                        stop = SeqStatus.FINISHED_STOPPED
                if first:
                    self.metrics.on_first_token(seq.ttft)
                else:
                    self.metrics.on_token()
                out = RequestOutput(seq.request_id, [tok], text, seq=seq)
                if stop is not None:
                    tail = detok.flush() if stop == SeqStatus.FINISHED_LENGTH else ""
                    out.text += tail
                    out.finished, out.finish_reason = True, stop.value
                    seq.finish_time = now
                    self.scheduler.finish(seq, stop)
                    self.requests.pop(seq.request_id, None)
                    self.metrics.on_finish(seq)
                outs.append(out)
                self._emit(cb, out)
        self.metrics.on_phase(t_launch, now - t_wait, time.perf_counter() - now)
        if self._profiler is not None:
            self._profiler.step()
            self._profile_left -= 1
            if self._profile_left <= 0:
                self._stop_profiler()
        return outs

    # ---- torch.profiler hook: SYMMETRY_PROFILE=<dir> [SYMMETRY_PROFILE_STEPS=N] ----------
    def _start_profiler(self) -> None:
        from torch.profiler import ProfilerActivity, profile

        acts = [ProfilerActivity.CPU] + ([ProfilerActivity.CUDA] if self.device.type != "cpu" else [])
        self._profiler = profile(activities=acts, record_shapes=False)
        self._profiler.__enter__()

    def _stop_profiler(self) -> None:
        prof, self._profiler = self._profiler, None
        prof.__exit__(None, None, None)
        os.makedirs(_PROFILE_DIR, exist_ok=True)
        path = os.path.join(_PROFILE_DIR, f"engine_trace_rank{self.cfg.tp_rank}_{os.getpid()}.json")
        prof.export_chrome_trace(path)
        self.profile_trace = path

    def warmup(self, prompt_lens=None) -> float:
        """Provider start-up pass: one prefill per size class (library GEMM heuristics and code objects
        load here, not in the first client's TTFT), then capture the decode hipGraphs.  Returns seconds."""
        t0 = time.perf_counter()
        budget = self.scheduler.cfg.max_num_batched_tokens
        seq_cap = self.scheduler.cfg.max_model_len - 4
        lens = prompt_lens or [n for n in (1, 16, 64, 128, 256, 512, 1024, 2048, 4096, 8192) if n <= budget]
        vocab = self.model_cfg.vocab_size
        for n in lens:
            n = min(n, budget)
            # a size class larger than one sequence may hold is warmed as several prompts in one step
            k = max(1, -(-n // seq_cap))
            seqs = []
            for j in range(k):
                m = n // k + (1 if j < n % k else 0)
                ids = [(7 * i + 3 * j) % (vocab - 1) + 1 for i in range(m)]
                seqs.append(self.add_request(f"__warmup-{n}-{j}", ids, SamplingParams(max_tokens=2, ignore_eos=True)))
            while not all(s.status.finished for s in seqs):
                self.step()
        self.runner.capture_all()
        self.metrics = EngineMetrics()
        return time.perf_counter() - t0

    def generate(self, prompt_ids: list, params: SamplingParams | None = None) -> list[int]:
        """Blocking single-request helper (tests, smoke)."""
        rid = f"gen-{time.monotonic_ns()}"
        seq = self.add_request(rid, prompt_ids, params)
        while not seq.status.finished:
            self.step()
        return list(seq.output_ids)

    def shutdown(self) -> None:
        if self.health is not None:
            # an orderly stop: the workers leaving after the stop broadcast is not a fault
            self.health.stop()
        self.runner.broadcast_stop()


def _deliver_all(items) -> None:
    for deliver, out in items:
        deliver(out)


class AsyncEngine:
    """Runs :class:`LLMEngine` on a dedicated thread; asyncio-facing ``generate``.

    The outputs of one engine step reach each event loop as ONE batch (one cross-thread wake-up per step,
    not one per token; ``SYMMETRY_BATCH_DELIVERY=0`` restores per-token wake-ups): it halves the engine
    thread's per-step postprocess time (profiles/e2e_delivery_ab_r2.jsonl).  ``SYMMETRY_GIL_SWITCH_US``
    optionally shortens the interpreter's GIL switch interval (default: Python's 5 ms; 500 us measured no
    gain in the same A/B)."""

    def __init__(self, engine: LLMEngine, queue_limit: int = 4096):
        self.engine = engine
        self.queue_limit = queue_limit
        self._wake = threading.Event()
        self._stop = False
        self._thread = threading.Thread(target=self._loop, name="symmetry-engine", daemon=True)
        self._started = False
        self._pending: list = []  # (loop, deliver, output) of the current step, engine thread only
        self._batch = os.environ.get("SYMMETRY_BATCH_DELIVERY", "1") != "0"

    def start(self) -> None:
        if not self._started:
            self._started = True
            us = int(os.environ.get("SYMMETRY_GIL_SWITCH_US", "0"))
            if us > 0:
                sys.setswitchinterval(us * 1e-6)
            self._thread.start()

    def _loop(self) -> None:
        idle = True
        while not self._stop:
            if self.engine.fatal is not None:  # fault containment: fail whatever is left, then serve nothing
                self.engine.step()
                self._flush()
                self._wake.wait(0.05)
                self._wake.clear()
                continue
            if not self.engine.has_unfinished():
                idle = True
                self._wake.wait(0.05)
                self._wake.clear()
                continue
            if idle:
                self._coalesce()
                idle = False
            self.engine.step()
            self._flush()

    def _coalesce(self) -> None:
        """Idle -> busy: let a burst of simultaneous requests finish arriving (EngineConfig.arrival_*)."""
        cfg = self.engine.cfg
        quiet, window = cfg.arrival_quiet_us * 1e-6, cfg.arrival_window_us * 1e-6
        if quiet <= 0:
            return
        t0 = time.perf_counter()
        while not self._stop:
            now = time.perf_counter()
            if now - self.engine.last_arrival >= quiet or now - t0 >= window:
                return
            time.sleep(min(quiet, 1e-4))

    def _flush(self) -> None:
        """Hand this step's outputs to their event loops, one call per loop."""
        if not self._pending:
            return
        by_loop: dict = {}
        for loop, deliver, out in self._pending:
            by_loop.setdefault(loop, []).append((deliver, out))
        self._pending = []
        for loop, items in by_loop.items():
            try:
                loop.call_soon_threadsafe(_deliver_all, items)
            except RuntimeError:  # the loop is closed: its consumers are gone
                pass

    def stop(self) -> None:
        self._stop = True
        self._wake.set()
        if self._started:
            self._thread.join(timeout=10)
        self.engine.shutdown()

    def submit(self, request_id: str, on_output, messages: list | None = None, prompt_ids: list | None = None,
               params: SamplingParams | None = None, cache_scope: bytes = b"") -> None:
        """Callback form of :meth:`generate` for the serving hot path: ``on_output(out)`` runs on the calling
        event loop for every output (a step's outputs arrive as one batch, see the class note), with no
        per-token task switch or async-generator hop.  The caller aborts through :meth:`abort`."""
        loop = asyncio.get_running_loop()

        def cb(out: RequestOutput) -> None:
            out.t_engine = time.perf_counter()  # (request-path timing: NativeBackend.timings)
            if self._batch and threading.current_thread() is self._thread:
                self._pending.append((loop, on_output, out))
            else:
                loop.call_soon_threadsafe(on_output, out)

        if prompt_ids is None:
            prompt_ids = self.engine.tokenizer.apply_chat_template(messages or [])
        self.engine.add_request(request_id, prompt_ids, params, cb, cache_scope=cache_scope)
        self.start()
        self._wake.set()

    def abort(self, request_id: str) -> None:
        self.engine.abort(request_id)

    async def generate(self, request_id: str, messages: list | None = None, prompt_ids: list | None = None,
                       params: SamplingParams | None = None, cache_scope: bytes = b""):
        """Async iterator of RequestOutput for one request; aborts the sequence if the consumer goes away.

        The engine thread never blocks on a consumer: outputs are buffered, and a consumer that falls
        more than ``queue_limit`` outputs behind (a stalled / slow reader) has its request aborted with
        an error output, so its KV blocks return to the pool (SURVEY.md §7.4 risk 6)."""
        loop = asyncio.get_running_loop()
        q: asyncio.Queue = asyncio.Queue()
        state = {"overflow": False}

        def deliver(out: RequestOutput) -> None:
            if state["overflow"]:
                return
            if not out.finished and q.qsize() >= self.queue_limit:
                state["overflow"] = True
                self.engine.abort(request_id)
                q.put_nowait(RequestOutput(request_id, [], "", True, "error",
                                           error=f"client too slow: more than {self.queue_limit} outputs behind"))
                return
            q.put_nowait(out)

        def cb(out: RequestOutput) -> None:
            out.t_engine = time.perf_counter()  # (request-path timing: NativeBackend.timings)
            if self._batch and threading.current_thread() is self._thread:
                self._pending.append((loop, deliver, out))  # flushed after the engine step
            else:
                loop.call_soon_threadsafe(deliver, out)

        if prompt_ids is None:
            prompt_ids = self.engine.tokenizer.apply_chat_template(messages or [])
        self.engine.add_request(request_id, prompt_ids, params, cb, cache_scope=cache_scope)
        self.start()
        self._wake.set()
        finished = False
        try:
            while True:
                out = await q.get()
                yield out
                if out.finished:
                    finished = True
                    return
        finally:
            if not finished:
                self.engine.abort(request_id)
