"""Engine / provider metrics.

The reference only logs (``src/logger.ts``); the native provider also keeps
counters and latency distributions: TTFT, inter-token latency, tokens/s,
batch size, KV utilisation, queue depth, active peers.  ``summary()`` is
what the bench and the periodic metrics log line print.
"""
from __future__ import annotations

import statistics
import threading
import time
from collections import deque


def percentile(xs, q: float):
    if not xs:
        return None
    s = sorted(xs)
    k = (len(s) - 1) * q
    f = int(k)
    c = min(f + 1, len(s) - 1)
    return s[f] + (s[c] - s[f]) * (k - f)


class EngineMetrics:
    def __init__(self, window: int = 4096):
        self.lock = threading.Lock()
        self.t_start = time.perf_counter()
        self.requests = 0
        self.finished = 0
        self.tokens = 0
        self.steps = {"prefill": 0, "decode": 0}
        self.step_time = {"prefill": 0.0, "decode": 0.0}
        self.ttft = deque(maxlen=window)
        self.itl = deque(maxlen=window)
        self.batch = deque(maxlen=window)
        self.kv_util = 0.0
        self.prefix_hits = 0      # prompt tokens whose prefill was skipped (adopted cached KV blocks)
        self.prefix_queries = 0   # prompt tokens looked up in the prefix cache
        self.queue_depth = 0
        self.active_peers = 0
        # engine step timer (seconds): host scheduling + enqueue, host blocked on the GPU, streaming out
        self.phase = {"launch": 0.0, "wait": 0.0, "postprocess": 0.0}
        self.aborted = 0
        self.errors = 0

    def on_arrival(self):
        with self.lock:
            self.requests += 1

    def on_step(self, kind, nseq, ntok, dt, kv_util, qdepth):
        with self.lock:
            self.steps[kind] += 1
            self.step_time[kind] += dt
            if kind == "decode":
                self.batch.append(nseq)
                self.itl.append(dt)
            self.kv_util = kv_util
            self.queue_depth = qdepth

    def on_first_token(self, ttft):
        with self.lock:
            self.tokens += 1
            if ttft is not None:
                self.ttft.append(ttft)

    def on_token(self):
        with self.lock:
            self.tokens += 1

    def on_finish(self, seq):
        with self.lock:
            self.finished += 1

    def on_phase(self, launch: float, wait: float, postprocess: float):
        with self.lock:
            self.phase["launch"] += launch
            self.phase["wait"] += wait
            self.phase["postprocess"] += postprocess

    def on_abort(self, error: bool = False):
        with self.lock:
            if error:
                self.errors += 1
            else:
                self.aborted += 1

    def summary(self) -> dict:
        with self.lock:
            el = time.perf_counter() - self.t_start
            return {
                "requests": self.requests,
                "finished": self.finished,
                "tokens": self.tokens,
                "tokens_per_s": self.tokens / el if el > 0 else 0.0,
                "p50_ttft_ms": None if not self.ttft else 1e3 * percentile(list(self.ttft), 0.5),
                "p99_ttft_ms": None if not self.ttft else 1e3 * percentile(list(self.ttft), 0.99),
                "p50_itl_ms": None if not self.itl else 1e3 * percentile(list(self.itl), 0.5),
                "mean_decode_batch": statistics.fmean(self.batch) if self.batch else 0.0,
                "prefill_steps": self.steps["prefill"],
                "decode_steps": self.steps["decode"],
                "kv_utilization": round(self.kv_util, 4),
                "prefix_cache_hit_tokens": self.prefix_hits,
                "prefix_cache_hit_rate": round(self.prefix_hits / self.prefix_queries, 4) if self.prefix_queries else 0.0,
                "queue_depth": self.queue_depth,
                "active_peers": self.active_peers,
                "aborted": self.aborted,
                "errors": self.errors,
                "step_phase_ms": {k: round(1e3 * v / max(1, sum(self.steps.values())), 4)
                                  for k, v in self.phase.items()},
            }


class MetricsReporter:
    """Periodic metrics: one ``📊`` log line and (optionally) a JSON snapshot file every ``interval_s``.

    ``source`` returns the dict to report (engine summary merged with provider counters)."""

    def __init__(self, source, interval_s: float = 60.0, path: str | None = None, log=None):
        self.source, self.interval_s, self.path, self.log = source, interval_s, path, log
        self._task = None

    def snapshot(self) -> dict:
        snap = dict(self.source())
        snap["ts"] = time.time()
        if self.path:
            import json
            import os

            tmp = self.path + ".tmp"
            with open(tmp, "w") as f:
                json.dump(snap, f)
            os.replace(tmp, self.path)
        if self.log is not None:
            keys = ("tokens_per_s", "p50_ttft_ms", "p50_itl_ms", "mean_decode_batch", "kv_utilization",
                    "queue_depth", "active_peers")
            self.log(" ".join(f"{k}={snap[k]:.4g}" if isinstance(snap.get(k), float) else f"{k}={snap.get(k)}"
                              for k in keys if k in snap))
        return snap

    def start(self) -> None:
        import asyncio

        async def loop():
            while True:
                await asyncio.sleep(self.interval_s)
                try:
                    self.snapshot()
                except Exception:  # metrics must never take the provider down
                    pass

        if self.interval_s and self.interval_s > 0:
            self._task = asyncio.ensure_future(loop())

    def stop(self) -> None:
        if self._task is not None:
            self._task.cancel()
            self._task = None
