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
        self.queue_depth = 0
        self.active_peers = 0

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
                "queue_depth": self.queue_depth,
                "active_peers": self.active_peers,
            }
