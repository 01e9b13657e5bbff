"""Time one short prefill (Llama-3-8B, random init) end to end and per GPU step, for rocprofv3 kernel traces.

    python bench/host/prefill_step.py --tokens 128 --reps 20 [--no-graphs]

Each rep is a fresh prompt of ``--tokens`` tokens (distinct ids: no prefix-cache hit) generating ONE token,
so the step is exactly the prefill (+ its fused lm_head / sampler).  Prints one JSON line: host launch ->
GPU done per prefill (median), and the engine's launch / enqueue split.
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3:8b")
    ap.add_argument("--tokens", type=int, default=128)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--no-graphs", action="store_true")
    args = ap.parse_args()

    import torch

    from symmetry_amd.engine.llm_engine import EngineConfig, LLMEngine
    from symmetry_amd.engine.sequence import SamplingParams

    eng = LLMEngine(EngineConfig(model=args.model, device="auto", max_num_seqs=4, max_model_len=2048,
                                 use_graphs=not args.no_graphs))
    eng.warmup([args.tokens])
    vocab = eng.model_cfg.vocab_size
    times, enq = [], []
    for r in range(args.reps + 2):
        ids = [(1000 + 97 * r + 13 * i) % (vocab - 1) + 1 for i in range(args.tokens)]
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        eng.generate(ids, SamplingParams(max_tokens=1, ignore_eos=True))
        t1 = time.perf_counter()
        tr = eng.step_trace[-1]
        if r >= 2:
            times.append((t1 - t0) * 1e3)
            enq.append((tr[5] - tr[0]) * 1e3)
    print(json.dumps({"model": args.model, "tokens": args.tokens, "graphs": not args.no_graphs,
                      "prefill_ms_median": round(statistics.median(times), 3), "prefill_ms_min": round(min(times), 3),
                      "host_enqueue_ms_median": round(statistics.median(enq), 3), "reps": args.reps}), flush=True)


if __name__ == "__main__":
    main()
