#!/usr/bin/env python3
"""End-to-end provider benchmark over the encrypted swarm (SURVEY.md §4.2 'E2E bench', BASELINE configs 2-5).

Process layout (everything on 127.0.0.1):
  * main process: discovery node + Symmetry server + ``symmetry-cli``-equivalent provider (native backend,
    the MI355X engine) -- exactly the objects ``symmetry-cli -c provider.yaml`` builds;
  * a separate client process: C Symmetry clients, each ``requestProvider`` (model-based assignment by
    the server), connect to the provider's topic (Noise XX + secretstream), send ``newConversation`` +
    ``inference``, then read the ``symmetryEmitterKey`` header, one SSE event per token and
    ``inferenceEnded``.

Per client: TTFT = ``inference`` write -> first content delta on the client's socket; tokens/s =
(content events - 1) / (last event - first event).  Prints one JSON line (p50 TTFT, per-client and
aggregate streamed tokens/s) -- the BASELINE.json metric measured at the client end of the socket
(``symmetry_amd/testing/e2e.py``; ``bench.py`` runs the same measurement after its engine-step timing).

  python bench/e2e.py --model llama3:8b --clients 10 --max-tokens 256      # config 3
  python bench/e2e.py --model llama3:8b --clients 1                        # config 2
  python bench/e2e.py --model mixtral:8x7b --clients 4 --data-collection   # config 5 (public + collection)
"""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


async def _serve(args):
    from symmetry_amd.engine.llm_engine import EngineConfig, LLMEngine
    from symmetry_amd.testing.e2e import client_end_run

    t0 = time.perf_counter()
    cfg = {"modelName": args.model, "maxConnections": args.clients}
    if args.decode_weights:
        cfg["decodeWeights"] = args.decode_weights
    eng = LLMEngine(EngineConfig.from_provider(cfg, max_model_len=args.max_model_len, device="auto",
                                               max_num_batched_tokens=max(8192, args.clients * 512)))
    warm = eng.warmup() if eng.device.type != "cpu" else 0.0
    load_s = time.perf_counter() - t0
    out = {"metric": "streamed tokens/sec + p50 TTFT per client (over the encrypted swarm)", "model": args.model}
    out.update(await client_end_run(eng, args.model, args.clients, prompt_tokens=args.prompt_tokens,
                                    max_tokens=args.max_tokens, data_collection=args.data_collection))
    out.update({"load_and_warmup_s": round(load_s, 1), "warmup_s": round(warm, 1),
                "weight_layout": "single preshuffled copy" if eng.model.single_copy else
                ("row-major + preshuffled copy" if eng.model.dgw else "row-major"),
                "dtype": "bf16", "data": "synthetic prompts, random-init weights"})
    eng.shutdown()
    print(json.dumps(out), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3:8b")
    ap.add_argument("--clients", type=int, default=10)
    ap.add_argument("--max-tokens", type=int, default=256)
    ap.add_argument("--prompt-tokens", type=int, default=128)
    ap.add_argument("--max-model-len", type=int, default=4096)
    ap.add_argument("--data-collection", action="store_true")
    ap.add_argument("--decode-weights", default=None, choices=("auto", "preshuffled", "replace", "shared"),
                    help="weight layout (engine default: auto)")
    args = ap.parse_args()
    asyncio.run(_serve(args))


if __name__ == "__main__":
    main()
