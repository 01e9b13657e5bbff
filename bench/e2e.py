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
aggregate streamed tokens/s) -- the BASELINE.json metric measured at the client end of the socket.

  python bench/e2e.py --model llama3:8b --clients 10 --max-tokens 256      # config 3
  python bench/e2e.py --model llama3:8b --clients 1                        # config 2
  python bench/e2e.py --model mixtral:8x7b --clients 4 --data-collection   # config 5 (public + collection)
"""
from __future__ import annotations

import argparse
import asyncio
import json
import multiprocessing as mp
import os
import statistics
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def _client_proc(boot, server_key, model, n, prompt_words, max_tokens, out_q, start_evt):
    async def one(i):
        from symmetry_amd.testing.mock_client import SymmetryClient

        c = SymmetryClient(boot, server_key)
        await c.start()
        try:
            det = await c.request_provider(model)
            conn = await c.connect_provider(det["discoveryKey"])
            words = " ".join(f"w{(i * 7919 + k) % 997}" for k in range(prompt_words))
            r = await c.chat(conn, [{"role": "user", "content": words}],
                             extra={"max_tokens": max_tokens, "ignore_eos": True, "temperature": 0.0},
                             timeout=600)
            return {"ttft_ms": None if r.ttft_s is None else r.ttft_s * 1e3, "tokens_per_s": r.tokens_per_s,
                    "events": r.content_events, "ended": r.ended, "error": r.error,
                    "wall_s": r.t_end - r.t_start}
        finally:
            await c.stop()

    async def main():
        start_evt.wait()
        return await asyncio.gather(*(one(i) for i in range(n)))

    try:
        out_q.put(asyncio.run(main()))
    except Exception as exc:  # report, never hang the parent
        import traceback

        out_q.put(f"client process failed: {exc}\n{traceback.format_exc()}")


async def _serve(args):
    import yaml

    from symmetry_amd.backends.native import NativeBackend
    from symmetry_amd.engine.llm_engine import EngineConfig, LLMEngine
    from symmetry_amd.net import DiscoveryServer
    from symmetry_amd.provider.node import SymmetryProvider
    from symmetry_amd.testing.mock_server import SymmetryServer

    ds = DiscoveryServer()
    await ds.start()
    boot = [ds.address]
    server = SymmetryServer(bootstrap=boot, ping_interval=5.0)
    await server.start()
    tmp = tempfile.mkdtemp(prefix="symmetry-e2e-")
    cfg = {"apiHostname": "127.0.0.1", "apiPath": "/v1/chat/completions", "apiPort": 0, "apiProtocol": "http",
           "apiProvider": "native", "dataCollectionEnabled": bool(args.data_collection),
           "maxConnections": args.clients, "modelName": args.model, "name": "e2e-provider",
           "path": os.path.join(tmp, "data"), "public": True, "serverKey": server.server_key,
           "metricsInterval": 0}
    path = os.path.join(tmp, "provider.yaml")
    with open(path, "w") as f:
        yaml.safe_dump(cfg, f)
    t0 = time.perf_counter()
    eng = LLMEngine(EngineConfig.from_provider(cfg, max_model_len=args.max_model_len, device="auto",
                                               max_num_batched_tokens=max(8192, args.clients * 512)))
    warm = eng.warmup() if eng.device.type != "cpu" else 0.0
    load_s = time.perf_counter() - t0
    provider = SymmetryProvider(path, backend=NativeBackend(cfg, engine=eng), bootstrap=boot)
    await provider.init()
    for _ in range(200):
        if server.providers(args.model):
            break
        await asyncio.sleep(0.05)

    ctx = mp.get_context("spawn")
    q, start_evt = ctx.Queue(), ctx.Event()
    p = ctx.Process(target=_client_proc, args=(boot, server.server_key, args.model, args.clients, args.prompt_words,
                                               args.max_tokens, q, start_evt))
    p.start()
    await asyncio.sleep(0.5)
    eng.metrics = type(eng.metrics)()
    t1 = time.perf_counter()
    start_evt.set()
    res = await asyncio.to_thread(q.get)
    wall = time.perf_counter() - t1
    p.join(30)
    stats = provider.stats()
    saved = len(provider.saved_files)
    await provider.destroy()
    await server.stop()
    await ds.stop()
    if isinstance(res, str):
        raise SystemExit(res)
    ttfts = sorted(r["ttft_ms"] for r in res if r["ttft_ms"] is not None)
    tps = [r["tokens_per_s"] for r in res]
    total_events = sum(r["events"] for r in res)
    out = {
        "metric": "streamed tokens/sec + p50 TTFT per client (over the encrypted swarm)",
        "model": args.model, "clients": args.clients, "max_tokens": args.max_tokens,
        "p50_ttft_ms": round(statistics.median(ttfts), 2) if ttfts else None,
        "p90_ttft_ms": round(ttfts[int(0.9 * (len(ttfts) - 1))], 2) if ttfts else None,
        "per_client_tokens_per_s_mean": round(statistics.fmean(tps), 2),
        "per_client_tokens_per_s_min": round(min(tps), 2),
        "aggregate_tokens_per_s": round(total_events / wall, 2),
        "all_ended": all(r["ended"] and not r["error"] for r in res),
        "data_collection_files": saved,
        "engine": {k: stats.get(k) for k in ("mean_decode_batch", "p50_itl_ms", "decode_steps", "step_phase_ms")},
        "load_and_warmup_s": round(load_s, 1), "warmup_s": round(warm, 1),
        "dtype": "bf16", "data": "synthetic prompts, random-init weights",
    }
    print(json.dumps(out), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3:8b")
    ap.add_argument("--clients", type=int, default=10)
    ap.add_argument("--max-tokens", type=int, default=256)
    ap.add_argument("--prompt-words", type=int, default=60)
    ap.add_argument("--max-model-len", type=int, default=4096)
    ap.add_argument("--data-collection", action="store_true")
    args = ap.parse_args()
    asyncio.run(_serve(args))


if __name__ == "__main__":
    main()
