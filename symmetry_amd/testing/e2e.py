"""Client-end measurement of the BASELINE.json metric: streamed tokens/s + p50 TTFT per client, read on
the clients' swarm sockets ("per-client streamed tok/s over the swarm socket, p50 TTFT from
the ``inference`` write to the first content event").

Process layout (everything on 127.0.0.1):
  * this process: discovery node + Symmetry server + the provider node (``symmetry-cli`` equivalent, native
    backend on the given, already warmed-up engine -- under TP, rank 0's engine with the workers mirroring);
  * a separate client process: C Symmetry clients, each ``requestProvider`` (model-based assignment by the
    server), join the provider's topic (Noise XX + secretstream), send ``newConversation`` + ``inference``,
    then read the ``symmetryEmitterKey`` header, one SSE event per token and ``inferenceEnded``
    (the reference's stream shape, ``/root/reference/src/provider.ts:234-262``).

Per client: TTFT = ``inference`` write -> first content delta on the client's socket; tokens/s =
(content events - 1) / (last event - first event).  Used by ``bench.py`` (its ``client_end`` fields) and
``bench/e2e.py``.
"""
from __future__ import annotations

import asyncio
import collections
import multiprocessing as mp
import os
import statistics
import tempfile
import time

# chat-template tokens around a single user message (byte tokenizer, llama3 format): begin, header(user),
# "\n\n" + content, eot, header(assistant) "\n\n"
_TEMPLATE_TOKENS = 23


def prompt_text(i: int, tokens: int) -> str:
    """ASCII user content that makes a ``tokens``-token chat prompt under the byte tokenizer."""
    n = max(1, tokens - _TEMPLATE_TOKENS)
    base = "".join(chr(0x61 + (i * 7 + k * 13) % 26) if (k + i) % 6 else " " for k in range(n))
    return base[:n]


def _client_proc(boot, server_key, model, n, prompt_tokens, max_tokens, out_q, start_evt):
    async def one(i):
        from symmetry_amd.testing.mock_client import SymmetryClient

        c = SymmetryClient(boot, server_key)
        await c.start()
        try:
            det = await c.request_provider(model)
            conn = await c.connect_provider(det["discoveryKey"])
            await ready.wait()
            r = await c.chat(conn, [{"role": "user", "content": prompt_text(i, prompt_tokens)}],
                             extra={"max_tokens": max_tokens, "ignore_eos": True, "temperature": 0.0},
                             timeout=600)
            return {"ttft_ms": None if r.ttft_s is None else r.ttft_s * 1e3, "tokens_per_s": r.tokens_per_s,
                    "events": r.content_events, "ended": r.ended, "error": r.error,
                    "wall_s": r.t_end - r.t_start, "client": i,
                    "t_write": r.t_start, "t_first": None if r.ttft_s is None else r.t_start + r.ttft_s}
        finally:
            await c.stop()

    async def main():
        nonlocal ready
        ready = asyncio.Event()
        tasks = [asyncio.create_task(one(i)) for i in range(n)]
        # every client has its provider connection before any sends: all requests arrive together
        await asyncio.to_thread(start_evt.wait)
        await asyncio.sleep(0.2)
        ready.set()
        return await asyncio.gather(*tasks)

    ready = None
    try:
        out_q.put(asyncio.run(main()))
    except Exception as exc:  # report, never hang the parent
        import traceback

        out_q.put(f"client process failed: {exc}\n{traceback.format_exc()}")


async def client_end_run(engine, model: str, clients: int, prompt_tokens: int = 128, max_tokens: int = 256,
                         data_collection: bool = False, public: bool = True, timeout: float = 600.0) -> dict:
    """Serve ``engine`` as a provider and measure ``clients`` concurrent streamed chats at the client end."""
    import yaml

    from ..backends.native import NativeBackend, timing_key
    from ..net import DiscoveryServer
    from ..provider.node import SymmetryProvider
    from .mock_server import SymmetryServer

    ds = DiscoveryServer()
    await ds.start()
    boot = [ds.address]
    server = SymmetryServer(bootstrap=boot, ping_interval=5.0)
    await server.start()
    tmp = tempfile.mkdtemp(prefix="symmetry-e2e-")
    cfg = {"apiHostname": "127.0.0.1", "apiPath": "/v1/chat/completions", "apiPort": 0, "apiProtocol": "http",
           "apiProvider": "native", "dataCollectionEnabled": bool(data_collection),
           "maxConnections": clients, "modelName": model, "name": "e2e-provider",
           "path": os.path.join(tmp, "data"), "public": bool(public), "serverKey": server.server_key,
           "metricsInterval": 0}
    path = os.path.join(tmp, "provider.yaml")
    with open(path, "w") as f:
        yaml.safe_dump(cfg, f)
    provider = SymmetryProvider(path, backend=NativeBackend(cfg, engine=engine, record_timings=True), bootstrap=boot)
    await provider.init()
    for _ in range(200):
        if server.providers(model):
            break
        await asyncio.sleep(0.05)
    ctx = mp.get_context("spawn")
    q, start_evt = ctx.Queue(), ctx.Event()
    p = ctx.Process(target=_client_proc, args=(boot, server.server_key, model, clients, prompt_tokens,
                                               max_tokens, q, start_evt), daemon=True)
    p.start()
    try:
        await asyncio.sleep(0.5)
        engine.metrics = type(engine.metrics)()
        tm0 = dict(engine.runner.timing, schedule=engine.host_phase["schedule"])
        t1 = time.perf_counter()
        start_evt.set()
        res = await asyncio.wait_for(asyncio.to_thread(q.get), timeout)
        wall = time.perf_counter() - t1
    finally:
        p.join(30)
        if p.is_alive():
            p.kill()
        stats = provider.stats()
        tm1 = dict(engine.runner.timing, schedule=engine.host_phase["schedule"])
        saved = len(provider.saved_files)
        timings = list(getattr(provider.backend, "timings", []))
        trace = list(getattr(engine, "step_trace", []))
        # the provider's backend stop would shut the engine down: detach it (the caller owns the engine)
        backend = provider.backend
        if getattr(backend, "aengine", None) is not None:
            ae, backend.aengine = backend.aengine, None
            ae._stop = True
            ae._wake.set()
            if ae._started:
                await asyncio.to_thread(ae._thread.join, 10)
        await provider.destroy()
        await server.stop()
        await ds.stop()
    if isinstance(res, str):
        raise RuntimeError(res)
    for r in res:  # the provider's timing key of each client's prompt (salted per process: computed here)
        r["key"] = timing_key(prompt_text(r["client"], prompt_tokens))
    ttfts = sorted(r["ttft_ms"] for r in res if r["ttft_ms"] is not None)
    tps = [r["tokens_per_s"] for r in res]
    total_events = sum(r["events"] for r in res)
    return {
        "clients": clients, "prompt_tokens": prompt_tokens, "max_tokens": max_tokens,
        "p50_ttft_ms": round(statistics.median(ttfts), 2) if ttfts else None,
        "p90_ttft_ms": round(ttfts[int(0.9 * (len(ttfts) - 1))], 2) if ttfts else None,
        "per_client_tokens_per_s_median": round(statistics.median(tps), 2) if tps else None,
        "per_client_tokens_per_s_min": round(min(tps), 2) if tps else None,
        "aggregate_tokens_per_s": round(total_events / wall, 2),
        "all_ended": all(r["ended"] and not r["error"] for r in res),
        "content_events": total_events,
        "data_collection_files": saved,
        "engine": {k: stats.get(k) for k in ("mean_decode_batch", "p50_itl_ms", "decode_steps", "step_phase_ms")},
        # host ms per engine step inside ModelRunner.launch during this run (pack / TP metadata push / H2D +
        # replay enqueue / D2H enqueue): what the engine thread spends outside scheduling and streaming
        "runner_host_ms_per_step": {k: round((tm1[k] - tm0[k]) / max(1, tm1["steps"] - tm0["steps"]) * 1e3, 4)
                                    for k in ("schedule", "fill", "send", "run", "graph_launch", "d2h")},
        "ttft_path_ms": ttft_breakdown(res, timings),
        "first_steps": first_steps(timings, trace),
    }


def first_steps(timings: list, trace: list, n: int = 5) -> list | None:
    """The engine's first n steps after the first request of the run arrived: (kind, sequences, tokens, launch,
    end of the host's enqueue and completion in ms after that arrival)."""
    recvs = [t["recv"] for t in timings if t.get("recv") is not None]
    if not recvs or not trace:
        return None
    t0 = min(recvs)
    steps = [s for s in trace if s[1] >= t0 - 0.05][:n]
    return [{"kind": k, "seqs": ns, "tokens": nt, "launch_ms": round((a - t0) * 1e3, 3),
             "enqueued_ms": round((q - t0) * 1e3, 3), "done_ms": round((b - t0) * 1e3, 3)}
            for a, b, k, ns, nt, q in steps]


def ttft_breakdown(res: list, timings: list) -> dict | None:
    """Median of each leg of the client-end TTFT (perf_counter is CLOCK_MONOTONIC, one clock for the client
    and provider processes of one host): client write -> provider receive -> engine submit -> first token on
    the engine thread -> first output callback on the event loop -> first SSE event written -> first content
    event read by the client; plus the spread of the receive times (how long the burst took to arrive)."""
    counts = collections.Counter(t.get("key") for t in timings)
    dup = {k for k, c in counts.items() if c > 1}  # (prompts repeat with a period of 78 clients: skip those)
    by_key = {t.get("key"): t for t in timings if t.get("key") is not None and t.get("key") not in dup}
    legs = {"write_to_recv": [], "recv_to_submit": [], "submit_to_engine_first": [], "engine_to_callback": [],
            "callback_to_written": [], "written_to_client": []}
    recvs = []
    for r in res:
        t = by_key.get(r.get("key"))
        if t is None or r.get("t_first") is None:
            continue
        pts = [r["t_write"], t.get("recv"), t.get("submitted"), t.get("engine_first"), t.get("callback_first"),
               t.get("written_first"), r["t_first"]]
        if any(p is None for p in pts):
            continue
        recvs.append(t["recv"])
        for (name, vals), a, b in zip(legs.items(), pts[:-1], pts[1:]):
            vals.append((b - a) * 1e3)
    if not recvs:
        return None
    out = {k: round(statistics.median(v), 3) for k, v in legs.items()}
    out["receive_spread"] = round((max(recvs) - min(recvs)) * 1e3, 3)
    out["matched"] = len(recvs)
    return out
