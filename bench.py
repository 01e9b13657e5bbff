#!/usr/bin/env python3
"""Headline benchmark: streamed tokens/s + p50 TTFT per client of a Llama-3-8B provider.

Metric and config come from BASELINE.json ("streamed tokens/sec + p50 TTFT per
client, Llama-3-8B provider, 1/2/4/8 MI355X"; config 3: maxConnections=10
concurrent clients, continuous batching, greedy decode).

One process per GPU for N > 1: either under ``torch.distributed.run`` (the
driver's form) or as plain ``python bench.py --gpus N``, which starts its own
torchrun child with N ranks (``_self_launch``).  bf16,
random-init weights of the real Llama-3-8B architecture, synthetic 128-token
prompts (no network for checkpoints/datasets).

Parallelism (``--parallel``; default ``tp`` for N > 1):
  * ``tp``: ONE provider over all N GPUs -- Llama-3-8B tensor-parallel (TP=N,
    Megatron column/row split, the decode all-reduces on the one-shot xGMI
    kernel, RCCL for the rest), rank 0 schedules and streams, ranks 1..N-1
    mirror each step from the shared-memory metadata ring (pipelined decode).
    ``--clients`` concurrent clients in total (default 10 = maxConnections):
    "strong" scaling -- each client's stream gets faster as GPUs are added.
  * ``dp``: N independent providers, one per GPU, ``--clients`` each: "weak"
    scaling of aggregate throughput.

Timing (the driver contract): the engine runs its start-up warmup (prefill
size classes, hipGraph capture); W warmup steps (the prefill of all prompts +
decode steps) are untimed; then exactly K decode steps (one token for every
client) are timed between sync points (every rank's GPU idle + a barrier) on
both sides; the max over ranks is reported.  Every generated token is
detokenized and SSE-encoded for its client inside the timed loop.

Headline ``value``: streamed tokens/s PER CLIENT (the metric's own unit), the median over the clients of
the client-end run below -- measured at the client sockets; the engine-side per-client rate (1000 /
ms_per_step) and the aggregate over all clients are reported next to it.

Client end (``--client-end``, default on): after the timed steps the same
engine serves as a real provider -- discovery node, Symmetry server, provider
node and ``--clients`` swarm clients in a separate process over Noise XX +
secretstream -- and per-client streamed tokens/s and p50 TTFT are measured on
the client sockets (``symmetry_amd/testing/e2e.py``), reported under
``client_end`` and as the top-level ``p50_ttft_ms`` / ``client_end_*`` fields.
"""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

METRIC = "streamed tokens/sec + p50 TTFT per client, Llama-3-8B provider, 1/2/4/8 MI355X"


def _args():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=64)
    ap.add_argument("--warmup", type=int, default=8)
    ap.add_argument("--model", default="llama3:8b")
    ap.add_argument("--parallel", choices=("auto", "tp", "dp"), default="auto",
                    help="tp: one provider over all GPUs (default for N > 1); dp: one provider per GPU")
    ap.add_argument("--clients", type=int, default=10,
                    help="concurrent clients (maxConnections): in total under tp, per GPU under dp")
    ap.add_argument("--prompt-len", type=int, default=128)
    ap.add_argument("--max-model-len", type=int, default=8192)
    ap.add_argument("--client-end", type=int, default=1, help="1: also measure at the client sockets")
    ap.add_argument("--client-tokens", type=int, default=256, help="tokens per client in the client-end run")
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--nt-weights", type=int, default=None, help="A/B: non-temporal decode weight loads (0/1)")
    ap.add_argument("--max-batched-tokens", type=int, default=None, help="A/B: token budget of a pure-prefill step")
    ap.add_argument("--mixed-prefill-tokens", type=int, default=None, help="A/B: prompt budget of mixed steps")
    ap.add_argument("--profile-steps", type=int, default=0, help="extra decode steps after timing (for rocprof)")
    ap.add_argument("--verify-clients", type=int, default=2,
                    help="after timing: check every token these clients received against the fp32 oracle (0: off)")
    ap.add_argument("--verify-tol", type=float, default=VERIFY_TOL)
    return ap.parse_args()


# A streamed token passes if its oracle logit is within this of the oracle's best at that position: the bf16
# engine and the fp32 oracle differ by rounding, and a near-tie may go either way (tests/test_tp_gpu.py
# _check_oracle).  A wrong kernel on the real shapes misses by whole logits, not by this.
VERIFY_TOL = 0.08


def verify_streams(eng, checks, group, tol):
    """Every rank: the fp32 oracle (models/reference_model.py, teacher-forced over the streamed tokens) on the
    engine's own weights; under TP each rank runs its shard and the oracle sums / gathers over ``group``.
    ``checks`` (rank 0: [(prompt_ids, output_ids)], others: None) is broadcast first.  Returns the summary."""
    import torch.distributed as dist

    from symmetry_amd.models import reference_model as rm

    if group is not None:
        box = [checks]
        dist.broadcast_object_list(box, src=0, group=eng.runner.cpu_group)
        checks = box[0]
    res = {"clients": len(checks), "tokens": 0, "mismatches": 0, "max_gap": 0.0, "tol": tol, "per_client": []}
    for prompt, out in checks:
        lg = rm.forward_logits(eng.weights, list(prompt) + list(out)[:-1], group=group)
        r = rm.check_tokens(lg, len(prompt), list(out), tol)
        del lg
        res["per_client"].append(r)
        res["tokens"] += r["tokens"]
        res["mismatches"] += r["mismatches"]
        res["max_gap"] = max(res["max_gap"], r["max_gap"])
    return res


SHARED_GPU_ENV = "SYMMETRY_BENCH_SHARED_GPU"


def _fail(args, msg: str) -> int:
    """One JSON line with an ``error`` (never a silently smaller measurement) and a non-zero exit."""
    print(json.dumps({"metric": METRIC, "value": None, "unit": "tokens/s per client", "n_gpus": args.gpus,
                      "steps": args.steps, "warmup": args.warmup, "error": msg}), flush=True)
    return 2


def visible_gpus() -> int:
    """GPUs this process may use, counted without initialising the HIP runtime (``device_count()`` only
    enumerates on this stack; ``HIP_VISIBLE_DEVICES`` restricts it)."""
    import torch

    return int(torch.cuda.device_count())


def launch_plan(args_argv: list, n: int, port: int) -> list:
    """argv of the ONE torchrun child that runs ``n`` ranks of this bench (one per GPU, 127.0.0.1 rendezvous)."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
            "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.join(ROOT, "bench.py"), *args_argv]


def _self_launch(args) -> int | None:
    """``python bench.py --gpus N`` (N > 1) outside a launcher: check the GPUs, then start the N ranks as one
    ``torch.distributed.run`` child -- before this process makes any GPU call, never an exec -- relay its output
    and exit with its return code.  Under a launcher: ``WORLD_SIZE`` must equal ``--gpus``.

    No GPUs visible (CPU container): the ranks run on the CPU (gloo), the rehearsal the tests use.  Fewer GPUs
    than asked: an error line, unless ``SYMMETRY_BENCH_SHARED_GPU=1`` lets the ranks share the visible GPUs
    (a one-GPU rehearsal: host-staged gloo collectives + the xGMI kernels between the processes + decode
    hipGraphs)."""
    world = os.environ.get("WORLD_SIZE")
    if world is not None:
        if int(world) != args.gpus:
            return _fail(args, f"--gpus {args.gpus} but the launcher started {world} ranks")
        return None
    if args.gpus <= 1:
        return None
    import socket
    import subprocess

    n = visible_gpus()
    env = dict(os.environ)
    if 0 < n < args.gpus:
        if os.environ.get(SHARED_GPU_ENV) != "1":
            return _fail(args, f"--gpus {args.gpus} needs {args.gpus} GPUs, {n} visible "
                               f"({SHARED_GPU_ENV}=1 rehearses the ranks on the visible GPUs)")
        for k, v in (("SYMMETRY_TP_COMM", "gloo"), ("SYMMETRY_XGMI", "1"), ("SYMMETRY_XGMI_GRAPHS", "1"),
                     ("SYMMETRY_DIST_BACKEND", "gloo")):
            env.setdefault(k, v)
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    p = subprocess.Popen(launch_plan(sys.argv[1:], args.gpus, port), env=env)
    try:
        return abs(p.wait())
    except KeyboardInterrupt:
        p.terminate()
        return abs(p.wait())


def main() -> int:
    args = _args()
    code = _self_launch(args)
    if code is not None:
        return code
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    parallel = args.parallel if args.parallel != "auto" else ("tp" if world > 1 else "dp")
    gpu = torch.cuda.is_available()
    if gpu:
        torch.cuda.set_device(local % torch.cuda.device_count())

    from symmetry_amd import ops
    from symmetry_amd.engine.llm_engine import EngineConfig, LLMEngine
    from symmetry_amd.engine.sequence import SamplingParams
    from symmetry_amd.protocol import sse

    if gpu and not ops.native_available():
        raise SystemExit("native kernels missing: run `python -m symmetry_amd._build` first")
    if args.nt_weights is not None and ops.native_available():
        from symmetry_amd.ops import _native
        _native.ops().decode_gemm_nt(int(args.nt_weights))

    C, P, W, K = args.clients, args.prompt_len, args.warmup, args.steps
    block = 64
    blocks = C * ((args.max_model_len + block - 1) // block) + 16
    cfg = EngineConfig(model=args.model, device="auto", seed=1234 + (0 if parallel == "tp" else rank),
                       max_num_seqs=C, max_model_len=args.max_model_len, block_size=block, num_kv_blocks=blocks,
                       use_graphs=not args.no_graphs, max_num_batched_tokens=max(8192, C * P))
    if args.max_batched_tokens is not None:
        cfg.max_num_batched_tokens = args.max_batched_tokens
    if args.mixed_prefill_tokens is not None:
        cfg.mixed_prefill_tokens = args.mixed_prefill_tokens

    t0 = time.perf_counter()
    if parallel == "tp" and world > 1:
        from symmetry_amd.parallel.launch import init_tp_engine

        eng, rank = init_tp_engine(cfg)
        group = eng.runner.cpu_group
    else:
        group = None
        if world > 1:
            # SYMMETRY_DIST_BACKEND=gloo rehearses the multi-rank flow with several ranks on one GPU (RCCL
            # refuses two ranks on one device); the driver's multi-GPU runs use RCCL
            backend = os.environ.get("SYMMETRY_DIST_BACKEND", "nccl" if gpu else "gloo")
            dist.init_process_group(backend, device_id=torch.device("cuda", local) if gpu and backend == "nccl"
                                    else None)
            group = dist.new_group(backend="gloo")
        eng = LLMEngine(cfg)
    t_load = time.perf_counter() - t0
    tp_worker = parallel == "tp" and world > 1 and rank != 0
    runner = eng.runner

    if tp_worker:
        # mirror rank 0 (warmup, graph capture, timed steps, client-end run) until it stops the plane
        runner.worker_loop()
        if args.verify_clients > 0:
            verify_streams(eng, None, dist.group.WORLD, args.verify_tol)
        elapsed = runner.sync_times[1] - runner.sync_times[0] if len(runner.sync_times) >= 2 else 0.0
        _reduce_and_exit(group, elapsed, [], world)
        return 0

    # provider start-up (not timed): prefill size classes + decode hipGraph capture
    t_cap = eng.warmup([n for n in (16, 128, 512, C * P) if n <= cfg.max_num_batched_tokens])

    def sync() -> float:
        if parallel == "tp" or world == 1:
            return runner.sync_point()
        if gpu:
            torch.cuda.synchronize()
        dist.barrier(group=group)
        if gpu:
            torch.cuda.synchronize()
        return time.perf_counter()

    # ---- clients: synthetic chat prompts of exactly P tokens, SSE-encoded streaming sinks
    g = torch.Generator().manual_seed(99 + rank)
    streams = {f"client-{i}": [] for i in range(C)}
    model_name = eng.model_cfg.name

    def sink(rid):
        buf = streams[rid]

        def cb(out):
            buf.append(sse.chunk_event(rid, model_name, out.text, finish_reason=out.finish_reason))
        return cb

    total_steps = W + K + args.profile_steps
    params = SamplingParams(max_tokens=total_steps + 2, temperature=0.0, ignore_eos=True)
    prefix = eng.tokenizer.apply_chat_template([{"role": "user", "content": ""}])
    seqs = []
    for i in range(C):
        body = torch.randint(256, max(257, eng.model_cfg.vocab_size - 1024), (max(1, P - len(prefix)),),
                             generator=g).tolist()
        seqs.append(eng.add_request(f"client-{i}", (prefix + body)[:P], params, sink(f"client-{i}")))

    # ---- warmup: prefill (TTFT) + W decode steps
    while any(s.first_token_time is None for s in seqs):
        eng.step()
    ttfts = sorted(s.ttft for s in seqs)
    for _ in range(W):
        eng.step()
    t1 = sync()
    tm0 = dict(runner.timing)
    for _ in range(K):
        eng.step()
    elapsed = sync() - t1
    host_ms = {k: round((runner.timing[k] - tm0[k]) / K * 1e3, 4)
               for k in ("fill", "send", "run", "graph_launch", "d2h")}
    for _ in range(args.profile_steps):
        eng.step()
    for s in seqs:
        eng.abort(s.request_id)
    while eng.has_unfinished():
        eng.step()
    events = sum(len(v) for v in streams.values())

    client_end = None
    if args.client_end and rank == 0:
        from symmetry_amd.testing.e2e import client_end_run

        try:
            client_end = asyncio.run(client_end_run(eng, args.model, C, prompt_tokens=P,
                                                    max_tokens=args.client_tokens))
        except Exception as exc:  # the engine-step measurement stands on its own
            client_end = {"error": f"{type(exc).__name__}: {exc}"}
    # what the clients received must be the model's output: every streamed token of the first clients against
    # the fp32 oracle of the same weights (a fast but wrong kernel fails the bench instead of posting a number)
    checks = [(list(s.prompt_ids), list(s.output_ids)) for s in seqs[:max(0, args.verify_clients)]]
    verified = None
    if parallel == "tp" and world > 1:
        eng.shutdown()
        if checks:
            verified = verify_streams(eng, checks, dist.group.WORLD, args.verify_tol)
    else:
        if checks:
            verified = verify_streams(eng, checks, None, args.verify_tol)
        if world > 1:
            dist.barrier(group=group)
    elapsed, ttfts, rank_elapsed = _reduce(group, elapsed, ttfts, world, gather_ttft=parallel == "dp")

    p50_ttft = ttfts[len(ttfts) // 2] * 1e3
    mean_ttft, max_ttft = sum(ttfts) / len(ttfts) * 1e3, ttfts[-1] * 1e3
    ms_step = elapsed / K * 1e3
    n_clients = C * (world if parallel == "dp" else 1)
    total_tps = n_clients * K / elapsed
    per_client = 1e3 / ms_step
    ce_ok = client_end is not None and client_end.get("per_client_tokens_per_s_median") is not None
    # the headline IS the metric's "per client" rate: measured at the client sockets (SSE over Noise XX +
    # secretstream, clients in another process) when the client-end run worked, else the engine-side rate
    value = client_end["per_client_tokens_per_s_median"] if ce_ok else round(per_client, 2)
    if rank == 0:
        line = {
            "metric": METRIC,
            "value": value,
            "unit": "tokens/s per client",
            "n_gpus": world,
            "steps": K,
            "warmup": W,
            "ms_per_step": round(ms_step, 4),
            "higher_is_better": True,
            "scaling": "strong" if parallel == "tp" and world > 1 else "weak",
            "vs_baseline": None,
            "dtype": "bf16",
            "data": "synthetic 128-token prompts, random-init weights (real Llama-3-8B architecture)",
            "config": {"model": args.model, "global_batch": n_clients, "seq_len": P,
                       "parallelism": f"{parallel}{world}", "clients": n_clients,
                       "clients_per_provider": C, "max_model_len": args.max_model_len,
                       "decode": "greedy", "hipgraphs": bool(runner.use_graphs),
                       "tp_comm": type(eng.model.tp).__name__ if eng.model.tp is not None else None,
                       "ops": ("torch-eager (baseline B1)" if ops.torch_mode() else
                               "native gfx950 HIP" if gpu else "torch reference (CPU)")},
            "value_source": "client_end (socket-measured median over clients)" if ce_ok else "engine timed steps",
            "aggregate_tokens_per_s": round(total_tps, 2),
            "engine_per_client_tokens_per_s": round(per_client, 2),
            "per_rank_ms_per_step": [round(e / K * 1e3, 4) for e in rank_elapsed],
            # rank 0's host time per timed step inside ModelRunner.launch: metadata packing, the TP metadata-plane
            # push, H2D copy + graph replay enqueue, D2H copy + event enqueue
            "host_ms_per_step": host_ms,
            "engine_p50_ttft_ms": round(p50_ttft, 2),
            "engine_mean_ttft_ms": round(mean_ttft, 2),
            "engine_max_ttft_ms": round(max_ttft, 2),
            "load_s": round(t_load, 1),
            "warmup_s": round(t_cap, 1),
            "sse_events_rank0": events,
        }
        if parallel == "tp" and world > 1:
            tp = eng.model.tp
            line["tp"] = {"xgmi_calls": dict(getattr(tp, "calls", {})),
                          "prefill_allreduce_bytes_per_rank": dict(eng.model.tp_reduced_bytes),
                          "metadata_plane": type(runner.meta).__name__}
        if verified is not None:
            line["verified"] = verified
        if client_end is not None:
            line["client_end"] = client_end
            line["p50_ttft_ms"] = client_end.get("p50_ttft_ms")
            line["client_end_per_client_tokens_per_s"] = client_end.get("per_client_tokens_per_s_median")
        else:
            line["p50_ttft_ms"] = round(p50_ttft, 2)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()
    if verified is not None and verified["mismatches"]:
        print(f"bench: {verified['mismatches']} of {verified['tokens']} streamed tokens disagree with the fp32 "
              "oracle", file=sys.stderr, flush=True)
        return 3
    return 0


def _reduce(group, elapsed, ttfts, world, gather_ttft):
    """Max elapsed over ranks (+ every rank's own); all ranks' TTFTs (dp: every rank has its own clients)."""
    import torch
    import torch.distributed as dist

    if world == 1:
        return elapsed, ttfts, [elapsed]
    tt = torch.tensor([elapsed], dtype=torch.float64)
    every = [torch.zeros_like(tt) for _ in range(world)]
    dist.all_gather(every, tt, group=group)
    per_rank = [float(t.item()) for t in every]
    if gather_ttft:
        tf = torch.tensor(ttfts, dtype=torch.float64)
        allt = [torch.zeros_like(tf) for _ in range(world)]
        dist.all_gather(allt, tf, group=group)
        ttfts = sorted(torch.cat(allt).tolist())
    return max(per_rank), ttfts, per_rank


def _reduce_and_exit(group, elapsed, ttfts, world):
    import torch.distributed as dist

    _reduce(group, elapsed, ttfts, world, gather_ttft=False)
    dist.destroy_process_group()


if __name__ == "__main__":
    sys.exit(main())
