#!/usr/bin/env python3
"""Headline benchmark: streamed tokens/s + p50 TTFT per client of a Llama-3-8B provider.

Metric and config come from BASELINE.json ("streamed tokens/sec + p50 TTFT per
client, Llama-3-8B provider, 1/2/4/8 MI355X"; config 3: maxConnections=10
concurrent clients, continuous batching, greedy decode).

Per GPU (one process per GPU, launched by torch.distributed.run for N > 1):
  * a native engine serving Llama-3-8B (bf16, random-init weights of the real
    architecture, synthetic prompts: no network for checkpoints/datasets);
  * ``--clients`` concurrent chat requests (default 10 = maxConnections);
  * every generated token is detokenized and encoded as one OpenAI SSE
    ``chat.completion.chunk`` event for its client (the provider's streaming
    path).
Scaling is data-parallel ("weak"): each GPU runs its own provider engine and
clients, so per-GPU work is fixed as N grows.

A *step* is one engine decode step (one token for every client).  The engine
first runs its start-up warmup (one prefill per size class, hipGraph capture),
as a provider does before it announces itself.  W warmup steps (the prefill
of all prompts + decode steps) are untimed; then exactly K decode steps are timed between
barrier + synchronize on both sides; the max over ranks is reported.
p50 TTFT is measured on the prefill (all clients arrive together).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

METRIC = "streamed tokens/sec + p50 TTFT per client, Llama-3-8B provider, 1/2/4/8 MI355X"


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=64)
    ap.add_argument("--warmup", type=int, default=8)
    ap.add_argument("--model", default="llama3:8b")
    ap.add_argument("--clients", type=int, default=10, help="concurrent clients per GPU (maxConnections)")
    ap.add_argument("--prompt-len", type=int, default=128)
    ap.add_argument("--max-model-len", type=int, default=8192)
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--persistent-mlp", action="store_true", help="O/gate_up/down as one persistent launch (A/B)")
    ap.add_argument("--attn-block", type=int, default=None, help="A/B: QKV -> attention -> O as one launch (0/1)")
    ap.add_argument("--nt-weights", type=int, default=None, help="A/B: non-temporal decode weight loads (0/1)")
    ap.add_argument("--max-batched-tokens", type=int, default=None, help="A/B: token budget of a pure-prefill step")
    ap.add_argument("--mixed-prefill-tokens", type=int, default=None, help="A/B: prompt budget of mixed steps")
    ap.add_argument("--profile-steps", type=int, default=0, help="extra decode steps after timing (for rocprof)")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if torch.cuda.is_available():
        torch.cuda.set_device(local % torch.cuda.device_count())
    if world > 1:
        # SYMMETRY_DIST_BACKEND=gloo rehearses the multi-rank flow with several ranks on one GPU (RCCL
        # refuses two ranks on one device); the driver's multi-GPU runs use RCCL
        backend = os.environ.get("SYMMETRY_DIST_BACKEND", "nccl" if torch.cuda.is_available() else "gloo")
        dist.init_process_group(backend, device_id=torch.device("cuda", local)
                                if torch.cuda.is_available() and backend == "nccl" else None)

    from symmetry_amd import ops
    from symmetry_amd.engine.llm_engine import EngineConfig, LLMEngine
    from symmetry_amd.engine.sequence import SamplingParams
    from symmetry_amd.protocol import sse

    if torch.cuda.is_available() and not ops.native_available():
        raise SystemExit("native kernels missing: run `python -m symmetry_amd._build` first")

    if args.nt_weights is not None and ops.native_available():
        from symmetry_amd.ops import _native
        _native.ops().decode_gemm_nt(int(args.nt_weights))

    C, P, W, K = args.clients, args.prompt_len, args.warmup, args.steps
    block = 64
    blocks = C * ((args.max_model_len + block - 1) // block) + 16
    cfg = EngineConfig(model=args.model, device="auto", seed=1234 + rank, max_num_seqs=C,
                       max_model_len=args.max_model_len, block_size=block, num_kv_blocks=blocks,
                       use_graphs=not args.no_graphs, max_num_batched_tokens=max(8192, C * P),
                       persistent_mlp=args.persistent_mlp)
    if args.max_batched_tokens is not None:
        cfg.max_num_batched_tokens = args.max_batched_tokens
    if args.mixed_prefill_tokens is not None:
        cfg.mixed_prefill_tokens = args.mixed_prefill_tokens
    if args.attn_block is not None:
        cfg.fused_attn_block = bool(args.attn_block)
    t0 = time.perf_counter()
    eng = LLMEngine(cfg)
    t_load = time.perf_counter() - t0
    # provider start-up (not timed): prefill size classes + decode hipGraph capture
    t_cap = eng.warmup([n for n in (16, 128, 512, C * P) if n <= cfg.max_num_batched_tokens])
    sync = torch.cuda.synchronize if torch.cuda.is_available() else (lambda: None)

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
        body = torch.randint(256, max(257, eng.model_cfg.vocab_size - 1024), (max(1, P - len(prefix)),), generator=g).tolist()
        seqs.append(eng.add_request(f"client-{i}", (prefix + body)[:P], params, sink(f"client-{i}")))

    # ---- warmup: prefill (TTFT) + W decode steps
    steps_done = 0
    while any(s.first_token_time is None for s in seqs):
        eng.step()
        steps_done += 1
    ttfts = sorted(s.ttft for s in seqs)
    for _ in range(W):
        eng.step()
        steps_done += 1
    sync()
    if world > 1:
        dist.barrier()
    sync()
    t1 = time.perf_counter()
    for _ in range(K):
        eng.step()
    sync()
    if world > 1:
        dist.barrier()
    sync()
    elapsed = time.perf_counter() - t1
    for _ in range(args.profile_steps):
        eng.step()
    sync()

    if world > 1:
        tt = torch.tensor([elapsed], device="cuda" if torch.cuda.is_available() else "cpu", dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
        tf = torch.tensor(ttfts, device=tt.device, dtype=torch.float64)
        allt = [torch.zeros_like(tf) for _ in range(world)]
        dist.all_gather(allt, tf)
        ttfts = sorted(torch.cat(allt).tolist())
    p50_ttft = ttfts[len(ttfts) // 2] * 1e3
    mean_ttft, max_ttft = sum(ttfts) / len(ttfts) * 1e3, ttfts[-1] * 1e3
    ms_step = elapsed / K * 1e3
    total_tps = world * C * K / elapsed
    per_client = 1e3 / ms_step
    events = sum(len(v) for v in streams.values())
    if rank == 0:
        print(json.dumps({
            "metric": METRIC,
            "value": round(total_tps, 2),
            "unit": "tokens/s",
            "n_gpus": world,
            "steps": K,
            "warmup": W,
            "ms_per_step": round(ms_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16",
            "data": "synthetic prompts, random-init weights (real Llama-3-8B architecture)",
            "config": {"model": args.model, "global_batch": world * C, "seq_len": P,
                       "parallelism": f"dp{world}", "clients_per_gpu": C, "max_model_len": args.max_model_len,
                       "decode": "greedy", "hipgraphs": bool(eng.runner.use_graphs),
                       "ops": ("torch-eager (baseline B1)" if ops.torch_mode() else
                               "native gfx950 HIP" if torch.cuda.is_available() else "torch reference (CPU)")},
            "per_client_tokens_per_s": round(per_client, 2),
            "p50_ttft_ms": round(p50_ttft, 2),
            "mean_ttft_ms": round(mean_ttft, 2),
            "max_ttft_ms": round(max_ttft, 2),
            "load_s": round(t_load, 1),
            "warmup_s": round(t_cap, 1),
            "sse_events_rank0": events,
        }), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
