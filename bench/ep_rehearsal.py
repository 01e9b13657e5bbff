#!/usr/bin/env python3
"""One-GPU expert-parallel rehearsal of Mixtral-8x7B (BASELINE config 5's EP form): N processes share cuda:0,
attention tensor-parallel and the experts expert-parallel over the N ranks (parallel/launch.py init_tp_engine),
random-init weights in the single-copy preshuffled layout.  For each prompt total T (C prompts of T / C tokens in
one prefill step) it reports the TTFT of the step and the bytes rank 0's MoE collectives pushed per layer, for
one combine mode per run (``--mode a2a``: the replicated-token owner exchange, models/moe.py forward_a2a;
``--mode allreduce``: the fp32 all-reduce combine).

What transfers to an 8-GPU node and what does not: the byte counts are exact (the same routing, the same
exchange); the owner exchange runs on the peer-memory a2a kernel (IPC buffers, here all on one HBM); the
all-reduce of prefill-sized partials and the owners' all-gather run on the host-staged gloo communicator (RCCL
refuses two ranks on one device), so their time here is a slow-transport stand-in, proportional to their bytes.
The ranks also share one GPU's CUs, so expert GEMM time is the full model's, not a shard's.

  python bench/ep_rehearsal.py --world 2 --mode a2a --tokens 64,128,256,512,1024 >> gpurun_out/ep.jsonl
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def _port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _entry(rank, world, port, args, q):
    import traceback

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK="0", SYMMETRY_TP_COMM="gloo", SYMMETRY_XGMI="1", SYMMETRY_MOE_A2A_STATS="1",
                      SYMMETRY_MOE_MODE=args.mode, SYMMETRY_XGMI_FUSED="0")
    try:
        import torch

        from symmetry_amd.engine.llm_engine import EngineConfig
        from symmetry_amd.engine.sequence import SamplingParams
        from symmetry_amd.parallel.launch import init_tp_engine

        tokens = [int(t) for t in args.tokens.split(",")]
        ecfg = EngineConfig(model=args.model, device=args.device, max_num_seqs=32, max_model_len=2048,
                            max_num_batched_tokens=max(max(tokens), 2048), num_kv_blocks=args.kv_blocks,
                            use_graphs=False, decode_weights="replace")
        eng, r = init_tp_engine(ecfg)
        moe = eng.runner.model.moe
        sync = torch.cuda.synchronize if args.device != "cpu" else (lambda: None)
        if r != 0:
            eng.runner.worker_loop()
            q.put((rank, moe.a2a_stats()))
            return
        layers = eng.model_cfg.num_layers
        vocab = eng.model_cfg.vocab_size
        rows = []
        try:
            for T in tokens:
                C = max(1, T // 128)
                L = T // C
                ts, bys = [], []
                for rep in range(args.reps + 1):  # rep 0: warmup (first use of this step shape)
                    base = 1000 + 7919 * rep + 131 * T
                    prompts = [[(base + 613 * c + 17 * i) % (vocab - 20) + 10 for i in range(L)] for c in range(C)]
                    s0 = moe.a2a_stats()
                    sync()
                    t0 = time.perf_counter()
                    for c, p in enumerate(prompts):
                        eng.add_request(f"ep-{T}-{rep}-{c}", p, SamplingParams(max_tokens=1, ignore_eos=True))
                    while eng.has_unfinished():
                        eng.step()
                    sync()
                    dt = time.perf_counter() - t0
                    s1 = moe.a2a_stats()
                    if rep:
                        ts.append(dt * 1e3)
                        bys.append({k: (s1[k] - s0[k]) / layers for k in s1})
                per_layer = {k: statistics.median(b[k] for b in bys) for k in bys[0]}
                pushed = per_layer["allreduce"] if args.mode == "allreduce" else (
                    per_layer["return"] + per_layer["gather"] + per_layer["dispatch"])
                rows.append({"world": world, "mode": args.mode, "tokens": C * L, "prompts": C,
                             "ttft_ms": round(statistics.median(ts), 2), "ttft_ms_min": round(min(ts), 2),
                             "bytes_per_layer_rank0": int(pushed),
                             "detail_per_layer": {k: int(v) for k, v in per_layer.items() if v},
                             "moe_calls": dict(moe.calls)})
                print(json.dumps(rows[-1]), flush=True)
        finally:
            eng.shutdown()
        q.put((rank, rows))
    except Exception:
        q.put((rank, traceback.format_exc()))
    finally:
        import torch.distributed as dist

        if dist.is_initialized():
            dist.destroy_process_group()


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=2)
    ap.add_argument("--mode", choices=["a2a", "allreduce"], default="a2a")
    ap.add_argument("--model", default="mixtral:8x7b")
    ap.add_argument("--tokens", default="64,128,256,512,1024")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--kv-blocks", type=int, default=256)
    ap.add_argument("--device", default="cuda", help="cpu: a gloo smoke run of the script (tiny models)")
    args = ap.parse_args()
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    port = _port()
    procs = [ctx.Process(target=_entry, args=(r, args.world, port, args, q)) for r in range(args.world)]
    for p in procs:
        p.start()
    res = dict(q.get() for _ in range(args.world))
    for p in procs:
        p.join(120)
    errs = [v for v in res.values() if isinstance(v, str)]
    if errs:
        sys.stderr.write(errs[0])
        return 1
    return 0


if __name__ == "__main__":
    sys.exit(main())
