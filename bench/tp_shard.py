#!/usr/bin/env python3
"""One TP rank's decode step on ONE GPU: the compute + collective-kernel time of a TP=N shard.

An N-GPU node is not available to this repo's development runs, so this measures what can be measured
on one MI355X: rank 0's shard of Llama-3-8B (or 70B) at TP=N -- the same sharded weights, the same fused
decode kernels at the shard shapes (e.g. QKV N = 768, O K = 512 at TP=8), the same hipGraph-captured
pipelined step -- with every collective running the real one-shot xGMI kernel on a world-1 communicator
(its push, flag and reduce on local HBM, no peer latency; the fused row-parallel GEMM + all-reduce launches
have no other rank's granules to wait for).  The step time is therefore a lower bound of
the TP=N step: real xGMI adds the peers' flag latency to each of the 2 per-layer collectives + the
sampling-keys one.  The model math is one shard's (outputs are not the full model's): timing only.

  python bench/tp_shard.py --tp 8 --clients 10 [--model llama3:70b]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


class LocalXgmi:
    """The XgmiComm interface over a world-1 xGMI communicator (every collective a real kernel launch)."""

    capturable = True

    def __init__(self, device, world: int, slot_bytes: int = 4 << 20):
        from symmetry_amd.ops import _native

        self.ops = _native.ops()
        self.rank, self.world = 0, world
        self.slot_bytes = slot_bytes
        self.handle = int(self.ops.xgmi_create(slot_bytes, 1, 0, device.index or 0))
        self.ops.xgmi_connect_local(self.handle, [self.handle])
        self.calls = {"all_reduce": 0, "add_prep": 0, "keys": 0}
        # the fused GEMM + all-reduce communicator (own slots of epoch-tagged granules, world 1: no peer granule
        # to wait for -- the launch is the GEMM + residual epilogue)
        self.xar = int(self.ops.xgmi_create(slot_bytes, 1, 0, device.index or 0))
        self.ops.xgmi_connect_local(self.xar, [self.xar])

    def all_reduce(self, t, op="sum"):
        # prefill-sized messages go to RCCL on a real node; a world-1 sum is the identity (not timed here)
        if op == "sum" and t.numel() * t.element_size() <= self.slot_bytes and t.numel() % 8 == 0:
            self.ops.xgmi_all_reduce(t, t, self.handle)
            self.calls["all_reduce"] += 1

    def all_reduce_add_prep(self, y, resid, w_next, xw, ss):
        self.ops.xgmi_add_prep(y, resid, w_next, xw, ss, self.handle)
        self.calls["add_prep"] += 1

    def argmax_keys(self, keys, ids):
        self.ops.xgmi_keys_max(keys, ids, self.handle)
        self.calls["keys"] += 1

    def gemm_ar_resid(self, x, W, wshuf, resid, w_next, xw, ss) -> bool:
        from symmetry_amd.parallel.comm import XAR

        if not XAR or x.shape[0] > 64 or x.shape[0] * resid.shape[1] * 8 > self.slot_bytes:
            return False
        ok = bool(self.ops.xgmi_gemm_ar_resid(x, W, bool(wshuf), resid, w_next, xw, ss, self.xar))
        if ok:
            self.calls["gemm_ar"] = self.calls.get("gemm_ar", 0) + 1
        return ok

    def all_gather(self, t):
        import torch

        return torch.cat([t] * self.world, 0)

    def error(self) -> int:
        return int(self.ops.xgmi_error(self.handle)) or int(self.ops.xgmi_error(self.xar))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3:8b")
    ap.add_argument("--tp", type=int, default=8)
    ap.add_argument("--clients", type=int, default=10)
    ap.add_argument("--prompt-len", type=int, default=128)
    ap.add_argument("--steps", type=int, default=64)
    ap.add_argument("--warmup", type=int, default=8)
    ap.add_argument("--max-model-len", type=int, default=2048)
    args = ap.parse_args()
    import torch

    from symmetry_amd.engine.llm_engine import EngineConfig, LLMEngine
    from symmetry_amd.engine.sequence import SamplingParams

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    C, P = args.clients, args.prompt_len
    comm = LocalXgmi(dev, args.tp)
    blocks = C * ((args.max_model_len + 63) // 64) + 16
    cfg = EngineConfig(model=args.model, device="cuda:0", max_num_seqs=C, max_model_len=args.max_model_len,
                       num_kv_blocks=blocks, tp_size=args.tp, tp_rank=0, weight_init="shard",
                       max_num_batched_tokens=max(8192, C * P))
    eng = LLMEngine(cfg, tp_comm=comm)
    print(f"loaded {args.model} TP={args.tp} shard", flush=True)
    eng.warmup([16, 128, C * P])
    print("warm", flush=True)
    params = SamplingParams(max_tokens=args.steps + args.warmup + 4, temperature=0.0, ignore_eos=True)
    seqs = [eng.add_request(f"c{i}", [(31 * i + 7 * k) % 100000 + 300 for k in range(P)], params) for i in range(C)]
    while any(s.first_token_time is None for s in seqs):
        if any(s.status.finished for s in seqs):
            raise SystemExit("a request failed (see the engine's traceback)")
        eng.step()
    for _ in range(args.warmup):
        eng.step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        eng.step()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / args.steps * 1e3
    err = comm.error()
    print(json.dumps({"model": args.model, "tp": args.tp, "rank_shard": 0, "clients": C,
                      "ms_per_step": round(ms, 4), "per_client_tokens_per_s_upper_bound": round(1e3 / ms, 1),
                      "collective_kernels": comm.calls, "xgmi_error": err, "hipgraphs": eng.runner.use_graphs,
                      "note": "one shard on one GPU, collectives on a world-1 xGMI communicator (no peer latency)"}),
          flush=True)


if __name__ == "__main__":
    main()
