#!/usr/bin/env python3
"""TTFT / prefill throughput of the native engine: C prompts of L tokens arriving together.

Reports the wall time of the prefill step(s) that produce every first token (= TTFT of the last client),
prefill tokens/s and achieved TFLOP/s (2 x params x tokens + attention), after the engine's start-up warmup.

  python bench/prefill.py --model llama3:8b --clients 10 --prompt-len 128 --reps 5
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3:8b")
    ap.add_argument("--clients", type=int, default=10)
    ap.add_argument("--prompt-len", type=int, default=128)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--ab-moe-grouped", action="store_true",
                    help="MoE: alternate grouped MFMA GEMMs / per-expert library GEMMs (host sync) per rep")
    ap.add_argument("--ab-moe-pg", action="store_true",
                    help="MoE: alternate the prefill GEMM kernel's grouped mode (ops.pg_grouped) / the grouped_gemm "
                         "kernels per rep")
    ap.add_argument("--ab-pgemm", action="store_true",
                    help="dense: alternate the prefill GEMM path (pgemm, fused epilogues) / the library path per rep")
    args = ap.parse_args()
    from symmetry_amd.engine.llm_engine import EngineConfig, LLMEngine

    C, L = args.clients, args.prompt_len
    eng = LLMEngine(EngineConfig(model=args.model, max_num_seqs=max(C, 1), max_model_len=max(2048, L + 64),
                                 max_num_batched_tokens=max(8192, C * L)))
    eng.warmup([16, 128, 512, C * L] if C * L > 512 else None)
    from symmetry_amd import ops
    from symmetry_amd.models import moe as moe_mod

    if args.ab_pgemm:
        def set_arm(a):
            ops._PGEMM_ON = a
    elif args.ab_moe_pg:
        def set_arm(a):
            moe_mod.PG_GROUPED = a
    else:
        def set_arm(a):
            moe_mod.GROUPED = a
    arms = [True, False] if (args.ab_moe_grouped or args.ab_pgemm or args.ab_moe_pg) else [moe_mod.GROUPED]
    times = {a: [] for a in arms}
    for r in range(args.reps):  # arms interleaved per rep: drift hits both
        for k, arm in enumerate(arms):
            set_arm(arm)
            times[arm].append(_once(eng, C, L, r, salt=k))
    res = {a: sorted(t)[len(t) // 2] for a, t in times.items()}
    cfg = eng.model_cfg
    toks = C * L
    vd = cfg.vocab_size * cfg.hidden_size
    body = cfg.num_params() - vd - (0 if cfg.tie_embeddings else vd)  # layers only: embedding is a gather
    flops = 2 * body * toks + 2 * vd * C + 4 * cfg.num_layers * cfg.num_heads * cfg.head_dim * C * L * L / 2
    for arm, t in res.items():
        out = {"model": args.model, "clients": C, "prompt_len": L, "ttft_ms": round(t * 1e3, 2),
               "prefill_tokens_per_s": round(toks / t), "tflops": round(flops / t / 1e12, 1)}
        if args.ab_pgemm:
            out["pgemm"] = arm
        elif args.ab_moe_pg:
            out["moe_pg_grouped"] = arm
        elif cfg.is_moe:
            out["moe_grouped_gemm"] = arm
        print(json.dumps(out), flush=True)


def _once(eng, C, L, r, salt=0):
    """TTFT of the last client of one burst (``salt`` / ``r`` keep the prompts apart: no prefix-cache hits)."""
    import torch

    from symmetry_amd.engine.sequence import SamplingParams

    seqs = [eng.add_request(f"p{salt}-{r}-{i}", [(97 * i + 13 * k + r + 1009 * salt) % 30000 + 300 for k in range(L)],
                            SamplingParams(max_tokens=1, ignore_eos=True)) for i in range(C)]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    while not all(s.output_ids for s in seqs):
        eng.step()
    torch.cuda.synchronize()
    t = time.perf_counter() - t0
    while eng.has_unfinished():
        eng.step()
    return t


if __name__ == "__main__":
    main()
