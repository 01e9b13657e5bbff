#!/usr/bin/env python3
"""Multi-turn chat TTFT: the reference's clients resend the whole conversation every turn
(REF src/provider.ts:312-316), so turn k's prompt = turn k-1's prompt + answer + a new user message.
Measures TTFT per turn with automatic prefix caching on and off (same engine settings otherwise).

  python bench/multiturn.py --turns 4 --system-len 1024 --user-len 64 --answer-len 64
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run(caching: bool, args):
    import torch

    from symmetry_amd.engine.llm_engine import EngineConfig, LLMEngine
    from symmetry_amd.engine.sequence import SamplingParams

    eng = LLMEngine(EngineConfig(model=args.model, max_num_seqs=4, max_model_len=8192, num_kv_blocks=1024,
                                 enable_prefix_caching=caching))
    eng.warmup([16, 128, 512, 2048])
    g = torch.Generator().manual_seed(5)
    rnd = lambda n: torch.randint(300, 30000, (n,), generator=g).tolist()  # noqa: E731
    convo = rnd(args.system_len)
    ttfts = []
    for t in range(args.turns):
        convo = convo + rnd(args.user_len)
        torch.cuda.synchronize()
        seq = eng.add_request(f"turn{t}-{caching}", convo, SamplingParams(max_tokens=args.answer_len, ignore_eos=True))
        t0 = time.perf_counter()
        while not seq.output_ids:
            eng.step()
        ttfts.append((time.perf_counter() - t0) * 1e3)
        while eng.has_unfinished():
            eng.step()
        convo = convo + list(seq.output_ids)
    res = {"prefix_caching": caching, "prompt_lens": None, "ttft_ms": [round(x, 2) for x in ttfts],
           "cache_hit_tokens": eng.blocks.hit_tokens}
    del eng
    import gc
    gc.collect()
    torch.cuda.empty_cache()
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3:8b")
    ap.add_argument("--turns", type=int, default=4)
    ap.add_argument("--system-len", type=int, default=1024)
    ap.add_argument("--user-len", type=int, default=64)
    ap.add_argument("--answer-len", type=int, default=64)
    args = ap.parse_args()
    for caching in (False, True):
        r = run(caching, args)
        r["prompt_lens"] = [args.system_len + (t + 1) * args.user_len + t * args.answer_len for t in range(args.turns)]
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
