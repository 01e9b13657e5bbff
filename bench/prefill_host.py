#!/usr/bin/env python3
"""Host vs device time of one prefill step (C prompts of L tokens): how long eng.step() takes to return
(host issue: Python + launches) against the step's wall time to the synchronised result.

  python bench/prefill_host.py --clients 1 --prompt-len 128
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
    ap.add_argument("--clients", type=int, nargs="+", default=[1, 2, 4, 10])
    ap.add_argument("--prompt-len", type=int, default=128)
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    import torch

    from symmetry_amd.engine.llm_engine import EngineConfig, LLMEngine
    from symmetry_amd.engine.sequence import SamplingParams

    L = args.prompt_len
    C_max = max(args.clients)
    eng = LLMEngine(EngineConfig(model=args.model, max_num_seqs=C_max, max_model_len=max(2048, L + 64),
                                 max_num_batched_tokens=max(8192, C_max * L)))
    eng.warmup([16, 128, 512, C_max * L])
    for C in args.clients:
        host, wall = [], []
        for r in range(args.reps):
            seqs = [eng.add_request(f"h{C}-{r}-{i}", [(97 * i + 13 * k + r) % 30000 + 300 for k in range(L)],
                                    SamplingParams(max_tokens=1, ignore_eos=True)) for i in range(C)]
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            eng.step()
            t1 = time.perf_counter()
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            host.append(t1 - t0)
            wall.append(t2 - t0)
            while eng.has_unfinished():
                eng.step()
        host.sort()
        wall.sort()
        print(json.dumps({"clients": C, "prompt_len": L, "host_issue_ms": round(host[len(host) // 2] * 1e3, 2),
                          "step_wall_ms": round(wall[len(wall) // 2] * 1e3, 2)}), flush=True)


if __name__ == "__main__":
    main()
