"""Microbenchmark: skinny decode GEMM variants on the Llama-3-8B projection shapes.

Weights are rotated over enough copies (>= 1 GiB) that every call streams
from HBM, as in a real decode step (the 256 MiB Infinity Cache would
otherwise serve repeated calls).  Variants are timed interleaved in one
process (cdna_hip_programming.md §5.4 rule 24).
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch

from symmetry_amd import ops

SHAPES = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336),
          "lm_head": (128256, 4096)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, nargs="+", default=[1, 10, 32])
    ap.add_argument("--variants", type=int, nargs="+", default=[0, 1, 2, 3])
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--splits", type=str, default="auto")
    args = ap.parse_args()
    dev = torch.device("cuda")
    res = []
    for name, (N, K) in SHAPES.items():
        nbytes = N * K * 2
        copies = max(2, (1 << 30) // nbytes + 1)
        ws = [torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02 for _ in range(copies)]
        for M in args.m:
            x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
            splits = [ops.choose_splits(N, K)] if args.splits == "auto" else [int(s) for s in args.splits.split(",")]
            for S in splits:
                if K % (256 * S):
                    continue
                y = torch.empty(S, M, N, device=dev)
                times = {v: [] for v in args.variants}
                for v in args.variants:  # warm
                    if v == 3 and N % 32:
                        continue
                    ops.skinny_gemm(x, ws[0], y, v)
                torch.cuda.synchronize()
                for it in range(args.iters):
                    for v in args.variants:
                        if v == 3 and N % 32:
                            continue
                        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                        w = ws[it % copies]
                        e0.record()
                        ops.skinny_gemm(x, w, y, v)
                        e1.record()
                        torch.cuda.synchronize()
                        times[v].append(e0.elapsed_time(e1))
                for v, t in times.items():
                    if not t:
                        continue
                    t = sorted(t)
                    med = t[len(t) // 2] * 1e-3
                    r = {"shape": name, "N": N, "K": K, "M": M, "S": S, "variant": v, "us": round(med * 1e6, 2),
                         "TBps": round(nbytes / med / 1e12, 3)}
                    res.append(r)
                    print(json.dumps(r), flush=True)
        del ws
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
