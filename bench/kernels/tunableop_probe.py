"""Probe: hipBLASLt's default heuristic vs PyTorch TunableOp-selected solutions for the prefill GEMMs of
Llama-3-8B (x @ W.T, bf16) at the bench's prefill step sizes.  Run twice: plain (default heuristic), then with
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 (tunes each shape on first use, then times it).
Output: one JSON line per (shape, M)."""
import argparse
import json
import os

import torch

SHAPES = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, nargs="+", default=[512, 768, 1024])
    ap.add_argument("--iters", type=int, default=50)
    args = ap.parse_args()
    dev = torch.device("cuda")
    tuned = os.environ.get("PYTORCH_TUNABLEOP_ENABLED", "0") == "1"
    for name, (N, K) in SHAPES.items():
        w = (torch.randn(N, K, device=dev) * 0.02).bfloat16()
        for M in args.m:
            x = torch.randn(M, K, device=dev).bfloat16()
            y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            for _ in range(3):
                torch.matmul(x, w.t(), out=y)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.iters):
                torch.matmul(x, w.t(), out=y)
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / args.iters
            print(json.dumps({"shape": name, "M": M, "N": N, "K": K, "tunableop": tuned, "us": round(us, 1),
                              "TFLOPs": round(2 * M * N * K / us / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
