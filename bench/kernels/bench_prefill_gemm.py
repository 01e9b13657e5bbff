"""Prefill GEMM shapes of Llama-3-8B: default hipBLASLt heuristic vs PyTorch TunableOp's measured pick.

  python bench/kernels/bench_prefill_gemm.py --m 1280 10240
"""
import argparse
import json
import os
import sys
import tempfile

import torch

SHAPES = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336)}


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, nargs="+", default=[1280, 10240])
    args = ap.parse_args()
    dev = torch.device("cuda")
    res = {}
    for M in args.m:
        for name, (N, K) in SHAPES.items():
            x = torch.randn(M, K, device=dev).bfloat16()
            w = torch.randn(N, K, device=dev).bfloat16()
            y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            res[(M, name, "default")] = timeit(lambda: torch.matmul(x, w.t(), out=y))
    tun = torch.cuda.tunable
    tun.enable(True)
    tun.tuning_enable(True)
    tun.set_filename(os.path.join(tempfile.mkdtemp(), "tunableop_results.csv"))
    for M in args.m:
        for name, (N, K) in SHAPES.items():
            x = torch.randn(M, K, device=dev).bfloat16()
            w = torch.randn(N, K, device=dev).bfloat16()
            y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            torch.matmul(x, w.t(), out=y)  # tunes this shape
            tun.tuning_enable(False)
            res[(M, name, "tuned")] = timeit(lambda: torch.matmul(x, w.t(), out=y))
            tun.tuning_enable(True)
    for M in args.m:
        for name, (N, K) in SHAPES.items():
            d, t = res[(M, name, "default")], res[(M, name, "tuned")]
            print(json.dumps({"M": M, "shape": name, "default_us": round(d, 1), "tuned_us": round(t, 1),
                              "tflops_default": round(2 * M * N * K / d / 1e6, 1),
                              "tflops_tuned": round(2 * M * N * K / t / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
