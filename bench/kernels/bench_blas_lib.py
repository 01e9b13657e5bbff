"""Prefill GEMMs (Llama-3-8B projections) on hipBLASLt vs rocBLAS (torch.backends.cuda.preferred_blas_library):
median us per GEMM over graph-replayed launches with a distinct weight per launch (cold weights, as in a
prefill step).

  python bench/kernels/bench_blas_lib.py --tokens 512 1280 4096
"""
import argparse
import json

import torch


def timed(fn, n, reps=5):
    fn(0)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for i in range(n):
            fn(i)
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3 / n)
    return sorted(ts)[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, nargs="+", default=[512, 1280, 4096])
    ap.add_argument("--copies", type=int, default=8)
    args = ap.parse_args()
    shapes = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336)}
    for T in args.tokens:
        for name, (N, K) in shapes.items():
            x = torch.randn(T, K, device="cuda").bfloat16()
            ws = [(torch.randn(N, K, device="cuda") * 0.02).bfloat16() for _ in range(args.copies)]
            y = torch.empty(T, N, device="cuda", dtype=torch.bfloat16)
            res = {"T": T, "gemm": name}
            for lib in ("cublaslt", "cublas"):
                torch.backends.cuda.preferred_blas_library(lib)
                us = timed(lambda i: torch.matmul(x, ws[i % len(ws)].t(), out=y), 2 * args.copies)
                res[{"cublaslt": "hipblaslt_us", "cublas": "rocblas_us"}[lib]] = round(us, 2)
                res[{"cublaslt": "hipblaslt_tflops", "cublas": "rocblas_tflops"}[lib]] = round(2 * T * N * K / us / 1e6, 1)
            torch.backends.cuda.preferred_blas_library("cublaslt")
            print(json.dumps(res), flush=True)
            del ws


if __name__ == "__main__":
    main()
