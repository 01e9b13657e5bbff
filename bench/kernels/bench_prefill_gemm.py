"""Prefill projection GEMMs (x[T,K] @ W[N,K]^T, bf16, hipBLASLt via torch.matmul) at the Llama-3-8B shapes:
default heuristic vs PyTorch TunableOp (every hipBLASLt/rocBLAS solution timed, best kept).

  python bench/kernels/bench_prefill_gemm.py --tokens 128 1280 --tune-file gpurun_out/tunableop.csv
"""
import argparse
import json

import torch

SHAPES = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336)}


def timeit(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(5):
            fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / (reps * 5)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, nargs="+", default=[128, 256, 512, 1280, 4096])
    ap.add_argument("--tune-file", default=None)
    ap.add_argument("--alt", action="store_true", help="also time the transposed orientation y^T = W x^T")
    args = ap.parse_args()
    dev = torch.device("cuda")
    ws = {k: torch.randn(n, kk, device=dev).bfloat16() * 0.02 for k, (n, kk) in SHAPES.items()}
    res = {}
    for T in args.tokens:
        for k, (N, K) in SHAPES.items():
            x = torch.randn(T, K, device=dev).bfloat16()
            y = torch.empty(T, N, device=dev, dtype=torch.bfloat16)
            res[(T, k)] = timeit(lambda: torch.matmul(x, ws[k].t(), out=y))
    if args.tune_file:
        torch.cuda.tunable.enable(True)
        torch.cuda.tunable.tuning_enable(True)
        torch.cuda.tunable.set_filename(args.tune_file)
        torch.cuda.tunable.set_max_tuning_duration(200)
    for T in args.tokens:
        for k, (N, K) in SHAPES.items():
            x = torch.randn(T, K, device=dev).bfloat16()
            y = torch.empty(T, N, device=dev, dtype=torch.bfloat16)
            d = res[(T, k)]
            row = {"T": T, "gemm": k, "N": N, "K": K, "default_us": round(d, 1),
                   "default_tflops": round(2 * T * N * K / d / 1e6, 1),
                   "default_TBps": round(2 * N * K / d / 1e6, 2)}
            if args.alt:
                yt = torch.empty(N, T, device=dev, dtype=torch.bfloat16)
                a = timeit(lambda: torch.matmul(ws[k], x.t(), out=yt))
                a2 = timeit(lambda: y.copy_(torch.matmul(ws[k], x.t(), out=yt).t()))
                row.update({"alt_us": round(a, 1), "alt_plus_transpose_us": round(a2, 1)})
            if args.tune_file:
                torch.matmul(x, ws[k].t(), out=y)  # tunes this shape
                torch.cuda.synchronize()
                t = timeit(lambda: torch.matmul(x, ws[k].t(), out=y))
                row.update({"tuned_us": round(t, 1), "tuned_tflops": round(2 * T * N * K / t / 1e6, 1)})
            print(json.dumps(row), flush=True)
    if args.tune_file:
        torch.cuda.tunable.write_file()


if __name__ == "__main__":
    main()
