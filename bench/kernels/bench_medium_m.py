"""Medium-M prefill projections (T = 65..256 tokens, Llama-3-8B shapes): hipBLASLt (torch.matmul, bf16 out)
vs the weight-streaming decode kernels run over 64-row chunks (dg_f32: fp32 out, plain [N, K] weights;
skinny_gemm: fp32 k-split slabs).  At these T the projections are weight-read bound, and hipBLASLt reaches
only 1.6-2.3 TB/s on three of the four (profiles/prefill_gemm_hipblaslt_r1.jsonl).

  python bench/kernels/bench_medium_m.py --tokens 96 128 192 256
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from symmetry_amd import ops  # noqa: E402

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
    ap.add_argument("--tokens", type=int, nargs="+", default=[96, 128, 192, 256])
    ap.add_argument("--chunk", type=int, default=64)
    args = ap.parse_args()
    dev = torch.device("cuda")
    ws = {k: (torch.randn(n, kk, device=dev) * 0.02).bfloat16() for k, (n, kk) in SHAPES.items()}
    for T in args.tokens:
        for k, (N, K) in SHAPES.items():
            x = (torch.randn(T, K, device=dev) * 0.5).bfloat16()
            y = torch.empty(T, N, device=dev, dtype=torch.bfloat16)
            yf = torch.empty(T, N, device=dev, dtype=torch.float32)
            ch = [(m0, min(T, m0 + args.chunk)) for m0 in range(0, T, args.chunk)]

            def dg():
                for m0, m1 in ch:
                    ops.dg_f32(x[m0:m1], ws[k], None, 0.0, yf[m0:m1])

            S = ops.choose_splits(N, K)
            slabs = [torch.empty(S, m1 - m0, N, device=dev, dtype=torch.float32) for m0, m1 in ch]

            def sk():
                for (m0, m1), s in zip(ch, slabs):
                    ops.skinny_gemm(x[m0:m1], ws[k], s)

            ref = x.float() @ ws[k].float().t()
            dg()
            err_dg = float((yf - ref).abs().max())
            sk()
            err_sk = float((torch.cat([s.sum(0) for s in slabs]) - ref).abs().max())
            d = timeit(lambda: torch.matmul(x, ws[k].t(), out=y))
            a = timeit(dg)
            b = timeit(sk)
            row = {"T": T, "gemm": k, "N": N, "K": K, "chunk": args.chunk, "hipblaslt_us": round(d, 1),
                   "dg_chunks_us": round(a, 1), "skinny_chunks_us": round(b, 1),
                   "hipblaslt_TBps": round(2 * N * K / d / 1e6, 2), "dg_err": err_dg, "skinny_err": err_sk}
            print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
