#!/usr/bin/env python3
"""The prefill step's bandwidth kernels outside the GEMMs (Llama-3-8B shapes): add + RMSNorm of the residual stream
(``ops.add_rms_norm``: bf16 delta + fp32 residual in, fp32 residual + bf16 normalised rows out) and RoPE + paged
K/V write (``ops.rope_cache``: bf16 qkv rows in, q rows + cache blocks out), at prefill row counts.  One JSON line
per (kernel, rows): median us of a hipGraph chain and the achieved HBM rate of the bytes each launch must move.

  python bench/kernels/bench_prefill_elementwise.py --rows 384 768 1280
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def timed(fn, chain=20, iters=10):
    import torch

    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(chain):
            fn()
    ts = []
    for _ in range(iters):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        g.replay()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3 / chain)
    ts.sort()
    return ts[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, nargs="+", default=[384, 768, 1280])
    ap.add_argument("--kernels", nargs="+", default=["add_rms_norm", "rope_cache"])
    args = ap.parse_args()
    import torch

    from symmetry_amd import ops
    from symmetry_amd.ops.reference import rope_table

    dev = torch.device("cuda")
    d, Hq, Hkv, D, BS = 4096, 32, 8, 128, 64
    cs = rope_table(8192, D, 500000.0, None, device=dev)
    for T in args.rows:
        if "add_rms_norm" in args.kernels:
            delta = torch.randn(T, d, device=dev).bfloat16()
            resid = torch.randn(T, d, device=dev)
            w = torch.rand(d, device=dev).bfloat16()
            out = torch.empty(T, d, device=dev, dtype=torch.bfloat16)
            us = timed(lambda: ops.add_rms_norm(delta, resid, w, 1e-5, out))
            nbytes = T * d * (2 + 4 + 4 + 2)
            print(json.dumps({"kernel": "add_rms_norm", "rows": T, "us": round(us, 2),
                              "TBps": round(nbytes / us / 1e6, 2)}), flush=True)
        if "rope_cache" in args.kernels:
            N = (Hq + 2 * Hkv) * D
            qkv = torch.randn(T, N, device=dev).bfloat16()
            nseq = max(1, T // 128)
            pos = torch.cat([torch.arange(T // nseq) for _ in range(nseq)] +
                            [torch.arange(T - nseq * (T // nseq))]).to(torch.int32).to(dev)
            nblk = (T + BS - 1) // BS + nseq + 1
            slots = torch.arange(T, dtype=torch.int32, device=dev)  # consecutive, block-aligned sequences
            q = torch.empty(T, Hq * D, device=dev, dtype=torch.bfloat16)
            kc = torch.zeros(nblk, Hkv, BS, D, device=dev, dtype=torch.bfloat16)
            vc = torch.zeros(nblk, Hkv, D, BS, device=dev, dtype=torch.bfloat16)
            us = timed(lambda: ops.rope_cache(qkv, pos, slots, cs, q, kc, vc, Hq, Hkv, perm=True))
            nbytes = T * N * 2 * 2
            print(json.dumps({"kernel": "rope_cache", "rows": T, "us": round(us, 2),
                              "TBps": round(nbytes / us / 1e6, 2)}), flush=True)


if __name__ == "__main__":
    main()
