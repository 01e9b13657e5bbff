"""Microbenchmark: fused decode GEMM (csrc/kernels/decode_gemm.hip) decomposition variants.

Each measurement is a hipGraph of ``chain`` dependent launches over rotated weight copies (>= 1 GiB,
so every call streams from HBM past the 256 MiB Infinity Cache), replayed ``iters`` times; the
reported time per launch therefore includes the kernel boundary, as in a captured decode step.
Variants are interleaved in one process.  Output: one JSON line per (shape, M, variant).
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch

from symmetry_amd import ops
from symmetry_amd.models.layout import gu_perm, qkv_perm
from symmetry_amd.ops import _native

# name: (epilogue, N, K) -- Llama-3-8B at TP=1, and the TP=8 shards
SHAPES = {
    "qkv": ("qkv", 6144, 4096), "o": ("resid", 4096, 4096), "gate_up": ("swiglu", 28672, 4096),
    "down": ("resid", 4096, 14336), "lm_head": ("argmax", 128256, 4096),
    "qkv_tp8": ("qkv", 768, 4096), "o_tp8": ("f32", 4096, 512), "gate_up_tp8": ("swiglu", 3584, 4096),
    "down_tp8": ("f32", 4096, 1792), "lm_head_tp8": ("argmax", 16032, 4096),
    # Llama-3-70B at TP=1 (config 4 on one GPU)
    "qkv_70b": ("qkv", 10240, 8192), "o_70b": ("resid", 8192, 8192), "gate_up_70b": ("swiglu", 57344, 8192),
    "down_70b": ("resid", 8192, 28672),
    # Llama-3-70B TP=8 shards (config 4: one rank's projections)
    "qkv_70b_tp8": ("qkv", 1280, 8192), "o_70b_tp8": ("f32", 8192, 1024), "gate_up_70b_tp8": ("swiglu", 7168, 8192),
    "down_70b_tp8": ("f32", 8192, 3584),
    # plain fp32-output twins: the difference to the fused shapes is the epilogue's cost
    "qkv_f32": ("f32", 6144, 4096), "o_f32": ("f32", 4096, 4096), "gate_up_f32": ("f32", 28672, 4096),
}


def make_call(epi, x, W, M, N, K, dev, sh=False):
    ss = torch.rand(M, K // 16, device=dev) + 0.5
    if epi == "f32":
        y = torch.empty(M, N, device=dev)
        return lambda w: ops.dg_f32(x, w, ss, 1e-5, y, wshuf=sh)
    if epi == "resid":
        resid = torch.zeros(M, N, device=dev)
        wn = torch.ones(N, device=dev, dtype=torch.bfloat16)
        xw = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        sso = torch.empty(M, N // 16, device=dev)
        return lambda w: ops.dg_resid(x, w, resid, wn, xw, sso, wshuf=sh)
    if epi == "swiglu":
        act = torch.empty(M, N // 2, device=dev, dtype=torch.bfloat16)
        return lambda w: ops.dg_swiglu(x, w, ss, 1e-5, act, wshuf=sh)
    if epi == "qkv":
        g = 8 if N in (10240, 1280) else 4  # Llama-3-70B (and its TP=8 shard): 64 q / 8 kv heads; 8B: 32 / 8
        hkv = N // 128 // (g + 2)
        hq = g * hkv
        cs = torch.rand(4096, 128, device=dev)
        pos = torch.arange(M, device=dev, dtype=torch.int32)
        slots = torch.arange(M, device=dev, dtype=torch.int32)
        q = torch.empty(M, hq, 128, device=dev, dtype=torch.bfloat16)
        kc = torch.zeros(4, hkv, 64, 128, device=dev, dtype=torch.bfloat16)
        vc = torch.zeros(4, hkv, 128, 64, device=dev, dtype=torch.bfloat16)
        return lambda w: ops.dg_qkv(x, w, ss, 1e-5, pos, slots, cs, q, kc, vc, hq, hkv, wshuf=sh)
    temps = torch.zeros(M, device=dev)
    seeds = torch.zeros(M, device=dev, dtype=torch.int64)
    step = torch.zeros(1, device=dev, dtype=torch.int64)
    tk = torch.empty(M * (N // 16), device=dev, dtype=torch.int64)
    keys = torch.empty(M, device=dev, dtype=torch.int64)
    ids = torch.empty(M, device=dev, dtype=torch.int32)
    return lambda w: ops.dg_argmax(x, w, ss, 1e-5, temps, seeds, step, tk, keys, ids, 0, None, wshuf=sh)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", nargs="+", default=["qkv", "o", "gate_up", "down", "lm_head"])
    ap.add_argument("--m", type=int, nargs="+", default=[1, 10, 32, 64])
    ap.add_argument("--variants", type=int, nargs="+", default=[0, 1, 2, 3, 4])
    ap.add_argument("--chain", type=int, default=16)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--warm", action="store_true", help="one weight copy: measures Infinity-Cache-resident weights")
    ap.add_argument("--layouts", nargs="+", default=["row"], choices=["row", "shuf"],
                    help="weight stream layout(s): row-major and/or MFMA-preshuffled")
    args = ap.parse_args()
    dev = torch.device("cuda")
    lib = _native.ops()
    for name in args.shapes:
        epi, N, K = SHAPES[name]
        nbytes = N * K * 2
        copies = 1 if args.warm else max(2, (1 << 30) // nbytes + 1)
        ws = [(torch.randn(N, K, device=dev) * 0.02).bfloat16() for _ in range(copies)]
        for M in args.m:
            x = torch.randn(M, K, device=dev).bfloat16()
            graphs = {}
            for lay in args.layouts:
                call = make_call(epi, x, ws[0], M, N, K, dev, sh=lay == "shuf")
                for v in args.variants:
                    lib.decode_gemm_variant(v)
                    for c in range(2):
                        call(ws[c % copies])
                    torch.cuda.synchronize()
                    g = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(g):
                        for c in range(args.chain):
                            call(ws[c % copies])
                    graphs[(lay, v)] = g
            lib.decode_gemm_variant(-1)
            times = {k: [] for k in graphs}
            for it in range(args.iters):
                for v, g in graphs.items():
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    g.replay()
                    e1.record()
                    torch.cuda.synchronize()
                    if it:
                        times[v].append(e0.elapsed_time(e1) * 1e3 / args.chain)
            for (lay, v), t in times.items():
                t.sort()
                us = t[len(t) // 2]
                print(json.dumps({"shape": name, "N": N, "K": K, "M": M, "layout": lay, "variant": v,
                                  "us": round(us, 2), "TBps": round(nbytes / us / 1e6, 3)}), flush=True)
            del graphs
        del ws
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
