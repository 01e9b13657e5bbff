"""Decode attention kernel alone (csrc/kernels/attention.hip, attn_decode): S sequences x ctx tokens,
Llama-3-8B heads (32 q / 8 kv, D = 128), paged cache of 64-token blocks; a hipGraph chain over `layers`
different caches (as in a decode step), so K/V stream from HBM.  Also reports the floor of a graph chain
of trivial launches (the per-kernel boundary).

  python bench/kernels/bench_attn_decode.py --seqs 10 --ctx 64 160 512 2048 8192
"""
import argparse
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from symmetry_amd import ops  # noqa: E402


def timed(fn, chain, reps=20):
    fn(0)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for i in range(chain):
            fn(i)
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / (reps * chain)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seqs", type=int, default=10)
    ap.add_argument("--ctx", type=int, nargs="+", default=[64, 160, 512, 2048, 8192])
    ap.add_argument("--layers", type=int, default=32)
    ap.add_argument("--span", type=int, default=0, help="block-table width in tokens (the graph's context "
                    "bucket; 0: just the context)")
    ap.add_argument("--wave", type=int, nargs="+", default=[-1],
                    help="attn_wave min-units settings to compare (-1: leave the default; 0: never; 1: always)")
    ap.add_argument("--heads", type=int, nargs=2, default=[32, 8], metavar=("HQ", "HKV"),
                    help="query / kv heads (one TP rank's shard: 4 1 for Llama-3-8B at TP=8, 8 1 for 70B)")
    args = ap.parse_args()
    dev = torch.device("cuda")
    ops._native.ops()  # load the extension (registers torch.ops.symmetry_amd)
    (Hq, Hkv), D, BS = args.heads, 128, 64
    S, L = args.seqs, args.layers
    tiny = torch.zeros(64, device=dev)
    print(json.dumps({"kernel": "trivial launch (graph chain floor)", "us": round(timed(lambda i: tiny.add_(1.0), 64), 2)}))
    for ctx in args.ctx:
        nb = (ctx + BS - 1) // BS
        NB = S * nb + 1
        kc = [torch.randn(NB, Hkv, BS, D, device=dev).bfloat16() for _ in range(L)]
        vc = [torch.randn(NB, Hkv, D, BS, device=dev).bfloat16() for _ in range(L)]
        bt = (torch.arange(S * nb, dtype=torch.int32, device=dev) + 1).view(S, nb)
        width = max(nb, args.span // BS)
        if width > nb:
            bt = torch.cat([bt, torch.zeros(S, width - nb, dtype=torch.int32, device=dev)], 1).contiguous()
            nb = width
        ctxs = torch.full((S,), ctx, dtype=torch.int32, device=dev)
        q = torch.randn(S, Hq, D, device=dev).bfloat16()
        out = torch.empty_like(q)
        parts = (nb * BS + ops.ATTN_DECODE_PART - 1) // ops.ATTN_DECODE_PART
        tmp_o = torch.empty(S, Hq, parts, D, device=dev)
        tmp_ml = torch.empty(S, Hq, parts, 2, device=dev)
        cnt = torch.zeros(S * Hkv, dtype=torch.int32, device=dev)
        for wv in args.wave:
            if wv >= 0:
                torch.ops.symmetry_amd.attn_wave(wv, 0)
            us = timed(lambda i: ops.attn_decode(q, kc[i % L], vc[i % L], bt, ctxs, out, tmp_o, tmp_ml, cnt,
                                                 1 / math.sqrt(D)), L)
            kv_bytes = 2 * S * ctx * Hkv * D * 2
            print(json.dumps({"kernel": "attn_decode", "heads": [Hq, Hkv], "seqs": S, "ctx": ctx, "span": nb * BS, "wave": wv,
                              "us": round(us, 2), "TBps": round(kv_bytes / us / 1e6, 3)}), flush=True)
        torch.ops.symmetry_amd.attn_wave(1024, 513)
        del kc, vc


if __name__ == "__main__":
    main()
