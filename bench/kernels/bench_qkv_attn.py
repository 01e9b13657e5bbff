#!/usr/bin/env python3
"""Fused QKV + decode attention launch (ops.qkv_attn) vs dg_qkv + attn_decode, Llama-3-8B shapes.

Both forms are captured in a hipGraph of ``--layers`` layers (distinct QKV weights per layer, so they stream
from HBM) and timed over replays; ``--stamps`` adds the per-workgroup s_memrealtime stamps of one fused launch
(us from the first workgroup's start; QKV role: start / tiles published / end, attention role: start / wait
done / end).  One JSON line per (M, context).

  python bench/kernels/bench_qkv_attn.py --m 10 --ctx 180 350 --stamps
"""
import argparse
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from symmetry_amd import ops  # noqa: E402
from symmetry_amd.models.layout import preshuffle, qkv_perm  # noqa: E402
from symmetry_amd.ops import reference as ref  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, nargs="+", default=[10])
    ap.add_argument("--ctx", type=int, nargs="+", default=[180, 350])
    ap.add_argument("--span", type=int, default=512, help="block-table span (the graph's context bucket)")
    ap.add_argument("--layers", type=int, default=16)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--stamps", action="store_true")
    args = ap.parse_args()
    dev = torch.device("cuda")
    Hq, Hkv, D, d, BS = 32, 8, 128, 4096, 64
    N = (Hq + 2 * Hkv) * D
    g = torch.Generator(device=dev).manual_seed(0)
    Ws = [preshuffle((torch.randn(N, d, device=dev, generator=g) / d ** 0.5).bfloat16()[qkv_perm(Hq, Hkv, D).to(dev)])
          for _ in range(args.layers)]
    cs = ref.rope_table(8192, D, 500000.0, device=dev)
    nat = ops._native.ops()
    for M in args.m:
        for c in args.ctx:
            max_blocks = args.span // BS
            NB = M * max_blocks + 2
            kc = torch.randn(NB, Hkv, BS, D, device=dev, generator=g).bfloat16()
            vc = torch.randn(NB, Hkv, D, BS, device=dev, generator=g).bfloat16()
            bt = torch.arange(M * max_blocks, dtype=torch.int32, device=dev).view(M, max_blocks)
            ctx = torch.full((M,), c, dtype=torch.int32, device=dev)
            pos = ctx - 1
            slots = (bt[:, (c - 1) // BS] * BS + (c - 1) % BS).int().contiguous()
            xw = torch.randn(M, d, device=dev, generator=g).bfloat16()
            ss = torch.rand(M, d // 16, device=dev, generator=g) + 1
            q = torch.empty(M, Hq, D, device=dev, dtype=torch.bfloat16)
            attn = torch.empty(M, Hq, D, device=dev, dtype=torch.bfloat16)
            mp = (args.span + 255) // 256
            tmp_o = torch.empty(M, Hq, mp, D, device=dev)
            tmp_ml = torch.empty(M, Hq, mp, 2, device=dev)
            cnt = torch.zeros(M * Hkv, dtype=torch.int32, device=dev)
            ctl = torch.zeros(ops.QKV_ATTN_CTL, dtype=torch.int32, device=dev)
            scale = 1 / math.sqrt(D)

            def two():
                for W in Ws:
                    ops.dg_qkv(xw, W, ss, 1e-5, pos, slots, cs, q, kc, vc, Hq, Hkv, wshuf=True)
                    ops.attn_decode(q, kc, vc, bt, ctx, attn, tmp_o, tmp_ml, cnt, scale)

            def one():
                for W in Ws:
                    assert ops.qkv_attn(xw, W, ss, 1e-5, pos, slots, cs, q, kc, vc, Hq, Hkv, True, bt, ctx, attn,
                                        tmp_o, tmp_ml, cnt, scale, ctl)

            res = {"M": M, "ctx": c, "span": args.span, "layers": args.layers}
            for name, fn in (("two_launches", two), ("fused", one)):
                s = torch.cuda.Stream()
                with torch.cuda.stream(s):
                    fn()
                    graph = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(graph, stream=s):
                        fn()
                torch.cuda.synchronize()
                for _ in range(3):
                    graph.replay()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(args.iters):
                    graph.replay()
                e1.record()
                torch.cuda.synchronize()
                res[f"{name}_us_per_layer"] = round(e0.elapsed_time(e1) * 1e3 / args.iters / args.layers, 2)
            res["ctl_ok"] = not bool(ctl.any())
            if args.stamps:
                st = torch.zeros(4096, 4, dtype=torch.int64, device=dev)
                nat.qkv_attn_stamps(st)
                one()
                torch.cuda.synchronize()
                nat.qkv_attn_stamps(None)
                st = st.cpu()
                st = st[st[:, 0] > 0]
                t0 = int(st[:, 0].min())
                qt = torch.tensor([0.0, 0.1, 0.5, 0.9, 1.0], dtype=torch.float64)
                for role, nm in ((0, "qkv"), (1, "attn")):
                    r = st[st[:, 3] == role]
                    res[f"{nm}_wgs"] = int(r.shape[0])
                    for k, col in (("start", 0), ("mid", 1), ("end", 2)):
                        v = (r[:, col] - t0).double()
                        res[f"{nm}_{k}_us"] = [round(x, 2) for x in (torch.quantile(v, qt) * 0.01).tolist()]
            print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
