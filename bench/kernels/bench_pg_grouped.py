#!/usr/bin/env python3
"""Grouped expert GEMMs of Mixtral 8x7B prefill: the prefill GEMM kernel in grouped mode (csrc/kernels/pgemm.hip,
``ops.pg_grouped``) per tile config against the current MoE path (``ops.grouped_gemm``: the 128 x 128 tile kernel,
or the weight-streaming kernel on the preshuffled copies where moe.py's PRE_ROWS thresholds pick it).  Segments are
uneven (0.4x .. 2.0x the mean, as top-2 routing of a few prompts gives).  One JSON line per (shape, rows, kernel):
median us over the reps, effective PFLOP/s on the routed rows, and the max error against the current path.

  python bench/kernels/bench_pg_grouped.py --rows 32,64,128,256
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

SKEW = (0.4, 2.0, 0.8, 1.2, 0.6, 1.4, 1.0, 0.6)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", default="32,64,128,256,512")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--shapes", default="w13_swiglu,w2_f32")
    ap.add_argument("--cfgs", default="auto,1,4,5,9,10")
    ap.add_argument("--current", default="policy", choices=["policy", "stream_pre", "tile128"],
                    help="the grouped_gemm kernel to compare with (policy: moe.py's PRE_ROWS thresholds)")
    args = ap.parse_args()
    import torch

    from symmetry_amd import ops
    from symmetry_amd.models import moe
    from symmetry_amd.models.layout import preshuffle

    dev = torch.device("cuda", 0)
    E, d, F = 8, 4096, 14336
    g = torch.Generator(device=dev).manual_seed(0)
    w13 = (torch.randn(E, 2 * F, d, device=dev, generator=g) * 0.02).bfloat16()
    w2 = (torch.randn(E, d, F, device=dev, generator=g) * 0.02).bfloat16()
    w13p = torch.stack([preshuffle(w13[e]) for e in range(E)])
    w2p = torch.stack([preshuffle(w2[e]) for e in range(E)])

    def timed(run):
        run()
        torch.cuda.synchronize()
        ts = []
        for _ in range(args.reps):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            run()
            b.record()
            b.synchronize()
            ts.append(a.elapsed_time(b) * 1e3)
        ts.sort()
        return ts[len(ts) // 2]

    for rows in [int(r) for r in args.rows.split(",")]:
        counts = [max(1, int(rows * f)) for f in SKEW]
        R = sum(counts)
        off = torch.zeros(E + 1, dtype=torch.int32)
        off[1:] = torch.cumsum(torch.tensor(counts), 0)
        offsets = off.to(dev)
        xs = torch.randn(R, d, device=dev, generator=g).bfloat16()
        act = (torch.randn(R, F, device=dev, generator=g) * 0.5).bfloat16()
        for name in args.shapes.split(","):
            if name == "w13_swiglu":
                N, K, x, wp = 2 * F, d, xs, w13p
                pre = R <= moe.PRE_ROWS_W13 * E if args.current == "policy" else args.current == "stream_pre"
                ref = torch.empty(R, F, device=dev, dtype=torch.bfloat16)
                cur = lambda: ops.grouped_gemm(xs, w13p if pre else w13, offsets, 0, ref, 2 + 4 * pre)  # noqa: E731
            else:
                N, K, x, wp = d, F, act, w2p
                pre = R <= moe.PRE_ROWS * E if args.current == "policy" else args.current == "stream_pre"
                ref = torch.empty(R, d, device=dev, dtype=torch.float32)
                cur = lambda: ops.grouped_gemm(act, w2p if pre else w2, offsets, 0, ref, 1 + 4 * pre)  # noqa: E731
            flops = 2.0 * R * N * K
            us = timed(cur)
            base = {"shape": name, "rows_per_expert": rows, "routed_rows": R}
            print(json.dumps({**base, "kernel": "stream_pre" if pre else "tile128", "us": round(us, 1),
                              "PF": round(flops / us / 1e9, 3)}), flush=True)
            refv = ref.float().clone()
            for c in args.cfgs.split(","):
                if c == "auto":
                    ch = ops.choose_pg_grouped(R, N, K, E, slabs=name == "w2_f32", even_wn=name == "w13_swiglu")
                    if ch is None:
                        continue
                    cfg, S = ch
                    plans = [(cfg, S, "auto")]
                else:
                    cfg = int(c)
                    bm, bn = ops.PG_CFG_SHAPES[cfg]
                    if N % bn:
                        continue
                    plans = [(cfg, S, "") for S in ((1, 2) if name == "w2_f32" else (1,)) if K % (64 * S) == 0]
                for cfg, S, tag in plans:
                    if name == "w13_swiglu":
                        y = torch.empty(R, F, device=dev, dtype=torch.bfloat16)
                        run = lambda y=y, cfg=cfg: ops.pg_grouped(xs, wp, offsets, 0, y, ops.PG_EPI_SWIGLU_SPLIT, cfg)  # noqa
                    else:
                        y = torch.empty(S, R, d, device=dev, dtype=torch.float32)
                        run = lambda y=y, cfg=cfg, S=S: ops.pg_grouped(act, wp, offsets, 0, y, ops.PG_EPI_F32, cfg, S)  # noqa
                    us = timed(run)
                    out = y.float() if y.dim() == 2 else y.sum(0)
                    err = ((out - refv).abs().max() / refv.abs().max().clamp_min(1e-6)).item()
                    print(json.dumps({**base, "kernel": f"pg_grouped{'_' + tag if tag else ''}", "cfg": cfg,
                                      "tile": ops.PG_CFG_SHAPES[cfg], "S": S, "us": round(us, 1),
                                      "PF": round(flops / us / 1e9, 3), "max_rel_err": round(err, 5)}), flush=True)


if __name__ == "__main__":
    main()
