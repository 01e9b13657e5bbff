#!/usr/bin/env python3
"""Grouped expert GEMM (csrc/kernels/moe.hip) on Mixtral 8x7B's expert shapes: the 128 x 128 tile kernel vs the
weight-streaming kernel, by routed rows per expert.  One JSON line per (shape, rows, kernel): median us over the
reps and the effective weight-read rate (every expert's weights once per launch).

  python bench/kernels/bench_grouped.py --rows 64,128,192,256
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", default="32,64,96,128,160,192,256")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--kernels", default="tile128,stream,stream_pre")
    ap.add_argument("--shapes", default="w13_swiglu,w2_f32")
    ap.add_argument("--skew", action="store_true", help="segments from 0.55x to 1.45x the mean")
    args = ap.parse_args()
    import torch

    from symmetry_amd import ops

    dev = torch.device("cuda", 0)
    E, d, F = 8, 4096, 14336
    g = torch.Generator(device=dev).manual_seed(0)
    w13 = (torch.randn(E, 2 * F, d, device=dev, generator=g) * 0.02).bfloat16()
    w2 = (torch.randn(E, d, F, device=dev, generator=g) * 0.02).bfloat16()
    from symmetry_amd.models.layout import preshuffle

    w13p = torch.stack([preshuffle(w13[e]) for e in range(E)])
    w2p = torch.stack([preshuffle(w2[e]) for e in range(E)])
    for rows in [int(r) for r in args.rows.split(",")]:
        # a mildly uneven split around the mean (+-15 %), as top-2 routing of a few prompts gives
        if args.skew:  # top-2 routing of a few prompts through a trained-like router: 0.55x .. 1.45x the mean
            counts = [max(1, int(rows * f)) for f in (0.55, 1.45, 0.85, 1.15, 0.7, 1.3, 1.0, 1.0)]
        else:
            counts = [max(1, int(rows * (1 + 0.15 * ((3 * e) % 5 - 2) / 2))) for e in range(E)]
        R = sum(counts)
        off = torch.zeros(E + 1, dtype=torch.int32)
        off[1:] = torch.cumsum(torch.tensor(counts), 0)
        offsets = off.to(dev)
        xs = torch.randn(R, d, device=dev, generator=g).bfloat16()
        act = torch.randn(R, F, device=dev, generator=g).bfloat16()
        y13 = torch.empty(R, F, device=dev, dtype=torch.bfloat16)
        y2 = torch.empty(R, d, device=dev, dtype=torch.float32)
        S13, S2 = ops.choose_splits(2 * F, d), ops.choose_splits(d, F)
        y13s = torch.empty(S13, R, 2 * F, device=dev)
        y2s = torch.empty(S2, R, d, device=dev)

        def skinny13():
            ops.grouped_skinny(xs, w13, offsets, 0, y13s)
            ops.swiglu(y13s, y13)

        skinny = {"w13_swiglu": skinny13, "w2_f32": lambda: ops.grouped_skinny(act, w2, offsets, 0, y2s)}
        for name, fn, wbytes in (("w13_swiglu", lambda pre=False: ops.grouped_gemm(xs, w13p if pre else w13, offsets, 0, y13,
                                                                                 2 + 4 * pre), w13.numel() * 2),
                                 ("w2_f32", lambda pre=False: ops.grouped_gemm(act, w2p if pre else w2, offsets, 0, y2,
                                                                             1 + 4 * pre), w2.numel() * 2)):
            if name not in args.shapes.split(","):
                continue
            for pol, kname in ((0, "tile128"), (2, "stream"), (2, "stream_pre"), (22, "stream_pre_rw2"),
                               (42, "stream_pre_rw4"), (1, "skinny"), (802, "stream_pre_mt8")):
                if kname not in args.kernels.split(","):
                    continue
                ops.grouped_stream_policy(pol)
                run = (lambda f=fn: f(True)) if kname.startswith("stream_pre") else (skinny[name] if kname == "skinny" else fn)
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
                us = ts[len(ts) // 2]
                print(json.dumps({"shape": name, "rows_per_expert": rows, "routed_rows": R, "skew": args.skew, "kernel": kname,
                                  "us": round(us, 1), "weight_TBps": round(wbytes / us / 1e6, 2)}), flush=True)
        ops.grouped_stream_policy(1)


if __name__ == "__main__":
    main()
