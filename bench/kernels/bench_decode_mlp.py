#!/usr/bin/env python3
"""Persistent decode MLP (one launch: O -> gate_up/SwiGLU -> down) vs the three fused decode GEMMs.

Both paths are captured in a hipGraph of ``--layers`` layer blocks (distinct weights per layer, so the
weights stream from HBM as in a real decode step) and timed over replays.  Prints one JSON line per M.

  python bench/kernels/bench_decode_mlp.py --ms 1 4 10 16
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from symmetry_amd import ops  # noqa: E402
from symmetry_amd.models.layout import preshuffle  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ms", type=int, nargs="+", default=[1, 4, 10, 16])
    ap.add_argument("--layers", type=int, default=8)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--d", type=int, default=4096)
    ap.add_argument("--F", type=int, default=14336)
    ap.add_argument("--row-major", action="store_true")
    ap.add_argument("--cfgs", type=int, nargs="+", default=[-1],
                    help="persistent configurations (launch_decode_mlp; -1 = default)")
    ap.add_argument("--xcfgs", type=int, nargs="+", default=[],
                    help="x-resident persistent kernel A/B knob bits (decode_gemm.hip g_mlp_xcfg)")
    ap.add_argument("--stamps", action="store_true",
                    help="x-resident kernel: per-phase s_memrealtime stamps of the last layer (us from launch start)")
    args = ap.parse_args()
    dev = torch.device("cuda")
    d, F, L = args.d, args.F, args.layers
    shuf = not args.row_major
    g = torch.Generator(device=dev).manual_seed(0)

    def w(n, k):
        t = (torch.randn(n, k, device=dev, generator=g) / k ** 0.5).bfloat16()
        return preshuffle(t) if shuf else t

    layers = [(w(d, d), w(2 * F, d), w(d, F)) for _ in range(L)]
    ln = (torch.rand(d, device=dev, generator=g) + 0.5).bfloat16()
    byts = L * 2 * (d * d + 2 * F * d + d * F)
    for M in args.ms:
        attn = torch.randn(M, d, device=dev, generator=g).bfloat16()
        resid = torch.randn(M, d, device=dev, generator=g)
        xw = torch.empty(M, d, device=dev, dtype=torch.bfloat16)
        ss = torch.empty(M, d // 16, device=dev)
        act = torch.empty(M, F, device=dev, dtype=torch.bfloat16)
        ctl = torch.zeros(ops.DECODE_MLP_CTL, device=dev, dtype=torch.int32)

        def seq():
            for wo, wgu, wd in layers:
                ops.dg_resid(attn, wo, resid, ln, xw, ss, wshuf=shuf)
                ops.dg_swiglu(xw, wgu, ss, 1e-5, act, wshuf=shuf)
                ops.dg_resid(act, wd, resid, ln, xw, ss, wshuf=shuf)

        def per():
            for wo, wgu, wd in layers:
                ops.decode_mlp(attn, wo, wgu, wd, resid, ln, ln, xw, ss, act, ctl, 1e-5, wshuf=shuf)

        res = {"M": M, "layers": L, "layout": "preshuffled" if shuf else "row-major"}
        lib = ops._native.ops()
        runs = [("three_launches", seq, None)] + [(f"persistent{'' if c < 0 else c}", per, c) for c in args.cfgs]
        runs += [(f"xres_x{x}", per, -1 - 1000 * (x + 1)) for x in args.xcfgs]
        for name, fn, c in runs:
            if c is not None and c <= -1000:
                lib.decode_gemm_variant(-1)
                lib.decode_gemm_variant(2000 + (-c // 1000 - 1))
            elif c is not None:
                lib.decode_gemm_variant(2000)
                lib.decode_gemm_variant(1000 + c if c >= 0 else -1)
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
            us = e0.elapsed_time(e1) * 1e3 / args.iters / L
            res[f"{name}_us_per_layer"] = round(us, 2)
            res[f"{name}_TBps"] = round(byts / L / (us * 1e-6) / 1e12, 2)
            res[f"{name}_ctl_ok"] = not bool(ctl.any())
        lib.decode_gemm_variant(-1)
        lib.decode_gemm_variant(2000)
        if args.stamps:
            st = torch.zeros(1024, 8, dtype=torch.int64, device=dev)
            lib.decode_mlp_stamps(st)
            for _ in range(2):
                per()
            torch.cuda.synchronize()
            lib.decode_mlp_stamps(None)
            st = st.cpu()
            st = st[st[:, 0] > 0]
            t0 = int(st[:, 0].min())
            names = ["start", "o_done", "gu_wait_done", "gu_done", "d_wait_done", "end"]
            q = torch.tensor([0.0, 0.1, 0.5, 0.9, 1.0])
            res["stamps_us_p0_10_50_90_100"] = {
                n: [round(v, 2) for v in (torch.quantile((st[:, k] - t0).double(), q.double()) * 0.01).tolist()]
                for k, n in enumerate(names)}
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
