"""Decode MoE routing launches alone (csrc/kernels/moe.hip): the one-launch moe_decode_route vs the general
path's rms_norm + router GEMM + moe_route_permute (three kernels), and moe_combine_prep vs moe_combine +
add_prep; hipGraph chains over 32 layers' router weights (Mixtral-8x7B shapes: d 4096, 8 experts, top-2).

  python bench/kernels/bench_moe_decode.py --t 1 4 8
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from symmetry_amd import ops  # noqa: E402


def timed(fn, chain=32, reps=20):
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
    ap.add_argument("--t", type=int, nargs="+", default=[1, 4, 8])
    args = ap.parse_args()
    dev = torch.device("cuda")
    d, E, k, L = 4096, 8, 2, 32
    routers = [(torch.randn(16, d, device=dev) * 0.05).bfloat16() for _ in range(L)]
    lnw = (torch.rand(d, device=dev) + 0.5).bfloat16()
    for T in args.t:
        R = T * k
        resid = torch.randn(T, d, device=dev)
        ids = torch.empty(R, dtype=torch.int32, device=dev)
        w = torch.empty(R, device=dev)
        dst = torch.empty(R, dtype=torch.int32, device=dev)
        counts = torch.empty(E, dtype=torch.int32, device=dev)
        offsets = torch.empty(E + 1, dtype=torch.int32, device=dev)
        cursor = torch.zeros(E, dtype=torch.int32, device=dev)
        xs = torch.empty(R, d, dtype=torch.bfloat16, device=dev)
        xn = torch.empty(T, d, dtype=torch.bfloat16, device=dev)
        S = ops.choose_splits(16, d)
        lg = torch.empty(S, T, 16, device=dev)

        def general(i):
            ops.rms_norm(resid, lnw, 1e-5, xn)
            ops.skinny_gemm(xn, routers[i], lg)
            ops.moe_route_permute(lg, xn, k, E, ids, w, counts, offsets, cursor, xs, dst)

        def fused(i):
            ops.moe_decode_route(resid, lnw, 1e-5, routers[i][:E], k, ids, w, counts, offsets, cursor, xs, dst)

        y = torch.randn(2, R, d, device=dev)
        out = torch.empty(T, d, device=dev)
        r2 = torch.randn(T, d, device=dev)
        xw = torch.empty(T, d, dtype=torch.bfloat16, device=dev)
        ss1, ssp = torch.empty(T, 1, device=dev), torch.empty(T, 8, device=dev)

        def comb_general(i):
            ops.moe_combine(y, dst, ids, 0, E, w, k, out)
            ops.add_prep(out, r2, lnw, xw, ss1)

        def comb_fused(i):
            ops.moe_combine_prep(y, dst, ids, E, w, k, r2, lnw, xw, ssp)

        print(json.dumps({"T": T, "route_general_us": round(timed(general), 2), "route_fused_us": round(timed(fused), 2),
                          "combine_prep_general_us": round(timed(comb_general), 2),
                          "combine_prep_fused_us": round(timed(comb_fused), 2)}), flush=True)


if __name__ == "__main__":
    main()
