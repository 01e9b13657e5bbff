"""Prefill projection GEMM (csrc/kernels/pgemm.hip) vs hipBLASLt (torch.matmul) at the Llama-3-8B shapes.

Every tile config x split that tiles the shape is timed (hipGraph of 5 launches, replayed; random operands),
checked once against an fp32 product, and printed as one JSON line per (tokens, projection):

  python bench/kernels/bench_pgemm.py --tokens 384 768 1280 --out gpurun_out/pgemm.jsonl
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from symmetry_amd.models.layout import preshuffle  # noqa: E402
from symmetry_amd.ops import _native  # noqa: E402

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
    ap.add_argument("--tokens", type=int, nargs="+", default=[384, 512, 640, 768, 1280])
    ap.add_argument("--shapes", nargs="+", default=list(SHAPES))
    ap.add_argument("--cfgs", type=int, nargs="+", default=list(range(16)))
    ap.add_argument("--splits", type=int, nargs="+", default=[1, 2, 4])
    ap.add_argument("--max-waves", type=float, default=2.2, help="skip grids above this many waves of 256 CUs")
    ap.add_argument("--out", default=None)
    ap.add_argument("--profile", type=int, nargs=2, default=None, metavar=("CFG", "S"),
                    help="rocprof mode: run only this config and the library GEMM, 10 plain launches each per shape")
    args = ap.parse_args()
    ops = _native.ops()
    dev = torch.device("cuda")
    torch.manual_seed(0)
    cfgs = [(c, tuple(ops.pgemm_shape(c))) for c in args.cfgs]
    cfgs = [(c, s) for c, s in cfgs if s]
    out = open(args.out, "a") if args.out else None
    if args.profile:
        c, S = args.profile
        bm, bn = cfgs[[cc for cc, _ in cfgs].index(c)][1]
        for name in args.shapes:
            N, K = SHAPES[name]
            w = preshuffle((torch.rand(N, K, device=dev) * 2 - 1).mul_(0.05).bfloat16())
            for T in args.tokens:
                x = (torch.rand(T, K, device=dev) * 2 - 1).bfloat16()
                y = torch.empty(T, N, device=dev, dtype=torch.bfloat16)
                tiles = -(-T // bm) * (N // bn)
                slab = torch.empty(S, T, N, device=dev) if S > 1 else None
                cnt = torch.zeros(tiles, dtype=torch.int32, device=dev) if S > 1 else None
                for _ in range(10):
                    ops.pgemm(x, w, y, c, S, slab, cnt)
                for _ in range(10):
                    torch.matmul(x, w.t(), out=y)
                torch.cuda.synchronize()
                print(json.dumps({"profiled": name, "T": T, "cfg": c, "S": S}), flush=True)
        return
    for name in args.shapes:
        N, K = SHAPES[name]
        w = (torch.rand(N, K, device=dev) * 2 - 1).mul_(0.05).bfloat16()
        wsh = preshuffle(w)
        for T in args.tokens:
            x = (torch.rand(T, K, device=dev) * 2 - 1).bfloat16()
            ref = x.float() @ w.float().t()
            y = torch.empty(T, N, device=dev, dtype=torch.bfloat16)
            lib = timeit(lambda: torch.matmul(x, w.t(), out=y))
            arms = []
            for c, (bm, bn) in cfgs:
                if N % bn:
                    continue
                tiles = -(-T // bm) * (N // bn)
                for S in args.splits:
                    if K % (64 * S) or tiles * S > args.max_waves * 256:
                        continue
                    slab = torch.empty(S, T, N, device=dev) if S > 1 else None
                    cnt = torch.zeros(tiles, dtype=torch.int32, device=dev) if S > 1 else None
                    yf = torch.empty(T, N, device=dev)
                    ops.pgemm(x, wsh, yf, c, S, slab, cnt)
                    torch.cuda.synchronize()
                    err = float((yf - ref).abs().max() / ref.abs().max())
                    t = timeit(lambda: ops.pgemm(x, wsh, y, c, S, slab, cnt))
                    arms.append({"cfg": c, "tile": [bm, bn], "S": S, "wgs": tiles * S, "us": round(t, 1),
                                 "pf": round(2 * T * N * K / t / 1e9, 3), "err": round(err, 5)})
            arms.sort(key=lambda a: a["us"])
            row = {"T": T, "gemm": name, "N": N, "K": K, "lib_us": round(lib, 1),
                   "lib_pf": round(2 * T * N * K / lib / 1e9, 3), "best": arms[0] if arms else None,
                   "speedup": round(lib / arms[0]["us"], 3) if arms else None, "arms": arms}
            line = json.dumps(row)
            print(json.dumps({k: v for k, v in row.items() if k != "arms"}), flush=True)
            if out:
                out.write(line + "\n")
                out.flush()


if __name__ == "__main__":
    main()
