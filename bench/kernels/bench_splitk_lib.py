"""Large-M prefill projections with few output tiles (o / down: N = 4096): hipBLASLt as one GEMM (bf16 out)
vs a k-split strided-batched GEMM (torch.bmm, fp32 slabs out), each followed by the real consumer
(add_rms_norm summing the slabs).  One JSON line per (T, gemm, arm), median us of graph-replayed launches."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from symmetry_amd import ops  # noqa: E402


def timed(fn, reps=10, rounds=5):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    ts = []
    for _ in range(rounds):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3 / reps)
    return sorted(ts)[len(ts) // 2]


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--t", type=int, nargs="+", default=[512, 1280, 2048, 4096])
    args = ap.parse_args()
    dev = torch.device("cuda")
    lnw = torch.ones(4096, device=dev, dtype=torch.bfloat16)
    for name, N, K in (("o", 4096, 4096), ("down", 4096, 14336), ("qkv", 6144, 4096)):
        w = ((torch.rand(N, K, device=dev) * 2 - 1) * 0.05).to(torch.bfloat16)
        for T in args.t:
            x = (torch.rand(T, K, device=dev) * 2 - 1).to(torch.bfloat16)
            resid = torch.zeros(T, 4096, device=dev)
            xo = torch.empty(T, 4096, device=dev, dtype=torch.bfloat16)
            yb = torch.empty(T, N, device=dev, dtype=torch.bfloat16)
            cons = (lambda y: ops.add_rms_norm(y, resid, lnw, 1e-5, xo)) if N == 4096 else (lambda y: None)
            t = timed(lambda: (torch.matmul(x, w.t(), out=yb), cons(yb)))
            print(json.dumps({"T": T, "gemm": name, "arm": "matmul", "us": round(t, 2)}), flush=True)
            ref = x.float() @ w.float().t()
            for S in (2, 4):
                kc = K // S
                xs = x.view(T, S, kc).permute(1, 0, 2)
                wt = w.view(N, S, kc).permute(1, 2, 0)
                ys = torch.empty(S, T, N, device=dev)
                fn = lambda: (torch.bmm(xs, wt, out_dtype=torch.float32, out=ys), cons(ys))
                try:
                    t = timed(fn)
                except Exception as e:  # noqa: BLE001
                    print(json.dumps({"T": T, "gemm": name, "arm": f"bmm S{S}", "error": str(e)[:200]}), flush=True)
                    continue
                err = (ys.sum(0) - ref).abs().max().item()
                print(json.dumps({"T": T, "gemm": name, "arm": f"bmm S{S}", "us": round(t, 2), "max_err": round(err, 4)}),
                      flush=True)
            del x, resid, xo, yb
        del w
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
