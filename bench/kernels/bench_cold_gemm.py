"""Weight-streaming projections with the Infinity Cache defeated: every launch of a captured graph reads a
different weight copy (>= 1.2 GB of copies in rotation), as a decode step does (each layer's weights are
read once per step).  Compares the fused decode GEMM's F32 epilogue (dg_f32, register-streamed weights)
with mgemm (LDS-DMA weight stream) at small M, us per launch and TB/s of weight bytes."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from symmetry_amd import ops  # noqa: E402
from symmetry_amd.models.layout import preshuffle  # noqa: E402


def timed_rot(fns, rounds=5):
    for f in fns:
        f()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for f in fns:
            f()
    ts = []
    for _ in range(rounds):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3 / len(fns))
    return sorted(ts)[len(ts) // 2]


def main():
    dev = torch.device("cuda")
    Ms = [int(m) for m in os.environ.get("CG_MS", "1,10,16,24,32,64").split(",")]
    for name, N, K in (("qkv", 6144, 4096), ("o", 4096, 4096), ("gate_up", 28672, 4096), ("down", 4096, 14336)):
        nbytes = N * K * 2
        copies = max(3, int(1.2e9 // nbytes) + 1)
        ws = [preshuffle(((torch.rand(N, K, device=dev) * 2 - 1) * 0.05).to(torch.bfloat16)) for _ in range(copies)]
        for M in Ms:
            x = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
            rec = {"gemm": name, "M": M, "copies": copies, "MB": round(nbytes / 1e6, 1)}
            if M <= 64:
                y = torch.empty(M, N, device=dev)
                us = timed_rot([lambda w=w: ops.dg_f32(x, w, None, 1e-5, y, wshuf=True) for w in ws * 2])
                rec["dg_f32_us"] = round(us, 2)
                rec["dg_f32_TBps"] = round(nbytes / us / 1e6, 2)
            pick = ops.choose_mgemm(M, N, K)
            cands = [pick] if pick else []
            for rw, S in ((1, 1), (2, 1), (1, 2), (2, 2), (4, 2)):
                if (rw, S) not in cands and N % (64 * rw) == 0 and 128 <= N // (64 * rw) * S <= 512:
                    cands.append((rw, S))
            for rw, S in cands:
                ys = torch.empty(S, M, N, device=dev)
                us = timed_rot([lambda w=w: ops.mgemm(x, w, ys, rw) for w in ws * 2])
                rec[f"mgemm_rw{rw}_S{S}_us"] = round(us, 2)
                rec[f"mgemm_rw{rw}_S{S}_TBps"] = round(nbytes / us / 1e6, 2)
            print(json.dumps(rec), flush=True)
        del ws
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
