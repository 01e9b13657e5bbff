"""Prefill attention kernel alone (csrc/kernels/attention.hip, attn_prefill): causal, paged K/V, GQA.

Reports us per launch and achieved TFLOP/s (4 * sum_q(visible keys) * D * Hq, causal) for a few prompt
shapes, hipGraph-replayed.   python bench/kernels/bench_attn_prefill.py
"""
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from symmetry_amd import ops  # noqa: E402


def run(lens, Hq=32, Hkv=8, BS=64, reps=20):
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    D = 128
    nblk = [(n + BS - 1) // BS for n in lens]
    NB = sum(nblk) + 1
    kc = torch.randn(NB, Hkv, BS, D, device=dev, generator=g).bfloat16()
    vc = torch.randn(NB, Hkv, D, BS, device=dev, generator=g).bfloat16()
    mb = max(nblk)
    bt = torch.zeros(len(lens), mb, dtype=torch.int32)
    i = 1
    for s, nb in enumerate(nblk):
        bt[s, :nb] = torch.arange(i, i + nb)
        i += nb
    bt = bt.to(dev)
    T = sum(lens)
    q = torch.randn(T, Hq, D, device=dev, generator=g).bfloat16()
    out = torch.empty_like(q)
    ctx = torch.tensor(lens, dtype=torch.int32, device=dev)
    cu = torch.tensor([0] + list(torch.tensor(lens).cumsum(0).tolist()), dtype=torch.int32, device=dev)
    tiles = []
    for s, n in enumerate(lens):
        for r in range(0, n, 64):
            tiles.append((s, r))
    tiles.sort(key=lambda t: -(t[1] + 64))  # heaviest first, as the engine orders them
    tiles = torch.tensor(tiles, dtype=torch.int32, device=dev).view(-1, 2)
    scale = 1 / math.sqrt(D)
    fn = lambda: ops.attn_prefill(q, kc, vc, bt, ctx, cu, tiles, out, scale)  # noqa: E731
    fn()
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, stream=s):
            for _ in range(10):
                fn()
    torch.cuda.synchronize()
    graph.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        graph.replay()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / (reps * 10)
    flops = sum(4 * (n * (n + 1) / 2) * D * Hq for n in lens)
    return {"lens": f"{len(lens)}x{lens[0]}", "us": round(us, 1), "tflops": round(flops / us / 1e6, 1)}


if __name__ == "__main__":
    shapes = {"1x128": [128], "6x128": [128] * 6, "10x128": [128] * 10, "4x256": [256] * 4, "10x1024": [1024] * 10, "1x4096": [4096], "4x2048": [2048] * 4, "1x8192": [8192]}
    for name in (sys.argv[1:] or list(shapes)):
        print(json.dumps(run(shapes[name])), flush=True)
