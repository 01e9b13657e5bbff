"""Fused decode attention block (QKV -> attention -> O, one launch) vs the three fused launches.

Llama-3-8B layer shapes, MFMA-preshuffled weights, M concurrent sequences of context C, L distinct layers
captured in one hipGraph and replayed (the engine's regime).  `--stamps` also prints the in-kernel role
timeline of one launch (s_memrealtime, 10 ns ticks): when QKV tiles end, when attention units see their
group complete / finish, when O tiles see the attention output / finish.

  python bench/kernels/bench_decode_block.py --M 10 --ctx 200 --cfgs 0 1 2 --stamps
"""
import argparse
import json
import math
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from symmetry_amd import ops  # noqa: E402
from symmetry_amd.models.layout import preshuffle, qkv_perm  # noqa: E402
from symmetry_amd.ops import reference as ref  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=10)
    ap.add_argument("--ctx", type=int, default=200)
    ap.add_argument("--layers", type=int, default=16)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--cfgs", type=int, nargs="+", default=[0])
    ap.add_argument("--stamps", action="store_true")
    args = ap.parse_args()
    dev = torch.device("cuda")
    M, C, L = args.M, args.ctx, args.layers
    Hq, Hkv, D, d, BS = 32, 8, 128, 4096, 64
    g = torch.Generator(device=dev).manual_seed(0)
    nblk = (C + BS - 1) // BS
    NB = M * nblk + 2
    kc = [torch.randn(NB, Hkv, BS, D, device=dev, generator=g).bfloat16() for _ in range(L)]
    vc = [torch.randn(NB, Hkv, D, BS, device=dev, generator=g).bfloat16() for _ in range(L)]
    bt = torch.arange(M * nblk, device=dev, dtype=torch.int32).view(M, nblk)
    ctx = torch.full((M,), C, device=dev, dtype=torch.int32)
    pos = ctx - 1
    slots = (bt[:, (C - 1) // BS] * BS + (C - 1) % BS).int()
    N = (Hq + 2 * Hkv) * D
    perm = qkv_perm(Hq, Hkv, D).to(dev)
    Wq = [preshuffle((torch.randn(N, d, device=dev, generator=g) / 64).bfloat16()[perm].contiguous()) for _ in range(L)]
    Wo = [preshuffle((torch.randn(d, Hq * D, device=dev, generator=g) / 64).bfloat16()) for _ in range(L)]
    ln2 = (torch.randn(d, device=dev, generator=g) * 0.1 + 1).bfloat16()
    cs = ref.rope_table(4096, D, 500000.0, device=dev)
    xw = torch.randn(M, d, device=dev, generator=g).bfloat16()
    ss = torch.rand(M, d // 16, device=dev, generator=g) * 16 + 1
    resid = torch.randn(M, d, device=dev, generator=g)
    q = torch.empty(M, Hq, D, device=dev, dtype=torch.bfloat16)
    attn = torch.empty(M, Hq, D, device=dev, dtype=torch.bfloat16)
    mp = (nblk * BS + ops.ATTN_DECODE_PART - 1) // ops.ATTN_DECODE_PART
    tmp_o = torch.empty(M, Hq, mp, D, device=dev)
    tmp_ml = torch.empty(M, Hq, mp, 2, device=dev)
    mpb = (nblk * BS + ops.ATTN_BLOCK_PART - 1) // ops.ATTN_BLOCK_PART
    tmp_ob = torch.empty(M, Hq, mpb, D, device=dev)
    tmp_mlb = torch.empty(M, Hq, mpb, 2, device=dev)
    cnt = torch.zeros(M * Hkv, device=dev, dtype=torch.int32)
    ctl = torch.zeros(ops.DECODE_BLOCK_CTL, device=dev, dtype=torch.int32)
    scale = 1 / math.sqrt(D)
    nat = ops._native.ops()

    def three(i):
        ops.dg_qkv(xw, Wq[i], ss, 1e-5, pos, slots, cs, q, kc[i], vc[i], Hq, Hkv, wshuf=True)
        ops.attn_decode(q, kc[i], vc[i], bt, ctx, attn, tmp_o, tmp_ml, cnt, scale)
        ops.dg_resid(attn.view(M, -1), Wo[i], resid, ln2, xw, ss, wshuf=True)

    def block(i, cfg, stamps=None):
        nat.decode_block(xw, Wq[i], ss, 1e-5, pos, slots, cs, q, kc[i], vc[i], bt, ctx, attn, tmp_ob, tmp_mlb, cnt,
                         scale, Wo[i], resid, ln2, xw, ss, ctl, True, stamps, cfg)

    def timed(fn):
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            for i in range(L):
                fn(i)
            torch.cuda.synchronize()
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph, stream=s):
                for i in range(L):
                    fn(i)
        torch.cuda.synchronize()
        for _ in range(3):
            graph.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.reps):
            graph.replay()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e3 / args.reps / L

    res = {"three_launch": round(timed(three), 2)}
    for cfg in args.cfgs:
        res[f"block_cfg{cfg}"] = round(timed(lambda i, c=cfg: block(i, c)), 2)
        assert not ctl.any(), "dependency wait gave up"
    print(json.dumps({"M": M, "ctx": C, "us_per_layer": res}), flush=True)
    if args.stamps:
        # stamps of every layer of a graph replay: per-layer WG span and the gap to the next layer's first WG
        grid = N // 16 + M * Hkv * mpb + d // 16
        for cfg in args.cfgs:
            st = torch.zeros(L, grid, 4, device=dev, dtype=torch.int64)
            s = torch.cuda.Stream()
            with torch.cuda.stream(s):
                graph = torch.cuda.CUDAGraph()
                with torch.cuda.graph(graph, stream=s):
                    for i in range(L):
                        block(i, cfg, st[i])
            torch.cuda.synchronize()
            for _ in range(3):
                graph.replay()
            torch.cuda.synchronize()
            t = st.cpu()
            spans, gaps, phases = [], [], []
            for i in range(L):
                r = t[i]
                t0, t1 = int(r[:, 0].min()), int(r[:, 2].max())
                spans.append((t1 - t0) / 100.0)
                if i + 1 < L:
                    gaps.append((int(t[i + 1][:, 0].min()) - t1) / 100.0)
                q_end = int(r[r[:, 3] == 0][:, 2].max())
                ar = r[(r[:, 3] == 1) & (r[:, 1] > 0)]
                a_end = int(ar[:, 2].max())
                o_wait = int(r[r[:, 3] == 2][:, 1].median())
                phases.append(((q_end - t0) / 100.0, (a_end - t0) / 100.0, (o_wait - t0) / 100.0))
            med = lambda xs: sorted(xs)[len(xs) // 2]
            r = t[L // 2]
            t0 = int(r[:, 0].min())
            detail = {}
            for role, name in ((0, "qkv"), (1, "attn"), (2, "o")):
                rr = r[r[:, 3] == role]
                if name == "attn":
                    rr = rr[rr[:, 1] > 0]
                row = {}
                for col, cname in ((0, "start"), (1, "wait_done"), (2, "end")):
                    v = rr[:, col]
                    v = v[v > 0]
                    if v.numel():
                        us = ((v - t0).double() / 100.0).sort().values
                        row[cname] = [round(float(us[int(q * (len(us) - 1))]), 2) for q in (0, 0.1, 0.5, 0.9, 1.0)]
                detail[name] = row
            print(json.dumps({"cfg": cfg, "layer_mid_pcts_0_10_50_90_100": detail}), flush=True)
            print(json.dumps({"cfg": cfg, "graph_span_us_med": med(spans), "gap_to_next_us_med": med(gaps) if gaps else None,
                              "qkv_end_attn_end_o_wait_med": [med([p[j] for p in phases]) for j in range(3)]}),
                  flush=True)


if __name__ == "__main__":
    main()
