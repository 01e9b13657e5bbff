#!/usr/bin/env python3
"""Decode-step engine (csrc/kernels/decode_layers.hip) phase timeline from in-kernel wall-clock stamps.

One TP rank's shard on one GPU (bench/tp_shard.py's world-1 communicator), eager decode steps; the last step runs
with stamps: every workgroup's 100 MHz wall clock when each phase's edge passed and when it signalled the phase.
Per phase: work span after the edge (median / max over workgroups), the edge latency (last producer's signal ->
first / median consumer release), and the layer period.

  python bench/kernels/bench_engine.py --tp 8 --clients 10
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "bench"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3:8b")
    ap.add_argument("--tp", type=int, default=8)
    ap.add_argument("--clients", type=int, default=10)
    ap.add_argument("--prompt-len", type=int, default=128)
    ap.add_argument("--steps", type=int, default=8)
    args = ap.parse_args()
    import torch

    from symmetry_amd.engine.llm_engine import EngineConfig, LLMEngine
    from symmetry_amd.engine.sequence import SamplingParams
    from symmetry_amd.models import transformer as tr
    from tp_shard import LocalXgmi

    tr.DECODE_ENGINE = "1"
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    C, P = args.clients, args.prompt_len
    comm = LocalXgmi(dev, args.tp)
    cfg = EngineConfig(model=args.model, device="cuda:0", max_num_seqs=C, max_model_len=2048,
                       num_kv_blocks=C * 32 + 16, tp_size=args.tp, tp_rank=0, weight_init="shard", use_graphs=False,
                       max_num_batched_tokens=max(8192, C * P))
    eng = LLMEngine(cfg, tp_comm=comm)
    params = SamplingParams(max_tokens=args.steps + 8, temperature=0.0, ignore_eos=True)
    seqs = [eng.add_request(f"c{i}", [(31 * i + 7 * k) % 100000 + 300 for k in range(P)], params) for i in range(C)]
    while any(s.first_token_time is None for s in seqs):
        eng.step()
    for _ in range(args.steps):
        eng.step()
    model = eng.model
    plan = model._engine_cache.get("plan")
    G, L = plan[2], model.cfg.num_layers
    st = torch.zeros(G * L * 5 * 8, dtype=torch.int64, device=dev)
    model.engine_stamps = st
    eng.step()
    torch.cuda.synchronize()
    model.engine_stamps = None
    s = st.view(G, L, 5, 8).cpu().double() / 100.0  # us
    names = ["qkv", "attn", "o", "gu", "down"]
    out = {"model": args.model, "tp": args.tp, "clients": C, "grid": G, "ksq": plan[0], "layers": L}
    t0 = s[:, 0, 0, 0].min()
    rows = {}
    mid = range(1, L - 1)
    for p, n in enumerate(names):
        work, edge_first, edge_med, skew = [], [], [], []
        for l in mid:
            passed, signed = s[:, l, p, 0], s[:, l, p, 1]
            work.append(float((signed - passed).median()))
            skew.append(float(signed.max() - signed.median()))
            nl, npx = (l, p + 1) if p + 1 < 5 else (l + 1, 0)
            nxt = s[:, nl, npx, 0]
            edge_first.append(float(nxt.min() - signed.max()))
            edge_med.append(float(nxt.median() - signed.max()))
        # sub-phase stamps of the first unit (2: operands landed, 3: after the reduce barrier / rope barrier, 4: epilogue
        # done / merge barrier), relative to the edge, median over the workgroups that have them
        sub, spread, split = {}, {}, {}
        n_attn = C * model.hkv * 8  # workgroups with an attention unit (decode_layers.hip DL_APARTS = 8)
        for k in (2, 3, 4):
            vals, q10, q90, va, vo = [], [], [], [], []
            for l in mid:
                v = s[:, l, p, k]
                ok = v > 0
                if ok.any():
                    rel = v[ok] - s[ok, l, p, 0]
                    vals.append(float(rel.median()))
                    q10.append(float(rel.quantile(0.1)))
                    q90.append(float(rel.quantile(0.9)))
                    idx = torch.nonzero(ok).flatten()
                    ra, ro = rel[idx < n_attn], rel[idx >= n_attn]
                    if len(ra) and len(ro):
                        va.append(float(ra.median()))
                        vo.append(float(ro.median()))
            if vals:
                sub[str(k)] = round(sum(vals) / len(vals), 2)
                spread[str(k)] = [round(sum(q10) / len(q10), 2), round(sum(q90) / len(q90), 2)]
            if va:
                split[str(k)] = [round(sum(va) / len(va), 2), round(sum(vo) / len(vo), 2)]
        rows[n] = {"sub_us": sub, "sub_p10_p90_us": spread, "sub_attn_wgs_vs_rest_us": split, "work_median_us": round(sum(work) / len(work), 2),
                   "last_signal_skew_us": round(sum(skew) / len(skew), 2),
                   "edge_release_first_us": round(sum(edge_first) / len(edge_first), 2),
                   "edge_release_median_us": round(sum(edge_med) / len(edge_med), 2)}
    period = [float(s[:, l + 1, 0, 0].median() - s[:, l, 0, 0].median()) for l in range(0, L - 1)]
    out["phases"] = rows
    out["layer_period_us"] = round(sum(period[1:]) / max(1, len(period) - 1), 2)
    out["launch_span_us"] = round(float(s[:, L - 1, 4, 1].max() - t0), 1)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
