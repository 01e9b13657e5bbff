"""Medium-M projections (65..256 tokens, Llama-3-8B shapes): mgemm (csrc/kernels/mgemm.hip) split-K slabs
vs hipBLASLt (torch.matmul), each followed by its real consumer kernel (qkv -> rope_cache, o / down ->
add_rms_norm, gate_up -> swiglu), which sums the slabs in its prologue.  Sweeps every (rw, S) the kernel
accepts with 128..1024 workgroups; one JSON line per (T, gemm, arm) with median us over graph-replayed
launches, plus the chooser's pick and max |err| of the slab sum vs an fp32 reference."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from symmetry_amd import ops  # noqa: E402
from symmetry_amd.models.layout import preshuffle  # noqa: E402
from symmetry_amd.ops import reference  # noqa: E402


def timed(fn, reps=20, rounds=5):
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


NTS = [0]


def main():
    dev = torch.device("cuda")
    torch.manual_seed(0)
    Ts = [int(t) for t in os.environ.get("MG_TS", "80,128,192,256").split(",")]
    global NTS
    NTS = [int(v) for v in os.environ.get("MG_NT", "0").split(",")]
    shapes = [("qkv", 6144, 4096), ("o", 4096, 4096), ("gate_up", 28672, 4096), ("down", 4096, 14336)]
    only = os.environ.get("MG_SHAPES")
    if only:
        shapes = [s for s in shapes if s[0] in only.split(",")]
    Hq, Hkv, D, BS = 32, 8, 128, 64
    cos_sin = reference.rope_table(4096, D, 500000.0, None, device=dev)
    kc = torch.zeros(64, Hkv, BS, D, device=dev, dtype=torch.bfloat16)
    vc = torch.zeros(64, Hkv, D, BS, device=dev, dtype=torch.bfloat16)
    lnw = torch.ones(4096, device=dev, dtype=torch.bfloat16)
    for name, N, K in shapes:
        w = ((torch.rand(N, K, device=dev) * 2 - 1) * 0.05).to(torch.bfloat16)
        ws = preshuffle(w)
        for T in Ts:
            x = (torch.rand(T, K, device=dev) * 2 - 1).to(torch.bfloat16)
            pos = torch.arange(T, device=dev, dtype=torch.int32)
            slots = torch.arange(T, device=dev, dtype=torch.int32)
            q = torch.empty(T, Hq, D, device=dev, dtype=torch.bfloat16)
            resid = torch.zeros(T, 4096, device=dev, dtype=torch.float32)
            xo = torch.empty(T, 4096, device=dev, dtype=torch.bfloat16)
            act = torch.empty(T, N // 2, device=dev, dtype=torch.bfloat16)

            def consume(y):
                if name == "qkv":
                    ops.rope_cache(y, pos, slots, cos_sin, q, kc, vc, Hq, Hkv, perm=True)
                elif name == "gate_up":
                    ops.swiglu(y, act, interleaved=True)
                else:
                    ops.add_rms_norm(y, resid, lnw, 1e-5, xo)

            ref = x.float() @ w.float().t()
            yb = torch.empty(T, N, device=dev, dtype=torch.bfloat16)
            t_lib = timed(lambda: torch.matmul(x, w.t(), out=yb))
            t_lib_c = timed(lambda: (torch.matmul(x, w.t(), out=yb), consume(yb)))
            print(json.dumps({"T": T, "gemm": name, "arm": "hipblaslt", "gemm_us": round(t_lib, 2),
                              "with_consumer_us": round(t_lib_c, 2)}), flush=True)
            if T <= 64:  # the general path's kernel below 65 rows: split-K skinny GEMM into slabs
                Ss = ops.choose_splits(N, K)
                ysk = torch.empty(Ss, T, N, device=dev, dtype=torch.float32)
                t_sk = timed(lambda: ops.skinny_gemm(x, w, ysk))
                t_sk_c = timed(lambda: (ops.skinny_gemm(x, w, ysk), consume(ysk)))
                print(json.dumps({"T": T, "gemm": name, "arm": f"skinny S{Ss}", "gemm_us": round(t_sk, 2),
                                  "with_consumer_us": round(t_sk_c, 2)}), flush=True)
                t_lib_c = min(t_lib_c, t_sk_c)
            pick = ops.choose_mgemm(T, N, K)
            for rw in (1, 2, 3, 4):
                if N % (64 * rw) or (T > 128 and rw > 2):
                    continue
                for S in (1, 2, 4, 7, 8, 14, 16, 28, 32, 56, 64):
                    if (K // 64) % S:
                        continue
                    wgs = N // (64 * rw) * S
                    if wgs < 128 or wgs > (512 if T <= 64 else 1024):
                        continue
                    y = torch.empty(S, T, N, device=dev, dtype=torch.float32)
                    ops.mgemm(x, ws, y, rw)
                    torch.cuda.synchronize()
                    err = (y.sum(0) - ref).abs().max().item()
                    for nt in NTS:
                        torch.ops.symmetry_amd.mgemm_nt(nt)
                        t = timed(lambda: ops.mgemm(x, ws, y, rw))
                        tc = timed(lambda: (ops.mgemm(x, ws, y, rw), consume(y)))
                        print(json.dumps({"T": T, "gemm": name, "arm": f"mgemm rw{rw} S{S}" + (" nt" if nt else ""),
                                          "wgs": wgs, "gemm_us": round(t, 2), "with_consumer_us": round(tc, 2),
                                          "speedup_vs_lib": round(t_lib_c / tc, 3), "max_err": round(err, 5),
                                          "chosen": pick == (rw, S)}), flush=True)
                    torch.ops.symmetry_amd.mgemm_nt(0)
                    del y
            del x
        del w, ws
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
