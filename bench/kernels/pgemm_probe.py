"""Ablation probe of the prefill GEMM's main loop (csrc/kernels/pgemm.hip built standalone with -DPG_PROBE):
full kernel vs no MFMAs (PG_ABLATE=1: DMA intake + LDS reads alone) vs no DMAs after the prologue (PG_ABLATE=2:
MFMAs on stale slots), per tile config -- which side bounds a k-step (cdna_hip_programming.md §5.4 rule 17).

  python bench/kernels/pgemm_probe.py --build     (CPU: compiles bench/kernels/pg_probe_*.so)
  python bench/kernels/pgemm_probe.py --tokens 768 --shape 28672 4096 --cfgs 0 1
  python bench/kernels/pgemm_probe.py --grouped 64 128 --shape 28672 4096 --cfgs 1 10 --variants full noskip
  (--grouped: rows per expert of 8 experts, segments 0.4x .. 2.0x the mean, weights [8, N, K])
"""
import argparse
import ctypes
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
VARIANTS = {"full": [], "no_mfma": ["-DPG_ABLATE=1"], "no_dma": ["-DPG_ABLATE=2"], "nosplit": ["-DPG_SPLIT_ISSUE=0"],
            "slots3": ["-DPG_MAX_SLOTS=3"], "slots5": ["-DPG_MAX_SLOTS=5"], "slots6": ["-DPG_MAX_SLOTS=6"]}


def build(names):
    src = os.path.join(ROOT, "csrc", "kernels", "pgemm.hip")
    for name in names:
        flags = VARIANTS[name]
        out = os.path.join(HERE, f"pg_probe_{name}.so")
        subprocess.run(["/opt/rocm/bin/hipcc", "-shared", "-fPIC", "-O3", "-std=c++17", "--offload-arch=gfx950",
                        "-ffp-contract=fast", "-munsafe-fp-atomics", "-DPG_PROBE", "-I", os.path.dirname(src), src,
                        "-o", out] + flags, check=True)
        print(out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--tokens", type=int, nargs="+", default=[768])
    ap.add_argument("--shape", type=int, nargs=2, default=[28672, 4096])
    ap.add_argument("--cfgs", type=int, nargs="+", default=[0])
    ap.add_argument("--S", type=int, default=1, help="k splits (> 1: fp32 slabs, no in-launch reduction)")
    ap.add_argument("--rounds", type=int, default=3, help="interleaved rounds over the variants (min reported)")
    ap.add_argument("--variants", nargs="+", default=list(VARIANTS))
    ap.add_argument("--grouped", type=int, nargs="+", default=None, metavar="ROWS")
    args = ap.parse_args()
    if args.build:
        return build(args.variants)
    import torch

    sys.path.insert(0, HERE)
    from bench_pgemm import timeit

    libs = {v: ctypes.CDLL(os.path.join(HERE, f"pg_probe_{v}.so")) for v in args.variants}
    N, K = args.shape
    dev = torch.device("cuda")
    if args.grouped:
        return grouped(args, libs, N, K, dev, timeit)
    w = ((torch.rand(N, K, device=dev) * 2 - 1) * 0.05).bfloat16()
    for T in args.tokens:
        x = (torch.rand(T, K, device=dev) * 2 - 1).bfloat16()
        y = torch.empty(args.S * T * N * (2 if args.S > 1 else 1), device=dev, dtype=torch.bfloat16)
        for c in args.cfgs:
            row = {"T": T, "N": N, "K": K, "cfg": c, "S": args.S}
            for _ in range(args.rounds):  # interleaved rounds in one process (rule 24): min per variant
                for v, lib in libs.items():
                    def run():
                        s = torch.cuda.current_stream().cuda_stream
                        rc = lib.pg_probe(c, ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(w.data_ptr()),
                                          ctypes.c_void_p(y.data_ptr()), T, N, K, args.S, ctypes.c_void_p(s))
                        assert rc == 0
                    t = round(timeit(run), 1)
                    row[v + "_us"] = min(row.get(v + "_us", 1e9), t)
            print(json.dumps(row), flush=True)


def grouped(args, libs, N, K, dev, timeit):
    import torch

    E = 8
    w = ((torch.rand(E, N, K, device=dev) * 2 - 1) * 0.05).bfloat16()
    for rows in args.grouped:
        counts = [max(1, int(rows * f)) for f in (0.4, 2.0, 0.8, 1.2, 0.6, 1.4, 1.0, 0.6)]
        R = sum(counts)
        off = torch.zeros(E + 1, dtype=torch.int32)
        off[1:] = torch.cumsum(torch.tensor(counts), 0)
        off = off.to(dev)
        x = (torch.rand(R, K, device=dev) * 2 - 1).bfloat16()
        y = torch.empty(R, N, device=dev, dtype=torch.bfloat16)
        for c in args.cfgs:
            row = {"grouped_rows": rows, "R": R, "N": N, "K": K, "cfg": c}
            for _ in range(args.rounds):
                for v, lib in libs.items():
                    def run():
                        s = torch.cuda.current_stream().cuda_stream
                        rc = lib.pg_probe_grouped(c, ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(w.data_ptr()),
                                                  ctypes.c_void_p(off.data_ptr()), E, ctypes.c_void_p(y.data_ptr()),
                                                  R, N, K, ctypes.c_void_p(s))
                        assert rc == 0
                    t = round(timeit(run), 1)
                    row[v + "_us"] = min(row.get(v + "_us", 1e9), t)
            print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
