"""Experimental prefill GEMM (prefill_gemm.hip in this directory) vs hipBLASLt (torch.matmul) at the Llama-3-8B prefill
projection shapes.  One JSON line per (T, gemm): median us over graph-replayed launches (random
[-1, 1) operands), TFLOP/s, max |err| vs an fp32 torch reference.  Both arms run interleaved in one
process (cdna_hip_programming.md §5.4 rule 24)."""
import ctypes
import json
import os
import subprocess
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(HERE)))
KDIR = os.path.join(ROOT, "csrc", "kernels")


def build():
    so = os.path.join(HERE, "pgemm_dev.so")
    srcs = [os.path.join(HERE, "prefill_gemm.hip"), os.path.join(HERE, "pgemm_capi.hip")]
    deps = srcs + [os.path.join(HERE, "pgemm.h"), os.path.join(KDIR, "common.h")]
    if not os.path.exists(so) or any(os.path.getmtime(d) > os.path.getmtime(so) for d in deps):
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-shared", "-fPIC",
                        "-I", KDIR, "-I", HERE] + srcs + ["-o", so], check=True)
    return ctypes.CDLL(so)


def timed(fn, reps=20, rounds=7):
    g = torch.cuda.CUDAGraph()
    fn()
    torch.cuda.synchronize()
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
    lib = build()
    if len(sys.argv) > 1 and sys.argv[1] == "--build-only":
        return
    if len(sys.argv) > 1 and sys.argv[1] == "--one":  # --one T N K [reps]: launches for rocprofv3 counters
        T, N, K = (int(a) for a in sys.argv[2:5])
        reps = int(sys.argv[5]) if len(sys.argv) > 5 else 20
        dev = torch.device("cuda")
        x = (torch.rand(T, K, device=dev) * 2 - 1).to(torch.bfloat16)
        w = (torch.rand(N, K, device=dev) * 2 - 1).to(torch.bfloat16)
        y = torch.empty(T, N, device=dev, dtype=torch.bfloat16)
        for _ in range(reps):
            lib.pg_bf16(ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(w.data_ptr()), ctypes.c_void_p(y.data_ptr()),
                        T, N, K, ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
            torch.matmul(x, w.t())
        torch.cuda.synchronize()
        return
    dev = torch.device("cuda")
    torch.manual_seed(0)
    shapes = [("qkv", 6144, 4096), ("o", 4096, 4096), ("gate_up", 28672, 4096), ("down", 4096, 14336)]
    Ts = [int(t) for t in os.environ.get("PG_TS", "128,256,512,1280,4096").split(",")]
    for T in Ts:
        for name, N, K in shapes:
            x = (torch.rand(T, K, device=dev) * 2 - 1).to(torch.bfloat16)
            w = (torch.rand(N, K, device=dev) * 2 - 1).to(torch.bfloat16)
            y = torch.empty(T, N, device=dev, dtype=torch.bfloat16)
            y2 = torch.empty_like(y)
            st = lambda: ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
            run = lambda: lib.pg_bf16(ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(w.data_ptr()),
                                      ctypes.c_void_p(y.data_ptr()), T, N, K, st())
            lib_ = lambda: torch.matmul(x, w.t(), out=y2)
            variants = [int(v) for v in os.environ.get("PG_VARIANTS", "0").split(",")]
            ref = x.float() @ w.float().t()
            rec = {"T": T, "gemm": name, "N": N, "K": K}
            fl = 2.0 * T * N * K
            t_lib = []
            t_var = {v: [] for v in variants}
            for v in variants:
                lib.pg_variant(v)
                y.fill_(float("nan"))
                run()
                torch.cuda.synchronize()
                rec[f"v{v}_err"] = round((y.float() - ref).abs().max().item(), 4)
            for _ in range(3):
                for v in variants:
                    lib.pg_variant(v)
                    t_var[v].append(timed(run))
                t_lib.append(timed(lib_))
            ul = sorted(t_lib)[1]
            rec["hipblaslt_us"] = round(ul, 1)
            rec["hipblaslt_tflops"] = round(fl / ul / 1e6, 1)
            for v in variants:
                us = sorted(t_var[v])[1]
                rec[f"v{v}_us"] = round(us, 1)
                rec[f"v{v}_tflops"] = round(fl / us / 1e6, 1)
                rec[f"v{v}_speedup"] = round(ul / us, 3)
            rec["ref_absmax"] = round(ref.abs().max().item(), 1)
            print(json.dumps(rec), flush=True)
            del x, w, y, y2, ref
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
