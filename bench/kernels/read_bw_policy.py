#!/usr/bin/env python3
"""Read-bandwidth probe by load path / cache policy (bench/kernels/read_bw.hip, run_read_variant): register
loads (default, nt) vs LDS-DMA (global_load_lds) rings (default, nt) streaming decode-GEMM-sized weights,
graph-replayed over rotating copies (the Infinity Cache defeated).  One JSON line per (size, variant, waves).

  python bench/kernels/read_bw_policy.py
"""
import ctypes
import json
import os
import subprocess

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
NAMES = {0: "reg_u8", 1: "reg_nt_u8", 2: "lds_r8", 3: "lds_r8_nt", 4: "lds_r16_nt", 5: "lds_r16", 6: "reg_nt_u16"}


def main():
    so = os.path.join(HERE, "read_bw.so")
    src = os.path.join(HERE, "read_bw.hip")
    if not os.path.exists(so) or os.path.getmtime(so) < os.path.getmtime(src):
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-shared", "-fPIC", src, "-o", so],
                       check=True)
    lib = ctypes.CDLL(so)
    dev = torch.device("cuda")
    sink = torch.zeros(4, dtype=torch.int32, device=dev)
    for name, mb in (("o", 32.0), ("down", 117.4), ("gate_up", 234.9)):
        nbytes = int(mb * 1e6) // (1 << 20) * (1 << 20)
        copies = max(2, (1 << 30) // nbytes + 1)
        ws = [torch.empty(nbytes // 2, dtype=torch.bfloat16, device=dev) for _ in range(copies)]
        for waves in (1024, 4096):
            for v in NAMES:
                if nbytes // 16 // waves % (64 * 16):
                    continue
                st = torch.cuda.current_stream().cuda_stream
                lib.run_read_variant(ctypes.c_void_p(ws[0].data_ptr()), ctypes.c_longlong(nbytes), waves, v,
                                     ctypes.c_void_p(sink.data_ptr()), ctypes.c_void_p(st))
                torch.cuda.synchronize()
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    st = torch.cuda.current_stream().cuda_stream
                    for c in range(16):
                        lib.run_read_variant(ctypes.c_void_p(ws[c % copies].data_ptr()), ctypes.c_longlong(nbytes),
                                             waves, v, ctypes.c_void_p(sink.data_ptr()), ctypes.c_void_p(st))
                ts = []
                for _ in range(6):
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    g.replay()
                    e1.record()
                    torch.cuda.synchronize()
                    ts.append(e0.elapsed_time(e1) * 1e3 / 16)
                us = sorted(ts)[len(ts) // 2]
                print(json.dumps({"shape": name, "MB": round(nbytes / 1e6, 1), "waves": waves, "variant": NAMES[v],
                                  "us": round(us, 2), "TBps": round(nbytes / us / 1e6, 3)}), flush=True)
            for aux in (0, 1, 2, 3, 16, 17, 18, 19):  # buffer loads by cache policy (CPol: 1 sc0, 2 nt, 16 sc1)
                if nbytes // 16 // waves % (64 * 8):
                    continue
                g = torch.cuda.CUDAGraph()
                lib.run_read_buf(ctypes.c_void_p(ws[0].data_ptr()), ctypes.c_longlong(nbytes), waves, aux,
                                 ctypes.c_void_p(sink.data_ptr()), ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
                torch.cuda.synchronize()
                with torch.cuda.graph(g):
                    st = torch.cuda.current_stream().cuda_stream
                    for c in range(16):
                        lib.run_read_buf(ctypes.c_void_p(ws[c % copies].data_ptr()), ctypes.c_longlong(nbytes), waves,
                                         aux, ctypes.c_void_p(sink.data_ptr()), ctypes.c_void_p(st))
                ts = []
                for _ in range(6):
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    g.replay()
                    e1.record()
                    torch.cuda.synchronize()
                    ts.append(e0.elapsed_time(e1) * 1e3 / 16)
                us = sorted(ts)[len(ts) // 2]
                print(json.dumps({"shape": name, "MB": round(nbytes / 1e6, 1), "waves": waves, "variant": f"buf_aux{aux}",
                                  "us": round(us, 2), "TBps": round(nbytes / us / 1e6, 3)}), flush=True)
        del ws
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
