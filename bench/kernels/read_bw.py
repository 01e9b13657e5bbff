"""Ceiling probe: how fast can a plain streaming read of a decode-GEMM-sized weight go on this chip?
Compares against bench_decode_gemm.py numbers (same bytes, same number of waves)."""
import ctypes
import json
import os
import subprocess

import torch

HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    so = os.path.join(HERE, "read_bw.so")
    if not os.path.exists(so):
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-shared", "-fPIC",
                        os.path.join(HERE, "read_bw.hip"), "-o", so], check=True)
    lib = ctypes.CDLL(so)
    dev = torch.device("cuda")
    sink = torch.zeros(4, dtype=torch.int32, device=dev)
    for name, mb in (("o", 33.5), ("qkv", 50.3), ("down", 117.4), ("gate_up", 234.9), ("lm_head", 1050.7)):
        nbytes = int(mb * 1e6) // (1 << 20) * (1 << 20)
        copies = max(2, (1 << 30) // nbytes + 1)
        ws = [torch.empty(nbytes // 2, dtype=torch.bfloat16, device=dev) for _ in range(copies)]
        for waves in (1024, 2048, 4096, 8192):
            for u in (4, 8, 16):
                if nbytes // 16 // waves % (64 * u):
                    continue
                st = torch.cuda.current_stream().cuda_stream
                g = torch.cuda.CUDAGraph()
                lib.run_read(ctypes.c_void_p(ws[0].data_ptr()), ctypes.c_longlong(nbytes), waves, u,
                             ctypes.c_void_p(sink.data_ptr()), ctypes.c_void_p(st))
                torch.cuda.synchronize()
                with torch.cuda.graph(g):
                    st = torch.cuda.current_stream().cuda_stream
                    for c in range(16):
                        lib.run_read(ctypes.c_void_p(ws[c % copies].data_ptr()), ctypes.c_longlong(nbytes), waves, u,
                                     ctypes.c_void_p(sink.data_ptr()), ctypes.c_void_p(st))
                ts = []
                for _ in range(6):
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    g.replay()
                    e1.record()
                    torch.cuda.synchronize()
                    ts.append(e0.elapsed_time(e1) * 1e3 / 16)
                us = sorted(ts)[len(ts) // 2]
                print(json.dumps({"shape": name, "MB": round(nbytes / 1e6, 1), "waves": waves, "U": u,
                                  "us": round(us, 2), "TBps": round(nbytes / us / 1e6, 3)}), flush=True)
        del ws
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
