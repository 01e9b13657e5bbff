"""Infinity-Cache prefetch probe (see mall_probe.hip).  Prints one JSON line per (shape, arm) with the
median over interleaved reps of:
  cold    stream W after a 1 GiB flush                               (HBM-served weight stream)
  warm    stream W right after streaming it once                     (Infinity-Cache-served)
  spin    5 us latency-bound launch (10 busy workgroups) then stream W, cold
  spin_pf the same launch carrying `pf` extra workgroups that read W, then stream W
For spin / spin_pf the JSON has the launch time, the stream time and their sum."""
import ctypes
import json
import os
import statistics
import subprocess
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    so = os.path.join(HERE, "mall_probe.so")
    src = os.path.join(HERE, "mall_probe.hip")
    if not os.path.exists(so) or os.path.getmtime(so) < os.path.getmtime(src):
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-shared", "-fPIC", src, "-o", so],
                       check=True)
    lib = ctypes.CDLL(so)
    dev = torch.device("cuda")
    sink = torch.zeros(8, dtype=torch.int32, device=dev)
    flush = torch.empty(1 << 29, dtype=torch.bfloat16, device=dev)  # 1 GiB
    S = lambda: ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    P = lambda t: ctypes.c_void_p(t.data_ptr())
    sk = P(sink)
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 15
    ticks = 500  # 5 us of the 100 MHz realtime clock
    for name, mb in (("o", 33.5), ("qkv", 50.3), ("down", 117.4)):
        nbytes = int(mb * 1e6) // (1 << 20) * (1 << 20)
        w = torch.empty(nbytes // 2, dtype=torch.bfloat16, device=dev)
        arms = ["cold", "warm", "spin"] + [f"spin_pf{p}" for p in (246, 502, 1014)]
        res = {a: [] for a in arms}
        for rep in range(reps + 2):
            for a in arms:
                lib.mp_flush(P(flush), ctypes.c_longlong(flush.numel() * 2), 2048, sk, S())
                if a == "warm":
                    lib.mp_stream(P(w), ctypes.c_longlong(nbytes), 1024, sk, S())
                e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
                e[0].record()
                if a.startswith("spin"):
                    pf = int(a[7:]) if a.startswith("spin_pf") else 0
                    lib.mp_spin(10, ctypes.c_longlong(ticks), pf, P(w), ctypes.c_longlong(nbytes), sk, S())
                e[1].record()
                lib.mp_stream(P(w), ctypes.c_longlong(nbytes), 1024, sk, S())
                e[2].record()
                torch.cuda.synchronize()
                if rep >= 2:
                    res[a].append((e[0].elapsed_time(e[1]) * 1e3, e[1].elapsed_time(e[2]) * 1e3))
        for a in arms:
            first = statistics.median(x for x, _ in res[a])
            second = statistics.median(y for _, y in res[a])
            tot = statistics.median(x + y for x, y in res[a])
            print(json.dumps({"shape": name, "MB": round(nbytes / 1e6, 1), "arm": a, "launch_us": round(first, 2),
                              "stream_us": round(second, 2), "total_us": round(tot, 2),
                              "stream_TBps": round(nbytes / second / 1e6, 2)}), flush=True)
        del w
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
