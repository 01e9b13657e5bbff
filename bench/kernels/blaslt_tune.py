"""Offline hipBLASLt solution sweep for the library prefill GEMMs, run IN the serving process's library.

    python bench/kernels/blaslt_tune.py --shapes 6144x4096,4096x4096,28672x4096,4096x14336 --ms 128,512,768 \
        > gpurun_out/blaslt_tune.jsonl
    python tools/blaslt_table.py gpurun_out/blaslt_tune.jsonl   # -> symmetry_amd/ops/blaslt_table.json

torch loads its own hipBLASLt build, and that is the library `csrc/kernels/blaslt.hip` calls (its solution
indices differ from the /opt/rocm build's: bench/kernels/blaslt_algos.cpp numbers them for that one), so the sweep
goes through the same op (`torch.ops.symmetry_amd.blaslt_tune`): every supported TN bf16 solution timed over 3
calls with the weight rotating over >= 1 GiB of random copies (each call reads it from HBM), the 6 fastest re-timed
over 11 calls next to the heuristic's pick.  One JSON line per (N, K, M).
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from symmetry_amd.ops import _native  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="6144x4096,4096x4096,28672x4096,4096x14336")
    ap.add_argument("--ms", default="96,128,192,256,320,384,448,512,640,768,896,1024,1280,1536,2048")
    args = ap.parse_args()
    dev = torch.device("cuda")
    ops = _native.ops()
    for shape in args.shapes.split(","):
        N, K = (int(v) for v in shape.split("x"))
        copies = max(2, (1 << 30) // (N * K * 2) + 1)
        ws = [((torch.rand(N, K, device=dev) * 2 - 1) * 0.05).to(torch.bfloat16) for _ in range(copies)]
        for M in (int(m) for m in args.ms.split(",")):
            x = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
            y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            idx, us = ops.blaslt_tune(x, ws, y)
            print(json.dumps({"N": N, "K": K, "M": M, "out": "bf16", "index": idx[0], "us": round(us[0], 2),
                              "default_index": idx[1], "default_us": round(us[1], 2), "supported": idx[2]}),
                  flush=True)
        del ws
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
