"""Latency of the one-shot peer-memory all-reduce (csrc/kernels/xgmi_ar.hip) on ONE MI355X.

The ranks of one process run as grid slices of one launch (tests/test_xgmi_gpu.py explains why), their
buffers mapped to each other: the protocol (push into every rank's slot, per-(workgroup, source) flags,
rank-order reduce) is the multi-GPU one, with local HBM in place of the xGMI links, so this is a lower
bound on the per-collective cost (launch + push + signal + reduce), not an xGMI measurement.
Message sizes are the TP decode all-reduces of Llama-3-70B (fp32 [rows, 8192]).
Prints one JSON line per (world, rows, op); add_prep_P<n>: n column parts per row (workgroups per row)."""
import json
import sys

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.dirname(
    __import__("os").path.abspath(__file__)))))
from symmetry_amd.ops import _native  # noqa: E402

ops = _native.ops()
dev = torch.device("cuda", 0)
d = 8192
ITERS = 200
for world in (2, 4):
    hs = [int(ops.xgmi_create(4 << 20, world, r, 0)) for r in range(world)]
    for h in hs:
        ops.xgmi_connect_local(h, hs)
    for rows in (1, 4, 10, 32, 64):
        ys = [torch.randn(rows, d, device=dev) for _ in range(world)]
        resid = [torch.randn(rows, d, device=dev) for _ in range(world)]
        xw = [torch.empty(rows, d, device=dev, dtype=torch.bfloat16) for _ in range(world)]
        sss = {P: [torch.empty(rows, P, device=dev) for _ in range(world)] for P in (1, 2, 4, 8, 16)}
        w = torch.ones(d, device=dev, dtype=torch.bfloat16)
        arms = [("all_reduce", lambda: ops.xgmi_all_reduce_multi(ys, ys, hs))]
        arms += [(f"add_prep_P{P}", (lambda P=P: ops.xgmi_add_prep_multi(ys, resid, w, xw, sss[P], hs)))
                 for P in (1, 2, 4, 8, 16) if world * rows * P <= 1024]  # slices must be co-resident
        for name, fn in arms:
            for _ in range(10):
                fn()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                for _ in range(ITERS):
                    fn()
            g.replay()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            g.replay()
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / ITERS
            assert all(ops.xgmi_error(h) == 0 for h in hs)
            print(json.dumps({"bench": "xgmi_local", "op": name, "world": world, "rows": rows,
                              "bytes_per_rank": rows * d * 4, "us_per_collective": round(us, 2)}), flush=True)
    for h in hs:
        ops.xgmi_destroy(h)
