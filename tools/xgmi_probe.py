"""Probe: do the xGMI all-reduce kernels of two in-process 'ranks' on two streams run concurrently?"""
import time

import torch

from symmetry_amd.ops import _native

ops = _native.ops()
dev = torch.device("cuda", 0)
for world in (1, 2):
    hs = [int(ops.xgmi_create(1 << 20, world, r, 0)) for r in range(world)]
    for h in hs:
        ops.xgmi_connect_local(h, hs)
    xs = [torch.ones(4096, device=dev) * (r + 1) for r in range(world)]
    outs = [torch.zeros(4096, device=dev) for _ in range(world)]
    streams = [torch.cuda.Stream() for _ in range(world)]
    torch.cuda.synchronize()
    for order in ("fwd", "rev"):
        t0 = time.perf_counter()
        rs = range(world) if order == "fwd" else reversed(range(world))
        for r in rs:
            with torch.cuda.stream(streams[r]):
                ops.xgmi_all_reduce(xs[r], outs[r], hs[r])
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        print(world, order, f"{dt*1e3:.1f} ms", [ops.xgmi_error(h) for h in hs], [float(o[0]) for o in outs], flush=True)
    for h in hs:
        ops.xgmi_destroy(h)

# same, with the streams ordered after the current stream (as tests/test_xgmi_gpu.py::_launch_all)
world = 2
hs = [int(ops.xgmi_create(1 << 20, world, r, 0)) for r in range(world)]
for h in hs:
    ops.xgmi_connect_local(h, hs)
for it in range(3):
    xs = [torch.randn(4096).to(dev) for r in range(world)]
    outs = [torch.zeros(4096, device=dev) for _ in range(world)]
    streams = [torch.cuda.Stream() for _ in range(world)]
    cur = torch.cuda.current_stream()
    for s in streams:
        s.wait_stream(cur)
    t0 = time.perf_counter()
    for r in range(world):
        with torch.cuda.stream(streams[r]):
            ops.xgmi_all_reduce(xs[r], outs[r], hs[r])
    for s in streams:
        cur.wait_stream(s)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print("wait_stream", it, f"{dt*1e3:.1f} ms", [ops.xgmi_error(h) for h in hs],
          float((outs[0] - (xs[0] + xs[1])).abs().max()), flush=True)
