"""Probe: replay tests/test_xgmi_gpu.py::test_xgmi_all_reduce's sequence; compare GPU reads of the outputs
(twice) with a host copy, to tell stale cache lines on the reading side from lost writes."""
import time

import torch

from symmetry_amd.ops import _native

ops = _native.ops()
dev = torch.device("cuda", 0)
for n in (4096, 8 * 3001, 262144):
    for dtype in (torch.float32, torch.bfloat16):
        for world in (2, 3):
            hs = [int(ops.xgmi_create(1 << 20, world, r, 0)) for r in range(world)]
            for h in hs:
                ops.xgmi_connect_local(h, hs)
            g = torch.Generator(device="cpu").manual_seed(n + world)
            for it in range(3):
                xs = [torch.randn(n, generator=g).to(dev, dtype) for _ in range(world)]
                outs = [torch.full_like(x, float("nan")) for x in xs]
                ops.xgmi_all_reduce_multi(xs, outs, hs)
                torch.cuda.synchronize()
                ref = torch.zeros(n, dtype=torch.float32, device=dev)
                for x in xs:
                    ref += x.float()
                ref = ref.to(dtype)
                refc = sum(x.cpu().float() for x in xs).to(dtype)
                res = []
                for r in range(world):
                    m1 = int((outs[r] != ref).sum())
                    torch.cuda.synchronize()
                    time.sleep(0.05)
                    m2 = int((outs[r] != ref).sum())
                    hc = outs[r].cpu()
                    mh = int((hc != refc).sum())
                    bad = (hc != refc).nonzero().flatten()[:2].tolist()
                    res.append((m1, m2, mh, bad, ops.xgmi_error(hs[r])))
                if any(v[0] or v[1] or v[2] for v in res):
                    print(n, dtype, world, it, res, flush=True)
            for h in hs:
                ops.xgmi_destroy(h)
print("done", flush=True)
