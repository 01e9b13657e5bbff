"""Probe: mismatches of the multi-rank xGMI all-reduce at 3 ranks x 262144 fp32."""
import torch

from symmetry_amd.ops import _native

ops = _native.ops()
dev = torch.device("cuda", 0)
for world, n in ((2, 262144), (3, 262144), (3, 65536), (3, 4096)):
    hs = [int(ops.xgmi_create(1 << 20, world, r, 0)) for r in range(world)]
    for h in hs:
        ops.xgmi_connect_local(h, hs)
    g = torch.Generator().manual_seed(1)
    for it in range(4):
        xs = [torch.randn(n, generator=g).to(dev) for _ in range(world)]
        outs = [torch.full_like(x, float("nan")) for x in xs]
        ops.xgmi_all_reduce_multi(xs, outs, hs)
        torch.cuda.synchronize()
        ref = xs[0].clone()
        for x in xs[1:]:
            ref += x
        torch.cuda.synchronize()
        res = []
        for r in range(world):
            m1 = int((outs[r] != ref).sum())
            nan = int(outs[r].isnan().sum())
            torch.cuda.synchronize()
            m2 = int((outs[r] != ref).sum())
            bad = (outs[r] != ref).nonzero().flatten()
            first = bad[:3].tolist()
            res.append((m1, m2, nan, first, ops.xgmi_error(hs[r])))
        print(world, n, it, res, flush=True)
    for h in hs:
        ops.xgmi_destroy(h)
