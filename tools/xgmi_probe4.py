"""Probe: classify the wrong outputs of the 3-rank x 262144 multi-rank xGMI all-reduce."""
import itertools

import torch

from symmetry_amd.ops import _native

ops = _native.ops()
dev = torch.device("cuda", 0)
world, n = 3, 262144
for trial in range(3):
    hs = [int(ops.xgmi_create(1 << 20, world, r, 0)) for r in range(world)]
    for h in hs:
        ops.xgmi_connect_local(h, hs)
    g = torch.Generator(device="cpu").manual_seed(trial)
    for it in range(4):
        xc = [torch.randn(n, generator=g) for _ in range(world)]
        xs = [x.to(dev) for x in xc]
        outs = [torch.full_like(x, float("nan")) for x in xs]
        ops.xgmi_all_reduce_multi(xs, outs, hs)
        torch.cuda.synchronize()
        full = xc[0] + xc[1] + xc[2]
        cands = {"nan": None}
        for k in range(world + 1):
            for sub in itertools.combinations(range(world), k):
                v = torch.zeros(n)
                for s in sub:
                    v = v + xc[s]
                cands["sum" + "".join(map(str, sub))] = v
        for r in range(world):
            gclone = outs[r].clone().cpu()
            hc = outs[r].cpu()
            for name, val in (("host", hc), ("gpuclone", gclone)):
                bad = (val != full)
                nb = int(bad.sum())
                if not nb:
                    continue
                idx = bad.nonzero().flatten()
                cls = {}
                for cname, cv in cands.items():
                    if cv is None:
                        m = int(val[idx].isnan().sum())
                    else:
                        m = int((val[idx] == cv[idx]).sum())
                    if m:
                        cls[cname] = m
                chunks = sorted(set((idx // 2048).tolist()))
                print(f"trial {trial} it {it} rank {r} {name}: {nb} bad, chunks {chunks[:12]}{'...' if len(chunks) > 12 else ''} "
                      f"({len(chunks)}), first {idx[:2].tolist()}, class {cls}", flush=True)
        print(f"trial {trial} it {it} err {[ops.xgmi_error(h) for h in hs]}", flush=True)
    for h in hs:
        ops.xgmi_destroy(h)
