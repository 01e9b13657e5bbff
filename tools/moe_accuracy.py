"""MoE block accuracy on the GPU: grouped MFMA path vs per-expert library path vs the fp32 CPU oracle."""
import sys

import torch

sys.path.insert(0, ".")
from symmetry_amd.models import moe as moe_mod  # noqa: E402
from symmetry_amd.models.config import resolve  # noqa: E402
from symmetry_amd.models.transformer import TransformerLM  # noqa: E402
from symmetry_amd.models.weights import ShardSpec, random_weights  # noqa: E402

cfg = resolve(sys.argv[1] if len(sys.argv) > 1 else "tiny-mixtral")
w = random_weights(cfg, ShardSpec(), seed=3, device="cuda")
m = TransformerLM(w, "cuda")
mc = TransformerLM(w.to("cpu"), "cpu")
g = torch.Generator().manual_seed(0)
for T in (40, 250, 700):
    x = torch.randn(T, cfg.hidden_size, generator=g).bfloat16()
    ref = mc.moe.forward(0, x).clone()
    ref_ids = mc.moe._buf("ids", (T * cfg.top_k,), torch.int32).clone().view(T, -1)
    out = {}
    for grouped in (True, False):
        moe_mod.GROUPED = grouped
        out[grouped] = m.moe.forward(0, x.cuda()).float().cpu().clone()
        ids = m.moe._buf("ids", (T * cfg.top_k,), torch.int32).cpu().view(T, -1)
    flips = (ids.sort(1).values != ref_ids.sort(1).values).any(1)
    row_err = {k: (v - ref).abs().max(1).values for k, v in out.items()}
    print(T, "routing flips vs oracle:", int(flips.sum()),
          {k: (float(e.max()), int(e.argmax()), float(e[~flips].max()) if (~flips).any() else None)
           for k, e in row_err.items()}, "grouped-vs-library", float((out[True] - out[False]).abs().max()), flush=True)
