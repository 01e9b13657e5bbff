"""Diagnostic: MoE block GPU vs CPU for the same inputs (skinny decode path and library prefill path)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from symmetry_amd.models.config import TINY_MIXTRAL
from symmetry_amd.models.weights import random_weights, ShardSpec, ModelWeights
from symmetry_amd.models.transformer import TransformerLM

w = random_weights(TINY_MIXTRAL, ShardSpec(), seed=0)
cpu = TransformerLM(w, "cpu")
wg = w.to("cuda")
gpu = TransformerLM(wg, "cuda")
for T in (1, 5, 8, 20, 33, 40, 100):
    x = torch.randn(T, 256, generator=torch.Generator().manual_seed(T)).bfloat16()
    for rep in range(3):
        oc = cpu.moe.forward(0, x).clone()
        og = gpu.moe.forward(0, x.cuda()).clone().cpu()
        err = (oc - og).abs().max().item()
        ids_g = gpu.moe._buf("ids", (T * 2,), torch.int32).cpu()
        ids_c = cpu.moe._buf("ids", (T * 2,), torch.int32)
        print(T, rep, "err", err, "ids_equal", torch.equal(ids_g, ids_c), "offs", gpu.moe._buf("offsets", (5,), torch.int32).tolist())
