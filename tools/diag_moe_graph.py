"""Diagnostic: MoE block eager vs hipGraph replay (state carried across replays?)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from symmetry_amd.models.config import TINY_MIXTRAL
from symmetry_amd.models.weights import random_weights, ShardSpec, ModelWeights
from symmetry_amd.models.transformer import TransformerLM

w = random_weights(TINY_MIXTRAL, ShardSpec(), seed=0)
wg = w.to("cuda")
gpu = TransformerLM(wg, "cuda")
T = 8
x = torch.randn(T, 256, generator=torch.Generator().manual_seed(1)).bfloat16().cuda()
ref = gpu.moe.forward(0, x).clone()
s = torch.cuda.Stream(); s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    gpu.moe.forward(0, x)
torch.cuda.current_stream().wait_stream(s); torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    out = gpu.moe.forward(0, x)
for r in range(4):
    g.replay(); torch.cuda.synchronize()
    cnt = gpu.moe._buf("counts", (4,), torch.int32).tolist()
    cur = gpu.moe._buf("cursor", (4,), torch.int32).tolist()
    print("replay", r, "err", (out - ref).abs().max().item(), "counts", cnt, "cursor", cur, flush=True)
