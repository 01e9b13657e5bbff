"""Numerics check of the decode GEMM variants (dg_f32) against an fp32 torch reference at 17..64 rows."""
import torch, json
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from symmetry_amd import ops
from symmetry_amd.ops import _native
lib = _native.ops()
dev = torch.device("cuda")
for (N, K) in [(6144, 4096), (4096, 4096), (28672, 4096), (4096, 14336)]:
    W = (torch.randn(N, K, device=dev) * 0.02).bfloat16()
    for M in [17, 33, 64]:
        x = torch.randn(M, K, device=dev).bfloat16()
        ref = x.float() @ W.float().t()
        for v in [12, 13, 14, 15, 16]:
            lib.decode_gemm_variant(v)
            y = torch.full((M, N), float("nan"), device=dev)
            ops.dg_f32(x, W, None, 0.0, y)
            torch.cuda.synchronize()
            err = float((y - ref).abs().max())
            print(json.dumps({"N": N, "K": K, "M": M, "v": v, "err": err}), flush=True)
            assert err < 1e-2, err
lib.decode_gemm_variant(-1)
print("OK")
