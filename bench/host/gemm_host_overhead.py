"""Host cost of enqueueing the prefill projections' library GEMMs (torch.matmul / the split-K bmm) vs a trivial
op: the GPU runs far behind (each GEMM is 30-150 us), so the loop's wall time is the host's enqueue cost.

  python bench/host/gemm_host_overhead.py
"""
import json
import time

import torch


def host_us(fn, n=40):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    return (t1 - t0) / n * 1e6


def main():
    dev = torch.device("cuda")
    M = 768
    x = torch.randn(M, 4096, device=dev).bfloat16()
    tiny = torch.zeros(64, device=dev)
    print(json.dumps({"op": "tiny add_", "host_us": round(host_us(lambda: tiny.add_(1.0)), 2)}))
    for name, N, K in (("qkv", 6144, 4096), ("o", 4096, 4096), ("gate_up", 28672, 4096), ("down", 4096, 14336)):
        w = torch.randn(N, K, device=dev).bfloat16()
        xx = x if K == 4096 else torch.randn(M, K, device=dev).bfloat16()
        out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        print(json.dumps({"op": f"matmul {name}", "host_us": round(host_us(lambda: torch.matmul(xx, w.t(), out=out)), 2)}))
        S = 2
        kc = K // S
        y = torch.empty(S, M, N, device=dev)
        f = lambda: torch.bmm(xx.view(M, S, kc).permute(1, 0, 2), w.view(N, S, kc).permute(1, 2, 0),  # noqa: E731
                              out_dtype=torch.float32, out=y)
        print(json.dumps({"op": f"bmm split-K {name}", "host_us": round(host_us(f), 2)}))
        del w, out, y


if __name__ == "__main__":
    main()
