"""Probe: can two processes on ONE GPU share device memory through HIP IPC (torch CUDA-tensor sharing)?"""
import torch
import torch.multiprocessing as mp


def child(q, r):
    t = q.get()
    t.add_(1.0)
    torch.cuda.synchronize()
    r.put(float(t.sum()))


if __name__ == "__main__":
    mp.set_start_method("spawn")
    q, r = mp.Queue(), mp.Queue()
    x = torch.zeros(1024, device="cuda")
    p = mp.Process(target=child, args=(q, r))
    p.start()
    q.put(x)
    print("child sum", r.get(timeout=60))
    p.join(timeout=60)
    torch.cuda.synchronize()
    print("parent sum", float(x.sum()))
