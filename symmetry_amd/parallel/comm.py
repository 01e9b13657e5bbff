"""Collective communication for tensor / expert parallelism (R1-R4).

Two interchangeable implementations of one small interface
(``all_reduce``, ``all_gather``, ``all_to_all_rows``, ``broadcast``):

* :class:`RcclComm` -- our C++ RCCL communicator (``csrc/bindings/rccl_comm.cpp``),
  collectives enqueued on torch's current HIP stream so they are captured
  into the decode hipGraph; rides xGMI on an MI355X node.
* :class:`TorchComm` -- ``torch.distributed`` on a process group (gloo on the
  CPU for the multi-process tests; RCCL through c10d on GPUs).
* :class:`XgmiComm` -- wraps one of the above: all-reduces that fit its slot
  (decode-sized) run as ONE one-shot kernel over xGMI peer memory
  (``csrc/kernels/xgmi_ar.hip``: every rank writes its partial into every
  peer's buffer, seven links at once, one hop), optionally fused with the
  residual add + next-norm prep of the row-parallel projections; everything
  else goes to the wrapped communicator.
* :class:`HostStagedComm` -- GPU tensors reduced through a gloo group on the
  host.  Not a fast path: it lets several ranks share ONE GPU (RCCL refuses
  duplicate devices), so the sharded HIP kernels of a TP/EP launch can be
  checked on a one-GPU box (``SYMMETRY_TP_COMM=gloo``; eager steps only).

xGMI is point-to-point (7 links x ~153 GB/s per GPU), so the per-layer
decode all-reduce (16 KiB x batch for 70B) is latency-bound: the model
issues exactly two per layer and keeps them inside the captured graph.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist


# Row-parallel decode projections under TP run GEMM + all-reduce + residual epilogue as ONE launch
# (XgmiComm.gemm_ar_resid); SYMMETRY_XGMI_FUSED=0 restores GEMM + the fused all-reduce / add_prep launch (A/B)
XAR = os.environ.get("SYMMETRY_XGMI_FUSED", "1") != "0"


class Comm:
    rank: int = 0
    world: int = 1
    capturable: bool = False  # every collective enqueues on the current HIP stream (hipGraph capture)

    def all_reduce(self, t: torch.Tensor, op: str = "sum") -> None:
        raise NotImplementedError

    def all_gather(self, t: torch.Tensor) -> torch.Tensor:
        raise NotImplementedError

    def all_to_all_rows(self, send: torch.Tensor, send_counts: list[int], recv_counts: list[int]) -> torch.Tensor:
        raise NotImplementedError

    def broadcast(self, t: torch.Tensor, src: int = 0) -> None:
        raise NotImplementedError

    def argmax_keys(self, keys: torch.Tensor, ids: torch.Tensor) -> None:
        """Vocab-parallel sampling combine: keys int64 [B] hold each rank's packed u64 (order-preserving
        value | inverted index) maxima; ids[:B] = the index of the global max.  Fused on XgmiComm."""
        sign = -(1 << 63)
        keys.bitwise_xor_(sign)  # signed MAX == unsigned max once the sign bit is flipped
        self.all_reduce(keys, op="max")
        keys.bitwise_xor_(sign)
        ids[: keys.numel()].copy_((0xFFFFFFFF - (keys & 0xFFFFFFFF)).to(torch.int32))

    def all_reduce_add_prep(self, y, resid, w_next, xw, ss) -> None:
        """resid += all_reduce(y); xw = bf16(resid * w_next); ss = row sums of resid^2 (decode epilogue
        of a row-parallel projection, ``ops.add_prep``).  Fused into the collective by XgmiComm."""
        from .. import ops

        self.all_reduce(y)
        ops.add_prep(y, resid, w_next, xw, ss)


_OPS = {"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX, "min": dist.ReduceOp.MIN}


class TorchComm(Comm):
    def __init__(self, group=None):
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)

    def all_reduce(self, t, op="sum"):
        dist.all_reduce(t, op=_OPS[op], group=self.group)

    def all_gather(self, t):
        out = [torch.empty_like(t) for _ in range(self.world)]
        dist.all_gather(out, t.contiguous(), group=self.group)
        return torch.cat(out, 0)

    def all_to_all_rows(self, send, send_counts, recv_counts):
        recv = send.new_empty((sum(recv_counts),) + tuple(send.shape[1:]))
        dist.all_to_all_single(recv, send.contiguous(), output_split_sizes=list(recv_counts),
                               input_split_sizes=list(send_counts), group=self.group)
        return recv

    def broadcast(self, t, src=0):
        dist.broadcast(t, src=src, group=self.group)


class HostStagedComm(Comm):
    """Collectives on device tensors via host copies and a gloo group (see module docstring)."""

    def __init__(self, group=None):
        self.inner = TorchComm(group)
        self.rank, self.world = self.inner.rank, self.inner.world

    def all_reduce(self, t, op="sum"):
        h = t.detach().cpu()
        self.inner.all_reduce(h, op)
        t.copy_(h)

    def all_gather(self, t):
        return self.inner.all_gather(t.detach().cpu()).to(t.device)

    def all_to_all_rows(self, send, send_counts, recv_counts):
        return self.inner.all_to_all_rows(send.detach().cpu(), send_counts, recv_counts).to(send.device)

    def broadcast(self, t, src=0):
        h = t.detach().cpu()
        self.inner.broadcast(h, src)
        t.copy_(h)


class RcclComm(Comm):
    """Graph-capturable RCCL communicator over the ranks of ``group`` (bootstrapped through it)."""

    capturable = True

    def __init__(self, group=None, bootstrap_group=None):
        from ..ops import _native

        self.ops = _native.ops()
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        boot = bootstrap_group if bootstrap_group is not None else group
        if self.rank == 0:
            uid = self.ops.rccl_unique_id()
        else:
            uid = torch.zeros(128, dtype=torch.uint8)
        if uid.numel() != 128:
            buf = torch.zeros(max(128, uid.numel()), dtype=torch.uint8)
            buf[: uid.numel()] = uid
            uid = buf
        dist.broadcast(uid, src=dist.get_global_rank(boot, 0) if boot is not None else 0, group=boot)
        self.handle = int(self.ops.rccl_init(uid[:128].contiguous(), self.world, self.rank))

    def all_reduce(self, t, op="sum"):
        self.ops.rccl_all_reduce(t, self.handle, op)

    def all_gather(self, t):
        out = t.new_empty((self.world,) + tuple(t.shape))
        self.ops.rccl_all_gather(t.contiguous(), out, self.handle)
        return out.reshape((self.world * t.shape[0],) + tuple(t.shape[1:])) if t.dim() else out

    def all_to_all_rows(self, send, send_counts, recv_counts):
        row = int(send[0].numel()) if send.shape[0] else int(torch.tensor(send.shape[1:]).prod())
        recv = send.new_empty((sum(recv_counts),) + tuple(send.shape[1:]))
        self.ops.rccl_all_to_all(send.contiguous(), recv, list(send_counts), list(recv_counts), row, self.handle)
        return recv

    def broadcast(self, t, src=0):
        self.ops.rccl_broadcast(t, src, self.handle)

    def destroy(self):
        self.ops.rccl_destroy(self.handle)


class XgmiComm(Comm):
    """One-shot all-reduce over xGMI peer memory for decode-sized messages (see module docstring).

    Every rank allocates one uncached buffer (flags + 2 x world slots of ``slot_bytes``), the IPC handles
    are all-gathered over ``group`` (gloo) and every peer buffer is mapped (``hipIpcOpenMemHandle``).
    Messages larger than a slot, non-sum ops and other dtypes go to ``inner`` (RCCL)."""

    def __init__(self, inner: Comm, group, device, slot_bytes: int = 4 << 20, barrier: bool = True):
        from ..ops import _native

        self.ops = _native.ops()
        self.inner = inner
        self.rank, self.world = inner.rank, inner.world
        self.capturable = inner.capturable  # the xGMI kernels are; the fallbacks are the inner ones
        dev = torch.device(device)
        self.slot_bytes = int(slot_bytes)
        # largest message on the one-shot kernels; ranks sharing one GPU (rehearsals) keep it to decode sizes: a
        # prefill-sized collective's grid (up to 4096 spinning workgroups) can fill the device before the other
        # rank's kernel starts, so neither makes progress until the wait limit
        self.oneshot_bytes = self.slot_bytes
        if torch.cuda.device_count() < self.world:
            self.oneshot_bytes = min(self.slot_bytes, 256 << 10)
        self.calls = {"all_reduce": 0, "add_prep": 0}  # collectives issued on the xGMI kernels (host count)
        self.xar = None  # the fused row-parallel GEMM + all-reduce communicator (attach_xar)
        self.a2a = None  # the expert all-to-all communicator (attach_a2a)
        try:
            self.handle = int(self.ops.xgmi_create(int(slot_bytes), self.world, self.rank, dev.index or 0))
            mine = self.ops.xgmi_ipc_handle(self.handle)
        except Exception:  # noqa: BLE001 -- still take part in the exchange below, then fail
            mine = None
            if not hasattr(self, "handle"):
                self.handle = None
        ref = mine if mine is not None else torch.zeros(64, dtype=torch.uint8)
        allh = [torch.zeros_like(ref) for _ in range(self.world)]
        dist.all_gather(allh, ref, group=group)  # every rank takes part, even one that failed to export
        if mine is None:
            raise RuntimeError("xgmi: hipIpcGetMemHandle failed")
        self.ops.xgmi_open(self.handle, torch.stack(allh))
        if barrier:
            dist.barrier(group=group)  # every rank mapped every buffer before the first collective

    def self_test(self) -> bool:
        """One all-reduce of known values through the peer buffers (every rank, collectively): True when it
        summed correctly and no rank gave up waiting.  Run once at startup, so a node whose links or IPC
        mappings misbehave falls back to RCCL instead of failing its first decode step."""
        dev = torch.device("cuda", torch.cuda.current_device())
        t = torch.full((4096,), float(self.rank + 1), device=dev)
        self.ops.xgmi_all_reduce(t, t, self.handle)
        torch.cuda.synchronize(dev)
        want = self.world * (self.world + 1) / 2
        return int(self.ops.xgmi_error(self.handle)) == 0 and bool((t == want).all())

    def xar_self_test(self, d: int, ks=(256,), rows=(4,), layouts=(False,)) -> bool:
        """The fused row-parallel projection + all-reduce + residual launch on exactly representable data
        (x = 1, W = (rank + 1) / 256, residual 0.5) for every (K, M, layout) given -- the production shapes (the
        row-parallel K of o and down, M = 1 and 16, row-major and preshuffled: a constant matrix is its own
        preshuffle) reach the launch variants the decode step will pick.  True when every row came back as
        0.5 + K / 256 * sum of (rank + 1), every launch fit (co-resident grid) and no rank gave up waiting."""
        dev = torch.device("cuda", torch.cuda.current_device())
        w_next = torch.ones(d, device=dev, dtype=torch.bfloat16)
        for K in ks:
            W = torch.full((d, K), (self.rank + 1) / 256, device=dev, dtype=torch.bfloat16)
            for M in rows:
                for wshuf in layouts:
                    x = torch.ones(M, K, device=dev, dtype=torch.bfloat16)
                    resid = torch.full((M, d), 0.5, device=dev)
                    xw = torch.empty(M, d, device=dev, dtype=torch.bfloat16)
                    ss = torch.empty(M, d // 16, device=dev)
                    if not self.gemm_ar_resid(x, W, wshuf, resid, w_next, xw, ss):
                        return False
                    torch.cuda.synchronize(dev)
                    self.calls["gemm_ar"] -= 1
                    want = 0.5 + K / 256 * self.world * (self.world + 1) / 2
                    if int(self.ops.xgmi_error(self.xar.handle)) != 0 or not bool((resid == want).all()):
                        return False
        return True

    def _fits(self, t) -> bool:
        return (t.is_cuda and t.dtype in (torch.float32, torch.bfloat16) and t.is_contiguous()
                and t.numel() % 8 == 0 and t.numel() * t.element_size() <= self.oneshot_bytes)

    def all_reduce(self, t, op="sum"):
        if op == "sum" and self._fits(t):
            self.ops.xgmi_all_reduce(t, t, self.handle)
            self.calls["all_reduce"] += 1
        else:
            self.inner.all_reduce(t, op)

    def all_reduce_add_prep(self, y, resid, w_next, xw, ss):
        if y.dtype == torch.float32 and self._fits(y) and y.numel() == resid.numel():
            self.ops.xgmi_add_prep(y, resid, w_next, xw, ss, self.handle)
            self.calls["add_prep"] += 1
        else:
            super().all_reduce_add_prep(y, resid, w_next, xw, ss)

    # ---- R3: unpadded expert all-to-all on a second peer-memory communicator ------------------------------
    def attach_a2a(self, group, cap: int, row_bytes: int) -> None:
        """Collective (every rank): a second xGMI communicator whose slots hold ``cap`` rows of up to
        ``row_bytes`` each (+ counts and side ints) for :meth:`a2a_rows`.  Mixtral prefill: cap = ceil(max
        tokens / N) * top_k rows, row_bytes = d * 4 (the fp32 return) -- ~0.5 GB of uncached HBM per rank."""
        slot = (int(self.ops.xgmi_a2a_slot(int(cap), int(row_bytes))) + 255) // 256 * 256
        self.a2a = XgmiComm(self.inner, group, torch.device("cuda", torch.cuda.current_device()), slot_bytes=slot,
                            barrier=False)  # the caller votes, then barriers (parallel/launch.py)
        self.a2a_cap, self.a2a_row_bytes = int(cap), int(row_bytes)
        self.calls["a2a"] = 0

    def a2a_fits(self, cap: int, row_bytes: int) -> bool:
        return self.a2a is not None and cap <= self.a2a_cap and row_bytes <= self.a2a_row_bytes

    def a2a_rows(self, src, counts, side, dst, dst_side=None, dst_counts=None) -> None:
        """Block q of ``src`` ([world * cap, ...] rows; its first ``counts[q]`` -- a DEVICE int32 [world] -- are
        real) becomes block ``rank`` of rank q's ``dst``; only real rows cross the links, no host sync."""
        cap = src.shape[0] // self.world
        self.ops.xgmi_a2a(src, counts, side, dst, dst_side, dst_counts, cap, self.a2a.handle)
        self.calls["a2a"] += 1

    def attach_xar(self, group, rows: int, d: int) -> None:
        """Collective (every rank): the communicator of the fused row-parallel decode projections -- slots of
        ``rows`` x ``d`` epoch-tagged 8-B granules (csrc/kernels/decode_epi.h, xar_push / xar_collect)."""
        self.xar = XgmiComm(self.inner, group, torch.device("cuda", torch.cuda.current_device()),
                            slot_bytes=(int(rows) * int(d) * 8 + 255) // 256 * 256, barrier=False)

    def gemm_ar_resid(self, x, W, wshuf, resid, w_next, xw, ss) -> bool:
        """Row-parallel decode projection + all-reduce + residual add + next-norm prep as ONE launch
        (``DECODE_EPI_XAR``): ``ss`` gets one sum-of-squares partial per 16 columns ([M, d / 16], the layout
        the single-GPU dg_resid writes).  False: shapes or occupancy do not fit (the caller runs GEMM +
        ``all_reduce_add_prep``)."""
        if not XAR or self.xar is None or not x.is_cuda or x.shape[0] > 64 or W.shape[0] % 16 or x.shape[1] % 256:
            return False
        if x.shape[0] * resid.shape[1] * 8 > self.xar.slot_bytes or ss.shape[1] != W.shape[0] // 16:
            return False
        ok = bool(self.ops.xgmi_gemm_ar_resid(x, W, bool(wshuf), resid, w_next, xw, ss, self.xar.handle))
        if ok:
            self.calls["gemm_ar"] = self.calls.get("gemm_ar", 0) + 1
        return ok

    def argmax_keys(self, keys, ids):
        if keys.is_cuda and keys.is_contiguous() and keys.numel() <= 4096:
            self.ops.xgmi_keys_max(keys, ids, self.handle)
            self.calls["keys"] = self.calls.get("keys", 0) + 1
        else:
            super().argmax_keys(keys, ids)

    def all_gather(self, t):
        return self.inner.all_gather(t)

    def all_to_all_rows(self, send, send_counts, recv_counts):
        return self.inner.all_to_all_rows(send, send_counts, recv_counts)

    def broadcast(self, t, src=0):
        self.inner.broadcast(t, src)

    def error(self) -> int:
        """1 + the source rank a collective gave up waiting for (or the code the host declared), else 0.  Sticky
        (the communicator stays failed); host-mapped, so it costs no device synchronisation: the model runner
        polls it after every step.  Covers the all-to-all communicator too."""
        e = int(self.ops.xgmi_error(self.handle))
        for sub in (self.xar, self.a2a):
            if not e and sub is not None:
                e = int(self.ops.xgmi_error(sub.handle))
        return e

    def set_error(self, code: int) -> None:
        """Declare a fault from the host (rank 0's health monitor): every spinning collective stops waiting."""
        self.ops.xgmi_set_error(self.handle, int(code))
        for sub in (self.xar, self.a2a):
            if sub is not None:
                self.ops.xgmi_set_error(sub.handle, int(code))

    def destroy(self, inner_too: bool = True):
        for name in ("xar", "a2a"):
            sub = getattr(self, name, None)
            if sub is not None:
                sub.destroy(inner_too=False)
                setattr(self, name, None)
        if self.handle is not None:
            self.ops.xgmi_destroy(self.handle)
        if inner_too and hasattr(self.inner, "destroy"):
            self.inner.destroy()
