"""R4: rank 0 -> TP workers step-metadata plane.

Rank 0 runs the scheduler; each step it sends one int32 message -- the step header plus the packed
metadata buffer of :class:`~symmetry_amd.engine.model_runner.ModelRunner` -- and every worker enqueues
the same step on its own GPU.

* :class:`ShmMetaPlane` (default): the native shared-memory ring of ``csrc/runtime/meta_ring.cpp``.  One
  memcpy + release store on rank 0, a polled acquire on the workers: rank 0 never waits for a worker's
  host (unless one falls a whole ring behind), so workers enqueue step N+1 while their GPU still runs
  step N -- the pipelined TP decode loop.  All ranks of a provider share one node (xGMI), so shared
  memory reaches every worker.
* :class:`GlooMetaPlane`: two gloo broadcasts per step (``SYMMETRY_META=gloo``, or when the native
  runtime is not built) -- the round-2 plane, kept for A/B and as the portable fallback.
"""
from __future__ import annotations

import os
import uuid

import numpy as np
import torch
import torch.distributed as dist


class MetaPlane:
    def send(self, header: np.ndarray, payload: np.ndarray | None) -> None:
        raise NotImplementedError

    def recv(self):
        """Workers: (header int32 [H], payload int32 [n]) of the next step, or None once rank 0 closed."""
        raise NotImplementedError

    def close(self) -> None:
        pass

    def faults(self) -> list:
        """Rank 0: [(worker rank, code)] of workers that reported a failure (code > 0) or whose process is
        gone (code -1).  The gloo plane has no back-channel: its broadcasts raise on a dead peer instead."""
        return []

    def report(self, code: int) -> None:
        """Worker: tell rank 0 this rank failed (before it exits)."""


class GlooMetaPlane(MetaPlane):
    def __init__(self, group, header_len: int):
        self.group, self.header_len = group, header_len

    def send(self, header, payload):
        n = 0 if payload is None else int(payload.size)
        h = torch.from_numpy(np.concatenate([header, [n]]).astype(np.int32))
        dist.broadcast(h, src=0, group=self.group)
        if n:
            dist.broadcast(torch.from_numpy(np.ascontiguousarray(payload, dtype=np.int32)), src=0, group=self.group)

    def recv(self):
        h = torch.zeros(self.header_len + 1, dtype=torch.int32)
        dist.broadcast(h, src=0, group=self.group)
        n = int(h[-1])
        buf = torch.zeros(n, dtype=torch.int32)
        if n:
            dist.broadcast(buf, src=0, group=self.group)
        return h[:-1].numpy(), buf.numpy()


class ShmMetaPlane(MetaPlane):
    """Shared-memory ring; created by rank 0, opened by ranks 1..world-1 (reader index rank - 1)."""

    def __init__(self, group, rank: int, world: int, header_len: int, slot_bytes: int, nslots: int = 16):
        from ..runtime import _runtime

        self.rank, self.header_len = rank, header_len
        name = [None]
        if rank == 0:
            name[0] = f"/symm-meta-{os.getpid()}-{uuid.uuid4().hex[:10]}"
            self.ring = _runtime.MetaRing(name[0], int(slot_bytes), int(nslots), world - 1, True)
        dist.broadcast_object_list(name, src=0, group=group)
        if rank != 0:
            self.ring = _runtime.MetaRing(name[0], 0, 0, world - 1, False)
        dist.barrier(group=group)
        if rank == 0:
            self.ring.unlink()  # every rank has it mapped: no name left behind in /dev/shm
        # liveness back-channel: rank 0 polls the workers' pids / error words (faults()), workers rank 0's pid
        self.ring.register_pid(rank - 1, os.getpid())
        dist.barrier(group=group)
        self._buf = np.zeros(1024, dtype=np.int32)

    def send(self, header, payload):
        n = 0 if payload is None else int(payload.size)
        need = self.header_len + n
        if self._buf.size < need:
            self._buf = np.zeros(max(need, 2 * self._buf.size), dtype=np.int32)
        msg = self._buf[:need]
        msg[:self.header_len] = header
        if n:
            msg[self.header_len:] = payload
        self.ring.push(msg)

    def recv(self):
        msg = self.ring.pop(self.rank - 1)
        if msg is None:
            return None
        return msg[:self.header_len], msg[self.header_len:]

    def close(self):
        if self.rank == 0:
            self.ring.shut()

    def faults(self):
        return [(int(r) + 1, int(c)) for r, c in self.ring.faults()]

    def report(self, code: int) -> None:
        if self.rank > 0:
            self.ring.report(self.rank - 1, int(code) or 1)


def make_metaplane(group, rank: int, world: int, header_len: int, slot_bytes: int) -> MetaPlane:
    """Every rank must pick the same plane: the shm ring only if all ranks can load the native runtime."""
    ok = os.environ.get("SYMMETRY_META", "shm").lower() != "gloo"
    if ok:
        try:
            from ..runtime import _runtime  # noqa: F401
        except ImportError:
            ok = False
    flag = torch.tensor([int(ok)], dtype=torch.int32)
    dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=group)
    if int(flag[0]):
        return ShmMetaPlane(group, rank, world, header_len, slot_bytes)
    return GlooMetaPlane(group, header_len)
