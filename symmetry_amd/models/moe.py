"""Mixtral sparse-MoE block (K10-K12) with expert parallelism (R3).

Routing, permutation into expert segments, the per-expert GEMMs and the
weighted combine run as HIP kernels (``csrc/kernels/moe.hip``); small routed
batches (<= 64 rows: every decode step) use the grouped skinny MFMA GEMM,
which reads the segment bounds from device memory -- no host sync, so the
decode step stays hipGraph-capturable.  Larger (prefill) batches read the
segment offsets once and run one library GEMM per expert.

Expert parallelism, ``ep_size = N`` ranks each owning ``E/N`` experts:

* ``mode="allreduce"`` (with tensor-parallel attention: every rank holds the
  same tokens) -- each rank applies only its own experts to all routed rows
  and the partial outputs are summed with one all-reduce (graph-capturable);
* ``mode="a2a"`` (with data-parallel attention: ranks hold different tokens)
  -- tokens are dispatched to the ranks owning their experts and the results
  combined back with two all-to-all exchanges over RCCL (``Comm.all_to_all_rows``).
"""
from __future__ import annotations

import torch

from .. import ops

SKINNY_ROWS = 64


class MoEBlock:
    def __init__(self, model, ep_comm=None, mode: str = "allreduce"):
        self.m = model
        cfg = model.cfg
        shard = model.w.shard
        self.E, self.k = cfg.num_experts, cfg.top_k
        self.ep, self.ep_rank = shard.ep_size, shard.ep_rank
        self.E_local = self.E // self.ep
        self.e_lo = self.ep_rank * self.E_local
        self.e_hi = self.e_lo + self.E_local
        self.comm = ep_comm if ep_comm is not None else model.tp
        self.mode = mode
        self.F = cfg.intermediate_size
        # router rows padded to a multiple of 16 for the skinny GEMM (padded logits are never read)
        self.router = {}
        Ep = (self.E + 15) // 16 * 16
        for i in range(cfg.num_layers):
            r = model.w.layer(i, "router")
            pad = torch.zeros(Ep, r.shape[1], dtype=r.dtype, device=r.device)
            pad[: self.E] = r
            self.router[i] = pad

    def _buf(self, name, shape, dtype):
        return self.m._buf("moe." + name, shape, dtype)

    def forward(self, i: int, x: torch.Tensor) -> torch.Tensor:
        if self.ep > 1 and self.mode == "a2a":
            return self.forward_a2a(i, x)
        return self._forward_local(i, x, reduce=self.ep > 1)

    # ------------------------------------------------------------------------------------------
    def _route(self, i, x):
        T, d = x.shape
        k, E = self.k, self.E
        R = T * k
        logits = self.m._linear("router", x, self.router[i])
        ids = self._buf("ids", (R,), torch.int32)
        w = self._buf("w", (R,), torch.float32)
        dst = self._buf("dst", (R,), torch.int32)
        counts = self._buf("counts", (E,), torch.int32)
        offsets = self._buf("offsets", (E + 1,), torch.int32)
        cursor = self._buf("cursor", (E,), torch.int32)
        xs = self._buf("xs", (R, d), torch.bfloat16)
        ops.moe_route_permute(logits, x, k, E, ids, w, counts, offsets, cursor, xs, dst)
        return ids, w, dst, offsets, xs

    def _experts(self, i, xs, offsets, e_lo, n_local):
        """Apply experts [e_lo, e_lo + n_local) to their segments of xs; returns a LinOut [.., R, d]."""
        R, d = xs.shape
        w13 = self.m.w.layer(i, "w13")
        w2 = self.m.w.layer(i, "w2")
        F = self.F
        act = self._buf("act", (R, F), torch.bfloat16)
        if R <= SKINNY_ROWS:
            s1 = ops.choose_splits(2 * F, d)
            y1 = self._buf("y1", (s1, R, 2 * F), torch.float32)
            ops.grouped_skinny(xs, w13, offsets, e_lo, y1)
            ops.swiglu(y1, act)
            s2 = ops.choose_splits(d, F)
            y2 = self._buf("y2", (s2, R, d), torch.float32)
            ops.grouped_skinny(act, w2, offsets, e_lo, y2)
            return y2
        offs = offsets.tolist()
        y1 = self._buf("y1b", (R, 2 * F), torch.bfloat16)
        y2 = self._buf("y2b", (R, d), torch.bfloat16)
        for e in range(n_local):
            a, b = offs[e_lo + e], offs[e_lo + e + 1]
            if b > a:
                ops.linear(xs[a:b], w13[e], out=y1[a:b])
        ops.swiglu(y1, act)
        for e in range(n_local):
            a, b = offs[e_lo + e], offs[e_lo + e + 1]
            if b > a:
                ops.linear(act[a:b], w2[e], out=y2[a:b])
        return y2

    def _forward_local(self, i, x, reduce: bool) -> torch.Tensor:
        T, d = x.shape
        ids, w, dst, offsets, xs = self._route(i, x)
        y2 = self._experts(i, xs, offsets, self.e_lo, self.E_local)
        out = self._buf("out", (T, d), torch.float32)
        ops.moe_combine(y2, dst, ids, self.e_lo, self.e_hi, w, self.k, out)
        if reduce:
            self.comm.all_reduce(out)
        return out

    # ------------------------------------------------------------------------------------------
    def forward_a2a(self, i: int, x: torch.Tensor) -> torch.Tensor:
        """Dispatch/combine over all-to-all.  x holds THIS rank's tokens (data-parallel attention)."""
        T, d = x.shape
        k, ep = self.k, self.ep
        ids, w, dst, offsets, xs = self._route(i, x)
        R = T * k
        # xs rows are grouped by expert == grouped by owner rank (owners own contiguous expert ranges)
        offs = offsets.to("cpu", torch.int64)
        bounds = [int(offs[r * self.E_local]) for r in range(ep)] + [R]
        send_counts = [bounds[r + 1] - bounds[r] for r in range(ep)]
        cnt = torch.tensor(send_counts, dtype=torch.int64, device=x.device).view(ep, 1)
        recv_cnt = self.comm.all_to_all_rows(cnt, [1] * ep, [1] * ep).view(-1).tolist()
        # expert id of every sent row (rows of xs are sorted by expert)
        row_expert = torch.repeat_interleave(torch.arange(self.E, device=x.device),
                                             (offs[1:] - offs[:-1]).to(x.device))
        x_recv = self.comm.all_to_all_rows(xs[:R], send_counts, recv_cnt)
        e_recv = self.comm.all_to_all_rows(row_expert.view(-1, 1).to(torch.int64), send_counts, recv_cnt).view(-1)
        # local expert segments of the received rows (stable sort keeps per-source order)
        order = torch.argsort(e_recv, stable=True)
        xr = x_recv.index_select(0, order).contiguous()
        local = e_recv.index_select(0, order) - self.e_lo
        cnt_local = torch.bincount(local, minlength=self.E_local)[: self.E_local]
        loc_off = torch.zeros(self.E + 1, dtype=torch.int32, device=x.device)
        loc_off[self.e_lo + 1 : self.e_lo + self.E_local + 1] = torch.cumsum(cnt_local, 0).to(torch.int32)
        loc_off[self.e_lo + self.E_local + 1 :] = loc_off[self.e_lo + self.E_local]
        yl = self._experts(i, xr, loc_off, self.e_lo, self.E_local)
        ylf = ops.reference.linout_sum(yl) if yl.dim() == 3 else yl.float()
        y_sorted_back = torch.empty_like(ylf)
        y_sorted_back[order] = ylf  # undo the local sort: rows back in received order
        y_back = self.comm.all_to_all_rows(y_sorted_back.contiguous(), recv_cnt, send_counts)
        out = self._buf("out", (T, d), torch.float32)
        ops.moe_combine(y_back, dst, ids, 0, self.E, w, k, out)
        return out
