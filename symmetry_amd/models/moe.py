"""Mixtral sparse-MoE block (K10-K12) with expert parallelism (R3).

Routing, permutation into expert segments, the per-expert GEMMs and the weighted combine run as HIP
kernels (``csrc/kernels/moe.hip``) whose segment bounds live in device memory: no host sync anywhere in
the block, so every step (decode and prefill, with or without expert parallelism) is hipGraph-capturable.
Small routed batches (<= 64 rows: decode steps) use the grouped skinny MFMA GEMM or the weight-streaming kernel;
prefill-sized ones the prefill GEMM kernel in grouped mode (``ops.pg_grouped``, csrc/kernels/pgemm.hip) or, below
its row thresholds, the weight-streaming / 128 x 128 tile grouped GEMMs (``ops.grouped_gemm``), SwiGLU fused into
the gate/up epilogue everywhere.

Expert parallelism, ``ep_size = N`` ranks each owning ``E / N`` experts (attention is tensor-parallel, so
every rank holds the same T tokens when the block starts):

* all-reduce combine (``mode="allreduce"``, and ``"auto"`` below ``A2A_ROWS`` rows -- the default): each
  rank applies its own experts to all routed rows and one all-reduce sums the partial outputs (on the
  one-shot xGMI kernel at decode sizes);
* owner exchange (``mode="a2a"``, and ``"auto"`` from ``A2A_ROWS`` rows -- opt-in; :meth:`forward_a2a`):
  no dispatch leg (every rank already holds the tokens) -- every rank routes all T tokens and runs its own
  experts on its own routed rows; per token with a local expert ONE fp32 row (the weighted partial over those
  experts) goes to the token's slice owner (``XgmiComm.a2a_rows``: only counted rows cross the links, counts
  on the device); the owners sum in rank order and a bf16 all-gather rebuilds [T, d].  Elsewhere (RCCL / gloo)
  whole capacity blocks move, empty slots marked -1.
* :meth:`MoEBlock.forward_tokens` is the exchange for ranks that hold DIFFERENT tokens (data-parallel attention
  in front of expert-parallel MoE): dispatch of routed rows to their owners, expert GEMMs, return, combine.
"""
from __future__ import annotations

import os

import torch

from .. import ops

SKINNY_ROWS = 64
# mean routed rows per expert up to which prefill takes the weight-streaming grouped GEMM on the preshuffled expert
# copies (bench/kernels/bench_grouped.py, profiles/r5/grouped_stream.jsonl: at 64 rows w13 469 -> 358 us, w2 300 ->
# 165; from ~128 rows the tile kernel is as fast on w13, and on w2 once uneven routing spills segments past the
# 256-row unit: Mixtral 4 x 128-token prefill w2 324 vs 318 us, profiles/r5/prof_mixtral_prefill_4x128_stream.csv)
PRE_ROWS = int(os.environ.get("SYMMETRY_MOE_PRE_ROWS", "100"))
# gate/up (+ SwiGLU) streams further: 128-row units with 4 weight tiles per wave, longer segments in two units
# (w13 at 128 rows per expert 468 vs 598-614 us on the tile kernel, at 160 rows 619-650 vs 673-707)
PRE_ROWS_W13 = int(os.environ.get("SYMMETRY_MOE_PRE_ROWS_W13", "176"))
# mean routed rows per local expert from which prefill runs an expert GEMM on the prefill GEMM kernel's grouped mode
# (ops.pg_grouped) instead of the two kernels above (A/B switch: SYMMETRY_MOE_PG=0).  Mixtral shapes, segments
# 0.4x .. 2.0x the mean (bench/kernels/bench_pg_grouped.py, profiles/r6/pg_grouped_sweep*.jsonl): w2 at 80 rows
# 206 vs 247 us (streaming), at 128 236 vs 350, at 256 336 vs 594 (tile); at 48 / 64 rows streaming keeps a 5-9 %
# lead.  w13 + SwiGLU even at 80-96 rows, 421 vs 475 at 112, 451 vs 474 at 128, 649 vs 889 at 256.
PG_GROUPED = os.environ.get("SYMMETRY_MOE_PG", "1") != "0"
PG_ROWS_W13 = int(os.environ.get("SYMMETRY_MOE_PG_ROWS_W13", "100"))
PG_ROWS_W2 = int(os.environ.get("SYMMETRY_MOE_PG_ROWS_W2", "72"))
# decode steps stream the preshuffled copies from this many routed rows per local expert (every expert routed)
STREAM_DECODE_ROWS = int(os.environ.get("SYMMETRY_MOE_STREAM_DECODE_ROWS", "4"))
# "auto": the owner exchange (forward_a2a) from this many tokens, the fp32 all-reduce combine below.  Off by default:
# the one-GPU rehearsal (bench/ep_rehearsal.py, profiles/r6/ep_crossover.jsonl) found no crossover up to 1024 tokens
# at 2 and 4 ranks -- the exchange moves 35-51 % fewer bytes per rank (world 4, 1024 tokens: 12.2 vs 25.2 MB per
# layer) but costs three collectives and a counts readback per layer against one all-reduce (TTFT 1016 vs 299 ms at
# world 2 on the shared GPU's host-staged transport); a node with one GPU per rank and the peer-memory exchange
# kernel is the measurement that could set it lower (SYMMETRY_MOE_A2A_ROWS / SYMMETRY_MOE_MODE=a2a)
A2A_ROWS = int(os.environ.get("SYMMETRY_MOE_A2A_ROWS", str(1 << 30)))
GROUPED = os.environ.get("SYMMETRY_MOE_GROUPED", "1") != "0"  # A/B: 0 = per-expert library GEMMs (host sync)
# count the bytes this rank's MoE collectives push (device-side counts are summed lazily: ``a2a_stats()`` syncs
# once per call -- tests / benches read it once per step)
A2A_STATS = os.environ.get("SYMMETRY_MOE_A2A_STATS", "0") == "1"
# decode steps: routing in one launch and the combine fused with the residual prep (A/B: 0 = five routing launches
# + combine + add_prep; profiles/r4/moe_decode_fused.jsonl)
DECODE_FUSED = os.environ.get("SYMMETRY_MOE_DECODE_FUSED", "1") != "0"
# rows up to which the routing runs as the one-workgroup launch: 8.8 vs 12.0 us at 1 row, 12.8 vs 14.0 at 4,
# 17.8 vs 14.1 at 8 (profiles/r4/moe_decode_fused.jsonl)
ROUTE_FUSED_ROWS = int(os.environ.get("SYMMETRY_MOE_ROUTE_FUSED_ROWS", "4"))


class MoEBlock:
    def __init__(self, model, ep_comm=None, mode: str | None = None):
        self.m = model
        cfg = model.cfg
        shard = model.w.shard
        self.E, self.k = cfg.num_experts, cfg.top_k
        self.ep, self.ep_rank = shard.ep_size, shard.ep_rank
        self.E_local = self.E // self.ep
        self.e_lo = self.ep_rank * self.E_local
        self.e_hi = self.e_lo + self.E_local
        self.comm = ep_comm if ep_comm is not None else model.tp
        self.mode = mode or os.environ.get("SYMMETRY_MOE_MODE", "auto")
        self.F = cfg.intermediate_size
        self.calls = {"allreduce": 0, "a2a": 0}
        self.a2a_bytes = {"dispatch": 0, "return": 0, "routed_rows": 0, "padded_dispatch": 0, "gather": 0,
                          "allreduce": 0}
        self._pending = []  # (key, device int64 scalar) byte / row counts not yet read back
        # router rows padded to a multiple of 16 for the skinny GEMM (padded logits are never read)
        self.router = {}
        self.single_copy = False  # adopt_single_copy: the expert tensors themselves are preshuffled
        self.pre = self._preshuffled_copies(model)
        pol = os.environ.get("SYMMETRY_MOE_STREAM_POLICY")  # A/B: grouped_gemm's row-major streaming policy
        if pol is not None and model.device.type == "cuda":
            ops.grouped_stream_policy(int(pol))
        Ep = (self.E + 15) // 16 * 16
        for i in range(cfg.num_layers):
            r = model.w.layer(i, "router")
            pad = torch.zeros(Ep, r.shape[1], dtype=r.dtype, device=r.device)
            pad[: self.E] = r
            self.router[i] = pad

    @staticmethod
    def _preshuffled_copies(model) -> dict:
        """MFMA-preshuffled copies of the expert weights for the weight-streaming grouped GEMM of prefill-sized
        routed batches (csrc/kernels/moe.hip grouped_stream_kernel: fragment loads of 1 KB contiguous; Mixtral at
        64-128 rows per expert: w2 303 -> 153 / 331 -> 212 us, w13 430 -> 352 us, profiles/r5/grouped_stream.jsonl).
        Decode steps stream them too (1-8 rows per expert: w13 320 -> 299 us, w2 162 -> 144).  The row-major
        tensors stay for the tile kernel (long segments), so this is one extra copy: w2 first (the larger win),
        then w13, from the HBM left after the KV cache's need (admission limit x context) and a workspace reserve
        (transformer.copy_budget; Mixtral on one GPU at 64 seqs x 8K: both copies, 90 GB)."""
        mode = os.environ.get("SYMMETRY_MOE_PRESHUFFLE", "auto")
        dev = model.device
        if mode == "0" or dev.type != "cuda" or not GROUPED or getattr(model, "plan_single_copy", False):
            return {}  # (single copy: adopt_single_copy preshuffles the stacks in place instead)
        cfg = model.cfg
        from .transformer import copy_budget

        budget = float("inf") if mode == "1" else copy_budget(dev, getattr(model, "kv_reserve", 0))
        out = {}
        for name in ("w2", "w13"):
            ws = [model.w.layer(i, name) for i in range(cfg.num_layers)]
            E, N, K = ws[0].shape  # the streaming kernel's tiling: <= 8 local experts, K % 256, 128-row n-blocks
            if E > 8 or K % 256 or ((N // 2) % 64 if name == "w13" else N % 128):
                continue
            need = sum(w.numel() * 2 for w in ws)
            if need > budget:
                break
            budget -= need
            for i, w in enumerate(ws):
                E, N, K = w.shape
                out[(i, name)] = w.reshape(E, N // 16, 16, K // 32, 4, 8).permute(0, 1, 3, 4, 2, 5).contiguous().view(E, N, K)
        return out

    def single_copy_ok(self) -> bool:
        """The expert shapes tile for the kernels that read the preshuffled layout (streaming: <= 8 local experts,
        K % 256, 128-row n-blocks; the grouped prefill GEMM: 64-deep k steps)."""
        cfg = self.m.cfg
        d, F = cfg.hidden_size, self.F
        return GROUPED and self.E_local <= 8 and d % 256 == 0 and F % 256 == 0 and F % 64 == 0 and d % 128 == 0

    def adopt_single_copy(self) -> list:
        """decode_weights="replace": the expert weights exist ONLY preshuffled (per expert, models/layout.py) -- an
        existing copy becomes the weight and the row-major tensor is released, else the tensor is preshuffled in
        place.  Every expert GEMM then reads that layout: decode steps the weight-streaming kernel, prefill the
        streaming or the grouped prefill GEMM kernel.  Returns the tensor names now stored preshuffled."""
        from .layout import preshuffle

        w = self.m.w
        keys = []
        for i in range(self.m.cfg.num_layers):
            for name in ("w13", "w2"):
                key = f"layers.{i}.{name}"
                t = self.pre.get((i, name))
                if t is None:
                    t = preshuffle(w.tensors[key])
                w.tensors[key] = t
                self.pre[(i, name)] = t
                keys.append(key)
        self.single_copy = True
        return keys

    def _stat(self, key: str, v) -> None:
        """Add ``v`` (an int, or a device scalar: no sync here) to a2a_bytes[key] when A2A_STATS is on."""
        if A2A_STATS:
            if isinstance(v, torch.Tensor):
                self._pending.append((key, v.to(torch.int64)))
            else:
                self.a2a_bytes[key] += int(v)

    def a2a_stats(self) -> dict:
        """The byte / row counters with every pending device count read back in ONE transfer."""
        if self._pending:
            keys = [k for k, _ in self._pending]
            vals = torch.stack([v.reshape(()) for _, v in self._pending]).tolist()
            for k, v in zip(keys, vals):
                self.a2a_bytes[k] += int(v)
            self._pending = []
        return dict(self.a2a_bytes)

    @staticmethod
    def _block_rows(counts, cap: int, dev) -> torch.Tensor:
        """Row indices of the first counts[q] rows of every cap-row block q."""
        idx = [torch.arange(q * cap, q * cap + int(c)) for q, c in enumerate(counts) if c]
        return (torch.cat(idx) if idx else torch.zeros(0, dtype=torch.int64)).to(dev)

    def _exchange_counted(self, send: torch.Tensor, counts, recv_counts, cap: int, fill=None) -> torch.Tensor:
        """All-to-all of block-laid-out rows on RCCL / gloo with the real counts as splits (all_to_all_single):
        block q of ``send`` ([N * cap, ...]) holds counts[q] real rows for rank q; the result has block s = the
        recv_counts[s] rows rank s sent here, the rest ``fill`` (or unset).  Only real rows cross the links."""
        N, dev = self.ep, send.device
        payload = send.index_select(0, self._block_rows(counts, cap, dev))
        got = self.comm.all_to_all_rows(payload, list(counts), list(recv_counts))
        shape = (N * cap,) + tuple(send.shape[1:])
        recv = torch.empty(shape, dtype=send.dtype, device=dev) if fill is None else \
            torch.full(shape, fill, dtype=send.dtype, device=dev)
        recv.index_copy_(0, self._block_rows(recv_counts, cap, dev), got)
        return recv

    def _counts_exchange(self, cursor: torch.Tensor):
        """(send counts, receive counts) as host lists: the per-peer counts all-to-all (one int each) + ONE
        readback -- the split sizes all_to_all_single needs."""
        N = self.ep
        rc = self.comm.all_to_all_rows(cursor.view(N, 1).contiguous(), [1] * N, [1] * N).view(N)
        both = torch.cat([cursor.view(N).to(rc.device), rc]).tolist()
        return [int(v) for v in both[:N]], [int(v) for v in both[N:]]

    def _buf(self, name, shape, dtype):
        return self.m._buf("moe." + name, shape, dtype)

    def use_a2a(self, T: int) -> bool:
        if self.ep <= 1:
            return False
        return self.mode == "a2a" or (self.mode == "auto" and T >= A2A_ROWS)

    def forward(self, i: int, x: torch.Tensor) -> torch.Tensor:
        if self.use_a2a(x.shape[0]):
            self.calls["a2a"] += 1
            return self.forward_a2a(i, x)
        self.calls["allreduce"] += 1
        return self._forward_local(i, x, reduce=self.ep > 1)

    def decode_fused_ok(self, T: int, d: int) -> bool:
        """The one-launch routing (+ fused combine / residual prep) of a decode step applies."""
        return (DECODE_FUSED and T <= 8 and not self.use_a2a(T) and self.E <= 64 and self.k <= 8 and d % 8 == 0
                and d <= 4096)

    def forward_decode(self, i: int, resid, lnw, eps: float, w_next, xw, ss_1) -> torch.Tensor:
        """A decode step's MoE block straight off the fp32 residual stream: ONE routing launch (RMSNorm + router
        + top-k + segments + permuted rows, ``ops.moe_decode_route``), the grouped expert GEMMs, and the weighted
        combine fused with the residual add + next-norm prep (``ops.moe_combine_prep``); under expert
        parallelism the combine stays separate (its partial sum is all-reduced first).  resid += MoE(RMSNorm(
        resid)); xw and the returned sum-of-squares partials ([T, P]; ``ss_1`` [T, 1] under EP): the next layer's
        deferred-norm inputs."""
        self.calls["allreduce"] += 1
        T, d = resid.shape
        k, E = self.k, self.E
        R = T * k
        ids = self._buf("ids", (R,), torch.int32)
        w = self._buf("w", (R,), torch.float32)
        dst = self._buf("dst", (R,), torch.int32)
        counts = self._buf("counts", (E,), torch.int32)
        offsets = self._buf("offsets", (E + 1,), torch.int32)
        cursor = self._buf("cursor", (E,), torch.int32)
        xs = self._buf("xs", (R, d), torch.bfloat16)
        if T <= ROUTE_FUSED_ROWS:
            ops.moe_decode_route(resid, lnw, eps, self.router[i][:E], k, ids, w, counts, offsets, cursor, xs, dst)
        else:  # the one-workgroup routing launch stops paying off past a few rows (bench_moe_decode.py)
            xn = self._buf("xn", (T, d), torch.bfloat16)
            ops.rms_norm(resid, lnw, eps, xn)
            logits = self._router_logits(i, xn)
            ops.moe_route_permute(logits, xn, k, E, ids, w, counts, offsets, cursor, xs, dst)
        y2 = self._experts(i, xs, offsets, self.e_lo, self.E_local, out_f32=True)
        if self.ep > 1:
            out = self._buf("out", (T, d), torch.float32)
            ops.moe_combine(y2, dst, ids, self.e_lo, self.e_hi, w, k, out)
            self.comm.all_reduce(out)
            ops.add_prep(out, resid, w_next, xw, ss_1)
            return ss_1
        nv = d // 8
        P = nv // 64 if nv % 64 == 0 and nv >= 64 else 1  # one 8-column vector per thread of a 64-thread part
        ss = self._buf("ss_parts", (T, P), torch.float32)
        ops.moe_combine_prep(y2, dst, ids, E, w, k, resid, w_next, xw, ss)
        return ss

    # ------------------------------------------------------------------------------------------
    def _router_logits(self, i, x):
        """Router logits of x's rows: the 16-expert-row MFMA kernel (fp32, one launch) where the padded router is
        16 rows, else the projection path."""
        if self.router[i].shape[0] == 16 and x.shape[1] % 128 == 0 and x.is_contiguous():
            logits = self._buf("router_logits", (x.shape[0], 16), torch.float32)
            ops.moe_router(x, self.router[i], logits)
            return logits
        return self.m._linear("router", x, self.router[i])

    def _route(self, i, x):
        T, d = x.shape
        k, E = self.k, self.E
        R = T * k
        logits = self._router_logits(i, x)
        ids = self._buf("ids", (R,), torch.int32)
        w = self._buf("w", (R,), torch.float32)
        dst = self._buf("dst", (R,), torch.int32)
        counts = self._buf("counts", (E,), torch.int32)
        offsets = self._buf("offsets", (E + 1,), torch.int32)
        cursor = self._buf("cursor", (E,), torch.int32)
        xs = self._buf("xs", (R, d), torch.bfloat16)
        ops.moe_route_permute(logits, x, k, E, ids, w, counts, offsets, cursor, xs, dst)
        return ids, w, dst, offsets, xs

    def _grouped_ok(self, d: int) -> bool:
        return d % 128 == 0 and self.F % 64 == 0 and GROUPED



    def _experts(self, i, xs, offsets, e_lo, n_local, out_f32: bool = False):
        """Apply experts [e_lo, e_lo + n_local) to their segments of xs (segment bounds: ``offsets``, device
        memory, global expert numbering); returns a LinOut [.., R, d]."""
        R, d = xs.shape
        w13 = self.m.w.layer(i, "w13")
        w2 = self.m.w.layer(i, "w2")
        F = self.F
        act = self._buf("act", (R, F), torch.bfloat16)
        if STREAM_DECODE_ROWS * n_local <= R <= SKINNY_ROWS and ((i, "w13") in self.pre or (i, "w2") in self.pre):
            # decode sizes on the preshuffled copies: the weight-streaming kernel (1 KB fragment loads, one unit per
            # populated expert and n-block) beats the grouped skinny GEMM at 1-8 rows per expert when every expert
            # is routed: w13 + SwiGLU 320 -> 299 us, w2 162 -> 144 (profiles/r5/grouped_stream.jsonl); with a few
            # tokens (config 5: 4 clients, ~3 of 8 experts idle) its units leave a partial last round and the
            # skinny GEMM's per-(tile, expert) grid balances better (85.6 vs 87.9 tok/s per client end to end)
            p13, p2 = self.pre.get((i, "w13")), self.pre.get((i, "w2"))
            if p13 is not None:
                ops.grouped_gemm(xs, p13, offsets, e_lo, act, ops.GROUPED_SWIGLU + ops.GROUPED_PRESHUFFLED)
            else:
                s1 = ops.choose_splits(2 * F, d)
                y1 = self._buf("y1", (s1, R, 2 * F), torch.float32)
                ops.grouped_skinny(xs, w13, offsets, e_lo, y1)
                ops.swiglu(y1, act)
            if p2 is not None:
                y2 = self._buf("y2f" if out_f32 else "y2b", (R, d), torch.float32 if out_f32 else torch.bfloat16)
                ops.grouped_gemm(act, p2, offsets, e_lo, y2, (ops.GROUPED_F32 if out_f32 else ops.GROUPED_BF16)
                                 + ops.GROUPED_PRESHUFFLED)
                return y2
            s2 = ops.choose_splits(d, F)
            y2 = self._buf("y2", (s2, R, d), torch.float32)
            ops.grouped_skinny(act, w2, offsets, e_lo, y2)
            return y2
        if R <= SKINNY_ROWS:  # (single copy: the skinny GEMM reads the preshuffled expert stacks)
            s1 = ops.choose_splits(2 * F, d)
            y1 = self._buf("y1", (s1, R, 2 * F), torch.float32)
            ops.grouped_skinny(xs, w13, offsets, e_lo, y1, wshuf=self.single_copy)
            ops.swiglu(y1, act)
            s2 = ops.choose_splits(d, F)
            y2 = self._buf("y2", (s2, R, d), torch.float32)
            ops.grouped_skinny(act, w2, offsets, e_lo, y2, wshuf=self.single_copy)
            return y2
        if self._grouped_ok(d):
            # prefill-sized.  From PG_ROWS_* mean routed rows per local expert: the prefill GEMM kernel in grouped mode
            # on the preshuffled copies (csrc/kernels/pgemm.hip: block -> (expert, m-tile) from the device offsets)
            # -- SwiGLU of the [gate; up] halves in the gate/up epilogue, w2 into fp32 k-split slabs the combine
            # sums.  Below: the weight-streaming kernel on the preshuffled copies up to PRE_ROWS* rows, the 128 x 128
            # tile kernel beyond
            rpe = R / max(1, n_local)
            pg13 = self.pre.get((i, "w13")) if PG_GROUPED and rpe >= PG_ROWS_W13 else None
            pg2 = self.pre.get((i, "w2")) if PG_GROUPED and rpe >= PG_ROWS_W2 else None
            c13 = ops.choose_pg_grouped(R, 2 * F, d, n_local, even_wn=True) if pg13 is not None else None
            c2 = ops.choose_pg_grouped(R, d, F, n_local, slabs=out_f32) if pg2 is not None else None
            if c13 is not None:
                ops.pg_grouped(xs, pg13, offsets, e_lo, act, ops.PG_EPI_SWIGLU_SPLIT, c13[0])
            else:
                p13 = self.pre.get((i, "w13")) if self.single_copy or R <= PRE_ROWS_W13 * self.E else None
                ops.grouped_gemm(xs, w13 if p13 is None else p13, offsets, e_lo, act,
                                 ops.GROUPED_SWIGLU + (0 if p13 is None else ops.GROUPED_PRESHUFFLED))
            if c2 is not None:
                cfg2, s2 = c2
                if out_f32:
                    y2 = self._buf(f"y2pg{s2}", (s2, R, d), torch.float32)
                    ops.pg_grouped(act, pg2, offsets, e_lo, y2, ops.PG_EPI_F32, cfg2, s2)
                else:
                    y2 = self._buf("y2b", (R, d), torch.bfloat16)
                    ops.pg_grouped(act, pg2, offsets, e_lo, y2, ops.PG_EPI_BF16, cfg2)
                return y2
            p2 = self.pre.get((i, "w2")) if self.single_copy or R <= PRE_ROWS * self.E else None
            y2 = self._buf("y2f" if out_f32 else "y2b", (R, d), torch.float32 if out_f32 else torch.bfloat16)
            ops.grouped_gemm(act, w2 if p2 is None else p2, offsets, e_lo, y2,
                             (ops.GROUPED_F32 if out_f32 else ops.GROUPED_BF16)
                             + (0 if p2 is None else ops.GROUPED_PRESHUFFLED))
            return y2
        # shapes outside the grouped kernel's tiling (not the registered models): per-expert library GEMMs
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
        y2 = self._experts(i, xs, offsets, self.e_lo, self.E_local, out_f32=True)
        out = self._buf("out", (T, d), torch.float32)
        ops.moe_combine(y2, dst, ids, self.e_lo, self.e_hi, w, self.k, out)
        if reduce:
            self.comm.all_reduce(out)
            self._stat("allreduce", self.allreduce_bytes(T, d))
        return out

    def allreduce_bytes(self, T: int, d: int) -> int:
        """Bytes one rank pushes for the fp32 [T, d] all-reduce combine: the one-shot xGMI kernel writes its
        partial into every peer ((N - 1) T d 4, decode sizes), a ring all-reduce 2 (N - 1) / N T d 4."""
        N = self.ep
        if T * d * 4 <= getattr(self.comm, "oneshot_bytes", 0):
            return (N - 1) * T * d * 4
        return 2 * (N - 1) * T * d * 4 // N

    # ------------------------------------------------------------------------------------------
    def forward_a2a(self, i: int, x: torch.Tensor) -> torch.Tensor:
        """Expert parallelism over REPLICATED tokens (x [T, d] identical on every rank: the attention is tensor-
        parallel).  No dispatch leg: every rank routes all T tokens (deterministic kernels, identical routing),
        runs its own experts on its own routed rows, and pushes, per token with a local expert, ONE fp32 row --
        the weighted partial over its local experts -- to the token's slice owner (rank t // S, S = ceil(T / N));
        the owner sums the partials in rank order and a bf16 all-gather rebuilds [T, d] on every rank.  Bytes
        per rank: ~T k / N rows x d x 4 to the owners (only counted rows cross the links on the xGMI
        communicator) + (N - 1) / N x T x d x 2 gathered, against 2 (N - 1) / N x T x d x 4 for the fp32
        all-reduce combine.  Elsewhere (RCCL / gloo) whole capacity blocks move, empty slots marked -1."""
        T, d = x.shape
        N, r, k = self.ep, self.ep_rank, self.k
        S = -(-T // N)
        lo, hi = min(T, r * S), min(T, (r + 1) * S)
        ids, w, dst, offsets, xs = self._route(i, x)
        y = self._experts(i, xs, offsets, self.e_lo, self.E_local, out_f32=True)
        cap = S  # a token sends at most one (pre-combined) row to its owner
        send = self._buf("own.send", (N * cap, d), torch.float32)
        side = self._buf("own.side", (N * cap,), torch.int32)
        cursor = self._buf("own.cursor", (N,), torch.int32)
        xg = getattr(self.comm, "a2a_fits", None)
        xg = xg is not None and xg(cap, d * 4)
        ops.moe_owner_pack(y, dst, ids, w, self.e_lo, self.e_hi, k, S, cursor, send, side)
        if xg:
            recv = self._buf("own.recv", (N * cap, d), torch.float32)
            rside = self._buf("own.rside", (N * cap,), torch.int32)
            rcnt = self._buf("own.rcnt", (N,), torch.int32)
            self.comm.a2a_rows(send, cursor, side, recv, rside, rcnt)
            self._stat("return", (cursor.sum() - cursor[r]) * (d * 4))  # rows that left this GPU (device count)
            self._stat("routed_rows", cursor.sum())
        else:
            # RCCL / gloo: the per-owner counts first, then all_to_all_single with them as splits (the side ints
            # ride as one extra fp32 column): only the real rows move
            sc, rc = self._counts_exchange(cursor)
            packed = torch.cat([send, side.view(-1, 1).view(torch.float32)], 1)
            got = self._exchange_counted(packed, sc, rc, cap)
            recv = got[:, :d].contiguous()
            rside = got[:, d:].contiguous().view(torch.int32).view(-1)
            rcnt = torch.tensor(rc, dtype=torch.int32, device=x.device)
            self._stat("return", (sum(sc) - sc[r]) * (d * 4 + 4))
            self._stat("routed_rows", sum(sc))
        pos = self._buf("own.pos", (N * S,), torch.int32)
        mine = self._buf("own.slice", (S, d), torch.bfloat16)
        ops.moe_owner_combine(recv, rside, rcnt, hi - lo, pos, mine)
        g = self.comm.all_gather(mine)  # [N * S, d] bf16
        self._stat("gather", (N - 1) * S * d * 2)
        return g[:T]

    def forward_tokens(self, i: int, x: torch.Tensor, S: int) -> torch.Tensor:
        """Dispatch -> owners' expert GEMMs -> return -> combine for THIS rank's tokens x [T_r <= S, d] (ranks
        may hold different tokens; S: the per-rank row bound every rank uses, which fixes the capacity)."""
        Tr, d = x.shape
        N, k, E, El = self.ep, self.k, self.E, self.E_local
        cap = S * k                       # rows this rank can send to one owner
        dev = x.device
        R = Tr * k
        # ---- route my tokens; group the routed rows by OWNER rank into fixed capacity blocks
        ids = self._buf("a2a.ids", (max(R, 1),), torch.int32)
        w = self._buf("a2a.w", (max(R, 1),), torch.float32)
        dst = self._buf("a2a.dst", (max(R, 1),), torch.int32)
        send = self._buf("a2a.send", (N * cap, d), torch.bfloat16)
        send_e = self._buf("a2a.send_e", (N * cap, 1), torch.int32)
        cursor = self._buf("a2a.cursor", (N,), torch.int32)  # after moe_scatter: routed rows per owner
        cursor.zero_()
        # only the routed rows cross the links: on xGMI with the counts on the device, on RCCL / gloo with the
        # counts exchanged first and used as all_to_all_single splits (slots past a count read "empty", -1)
        xg = getattr(self.comm, "a2a_fits", None)
        xg = xg is not None and xg(cap, d * 4)
        if Tr > 0:
            logits = self._router_logits(i, x)
            ops.moe_route(logits, Tr, k, E, ids, w)
            owner = self._buf("a2a.owner", (R,), torch.int32)
            torch.floor_divide(ids[:R], El, out=owner)
            blocks = self._blocks(N, cap, dev)
            ops.moe_scatter(x, owner, k, N, blocks, cursor, send, dst)
            send_e.view(-1).index_copy_(0, dst[:R].long(), ids[:R])
        # ---- dispatch: block q of every rank's send buffer goes to rank q
        if xg:
            recv = self._buf("a2a.recv", (N * cap, d), torch.bfloat16)
            recv_e = self._buf("a2a.recv_e", (N * cap,), torch.int32)
            rcnt = self._buf("a2a.rcnt", (N,), torch.int32)
            self.comm.a2a_rows(send, cursor, send_e.view(-1), recv, recv_e, rcnt)
        else:
            sc, rc = self._counts_exchange(cursor)
            # the expert id rides as two bf16 columns of the row; empty slots decode as -1
            packed = torch.cat([send, send_e.view(torch.bfloat16)], 1)
            fill_row = torch.cat([torch.zeros(d, dtype=torch.bfloat16),
                                  torch.tensor([-1], dtype=torch.int32).view(torch.bfloat16)])
            got = self._exchange_counted(packed, sc, rc, cap)
            empty = torch.ones(N * cap, dtype=torch.bool, device=dev)
            empty[self._block_rows(rc, cap, dev)] = False
            got[empty] = fill_row.to(dev)
            recv = got[:, :d].contiguous()                                      # [N * cap, d]  (src-major)
            recv_e = got[:, d:].contiguous().view(torch.int32).view(-1)         # expert id per slot, -1 = empty
        # ---- group the received rows by local expert, run the grouped GEMMs
        counts = self._buf("a2a.counts", (E,), torch.int32)
        offsets = self._buf("a2a.offsets", (E + 1,), torch.int32)
        cursor_e = self._buf("a2a.cursor_e", (E,), torch.int32)
        ops.moe_align(recv_e, E, counts, offsets, cursor_e)
        xs = self._buf("a2a.xs", (N * cap, d), torch.bfloat16)
        ldst = self._buf("a2a.ldst", (N * cap,), torch.int32)
        ldst.zero_()  # empty slots keep row 0 (returned, never combined)
        ops.moe_scatter(recv, recv_e, 1, E, offsets, cursor_e, xs, ldst)
        y = self._experts(i, xs, offsets, self.e_lo, El, out_f32=True)
        if y.dim() == 3:  # skinny-path slabs -> [N * cap, d] fp32, rows in local expert order
            yl = self._buf("a2a.ysum", (N * cap, d), torch.float32)
            torch.sum(y, 0, out=yl)
        else:
            yl = y
        # ---- return: every received slot's result goes back to the slot it came from
        back = self._buf("a2a.back", (N * cap, d), torch.float32)
        torch.index_select(yl, 0, ldst.long(), out=back)
        if xg:  # the return is the transpose: block s of `back` holds rcnt[s] real rows for rank s
            ret = self._buf("a2a.ret", (N * cap, d), torch.float32)
            self.comm.a2a_rows(back, rcnt, None, ret)
            r = self.ep_rank  # rows a rank keeps never cross a link
            self._stat("dispatch", (cursor.sum() - cursor[r]) * (d * 2))
            self._stat("return", (rcnt.sum() - rcnt[r]) * (d * 4))
        else:
            ret = self._exchange_counted(back, rc, sc, cap)                    # [N * cap, d]: my slots' results
            r = self.ep_rank
            self._stat("dispatch", (sum(sc) - sc[r]) * (d * 2 + 4))
            self._stat("return", (sum(rc) - rc[r]) * (d * 4))
        self._stat("routed_rows", R)
        self._stat("padded_dispatch", N * cap * d * 2)
        out = self._buf("a2a.out", (max(Tr, 1), d), torch.float32)[:Tr]
        if Tr > 0:
            ops.moe_combine(ret, dst, ids, 0, E, w, k, out)
        return out

    def _blocks(self, N: int, cap: int, dev) -> torch.Tensor:
        """Fixed segment starts q * cap of the per-owner send blocks (built once per capacity)."""
        key = ("moe.a2a.blocks", N, cap)
        b = self.m.ws.buffers.get(key)
        if b is None:
            b = torch.arange(N + 1, dtype=torch.int32, device=dev) * cap
            self.m.ws.buffers[key] = b
        return b
