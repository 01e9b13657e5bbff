"""Llama-3 / Mixtral decoder forward built on the symmetry_amd ops.

One code path serves CPU (torch references, tests) and MI355X (HIP kernels).
Per layer::

    K1 add+RMSNorm -> QKV proj -> K2/K3 RoPE+paged-cache write -> K4/K5 attention
    -> O proj -> [R1 all-reduce] -> K1 add+RMSNorm -> gate_up proj -> K7 SwiGLU
    -> down proj -> [R1 all-reduce]            (Mixtral: K10-K12 MoE block, R3 all-to-all)

Two paths over the same weights (stored in the decode layout, models/layout.py):

* fused (decode steps and short prefills below GENERAL_ROWS rows) -- five launches per dense layer::

      dg_qkv (norm scale + RoPE + KV write) -> attention -> dg_resid (O, residual add, ln2 prep)
      -> dg_swiglu (norm scale + SwiGLU) -> dg_resid (down, residual add, next-ln1 prep)

  with RMSNorm deferred into the consuming GEMM (csrc/kernels/decode_gemm.hip) and the final
  norm + lm_head + sampling in dg_argmax.  Under TP the row-parallel projections write fp32,
  are all-reduced, and add_prep does the residual + norm prep.
* general (prefills, and decode steps of GENERAL_ROWS..256 rows): projections of up to 256 rows on the
  medium-M split-K kernel (mgemm, where it beats the library: ops.choose_mgemm), longer ones on the
  library GEMM (hipBLASLt through torch.matmul), + fused elementwise kernels that also sum the split-K
  slabs, with the layout flags on rope_cache / swiglu; batches wider than 64 rows sample from one fp32
  logits GEMM (logits_argmax: the fused sampler's keys and RNG).

All intermediates live in a preallocated :class:`Workspace`, so the decode forward is
hipGraph-capturable.
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass, field

import torch

from .. import ops
from ..ops import reference
from .config import ModelConfig
from .layout import apply_decode_layout
from .weights import ModelWeights

SKINNY_MAX_M = 64
# TP prefill: row-parallel partials all-reduced in bf16 (SYMMETRY_TP_REDUCE_BF16=0: fp32, the A/B reference)
TP_REDUCE_BF16 = os.environ.get("SYMMETRY_TP_REDUCE_BF16", "1") != "0"
# Decode steps with at least this many rows run the O and down projections as k-split skinny GEMMs into
# fp32 slabs (summed by add_prep) instead of one fused dg_resid launch: those projections have only
# N / 16 = 256 row tiles, so every workgroup re-reads all M rows of x over the full K range and the x
# traffic outgrows the weight stream as M grows (bench.py ms/step, fused vs split: 24 rows 4.38 vs 4.42,
# 32 rows 4.75 vs 4.66, 64 rows 6.86 vs 6.12; profiles/decode_splitk_resid_r1.jsonl).  With the
# column-sliced add_prep the crossover moved to 21..24 rows (fused vs split: 20 rows 4.15 vs 4.19,
# 24 rows 4.34 vs 4.32, 28 rows 4.45 vs 4.44; 1/10/16 rows stay fused; profiles/decode_splitk_small_m_r1.jsonl).
# Re-checked with 3 alternating runs per arm (profiles/decode_splitk_threshold_ab_r2.jsonl, mean [min, max]):
# 24 rows fused 4.323 [4.317, 4.330] vs split 4.288 [4.285, 4.289] ms/step, p50 TTFT 40.43 vs 40.49 ms;
# 28 rows 4.443 [4.433, 4.453] vs 4.427 [4.417, 4.435], TTFT 47.07 vs 46.89: the split path wins by more than
# the run-to-run spread at 24 rows and TTFT does not move, so the threshold stays at 24.
# SYMMETRY_SPLITK_RESID_ROWS=0 disables it (A/B).
SPLITK_RESID_ROWS = int(os.environ.get("SYMMETRY_SPLITK_RESID_ROWS", "24"))
# Steps with at least this many rows run the general path -- medium-M projections (mgemm) +
# consumer kernels -- instead of the fused decode GEMMs, whose per-row-tile x re-reads grow with M.
# bench.py ms/step, fused vs general, 2 alternating runs each (profiles/general_rows_ab_r2.jsonl):
# 10 rows 3.22 vs 3.90, 16 3.42 vs 3.94, 24 4.30 vs 3.98, 32 4.52 vs 4.07, 48 5.11 vs 4.37, 64 5.78 vs 4.63.
# Decode batches are padded to buckets (.., 16, 24, ..), so 17..24-row steps run as 24.  0 disables.
GENERAL_ROWS = int(os.environ.get("SYMMETRY_GENERAL_ROWS", "20"))  # profiles/general_rows_ab_r2.jsonl
MAX_STEP_SEQS = 4096  # sequences per step (rows of last_ids)
# decode steps on the general path run rope_cache's per-row form (A/B knob)
ROPE_DECODE_ROWS = os.environ.get("SYMMETRY_ROPE_DECODE_ROWS", "1") != "0"
# general path (20-256 rows): which projections run on mgemm with the fused decode epilogue (in-launch split-K
# reduction; RoPE + KV write, residual + norm prep, SwiGLU in the GEMM) instead of slabs + a consumer kernel.
#   "all": all four (5 launches per layer instead of 9), "gu" (default): gate_up + SwiGLU only (o's consumer
#   becomes add_prep: deferred norm for gate_up), "0": none.  profiles/r3/mg_fused_ab.jsonl (alternating
#   runs): 64 clients 4.84 / 4.30-4.33 / 4.46 ms per step, 32 clients 3.95 / 3.80 / 3.91 for all / gu / 0:
#   the in-launch reduction's tail (one of S workgroups per column group sums the slabs) costs o / down /
#   qkv more than the separate consumer kernel they save.
MG_FUSED_MODE = os.environ.get("SYMMETRY_MG_FUSED", "gu")
MG_FUSED = MG_FUSED_MODE in ("1", "all")
MG_FUSED_GU = MG_FUSED_MODE == "gu"
# MFMA-preshuffled copy of the lm_head for the fused decode path's dg_argmax (1 KB per wave load like the layer
# weights; +1 GB for Llama-3-8B): SYMMETRY_LMHEAD_SHUF=0 keeps the row-major stream
LMHEAD_SHUF = os.environ.get("SYMMETRY_LMHEAD_SHUF", "1") != "0"


def copy_budget(device, kv_reserve: int, workspace: int = 6 << 30) -> float:
    """HBM an optional weight-layout copy may take: free memory minus the KV cache's need and a workspace reserve
    (the copies used to take half of the free HBM before the KV cache was sized)."""
    return max(0.0, float(torch.cuda.mem_get_info(device)[0]) - kv_reserve - workspace)


@dataclass
class ForwardBatch:
    """Device-side metadata of one engine step.

    ``kind`` is ``"decode"`` (one new token per sequence, T == num_seqs) or
    ``"prefill"`` (packed varlen prompts / prompt chunks).
    """

    kind: str
    input_ids: torch.Tensor      # [T] int32
    positions: torch.Tensor      # [T] int32
    slot_mapping: torch.Tensor   # [T] int32 (-1: no cache write)
    block_tables: torch.Tensor   # [num_seqs, max_blocks] int32
    ctx_lens: torch.Tensor       # [num_seqs] int32 (context incl. this step's tokens)
    temps: torch.Tensor          # [num_seqs] f32 (0 = greedy)
    seeds: torch.Tensor          # [num_seqs] i64
    step: torch.Tensor           # [1] i64 sampling step counter
    num_seqs: int
    # prefill only
    cu_q: torch.Tensor | None = None        # [num_seqs + 1] int32
    tiles: torch.Tensor | None = None       # [n_tiles, 2] int32
    last_idx: torch.Tensor | None = None    # [num_seqs] int64 row of each sequence's last token
    need_logits: bool = False
    src: torch.Tensor | None = None         # [T] int32: >= 0 -> token = previous step's sample in that row
    top_k: torch.Tensor | None = None       # [num_seqs] int32 (0 = off)
    top_p: torch.Tensor | None = None       # [num_seqs] f32 (1 = off)
    filtered: bool = False                  # some row needs the top-k / top-p resampler

    @property
    def num_tokens(self) -> int:
        return int(self.input_ids.numel())


class KVCache:
    """Paged KV cache: k [L, NB, Hkv, BS, D] (token-major), v [L, NB, Hkv, D, BS] (dim-major).

    Zero-initialised: every cache byte is finite, so masked tail tokens of a
    block contribute exactly 0 to P.V.
    """

    def __init__(self, num_layers: int, num_blocks: int, num_kv_heads: int, head_dim: int, block_size: int,
                 device, dtype=torch.bfloat16):
        self.num_layers, self.num_blocks, self.block_size = num_layers, num_blocks, block_size
        self.k = torch.zeros(num_layers, num_blocks, num_kv_heads, block_size, head_dim, device=device, dtype=dtype)
        self.v = torch.zeros(num_layers, num_blocks, num_kv_heads, head_dim, block_size, device=device, dtype=dtype)

    def nbytes(self) -> int:
        return 2 * self.k.numel() * self.k.element_size()


@dataclass
class Workspace:
    """Named scratch buffers that only grow.

    A replaced buffer is kept alive (``retired``): hipGraphs captured earlier
    hold its raw address, so it must never return to the allocator.
    """

    buffers: dict = field(default_factory=dict)
    retired: list = field(default_factory=list)

    def get(self, name: str, shape, dtype, device, zeros: bool = False) -> torch.Tensor:
        """``zeros``: zero-fill on (re)allocation only -- for state the kernels keep re-armed themselves."""
        numel = math.prod(shape)
        buf = self.buffers.get((name, dtype))
        if buf is None or buf.numel() < numel:
            if buf is not None:
                self.retired.append(buf)
            buf = (torch.zeros if zeros else torch.empty)(numel, dtype=dtype, device=device)
            self.buffers[(name, dtype)] = buf
        return buf[:numel].view(*shape)

    def nbytes(self) -> int:
        return sum(b.numel() * b.element_size() for b in list(self.buffers.values()) + self.retired)


class TransformerLM:
    def __init__(self, weights: ModelWeights, device, tp_comm=None, ep_comm=None, max_decode_ctx: int | None = None,
                 decode_weights: str = "auto", kv_reserve_bytes: int = 0):
        self.cfg: ModelConfig = weights.cfg
        self.w = weights
        self.device = torch.device(device)
        self.tp = tp_comm
        self.ep = ep_comm
        self.tp_size = weights.shard.tp_size
        self.tp_rank = weights.shard.tp_rank
        cfg = self.cfg
        self.hq = cfg.num_heads // self.tp_size
        self.hkv = cfg.num_kv_heads // self.tp_size
        self.D = cfg.head_dim
        self.scale = 1.0 / math.sqrt(cfg.head_dim)
        self.vocab_shard = cfg.vocab_size // self.tp_size
        max_pos = min(cfg.max_position, max_decode_ctx or cfg.max_position)
        self.cos_sin = reference.rope_table(max_pos, cfg.head_dim, cfg.rope_theta, cfg.rope_scaling,
                                            device=self.device)
        self.ws = Workspace()
        # HBM the KV cache needs (admission limit x context): the optional layout copies never eat into it
        self.kv_reserve = int(kv_reserve_bytes)
        self.moe = None
        # MoE models default to ONE preshuffled copy of every weight: the expert stacks are read only by kernels
        # that take that layout (measured equal to the two-copy layout end to end, 90 GB less on one GPU:
        # profiles/r6/e2e_mixtral_c5_single_copy.jsonl), so MoEBlock makes no separate copies
        self.plan_single_copy = self._fused_supported() and (decode_weights == "replace" or (
            decode_weights == "auto" and cfg.is_moe and self.device.type != "cpu"))
        if cfg.is_moe:
            from .moe import MoEBlock

            self.moe = MoEBlock(self, ep_comm)
        apply_decode_layout(weights)
        self.fused = self._fused_supported()
        # Sampled ids of the most recent step live at a fixed device address: every step writes its
        # samples here and the next step's embedding reads pending input tokens from here (src map),
        # so the host can enqueue step N+1 before it has seen step N's tokens (pipelined decode).
        self.last_ids = torch.zeros(MAX_STEP_SEQS, dtype=torch.int32, device=self.device)
        if self.device.type != "cpu":
            ops.decode_ks_ws(self.device)  # allocated before any graph capture (stable address)
        self.single_copy = False  # decode_weights="replace": the layer weights exist only MFMA-preshuffled
        self.dgw = self._decode_copies(decode_weights)
        self.tp_reduced_bytes: dict[str, int] = {}  # bytes per rank of the last general-path all-reduce

    def _decode_copies(self, mode: str) -> dict:
        """MFMA-preshuffled decode-GEMM weights (1 KB contiguous per wave load: profiles/decode_gemm_preshuffle_r1.jsonl,
        -9 % per layer).  ``mode``:

        * "preshuffled": an extra copy next to the row-major tensors, which stay for the hipBLASLt prefill GEMMs
          (8B: +14.5 GB of 288 GB);
        * "replace": ONE copy -- the layer weights are preshuffled in place (models with the fused decode GEMMs)
          and every consumer reads that layout: decode GEMMs, mgemm / the prefill GEMM (pgemm) for prefill,
          dg_f32 for the few-row projections; MoE experts likewise (MoEBlock.adopt_single_copy: the streaming and
          grouped prefill GEMM kernels); the fp32 oracle and exports unshuffle (layout.natural_tensors);
        * "shared": row-major only (the decode GEMMs' row-major variants);
        * "auto": MoE models "replace" (profiles/r6/e2e_mixtral_c5_single_copy.jsonl: equal end to end, 90 GB
          less); dense models "preshuffled" when the copy fits next to the KV cache's need (transformer.copy_budget;
          their prefill is faster on the library GEMMs), "replace" otherwise (70B on one GPU: 141 GB of layer
          weights), row-major only where neither applies."""
        if not self.fused or mode == "shared" or (self.device.type == "cpu" and mode != "replace"):
            return {}
        names = ["wqkv", "wo"] + ([] if self.cfg.is_moe else ["w_gu", "w_down"])
        extra = sum(self.w.layer(i, n).numel() * 2 for i in range(self.cfg.num_layers) for n in names)
        head = self.w["lm_head"] if LMHEAD_SHUF else None
        if head is not None and (head.shape[0] % 16 or head.shape[1] % 32):
            head = None
        if mode == "auto":
            # the layer copies first (-9 % per layer); the head copy (~1 GB for Llama-3-8B, -12 % of one lm_head
            # launch) only from what the same budget has left, so it never costs a model its layer copies.  The
            # budget: what is left after the KV cache's need and a 6 GB workspace reserve
            budget = copy_budget(self.device, self.kv_reserve)
            if self.moe is not None:
                mode = "replace" if self.moe.single_copy_ok() else "shared"
                if mode == "shared":
                    return {}
            elif extra > budget:
                mode = "replace"
            if head is not None and (mode == "replace" or extra + head.numel() * 2 > budget):
                head = None
        from .layout import preshuffle

        out = {}
        if mode == "replace":
            if self.moe is not None and not self.moe.single_copy_ok():
                raise ValueError("decode_weights=replace: the expert shapes do not tile for the preshuffled kernels")
            for i in range(self.cfg.num_layers):
                for n in names:
                    key = f"layers.{i}.{n}"
                    t = preshuffle(self.w.tensors[key])
                    self.w.tensors[key] = t  # the row-major tensor is released here
                    out[(i, n)] = t
            shuffled = {f"layers.{i}.{n}" for i in range(self.cfg.num_layers) for n in names}
            if self.moe is not None:
                shuffled |= set(self.moe.adopt_single_copy())
            self.w.shuffled = frozenset(shuffled)
            self.single_copy = True
            return out
        for i in range(self.cfg.num_layers):
            for n in names:
                out[(i, n)] = preshuffle(self.w.layer(i, n))
        if head is not None:
            out[(-1, "lm_head")] = preshuffle(head)
        return out

    def _row_major(self, i: int, name: str):
        """The row-major layer weight, or None when only the preshuffled layout exists (decode_weights="replace")."""
        return None if self.single_copy else self.w.layer(i, name)

    def extra_weight_bytes(self) -> int:
        """Bytes of the optional layout copies (preshuffled decode weights, preshuffled expert streams); 0 for the
        layer weights of a single-copy model (decode_weights="replace": the preshuffled tensors ARE the weights)."""
        n = sum(t.numel() * t.element_size() for k, t in self.dgw.items() if not (self.single_copy and k[0] >= 0))
        if self.moe is not None and not self.single_copy:
            n += sum(t.numel() * t.element_size() for t in self.moe.pre.values())
        return n

    def _lm_head(self, rows: int):
        """(weight, wshuf) of the decode lm_head for a ``rows``-row sampling launch: the MFMA-preshuffled copy up
        to 16 rows, the row-major stream's row-tile variants above (profiles/r3/lmhead_preshuffle_ab.jsonl: 1 row
        189.5 -> 175.1 us, 6 rows 192.9 -> 168.8; 24 rows 222.6 vs 232.3, 32 rows 220 vs 228; 64 rows even)."""
        return self._dgw(-1, "lm_head") if rows <= 16 else (self.w["lm_head"], False)

    def _dgw(self, i: int, name: str):
        """(weight, wshuf) for decode GEMM `name` of layer i (i = -1: the lm_head)."""
        t = self.dgw.get((i, name))
        if t is not None:
            return t, True
        return (self.w[name] if i < 0 else self.w.layer(i, name)), False

    def _shuf(self, i: int, name: str):
        """The MFMA-preshuffled copy of weight `name` of layer i, or None (medium-M prefill GEMMs)."""
        return self.dgw.get((i, name))

    def _fused_supported(self) -> bool:
        """Shape contract of the fused decode GEMMs: D == 128, every K % 256 == 0, every N % 16 == 0."""
        cfg = self.cfg
        ks = [cfg.hidden_size, self.hq * self.D]
        if not cfg.is_moe:
            ks.append(self.w.layer(0, "w_gu").shape[0] // 2)
        return (self.D == 128 and all(k % 256 == 0 for k in ks) and cfg.hidden_size % 16 == 0
                and self.vocab_shard % 16 == 0)

    # ------------------------------------------------------------------------------------------
    def _buf(self, name, shape, dtype):
        return self.ws.get(name, shape, dtype, self.device)

    def _linear(self, name: str, x: torch.Tensor, w: torch.Tensor, reduce: bool = False,
                wshuf: torch.Tensor | None = None) -> torch.Tensor:
        """x [T, K] bf16 -> LinOut: fp32 slabs [S, T, N] (skinny / medium-M) or bf16 [T, N] (library GEMM).
        ``wshuf``: the MFMA-preshuffled copy of ``w`` if one exists (enables the medium-M kernel)."""
        T, K = x.shape
        N = (w if w is not None else wshuf).shape[0]
        pick = ops.choose_mgemm(T, N, K) if wshuf is not None else None
        if pick is not None:
            rw, S = pick
            y = self._buf(name + ".slab", (S, T, N), torch.float32)
            ops.mgemm(x, wshuf, y, rw)
        elif w is None and T <= SKINNY_MAX_M:
            # only the preshuffled layout exists: the decode GEMM's fp32 form (one slab)
            y = self._buf(name + ".slab", (1, T, N), torch.float32)
            ops.dg_f32(x, wshuf, None, 0.0, y.view(T, N), wshuf=True)
        elif w is None:
            # ... and the prefill GEMM past the medium range: k-split fp32 slabs where they pay, else bf16 out
            cfg, S = ops.choose_pgemm(max(T, ops.PGEMM_MIN_M), N, K, slabs=True, force=True)
            if S > 1:
                y = self._buf(name + ".slab", (S, T, N), torch.float32)
            else:
                y = self._buf(name + ".bf16", (T, N), torch.bfloat16)
            ops.pgemm(x, wshuf, y, cfg, S)
        elif T <= SKINNY_MAX_M:
            S = ops.choose_splits(N, K)
            y = self._buf(name + ".slab", (S, T, N), torch.float32)
            ops.skinny_gemm(x, w, y)
        elif not self.cfg.is_moe and (S := ops.lib_splits(T, N, K)) > 1 and K % S == 0:
            # (dense models only: fp32 slabs instead of bf16 GEMM outputs shift MoE router logits enough to
            # flip near-tied top-2 choices against the fp32 oracle of the tiny random test model)
            y = self._buf(name + ".slab", (S, T, N), torch.float32)
            ops.linear_splitk(x, w, y)
        else:
            y = self._buf(name + ".bf16", (T, N), torch.bfloat16)
            ops.linear(x, w, out=y)
        if reduce and self.tp is not None and self.tp_size > 1:
            if y.dim() == 3 and y.shape[0] > 1:
                # sum the split-K slabs locally first: the collective then moves one [T, N] fp32 partial per
                # rank instead of S of them (S x fewer bytes over xGMI on every row-parallel projection)
                ys = self._buf(name + ".red", (1, T, N), torch.float32)
                torch.sum(y, dim=0, keepdim=True, out=ys)
                y = ys
            if TP_REDUCE_BF16 and T > SKINNY_MAX_M and y.dtype == torch.float32:
                # prefill-sized: all-reduce the partial in bf16 -- half the bytes of every row-parallel collective
                # (the TP=1 library GEMM of these shapes writes bf16 too); decode-sized ones stay fp32 (one-shot
                # xGMI kernels, fused with the residual epilogue)
                yb = self._buf(name + ".redbf", (T, N), torch.bfloat16)
                yb.copy_(y.view(T, N))
                y = yb
            self.tp_reduced_bytes[name] = y.numel() * y.element_size()
            self.tp.all_reduce(y)
        return y

    # ------------------------------------------------------------------------------------------
    def _attention(self, b: ForwardBatch, kv: KVCache, i: int, q: torch.Tensor, attn: torch.Tensor) -> None:
        if b.kind == "decode":
            span = b.block_tables.shape[1] * kv.block_size
            max_parts = (span + ops.ATTN_DECODE_PART - 1) // ops.ATTN_DECODE_PART
            tmp_o = self._buf("tmp_o", (b.num_seqs, self.hq, max_parts, self.D), torch.float32)
            tmp_ml = self._buf("tmp_ml", (b.num_seqs, self.hq, max_parts, 2), torch.float32)
            cnt = self.ws.get("attn_counters", (b.num_seqs * self.hkv,), torch.int32, self.device, zeros=True)
            ops.attn_decode(q, kv.k[i], kv.v[i], b.block_tables, b.ctx_lens, attn, tmp_o, tmp_ml, cnt, self.scale)
        else:
            ops.attn_prefill(q, kv.k[i], kv.v[i], b.block_tables, b.ctx_lens, b.cu_q, b.tiles, attn, self.scale)

    @torch.no_grad()
    def forward(self, b: ForwardBatch, kv: KVCache) -> torch.Tensor:
        """Run one step; returns sampled token ids [num_seqs] int32 (device)."""
        if self.fused and b.num_tokens <= SKINNY_MAX_M and not self._general_rows(b.num_tokens):
            return self._forward_fused(b, kv)
        mgs = self._mg_plan(b)
        if mgs is not None:
            return self._forward_general_fused(b, kv, mgs)
        return self._forward_general(b, kv)

    def _pg_gate_up(self, T: int):
        """Tile config of the prefill GEMM (csrc/kernels/pgemm.hip) for this step's gate_up + SwiGLU, or None (library
        GEMM + swiglu kernel).  Dense model on one GPU with the preshuffled copies, PGEMM_GU_MIN_M..PGEMM_GU_MAX_M
        rows: where one wave of 320 / 384 x 224 tiles covers the projection it beats hipBLASLt + the swiglu launch
        (768 rows: 149 vs 155.5 + 13.8 us per layer, profiles/r6/prof_prefill768_pg_gu.csv); elsewhere the library
        wins (profiles/r6/pgemm_gu_sweep.jsonl, prefill_pgemm_ab3.jsonl).  The other three projections measured faster on
        the library path even against fused pgemm epilogues (profiles/r6/prof_prefill768_pg_all4_fused.csv: qkv 76 vs
        59, o 56 vs 45, down 99 vs 81 us with their consumers), so they stay there.  (Single-copy models at every
        prefill size instead of pgemm + swiglu measured even: Llama-3-70B 4 x 128-token TTFT 76.98 vs 76.5 ms.)"""
        if (self.cfg.is_moe or self._tp_active() or not self.dgw or self.device.type == "cpu"
                or not ops.PGEMM_GU_MIN_M <= T <= ops.PGEMM_GU_MAX_M):
            return None
        pick = ops.choose_pgemm(T, self.dgw[(0, "w_gu")].shape[0], self.cfg.hidden_size, force=self.single_copy)
        return None if pick is None else pick[0]

    def _mg_plan(self, b: ForwardBatch, names=("qkv", "o", "gu", "down"), need_all: bool = True,
                 any_kind: bool = False):
        """mgemm (rw, split) + scratch per projection for the fused general path, or None."""
        # under TP only the column-parallel projections (qkv, gate_up: no collective in their epilogue)
        tp_ok = not self._tp_active() or set(names) <= {"qkv", "gu"}
        if not ((MG_FUSED or any_kind) and (b.kind == "decode" or any_kind) and self.dgw
                and self.device.type != "cpu" and not self.cfg.is_moe and tp_ok and b.num_tokens <= 256):
            return None
        T, d, dq = b.num_tokens, self.cfg.hidden_size, self.hq * self.D
        wgu = self.w.layer(0, "w_gu")
        shapes = {"qkv": (self.w.layer(0, "wqkv").shape[0], d), "o": (d, dq), "gu": (wgu.shape[0], d),
                  "down": (d, wgu.shape[0] // 2)}
        plan = {}
        for name, (N, K) in shapes.items():
            if name not in names:
                continue
            pick = ops.choose_mgemm(T, N, K, fused=True)
            if pick is None:
                if need_all:
                    return None
                continue
            rw, S = pick
            slab = self._buf("mg.slab", (S, T, N), torch.float32)
            cnt = self.ws.get("mg.cnt." + name, (N // 64,), torch.int32, self.device, zeros=True)
            plan[name] = (slab, cnt, rw)
        return plan

    def _general_rows(self, T: int) -> bool:
        """Steps of GENERAL_ROWS..64 rows take the general path (medium-M projections + consumer kernels)
        instead of the fused decode GEMMs: dense model on one GPU with the preshuffled weight copies."""
        return (0 < GENERAL_ROWS <= T and bool(self.dgw) and not self.cfg.is_moe and not self._tp_active())

    # ------------------------------------------------------------------------------------------
    def _tp_active(self) -> bool:
        return self.tp is not None and self.tp_size > 1

    def _resid_proj(self, name, x, Wsh, resid, w_next, xw, ss_t, ss_1, w_row=None) -> torch.Tensor:
        """Row-parallel projection + residual add + next-norm prep; returns the ss partials to use."""
        W, sh = Wsh
        M = x.shape[0]
        if w_row is not None and not self._tp_active() and 0 < SPLITK_RESID_ROWS <= M:
            N, K = w_row.shape
            y = self._buf(name + ".slab", (ops.choose_splits(N, K), M, N), torch.float32)
            ops.skinny_gemm(x, w_row, y)
            # four workgroups per row (64 rows x 1 workgroup is latency-bound), four ss partials per row
            parts = 4 if N % 32 == 0 else 1
            ss_p = self._buf("ss_p", (M, parts), torch.float32)
            ops.add_prep(y, resid, w_next, xw, ss_p)
            return ss_p
        if self._tp_active():
            fused = getattr(self.tp, "gemm_ar_resid", None)
            if fused is not None and fused(x, W, sh, resid, w_next, xw, ss_t):
                # GEMM + all-reduce + residual + next-norm prep in ONE launch (DECODE_EPI_XAR): ss per 16 columns
                return ss_t
            # all-reduce + residual add + next-norm prep (one launch on the xGMI communicator); P column
            # parts per row = P workgroups per row (8 up to 16 rows, 4 beyond:
            # profiles/xgmi_allreduce_local_r2.jsonl, add_prep_P*), P sum-of-squares partials per row
            d = resid.shape[1]
            P = next((p for p in ((8, 4, 2) if M <= 16 else (4, 2)) if d % (16 * p) == 0), 1)
            ss_p = self._buf(f"ss_tp{P}", (M, P), torch.float32)
            y = self._buf(name + ".f32", (x.shape[0], W.shape[0]), torch.float32)
            ops.dg_f32(x, W, None, 0.0, y, wshuf=sh)
            self.tp.all_reduce_add_prep(y, resid, w_next, xw, ss_p)
            return ss_p
        ops.dg_resid(x, W, resid, w_next, xw, ss_t, wshuf=sh)
        return ss_t

    def _forward_fused(self, b: ForwardBatch, kv: KVCache) -> torch.Tensor:
        cfg, w = self.cfg, self.w
        T, d, eps = b.num_tokens, cfg.hidden_size, cfg.rms_eps
        resid = self._buf("resid", (T, d), torch.float32)
        xw = self._buf("xw", (T, d), torch.bfloat16)
        ss_t = self._buf("ss_t", (T, d // 16), torch.float32)
        ss_1 = self._buf("ss_1", (T, 1), torch.float32)
        q = self._buf("q", (T, self.hq, self.D), torch.bfloat16)
        attn = self._buf("attn", (T, self.hq, self.D), torch.bfloat16)
        ops.embed_prep(b.input_ids, w["embed"], resid, w.layer(0, "ln1"), xw, ss_1, b.src, self.last_ids)
        ss = ss_1
        for i in range(cfg.num_layers):
            wq, shq = self._dgw(i, "wqkv")
            attn2d = attn.view(T, self.hq * self.D)
            nxt = w.layer(i + 1, "ln1") if i + 1 < cfg.num_layers else w["norm"]
            ops.dg_qkv(xw, wq, ss, eps, b.positions, b.slot_mapping, self.cos_sin, q, kv.k[i], kv.v[i], self.hq,
                       self.hkv, wshuf=shq)
            self._attention(b, kv, i, q, attn)
            ss = self._resid_proj("o", attn2d, self._dgw(i, "wo"), resid, w.layer(i, "ln2"), xw, ss_t, ss_1,
                                  self._row_major(i, "wo"))
            if cfg.is_moe:
                if self.moe.decode_fused_ok(T, d):
                    ss = self.moe.forward_decode(i, resid, w.layer(i, "ln2"), eps, nxt, xw, ss_1)
                else:
                    # router + experts are not decode GEMMs: materialise RMSNorm(resid) (one bf16 rounding)
                    xn = self._buf("x", (T, d), torch.bfloat16)
                    ops.rms_norm(resid, w.layer(i, "ln2"), eps, xn)
                    ops.add_prep(self.moe.forward(i, xn), resid, nxt, xw, ss_1)
                    ss = ss_1
            else:
                w_gu, shg = self._dgw(i, "w_gu")
                act = self._buf("act", (T, w_gu.shape[0] // 2), torch.bfloat16)
                ops.dg_swiglu(xw, w_gu, ss, eps, act, wshuf=shg)
                ss = self._resid_proj("down", act, self._dgw(i, "w_down"), resid, nxt, xw, ss_t, ss_1,
                                      self._row_major(i, "w_down"))
        n = b.num_seqs
        if b.kind == "decode":
            xl, sl = xw, ss
        else:
            xl, sl = xw.index_select(0, b.last_idx), ss.index_select(0, b.last_idx)
        ids = self.last_ids[:n]
        keys = self._buf("keys", (n,), torch.int64)
        tk = self._buf("tile_keys", (n * (self.vocab_shard // 16),), torch.int64)
        logits = self._buf("logits", (n, self.vocab_shard), torch.float32) if b.need_logits or b.filtered else None
        head, hsh = self._lm_head(n)
        ops.dg_argmax(xl, head, sl, eps, b.temps, b.seeds, b.step, tk, keys, ids,
                      self.tp_rank * self.vocab_shard, logits, wshuf=hsh)
        return self._finish_sampling(b, ids, keys, logits)

    def _forward_general_fused(self, b: ForwardBatch, kv: KVCache, mgs: dict) -> torch.Tensor:
        """Decode steps of 20..256 rows: the fused path's dataflow (deferred RMSNorm, epilogues in the GEMMs) on
        the medium-M GEMM -- qkv (+ RoPE, paged K/V write) -> attention -> o (+ residual, ln2 prep) -> gate_up
        (+ SwiGLU) -> down (+ residual, next-ln1 prep), each projection ONE mgemm launch whose last k-split
        workgroup per column group reduces the fp32 split slabs and runs the epilogue."""
        cfg, w = self.cfg, self.w
        T, d, eps = b.num_tokens, cfg.hidden_size, cfg.rms_eps
        resid = self._buf("resid", (T, d), torch.float32)
        xw = self._buf("xw", (T, d), torch.bfloat16)
        ss_t = self._buf("ss_t", (T, d // 16), torch.float32)
        ss_1 = self._buf("ss_1", (T, 1), torch.float32)
        q = self._buf("q", (T, self.hq, self.D), torch.bfloat16)
        attn = self._buf("attn", (T, self.hq, self.D), torch.bfloat16)
        ops.embed_prep(b.input_ids, w["embed"], resid, w.layer(0, "ln1"), xw, ss_1, b.src, self.last_ids)
        ss = ss_1
        for i in range(cfg.num_layers):
            nxt = w.layer(i + 1, "ln1") if i + 1 < cfg.num_layers else w["norm"]
            ops.dg_qkv(xw, self.dgw[(i, "wqkv")], ss, eps, b.positions, b.slot_mapping, self.cos_sin, q, kv.k[i],
                       kv.v[i], self.hq, self.hkv, wshuf=True, mg=mgs["qkv"])
            self._attention(b, kv, i, q, attn)
            ops.dg_resid(attn.view(T, self.hq * self.D), self.dgw[(i, "wo")], resid, w.layer(i, "ln2"), xw, ss_t,
                         wshuf=True, mg=mgs["o"])
            w_gu = self.dgw[(i, "w_gu")]
            act = self._buf("act", (T, w_gu.shape[0] // 2), torch.bfloat16)
            ops.dg_swiglu(xw, w_gu, ss_t, eps, act, wshuf=True, mg=mgs["gu"])
            ops.dg_resid(act, self.dgw[(i, "w_down")], resid, nxt, xw, ss_t, wshuf=True, mg=mgs["down"])
            ss = ss_t
        # normalise first: the lm_head's own row-scale prologue (4 waves x 16 rows of partial sums behind its weight
        # loads) cost 295 vs 230 us at 64 rows (profiles/r3/prof_all64.csv)
        x = self._buf("x", (T, d), torch.bfloat16)
        ops.rownorm(xw, ss, eps, x)
        return self.sample(b, x)

    # ------------------------------------------------------------------------------------------
    def _forward_general(self, b: ForwardBatch, kv: KVCache) -> torch.Tensor:
        cfg, w = self.cfg, self.w
        T = b.num_tokens
        d = cfg.hidden_size
        eps = cfg.rms_eps
        resid = self._buf("resid", (T, d), torch.float32)
        x = self._buf("x", (T, d), torch.bfloat16)
        q = self._buf("q", (T, self.hq, self.D), torch.bfloat16)
        attn = self._buf("attn", (T, self.hq, self.D), torch.bfloat16)
        # pipelined decode rows read their token from the previous step's samples on the device
        src = b.src if b.src is not None and b.kind == "decode" else None
        ops.embed_rms_norm(b.input_ids, w["embed"], resid, w.layer(0, "ln1"), eps, x, src,
                           self.last_ids if src is not None else None)
        pg_gu = self._pg_gate_up(T) if b.kind != "decode" else None
        gu_plan = None
        if MG_FUSED_GU and self.dgw and self.device.type != "cpu" and not cfg.is_moe and T <= 256:
            gu_plan = (self._mg_plan(b, names=("gu",), need_all=False, any_kind=True) or {}).get("gu")
        if gu_plan is not None:
            xw = self._buf("xw", (T, d), torch.bfloat16)
            ss_p = self._buf("ss_pgu", (T, 4 if d % 32 == 0 else 1), torch.float32)
        # single-copy models past the medium-M range: QKV + RoPE + paged K/V write in one prefill-GEMM launch (the
        # pgemm path would write fp32 k-split slabs that rope_cache then reads: Mixtral 4 x 128 tokens, rope 9.4 ->
        # 19.8 us per layer, profiles/r6/prof_mixtral_prefill_4x128_r6b.csv)
        pg_qkv = None
        if self.single_copy and T >= ops.PGEMM_MIN_M and b.kind != "decode" and self.device.type != "cpu":
            pick = ops.choose_pgemm(T, (self.hq + 2 * self.hkv) * self.D, d, align=128, force=True)
            pg_qkv = None if pick is None else pick[0]
        for i in range(cfg.num_layers):
            if pg_qkv is not None:
                ops.pg_qkv(x, self.dgw[(i, "wqkv")], None, eps, b.positions, b.slot_mapping, self.cos_sin, q, kv.k[i],
                           kv.v[i], self.hq, self.hkv, pg_qkv)
            else:
                qkv = self._linear("qkv", x, self._row_major(i, "wqkv"), wshuf=self._shuf(i, "wqkv"))
                ops.rope_cache(qkv, b.positions, b.slot_mapping, self.cos_sin, q, kv.k[i], kv.v[i], self.hq,
                               self.hkv, perm=True, decode=ROPE_DECODE_ROWS and b.kind == "decode")
            self._attention(b, kv, i, q, attn)
            o = self._linear("o", attn.view(T, self.hq * self.D), self._row_major(i, "wo"), reduce=True,
                             wshuf=self._shuf(i, "wo"))
            if gu_plan is not None:
                # deferred norm into gate_up + SwiGLU epilogue (one mgemm launch instead of GEMM + swiglu)
                ops.add_prep(o, resid, w.layer(i, "ln2"), xw, ss_p)
                w_gu = self.dgw[(i, "w_gu")]
                act = self._buf("act", (T, w_gu.shape[0] // 2), torch.bfloat16)
                ops.dg_swiglu(xw, w_gu, ss_p, eps, act, wshuf=True, mg=gu_plan)
                mlp = self._linear("down", act, self._row_major(i, "w_down"), reduce=True, wshuf=self._shuf(i, "w_down"))
            elif cfg.is_moe:
                ops.add_rms_norm(o, resid, w.layer(i, "ln2"), eps, x)
                mlp = self.moe.forward(i, x)
            else:
                ops.add_rms_norm(o, resid, w.layer(i, "ln2"), eps, x)
                if pg_gu is not None:
                    # gate_up + SwiGLU in one prefill-GEMM launch on the preshuffled copy (no [T, 2F] intermediate)
                    w_gu = self.dgw[(i, "w_gu")]
                    act = self._buf("act", (T, w_gu.shape[0] // 2), torch.bfloat16)
                    ops.pg_swiglu(x, w_gu, None, eps, act, pg_gu)
                else:
                    gu = self._linear("gu", x, self._row_major(i, "w_gu"), wshuf=self._shuf(i, "w_gu"))
                    F = gu.shape[-1] // 2
                    act = self._buf("act", (T, F), torch.bfloat16)
                    ops.swiglu(gu, act, interleaved=True)
                mlp = self._linear("down", act, self._row_major(i, "w_down"), reduce=True, wshuf=self._shuf(i, "w_down"))
            nxt = w.layer(i + 1, "ln1") if i + 1 < cfg.num_layers else w["norm"]
            ops.add_rms_norm(mlp, resid, nxt, eps, x)
        return self.sample(b, x)

    def sample(self, b: ForwardBatch, x: torch.Tensor) -> torch.Tensor:
        """Fused lm_head + greedy/Gumbel sampling on each sequence's last row."""
        n = b.num_seqs
        xl = x if b.kind == "decode" else x.index_select(0, b.last_idx)
        ids = self.last_ids[:n]
        keys = self._buf("keys", (n,), torch.int64)
        ntiles = self.vocab_shard // 16
        logits = self._buf("logits", (n, self.vocab_shard), torch.float32) if b.need_logits or b.filtered else None
        if self.fused and n <= SKINNY_MAX_M:
            # the decode lm_head kernel (row-tile variants for wide batches), on already-normalised rows
            tk = self._buf("tile_keys", (n * ntiles,), torch.int64)
            head, hsh = self._lm_head(n)
            ops.dg_argmax(xl, head, None, self.cfg.rms_eps, b.temps, b.seeds, b.step, tk, keys, ids,
                          self.tp_rank * self.vocab_shard, logits, wshuf=hsh)
            return self._finish_sampling(b, ids, keys, logits)
        if n <= SKINNY_MAX_M:
            tk = self._buf("tile_keys", (n * ntiles,), torch.int64)
            ops.lm_head_sample(xl, self.w["lm_head"], b.temps, b.seeds, b.step, tk, keys, ids,
                               self.tp_rank * self.vocab_shard, logits)
            return self._finish_sampling(b, ids, keys, logits)
        # wide batches (> 64 rows): the lm_head becomes compute-shaped -- one library GEMM into fp32
        # logits, then the fused epilogue's greedy / Gumbel-max keys over each row
        logits = self._buf("logits", (n, self.vocab_shard), torch.float32)
        ops.linear_splitk(xl.contiguous(), self.w["lm_head"], logits.view(1, n, self.vocab_shard))
        ops.logits_argmax(logits, b.temps, b.seeds, b.step, keys, ids, self.tp_rank * self.vocab_shard)
        return self._finish_sampling(b, ids, keys, logits)

    def _finish_sampling(self, b: ForwardBatch, ids, keys, logits) -> torch.Tensor:
        """TP combine of the fused sampler's keys, then the top-k / top-p resampler for rows that ask."""
        ids = self._combine_tp(ids, keys, logits)
        if b.filtered:
            full = logits
            if self._tp_active():
                g = self.tp.all_gather(logits)  # [tp * n, V / tp]
                full = g.view(self.tp_size, logits.shape[0], -1).permute(1, 0, 2).reshape(logits.shape[0], -1)
            ops.sample_filtered(full, b.temps, b.top_k, b.top_p, b.seeds, b.step, ids)
        return ids

    def _combine_tp(self, ids, keys, logits) -> torch.Tensor:
        if self._tp_active():
            self.tp.argmax_keys(keys, ids)  # global argmax over the vocabulary shards (one kernel on xGMI)
        self.last_logits = logits
        return ids
