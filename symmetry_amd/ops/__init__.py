"""Op layer: one Python entry point per kernel.

Dispatch rule (no silent fallback): a GPU tensor always runs the CDNA4 HIP
kernel from ``_C.so`` (``torch.ops.symmetry_amd.*``) and raises if the
library is not built/loadable; a CPU tensor runs the fp32 torch reference
(:mod:`symmetry_amd.ops.reference`).  The only exception is the explicit
``SYMMETRY_OPS=torch`` switch: the "unoptimised native" baseline B1
 that runs the torch reference ops, eagerly, on the GPU.  All ops write into caller-provided
outputs and allocate nothing on the GPU path, so the model runner can capture
them in a hipGraph.
"""
from __future__ import annotations

import os

import torch

from . import _native, reference

_TORCH_MODE = os.environ.get("SYMMETRY_OPS", "native").lower() == "torch"


def torch_mode() -> bool:
    """True under SYMMETRY_OPS=torch (eager torch ops on the GPU: baseline B1, no hipGraphs)."""
    return _TORCH_MODE

__all__ = [
    "native_available",
    "rms_norm",
    "add_rms_norm",
    "embed_rms_norm",
    "rope_cache",
    "attn_decode",
    "attn_prefill",
    "skinny_gemm",
    "mgemm",
    "choose_mgemm",
    "lm_head_sample",
    "swiglu",
    "moe_route_permute",
    "grouped_skinny",
    "moe_combine",
    "dg_f32",
    "dg_qkv",
    "dg_resid",
    "dg_swiglu",
    "dg_argmax",
    "embed_prep",
    "add_prep",
    "rownorm",
    "sample_filtered",
    "linear",
    "lib_splits",
    "linear_splitk",
    "choose_splits",
]


def native_available() -> bool:
    return _native.available()


def _gpu(t: torch.Tensor) -> bool:
    return t.device.type != "cpu" and not _TORCH_MODE


def rms_norm(x, w, eps, out):
    if _gpu(out):
        return _native.ops().rms_norm(x, w, float(eps), out)
    return reference.rms_norm(x, w, eps, out)


def add_rms_norm(delta, residual, w, eps, out):
    if _gpu(residual):
        return _native.ops().add_rms_norm(delta, residual, w, float(eps), out)
    return reference.add_rms_norm(delta, residual, w, eps, out)


def embed_rms_norm(ids, table, residual, w, eps, out, src=None, prev=None):
    """``src``/``prev``: rows with src >= 0 take the token prev[src] (the previous step's on-device sample)."""
    if _gpu(residual):
        return _native.ops().embed_rms_norm(ids, table, residual, w, float(eps), out, src, prev)
    return reference.embed_rms_norm(reference.resolve_ids(ids, src, prev), table, residual, w, eps, out)


def rope_cache(qkv, positions, slots, cos_sin, q_out, k_cache, v_cache, Hq, Hkv, perm=False, decode=False):
    """RoPE + paged K/V write.  ``decode``: rows of different sequences (a decode step): skips the prefill
    form's 8-row V token-run grouping for more workgroups per row."""
    if _gpu(q_out):
        return _native.ops().rope_cache(qkv, positions, slots, cos_sin, q_out, k_cache, v_cache, int(Hq), int(Hkv),
                                        bool(perm), bool(decode))
    return reference.rope_cache(qkv, positions, slots, cos_sin, q_out, k_cache, v_cache, Hq, Hkv, perm)


ATTN_DECODE_PART = 256  # context tokens per split-KV partition of attn_decode (csrc/kernels/attn_decode.h PART)


def attn_decode(q, k_cache, v_cache, block_tables, ctx_lens, out, tmp_o, tmp_ml, counters, scale):
    """Split-KV paged decode attention.  ``counters``: int32 [>= num_seqs * Hkv], zero-initialised once;
    the kernel re-arms it (graph-replay safe)."""
    if _gpu(q):
        return _native.ops().attn_decode(q, k_cache, v_cache, block_tables, ctx_lens, out, tmp_o, tmp_ml, counters,
                                         float(scale))
    return reference.attn_decode(q, k_cache, v_cache, block_tables, ctx_lens, out, tmp_o, tmp_ml, scale)


def attn_prefill(q, k_cache, v_cache, block_tables, ctx_lens, cu_q, tiles, out, scale):
    if _gpu(q):
        return _native.ops().attn_prefill(q, k_cache, v_cache, block_tables, ctx_lens, cu_q, tiles, out,
                                          float(scale))
    return reference.attn_prefill(q, k_cache, v_cache, block_tables, ctx_lens, cu_q, tiles, out, scale)


def skinny_gemm(x, w, y, variant: int = 0):
    if _gpu(x):
        return _native.ops().skinny_gemm(x, w, y, int(variant))
    return reference.skinny_gemm(x, w, y)


MGEMM_MAX_M = 256
_MGEMM_ON = os.environ.get("SYMMETRY_MGEMM", "1") != "0"  # A/B switch: 0 keeps every prefill on the library


def mgemm(x, w_shuf, y, rw: int):
    """Medium-M (65..256 rows) projection into fp32 split-K slabs y [S, M, N] (the skinny_gemm contract,
    summed by the LinOut consumers); ``w_shuf`` is the MFMA-preshuffled weight (models/layout.py)."""
    if _gpu(x):
        return _native.ops().mgemm(x, w_shuf, y, int(rw))
    return reference.skinny_gemm(x, reference.unshuffled(w_shuf, True), y)


def choose_mgemm(M: int, N: int, K: int, cus: int = 256, fused: bool = False):
    """(rw, S) of mgemm for an [M, K] x [N, K]^T projection, or None where another kernel is the better
    choice.  Measured on MI355X (profiles/mgemm_r2.jsonl, mgemm_small_r2.jsonl; each arm followed by its
    real consumer kernel): up to 64 rows mgemm beats both the split-K skinny GEMM and hipBLASLt on every
    Llama-3-8B projection; above 64 rows it wins for the narrow ones (N <= 8192: qkv / o / down) up to 192
    rows and for long-K or wider ones (down, qkv) up to 256, while the wide gate_up (N = 28672) stays on
    hipBLASLt.  A second wave of workgroups always lost, so only grids of 128..256 workgroups are
    considered, ranked by a linear model fitted to those sweeps: per-workgroup intake (64 rw weight rows +
    M activation rows over the k slice) at a per-CU rate that drops with the LDS ring depth (fewer slots
    at more rows), plus the S fp32 slabs written here and summed by the consumer, plus a fixed cost per
    workgroup spread over the grid."""
    if not _MGEMM_ON or M > MGEMM_MAX_M or K % 64:
        return None
    if M > 64 and (N > 8192 or (M > 192 and K < 8192 and N < 6144)):
        return None
    mt = 2 if M <= 32 else 4 if M <= 64 else 8 if M <= 128 else 16
    a_us_mb, b_us_mb = {2: (11.5, 2.2), 4: (11.5, 2.2), 8: (20.0, 1.0), 16: (30.0, 1.0)}[mt]
    best = None
    for rw in (1, 2, 3, 4):
        if N % (64 * rw) or (mt == 16 and rw > 2):
            continue
        for S in range(1, K // 64 + 1):
            if (K // 64) % S:
                continue
            wgs = N // (64 * rw) * S
            if wgs < cus // 2 or wgs > cus:
                continue
            slabs = b_us_mb * S * M * N * 4 / 1e6
            t = (a_us_mb * (64 * rw + M) * (K // S) * 2 / 1e6 + slabs
                 + 1000.0 / wgs)  # per-workgroup fixed cost (prologue, epilogue), spread over the grid
            if best is None or t < best[0]:
                best = (t, rw, S)
    return None if best is None else (best[1], best[2])


# ---- prefill projection GEMM (csrc/kernels/pgemm.hip): hundreds+ rows on the MFMA-preshuffled weights -------
def pgemm_shape(cfg: int):
    """(BM, BN) of tile config ``cfg`` (tokens x features per 512-thread block), or None."""
    if not native_available():
        return PG_CFG_SHAPES.get(cfg)
    s = _native.ops().pgemm_shape(int(cfg))
    return tuple(s) if s else None


# kept in sync with csrc/kernels/pgemm.hip PG_CFGS (used off-GPU, e.g. by the planner's CPU tests)
PG_CFG_SHAPES = {0: (384, 224), 1: (256, 256), 2: (192, 192), 3: (192, 128), 4: (256, 128), 5: (128, 128),
                 6: (320, 224), 7: (256, 224), 8: (192, 224), 9: (192, 256), 10: (128, 256)}


def pgemm(x, w_shuf, y, cfg: int, S: int = 1, slab=None, counters=None):
    """y [M, N] (bf16 or fp32) = x @ W^T with W MFMA-preshuffled; tile config ``cfg``, ``S`` k-splits (S > 1: fp32
    ``slab`` [S, M, N] scratch + int32 ``counters`` [tiles], zero before the first launch)."""
    if _gpu(x):
        return _native.ops().pgemm(x, w_shuf, y, int(cfg), int(S), slab, counters)
    w = reference.unshuffled(w_shuf, True)
    if y.dim() == 3:  # split-K slabs
        return reference.skinny_gemm(x, w, y)
    y.copy_(x.float() @ w.float().t())
    return y


_PGEMM_ON = os.environ.get("SYMMETRY_PGEMM", "1") != "0"  # A/B switch: 0 keeps long prefills on the library path
PGEMM_MIN_M = int(os.environ.get("SYMMETRY_PGEMM_MIN_M", "257"))  # below: mgemm (medium-M, weight-streaming)
# gate_up + SwiGLU on pgemm for prefill steps of PGEMM_GU_MIN_M..PGEMM_GU_MAX_M rows (one wave of 320 / 384 x 224
# tiles); 384 / 512 rows measured 4 / 1 % slower than the library + swiglu, 600 / 768 rows 4.5 / 3 % faster
# (profiles/r6/prefill_pgemm_ab3.jsonl), 1024+ the library's tiles win (profiles/r6/pgemm_gu_sweep.jsonl)
PGEMM_GU_MIN_M = int(os.environ.get("SYMMETRY_PGEMM_GU_MIN_M", "576"))
PGEMM_GU_MAX_M = int(os.environ.get("SYMMETRY_PGEMM_GU_MAX_M", "896"))


def choose_pgemm(M: int, N: int, K: int, slabs: bool = False, cus: int = 256, align: int = 16, force: bool = False):
    """(cfg, S) of the prefill GEMM for an [M, K] x [N, K]^T projection, or None.  ``slabs``: the consumer can sum
    fp32 split-K slabs (S > 1 allowed; fused epilogues need S = 1).  ``align``: the tile width must be a multiple
    of it (the QKV epilogue writes whole 128-dim heads).  ``force``: plan even where the library would be chosen
    (single-copy weights: the preshuffled layout is all there is).

    Cost model fitted to the 768-row sweeps on MI355X (bench/kernels/bench_pgemm.py, pgemm_probe.py;
    profiles/r6/pgemm_*.jsonl): a k-step (32 deep) of a BM x BN tile is bound by the per-CU LDS-DMA intake --
    ~50 GB/s per CU while at most 3/4 of the CUs stream, ~35 GB/s with all of them (L2 / fabric contention)
    -- or by its MFMAs at ~6.5 TFLOP/s per CU; plus ~3 us of prologue + epilogue per wave of blocks and the
    slabs written for the consumer."""
    if K % 64 or (not force and (not _PGEMM_ON or M < PGEMM_MIN_M)):
        return None
    best = None
    for cfg, (bm, bn) in PG_CFG_SHAPES.items():
        if N % bn or bn % align:
            continue
        for S in ((1, 2, 4) if slabs else (1,)):
            if K % (64 * S):
                continue
            tiles = -(-M // bm) * (N // bn) * S
            waves = -(-tiles // cus)
            busy = min(tiles, cus)
            rate = 50e9 if busy <= 3 * cus // 4 else 35e9
            step = max((bm + bn) * 64 / rate, 2 * bm * bn * 32 / 6.5e12)
            t = waves * (K // S // 32) * step + waves * 3e-6 + (S * M * N * 4 / 10e12 if S > 1 else 0.0)
            if best is None or t < best[0]:
                best = (t, cfg, S)
    return None if best is None else (best[1], best[2])


def _pg_resid_ref(x, W, resid, w_next, xw_out, ss_out):
    M = x.shape[0]
    r = resid[:M]
    r.add_(x.float() @ W.float().t())
    xw_out[:M].copy_((r * w_next.float()).to(xw_out.dtype))
    ss_out[:M].copy_(r.pow(2).view(M, ss_out.shape[1], -1).sum(-1))


def pg_qkv(x, W, ss_in, eps, positions, slots, cos_sin, q_out, k_cache, v_cache, Hq, Hkv, cfg):
    """Prefill QKV projection (W preshuffled, decode row layout) + deferred-norm row scale + RoPE + paged K/V write."""
    if _gpu(x):
        return _native.ops().pg_qkv(x, W, ss_in, float(eps), positions, slots, cos_sin, q_out, k_cache, v_cache,
                                    int(Hq), int(Hkv), int(cfg))
    return reference.dg_qkv(x, reference.unshuffled(W, True), ss_in, eps, positions, slots, cos_sin, q_out, k_cache,
                            v_cache, Hq, Hkv)


def pg_swiglu(x, W, ss_in, eps, act, cfg):
    """Prefill gate_up projection (tile-interleaved gate/up rows, preshuffled) + row scale + SwiGLU -> act."""
    if _gpu(x):
        return _native.ops().pg_swiglu(x, W, ss_in, float(eps), act, int(cfg))
    return reference.dg_swiglu(x, reference.unshuffled(W, True), ss_in, eps, act)


def pg_resid(x, W, resid, w_next, xw_out, ss_out, cfg):
    """Prefill row-parallel projection + residual add + next-norm prep; ss_out [M, N / BN]: one sum-of-squares
    partial per row and block column of tile config ``cfg``."""
    if _gpu(x):
        return _native.ops().pg_resid(x, W, resid, w_next, xw_out, ss_out, int(cfg))
    return _pg_resid_ref(x, reference.unshuffled(W, True), resid, w_next, xw_out, ss_out)


# grouped-expert mode (MoE prefill): tile configs instantiated for it (csrc/kernels/pgemm.hip PG_GRP_CFGS) and the
# epilogues (launchers.h DECODE_EPI_*)
PG_GRP_CFGS = (1, 4, 5, 9, 10)
PG_EPI_F32, PG_EPI_BF16, PG_EPI_SWIGLU_SPLIT = 0, 7, 8


def pg_grouped(xs, W, offsets, e_lo: int, y, epi: int, cfg: int, S: int = 1):
    """Grouped expert GEMM on the prefill GEMM kernel: expert e of W [E, N, K] (MFMA-preshuffled per expert) applied
    to rows [offsets[e_lo + e], offsets[e_lo + e + 1]) of xs [R, K].  epi PG_EPI_SWIGLU_SPLIT: act [R, N / 2] =
    silu(gate) * up of the [gate; up] halves; PG_EPI_BF16: y [R, N]; PG_EPI_F32: y [R, N] fp32 or [S, R, N] k-split
    partial slabs (LinOut).  Rows outside the segments are left untouched."""
    if _gpu(xs):
        return _native.ops().pg_grouped(xs, W, offsets, int(e_lo), y, int(epi), int(cfg), int(S))
    from ..models.layout import unshuffle

    offs = [int(v) for v in offsets[e_lo: e_lo + W.shape[0] + 1].tolist()]
    for e in range(W.shape[0]):
        a, b = offs[e], offs[e + 1]
        if b <= a:
            continue
        p = xs[a:b].float() @ unshuffle(W[e]).float().t()
        if epi == PG_EPI_SWIGLU_SPLIT:
            F = p.shape[1] // 2
            p = torch.nn.functional.silu(p[:, :F]) * p[:, F:]
        if y.dim() == 3:
            y[:, a:b] = 0
            y[0, a:b] = p
        else:
            y[a:b] = p.to(y.dtype)
    return y


def choose_pg_grouped(R: int, N: int, K: int, E: int, slabs: bool = False, cus: int = 256, even_wn: bool = False):
    """(cfg, S) of the grouped prefill GEMM for R routed rows over E local experts ([N, K] weights each), or None.
    The m-tile count is not known on the host (segment bounds live on the device): the estimate ceil(R / BM) + E / 2
    covers one partial tile per expert on average; otherwise choose_pgemm's cost model.  ``even_wn``: the split
    SwiGLU epilogue pairs a wave's tiles."""
    if K % 64:
        return None
    best = None
    for cfg in PG_GRP_CFGS:
        bm, bn = PG_CFG_SHAPES[cfg]
        if N % bn or (even_wn and (bn // 32) % 2):
            continue
        for S in ((1, 2, 4) if slabs else (1,)):
            if K % (64 * S):
                continue
            mt = -(-R // bm) + E // 2
            tiles = mt * (N // bn) * S
            waves = -(-tiles // cus)
            busy = min(tiles, cus)
            rate = 50e9 if busy <= 3 * cus // 4 else 35e9
            step = max((bm + bn) * 64 / rate, 2 * bm * bn * 32 / 6.5e12)
            t = waves * (K // S // 32) * step + waves * 3e-6 + (S * R * N * 4 / 10e12 if S > 1 else 0.0)
            if best is None or t < best[0]:
                best = (t, cfg, S)
    return None if best is None else (best[1], best[2])


def lm_head_sample(x, w, temps, seeds, step, tile_keys, out_keys, out_ids, n_offset=0, logits=None):
    if _gpu(x):
        return _native.ops().lm_head_sample(x, w, temps, seeds, step, tile_keys, out_keys, out_ids, int(n_offset),
                                            logits)
    return reference.lm_head_sample(x, w, temps, seeds, step, tile_keys, out_keys, out_ids, n_offset, logits)


def swiglu(gu, out, interleaved=False):
    if _gpu(out):
        return _native.ops().swiglu(gu, out, bool(interleaved))
    return reference.swiglu(gu, out, interleaved)


# ---- fused decode GEMMs: M <= 64 rows, weights in the decode layout (models/layout.py) ----------
# ss_in: per-(row, tile) sums of squares of the residual [>=M, tiles] (deferred RMSNorm) or None.
def dg_f32(x, W, ss_in, eps, y, wshuf=False):
    if _gpu(x):
        return _native.ops().dg_f32(x, W, ss_in, float(eps), y, bool(wshuf))
    return reference.dg_f32(x, reference.unshuffled(W, wshuf), ss_in, eps, y)


_KS_WS = {}
KS_WS_FLOATS = 1 << 20  # 4 MB: 4096 (tile, split) partials
KS_WS_TILES = 1 << 14


def decode_ks_ws(device):
    """The decode GEMMs' split-K workspace on ``device`` (fp32 partials + per-tile arrival counters, zeroed
    once and re-armed by the kernel): one per device for the process, so its address is stable across hipGraph
    captures.  Call it before capturing (the engine's model init does)."""
    key = (device.type, device.index)
    ws = _KS_WS.get(key)
    if ws is None:
        ws = (torch.empty(KS_WS_FLOATS, dtype=torch.float32, device=device),
              torch.zeros(KS_WS_TILES, dtype=torch.int32, device=device), 0)
        _KS_WS[key] = ws
    return ws


# mg: (slab [S, M, N] fp32, counters int32, rw) -> run the projection on the medium-M GEMM (mgemm, up to 256
# rows, preshuffled weights) with the same fused epilogue after an in-launch split-K reduction.  Without mg the
# decode GEMM gets the device's split-K workspace (decode_gemm.hip go_xres: k split across workgroups where
# whole 16-row tiles would leave CUs idle).
def dg_qkv(x, W, ss_in, eps, positions, slots, cos_sin, q_out, k_cache, v_cache, Hq, Hkv, wshuf=False, mg=None):
    if _gpu(x):
        slab, cnt, rw = mg if mg is not None else decode_ks_ws(x.device)
        return _native.ops().dg_qkv(x, W, ss_in, float(eps), positions, slots, cos_sin, q_out, k_cache, v_cache,
                                    int(Hq), int(Hkv), bool(wshuf), slab, cnt, int(rw))
    return reference.dg_qkv(x, reference.unshuffled(W, wshuf), ss_in, eps, positions, slots, cos_sin, q_out,
                            k_cache, v_cache, Hq, Hkv)


def dg_resid(x, W, resid, w_next, xw_out, ss_out, wshuf=False, mg=None):
    if _gpu(x):
        slab, cnt, rw = mg if mg is not None else decode_ks_ws(x.device)
        return _native.ops().dg_resid(x, W, resid, w_next, xw_out, ss_out, bool(wshuf), slab, cnt, int(rw))
    return reference.dg_resid(x, reference.unshuffled(W, wshuf), resid, w_next, xw_out, ss_out)


def dg_swiglu(x, W, ss_in, eps, act, wshuf=False, mg=None):
    if _gpu(x):
        slab, cnt, rw = mg if mg is not None else decode_ks_ws(x.device)
        return _native.ops().dg_swiglu(x, W, ss_in, float(eps), act, bool(wshuf), slab, cnt, int(rw))
    return reference.dg_swiglu(x, reference.unshuffled(W, wshuf), ss_in, eps, act)


def dg_argmax(x, W, ss_in, eps, temps, seeds, step, tile_keys, out_keys, out_ids, n_offset=0, logits=None,
              wshuf=False):
    if _gpu(x):
        return _native.ops().dg_argmax(x, W, ss_in, float(eps), temps, seeds, step, tile_keys, out_keys, out_ids,
                                       int(n_offset), logits, bool(wshuf))
    return reference.dg_argmax(x, reference.unshuffled(W, wshuf), ss_in, eps, temps, seeds, step, tile_keys,
                               out_keys, out_ids, n_offset, logits)


def embed_prep(ids, table, resid, w, xw, ss, src=None, prev=None):
    """Embedding gather + deferred-norm prep; with ``src``/``prev`` a row whose src >= 0 takes its token
    from ``prev[src]`` (the previous step's device-resident samples: pipelined decode)."""
    if _gpu(resid):
        return _native.ops().embed_prep(ids, table, resid, w, xw, ss, src, prev)
    return reference.embed_prep(ids, table, resid, w, xw, ss, src, prev)


def add_prep(delta, resid, w, xw, ss):
    if _gpu(resid):
        return _native.ops().add_prep(delta, resid, w, xw, ss)
    return reference.add_prep(delta, resid, w, xw, ss)


def rownorm(xw, ss, eps, out):
    if _gpu(out):
        return _native.ops().rownorm(xw, ss, float(eps), out)
    return reference.rownorm(xw, ss, eps, out)


def moe_route_permute(logits, x, k, E, ids, w, counts, offsets, cursor, xs, dst):
    if _gpu(x):
        return _native.ops().moe_route_permute(logits, x, int(k), int(E), ids, w, counts, offsets, cursor, xs, dst)
    return reference.moe_route_permute(logits, x, k, E, ids, w, counts, offsets, cursor, xs, dst)


def moe_route(logits, T, k, E, ids, w):
    if _gpu(ids):
        return _native.ops().moe_route(logits, int(T), int(k), int(E), ids, w)
    return reference.moe_route(logits, T, k, E, ids, w)


def moe_align(ids, G, counts, offsets, cursor):
    if _gpu(ids):
        return _native.ops().moe_align(ids, int(G), counts, offsets, cursor)
    return reference.moe_align(ids, G, counts, offsets, cursor)


def moe_scatter(x, ids, k, G, offsets, cursor, xs, dst, src_tok=None):
    """Rows of x into group segments starting at offsets[g] (``cursor`` zero); dst[a] = row of assignment a."""
    if _gpu(x):
        return _native.ops().moe_scatter(x, ids, int(k), int(G), offsets, cursor, xs, dst, src_tok)
    return reference.moe_scatter(x, ids, k, G, offsets, cursor, xs, dst, src_tok)


GROUPED_BF16, GROUPED_F32, GROUPED_SWIGLU = 0, 1, 2
GROUPED_PRESHUFFLED = 4  # + mode: W MFMA-preshuffled per expert (models/layout.py::preshuffle)


def grouped_gemm(xs, W, offsets, e0, y, mode):
    """Grouped MFMA GEMM over expert segments for any routed row count (segment bounds on the device)."""
    if _gpu(xs):
        return _native.ops().grouped_gemm(xs, W, offsets, int(e0), y, int(mode))
    return reference.grouped_gemm(xs, W, offsets, e0, y, mode)


def grouped_stream_policy(p: int) -> None:
    """grouped_gemm's weight-streaming kernel on row-major weights (csrc/kernels/moe.hip grouped_stream_kernel):
    0 never, 1 where it measured faster (default), 2 always (where the shapes tile); + 10 x (2 or 4): weight tiles
    per wave instead of the automatic choice.  Preshuffled weights always take the streaming kernel."""
    _native.ops().grouped_stream_policy(int(p))


def moe_router(x, Wr, logits):
    """Router logits fp32 [T, 16] = x [T, d] @ Wr[16, d]^T (router rows padded to 16; csrc/kernels/moe.hip)."""
    if _gpu(x):
        return _native.ops().moe_router(x, Wr, logits)
    logits.copy_(x.float() @ Wr.float().t())
    return logits


def grouped_skinny(xs, W, offsets, e0, y, wshuf: bool = False):
    """``wshuf``: W MFMA-preshuffled per expert (models/layout.py::preshuffle)."""
    if _gpu(xs):
        return _native.ops().grouped_skinny(xs, W, offsets, int(e0), y, bool(wshuf))
    if wshuf:
        from ..models.layout import unshuffle

        W = unshuffle(W)
    return reference.grouped_skinny(xs, W, offsets, e0, y)


def moe_decode_route(resid, lnw, eps, Wr, k, ids, w, counts, offsets, cursor, xs, dst):
    """Decode MoE routing in one launch: RMSNorm(resid) rows -> router logits -> top-k -> expert segments ->
    xs (the normalised rows permuted into their segments, token order within a segment)."""
    if _gpu(resid):
        return _native.ops().moe_decode_route(resid, lnw, float(eps), Wr, int(k), ids, w, counts, offsets, cursor,
                                              xs, dst)
    return reference.moe_decode_route(resid, lnw, eps, Wr, k, ids, w, counts, offsets, cursor, xs, dst)


def moe_combine_prep(y, dst, ids, E, w, k, resid, w_next, xw, ss):
    """moe_combine over every expert fused with add_prep (decode, experts all on this rank)."""
    if _gpu(resid):
        return _native.ops().moe_combine_prep(y, dst, ids, int(E), w, int(k), resid, w_next, xw, ss)
    return reference.moe_combine_prep(y, dst, ids, E, w, k, resid, w_next, xw, ss)


def moe_combine(y, dst, ids, e_lo, e_hi, w, k, out, accumulate=False):
    if _gpu(out):
        return _native.ops().moe_combine(y, dst, ids, int(e_lo), int(e_hi), w, int(k), out, bool(accumulate))
    return reference.moe_combine(y, dst, ids, e_lo, e_hi, w, k, out, accumulate)


def moe_owner_pack(y, dst, ids, w, e_lo, e_hi, k, S, cursor, send, side):
    """Expert parallelism over replicated tokens: the weighted partial of each token's local experts, one fp32
    row per token, grouped by slice owner (t // S) into ``send`` [N * cap, d]; ``cursor`` [N] = rows per owner."""
    if _gpu(send):
        return _native.ops().moe_owner_pack(y, dst, ids, w, int(e_lo), int(e_hi), int(k), int(S), cursor, send, side)
    return reference.moe_owner_pack(y, dst, ids, w, e_lo, e_hi, k, S, cursor, send, side)


def moe_owner_combine(recv, side, rcnt, Tr, pos, out):
    """The slice owner's rank-ordered sum of the received partials -> bf16 [S, d] (rows >= Tr zero)."""
    if _gpu(out):
        return _native.ops().moe_owner_combine(recv, side, rcnt, int(Tr), pos, out)
    return reference.moe_owner_combine(recv, side, rcnt, Tr, pos, out)


def sample_filtered(logits, temps, top_k, top_p, seeds, step, out_ids):
    """Resample rows that request top-k / top-p (temperature > 0) from full-vocab fp32 logits."""
    if _gpu(logits):
        return _native.ops().sample_filtered(logits, temps, top_k, top_p, seeds, step, out_ids)
    return reference.sample_filtered(logits, temps, top_k, top_p, seeds, step, out_ids)


def logits_argmax(logits, temps, seeds, step, out_keys, out_ids, n_offset=0):
    """Greedy / temperature (Gumbel-max) sampling over fp32 logits [B, V]: the keys and RNG of the fused
    lm_head epilogue, for decode batches wider than the fused kernels (> 64 rows)."""
    if _gpu(logits):
        return _native.ops().logits_argmax(logits, temps, seeds, step, int(n_offset), out_keys, out_ids)
    return reference.logits_argmax(logits, temps, seeds, step, out_keys, out_ids, n_offset)


def linear(x: torch.Tensor, w: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    """Plain library GEMM ``x @ w.T`` for prefill-sized M (hipBLASLt through torch, the library heuristic; a
    tuned-solution table measured neutral end to end and was removed: profiles/r4/blaslt_tuned_ab.jsonl)."""
    return torch.matmul(x, w.t(), out=out)


def lib_splits(M: int, N: int, K: int) -> int:
    """k split of a library prefill GEMM run as one strided-batched GEMM into fp32 slabs (linear_splitk).
    The narrow projections (N <= 8192) of 257..768-token prefills (and long-K ones up to 1536) leave most CUs
    idle as one GEMM; measured (profiles/prefill_splitk_lib_r2.jsonl, each with its consumer): 512 tokens
    down 81 -> 65 us (S = 4), o 34 -> 32, qkv 32 -> 28 (S = 2); 1280 tokens down 141 -> 132 (S = 2); beyond,
    the single GEMM wins."""
    if N > 8192 or N < 256 or not _MGEMM_ON:  # (N < 256: MoE routers keep their single GEMM)
        return 1
    if M <= 768:
        return 4 if K >= 8192 else 2
    if M <= 1536 and K >= 8192:
        return 2
    return 1


def linear_splitk(x: torch.Tensor, w: torch.Tensor, y: torch.Tensor) -> None:
    """y [S, M, N] fp32 = the S k-slice partial products of x @ w.T (the skinny_gemm slab contract) as one
    strided-batched library GEMM with fp32 output (hipBLASLt), summed by the LinOut consumer."""
    S, M, N = y.shape
    K = x.shape[1]
    if x.device.type == "cpu":
        return reference.skinny_gemm(x, w, y)
    kc = K // S
    torch.bmm(x.view(M, S, kc).permute(1, 0, 2), w.view(N, S, kc).permute(1, 2, 0), out_dtype=torch.float32, out=y)


def choose_splits(N: int, K: int, target_wgs: int = 1024, min_k_per_wave: int = 128) -> int:
    """k-split S of the skinny GEMM: the smallest divisor of K/256 giving >= target_wgs workgroups,
    keeping each wave's k range >= min_k_per_wave (2 MFMA k-blocks)."""
    tiles = max(1, N // 16)
    if K % 256:
        raise ValueError(f"skinny GEMM needs K % 256 == 0, got {K}")
    best = 1
    for s in range(1, K // 256 + 1):
        if (K // 256) % s or (K // s) // 4 < min_k_per_wave:
            continue
        best = s
        if tiles * s >= target_wgs:
            break
    return best
