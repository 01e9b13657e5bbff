"""Decode weight layout (the contract of csrc/kernels/decode_gemm.hip).

* ``wqkv``: rows of every q and k head are permuted so that 16-row tile j of a head holds
  dims 8j..8j+7 followed by dims D/2+8j..D/2+8j+7 -- both halves of each rotate-half RoPE
  pair in one MFMA tile (lanes l and l^32), so RoPE runs in the GEMM epilogue.  v heads stay
  in natural order.
* ``w_gu``: gate rows 8j..8j+7 followed by up rows 8j..8j+7 in tile j, so SwiGLU runs in the
  GEMM epilogue.
The library-GEMM (prefill) path reads the same tensors through the ``perm`` / ``interleaved``
flags of ``rope_cache`` / ``swiglu``.  The layout is applied once, in place, per TP shard.
"""
from __future__ import annotations

import torch

from .weights import ModelWeights


def _pair_perm(half: int) -> torch.Tensor:
    """Row order of one interleaved block: position p -> source row."""
    p = torch.arange(2 * half)
    jt, r = p // 16, p % 16
    return torch.where(r < 8, 8 * jt + r, half + 8 * jt + (r - 8))


def qkv_perm(hq: int, hkv: int, D: int) -> torch.Tensor:
    head = _pair_perm(D // 2)
    parts = [h * D + head for h in range(hq + hkv)]
    parts.append(torch.arange((hq + hkv) * D, (hq + 2 * hkv) * D))
    return torch.cat(parts)


def gu_perm(F: int) -> torch.Tensor:
    return _pair_perm(F)


def _inverse(perm: torch.Tensor) -> torch.Tensor:
    inv = torch.empty_like(perm)
    inv[perm] = torch.arange(perm.numel())
    return inv


def apply_decode_layout(w: ModelWeights) -> None:
    if getattr(w, "layout", "natural") == "decode":
        return
    cfg, tp = w.cfg, w.shard.tp_size
    hq, hkv = cfg.num_heads // tp, cfg.num_kv_heads // tp
    for i in range(cfg.num_layers):
        k = f"layers.{i}.wqkv"
        t = w.tensors[k]
        w.tensors[k] = t.index_select(0, qkv_perm(hq, hkv, cfg.head_dim).to(t.device)).contiguous()
        k = f"layers.{i}.w_gu"
        if k in w.tensors:
            t = w.tensors[k]
            w.tensors[k] = t.index_select(0, gu_perm(t.shape[0] // 2).to(t.device)).contiguous()
    w.layout = "decode"


def natural_tensors(w: ModelWeights) -> dict:
    """Tensors in natural (HF) row order, whatever layout ``w`` is stored in (reference model, export): preshuffled
    tensors (decode_weights="replace") are unshuffled first, then the decode row permutations undone."""
    shuffled = getattr(w, "shuffled", frozenset())
    if getattr(w, "layout", "natural") != "decode" and not shuffled:
        return w.tensors
    cfg, tp = w.cfg, w.shard.tp_size
    hq, hkv = cfg.num_heads // tp, cfg.num_kv_heads // tp
    out = dict(w.tensors)
    for k in shuffled:
        out[k] = unshuffle(out[k])
    if getattr(w, "layout", "natural") != "decode":
        return out
    for i in range(cfg.num_layers):
        k = f"layers.{i}.wqkv"
        t = out[k]
        out[k] = t.index_select(0, _inverse(qkv_perm(hq, hkv, cfg.head_dim)).to(t.device))
        k = f"layers.{i}.w_gu"
        if k in out:
            t = out[k]
            out[k] = t.index_select(0, _inverse(gu_perm(t.shape[0] // 2)).to(t.device))
    return out


# ---- MFMA-preshuffled weight stream (csrc/kernels/decode_gemm.hip, DecodeEpi::wshuf) -----------------
def preshuffle(w: torch.Tensor) -> torch.Tensor:
    """[..., N, K] row-major -> the same elements ordered [N/16][K/32][lane 64][8] per leading index (an expert
    stack [E, N, K] is preshuffled per expert): block (t, kb) holds rows 16t.. and k 32kb.. with lane l =
    16 * (k8 group) + row, i.e. exactly the MFMA 16x16x32 A-fragment order, so one wave load instruction reads 1 KB
    contiguous.  Returned with the original shape."""
    *lead, N, K = w.shape
    L = len(lead)
    perm = list(range(L)) + [L, L + 2, L + 3, L + 1, L + 4]
    return w.reshape(*lead, N // 16, 16, K // 32, 4, 8).permute(*perm).contiguous().view(w.shape)


def unshuffle(w: torch.Tensor) -> torch.Tensor:
    *lead, N, K = w.shape
    L = len(lead)
    perm = list(range(L)) + [L, L + 3, L + 1, L + 2, L + 4]
    return w.reshape(*lead, N // 16, K // 32, 4, 16, 8).permute(*perm).contiguous().view(w.shape)
