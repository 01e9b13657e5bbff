"""Naive full-recompute fp32 forward of the same weights (no KV cache, no paging,
no fused ops): the independent oracle the engine's outputs are tested against.
"""
from __future__ import annotations

import math

import torch

from ..ops.reference import rope_table
from .weights import ModelWeights


def _rms(x, w, eps):
    return x * torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + eps) * w.float()


def _moe(cfg, w, i, h, gaps=None):
    router = w.layer(i, "router").float()
    w13 = w.layer(i, "w13").float()
    w2 = w.layer(i, "w2").float()
    logits = h @ router.t()
    if gaps is not None and cfg.top_k < cfg.num_experts:  # margin of the k-th choice over the (k+1)-th
        top = logits.topk(cfg.top_k + 1, dim=-1).values
        gaps.append(top[:, cfg.top_k - 1] - top[:, cfg.top_k])
    topv, topi = logits.topk(cfg.top_k, dim=-1)
    gates = torch.softmax(topv, dim=-1)
    out = torch.zeros_like(h)
    F = cfg.intermediate_size
    for t in range(h.shape[0]):
        for j in range(cfg.top_k):
            e = int(topi[t, j])
            gu = w13[e] @ h[t]
            a = torch.nn.functional.silu(gu[:F]) * gu[F:]
            out[t] += gates[t, j] * (w2[e] @ a)
    return out


@torch.no_grad()
def forward_logits(w: ModelWeights, ids: list[int], router_gaps: list | None = None) -> torch.Tensor:
    """Logits [len(ids), V] for a single sequence (tp=1 weights).  ``router_gaps`` (MoE): receives, per
    layer, each position's router margin between its k-th and (k+1)-th expert -- a near-zero margin is a
    routing near-tie that bf16 activations may resolve the other way."""
    from .layout import natural_tensors

    if getattr(w, "layout", "natural") != "natural":
        w = ModelWeights(w.cfg, w.shard, natural_tensors(w))
    cfg = w.cfg
    T = len(ids)
    D, Hq, Hkv = cfg.head_dim, cfg.num_heads, cfg.num_kv_heads
    cs = rope_table(T, D, cfg.rope_theta, cfg.rope_scaling)
    cos, sin = cs[:, None, : D // 2], cs[:, None, D // 2 :]
    x = w["embed"].float()[torch.tensor(ids)]
    mask = torch.full((T, T), float("-inf")).triu(1)
    for i in range(cfg.num_layers):
        h = _rms(x, w.layer(i, "ln1"), cfg.rms_eps)
        qkv = h @ w.layer(i, "wqkv").float().t()
        q = qkv[:, : Hq * D].view(T, Hq, D)
        k = qkv[:, Hq * D : (Hq + Hkv) * D].view(T, Hkv, D)
        v = qkv[:, (Hq + Hkv) * D :].view(T, Hkv, D)

        def rot(t):
            a, b = t[..., : D // 2], t[..., D // 2 :]
            return torch.cat([a * cos - b * sin, b * cos + a * sin], -1)

        q, k = rot(q), rot(k)
        G = Hq // Hkv
        k = k.repeat_interleave(G, 1)
        v = v.repeat_interleave(G, 1)
        s = torch.einsum("qhd,khd->hqk", q, k) / math.sqrt(D) + mask
        o = torch.einsum("hqk,khd->qhd", torch.softmax(s, -1), v).reshape(T, Hq * D)
        x = x + o @ w.layer(i, "wo").float().t()
        h = _rms(x, w.layer(i, "ln2"), cfg.rms_eps)
        if cfg.is_moe:
            x = x + _moe(cfg, w, i, h, router_gaps)
        else:
            gu = h @ w.layer(i, "w_gu").float().t()
            F = gu.shape[-1] // 2
            x = x + (torch.nn.functional.silu(gu[:, :F]) * gu[:, F:]) @ w.layer(i, "w_down").float().t()
    x = _rms(x, w["norm"], cfg.rms_eps)
    return x @ w["lm_head"].float().t()


def greedy(w: ModelWeights, prompt: list[int], n: int) -> list[int]:
    ids = list(prompt)
    out = []
    for _ in range(n):
        t = int(forward_logits(w, ids)[-1].argmax())
        out.append(t)
        ids.append(t)
    return out
