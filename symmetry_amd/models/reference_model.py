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


def _all_reduce(t: torch.Tensor, group) -> torch.Tensor:
    """Sum over the TP ranks (the row-parallel partials of the oracle).  A gloo group moves GPU tensors
    through the host."""
    import torch.distributed as dist

    if group is None:
        return t
    if t.is_cuda and dist.get_backend(group) == "gloo":
        c = t.cpu()
        dist.all_reduce(c, group=group)
        return t.copy_(c)
    dist.all_reduce(t, group=group)
    return t


def _all_gather_cols(t: torch.Tensor, group) -> torch.Tensor:
    """[T, V / tp] vocabulary shard of every rank -> [T, V] (rank order)."""
    import torch.distributed as dist

    if group is None:
        return t
    world = dist.get_world_size(group)
    src = t.cpu() if t.is_cuda and dist.get_backend(group) == "gloo" else t
    parts = [torch.empty_like(src) for _ in range(world)]
    dist.all_gather(parts, src.contiguous(), group=group)
    return torch.cat(parts, dim=1).to(t.device)


@torch.no_grad()
def forward_logits(w: ModelWeights, ids: list[int], router_gaps: list | None = None, group=None) -> torch.Tensor:
    """Logits [len(ids), V] for a single sequence, computed in fp32 on the device the weights live on.

    ``group``: a TP process group whose ranks each call this with their own shard (``w.shard``): the column-
    parallel heads / intermediate columns stay local, the row-parallel partials (o, down) are summed over the
    group and the vocabulary shards of the lm_head gathered, so every rank returns the full model's logits.
    ``router_gaps`` (MoE, tp = 1): receives, per layer, each position's router margin between its k-th and
    (k+1)-th expert -- a near-zero margin is a routing near-tie that bf16 activations may resolve the other
    way."""
    from .layout import natural_tensors

    if getattr(w, "layout", "natural") != "natural" or getattr(w, "shuffled", None):
        w = ModelWeights(w.cfg, w.shard, natural_tensors(w), "natural")
    cfg = w.cfg
    tp = w.shard.tp_size if group is not None else 1
    if cfg.is_moe and tp > 1:
        raise NotImplementedError("the fp32 oracle shards dense models only")
    dev = w["embed"].device
    T = len(ids)
    D, Hq, Hkv = cfg.head_dim, cfg.num_heads // tp, cfg.num_kv_heads // tp
    cs = rope_table(T, D, cfg.rope_theta, cfg.rope_scaling).to(dev)
    cos, sin = cs[:, None, : D // 2], cs[:, None, D // 2 :]
    x = w["embed"].float()[torch.tensor(ids, device=dev)]
    mask = torch.full((T, T), float("-inf"), device=dev).triu(1)
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
        x = x + _all_reduce(o @ w.layer(i, "wo").float().t(), group)
        h = _rms(x, w.layer(i, "ln2"), cfg.rms_eps)
        if cfg.is_moe:
            x = x + _moe(cfg, w, i, h, router_gaps)
        else:
            gu = h @ w.layer(i, "w_gu").float().t()
            F = gu.shape[-1] // 2
            x = x + _all_reduce((torch.nn.functional.silu(gu[:, :F]) * gu[:, F:]) @ w.layer(i, "w_down").float().t(),
                                group)
    x = _rms(x, w["norm"], cfg.rms_eps)
    return _all_gather_cols(x @ w["lm_head"].float().t(), group)


def check_tokens(logits: torch.Tensor, prompt_len: int, out: list[int], tol: float = 0.08) -> dict:
    """Every generated token against the oracle's logits of the same sequence (teacher-forced over the engine's
    own outputs, so one miss does not cascade): token j must lie within ``tol`` of the best logit at its
    position (bf16 noise vs fp32; a near-tie may legitimately go either way)."""
    gaps = []
    for j, t in enumerate(out):
        row = logits[prompt_len - 1 + j]
        gaps.append(float(row.max() - row[t]))
    bad = [j for j, g in enumerate(gaps) if g > tol]
    return {"tokens": len(out), "mismatches": len(bad), "first_mismatch": bad[0] if bad else None,
            "max_gap": round(max(gaps), 4) if gaps else 0.0, "tol": tol}


def greedy(w: ModelWeights, prompt: list[int], n: int) -> list[int]:
    ids = list(prompt)
    out = []
    for _ in range(n):
        t = int(forward_logits(w, ids)[-1].argmax())
        out.append(t)
        ids.append(t)
    return out
