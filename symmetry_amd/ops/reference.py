"""Plain-PyTorch fp32 reference implementations of every symmetry_amd kernel.

They define the semantics the HIP kernels in ``csrc/kernels`` must match
(tests compare the two) and are the execution path for CPU tensors (unit
tests, the tiny CPU models).  Layout conventions are identical to the
kernels':

* ``LinOut``: a projection output is bf16 ``[T, N]`` or fp32 split-K slabs
  ``[S, T, N]`` (summed by the consumer);
* ``k_cache [NB, Hkv, BS, D]`` token-major, ``v_cache [NB, Hkv, D, BS]``
  dim-major;
* RoPE uses the rotate-half convention with a ``[max_pos, D]`` table
  ``[cos | sin]``.
"""
from __future__ import annotations

import math

import torch

MASK32 = 0xFFFFFFFF


def _mm(x: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """x @ w.T in fp32.  On the CPU (the numerics oracle) both operands are upcast; on a GPU (only in the
    SYMMETRY_OPS=torch eager baseline) the product runs as a bf16 library GEMM with fp32 output, so the
    baseline never materialises fp32 copies of the weights."""
    if x.device.type == "cpu":
        return x.float() @ w.float().t()
    return (x.to(w.dtype) @ w.t()).float()


def linout_sum(x: torch.Tensor) -> torch.Tensor:
    """Collapse a LinOut to fp32 ``[T, N]``."""
    if x.dtype == torch.float32 and x.dim() == 3:
        return x.sum(0)
    return x.float()


def rms_norm(x: torch.Tensor, w: torch.Tensor, eps: float, out: torch.Tensor) -> None:
    xf = linout_sum(x)
    y = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps) * w.float()
    out.copy_(y.view_as(out).to(out.dtype))


def add_rms_norm(delta, residual, w, eps, out) -> None:
    residual.add_(linout_sum(delta).view_as(residual))
    rms_norm(residual, w, eps, out)


def embed_rms_norm(ids, table, residual, w, eps, out) -> None:
    residual.copy_(table[ids.long()].float())
    rms_norm(residual, w, eps, out)


def _unperm_qk(x: torch.Tensor, nqk: int, D: int) -> torch.Tensor:
    """Undo the decode layout (models/layout.py) of the first ``nqk`` heads of x [T, H, D]."""
    from ..models.layout import _pair_perm

    inv = torch.empty(D, dtype=torch.long)
    inv[_pair_perm(D // 2)] = torch.arange(D)
    x = x.clone()
    x[:, :nqk] = x[:, :nqk].index_select(-1, inv.to(x.device))
    return x


def rope_cache(qkv, positions, slots, cos_sin, q_out, k_cache, v_cache, Hq: int, Hkv: int, perm: bool = False) -> None:
    T = positions.numel()
    D = k_cache.shape[3]
    BS = k_cache.shape[2]
    x = linout_sum(qkv).view(T, Hq + 2 * Hkv, D)
    if perm:
        x = _unperm_qk(x, Hq + Hkv, D)
    cs = cos_sin[positions.long()]  # [T, D]
    half = D // 2
    cos, sin = cs[:, None, :half], cs[:, None, half:]
    qk = x[:, : Hq + Hkv]
    x1, x2 = qk[..., :half], qk[..., half:]
    rot = torch.cat([x1 * cos - x2 * sin, x2 * cos + x1 * sin], dim=-1)
    q_out.copy_(rot[:, :Hq].reshape(q_out.shape).to(q_out.dtype))
    k = rot[:, Hq:].to(k_cache.dtype)
    v = x[:, Hq + Hkv:].to(v_cache.dtype)
    s = slots.long()
    valid = s >= 0
    if valid.any():
        s, k, v = s[valid], k[valid], v[valid]
        blk, off = s // BS, s % BS
        k_cache[blk, :, off, :] = k
        v_cache[blk, :, :, off] = v


def _gather_kv(k_cache, v_cache, block_table, ctx: int):
    """Contiguous K, V [ctx, Hkv, D] of one sequence (fp32)."""
    BS = k_cache.shape[2]
    nb = (ctx + BS - 1) // BS
    blocks = block_table[:nb].long()
    k = k_cache[blocks].permute(0, 2, 1, 3).reshape(nb * BS, k_cache.shape[1], -1)[:ctx]
    v = v_cache[blocks].permute(0, 3, 1, 2).reshape(nb * BS, v_cache.shape[1], -1)[:ctx]
    return k.float(), v.float()


def _attend(q, k, v, scale, causal_offset=None):
    """q [n, Hq, D], k/v [ctx, Hkv, D] -> [n, Hq, D] fp32 (GQA by repeat)."""
    Hq, Hkv = q.shape[1], k.shape[1]
    G = Hq // Hkv
    k = k.repeat_interleave(G, dim=1)
    v = v.repeat_interleave(G, dim=1)
    s = torch.einsum("qhd,khd->hqk", q.float(), k) * scale
    if causal_offset is not None:
        n, ctx = q.shape[0], k.shape[0]
        qpos = torch.arange(n, device=q.device)[:, None] + causal_offset
        kpos = torch.arange(ctx, device=q.device)[None, :]
        s = s.masked_fill(kpos > qpos, float("-inf"))
    p = torch.softmax(s, dim=-1)
    return torch.einsum("hqk,khd->qhd", p, v)


def attn_decode(q, k_cache, v_cache, block_tables, ctx_lens, out, tmp_o=None, tmp_ml=None, scale=1.0) -> None:
    S = q.shape[0]
    res = torch.empty(q.shape, dtype=torch.float32, device=q.device)
    for i in range(S):
        ctx = int(ctx_lens[i])
        k, v = _gather_kv(k_cache, v_cache, block_tables[i], ctx)
        res[i] = _attend(q[i : i + 1], k, v, scale)[0]
    out.copy_(res.view_as(out).to(out.dtype))


def attn_prefill(q, k_cache, v_cache, block_tables, ctx_lens, cu_q, tiles, out, scale) -> None:
    nseq = ctx_lens.numel()
    res = torch.zeros(q.shape, dtype=torch.float32, device=q.device)
    for i in range(nseq):
        a, b = int(cu_q[i]), int(cu_q[i + 1])
        if b == a:
            continue
        ctx = int(ctx_lens[i])
        k, v = _gather_kv(k_cache, v_cache, block_tables[i], ctx)
        res[a:b] = _attend(q[a:b], k, v, scale, causal_offset=ctx - (b - a))
    out.copy_(res.view_as(out).to(out.dtype))


def skinny_gemm(x, w, y) -> None:
    S = y.shape[0]
    K = x.shape[1]
    kc = K // S
    for s in range(S):
        y[s] = _mm(x[:, s * kc : (s + 1) * kc], w[:, s * kc : (s + 1) * kc])


# ----- sampling: same counter-based RNG and packed keys as the kernel ----------------------------
def _u32(x):
    return x & MASK32


def uniform01(seed: torch.Tensor, counter: torch.Tensor) -> torch.Tensor:
    """Bit-exact torch port of ``uniform01`` in csrc/kernels/common.h (int64 tensors)."""
    x0 = _u32(counter)
    x1 = _u32(counter >> 32)
    k0 = _u32(seed).expand_as(x0).clone()
    k1 = _u32(seed >> 32).expand_as(x0).clone()
    for _ in range(7):
        p0h, p0l = _mulhilo(x0, 0xD2511F53)
        p1h, p1l = _mulhilo(x1, 0xCD9E8D57)
        n0 = p1h ^ k0 ^ p0l
        n1 = p0h ^ k1 ^ p1l
        x0, x1 = n0, n1
        k0 = _u32(k0 + 0x9E3779B9)
        k1 = _u32(k1 + 0xBB67AE85)
    return ((x0 >> 8).double() + 0.5) * (1.0 / 16777216.0)


def _mulhilo(a: torch.Tensor, b: int):
    """Unsigned 32x32->64 multiply of int64 tensors holding u32 values."""
    al, ah = a & 0xFFFF, a >> 16
    bl, bh = b & 0xFFFF, b >> 16
    ll = al * bl
    lh = al * bh
    hl = ah * bl
    hh = ah * bh
    mid = (ll >> 16) + (lh & 0xFFFF) + (hl & 0xFFFF)
    lo = _u32((mid << 16) | (ll & 0xFFFF))
    hi = _u32(hh + (lh >> 16) + (hl >> 16) + (mid >> 16))
    return hi, lo


def _ordered_bits(v: torch.Tensor) -> torch.Tensor:
    u = v.float().view(torch.int32).long() & MASK32
    neg = (u & 0x80000000) != 0
    return torch.where(neg, _u32(~u), u | 0x80000000)


def sample_keys(logits: torch.Tensor, temps: torch.Tensor, seeds: torch.Tensor, step: int, n_offset: int = 0):
    """Packed argmax keys (int64 bit pattern of the kernel's u64) and token ids per row."""
    M, N = logits.shape
    gidx = torch.arange(N, device=logits.device, dtype=torch.int64) + n_offset
    vals = logits.float().clone()
    for m in range(M):
        t = float(temps[m])
        if t > 0:
            seed = int(seeds[m]) & 0xFFFFFFFFFFFFFFFF
            mixed = seed ^ ((step << 20) & 0xFFFFFFFFFFFFFFFF)
            if mixed >= 1 << 63:
                mixed -= 1 << 64
            u = uniform01(torch.tensor(mixed, dtype=torch.int64, device=gidx.device), gidx).float()
            vals[m] = vals[m] / t - torch.log(-torch.log(u))
    ob = _ordered_bits(vals)
    low = 0xFFFFFFFF - gidx
    ids = torch.empty(M, dtype=torch.int64, device=logits.device)
    keys = torch.empty(M, dtype=torch.int64, device=logits.device)
    for m in range(M):
        # max over (ob, low) lexicographic == max key
        best = ob[m].max()
        cand = torch.nonzero(ob[m] == best).flatten()
        j = int(cand.min())  # smallest index wins ties (largest ~idx)
        ids[m] = int(gidx[j])
        key = (int(best) << 32) | int(low[j])
        keys[m] = key - (1 << 64) if key >= 1 << 63 else key
    return keys, ids


def lm_head_sample(x, w, temps, seeds, step, tile_keys, out_keys, out_ids, n_offset: int, logits=None) -> None:
    lg = _mm(x, w)
    if logits is not None:
        logits.copy_(lg)
    keys, ids = sample_keys(lg, temps, seeds, int(step.reshape(-1)[0]), n_offset)
    M = x.shape[0]
    out_keys[:M].copy_(keys)
    out_ids[:M].copy_(ids.to(out_ids.dtype))


def logits_argmax(logits, temps, seeds, step, out_keys, out_ids, n_offset: int = 0) -> None:
    keys, ids = sample_keys(logits, temps, seeds, int(step.reshape(-1)[0]), n_offset)
    M = logits.shape[0]
    out_keys[:M].copy_(keys)
    out_ids[:M].copy_(ids.to(out_ids.dtype))


def swiglu(gu, out, interleaved: bool = False) -> None:
    g = linout_sum(gu)
    F = out.shape[1]
    if interleaved:
        from ..models.layout import _inverse, gu_perm

        g = g.index_select(-1, _inverse(gu_perm(F)).to(g.device))
    y = torch.nn.functional.silu(g[:, :F]) * g[:, F:]
    out.copy_(y.to(out.dtype))


# ----- fused decode GEMMs (csrc/kernels/decode_gemm.hip) -----------------------------------------
def unshuffled(W, wshuf: bool):
    """Row-major view of a decode weight stored MFMA-preshuffled (models/layout.py::preshuffle)."""
    if not wshuf:
        return W
    from ..models.layout import unshuffle

    return unshuffle(W)


def _row_scale(ss_in, eps: float, K: int, M: int):
    if ss_in is None:
        return None
    return torch.rsqrt(ss_in[:M].float().sum(-1, keepdim=True) / K + eps)


def _dg(x, W, ss_in, eps):
    y = _mm(x, W)
    rn = _row_scale(ss_in, eps, x.shape[1], x.shape[0])
    return y if rn is None else y * rn


def dg_f32(x, W, ss_in, eps, y) -> None:
    y[: x.shape[0]].copy_(_dg(x, W, ss_in, eps))


def dg_qkv(x, W, ss_in, eps, positions, slots, cos_sin, q_out, k_cache, v_cache, Hq: int, Hkv: int) -> None:
    rope_cache(_dg(x, W, ss_in, eps), positions, slots, cos_sin, q_out, k_cache, v_cache, Hq, Hkv, perm=True)


def dg_resid(x, W, resid, w_next, xw_out, ss_out) -> None:
    M = x.shape[0]
    r = resid[:M]
    r.add_(_mm(x, W))
    xw_out[:M].copy_((r * w_next.float()).to(xw_out.dtype))
    ss_out[:M].copy_(r.pow(2).view(M, -1, 16).sum(-1))


def dg_swiglu(x, W, ss_in, eps, act) -> None:
    swiglu(_dg(x, W, ss_in, eps), act[: x.shape[0]], interleaved=True)


def dg_argmax(x, W, ss_in, eps, temps, seeds, step, tile_keys, out_keys, out_ids, n_offset: int, logits=None) -> None:
    lg = _dg(x, W, ss_in, eps)
    if logits is not None:
        logits[: x.shape[0]].copy_(lg)
    keys, ids = sample_keys(lg, temps, seeds, int(step.reshape(-1)[0]), n_offset)
    M = x.shape[0]
    out_keys[:M].copy_(keys)
    out_ids[:M].copy_(ids.to(out_ids.dtype))


def resolve_ids(ids, src=None, prev=None):
    """Token per row: prev[src] where src >= 0 (previous step's on-device samples), else ids."""
    if src is None:
        return ids.long()
    s = src[: ids.numel()].long()
    return torch.where(s >= 0, prev.long()[s.clamp(min=0)], ids.long())


def embed_prep(ids, table, resid, w, xw, ss, src=None, prev=None) -> None:
    T = ids.numel()
    r = table[resolve_ids(ids, src, prev)].float()
    resid[:T].copy_(r)
    xw[:T].copy_((r * w.float()).to(xw.dtype))
    if ss.dim() == 2 and ss.shape[1] > 1:  # [>=T, P]: partial sums over P column slices of each row
        ss[:T].copy_(r.pow(2).view(T, ss.shape[1], -1).sum(-1))
    else:
        ss.view(-1)[:T].copy_(r.pow(2).sum(-1))  # ss: [>=T] or [>=T, 1] (one tile per row)


def add_prep(delta, resid, w, xw, ss) -> None:
    d = linout_sum(delta)
    T = d.shape[0]
    r = resid[:T]
    r.add_(d)
    xw[:T].copy_((r * w.float()).to(xw.dtype))
    if ss.dim() == 2 and ss.shape[1] > 1:  # [>=T, P]: partial sums over P column slices of each row
        ss[:T].copy_(r.pow(2).view(T, ss.shape[1], -1).sum(-1))
    else:
        ss.view(-1)[:T].copy_(r.pow(2).sum(-1))  # ss: [>=T] or [>=T, 1] (one tile per row)


def rownorm(xw, ss, eps, out) -> None:
    T, d = out.shape
    rn = torch.rsqrt(ss[:T].float().sum(-1, keepdim=True) / d + eps)
    out.copy_((xw[:T].float() * rn).to(out.dtype))


def rope_table(max_pos: int, head_dim: int, theta: float, scaling: dict | None = None,
               device="cpu") -> torch.Tensor:
    """``[max_pos, D]`` fp32 table ``[cos | sin]`` incl. Llama-3.1 NTK-by-parts scaling."""
    inv = 1.0 / (theta ** (torch.arange(0, head_dim, 2, dtype=torch.float64) / head_dim))
    if scaling and scaling.get("rope_type", scaling.get("type")) == "llama3":
        factor = scaling["factor"]
        lo, hi = scaling.get("low_freq_factor", 1.0), scaling.get("high_freq_factor", 4.0)
        old = scaling.get("original_max_position_embeddings", 8192)
        lo_wl, hi_wl = old / lo, old / hi
        wl = 2 * math.pi / inv
        smooth = (old / wl - lo) / (hi - lo)
        scaled = torch.where(wl > lo_wl, inv / factor, inv)
        mid = (wl <= lo_wl) & (wl >= hi_wl)
        scaled = torch.where(mid, (1 - smooth) * inv / factor + smooth * inv, scaled)
        inv = scaled
    pos = torch.arange(max_pos, dtype=torch.float64)
    ang = pos[:, None] * inv[None, :]
    return torch.cat([ang.cos(), ang.sin()], dim=-1).float().to(device)


# ----- MoE ---------------------------------------------------------------------------------------
def moe_route_permute(logits, x, k: int, E: int, ids, w, counts, offsets, cursor, xs, dst) -> None:
    """Top-k routing (softmax over the selected logits), expert segments in token order."""
    T = x.shape[0]
    lg = linout_sum(logits)[:, :E]
    topv, topi = torch.topk(lg, k, dim=-1)  # ties -> lower index first (same as the kernel)
    wt = torch.softmax(topv, dim=-1)
    ids[: T * k].copy_(topi.reshape(-1).to(ids.dtype))
    w[: T * k].copy_(wt.reshape(-1))
    flat = topi.reshape(-1)
    cnt = torch.bincount(flat, minlength=E)[:E]
    counts[:E].copy_(cnt.to(counts.dtype))
    off = torch.zeros(E + 1, dtype=torch.int64)
    off[1:] = torch.cumsum(cnt, 0)
    offsets[: E + 1].copy_(off.to(offsets.dtype))
    cur = off[:-1].clone()
    rows = torch.empty(T * k, dtype=torch.int64)
    for a in range(T * k):
        e = int(flat[a])
        rows[a] = cur[e]
        cur[e] += 1
    dst[: T * k].copy_(rows.to(dst.dtype))
    xs[rows] = x[torch.arange(T * k) // k].to(xs.dtype)


def moe_route(logits, T: int, k: int, E: int, ids, w) -> None:
    lg = linout_sum(logits)[:T, :E]
    topv, topi = torch.topk(lg, k, dim=-1)  # ties -> lower index first (same as the kernel)
    ids[: T * k].copy_(topi.reshape(-1).to(ids.dtype))
    w[: T * k].copy_(torch.softmax(topv, dim=-1).reshape(-1))


def moe_align(ids, G: int, counts, offsets, cursor) -> None:
    v = ids.long()
    v = v[(v >= 0) & (v < G)]
    cnt = torch.bincount(v, minlength=G)[:G]
    counts[:G].copy_(cnt.to(counts.dtype))
    off = torch.zeros(G + 1, dtype=torch.int64)
    off[1:] = torch.cumsum(cnt, 0)
    offsets[: G + 1].copy_(off.to(offsets.dtype))
    cursor[:G].zero_()


def moe_scatter(x, ids, k: int, G: int, offsets, cursor, xs, dst, src_tok=None) -> None:
    """Rows into group segments in assignment order (the kernel's order within a segment varies; every
    consumer indexes through dst, so results agree)."""
    T = x.shape[0]
    R = xs.shape[0]
    for a in range(T * k):
        g = int(ids[a])
        if g < 0 or g >= G:
            continue
        row = int(offsets[g]) + int(cursor[g])
        cursor[g] += 1
        dst[a] = row
        if 0 <= row < R:
            xs[row] = x[a // k].to(xs.dtype)
            if src_tok is not None:
                src_tok[row] = a // k


def grouped_gemm(xs, W, offsets, e0: int, y, mode: int) -> None:
    """Y[rows of e] = Xs[rows of e] . W[e]^T (mode 0 bf16 / 1 fp32), or SwiGLU of the [gate; up] product;
    mode + 4: W MFMA-preshuffled per expert."""
    if mode & 4:
        from ..models.layout import unshuffle

        W = torch.stack([unshuffle(W[e]) for e in range(W.shape[0])])
        mode &= 3
    for e in range(W.shape[0]):
        a, b = int(offsets[e0 + e]), int(offsets[e0 + e + 1])
        if b <= a:
            continue
        p = _mm(xs[a:b], W[e])
        if mode == 2:
            F = p.shape[1] // 2
            p = torch.nn.functional.silu(p[:, :F]) * p[:, F:]
        y[a:b] = p.to(y.dtype)


def grouped_skinny(xs, W, offsets, e0: int, y) -> None:
    S = y.shape[0]
    y.zero_()
    for e in range(W.shape[0]):
        a, b = int(offsets[e0 + e]), int(offsets[e0 + e + 1])
        if b > a:
            y[0, a:b] = _mm(xs[a:b], W[e])


def moe_combine(y, dst, ids, e_lo: int, e_hi: int, w, k: int, out, accumulate: bool) -> None:
    T, d = out.shape
    yy = linout_sum(y)
    res = torch.zeros(T, d, dtype=torch.float32)
    for t in range(T):
        for j in range(k):
            a = t * k + j
            e = int(ids[a])
            if e_lo <= e < e_hi and int(dst[a]) >= 0:
                res[t] += float(w[a]) * yy[int(dst[a])]
    if accumulate:
        out.add_(res)
    else:
        out.copy_(res)


def moe_owner_pack(y, dst, ids, w, e_lo: int, e_hi: int, k: int, S: int, cursor, send, side) -> None:
    """Weighted partial over each token's local experts ([e_lo, e_hi)), one row per token that has one, pushed
    into its slice owner's block (owner = t // S; token order here, arrival order on the GPU: the owner's
    combine does not depend on it); side = the token's index in the owner's slice."""
    N = cursor.numel()
    cap = send.shape[0] // N
    T = dst.numel() // k
    yy = linout_sum(y)
    cursor.zero_()
    for t in range(T):
        row = None
        for j in range(k):
            a = t * k + j
            e = int(ids[a])
            if e_lo <= e < e_hi and int(dst[a]) >= 0:
                v = float(w[a]) * yy[int(dst[a])]
                row = v if row is None else row + v
        if row is None:
            continue
        o = t // S
        c = int(cursor[o])
        cursor[o] += 1
        send[o * cap + c] = row
        side[o * cap + c] = t - o * S


def moe_owner_combine(recv, side, rcnt, Tr: int, pos, out) -> None:
    """out [S, d] bf16: row t = sum over sources (rank order) of the received partial for slice token t."""
    N = rcnt.numel()
    cap = recv.shape[0] // N
    S, d = out.shape
    acc = torch.zeros(S, d, dtype=torch.float32)
    pos.view(-1)[: N * S] = -1
    for s in range(N):
        for i in range(min(int(rcnt[s]), cap)):
            t = int(side[s * cap + i])
            if 0 <= t < S:
                pos[s * S + t] = i
    for t in range(Tr):
        for s in range(N):
            p = int(pos[s * S + t])
            if p >= 0:
                acc[t] += recv[s * cap + p].float()
    out.copy_(acc.to(out.dtype))


def sample_filtered(logits, temps, top_k, top_p, seeds, step, out_ids) -> None:
    """Temperature + top-k + top-p (nucleus) resampling of full-vocab rows (csrc/kernels/sampling.hip).

    Kept set = {tokens whose logit >= the k-th largest} intersected with the smallest descending prefix
    whose probability mass reaches top_p (ties at the threshold are kept).  Rows with t == 0 or without a
    filter are left untouched.  Same RNG stream as the fused lm_head sampler."""
    st = int(step.reshape(-1)[0])
    B, V = logits.shape
    for r in range(B):
        t, k, p = float(temps[r]), int(top_k[r]), float(top_p[r])
        use_k, use_p = 0 < k < V, p < 1.0
        if t <= 0 or not (use_k or use_p):
            continue
        l = logits[r].float()
        thr = -float("inf")
        srt = torch.sort(l, descending=True).values
        if use_k:
            thr = max(thr, float(srt[k - 1]))
        if use_p:
            w = torch.exp((srt - srt[0]) / t)
            cum = torch.cumsum(w, 0)
            j = int(torch.searchsorted(cum, max(p, 0.0) * float(w.sum())).clamp(max=V - 1))
            thr = max(thr, float(srt[j]))
        seed = int(seeds[r]) & 0xFFFFFFFFFFFFFFFF
        mixed = seed ^ ((st << 20) & 0xFFFFFFFFFFFFFFFF)
        if mixed >= 1 << 63:
            mixed -= 1 << 64
        u = uniform01(torch.tensor(mixed, dtype=torch.int64), torch.arange(V, dtype=torch.int64)).float()
        v = l / t - torch.log(-torch.log(u.to(l.device)))
        v = torch.where(l >= thr, v, torch.full_like(v, -float("inf")))
        out_ids[r] = int(torch.argmax(v))


def moe_decode_route(resid, lnw, eps, Wr, k: int, ids, w, counts, offsets, cursor, xs, dst) -> None:
    """rms_norm + router logits + moe_route_permute (the fused decode routing kernel's contract)."""
    T, d = resid.shape
    xn = torch.empty(T, d, dtype=torch.bfloat16)
    rms_norm(resid, lnw, eps, xn)
    logits = _mm(xn, Wr)
    moe_route_permute(logits, xn, k, Wr.shape[0], ids, w, counts, offsets, cursor, xs, dst)


def moe_combine_prep(y, dst, ids, E: int, w, k: int, resid, w_next, xw, ss) -> None:
    """moe_combine over every expert + add_prep (one sum-of-squares partial per row)."""
    T, d = resid.shape
    out = torch.empty(T, d, dtype=torch.float32)
    moe_combine(y, dst, ids, 0, E, w, k, out, False)
    add_prep(out, resid, w_next, xw, ss)
