"""Numerics of every CDNA4 HIP kernel against the plain-PyTorch fp32 reference.

Each test builds inputs on the GPU, runs the native op (torch.ops.symmetry_amd)
and the reference (symmetry_amd.ops.reference) on fp32 copies, and compares.
"""
import math

import pytest
import torch

from symmetry_amd import ops
from symmetry_amd.ops import reference as ref

pytestmark = pytest.mark.gpu


def _close(a, b, atol, rtol=0.0):
    a, b = a.float().cpu(), b.float().cpu()
    err = (a - b).abs()
    tol = atol + rtol * b.abs()
    assert torch.isfinite(a).all(), "non-finite output"
    assert (err <= tol).all(), f"max err {err.max().item():.4g} (atol {atol}, rtol {rtol})"


@pytest.mark.parametrize("T,d", [(1, 4096), (7, 4096), (33, 8192), (3, 128)])
@pytest.mark.parametrize("kind", ["bf16", "slabs"])
def test_rms_norm_family(gpu, T, d, kind):
    g = torch.Generator(device=gpu).manual_seed(0)
    w = (torch.randn(d, device=gpu, generator=g) * 0.1 + 1).bfloat16()
    if kind == "bf16":
        x = torch.randn(T, d, device=gpu, generator=g).bfloat16()
    else:
        x = torch.randn(3, T, d, device=gpu, generator=g)
    out = torch.empty(T, d, device=gpu, dtype=torch.bfloat16)
    ops.rms_norm(x, w, 1e-5, out)
    ref_out = torch.empty(T, d, dtype=torch.bfloat16)
    ref.rms_norm(x.cpu(), w.cpu(), 1e-5, ref_out)
    _close(out, ref_out, atol=2e-2, rtol=1e-2)

    res = torch.randn(T, d, device=gpu, generator=g)
    res_ref = res.cpu().clone()
    ops.add_rms_norm(x, res, w, 1e-5, out)
    ref.add_rms_norm(x.cpu(), res_ref, w.cpu(), 1e-5, ref_out)
    _close(res, res_ref, atol=1e-4, rtol=1e-5)
    _close(out, ref_out, atol=2e-2, rtol=1e-2)


def test_embed_rms_norm(gpu):
    V, d, T = 1000, 4096, 9
    g = torch.Generator(device=gpu).manual_seed(1)
    table = torch.randn(V, d, device=gpu, generator=g).bfloat16()
    ids = torch.randint(0, V, (T,), device=gpu, generator=g, dtype=torch.int32)
    w = torch.randn(d, device=gpu, generator=g).bfloat16()
    res = torch.empty(T, d, device=gpu)
    out = torch.empty(T, d, device=gpu, dtype=torch.bfloat16)
    ops.embed_rms_norm(ids, table, res, w, 1e-5, out)
    res_ref = torch.empty(T, d)
    out_ref = torch.empty(T, d, dtype=torch.bfloat16)
    ref.embed_rms_norm(ids.cpu(), table.cpu(), res_ref, w.cpu(), 1e-5, out_ref)
    _close(res, res_ref, atol=0)
    _close(out, out_ref, atol=3e-2, rtol=1e-2)


def _make_cache(gpu, NB, Hkv, BS, D=128):
    k = torch.zeros(NB, Hkv, BS, D, device=gpu, dtype=torch.bfloat16)
    v = torch.zeros(NB, Hkv, D, BS, device=gpu, dtype=torch.bfloat16)
    return k, v


@pytest.mark.parametrize("kind", ["bf16", "slabs"])
def test_rope_cache(gpu, kind):
    T, Hq, Hkv, D, BS, NB = 11, 32, 8, 128, 64, 8
    g = torch.Generator(device=gpu).manual_seed(2)
    N = (Hq + 2 * Hkv) * D
    qkv = torch.randn(T, N, device=gpu, generator=g).bfloat16() if kind == "bf16" else torch.randn(
        2, T, N, device=gpu, generator=g)
    pos = torch.randint(0, 4000, (T,), device=gpu, generator=g, dtype=torch.int32)
    slots = torch.randperm(NB * BS, device=gpu, generator=g)[:T].int()
    slots[3] = -1  # padding token: no cache write
    cs = ref.rope_table(8192, D, 500000.0).to(gpu)
    q = torch.empty(T, Hq, D, device=gpu, dtype=torch.bfloat16)
    kc, vc = _make_cache(gpu, NB, Hkv, BS)
    ops.rope_cache(qkv, pos, slots, cs, q, kc, vc, Hq, Hkv)
    q_r = torch.empty(T, Hq, D, dtype=torch.bfloat16)
    kc_r, vc_r = kc.new_zeros(kc.shape).cpu(), vc.new_zeros(vc.shape).cpu()
    ref.rope_cache(qkv.cpu(), pos.cpu(), slots.cpu(), cs.cpu(), q_r, kc_r, vc_r, Hq, Hkv)
    _close(q, q_r, atol=2e-2, rtol=1e-2)
    _close(kc, kc_r, atol=2e-2, rtol=1e-2)
    _close(vc, vc_r, atol=1e-2, rtol=1e-2)


@pytest.mark.parametrize("decode", [False, True])
@pytest.mark.parametrize("kind", ["bf16", "slabs"])
def test_rope_cache_prefill_groups(gpu, kind, decode):
    """Prefill-sized rope_cache (8-row groups): 16-byte V token runs for aligned consecutive slots, the
    per-token fallback for unaligned runs, scattered slots, padding rows and a ragged last group.
    decode=True: the same rows through the per-row form (several workgroups per row)."""
    Hq, Hkv, D, BS, NB = 32, 8, 128, 64, 12
    slots_l = list(range(3 * BS + 5, 3 * BS + 5 + 37)) + list(range(5 * BS, 5 * BS + 56))
    slots_l += [9 * BS + 1, -1, 7 * BS + 63, 10 * BS + 8, -1, 11 * BS, 2 * BS + 9]
    T = len(slots_l)  # 100: twelve full groups and a ragged one
    g = torch.Generator(device=gpu).manual_seed(12)
    N = (Hq + 2 * Hkv) * D
    qkv = torch.randn(T, N, device=gpu, generator=g).bfloat16() if kind == "bf16" else torch.randn(
        2, T, N, device=gpu, generator=g)
    pos = torch.randint(0, 4000, (T,), device=gpu, generator=g, dtype=torch.int32)
    slots = torch.tensor(slots_l, device=gpu, dtype=torch.int32)
    cs = ref.rope_table(8192, D, 500000.0).to(gpu)
    q = torch.empty(T, Hq, D, device=gpu, dtype=torch.bfloat16)
    kc, vc = _make_cache(gpu, NB, Hkv, BS)
    ops.rope_cache(qkv, pos, slots, cs, q, kc, vc, Hq, Hkv, decode=decode)
    q_r = torch.empty(T, Hq, D, dtype=torch.bfloat16)
    kc_r, vc_r = kc.new_zeros(kc.shape).cpu(), vc.new_zeros(vc.shape).cpu()
    ref.rope_cache(qkv.cpu(), pos.cpu(), slots.cpu(), cs.cpu(), q_r, kc_r, vc_r, Hq, Hkv)
    _close(q, q_r, atol=2e-2, rtol=1e-2)
    _close(kc, kc_r, atol=2e-2, rtol=1e-2)
    _close(vc, vc_r, atol=1e-2, rtol=1e-2)


def _random_paged(gpu, ctx_lens, Hkv, BS, g, extra_blocks=3):
    nseq = len(ctx_lens)
    max_blocks = max((c + BS - 1) // BS for c in ctx_lens) + 1
    NB = sum((c + BS - 1) // BS for c in ctx_lens) + extra_blocks
    kc = torch.randn(NB, Hkv, BS, 128, device=gpu, generator=g).bfloat16()
    vc = torch.randn(NB, Hkv, 128, BS, device=gpu, generator=g).bfloat16()
    perm = torch.randperm(NB, generator=torch.Generator().manual_seed(5)).tolist()
    bt = torch.zeros(nseq, max_blocks, dtype=torch.int32)
    i = 0
    for s, c in enumerate(ctx_lens):
        for b in range((c + BS - 1) // BS):
            bt[s, b] = perm[i]
            i += 1
    return kc, vc, bt.to(gpu)


@pytest.fixture(params=["grid", "stream"])
def attn_decode_kernel(request):
    """The grid split-KV kernel and the streaming long-context kernel (chosen by block-table span)."""
    torch.ops.symmetry_amd.attn_wave(0, 0)
    torch.ops.symmetry_amd.attn_stream_min(0 if request.param == "grid" else 1)
    yield request.param
    torch.ops.symmetry_amd.attn_stream_min(1024)
    torch.ops.symmetry_amd.attn_wave(1024, 513)


@pytest.mark.parametrize("Hq,Hkv", [(32, 8), (64, 8), (8, 1), (16, 16)])
@pytest.mark.parametrize("BS", [32, 64])
def test_attn_decode(gpu, attn_decode_kernel, Hq, Hkv, BS):
    g = torch.Generator(device=gpu).manual_seed(3)
    ctx_lens = [1, 17, 64, 255, 256, 257, 511, 512, 513, 1000, 2049, 4100]
    kc, vc, bt = _random_paged(gpu, ctx_lens, Hkv, BS, g)
    S = len(ctx_lens)
    q = torch.randn(S, Hq, 128, device=gpu, generator=g).bfloat16()
    ctx = torch.tensor(ctx_lens, device=gpu, dtype=torch.int32)
    max_parts = (bt.shape[1] * BS + ops.ATTN_DECODE_PART - 1) // ops.ATTN_DECODE_PART
    tmp_o = torch.empty(S, Hq, max_parts, 128, device=gpu)
    tmp_ml = torch.empty(S, Hq, max_parts, 2, device=gpu)
    out = torch.empty(S, Hq, 128, device=gpu, dtype=torch.bfloat16)
    cnt = torch.zeros(S * Hkv, device=gpu, dtype=torch.int32)
    scale = 1 / math.sqrt(128)
    ops.attn_decode(q, kc, vc, bt, ctx, out, tmp_o, tmp_ml, cnt, scale)
    out_r = torch.empty(S, Hq, 128, dtype=torch.bfloat16)
    ref.attn_decode(q.cpu(), kc.cpu(), vc.cpu(), bt.cpu(), ctx.cpu(), out_r, scale=scale)
    _close(out, out_r, atol=2e-2, rtol=2e-2)
    # the in-kernel split-KV combine re-arms its arrival counters: a second call is identical
    assert int(cnt.abs().sum()) == 0
    out2 = torch.empty_like(out)
    ops.attn_decode(q, kc, vc, bt, ctx, out2, tmp_o, tmp_ml, cnt, scale)
    assert torch.equal(out, out2)


@pytest.mark.parametrize("Hq,Hkv", [(32, 8), (64, 8), (8, 1), (16, 16)])
@pytest.mark.parametrize("BS", [32, 64])
def test_attn_decode_wave(gpu, Hq, Hkv, BS):
    """One wave per (seq, kv head) walking the whole context (wide decode batches, block tables of <= 64
    entries): forced on for a small batch, against the fp32 reference."""
    g = torch.Generator(device=gpu).manual_seed(4)
    ctx_lens = [c for c in (1, 17, 31, 32, 33, 64, 200, 255, 256, 257, 511, 700, 1000, 2000, 4000)
                if c <= 63 * BS]
    kc, vc, bt = _random_paged(gpu, ctx_lens, Hkv, BS, g)
    assert bt.shape[1] <= 64
    S = len(ctx_lens)
    q = torch.randn(S, Hq, 128, device=gpu, generator=g).bfloat16()
    ctx = torch.tensor(ctx_lens, device=gpu, dtype=torch.int32)
    max_parts = (bt.shape[1] * BS + ops.ATTN_DECODE_PART - 1) // ops.ATTN_DECODE_PART
    tmp_o = torch.empty(S, Hq, max_parts, 128, device=gpu)
    tmp_ml = torch.empty(S, Hq, max_parts, 2, device=gpu)
    out = torch.full((S, Hq, 128), float("nan"), device=gpu, dtype=torch.bfloat16)
    cnt = torch.zeros(S * Hkv, device=gpu, dtype=torch.int32)
    scale = 1 / math.sqrt(128)
    torch.ops.symmetry_amd.attn_wave(1, 0)
    try:
        ops.attn_decode(q, kc, vc, bt, ctx, out, tmp_o, tmp_ml, cnt, scale)
    finally:
        torch.ops.symmetry_amd.attn_wave(1024, 513)
    out_r = torch.empty(S, Hq, 128, dtype=torch.bfloat16)
    ref.attn_decode(q.cpu(), kc.cpu(), vc.cpu(), bt.cpu(), ctx.cpu(), out_r, scale=scale)
    _close(out, out_r, atol=2e-2, rtol=2e-2)


@pytest.mark.parametrize("Hq,Hkv", [(32, 8), (8, 8), (64, 8), (16, 8)])
@pytest.mark.parametrize("BS", [32, 64])
def test_attn_prefill(gpu, Hq, Hkv, BS):
    g = torch.Generator(device=gpu).manual_seed(4)
    # (new tokens, total context): fresh prompts and chunked continuations
    specs = [(5, 5), (64, 64), (100, 100), (37, 300), (130, 130), (1, 77), (200, 457)]
    ctx_lens = [c for _, c in specs]
    kc, vc, bt = _random_paged(gpu, ctx_lens, Hkv, BS, g)
    qlens = [n for n, _ in specs]
    cu = [0]
    for n in qlens:
        cu.append(cu[-1] + n)
    T = cu[-1]
    q = torch.randn(T, Hq, 128, device=gpu, generator=g).bfloat16()
    tiles = []
    for s, n in enumerate(qlens):
        for r in range(0, n, 64):
            tiles.append((s, r))
    tiles_t = torch.tensor(tiles, dtype=torch.int32, device=gpu)
    out = torch.empty_like(q)
    scale = 1 / math.sqrt(128)
    ctx = torch.tensor(ctx_lens, dtype=torch.int32, device=gpu)
    cu_t = torch.tensor(cu, dtype=torch.int32, device=gpu)
    ops.attn_prefill(q, kc, vc, bt, ctx, cu_t, tiles_t, out, scale)
    out_r = torch.empty(q.shape, dtype=torch.bfloat16)
    ref.attn_prefill(q.cpu(), kc.cpu(), vc.cpu(), bt.cpu(), ctx.cpu(), cu_t.cpu(), tiles_t.cpu(), out_r, scale)
    _close(out, out_r, atol=2e-2, rtol=2e-2)


@pytest.mark.parametrize("M", [1, 5, 16, 33, 64])
@pytest.mark.parametrize("N,K", [(6144, 4096), (4096, 14336), (1024, 512)])
def test_skinny_gemm(gpu, M, N, K):
    g = torch.Generator(device=gpu).manual_seed(6)
    x = torch.randn(M, K, device=gpu, generator=g).bfloat16()
    w = (torch.randn(N, K, device=gpu, generator=g) * 0.02).bfloat16()
    S = ops.choose_splits(N, K)
    y = torch.empty(S, M, N, device=gpu)
    ops.skinny_gemm(x, w, y)
    ref_y = x.float() @ w.float().t()
    _close(y.sum(0), ref_y, atol=2e-3 * math.sqrt(K) * 0.1 + 1e-3, rtol=1e-3)


@pytest.mark.parametrize("M", [1, 17, 40, 64, 65, 100, 128, 129, 200, 256])
@pytest.mark.parametrize("N,K,rw,S", [(512, 1024, 1, 4), (768, 2048, 3, 8), (1024, 3584, 2, 7), (512, 512, 4, 1)])
def test_mgemm(gpu, M, N, K, rw, S):
    """Medium-M split-K GEMM on the preshuffled weight: every slab is the partial product over its k slice
    (fp32 reference), rows past M untouched; ragged M (not a multiple of 16) exercises the zero-filled rows."""
    from symmetry_amd.models.layout import preshuffle

    if M > 128 and rw > 2:
        pytest.skip("rw <= 2 above 128 rows")
    g = torch.Generator(device=gpu).manual_seed(M * 7 + N)
    x = torch.randn(M, K, device=gpu, generator=g).bfloat16()
    w = (torch.randn(N, K, device=gpu, generator=g) * 0.02).bfloat16()
    y = torch.full((S, M, N), float("nan"), device=gpu)
    ops.mgemm(x, preshuffle(w), y, rw)
    kc = K // S
    for s in range(S):
        ref_s = x[:, s * kc:(s + 1) * kc].float() @ w[:, s * kc:(s + 1) * kc].float().t()
        _close(y[s], ref_s, atol=2e-3 * math.sqrt(kc) * 0.1 + 1e-3, rtol=1e-3)


def test_lm_head_sample(gpu):
    M, N, K = 10, 128256 // 16 * 16, 4096
    g = torch.Generator(device=gpu).manual_seed(7)
    x = torch.randn(M, K, device=gpu, generator=g).bfloat16()
    w = (torch.randn(N, K, device=gpu, generator=g) * 0.02).bfloat16()
    temps = torch.zeros(M, device=gpu)
    temps[5:] = 0.8
    seeds = torch.arange(M, device=gpu, dtype=torch.int64) * 7919 + 3
    step = torch.tensor([11], device=gpu, dtype=torch.int64)
    tile_keys = torch.empty(M * (N // 16), device=gpu, dtype=torch.int64)
    out_keys = torch.empty(M, device=gpu, dtype=torch.int64)
    out_ids = torch.empty(M, device=gpu, dtype=torch.int32)
    logits = torch.empty(M, N, device=gpu)
    ops.lm_head_sample(x, w, temps, seeds, step, tile_keys, out_keys, out_ids, 0, logits)
    ref_logits = x.float() @ w.float().t()
    _close(logits, ref_logits, atol=2e-3, rtol=1e-3)
    # greedy rows: kernel argmax must be the argmax of its own logits
    ids = out_ids.cpu().long()
    own = logits.cpu()
    assert torch.equal(ids[:5], own[:5].argmax(-1))
    # sampled rows: same RNG as the torch port (compare on the kernel's own logits)
    _, ids_ref = ref.sample_keys(own, temps.cpu(), seeds.cpu(), 11)
    assert (ids[5:] == ids_ref[5:]).float().mean() >= 0.8


def test_logits_argmax(gpu):
    """Wide-batch sampler over materialised fp32 logits: the fused epilogue's keys and RNG (greedy rows
    and Gumbel-max rows, with a vocab-shard offset) against the torch port: the same tokens, keys equal
    up to a few ulps of the noised value (device __logf)."""
    M, N = 70, 32000
    g = torch.Generator(device=gpu).manual_seed(17)
    logits = torch.randn(M, N, device=gpu, generator=g) * 3
    logits[3, 100] = logits[3, 200] = 1e3  # tie: the smaller vocab index wins
    temps = torch.zeros(M, device=gpu)
    temps[40:] = 0.7
    seeds = torch.arange(M, device=gpu, dtype=torch.int64) * 104729 - 5
    step = torch.tensor([23], device=gpu, dtype=torch.int64)
    out_keys = torch.empty(M, device=gpu, dtype=torch.int64)
    out_ids = torch.empty(M, device=gpu, dtype=torch.int32)
    ops.logits_argmax(logits, temps, seeds, step, out_keys, out_ids, n_offset=64000)
    keys_ref, ids_ref = ref.sample_keys(logits.cpu(), temps.cpu(), seeds.cpu(), 23, 64000)
    assert int(out_ids[3]) == 64100
    assert torch.equal(out_ids.cpu().long(), ids_ref)
    kk = out_keys.cpu()
    assert torch.equal(kk & 0xFFFFFFFF, keys_ref & 0xFFFFFFFF)  # same winning index
    assert int(((kk >> 32) - (keys_ref >> 32)).abs().max()) <= 4  # value bits: __logf vs torch.log ulps


def test_swiglu(gpu):
    T, F = 7, 14336
    g = torch.Generator(device=gpu).manual_seed(8)
    gu = torch.randn(4, T, 2 * F, device=gpu, generator=g)
    out = torch.empty(T, F, device=gpu, dtype=torch.bfloat16)
    ops.swiglu(gu, out)
    out_r = torch.empty(T, F, dtype=torch.bfloat16)
    ref.swiglu(gu.cpu(), out_r)
    _close(out, out_r, atol=2e-2, rtol=1e-2)
    gb = gu[0].bfloat16()
    ops.swiglu(gb, out)
    ref.swiglu(gb.cpu(), out_r)
    _close(out, out_r, atol=2e-2, rtol=1e-2)


@pytest.mark.parametrize("N,T,E,k", [(2, 243, 8, 2), (8, 1000, 8, 2), (4, 37, 8, 2)])
def test_moe_owner_pack_and_combine(gpu, N, T, E, k):
    """Replicated-token expert exchange kernels (moe.hip moe_owner_*): every rank packs the weighted partials of
    its local experts by slice owner; routing them like the xGMI a2a would (block s of rank q's send -> block q
    of rank s's recv) and combining must give each owner exactly the fp32 full MoE combine of its slice (up to
    one bf16 rounding), whatever order the atomics placed the rows in."""
    from symmetry_amd.ops import reference

    d = 256
    S = -(-T // N)
    g = torch.Generator(device="cpu").manual_seed(T + N)
    R = T * k
    ids = torch.stack([torch.randperm(E, generator=g)[:k] for _ in range(T)]).view(-1).int()
    w = torch.rand(R, generator=g)
    dst = torch.randperm(R, generator=g).int()  # row of each (token, slot) in the expert-sorted buffer
    y = torch.randn(R, d, generator=g)
    full = torch.zeros(T, d)
    reference.moe_combine(y, dst, ids, 0, E, w, k, full, False)
    El = E // N
    sends, sides, counts = [], [], []
    for q in range(N):
        send = torch.full((N * S, d), float("nan"), device=gpu)
        side = torch.full((N * S,), -1, dtype=torch.int32, device=gpu)
        cursor = torch.full((N,), 99, dtype=torch.int32, device=gpu)
        ops.moe_owner_pack(y.to(gpu), dst.to(gpu), ids.to(gpu), w.to(gpu), q * El, (q + 1) * El, k, S, cursor, send,
                           side)
        torch.cuda.synchronize()
        sends.append(send.cpu())
        sides.append(side.cpu())
        counts.append(cursor.cpu())
    for s in range(N):  # owner s
        recv = torch.zeros(N * S, d)
        rside = torch.full((N * S,), -1, dtype=torch.int32)
        rcnt = torch.zeros(N, dtype=torch.int32)
        for q in range(N):
            n = int(counts[q][s])
            recv[q * S:q * S + n] = sends[q][s * S:s * S + n]
            rside[q * S:q * S + n] = sides[q][s * S:s * S + n]
            rcnt[q] = n
        lo, hi = min(T, s * S), min(T, (s + 1) * S)
        out = torch.full((S, d), float("nan"), device=gpu, dtype=torch.bfloat16)
        pos = torch.empty(N * S, dtype=torch.int32, device=gpu)
        ops.moe_owner_combine(recv.to(gpu), rside.to(gpu), rcnt.to(gpu), hi - lo, pos, out)
        torch.cuda.synchronize()
        want = full[lo:hi]
        got = out[: hi - lo].float().cpu()
        assert ((got - want).abs() <= 1e-5 + want.abs() * 2.0 ** -8).all(), float((got - want).abs().max())
        assert (out[hi - lo:] == 0).all()
