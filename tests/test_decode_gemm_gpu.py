"""Fused decode GEMMs (csrc/kernels/decode_gemm.hip) against the fp32 references.

Shapes cover the 8-wave (K % 512 == 0) and 4-wave (K = 256, K = 1792: Llama-3-8B down_proj at
TP=8) decompositions and 1..4 column tiles (M = 1, 7, 16, 33, 64).
"""
import pytest
import torch

from symmetry_amd import ops
from symmetry_amd.models.layout import gu_perm, qkv_perm
from symmetry_amd.ops import reference as ref

pytestmark = pytest.mark.gpu

MS = [1, 7, 16, 33, 64]


def _close(a, b, atol, rtol=0.0):
    a, b = a.float().cpu(), b.float().cpu()
    err = (a - b).abs()
    assert torch.isfinite(a).all(), "non-finite output"
    assert (err <= atol + rtol * b.abs()).all(), f"max err {err.max().item():.4g}"


def _inputs(gpu, M, N, K, seed=0, ss=True):
    g = torch.Generator(device=gpu).manual_seed(seed)
    x = torch.randn(M, K, device=gpu, generator=g).bfloat16()
    W = (torch.randn(N, K, device=gpu, generator=g) / K ** 0.5).bfloat16()
    s = (torch.rand(M, K // 16, device=gpu, generator=g) * 16 + 1) if ss else None
    return x, W, s


@pytest.mark.parametrize("M", MS)
@pytest.mark.parametrize("N,K", [(4096, 4096), (512, 256), (4096, 1792)])
def test_dg_f32(gpu, M, N, K):
    x, W, s = _inputs(gpu, M, N, K)
    y = torch.empty(M, N, device=gpu)
    ops.dg_f32(x, W, s, 1e-5, y)
    y_ref = torch.empty(M, N)
    ref.dg_f32(x.cpu(), W.cpu(), s.cpu(), 1e-5, y_ref)
    _close(y, y_ref, atol=2e-3, rtol=1e-2)
    ops.dg_f32(x, W, None, 0.0, y)
    ref.dg_f32(x.cpu(), W.cpu(), None, 0.0, y_ref)
    _close(y, y_ref, atol=2e-3, rtol=1e-2)


@pytest.mark.parametrize("M", MS)
@pytest.mark.parametrize("N,K", [(4096, 4096), (1024, 1792)])
def test_dg_resid(gpu, M, N, K):
    x, W, _ = _inputs(gpu, M, N, K, seed=1)
    g = torch.Generator(device=gpu).manual_seed(2)
    resid = torch.randn(M, N, device=gpu, generator=g)
    wn = (torch.randn(N, device=gpu, generator=g) * 0.1 + 1).bfloat16()
    xw = torch.empty(M, N, device=gpu, dtype=torch.bfloat16)
    ss = torch.empty(M, N // 16, device=gpu)
    r_ref, xw_ref, ss_ref = resid.cpu().clone(), torch.empty(M, N, dtype=torch.bfloat16), torch.empty(M, N // 16)
    ops.dg_resid(x, W, resid, wn, xw, ss)
    ref.dg_resid(x.cpu(), W.cpu(), r_ref, wn.cpu(), xw_ref, ss_ref)
    _close(resid, r_ref, atol=2e-3, rtol=1e-3)
    _close(xw, xw_ref, atol=2e-2, rtol=1e-2)
    _close(ss, ss_ref, atol=1e-2, rtol=1e-3)


@pytest.mark.parametrize("M", MS)
@pytest.mark.parametrize("F,K", [(1792, 4096), (512, 256), (14336, 4096)])
def test_dg_swiglu(gpu, M, F, K):
    x, W, s = _inputs(gpu, M, 2 * F, K, seed=3)
    W = W[gu_perm(F).to(gpu)].contiguous()
    act = torch.empty(M, F, device=gpu, dtype=torch.bfloat16)
    ops.dg_swiglu(x, W, s, 1e-5, act)
    act_ref = torch.empty(M, F, dtype=torch.bfloat16)
    ref.dg_swiglu(x.cpu(), W.cpu(), s.cpu(), 1e-5, act_ref)
    _close(act, act_ref, atol=1e-2, rtol=2e-2)


@pytest.mark.parametrize("M", MS)
# (8, 1, 8192): the Llama-3-70B TP=8 shard (64 / 8 q heads, ONE kv head per rank, d = 8192)
@pytest.mark.parametrize("Hq,Hkv,K", [(32, 8, 4096), (4, 1, 512), (2, 1, 256), (8, 1, 8192)])
def test_dg_qkv(gpu, M, Hq, Hkv, K):
    D, BS, NB = 128, 32, 8
    N = (Hq + 2 * Hkv) * D
    x, W, s = _inputs(gpu, M, N, K, seed=4)
    W = W[qkv_perm(Hq, Hkv, D).to(gpu)].contiguous()
    cs = ref.rope_table(1024, D, 500000.0, device=gpu)
    g = torch.Generator(device=gpu).manual_seed(5)
    pos = torch.randint(0, 1024, (M,), device=gpu, generator=g, dtype=torch.int32)
    slots = torch.randperm(NB * BS, device=gpu, generator=g)[:M].int()
    slots[0] = -1  # a row without a cache write
    q = torch.empty(M, Hq, D, device=gpu, dtype=torch.bfloat16)
    kc = torch.zeros(NB, Hkv, BS, D, device=gpu, dtype=torch.bfloat16)
    vc = torch.zeros(NB, Hkv, D, BS, device=gpu, dtype=torch.bfloat16)
    ops.dg_qkv(x, W, s, 1e-5, pos, slots, cs, q, kc, vc, Hq, Hkv)
    q_r, kc_r, vc_r = torch.empty(M, Hq, D, dtype=torch.bfloat16), torch.zeros_like(kc.cpu()), torch.zeros_like(vc.cpu())
    ref.dg_qkv(x.cpu(), W.cpu(), s.cpu(), 1e-5, pos.cpu(), slots.cpu(), cs.cpu(), q_r, kc_r, vc_r, Hq, Hkv)
    _close(q, q_r, atol=2e-2, rtol=2e-2)
    _close(kc, kc_r, atol=2e-2, rtol=2e-2)
    _close(vc, vc_r, atol=2e-2, rtol=2e-2)


# 16032: Llama-3 vocab shard at TP=8; 128256: the full vocabulary (4-row-tile variant above 16 rows)
@pytest.mark.parametrize("M,N", [(m, 16032) for m in MS] + [(33, 128256), (64, 128256)])
def test_dg_argmax(gpu, M, N):
    K = 4096
    x, W, s = _inputs(gpu, M, N, K, seed=6)
    g = torch.Generator(device=gpu).manual_seed(7)
    temps = torch.where(torch.arange(M, device=gpu) % 2 == 0, 0.0, 0.8).float()
    seeds = torch.randint(0, 1 << 62, (M,), device=gpu, generator=g)
    step = torch.tensor([3], device=gpu, dtype=torch.int64)
    tk = torch.empty(M * (N // 16), device=gpu, dtype=torch.int64)
    keys = torch.empty(M, device=gpu, dtype=torch.int64)
    ids = torch.empty(M, device=gpu, dtype=torch.int32)
    logits = torch.empty(M, N, device=gpu)
    ops.dg_argmax(x, W, s, 1e-5, temps, seeds, step, tk, keys, ids, 100, logits)
    lg_ref = torch.empty(M, N)
    ref.dg_f32(x.cpu(), W.cpu(), s.cpu(), 1e-5, lg_ref)
    _close(logits, lg_ref, atol=2e-3, rtol=1e-2)
    # sample from the kernel's own logits (ties at fp32 rounding are not a kernel property)
    k_ref, i_ref = ref.sample_keys(logits.cpu(), temps.cpu(), seeds.cpu(), 3, 100)
    assert torch.equal(ids.cpu().long(), i_ref)
    greedy = temps.cpu() == 0  # sampled rows use __logf for the Gumbel noise: ids match, key bits may not
    assert torch.equal(keys.cpu()[greedy], k_ref[greedy])


@pytest.mark.parametrize("M,N", [(1, 128256), (10, 128256), (16, 16032), (33, 128256)])
def test_dg_argmax_preshuffled(gpu, M, N):
    """The lm_head as an MFMA-preshuffled copy (fused decode path): same logits / ids as the row-major weight."""
    from symmetry_amd.models.layout import preshuffle

    K = 4096
    x, W, s = _inputs(gpu, M, N, K, seed=16)
    temps = torch.zeros(M, device=gpu)
    seeds = torch.zeros(M, device=gpu, dtype=torch.int64)
    step = torch.tensor([1], device=gpu, dtype=torch.int64)
    outs = []
    for sh in (False, True):
        tk = torch.empty(M * (N // 16), device=gpu, dtype=torch.int64)
        keys = torch.empty(M, device=gpu, dtype=torch.int64)
        ids = torch.empty(M, device=gpu, dtype=torch.int32)
        logits = torch.empty(M, N, device=gpu)
        ops.dg_argmax(x, preshuffle(W) if sh else W, s, 1e-5, temps, seeds, step, tk, keys, ids, 0, logits, wshuf=sh)
        outs.append((logits, ids))
    lg_ref = torch.empty(M, N)
    ref.dg_f32(x.cpu(), W.cpu(), s.cpu(), 1e-5, lg_ref)
    _close(outs[1][0], lg_ref, atol=2e-3, rtol=1e-2)
    assert torch.equal(outs[1][1].cpu().long(), outs[1][0].cpu().argmax(1))


@pytest.mark.parametrize("T,P", [(33, 4), (64, 4), (3, 2)])
def test_add_prep_partial_sums_from_slabs(gpu, T, P):
    """add_prep over fp32 k-split slabs with P workgroups per row: ss holds P column-slice partials."""
    d = 4096
    g = torch.Generator(device=gpu).manual_seed(9)
    w = (torch.randn(d, device=gpu, generator=g) * 0.1 + 1).bfloat16()
    resid = torch.randn(T, d, device=gpu, generator=g)
    slabs = torch.randn(4, T, d, device=gpu, generator=g)
    xw = torch.empty(T, d, device=gpu, dtype=torch.bfloat16)
    ss = torch.empty(T, P, device=gpu)
    r_ref, xw_ref, ss_ref = resid.cpu(), torch.empty(T, d, dtype=torch.bfloat16), torch.empty(T, P)
    ops.add_prep(slabs, resid, w, xw, ss)
    ref.add_prep(slabs.cpu(), r_ref, w.cpu(), xw_ref, ss_ref)
    _close(resid, r_ref, atol=1e-5)
    _close(xw, xw_ref, atol=1e-2, rtol=1e-2)
    _close(ss, ss_ref, atol=1e-2, rtol=1e-4)
    assert torch.allclose(ss.sum(1).cpu(), r_ref.pow(2).sum(1), rtol=1e-4)


@pytest.mark.parametrize("T,P", [(33, 4), (3, 2)])
def test_embed_prep_partial_sums(gpu, T, P):
    """embed_prep with ss [T, P]: P column-slice partials per row, the same layout as add_prep."""
    d = 4096
    g = torch.Generator(device=gpu).manual_seed(10)
    table = torch.randn(300, d, device=gpu, generator=g).bfloat16()
    ids = torch.randint(0, 300, (T,), device=gpu, generator=g, dtype=torch.int32)
    w = (torch.randn(d, device=gpu, generator=g) * 0.1 + 1).bfloat16()
    resid = torch.empty(T, d, device=gpu)
    xw = torch.empty(T, d, device=gpu, dtype=torch.bfloat16)
    ss = torch.full((T, P), float("nan"), device=gpu)
    ops.embed_prep(ids, table, resid, w, xw, ss)
    r_ref, xw_ref, ss_ref = torch.empty(T, d), torch.empty(T, d, dtype=torch.bfloat16), torch.empty(T, P)
    ref.embed_prep(ids.cpu(), table.cpu(), r_ref, w.cpu(), xw_ref, ss_ref)
    _close(resid, r_ref, atol=0)
    _close(xw, xw_ref, atol=1e-2, rtol=1e-2)
    _close(ss, ss_ref, atol=1e-2, rtol=1e-4)


@pytest.mark.parametrize("T,d", [(1, 4096), (13, 4096), (5, 256)])
def test_prep_and_rownorm(gpu, T, d):
    g = torch.Generator(device=gpu).manual_seed(8)
    table = torch.randn(300, d, device=gpu, generator=g).bfloat16()
    ids = torch.randint(0, 300, (T,), device=gpu, generator=g, dtype=torch.int32)
    w = (torch.randn(d, device=gpu, generator=g) * 0.1 + 1).bfloat16()
    resid = torch.empty(T, d, device=gpu)
    xw = torch.empty(T, d, device=gpu, dtype=torch.bfloat16)
    ss = torch.empty(T, 1, device=gpu)
    ops.embed_prep(ids, table, resid, w, xw, ss)
    r_ref, xw_ref, ss_ref = torch.empty(T, d), torch.empty(T, d, dtype=torch.bfloat16), torch.empty(T, 1)
    ref.embed_prep(ids.cpu(), table.cpu(), r_ref, w.cpu(), xw_ref, ss_ref)
    _close(resid, r_ref, atol=0)
    _close(xw, xw_ref, atol=1e-2, rtol=1e-2)
    _close(ss, ss_ref, atol=1e-2, rtol=1e-4)
    delta = torch.randn(T, d, device=gpu, generator=g).bfloat16()
    ops.add_prep(delta, resid, w, xw, ss)
    ref.add_prep(delta.cpu(), r_ref, w.cpu(), xw_ref, ss_ref)
    _close(resid, r_ref, atol=1e-5)
    _close(xw, xw_ref, atol=1e-2, rtol=1e-2)
    _close(ss, ss_ref, atol=1e-2, rtol=1e-4)
    out = torch.empty(T, d, device=gpu, dtype=torch.bfloat16)
    ops.rownorm(xw, ss, 1e-5, out)
    out_ref = torch.empty(T, d, dtype=torch.bfloat16)
    ref.rownorm(xw_ref, ss_ref, 1e-5, out_ref)
    _close(out, out_ref, atol=2e-2, rtol=2e-2)


def test_rope_cache_perm_and_swiglu_interleaved(gpu):
    """Library-GEMM path consumers of the decode layout."""
    T, Hq, Hkv, D, BS = 9, 4, 2, 128, 32
    g = torch.Generator(device=gpu).manual_seed(9)
    qkv = torch.randn(T, (Hq + 2 * Hkv) * D, device=gpu, generator=g).bfloat16()
    cs = ref.rope_table(64, D, 500000.0, device=gpu)
    pos = torch.arange(T, device=gpu, dtype=torch.int32)
    slots = torch.arange(T, device=gpu, dtype=torch.int32)
    q = torch.empty(T, Hq, D, device=gpu, dtype=torch.bfloat16)
    kc = torch.zeros(1, Hkv, BS, D, device=gpu, dtype=torch.bfloat16)
    vc = torch.zeros(1, Hkv, D, BS, device=gpu, dtype=torch.bfloat16)
    ops.rope_cache(qkv, pos, slots, cs, q, kc, vc, Hq, Hkv, perm=True)
    q_r, kc_r, vc_r = torch.empty(T, Hq, D, dtype=torch.bfloat16), torch.zeros_like(kc.cpu()), torch.zeros_like(vc.cpu())
    ref.rope_cache(qkv.cpu(), pos.cpu(), slots.cpu(), cs.cpu(), q_r, kc_r, vc_r, Hq, Hkv, perm=True)
    _close(q, q_r, atol=2e-2, rtol=1e-2)
    _close(kc, kc_r, atol=2e-2, rtol=1e-2)
    _close(vc, vc_r, atol=0)
    F = 256
    gu = torch.randn(T, 2 * F, device=gpu, generator=g).bfloat16()
    a = torch.empty(T, F, device=gpu, dtype=torch.bfloat16)
    ops.swiglu(gu, a, interleaved=True)
    a_r = torch.empty(T, F, dtype=torch.bfloat16)
    ref.swiglu(gu.cpu(), a_r, interleaved=True)
    _close(a, a_r, atol=2e-2, rtol=1e-2)


@pytest.mark.parametrize("M", [1, 10, 33, 64])
def test_preshuffled_weight_stream(gpu, M):
    """MFMA-preshuffled weights (1 KB contiguous per wave load) give the row-major result exactly."""
    from symmetry_amd.models.layout import preshuffle
    from symmetry_amd.ops import _native

    lib = _native.ops()
    try:
        for v in (0, 3, 4, 7, 12, 13, 14):  # same decomposition on both layouts -> same summation order -> bitwise equal
            lib.decode_gemm_variant(v)
            for N, K in ((4096, 4096), (28672, 4096), (4096, 1792)):
                x, W, s = _inputs(gpu, M, N, K, seed=12)
                y0 = torch.empty(M, N, device=gpu)
                y1 = torch.empty(M, N, device=gpu)
                ops.dg_f32(x, W, s, 1e-5, y0)
                ops.dg_f32(x, preshuffle(W), s, 1e-5, y1, wshuf=True)
                assert torch.equal(y0, y1), (v, N, K)
    finally:
        lib.decode_gemm_variant(-1)


@pytest.mark.parametrize("M", [1, 4, 10, 16])
@pytest.mark.parametrize("shuf", [False, True])
def test_decode_mlp_persistent(gpu, M, shuf):
    """Persistent O -> gate_up/SwiGLU -> down launch == the three separate fused GEMMs (and the fp32 ref);
    the control block re-arms itself (ctl all zero after every launch, including graph replays)."""
    from symmetry_amd.models.layout import preshuffle

    d, dq, F = 4096, 4096, 14336
    g = torch.Generator(device=gpu).manual_seed(21 + M)
    attn = torch.randn(M, dq, device=gpu, generator=g).bfloat16()
    Wo = (torch.randn(d, dq, device=gpu, generator=g) / dq ** 0.5).bfloat16()
    Wgu = (torch.randn(2 * F, d, device=gpu, generator=g) / d ** 0.5).bfloat16()[gu_perm(F).to(gpu)].contiguous()
    Wd = (torch.randn(d, F, device=gpu, generator=g) / F ** 0.5).bfloat16()
    resid0 = torch.randn(M, d, device=gpu, generator=g)
    ln2 = (torch.randn(d, device=gpu, generator=g) * 0.1 + 1).bfloat16()
    wn = (torch.randn(d, device=gpu, generator=g) * 0.1 + 1).bfloat16()
    W3 = [preshuffle(w) for w in (Wo, Wgu, Wd)] if shuf else [Wo, Wgu, Wd]

    def buffers():
        return (resid0.clone(), torch.empty(M, d, device=gpu, dtype=torch.bfloat16),
                torch.empty(M, d // 16, device=gpu), torch.empty(M, F, device=gpu, dtype=torch.bfloat16))

    # sequential fused path
    r_s, xw_s, ss_s, act_s = buffers()
    ops.dg_resid(attn, W3[0], r_s, ln2, xw_s, ss_s, wshuf=shuf)
    ops.dg_swiglu(xw_s, W3[1], ss_s, 1e-5, act_s, wshuf=shuf)
    ops.dg_resid(act_s, W3[2], r_s, wn, xw_s, ss_s, wshuf=shuf)
    # persistent
    ctl = torch.zeros(ops.DECODE_MLP_CTL, device=gpu, dtype=torch.int32)
    r_p, xw_p, ss_p, act_p = buffers()
    ops.decode_mlp(attn, *W3, r_p, ln2, wn, xw_p, ss_p, act_p, ctl, 1e-5, wshuf=shuf)
    torch.cuda.synchronize()
    assert not ctl.any(), ctl.tolist()
    _close(act_p, act_s, atol=3e-2, rtol=2e-2)
    _close(r_p, r_s, atol=3e-3, rtol=1e-3)
    _close(xw_p, xw_s, atol=3e-2, rtol=2e-2)
    _close(ss_p, ss_s, atol=1e-2, rtol=2e-3)
    # fp32 reference
    r_r, xw_r, ss_r = resid0.cpu().clone(), torch.empty(M, d, dtype=torch.bfloat16), torch.empty(M, d // 16)
    act_r = torch.empty(M, F, dtype=torch.bfloat16)
    ref.decode_mlp(attn.cpu(), Wo.cpu(), Wgu.cpu(), Wd.cpu(), r_r, ln2.cpu(), wn.cpu(), xw_r, ss_r, act_r, 1e-5)
    _close(r_p, r_r, atol=5e-3, rtol=2e-3)
    # graph replays: same inputs -> same outputs, counters re-armed each time
    r_g, xw_g, ss_g, act_g = buffers()
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, stream=s):
            ops.decode_mlp(attn, *W3, r_g, ln2, wn, xw_g, ss_g, act_g, ctl, 1e-5, wshuf=shuf)
    torch.cuda.synchronize()
    for _ in range(3):
        r_g.copy_(resid0)
        graph.replay()
        torch.cuda.synchronize()
        assert not ctl.any(), ctl.tolist()
        assert torch.equal(r_g, r_p) and torch.equal(act_g, act_p) and torch.equal(ss_g, ss_p)


@pytest.mark.parametrize("M", [1, 4, 10, 16])
@pytest.mark.parametrize("Hq,Hkv,d,shuf", [(32, 8, 4096, True), (32, 8, 4096, False), (16, 2, 2048, True)])
def test_decode_block_fused_equals_three_launches(gpu, M, Hq, Hkv, d, shuf):
    """QKV -> attention -> O in one launch (decode_block) vs dg_qkv + attn_decode + dg_resid with decode_gemm
    variant 0: the QKV tiles (q, K/V cache) are bitwise equal; attention uses 256-token partitions (one
    32-token group per wave) instead of 512, so its output and what follows match to bf16 rounding,
    including multi-partition contexts (split-KV combine inside the launch).  The O tile given the SAME
    attention rows is bitwise equal; the control block re-arms itself, also under graph replay."""
    import math

    from symmetry_amd.models.layout import preshuffle
    from symmetry_amd.ops import _native

    D, BS = 128, 64
    g = torch.Generator(device=gpu).manual_seed(100 + M)
    ctx_lens = [(37 * i * i + 100 * i + 1) % 2100 + 1 for i in range(M)]
    max_blocks = max((c + BS - 1) // BS for c in ctx_lens) + 1
    NB = sum((c + BS - 1) // BS for c in ctx_lens) + 3
    kc0 = torch.randn(NB, Hkv, BS, D, device=gpu, generator=g).bfloat16()
    vc0 = torch.randn(NB, Hkv, D, BS, device=gpu, generator=g).bfloat16()
    perm = torch.randperm(NB, generator=torch.Generator().manual_seed(5)).tolist()
    bt = torch.zeros(M, max_blocks, dtype=torch.int32)
    i = 0
    for s, c in enumerate(ctx_lens):
        for blk in range((c + BS - 1) // BS):
            bt[s, blk] = perm[i]
            i += 1
    pos = torch.tensor([c - 1 for c in ctx_lens], dtype=torch.int32)
    slots = torch.tensor([int(bt[s, p // BS]) * BS + p % BS for s, p in enumerate(pos.tolist())], dtype=torch.int32)
    bt, pos, slots = bt.to(gpu), pos.to(gpu), slots.to(gpu)
    ctx = torch.tensor(ctx_lens, device=gpu, dtype=torch.int32)
    N = (Hq + 2 * Hkv) * D
    xw = torch.randn(M, d, device=gpu, generator=g).bfloat16()
    ss_in = torch.rand(M, d // 16, device=gpu, generator=g) * 16 + 1
    Wqkv = (torch.randn(N, d, device=gpu, generator=g) / d ** 0.5).bfloat16()[qkv_perm(Hq, Hkv, D).to(gpu)].contiguous()
    Wo = (torch.randn(d, Hq * D, device=gpu, generator=g) / (Hq * D) ** 0.5).bfloat16()
    if shuf:
        Wqkv, Wo = preshuffle(Wqkv), preshuffle(Wo)
    resid0 = torch.randn(M, d, device=gpu, generator=g)
    ln2 = (torch.randn(d, device=gpu, generator=g) * 0.1 + 1).bfloat16()
    cs = ref.rope_table(4096, D, 500000.0, device=gpu)
    scale = 1 / math.sqrt(D)
    max_parts = (max_blocks * BS + ops.ATTN_BLOCK_PART - 1) // ops.ATTN_BLOCK_PART

    def state():
        return dict(kc=kc0.clone(), vc=vc0.clone(), q=torch.empty(M, Hq, D, device=gpu, dtype=torch.bfloat16),
                    attn=torch.empty(M, Hq, D, device=gpu, dtype=torch.bfloat16), resid=resid0.clone(),
                    xw=xw.clone(), ss=ss_in.clone(), tmp_o=torch.empty(M, Hq, max_parts, D, device=gpu),
                    tmp_ml=torch.empty(M, Hq, max_parts, 2, device=gpu),
                    cnt=torch.zeros(M * Hkv, device=gpu, dtype=torch.int32))

    nat = _native.ops()
    nat.decode_gemm_variant(0)
    try:
        a = state()
        ss_t = torch.empty(M, d // 16, device=gpu)
        ops.dg_qkv(a["xw"], Wqkv, a["ss"], 1e-5, pos, slots, cs, a["q"], a["kc"], a["vc"], Hq, Hkv, wshuf=shuf)
        ops.attn_decode(a["q"], a["kc"], a["vc"], bt, ctx, a["attn"], a["tmp_o"], a["tmp_ml"], a["cnt"], scale)
        ops.dg_resid(a["attn"].view(M, -1), Wo, a["resid"], ln2, a["xw"], ss_t, wshuf=shuf)
        a["ss"] = ss_t
        bf = state()
        ctl = torch.zeros(ops.DECODE_BLOCK_CTL, device=gpu, dtype=torch.int32)
        # ss_in and ss_out alias, xw and xw_out alias: the engine's buffers
        ops.decode_block(bf["xw"], Wqkv, bf["ss"], 1e-5, pos, slots, cs, bf["q"], bf["kc"], bf["vc"], bt, ctx,
                         bf["attn"], bf["tmp_o"], bf["tmp_ml"], bf["cnt"], scale, Wo, bf["resid"], ln2, bf["xw"],
                         bf["ss"], ctl, wshuf=shuf)
        torch.cuda.synchronize()
        assert not ctl.any(), ctl.nonzero().flatten().tolist()
        assert not bf["cnt"].any()
        for k in ("q", "kc", "vc"):
            assert torch.equal(bf[k], a[k]), k
        _close(bf["attn"], a["attn"], atol=2e-2, rtol=2e-2)
        _close(bf["resid"], a["resid"], atol=2e-2, rtol=1e-2)
        # the O tile itself is bitwise the 3-launch one: feed the fused attention rows to dg_resid
        r2, xw2, ss2 = resid0.clone(), torch.empty_like(xw), torch.empty(M, d // 16, device=gpu)
        ops.dg_resid(bf["attn"].view(M, -1), Wo, r2, ln2, xw2, ss2, wshuf=shuf)
        assert torch.equal(r2, bf["resid"]) and torch.equal(xw2, bf["xw"]) and torch.equal(ss2, bf["ss"])
        # attention against the fp32 reference
        at_r = torch.empty(M, Hq, D, dtype=torch.bfloat16)
        ref.attn_decode(bf["q"].cpu(), bf["kc"].cpu(), bf["vc"].cpu(), bt.cpu(), ctx.cpu(), at_r, scale=scale)
        _close(bf["attn"], at_r, atol=2e-2, rtol=2e-2)
        # graph replays from the same inputs: identical outputs, counters re-armed every time
        gr = state()
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph, stream=s):
                ops.decode_block(gr["xw"], Wqkv, gr["ss"], 1e-5, pos, slots, cs, gr["q"], gr["kc"], gr["vc"], bt, ctx,
                                 gr["attn"], gr["tmp_o"], gr["tmp_ml"], gr["cnt"], scale, Wo, gr["resid"], ln2,
                                 gr["xw"], gr["ss"], ctl, wshuf=shuf)
        torch.cuda.synchronize()
        for _ in range(3):
            gr["resid"].copy_(resid0)
            gr["xw"].copy_(xw)
            gr["ss"].copy_(ss_in)
            graph.replay()
            torch.cuda.synchronize()
            assert not ctl.any()
            for k in ("q", "attn", "resid", "xw", "ss"):
                assert torch.equal(gr[k], bf[k]), k
    finally:
        nat.decode_gemm_variant(-1)


def _mg(gpu, M, N, K):
    """(slab, counters, rw) for the mgemm-with-epilogue form of a projection (ops.choose_mgemm's pick, or a
    forced 4-way split when the chooser declines: the in-launch reduction is what is under test)."""
    pick = ops.choose_mgemm(M, N, K) or (1, 4 if K % 256 == 0 else 1)
    rw, S = pick
    return (torch.full((S, M, N), float("nan"), device=gpu), torch.zeros(N // 64, dtype=torch.int32, device=gpu),
            rw), S


@pytest.mark.parametrize("M", [1, 20, 33, 64, 100])
@pytest.mark.parametrize("kind", ["qkv", "resid", "swiglu"])
def test_mgemm_fused_epilogues(gpu, M, kind):
    """mgemm with the fused decode epilogues (the general decode path of 20-256 rows): the last k-split
    workgroup of each column group reduces the fp32 slabs in split order and runs the same epilogue as the
    decode GEMMs, against the fp32 references; run twice (the counters re-arm themselves)."""
    from symmetry_amd.models.layout import preshuffle

    if kind == "qkv":
        Hq, Hkv, K, D = 32, 8, 4096, 128
        N = (Hq + 2 * Hkv) * D
    elif kind == "resid":
        N, K = 4096, 4096
    else:
        N, K = 2 * 1792, 4096
    x, W, s = _inputs(gpu, M, N, K, seed=7)
    if kind == "qkv":
        W = W[qkv_perm(Hq, Hkv, D).to(gpu)].contiguous()
    elif kind == "swiglu":
        W = W[gu_perm(N // 2).to(gpu)].contiguous()
    Ws = preshuffle(W)
    mg, S = _mg(gpu, M, N, K)
    for rep in range(2):
        if kind == "qkv":
            BS, NB = 32, 16
            cs = ref.rope_table(1024, D, 500000.0, device=gpu)
            g = torch.Generator(device=gpu).manual_seed(5)
            pos = torch.randint(0, 1024, (M,), device=gpu, generator=g, dtype=torch.int32)
            slots = torch.randperm(NB * BS, device=gpu, generator=g)[:M].int()
            slots[0] = -1
            q = torch.empty(M, Hq, D, device=gpu, dtype=torch.bfloat16)
            kc = torch.zeros(NB, Hkv, BS, D, device=gpu, dtype=torch.bfloat16)
            vc = torch.zeros(NB, Hkv, D, BS, device=gpu, dtype=torch.bfloat16)
            ops.dg_qkv(x, Ws, s, 1e-5, pos, slots, cs, q, kc, vc, Hq, Hkv, wshuf=True, mg=mg)
            q_r, kc_r, vc_r = torch.empty(M, Hq, D, dtype=torch.bfloat16), torch.zeros_like(kc.cpu()), torch.zeros_like(vc.cpu())
            ref.dg_qkv(x.cpu(), W.cpu(), s.cpu(), 1e-5, pos.cpu(), slots.cpu(), cs.cpu(), q_r, kc_r, vc_r, Hq, Hkv)
            _close(q, q_r, atol=2e-2, rtol=2e-2)
            _close(kc, kc_r, atol=2e-2, rtol=2e-2)
            _close(vc, vc_r, atol=2e-2, rtol=2e-2)
        elif kind == "resid":
            g = torch.Generator(device=gpu).manual_seed(2)
            resid = torch.randn(M, N, device=gpu, generator=g)
            wn = (torch.randn(N, device=gpu, generator=g) * 0.1 + 1).bfloat16()
            xw = torch.empty(M, N, device=gpu, dtype=torch.bfloat16)
            ss = torch.empty(M, N // 16, device=gpu)
            r_ref, xw_ref, ss_ref = resid.cpu().clone(), torch.empty(M, N, dtype=torch.bfloat16), torch.empty(M, N // 16)
            ops.dg_resid(x, Ws, resid, wn, xw, ss, wshuf=True, mg=mg)
            ref.dg_resid(x.cpu(), W.cpu(), r_ref, wn.cpu(), xw_ref, ss_ref)
            _close(resid, r_ref, atol=2e-3, rtol=1e-3)
            _close(xw, xw_ref, atol=2e-2, rtol=1e-2)
            _close(ss, ss_ref, atol=1e-2, rtol=1e-3)
        else:
            act = torch.empty(M, N // 2, device=gpu, dtype=torch.bfloat16)
            ops.dg_swiglu(x, Ws, s, 1e-5, act, wshuf=True, mg=mg)
            act_ref = torch.empty(M, N // 2, dtype=torch.bfloat16)
            ref.dg_swiglu(x.cpu(), W.cpu(), s.cpu(), 1e-5, act_ref)
            _close(act, act_ref, atol=1e-2, rtol=2e-2)
        torch.cuda.synchronize()
        assert int(mg[1].abs().sum()) == 0, "split-K counters must re-arm to zero"


@pytest.mark.parametrize("M", [1, 10, 16])
# (32, 8): Llama-3-8B QKV (384 tiles -> 768 half-K units); (4, 1): its TP=8 shard (48 tiles -> 192 quarter-K
# units); (16, 4, 2048): K = 2048 (U = 1 per split)
@pytest.mark.parametrize("Hq,Hkv,K", [(32, 8, 4096), (4, 1, 4096), (16, 4, 2048)])
def test_dg_qkv_ksplit_xres(gpu, M, Hq, Hkv, K):
    """x-resident decode GEMM with K split across workgroups (in-launch last-arriver reduction, decode_gemm.hip
    go_xres): same outputs as the fp32 reference and as the whole-K kernel, repeated launches (counters re-arm)."""
    from symmetry_amd.models.layout import preshuffle

    D, BS, NB = 128, 32, 8
    N = (Hq + 2 * Hkv) * D
    x, W, s = _inputs(gpu, M, N, K, seed=21)
    W = W[qkv_perm(Hq, Hkv, D).to(gpu)].contiguous()
    Ws = preshuffle(W)
    cs = ref.rope_table(1024, D, 500000.0, device=gpu)
    g = torch.Generator(device=gpu).manual_seed(22)
    pos = torch.randint(0, 1024, (M,), device=gpu, generator=g, dtype=torch.int32)
    slots = torch.randperm(NB * BS, device=gpu, generator=g)[:M].int()

    def run(mg):
        q = torch.empty(M, Hq, D, device=gpu, dtype=torch.bfloat16)
        kc = torch.zeros(NB, Hkv, BS, D, device=gpu, dtype=torch.bfloat16)
        vc = torch.zeros(NB, Hkv, D, BS, device=gpu, dtype=torch.bfloat16)
        ops.dg_qkv(x, Ws, s, 1e-5, pos, slots, cs, q, kc, vc, Hq, Hkv, wshuf=True, mg=mg)
        return q, kc, vc

    from symmetry_amd.ops import _native

    whole = run((None, None, 0))
    _native.ops().decode_ksplit(1)
    try:
        for _ in range(3):
            split = run(None)  # the device workspace: remainder tiles split over K
            for a, b in zip(split, whole):
                _close(a, b, atol=2e-2, rtol=2e-2)
    finally:
        _native.ops().decode_ksplit(0)
    assert int(ops.decode_ks_ws(x.device)[1].abs().sum()) == 0  # every tile's counter re-armed
    q_r, kc_r, vc_r = torch.empty(M, Hq, D, dtype=torch.bfloat16), torch.zeros(NB, Hkv, BS, D, dtype=torch.bfloat16), \
        torch.zeros(NB, Hkv, D, BS, dtype=torch.bfloat16)
    ref.dg_qkv(x.cpu(), W.cpu(), s.cpu(), 1e-5, pos.cpu(), slots.cpu(), cs.cpu(), q_r, kc_r, vc_r, Hq, Hkv)
    for a, b in zip(split, (q_r, kc_r, vc_r)):
        _close(a, b, atol=2e-2, rtol=2e-2)


@pytest.mark.parametrize("M", [1, 10])
def test_dg_resid_swiglu_ksplit_xres(gpu, M):
    """RESID / SWIGLU epilogues on the split-K x-resident kernel: N = 2048 at K = 4096 is 128 whole tiles (half
    the CUs) or 256 half-K units."""
    from symmetry_amd.models.layout import preshuffle

    F, K = 1024, 4096
    x, W, s = _inputs(gpu, M, 2 * F, K, seed=23)
    W = W[gu_perm(F).to(gpu)].contiguous()
    Ws = preshuffle(W)
    outs = []
    from symmetry_amd.ops import _native

    lib = _native.ops()
    for mg in ((None, None, 0), None):
        act = torch.empty(M, F, device=gpu, dtype=torch.bfloat16)
        lib.decode_ksplit(int(mg is None))
        try:
            ops.dg_swiglu(x, Ws, s, 1e-5, act, wshuf=True, mg=mg)
        finally:
            lib.decode_ksplit(0)
        outs.append(act)
    act_ref = torch.empty(M, F, dtype=torch.bfloat16)
    ref.dg_swiglu(x.cpu(), W.cpu(), s.cpu(), 1e-5, act_ref)
    for a in outs:
        _close(a, act_ref, atol=1e-2, rtol=2e-2)
    N = 2048
    x, W, _ = _inputs(gpu, M, N, K, seed=24)
    g = torch.Generator(device=gpu).manual_seed(25)
    resid0 = torch.randn(M, N, device=gpu, generator=g)
    wn = (torch.randn(N, device=gpu, generator=g) * 0.1 + 1).bfloat16()
    r_ref, xw_ref, ss_ref = resid0.cpu().clone(), torch.empty(M, N, dtype=torch.bfloat16), torch.empty(M, N // 16)
    ref.dg_resid(x.cpu(), W.cpu(), r_ref, wn.cpu(), xw_ref, ss_ref)
    for mg in ((None, None, 0), None):
        resid = resid0.clone()
        xw = torch.empty(M, N, device=gpu, dtype=torch.bfloat16)
        ss = torch.empty(M, N // 16, device=gpu)
        lib.decode_ksplit(int(mg is None))
        try:
            ops.dg_resid(x, preshuffle(W), resid, wn, xw, ss, wshuf=True, mg=mg)
        finally:
            lib.decode_ksplit(0)
        _close(resid, r_ref, atol=2e-3, rtol=1e-3)
        _close(xw, xw_ref, atol=2e-2, rtol=1e-2)
        _close(ss, ss_ref, atol=1e-2, rtol=1e-3)


@pytest.mark.parametrize("M", [1, 10, 16])
@pytest.mark.parametrize("Hq,Hkv,d", [(32, 8, 4096), (16, 2, 2048), (8, 1, 1024)])
def test_qkv_attn_fused_equals_two_launches(gpu, M, Hq, Hkv, d):
    """QKV + decode attention in one launch (qkv_attn: the attention units on the CUs the x-resident QKV grid
    leaves idle) vs dg_qkv + attn_decode: q, the paged K/V cache and the attention output are bitwise equal,
    including multi-partition contexts (split-KV combine in the launch); the control block and the split-KV
    counters re-arm themselves, also under graph replay; a block-table span the grid attention kernel does
    not serve (the streaming kernel's >= 1024 tokens) falls back (False, nothing enqueued)."""
    import math

    from symmetry_amd.models.layout import preshuffle

    D, BS = 128, 64
    g = torch.Generator(device=gpu).manual_seed(300 + M + Hq)
    ctx_lens = [(97 * i * i + 131 * i + 5) % 890 + 1 for i in range(M)]
    max_blocks = max((c + BS - 1) // BS for c in ctx_lens) + 1  # span < 1024: the grid attention kernel
    NB = sum((c + BS - 1) // BS for c in ctx_lens) + 3
    kc0 = torch.randn(NB, Hkv, BS, D, device=gpu, generator=g).bfloat16()
    vc0 = torch.randn(NB, Hkv, D, BS, device=gpu, generator=g).bfloat16()
    perm = torch.randperm(NB, generator=torch.Generator().manual_seed(7)).tolist()
    bt = torch.zeros(M, max_blocks, dtype=torch.int32)
    i = 0
    for s, c in enumerate(ctx_lens):
        for blk in range((c + BS - 1) // BS):
            bt[s, blk] = perm[i]
            i += 1
    pos = torch.tensor([c - 1 for c in ctx_lens], dtype=torch.int32)
    slots = torch.tensor([int(bt[s, p // BS]) * BS + p % BS for s, p in enumerate(pos.tolist())], dtype=torch.int32)
    bt, pos, slots = bt.to(gpu), pos.to(gpu), slots.to(gpu)
    ctx = torch.tensor(ctx_lens, device=gpu, dtype=torch.int32)
    N = (Hq + 2 * Hkv) * D
    xw = torch.randn(M, d, device=gpu, generator=g).bfloat16()
    ss_in = torch.rand(M, d // 16, device=gpu, generator=g) * 16 + 1
    Wqkv = (torch.randn(N, d, device=gpu, generator=g) / d ** 0.5).bfloat16()[qkv_perm(Hq, Hkv, D).to(gpu)].contiguous()
    Wqkv = preshuffle(Wqkv)
    cs = ref.rope_table(4096, D, 500000.0, device=gpu)
    scale = 1 / math.sqrt(D)
    max_parts = (max_blocks * BS + ops.ATTN_DECODE_PART - 1) // ops.ATTN_DECODE_PART

    def state():
        return dict(kc=kc0.clone(), vc=vc0.clone(), q=torch.empty(M, Hq, D, device=gpu, dtype=torch.bfloat16),
                    attn=torch.full((M, Hq, D), float("nan"), device=gpu, dtype=torch.bfloat16),
                    tmp_o=torch.empty(M, Hq, max_parts, D, device=gpu), tmp_ml=torch.empty(M, Hq, max_parts, 2, device=gpu),
                    cnt=torch.zeros(M * Hkv, device=gpu, dtype=torch.int32))

    def fused(st, ctl):
        return ops.qkv_attn(xw, Wqkv, ss_in, 1e-5, pos, slots, cs, st["q"], st["kc"], st["vc"], Hq, Hkv, True, bt, ctx,
                            st["attn"], st["tmp_o"], st["tmp_ml"], st["cnt"], scale, ctl)

    a = state()
    ops.dg_qkv(xw, Wqkv, ss_in, 1e-5, pos, slots, cs, a["q"], a["kc"], a["vc"], Hq, Hkv, wshuf=True)
    ops.attn_decode(a["q"], a["kc"], a["vc"], bt, ctx, a["attn"], a["tmp_o"], a["tmp_ml"], a["cnt"], scale)
    bf = state()
    ctl = torch.zeros(ops.QKV_ATTN_CTL, device=gpu, dtype=torch.int32)
    assert fused(bf, ctl)
    torch.cuda.synchronize()
    assert not ctl.any(), ctl.nonzero().flatten().tolist()
    assert not bf["cnt"].any()
    for k in ("q", "kc", "vc", "attn"):
        assert torch.equal(bf[k], a[k]), k
    at_r = torch.empty(M, Hq, D, dtype=torch.bfloat16)
    ref.attn_decode(bf["q"].cpu(), bf["kc"].cpu(), bf["vc"].cpu(), bt.cpu(), ctx.cpu(), at_r, scale=scale)
    _close(bf["attn"], at_r, atol=2e-2, rtol=2e-2)
    # graph replays from the same inputs: identical outputs, control words re-armed every time
    gr = state()
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, stream=s):
            assert fused(gr, ctl)
    torch.cuda.synchronize()
    for _ in range(3):
        gr["attn"].fill_(float("nan"))
        gr["kc"].copy_(kc0)
        gr["vc"].copy_(vc0)
        graph.replay()
        torch.cuda.synchronize()
        assert not ctl.any() and not gr["cnt"].any()
        for k in ("q", "kc", "vc", "attn"):
            assert torch.equal(gr[k], bf[k]), k
    # a 1024-token span: the standalone launch would stream (another kernel): not fused, nothing enqueued
    bt_long = torch.zeros(M, 16, dtype=torch.int32, device=gpu)
    bt_long[:, :max_blocks] = bt
    st = state()
    st["tmp_o"] = torch.empty(M, Hq, 4, D, device=gpu)
    st["tmp_ml"] = torch.empty(M, Hq, 4, 2, device=gpu)
    q_before = st["q"].clone()
    assert not ops.qkv_attn(xw, Wqkv, ss_in, 1e-5, pos, slots, cs, st["q"], st["kc"], st["vc"], Hq, Hkv, True,
                            bt_long, ctx, st["attn"], st["tmp_o"], st["tmp_ml"], st["cnt"], scale, ctl)
    torch.cuda.synchronize()
    assert torch.equal(st["kc"], kc0) and torch.equal(st["q"].view(-1)[:8], q_before.view(-1)[:8])


@pytest.mark.parametrize("M", [1, 10, 16])
# 8B QKV (384 tiles: 256 whole + 256 row halves), its TP=4 / TP=8 shards (96 / 48 tiles: halves only), and
# gate_up under TP=2 (896 tiles: 3 whole + 1 half per CU)
@pytest.mark.parametrize("what,Hq,Hkv,N", [("qkv", 32, 8, 0), ("qkv", 8, 2, 0), ("qkv", 4, 1, 0), ("gu", 0, 0, 14336)])
def test_xres_row_halves_bitwise(gpu, M, what, Hq, Hkv, N):
    """x-resident decode GEMM with remainder tiles split into row halves (rows {0-3, 8-11} / {4-7, 12-15} of a
    16-row MFMA tile in two workgroups, the other half's weight lanes masked off): bitwise equal to whole
    tiles (same sums, same order) for the QKV (RoPE pairs r / r + 8) and SwiGLU (gate / up rows r / r + 8)
    epilogues, and close to the fp32 reference."""
    from symmetry_amd.models.layout import preshuffle

    D, BS, NB, K = 128, 64, 8, 4096
    lib = ops._native.ops()
    g = torch.Generator(device=gpu).manual_seed(40 + M)
    if what == "qkv":
        N = (Hq + 2 * Hkv) * D
        x, W, s = _inputs(gpu, M, N, K, seed=41)
        W = W[qkv_perm(Hq, Hkv, D).to(gpu)].contiguous()
        cs = ref.rope_table(1024, D, 500000.0, device=gpu)
        pos = torch.randint(0, 1024, (M,), device=gpu, generator=g, dtype=torch.int32)
        slots = torch.randperm(NB * BS, device=gpu, generator=g)[:M].int()

        def run():
            q = torch.full((M, Hq, D), float("nan"), device=gpu, dtype=torch.bfloat16)
            kc = torch.zeros(NB, Hkv, BS, D, device=gpu, dtype=torch.bfloat16)
            vc = torch.zeros(NB, Hkv, D, BS, device=gpu, dtype=torch.bfloat16)
            ops.dg_qkv(x, preshuffle(W), s, 1e-5, pos, slots, cs, q, kc, vc, Hq, Hkv, wshuf=True)
            torch.cuda.synchronize()
            return q, kc, vc
    else:
        x, W, s = _inputs(gpu, M, N, K, seed=42)
        W = W[gu_perm(N // 2).to(gpu)].contiguous()

        def run():
            act = torch.full((M, N // 2), float("nan"), device=gpu, dtype=torch.bfloat16)
            ops.dg_swiglu(x, preshuffle(W), s, 1e-5, act, wshuf=True)
            torch.cuda.synchronize()
            return (act,)

    try:
        lib.decode_halves(1)
        halves = run()
        lib.decode_halves(0)
        whole = run()
    finally:
        lib.decode_halves(0)
    for a, b in zip(halves, whole):
        assert not torch.isnan(a.float()).any()
        assert torch.equal(a, b)
    if what == "qkv":
        q_r, kc_r, vc_r = (torch.empty(M, Hq, D, dtype=torch.bfloat16), torch.zeros(NB, Hkv, BS, D, dtype=torch.bfloat16),
                           torch.zeros(NB, Hkv, D, BS, dtype=torch.bfloat16))
        ref.dg_qkv(x.cpu(), W.cpu(), s.cpu(), 1e-5, pos.cpu(), slots.cpu(), cs.cpu(), q_r, kc_r, vc_r, Hq, Hkv)
        _close(halves[0], q_r, atol=2e-2, rtol=2e-2)
        _close(halves[1], kc_r, atol=2e-2, rtol=2e-2)
        _close(halves[2], vc_r, atol=2e-2, rtol=2e-2)
    else:
        act_r = torch.empty(M, N // 2, dtype=torch.bfloat16)
        ref.dg_swiglu(x.cpu(), W.cpu(), s.cpu(), 1e-5, act_r)
        _close(halves[0], act_r, atol=3e-2, rtol=2e-2)
