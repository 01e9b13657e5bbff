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


@pytest.mark.parametrize("M", [1, 10, 33])
def test_gemm_tile_split_k(gpu, M):
    """gemm_tile split across workgroups in k (variants 21..24: 2 / 4 splits at 4 / 8 waves; the default for
    few-tile long-K shards such as Llama-3-70B's TP=8 QKV): every fused epilogue matches the fp32 reference,
    repeat launches are bitwise equal (fixed split order) and every tile's arrival counter is re-armed."""
    from symmetry_amd.ops import _native

    lib = _native.ops()
    D, BS, NB, Hq, Hkv, K = 128, 32, 8, 8, 1, 8192
    try:
        for v in (21, 22, 23, 24):
            lib.decode_gemm_variant(v)
            x, W, s = _inputs(gpu, M, 1280, K, seed=40 + v)
            y0, y1 = torch.empty(M, 1280, device=gpu), torch.empty(M, 1280, device=gpu)
            ops.dg_f32(x, W, s, 1e-5, y0)
            ops.dg_f32(x, W, s, 1e-5, y1)
            assert torch.equal(y0, y1), v
            y_ref = torch.empty(M, 1280)
            ref.dg_f32(x.cpu(), W.cpu(), s.cpu(), 1e-5, y_ref)
            _close(y0, y_ref, atol=2e-3, rtol=1e-2)

            Wq = W[qkv_perm(Hq, Hkv, D).to(gpu)].contiguous()
            cs = ref.rope_table(1024, D, 500000.0, device=gpu)
            pos = torch.arange(M, device=gpu, dtype=torch.int32) * 7
            slots = torch.randperm(NB * BS, device=gpu)[:M].int()
            q = torch.empty(M, Hq, D, device=gpu, dtype=torch.bfloat16)
            kc = torch.zeros(NB, Hkv, BS, D, device=gpu, dtype=torch.bfloat16)
            vc = torch.zeros(NB, Hkv, D, BS, device=gpu, dtype=torch.bfloat16)
            ops.dg_qkv(x, Wq, s, 1e-5, pos, slots, cs, q, kc, vc, Hq, Hkv)
            q_r, kc_r, vc_r = torch.empty(M, Hq, D, dtype=torch.bfloat16), torch.zeros_like(kc.cpu()), \
                torch.zeros_like(vc.cpu())
            ref.dg_qkv(x.cpu(), Wq.cpu(), s.cpu(), 1e-5, pos.cpu(), slots.cpu(), cs.cpu(), q_r, kc_r, vc_r, Hq, Hkv)
            _close(q, q_r, atol=2e-2, rtol=2e-2)
            _close(kc, kc_r, atol=2e-2, rtol=2e-2)
            _close(vc, vc_r, atol=2e-2, rtol=2e-2)

            xr, Wr, _ = _inputs(gpu, M, 1024, 4096, seed=50 + v)
            g = torch.Generator(device=gpu).manual_seed(v)
            resid = torch.randn(M, 1024, device=gpu, generator=g)
            wn = (torch.randn(1024, device=gpu, generator=g) * 0.1 + 1).bfloat16()
            xw = torch.empty(M, 1024, device=gpu, dtype=torch.bfloat16)
            ss = torch.empty(M, 64, device=gpu)
            r_ref, xw_ref, ss_ref = resid.cpu().clone(), torch.empty(M, 1024, dtype=torch.bfloat16), torch.empty(M, 64)
            ops.dg_resid(xr, Wr, resid, wn, xw, ss)
            ref.dg_resid(xr.cpu(), Wr.cpu(), r_ref, wn.cpu(), xw_ref, ss_ref)
            _close(resid, r_ref, atol=2e-3, rtol=1e-3)
            _close(xw, xw_ref, atol=2e-2, rtol=1e-2)
            _close(ss, ss_ref, atol=1e-2, rtol=1e-3)

            F = 640
            Wg = W[gu_perm(F).to(gpu)].contiguous()
            act = torch.empty(M, F, device=gpu, dtype=torch.bfloat16)
            ops.dg_swiglu(x, Wg, s, 1e-5, act)
            act_ref = torch.empty(M, F, dtype=torch.bfloat16)
            ref.dg_swiglu(x.cpu(), Wg.cpu(), s.cpu(), 1e-5, act_ref)
            _close(act, act_ref, atol=1e-2, rtol=2e-2)
        torch.cuda.synchronize()
        assert int(ops.decode_ks_ws(gpu)[1].abs().sum()) == 0
    finally:
        lib.decode_gemm_variant(-1)


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
