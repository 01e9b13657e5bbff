"""Prefill projection GEMM (csrc/kernels/pgemm.hip) against the fp32 product: every tile config, split-K, ragged
row counts (rows past M padded in-kernel), bf16 and fp32 outputs, and the fused epilogues."""
import math

import pytest
import torch

from symmetry_amd import ops
from symmetry_amd.models.layout import preshuffle

pytestmark = pytest.mark.gpu


def _close(a, b, atol, rtol=0.0):
    err = (a.float() - b.float()).abs()
    assert torch.isfinite(a.float()).all(), "non-finite output"
    bad = err > atol + rtol * b.float().abs()
    assert not bad.any(), f"max err {err.max().item():.4g} at {bad.nonzero()[0].tolist()} (atol {atol})"


@pytest.mark.parametrize("cfg", sorted(ops.PG_CFG_SHAPES))
@pytest.mark.parametrize("M", [1, 100, 383, 768, 1290])
@pytest.mark.parametrize("S", [1, 2])
def test_pgemm_vs_fp32(gpu, cfg, M, S):
    bm, bn = ops.pgemm_shape(cfg)
    N, K = 2 * bn, 1024
    g = torch.Generator(device=gpu).manual_seed(cfg * 100 + M + S)
    x = (torch.rand(M, K, device=gpu, generator=g) * 2 - 1).bfloat16()
    w = ((torch.rand(N, K, device=gpu, generator=g) * 2 - 1) * 0.05).bfloat16()
    ref = x.float() @ w.float().t()
    tiles = -(-M // bm) * (N // bn)
    slab = torch.empty(S, M, N, device=gpu) if S > 1 else None
    cnt = torch.zeros(tiles, dtype=torch.int32, device=gpu) if S > 1 else None
    y = torch.full((M, N), float("nan"), device=gpu)
    ops.pgemm(x, preshuffle(w), y, cfg, S, slab, cnt)
    _close(y, ref, atol=1e-3 * math.sqrt(K) * 0.05 + 1e-4, rtol=1e-3)
    yb = torch.full((M, N), float("nan"), device=gpu, dtype=torch.bfloat16)
    ops.pgemm(x, preshuffle(w), yb, cfg, S, slab, cnt)  # counters re-armed by the previous launch
    _close(yb, ref, atol=2e-2, rtol=8e-3)


def _inputs(gpu, M, N, K, seed):
    g = torch.Generator(device=gpu).manual_seed(seed)
    x = (torch.rand(M, K, device=gpu, generator=g) * 2 - 1).bfloat16()
    w = ((torch.rand(N, K, device=gpu, generator=g) * 2 - 1) * 0.05).bfloat16()
    return g, x, w


@pytest.mark.parametrize("M", [300, 768])
def test_pg_swiglu_with_row_scale(gpu, M):
    """gate_up + deferred-norm row scale + SwiGLU on the decode layout's tile-interleaved rows vs fp32."""
    from symmetry_amd.ops import reference

    N, K = 7168, 1024
    g, x, w = _inputs(gpu, M, N, K, M)
    ss = torch.rand(M, 32, device=gpu, generator=g) * 40
    cfg, _ = ops.choose_pgemm(M, N, K)
    act = torch.full((M, N // 2), float("nan"), device=gpu, dtype=torch.bfloat16)
    ops.pg_swiglu(x, preshuffle(w), ss, 1e-5, act, cfg)
    want = torch.empty(M, N // 2, device=gpu, dtype=torch.bfloat16)
    reference.dg_swiglu(x, w, ss, 1e-5, want)
    _close(act, want, atol=1.5e-2, rtol=2e-2)


@pytest.mark.parametrize("cfg", [5, 3, 4, 9])
def test_pg_resid_partials(gpu, cfg):
    """o / down + residual add + next-norm prep: resid, xw and one sum-of-squares partial per row and block column."""
    M, N, K = 700, 4096, 2048
    bn = ops.pgemm_shape(cfg)[1]
    g, x, w = _inputs(gpu, M, N, K, cfg)
    resid = torch.randn(M, N, device=gpu, generator=g)
    w_next = (torch.rand(N, device=gpu, generator=g) + 0.5).bfloat16()
    r0 = resid.clone()
    xw = torch.empty(M, N, device=gpu, dtype=torch.bfloat16)
    ss = torch.full((M, N // bn), float("nan"), device=gpu)
    ops.pg_resid(x, preshuffle(w), resid, w_next, xw, ss, cfg)
    want_r = r0 + x.float() @ w.float().t()
    _close(resid, want_r, atol=2e-3, rtol=1e-4)
    _close(xw, want_r * w_next.float(), atol=3e-2, rtol=8e-3)
    _close(ss, want_r.pow(2).view(M, N // bn, bn).sum(-1), atol=1e-1, rtol=1e-4)


@pytest.mark.parametrize("M", [300, 768])
@pytest.mark.parametrize("consecutive", [False, True])
def test_pg_qkv_rope_cache(gpu, M, consecutive):
    """QKV + row scale + RoPE + paged K/V write vs the reference op (decode row layout of wqkv)."""
    from symmetry_amd.models.layout import qkv_perm
    from symmetry_amd.ops import reference

    Hq, Hkv, D, K, BS = 8, 2, 128, 1024, 64
    N = (Hq + 2 * Hkv) * D
    g, x, w = _inputs(gpu, M, N, K, M + 1)
    w = w[qkv_perm(Hq, Hkv, D).to(gpu)].contiguous()
    ss = torch.rand(M, 4, device=gpu, generator=g) * 300
    pos = torch.arange(M, device=gpu, dtype=torch.int32) + 5
    if consecutive:  # a prefill sequence's tokens: 8-token runs of V go out as one 16-B store
        slots = torch.arange(M, device=gpu, dtype=torch.int32) + 3 * BS
    else:
        slots = torch.randperm(M + 64, device=gpu)[:M].int()
    slots[7] = -1  # a row without a cache slot
    cs = reference.rope_table(2048, D, 500000.0, device=gpu)
    nb = (M + 64) // BS + 4
    kc = torch.zeros(nb, Hkv, BS, D, device=gpu, dtype=torch.bfloat16)
    vc = torch.zeros(nb, Hkv, D, BS, device=gpu, dtype=torch.bfloat16)
    q = torch.zeros(M, Hq, D, device=gpu, dtype=torch.bfloat16)
    kr, vr, qr = kc.clone(), vc.clone(), q.clone()
    cfg, _ = ops.choose_pgemm(M, N, K, align=D)
    ops.pg_qkv(x, preshuffle(w), ss, 1e-5, pos, slots, cs, q, kc, vc, Hq, Hkv, cfg)
    reference.dg_qkv(x, w, ss, 1e-5, pos, slots, cs, qr, kr, vr, Hq, Hkv)
    _close(q, qr, atol=2e-2, rtol=2e-2)
    _close(kc, kr, atol=2e-2, rtol=2e-2)
    _close(vc, vr, atol=2e-2, rtol=2e-2)


def test_engine_long_prefill_on_pgemm_matches_oracle(gpu, monkeypatch):
    """small-llama (head dim 128, real tile shapes) with a 500-token and a 200-token prompt in one prefill step whose
    gate_up + SwiGLU runs on the prefill GEMM, decode under hipGraphs: every token within bf16 noise of the fp32
    oracle."""
    from symmetry_amd.engine.llm_engine import EngineConfig, LLMEngine
    from symmetry_amd.engine.sequence import SamplingParams
    from symmetry_amd.models import reference_model as rm

    calls = []
    real = ops.pg_swiglu
    monkeypatch.setattr(ops, "pg_swiglu", lambda *a: calls.append(a[0].shape[0]) or real(*a))
    eng = LLMEngine(EngineConfig(model="small-llama", device="cuda:0", max_num_seqs=4, max_model_len=2048,
                                 num_kv_blocks=128, use_graphs=True))
    prompts = [[5 + (13 * i) % 30000 for i in range(500)], [9 + (7 * i) % 30000 for i in range(200)]]
    seqs = [eng.add_request(f"p{i}", p, SamplingParams(max_tokens=8, ignore_eos=True)) for i, p in enumerate(prompts)]
    while eng.has_unfinished():
        eng.step()
    assert calls and calls[0] == 700, calls
    w = eng.weights.to("cpu")
    for p, s in zip(prompts, seqs):
        lg = rm.forward_logits(w, p + s.output_ids[:-1])
        r = rm.check_tokens(lg, len(p), s.output_ids)
        assert r["mismatches"] == 0, r


@pytest.mark.parametrize("cfg", list(ops.PG_GRP_CFGS))
@pytest.mark.parametrize("case", ["skewed", "sparse_ep"])
def test_pg_grouped_vs_fp32(gpu, cfg, case):
    """Grouped experts (MoE prefill): uneven segments (one longer than two tiles, one empty, one of a single row),
    experts [e_lo, e_lo + E) of a global numbering (expert parallelism: rows of other ranks' experts untouched);
    split SwiGLU of [gate; up] halves, bf16, fp32 and fp32 k-split slabs against the fp32 product."""
    bm, bn = ops.pgemm_shape(cfg)
    E, K = 4, 512
    if case == "skewed":
        counts, e_lo, pre = [2 * bm + 37, 1, 0, bm - 5], 0, 0
    else:  # two foreign experts' rows in front of and behind the local ones
        counts, e_lo, pre = [70, 3, bm + 9, 0, 130, 19], 1, 70
        E = 4
    offs = [0]
    for c in counts:
        offs.append(offs[-1] + c)
    R = offs[-1]
    offsets = torch.tensor(offs, dtype=torch.int32, device=gpu)
    g = torch.Generator(device=gpu).manual_seed(cfg * 7 + len(case))
    xs = (torch.rand(R, K, device=gpu, generator=g) * 2 - 1).bfloat16()
    N = 2 * bn
    W = ((torch.rand(E, N, K, device=gpu, generator=g) * 2 - 1) * 0.05).bfloat16()
    Wp = torch.stack([preshuffle(W[e]) for e in range(E)])
    ref = torch.full((R, N), float("nan"), device=gpu)
    for e in range(E):
        a, b = offs[e_lo + e], offs[e_lo + e + 1]
        ref[a:b] = xs[a:b].float() @ W[e].float().t()
    own = ~torch.isnan(ref[:, 0])
    assert own.sum() == offs[e_lo + E] - offs[e_lo] and (pre == 0 or not own[:pre].any())
    sentinel = -7.0
    y = torch.full((R, N), sentinel, device=gpu)
    ops.pg_grouped(xs, Wp, offsets, e_lo, y, ops.PG_EPI_F32, cfg)
    _close(y[own], ref[own], atol=1e-3 * math.sqrt(K) * 0.05 + 1e-4, rtol=1e-3)
    assert (y[~own] == sentinel).all(), "rows of foreign experts written"
    yb = torch.full((R, N), sentinel, device=gpu, dtype=torch.bfloat16)
    ops.pg_grouped(xs, Wp, offsets, e_lo, yb, ops.PG_EPI_BF16, cfg)
    _close(yb[own], ref[own], atol=2e-2, rtol=8e-3)
    ys = torch.full((2, R, N), sentinel, device=gpu)
    ops.pg_grouped(xs, Wp, offsets, e_lo, ys, ops.PG_EPI_F32, cfg, 2)
    _close(ys.sum(0)[own], ref[own], atol=1e-3 * math.sqrt(K) * 0.05 + 1e-4, rtol=1e-3)
    if (bn // 32) % 2 == 0:
        F = N // 2
        act = torch.full((R, F), sentinel, device=gpu, dtype=torch.bfloat16)
        ops.pg_grouped(xs, Wp, offsets, e_lo, act, ops.PG_EPI_SWIGLU_SPLIT, cfg)
        want = torch.nn.functional.silu(ref[:, :F]) * ref[:, F:]
        _close(act[own], want[own], atol=1.5e-2, rtol=2e-2)
        assert (act[~own] == sentinel).all()
