"""Medium-M projection path (ops.mgemm / ops.choose_mgemm) on the CPU: the tile chooser only returns
configurations the kernel accepts, the CPU op matches the split-K slab contract, and the general forward
gives the same logits with its projections routed through mgemm slabs."""
import pytest
import torch

from symmetry_amd import ops
from symmetry_amd.models.layout import preshuffle
from symmetry_amd.ops import reference


@pytest.mark.parametrize("M", [65, 80, 128, 129, 192, 256])
@pytest.mark.parametrize("N,K", [(6144, 4096), (4096, 4096), (4096, 14336), (28672, 4096), (1536, 1024),
                                 (1024, 3584), (7168, 1024), (10240, 8192), (8192, 28672)])
def test_chooser_respects_kernel_contract(M, N, K):
    pick = ops.choose_mgemm(M, N, K)
    if pick is None:
        return
    rw, S = pick
    assert 1 <= rw <= 4 and (M <= 128 or rw <= 2)
    assert N % (64 * rw) == 0 and K % (64 * S) == 0
    assert 128 <= N // (64 * rw) * S <= 256


def test_chooser_keeps_wide_and_long_prefills_on_the_library():
    assert ops.choose_mgemm(128, 28672, 4096) is None  # gate_up: hipBLASLt streams it at ~5.5 TB/s
    assert ops.choose_mgemm(300, 4096, 4096) is None   # beyond the medium range
    assert ops.choose_mgemm(256, 4096, 4096) is None   # o at 256 rows: library measured faster
    assert ops.choose_mgemm(128, 4096, 14336) == (2, 8)


def test_cpu_op_matches_slab_contract():
    g = torch.Generator().manual_seed(3)
    x = torch.randn(100, 512, generator=g).bfloat16()
    w = (torch.randn(256, 512, generator=g) * 0.05).bfloat16()
    y = torch.empty(4, 100, 256)
    ops.mgemm(x, preshuffle(w), y, 1)
    ref = torch.empty_like(y)
    reference.skinny_gemm(x, w, ref)
    assert torch.allclose(y, ref)


def test_general_forward_through_mgemm_slabs(monkeypatch):
    """An 80-token prefill on the general path with the projections routed through mgemm slabs (CPU op on
    preshuffled copies) generates the fp32 oracle's greedy tokens."""
    from symmetry_amd.engine.llm_engine import EngineConfig, LLMEngine
    from symmetry_amd.engine.sequence import SamplingParams
    from symmetry_amd.models import reference_model as rm

    calls = []
    real = ops.mgemm
    monkeypatch.setattr(ops, "choose_mgemm", lambda M, N, K, cus=256: (1, 2) if N % 64 == 0 and M > 64 else None)
    monkeypatch.setattr(ops, "mgemm", lambda *a: calls.append(a[0].shape[0]) or real(*a))
    eng = LLMEngine(EngineConfig(model="tiny-llama", device="cpu", max_num_seqs=2, max_model_len=256,
                                 num_kv_blocks=32, block_size=16, use_graphs=False, seed=0))
    m = eng.model
    m.fused = False
    m.dgw = {(i, n): preshuffle(m.w.layer(i, n)) for i in range(m.cfg.num_layers)
             for n in ("wqkv", "wo", "w_gu", "w_down")}
    prompt = [3 + (7 * i) % 400 for i in range(80)]
    out = eng.generate(prompt, SamplingParams(max_tokens=5, temperature=0.0))
    assert calls and set(calls) == {80}
    lg = rm.forward_logits(eng.weights.to("cpu"), prompt + out[:-1])
    for j, t in enumerate(out):
        row = lg[len(prompt) - 1 + j]
        assert float(row.max() - row[t]) <= 0.05, (j, t, int(row.argmax()))


def test_general_rows_decode_matches_fused(monkeypatch):
    """Decode steps routed to the general path (GENERAL_ROWS: mgemm projections, consumer kernels, the
    decode lm_head kernel on normalised rows) generate the oracle's greedy tokens, as the fused path does."""
    from symmetry_amd.engine.llm_engine import EngineConfig, LLMEngine
    from symmetry_amd.engine.sequence import SamplingParams
    from symmetry_amd.models import reference_model as rm
    from symmetry_amd.models import transformer

    outs = []
    for general in (0, 1):
        monkeypatch.setattr(transformer, "GENERAL_ROWS", general)
        eng = LLMEngine(EngineConfig(model="small-llama", device="cpu", max_num_seqs=3, max_model_len=128,
                                     num_kv_blocks=16, block_size=32, use_graphs=False, seed=0))
        m = eng.model
        assert m.fused
        m.dgw = {(i, n): preshuffle(m.w.layer(i, n)) for i in range(m.cfg.num_layers)
                 for n in ("wqkv", "wo", "w_gu", "w_down")}
        prompts = [[5 + 3 * k + i for k in range(9 + 4 * i)] for i in range(3)]
        seqs = [eng.add_request(f"r{i}", p, SamplingParams(max_tokens=4, temperature=0.0)) for i, p in enumerate(prompts)]
        while eng.has_unfinished():
            eng.step()
        outs.append([s.output_ids for s in seqs])
        # both paths agree with the fp32 oracle to within bf16 noise (random weights give near-ties, so
        # token-for-token equality between the two roundings is not expected)
        lw = eng.weights.to("cpu")
        for p, s in zip(prompts, seqs):
            lg = rm.forward_logits(lw, p + s.output_ids[:-1])
            for j, t in enumerate(s.output_ids):
                row = lg[len(p) - 1 + j]
                assert float(row.max() - row[t]) <= 0.08, (general, j, t, int(row.argmax()))
    assert [o[0] for o in outs[0]] == [o[0] for o in outs[1]]


def test_splitk_library_prefill_matches_oracle(monkeypatch):
    """A 300-token prefill runs its narrow projections as k-split batched library GEMMs into fp32 slabs
    (ops.linear_splitk, summed by the consumers) and still generates the fp32 oracle's tokens."""
    from symmetry_amd.engine.llm_engine import EngineConfig, LLMEngine
    from symmetry_amd.engine.sequence import SamplingParams
    from symmetry_amd.models import reference_model as rm

    calls = []
    real = ops.linear_splitk
    monkeypatch.setattr(ops, "linear_splitk", lambda x, w, y: calls.append(tuple(y.shape)) or real(x, w, y))
    eng = LLMEngine(EngineConfig(model="tiny-llama", device="cpu", max_num_seqs=2, max_model_len=512,
                                 num_kv_blocks=32, block_size=16, use_graphs=False, seed=0))
    eng.model.fused = False
    prompt = [3 + (11 * i) % 450 for i in range(300)]
    out = eng.generate(prompt, SamplingParams(max_tokens=3, temperature=0.0))
    assert calls and all(c[0] == 2 and c[1] == 300 for c in calls), calls
    lg = rm.forward_logits(eng.weights.to("cpu"), prompt + out[:-1])
    for j, t in enumerate(out):
        row = lg[len(prompt) - 1 + j]
        assert float(row.max() - row[t]) <= 0.05, (j, t, int(row.argmax()))


def test_wide_decode_batches_sample_from_logits(monkeypatch):
    """Decode steps with more than 64 sequences (the GPU scheduler admits up to MAX_DECODE_ROWS for dense
    models) sample from one fp32 logits GEMM + logits_argmax and still follow the fp32 oracle; temperature
    rows draw the same token as the fused sampler's key on the same logits."""
    from symmetry_amd.engine.llm_engine import EngineConfig, LLMEngine
    from symmetry_amd.engine.model_runner import MAX_DECODE_ROWS
    from symmetry_amd.engine.sequence import SamplingParams
    from symmetry_amd.models import reference_model as rm

    rows = []
    real = ops.logits_argmax
    monkeypatch.setattr(ops, "logits_argmax", lambda lg, *a, **k: rows.append(lg.shape[0]) or real(lg, *a, **k))
    n = 70
    eng = LLMEngine(EngineConfig(model="tiny-llama", device="cpu", max_num_seqs=n, max_model_len=64,
                                 num_kv_blocks=2 * n + 8, block_size=16, use_graphs=False, seed=0))
    assert eng.scheduler.cfg.max_num_seqs == n <= MAX_DECODE_ROWS
    prompts = [[3 + (5 * i + 7 * k) % 400 for k in range(4 + i % 3)] for i in range(n)]
    seqs = [eng.add_request(f"w{i}", p, SamplingParams(max_tokens=3, temperature=0.0)) for i, p in enumerate(prompts)]
    while eng.has_unfinished():
        eng.step()
    assert rows and min(rows) == n  # the prefill and every decode step sampled all rows at once
    lw = eng.weights.to("cpu")
    for i in (0, 33, 69):
        p, s = prompts[i], seqs[i]
        lg = rm.forward_logits(lw, p + s.output_ids[:-1])
        for j, t in enumerate(s.output_ids):
            row = lg[len(p) - 1 + j]
            assert float(row.max() - row[t]) <= 0.05, (i, j, t, int(row.argmax()))
    # sampled rows: logits_argmax's key == the fused lm_head sampler's key on the same logits
    g = torch.Generator().manual_seed(5)
    x = torch.randn(3, 64, generator=g).bfloat16()
    w = (torch.randn(96, 64, generator=g) * 0.2).bfloat16()
    temps = torch.tensor([0.0, 0.9, 1.3])
    seeds = torch.tensor([11, -4, 77], dtype=torch.int64)
    step = torch.tensor([5], dtype=torch.int64)
    k1, i1 = torch.empty(3, dtype=torch.int64), torch.empty(3, dtype=torch.int32)
    k2, i2 = torch.empty(3, dtype=torch.int64), torch.empty(3, dtype=torch.int32)
    lg = torch.empty(3, 96)
    ops.lm_head_sample(x, w, temps, seeds, step, torch.empty(3 * 6, dtype=torch.int64), k1, i1, 32, lg)
    ops.logits_argmax(lg, temps, seeds, step, k2, i2, 32)
    assert torch.equal(k1, k2) and torch.equal(i1, i2)


def test_pgemm_planner_respects_kernel_contract():
    for M in (257, 384, 640, 768, 1290, 4096):
        for N, K in ((6144, 4096), (4096, 4096), (28672, 4096), (4096, 14336), (7168, 1024), (1536, 1024)):
            for slabs in (False, True):
                pick = ops.choose_pgemm(M, N, K, slabs=slabs)
                assert pick is not None
                cfg, S = pick
                bm, bn = ops.PG_CFG_SHAPES[cfg]
                assert N % bn == 0 and K % (64 * S) == 0 and (slabs or S == 1)
    assert ops.choose_pgemm(256, 4096, 4096) is None  # medium-M rows stay on mgemm


def test_long_prefill_gate_up_on_pgemm(monkeypatch):
    """A 300-token prefill with gate_up + SwiGLU on the prefill GEMM (CPU reference op on the preshuffled copy of the
    decode row layout) generates the fp32 oracle's greedy tokens."""
    from symmetry_amd.engine.llm_engine import EngineConfig, LLMEngine
    from symmetry_amd.engine.sequence import SamplingParams
    from symmetry_amd.models import reference_model as rm

    eng = LLMEngine(EngineConfig(model="small-llama", device="cpu", max_num_seqs=2, max_model_len=512,
                                 num_kv_blocks=64, block_size=16, use_graphs=False, seed=0))
    m = eng.model
    m.dgw = {(i, n): preshuffle(m.w.layer(i, n)) for i in range(m.cfg.num_layers)
             for n in ("wqkv", "wo", "w_gu", "w_down")}
    calls = []
    real = ops.pg_swiglu
    monkeypatch.setattr(m, "fused", False)
    monkeypatch.setattr(m, "_pg_gate_up", lambda T: ops.choose_pgemm(T, m.dgw[(0, "w_gu")].shape[0],
                                                                     m.cfg.hidden_size)[0] if T >= 257 else None)
    monkeypatch.setattr(ops, "pg_swiglu", lambda *a: calls.append(a[0].shape[0]) or real(*a))
    prompt = [3 + (7 * i) % 30000 for i in range(300)]
    out = eng.generate(prompt, SamplingParams(max_tokens=4, temperature=0.0))
    assert calls and set(calls) == {300}
    lg = rm.forward_logits(eng.weights.to("cpu"), prompt + out[:-1])
    for j, t in enumerate(out):
        row = lg[len(prompt) - 1 + j]
        assert float(row.max() - row[t]) <= 0.05, (j, t, int(row.argmax()))


def test_grouped_pgemm_planner_and_reference():
    """The grouped prefill GEMM's planner only returns instantiated configs that tile the shape (even tile pairs for
    the split SwiGLU), and its CPU reference agrees with the grouped GEMM reference on [gate; up] experts."""
    for R in (300, 1024, 4096):
        c13 = ops.choose_pg_grouped(R, 2 * 14336, 4096, 8, even_wn=True)
        c2 = ops.choose_pg_grouped(R, 4096, 14336, 8, slabs=True)
        for (cfg, S), (N, K) in ((c13, (2 * 14336, 4096)), (c2, (4096, 14336))):
            bm, bn = ops.PG_CFG_SHAPES[cfg]
            assert cfg in ops.PG_GRP_CFGS and N % bn == 0 and K % (64 * S) == 0
        assert (ops.PG_CFG_SHAPES[c13[0]][1] // 32) % 2 == 0 and c13[1] == 1
    g = torch.Generator().manual_seed(0)
    E, N, K = 3, 64, 64
    W = torch.randn(E, N, K, generator=g).bfloat16()
    xs = torch.randn(10, K, generator=g).bfloat16()
    offsets = torch.tensor([0, 2, 2, 7, 10], dtype=torch.int32)  # expert 0 foreign (e_lo = 1)
    Wp = torch.stack([preshuffle(W[e]) for e in range(E)])
    want = torch.zeros(10, N // 2)
    reference.grouped_gemm(xs, W, offsets, 1, want, ops.GROUPED_SWIGLU)
    got = torch.zeros(10, N // 2)
    ops.pg_grouped(xs, Wp, offsets, 1, got, ops.PG_EPI_SWIGLU_SPLIT, 5)
    assert torch.allclose(got, want, atol=1e-5)
    slabs = torch.full((2, 10, N), 5.0)
    ops.pg_grouped(xs, Wp, offsets, 1, slabs, ops.PG_EPI_F32, 5, 2)
    ref = torch.zeros(10, N)
    reference.grouped_gemm(xs, W, offsets, 1, ref, ops.GROUPED_F32)
    assert torch.allclose(slabs.sum(0)[2:], ref[2:], atol=1e-4) and (slabs[:, :2] == 5.0).all()
