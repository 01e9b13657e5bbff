"""Engine + MoE + RCCL on the MI355X: native kernels against the fp32 oracle."""
import math
import os

import pytest
import torch

from symmetry_amd import ops
from symmetry_amd.ops import reference as ref

pytestmark = pytest.mark.gpu


def _agree(weights, prompt, out, tol, router_tie=0.005):
    """Every generated token within ``tol`` of the fp32 oracle's best logit.  MoE: the check stops at the
    first position whose oracle routing has a near-tie (k-th vs (k+1)-th expert margin < ``router_tie`` in
    some layer, at or before it): bf16 activations may pick the other expert there, and the sequences
    legitimately diverge from that point on."""
    from symmetry_amd.models import reference_model as rm

    cpu = weights.to("cpu")
    gaps = []
    lg = rm.forward_logits(cpu, prompt + out[:-1], router_gaps=gaps)
    tie = None
    if gaps:
        g = torch.stack(gaps).min(0).values  # [positions]
        hit = (g < router_tie).nonzero()
        tie = int(hit[0]) if hit.numel() else None
    for j, t in enumerate(out):
        pos = len(prompt) - 1 + j
        if tie is not None and pos >= tie:
            break
        row = lg[pos]
        assert float(row.max() - row[t]) <= tol, (j, t, int(row.argmax()), float(row.max() - row[t]))


@pytest.mark.parametrize("model", ["tiny-llama", "small-llama", "tiny-mixtral"])
def test_engine_gpu_matches_oracle(gpu, model):
    from symmetry_amd.engine.llm_engine import EngineConfig, LLMEngine
    from symmetry_amd.engine.sequence import SamplingParams

    eng = LLMEngine(EngineConfig(model=model, device="cuda:0", max_num_seqs=8, max_model_len=1024,
                                 num_kv_blocks=64, use_graphs=True))
    prompts = [eng.tokenizer.apply_chat_template([{"role": "user", "content": f"question {i} " * (i + 1)}])
               for i in range(5)]
    seqs = [eng.add_request(f"g{i}", p, SamplingParams(max_tokens=12, ignore_eos=True)) for i, p in enumerate(prompts)]
    while eng.has_unfinished():
        eng.step()
    for p, s in zip(prompts, seqs):
        assert len(s.output_ids) == 12
        _agree(eng.weights, p, s.output_ids, tol=0.08)


@pytest.mark.parametrize("graphs", [False, True])
def test_splitk_resid_path_native(gpu, monkeypatch, graphs):
    """The k-split O/down chain on the GPU (skinny_gemm into fp32 slabs -> add_prep with P = 4 column
    partials -> dg_swiglu / dg_qkv / dg_argmax reading the 4-column ss) against the fp32 oracle; the
    threshold is lowered so a small batch takes the path the engine uses from SPLITK_RESID_ROWS rows."""
    from symmetry_amd.engine.llm_engine import EngineConfig, LLMEngine
    from symmetry_amd.engine.sequence import SamplingParams
    from symmetry_amd.models import transformer

    calls = []
    orig = ops.add_prep  # dense model, no TP: add_prep only runs on the split path
    monkeypatch.setattr(ops, "add_prep", lambda *a, **k: calls.append(1) or orig(*a, **k))
    monkeypatch.setattr(transformer, "SPLITK_RESID_ROWS", 2)
    eng = LLMEngine(EngineConfig(model="small-llama", device="cuda:0", max_num_seqs=6, max_model_len=1024,
                                 num_kv_blocks=64, use_graphs=graphs))
    prompts = [list(range(300 + 11 * i, 330 + 13 * i)) for i in range(5)]
    seqs = [eng.add_request(f"k{i}", p, SamplingParams(max_tokens=10, ignore_eos=True))
            for i, p in enumerate(prompts)]
    while eng.has_unfinished():
        eng.step()
    assert calls
    for p, s in zip(prompts, seqs):
        assert len(s.output_ids) == 10
        _agree(eng.weights, p, s.output_ids, tol=0.08)


@pytest.mark.parametrize("graphs", [False, True])
@pytest.mark.parametrize("mg_fused", ["0", "all", "gu"])
def test_general_rows_decode_native(gpu, monkeypatch, graphs, mg_fused):
    """Decode steps on the general path, as wide batches run it, against the fp32 oracle; the threshold is
    lowered so a small batch takes it.  "0": mgemm projections -> rope_cache / add_rms_norm / swiglu summing
    the slabs -> decode lm_head on normalised rows.  "all": each projection one mgemm launch with the decode
    epilogue fused after an in-launch split-K reduction.  "gu": only gate_up fused (SwiGLU epilogue, deferred
    norm from add_prep)."""
    from symmetry_amd.engine.llm_engine import EngineConfig, LLMEngine
    from symmetry_amd.engine.sequence import SamplingParams
    from symmetry_amd.models import transformer

    calls = []
    if mg_fused != "0":
        name = "dg_qkv" if mg_fused == "all" else "dg_swiglu"
        orig = getattr(ops, name)
        monkeypatch.setattr(ops, name, lambda *a, **k: (calls.append(a[0].shape[0]) if k.get("mg") else None)
                            or orig(*a, **k))
    else:
        orig = ops.mgemm
        monkeypatch.setattr(ops, "mgemm", lambda *a, **k: calls.append(a[0].shape[0]) or orig(*a, **k))
    monkeypatch.setattr(transformer, "GENERAL_ROWS", 1)
    monkeypatch.setattr(transformer, "MG_FUSED", mg_fused == "all")
    monkeypatch.setattr(transformer, "MG_FUSED_GU", mg_fused == "gu")
    eng = LLMEngine(EngineConfig(model="small-llama", device="cuda:0", max_num_seqs=6, max_model_len=1024,
                                 num_kv_blocks=64, use_graphs=graphs))
    prompts = [list(range(700 + 9 * i, 720 + 11 * i)) for i in range(5)]
    seqs = [eng.add_request(f"gr{i}", p, SamplingParams(max_tokens=8, ignore_eos=True))
            for i, p in enumerate(prompts)]
    while eng.has_unfinished():
        eng.step()
    assert calls and min(calls) <= 8  # decode steps went through mgemm
    for p, s in zip(prompts, seqs):
        assert len(s.output_ids) == 8
        _agree(eng.weights, p, s.output_ids, tol=0.08)


@pytest.mark.parametrize("graphs", [False, True])
def test_wide_decode_batches_native(gpu, monkeypatch, graphs):
    """More than 64 concurrent sequences: decode steps of 65..256 rows run the general path (mgemm
    projections, one graph per bucket) and sample from one fp32 logits GEMM + logits_argmax; spot-check
    sequences against the fp32 oracle."""
    from symmetry_amd.engine.llm_engine import EngineConfig, LLMEngine
    from symmetry_amd.engine.sequence import SamplingParams

    rows = []
    orig = ops.logits_argmax
    monkeypatch.setattr(ops, "logits_argmax", lambda lg, *a, **k: rows.append(lg.shape[0]) or orig(lg, *a, **k))
    n = 90
    eng = LLMEngine(EngineConfig(model="small-llama", device="cuda:0", max_num_seqs=n, max_model_len=256,
                                 num_kv_blocks=4 * n, use_graphs=graphs))
    assert eng.scheduler.cfg.max_num_seqs == n
    prompts = [list(range(300 + 7 * i, 300 + 7 * i + 10 + i % 5)) for i in range(n)]
    seqs = [eng.add_request(f"w{i}", p, SamplingParams(max_tokens=6, ignore_eos=True)) for i, p in enumerate(prompts)]
    while eng.has_unfinished():
        eng.step()
    assert rows and max(rows) >= 90  # prefill of all 90 and the 96-row decode bucket sampled wide
    for i in (0, 41, 89):
        assert len(seqs[i].output_ids) == 6
        _agree(eng.weights, prompts[i], seqs[i].output_ids, tol=0.08)


@pytest.mark.parametrize("lens", [(40, 45), (70, 60, 50), (256,)])
def test_medium_m_prefill_native(gpu, monkeypatch, lens):
    """Prefill steps of 65..256 tokens run their projections on mgemm (split-K slabs summed by rope_cache /
    add_rms_norm / swiglu, or gate_up as one mgemm launch with the SwiGLU epilogue) and still generate the
    oracle's tokens."""
    from symmetry_amd.engine.llm_engine import EngineConfig, LLMEngine
    from symmetry_amd.engine.sequence import SamplingParams

    calls = []
    orig, orig_sw = ops.mgemm, ops.dg_swiglu
    monkeypatch.setattr(ops, "mgemm", lambda *a, **k: calls.append(a[0].shape[0]) or orig(*a, **k))
    monkeypatch.setattr(ops, "dg_swiglu", lambda *a, **k: (k.get("mg") is not None and calls.append(a[0].shape[0]))
                        or orig_sw(*a, **k))
    eng = LLMEngine(EngineConfig(model="small-llama", device="cuda:0", max_num_seqs=4, max_model_len=1024,
                                 num_kv_blocks=64, use_graphs=True))
    prompts = [list(range(400 + 17 * i, 400 + 17 * i + n)) for i, n in enumerate(lens)]
    seqs = [eng.add_request(f"m{i}", p, SamplingParams(max_tokens=6, ignore_eos=True)) for i, p in enumerate(prompts)]
    while eng.has_unfinished():
        eng.step()
    assert calls and all(64 < m <= 256 for m in calls), calls
    for p, s in zip(prompts, seqs):
        assert len(s.output_ids) == 6
        _agree(eng.weights, p, s.output_ids, tol=0.08)


@pytest.mark.parametrize("lens", [(300,), (200, 400)])
def test_splitk_library_prefill_native(gpu, monkeypatch, lens):
    """257..768-token prefills: narrow projections as k-split strided-batched hipBLASLt GEMMs with fp32
    slabs (ops.linear_splitk) summed by the consumer kernels, against the fp32 oracle."""
    from symmetry_amd.engine.llm_engine import EngineConfig, LLMEngine
    from symmetry_amd.engine.sequence import SamplingParams

    calls = []
    orig = ops.linear_splitk
    monkeypatch.setattr(ops, "linear_splitk", lambda x, w, y: calls.append(tuple(y.shape)) or orig(x, w, y))
    eng = LLMEngine(EngineConfig(model="small-llama", device="cuda:0", max_num_seqs=4, max_model_len=1024,
                                 num_kv_blocks=64, use_graphs=True))
    prompts = [list(range(900 + 13 * i, 900 + 13 * i + n)) for i, n in enumerate(lens)]
    seqs = [eng.add_request(f"s{i}", p, SamplingParams(max_tokens=5, ignore_eos=True)) for i, p in enumerate(prompts)]
    while eng.has_unfinished():
        eng.step()
    assert calls
    for p, s in zip(prompts, seqs):
        assert len(s.output_ids) == 5
        _agree(eng.weights, p, s.output_ids, tol=0.08)


def test_graph_replay_equals_eager(gpu):
    from symmetry_amd.engine.llm_engine import EngineConfig, LLMEngine
    from symmetry_amd.engine.sequence import SamplingParams

    outs = []
    for graphs in (True, False):
        eng = LLMEngine(EngineConfig(model="small-llama", device="cuda:0", max_num_seqs=6, max_model_len=1024,
                                     num_kv_blocks=64, use_graphs=graphs))
        ps = [list(range(300, 340 + 7 * i)) for i in range(6)]
        seqs = [eng.add_request(f"e{i}", p, SamplingParams(max_tokens=20, ignore_eos=True)) for i, p in enumerate(ps)]
        while eng.has_unfinished():
            eng.step()
        outs.append([s.output_ids for s in seqs])
    assert outs[0] == outs[1]


@pytest.mark.parametrize("T", [1, 16, 37, 512])
def test_moe_router_logits_vs_fp32(gpu, T):
    """The 16-row router kernel (prefill routing) against the fp32 product; rows past T untouched."""
    d = 4096
    g = torch.Generator(device=gpu).manual_seed(T)
    x = torch.randn(T, d, device=gpu, generator=g).bfloat16()
    Wr = (torch.randn(16, d, device=gpu, generator=g) * 0.02).bfloat16()
    logits = torch.full((T, 16), float("nan"), device=gpu)
    ops.moe_router(x, Wr, logits)
    torch.testing.assert_close(logits, x.float() @ Wr.float().t(), atol=2e-3, rtol=2e-3)


def test_moe_kernels_vs_reference(gpu):
    T, d, E, k, F = 11, 256, 8, 2, 512
    g = torch.Generator(device=gpu).manual_seed(0)
    x = torch.randn(T, d, device=gpu, generator=g).bfloat16()
    logits = torch.randn(2, T, 16, device=gpu, generator=g)  # split-K slabs, padded router width
    R = T * k
    ids = torch.empty(R, dtype=torch.int32, device=gpu)
    w = torch.empty(R, device=gpu)
    dst = torch.empty(R, dtype=torch.int32, device=gpu)
    counts = torch.empty(E, dtype=torch.int32, device=gpu)
    offsets = torch.empty(E + 1, dtype=torch.int32, device=gpu)
    cursor = torch.empty(E, dtype=torch.int32, device=gpu)
    xs = torch.empty(R, d, dtype=torch.bfloat16, device=gpu)
    ops.moe_route_permute(logits, x, k, E, ids, w, counts, offsets, cursor, xs, dst)
    r_ids, r_w, r_dst = ids.cpu().clone(), w.cpu().clone(), dst.cpu().clone()
    c_ids, c_w, c_dst = torch.empty(R, dtype=torch.int32), torch.empty(R), torch.empty(R, dtype=torch.int32)
    c_cnt, c_off, c_cur = torch.empty(E, dtype=torch.int32), torch.empty(E + 1, dtype=torch.int32), torch.empty(
        E, dtype=torch.int32)
    c_xs = torch.empty(R, d, dtype=torch.bfloat16)
    ref.moe_route_permute(logits.cpu(), x.cpu(), k, E, c_ids, c_w, c_cnt, c_off, c_cur, c_xs, c_dst)
    assert torch.equal(r_ids, c_ids)
    assert torch.allclose(r_w, c_w, atol=1e-5)
    assert torch.equal(offsets.cpu(), c_off)
    # each assignment's row holds its token and lies in its expert's segment
    off = c_off.long()
    for a in range(R):
        row, e = int(r_dst[a]), int(r_ids[a])
        assert off[e] <= row < off[e + 1]
        assert torch.equal(xs[row].cpu(), x[a // k].cpu())
    W = (torch.randn(E, 2 * F, d, device=gpu, generator=g) * 0.05).bfloat16()
    S = ops.choose_splits(2 * F, d)
    y = torch.empty(S, R, 2 * F, device=gpu)
    ops.grouped_skinny(xs, W, offsets, 0, y)
    ref_y = torch.zeros(R, 2 * F)
    for e in range(E):
        a, b = int(off[e]), int(off[e + 1])
        ref_y[a:b] = xs[a:b].float().cpu() @ W[e].float().cpu().t()
    assert torch.allclose(y.sum(0).cpu(), ref_y, atol=2e-2, rtol=1e-2)
    # the same product on the per-expert MFMA-preshuffled stacks (single-copy expert weights)
    from symmetry_amd.models.layout import preshuffle

    ys = torch.full_like(y, float("nan"))
    ops.grouped_skinny(xs, preshuffle(W), offsets, 0, ys, wshuf=True)
    assert torch.equal(ys.sum(0), y.sum(0)), "preshuffled skinny GEMM differs from the row-major one"
    out = torch.empty(T, 2 * F, device=gpu)
    ops.moe_combine(y, dst, ids, 0, E, w, k, out)
    c_out = torch.empty(T, 2 * F)
    ref.moe_combine(y.cpu(), dst.cpu(), ids.cpu(), 0, E, w.cpu(), k, c_out, False)
    assert torch.allclose(out.cpu(), c_out, atol=1e-3, rtol=1e-3)
    # expert-range masking (EP): only experts 2..5 contribute
    ops.moe_combine(y, dst, ids, 2, 6, w, k, out)
    ref.moe_combine(y.cpu(), dst.cpu(), ids.cpu(), 2, 6, w.cpu(), k, c_out, False)
    assert torch.allclose(out.cpu(), c_out, atol=1e-3, rtol=1e-3)


@pytest.mark.parametrize("T,d,E,k", [(4, 4096, 8, 2), (8, 512, 8, 2), (1, 256, 64, 8), (7, 1024, 16, 4),
                                     (3, 4000, 20, 2)])
def test_moe_decode_fused_vs_reference(gpu, T, d, E, k):
    """The one-launch decode routing (RMSNorm + router + top-k + segments + permuted rows) and the combine fused
    with the residual prep against their fp32 compositions (reference.rms_norm / router / moe_route_permute;
    moe_combine + add_prep)."""
    g = torch.Generator(device=gpu).manual_seed(T * 31 + E)
    resid = torch.randn(T, d, device=gpu, generator=g) * 3
    lnw = (torch.rand(d, device=gpu, generator=g) + 0.5).bfloat16()
    Wr = (torch.randn(E, d, device=gpu, generator=g) * 0.05).bfloat16()
    R = T * k
    ids = torch.empty(R, dtype=torch.int32, device=gpu)
    w = torch.empty(R, device=gpu)
    dst = torch.empty(R, dtype=torch.int32, device=gpu)
    counts = torch.empty(E, dtype=torch.int32, device=gpu)
    offsets = torch.empty(E + 1, dtype=torch.int32, device=gpu)
    cursor = torch.full((E,), 7, dtype=torch.int32, device=gpu)
    xs = torch.empty(R, d, dtype=torch.bfloat16, device=gpu)
    ops.moe_decode_route(resid, lnw, 1e-5, Wr, k, ids, w, counts, offsets, cursor, xs, dst)
    c_ids, c_w, c_dst = torch.empty(R, dtype=torch.int32), torch.empty(R), torch.empty(R, dtype=torch.int32)
    c_cnt, c_off = torch.empty(E, dtype=torch.int32), torch.empty(E + 1, dtype=torch.int32)
    c_cur, c_xs = torch.empty(E, dtype=torch.int32), torch.empty(R, d, dtype=torch.bfloat16)
    ref.moe_decode_route(resid.cpu(), lnw.cpu(), 1e-5, Wr.cpu(), k, c_ids, c_w, c_cnt, c_off, c_cur, c_xs, c_dst)
    assert torch.equal(ids.cpu(), c_ids)  # random logits: no near-ties at this scale
    assert torch.allclose(w.cpu(), c_w, atol=1e-5)
    assert torch.equal(offsets.cpu(), c_off) and torch.equal(counts.cpu(), c_cnt)
    assert torch.equal(dst.cpu(), c_dst)  # segment rows in token order, like the reference
    assert int(cursor.abs().sum()) == 0
    assert (xs.cpu().float() - c_xs.float()).abs().max() <= 0.02 * c_xs.float().abs().max()
    # combine + residual prep (every expert local)
    y = torch.randn(2, R, d, device=gpu, generator=g)
    w_next = (torch.rand(d, device=gpu, generator=g) + 0.5).bfloat16()
    xw = torch.empty(T, d, dtype=torch.bfloat16, device=gpu)
    P = d // 8 // 64 if (d // 8) % 64 == 0 else 1
    ss = torch.empty(T, P, device=gpu)
    r0 = resid.clone()
    ops.moe_combine_prep(y, dst, ids, E, w, k, resid, w_next, xw, ss)
    c_r, c_xw, c_ss = r0.cpu().clone(), torch.empty(T, d, dtype=torch.bfloat16), torch.empty(T, P)
    ref.moe_combine_prep(y.cpu(), dst.cpu(), ids.cpu(), E, w.cpu(), k, c_r, w_next.cpu(), c_xw, c_ss)
    assert torch.allclose(resid.cpu(), c_r, atol=1e-4, rtol=1e-5)
    assert torch.allclose(xw.cpu().float(), c_xw.float(), atol=2e-2, rtol=1e-2)
    assert torch.allclose(ss.cpu(), c_ss, rtol=1e-4)


def test_rccl_single_rank_allreduce_and_capture(gpu):
    import socket

    import torch.distributed as dist

    from symmetry_amd.parallel.comm import RcclComm

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    if not dist.is_initialized():
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    comm = RcclComm()
    t = torch.arange(8, device=gpu, dtype=torch.float32)
    comm.all_reduce(t)
    torch.cuda.synchronize()
    assert torch.equal(t.cpu(), torch.arange(8, dtype=torch.float32))
    # the collective is capturable inside a hipGraph together with kernels
    g = torch.cuda.CUDAGraph()
    buf = torch.ones(1024, device=gpu)
    comm.all_reduce(buf)
    torch.cuda.synchronize()
    with torch.cuda.graph(g):
        buf.mul_(2.0)
        comm.all_reduce(buf, op="max")
    g.replay()
    torch.cuda.synchronize()
    assert float(buf[0]) == 2.0
    comm.destroy()
    dist.destroy_process_group()


def test_top_k_one_in_graph_equals_greedy(gpu):
    """The filtered-sampling decode graph variant (full logits + sample_filtered kernel) with top_k=1
    reproduces greedy decoding; a seeded top-p request is reproducible."""
    from symmetry_amd.engine.llm_engine import EngineConfig, LLMEngine
    from symmetry_amd.engine.sequence import SamplingParams

    eng = LLMEngine(EngineConfig(model="small-llama", device="cuda:0", max_num_seqs=4, max_model_len=512,
                                 num_kv_blocks=32, use_graphs=True))
    prompt = list(range(200, 237))
    greedy = eng.generate(prompt, SamplingParams(max_tokens=10, temperature=0.0, ignore_eos=True))
    k1 = eng.generate(prompt, SamplingParams(max_tokens=10, temperature=1.0, top_k=1, ignore_eos=True))
    assert k1 == greedy
    a = eng.generate(prompt, SamplingParams(max_tokens=10, temperature=0.9, top_p=0.8, seed=3, ignore_eos=True))
    b = eng.generate(prompt, SamplingParams(max_tokens=10, temperature=0.9, top_p=0.8, seed=3, ignore_eos=True))
    assert a == b
    # the filtered graph variant was captured and used (decode keys: (rows, blocks, filtered))
    assert any(k[2] for k in eng.runner.graphs if not isinstance(k[0], str))


def test_staggered_arrivals_mixed_steps_and_pipelining_match_oracle(gpu):
    """GPU engine with graphs + pipelined decode: a long prompt arrives while others decode (mixed
    prefill/decode steps), a short one arrives later; every sequence agrees with the fp32 oracle."""
    from symmetry_amd.engine.llm_engine import EngineConfig, LLMEngine
    from symmetry_amd.engine.sequence import SamplingParams

    eng = LLMEngine(EngineConfig(model="small-llama", device="cuda:0", max_num_seqs=6, max_model_len=1024,
                                 num_kv_blocks=64, use_graphs=True, mixed_prefill_tokens=96))
    prompts = {0: list(range(100, 140)), 1: list(range(500, 530)), 2: list(range(1000, 1300)), 3: [7, 8, 9]}
    arrive = {0: 0, 1: 0, 2: 4, 3: 9}
    seqs, step = {}, 0
    while step < 500:
        for i, t in arrive.items():
            if t == step:
                seqs[i] = eng.add_request(f"s{i}", prompts[i], SamplingParams(max_tokens=14, ignore_eos=True))
        if len(seqs) == len(prompts) and not eng.has_unfinished():
            break
        eng.step()
        step += 1
    for i, s in seqs.items():
        assert len(s.output_ids) == 14
        _agree(eng.weights, prompts[i], s.output_ids, tol=0.08)


@pytest.mark.parametrize("model", ["small-llama", "tiny-mixtral"])
def test_prefix_cache_multi_turn_on_gpu_matches_oracle(gpu, model):
    """Multi-turn chat on the native path: turn 2 adopts turn 1's cached KV blocks (prompt + answer) and
    prefills only the tail through the chunked-prefill attention kernel; outputs match the fp32 oracle."""
    from symmetry_amd.engine.llm_engine import EngineConfig, LLMEngine
    from symmetry_amd.engine.sequence import SamplingParams

    eng = LLMEngine(EngineConfig(model=model, device="cuda:0", max_num_seqs=4, max_model_len=1024,
                                 num_kv_blocks=64, block_size=32, use_graphs=True))
    turn1 = eng.tokenizer.apply_chat_template([{"role": "user", "content": "tell me about the swarm " * 6}])
    out1 = eng.generate(turn1, SamplingParams(max_tokens=24, ignore_eos=True))
    turn2 = turn1 + out1 + eng.tokenizer.encode(" and now the provider")
    hits0 = eng.blocks.hit_tokens
    out2 = eng.generate(turn2, SamplingParams(max_tokens=12, ignore_eos=True))
    assert eng.blocks.hit_tokens - hits0 >= (len(turn1) // 32) * 32
    _agree(eng.weights, turn1, out1, tol=0.08)
    _agree(eng.weights, turn2, out2, tol=0.08)


@pytest.mark.parametrize("path", ["fused", "general"])
def test_llama3_8b_shapes_two_layers_match_oracle(gpu, monkeypatch, path):
    """The headline model's real shapes (d = 4096, F = 14336, Hq / Hkv = 32 / 8, V = 128256) with two
    layers, through prefill, the decode hipGraphs and either decode path (fused decode GEMMs, or the
    general mgemm + consumer path that wide batches take), against the fp32 oracle."""
    from symmetry_amd.engine.llm_engine import EngineConfig, LLMEngine
    from symmetry_amd.engine.sequence import SamplingParams
    from symmetry_amd.models import transformer
    from symmetry_amd.models.config import LLAMA3_8B

    if path == "general":
        monkeypatch.setattr(transformer, "GENERAL_ROWS", 1)
    mcfg = LLAMA3_8B.replace(num_layers=2)
    eng = LLMEngine(EngineConfig(model="llama3:8b", model_config=mcfg, device="cuda:0", max_num_seqs=8,
                                 max_model_len=1024, num_kv_blocks=64, use_graphs=True))
    eng.warmup([16, 128])
    prompts = [eng.tokenizer.apply_chat_template([{"role": "user", "content": f"shape check {i} " * (2 * i + 1)}])
               for i in range(6)]
    seqs = [eng.add_request(f"s{i}", p, SamplingParams(max_tokens=8, ignore_eos=True))
            for i, p in enumerate(prompts)]
    while eng.has_unfinished():
        eng.step()
    assert eng.runner.graphs, "decode steps must replay captured hipGraphs"
    for p, s in zip(prompts, seqs):
        assert len(s.output_ids) == 8
        _agree(eng.weights, p, s.output_ids, tol=0.1)


def test_prefill_graphs_match_oracle(gpu, monkeypatch):
    """Short prefills replay hipGraphs captured at start-up per padded (tokens, context) bucket: padding token
    rows write no cache slot, padding attention tiles exit.  One-sequence prefills of 3..256 tokens (bucket edges
    included), a prefix-cache tail and a bucket replayed a second time, plus a two-sequence step (eager: not
    captured), all agree with the fp32 oracle; with the buckets off nothing is captured or replayed."""
    from symmetry_amd.engine import model_runner
    from symmetry_amd.engine.llm_engine import EngineConfig, LLMEngine
    from symmetry_amd.engine.sequence import SamplingParams

    groups = [[list(range(300, 303))], [list(range(10, 26))], [list(range(40, 57))], [list(range(60, 160))],
              [list(range(500, 756))], [list(range(900, 940)), list(range(1200, 1271))],
              [list(range(60, 160)) + [5, 6, 7]], [list(range(2000, 2090))]]

    def run(tokens):
        monkeypatch.setattr(model_runner, "PREFILL_GRAPH_TOKENS", tokens)
        eng = LLMEngine(EngineConfig(model="small-llama", device="cuda:0", max_num_seqs=4, max_model_len=1024,
                                     num_kv_blocks=64, block_size=32, use_graphs=True))
        eng.warmup([16, 128])  # start-up capture: decode graphs + one-sequence prefill buckets
        outs = []
        for gi, group in enumerate(groups):
            seqs = [eng.add_request(f"g{gi}-{j}", p, SamplingParams(max_tokens=6, ignore_eos=True))
                    for j, p in enumerate(group)]
            while eng.has_unfinished():
                eng.step()
            outs.append([list(s.output_ids) for s in seqs])
        return eng, outs

    eng, got = run(256)
    keys = [k for k in eng.runner.graphs if isinstance(k[0], str)]
    assert {k[1] for k in keys} == set(model_runner.PREFILL_GRAPH_BUCKETS) and {k[2] for k in keys} == {1}, keys
    # every one-sequence group replayed a start-up graph (the two-sequence one ran eagerly: not captured)
    assert eng.runner.prefill_graph_replays >= 7, eng.runner.prefill_graph_replays
    for group, outs in zip(groups, got):
        for p, o in zip(group, outs):
            assert len(o) == 6
            _agree(eng.weights, p, o, tol=0.08)
    eager, _ = run(0)
    assert not any(isinstance(k[0], str) for k in eager.runner.graphs) and eager.runner.prefill_graph_replays == 0


@pytest.mark.parametrize("policy", [0, 2])
@pytest.mark.parametrize("mode", [0, 1, 2])
@pytest.mark.parametrize("counts", [(300, 0, 129, 1, 640, 77, 0, 200), (3, 2, 1, 0, 0, 0, 0, 300),
                                    (90, 60, 100, 70, 95, 85, 80, 96), (150, 170, 180, 120, 160, 175, 140, 190)])
def test_grouped_gemm_vs_fp32(gpu, mode, counts, policy):
    """Grouped MFMA GEMM (K12) over uneven expert segments (empty ones, a 1-row one, multi-tile ones) with
    the segment bounds read on the device: bf16 / fp32 outputs and the fused SwiGLU epilogue, against fp32
    products; rows outside every segment are never written.  policy 0: the 128 x 128 tile kernel; 2: the
    weight-streaming kernel (its 128 / 192 / 256-row unit variants by the mean segment, segments longer than
    a unit split over several, an expert-parallel slice)."""
    ops.grouped_stream_policy(policy)
    try:
        _grouped_case(gpu, mode, counts)
    finally:
        ops.grouped_stream_policy(1)


def _grouped_case(gpu, mode, counts):
    E, d, F = 8, 512, 384
    g = torch.Generator(device=gpu).manual_seed(sum(counts) + mode)
    R = sum(counts)
    off = torch.zeros(E + 1, dtype=torch.int32)
    off[1:] = torch.cumsum(torch.tensor(counts), 0)
    offsets = off.to(gpu)
    xs = torch.randn(R + 16, d, device=gpu, generator=g).bfloat16()
    N = F if mode == 2 else 2 * F
    W = (torch.randn(E, 2 * F, d, device=gpu, generator=g) * 0.05).bfloat16()
    e0, El = (2, 4) if mode == 1 else (0, E)  # mode 1: an expert-parallel shard (experts 2..5)
    Wl = W[e0:e0 + El].contiguous()
    dt = torch.float32 if mode == 1 else torch.bfloat16
    y = torch.full((R + 16, N), 7.0, device=gpu, dtype=dt)
    ops.grouped_gemm(xs, Wl, offsets, e0, y, mode)
    torch.cuda.synchronize()
    yc, xc, Wc = y.float().cpu(), xs.float().cpu(), Wl.float().cpu()
    written = torch.zeros(R + 16, dtype=torch.bool)
    for e in range(El):
        a, b = int(off[e0 + e]), int(off[e0 + e + 1])
        if b <= a:
            continue
        p = xc[a:b] @ Wc[e].t()
        if mode == 2:
            p = torch.nn.functional.silu(p[:, :F]) * p[:, F:]
        tol = 2e-2 if mode != 1 else 2e-3
        torch.testing.assert_close(yc[a:b], p, atol=tol, rtol=tol)
        written[a:b] = True
    assert torch.all(yc[~written] == 7.0)


@pytest.mark.parametrize("pre", [False, True])
@pytest.mark.parametrize("mode", [1, 2])
def test_grouped_stream_mixtral_shapes(gpu, mode, pre):
    """The weight-streaming grouped GEMM on Mixtral's expert shapes (K = 4096 for w13 with the SwiGLU
    epilogue, K = 14336 for w2 with fp32 rows) at ~128 routed rows per expert, against fp32 products; row-major
    and MFMA-preshuffled expert weights."""
    E = 8
    K, Nw = (4096, 2 * 512) if mode == 2 else (14336, 512)
    counts = (131, 118, 140, 97, 126, 150, 110, 152)
    g = torch.Generator(device=gpu).manual_seed(mode)
    R = sum(counts)
    off = torch.zeros(E + 1, dtype=torch.int32)
    off[1:] = torch.cumsum(torch.tensor(counts), 0)
    xs = torch.randn(R, K, device=gpu, generator=g).bfloat16()
    W = (torch.randn(E, Nw, K, device=gpu, generator=g) * 0.02).bfloat16()
    N = Nw // 2 if mode == 2 else Nw
    y = torch.zeros(R, N, device=gpu, dtype=torch.float32 if mode == 1 else torch.bfloat16)
    ops.grouped_stream_policy(2)
    try:
        if pre:
            from symmetry_amd.models.layout import preshuffle

            Wp = torch.stack([preshuffle(W[e]) for e in range(E)])
            ops.grouped_gemm(xs, Wp, off.to(gpu), 0, y, mode + 4)
        else:
            ops.grouped_gemm(xs, W, off.to(gpu), 0, y, mode)
        torch.cuda.synchronize()
    finally:
        ops.grouped_stream_policy(1)
    yc, xc, Wc = y.float().cpu(), xs.float().cpu(), W.float().cpu()
    for e in range(E):
        a, b = int(off[e]), int(off[e + 1])
        p = xc[a:b] @ Wc[e].t()
        if mode == 2:
            p = torch.nn.functional.silu(p[:, :N]) * p[:, N:]
        tol = 2e-2 if mode == 2 else 2e-3
        torch.testing.assert_close(yc[a:b], p, atol=tol, rtol=tol)


@pytest.mark.parametrize("pg", [True, False])
def test_mixtral_prefill_grouped_path_matches_oracle(gpu, pg):
    """tiny-mixtral prefill of more than 64 routed rows: the grouped expert GEMMs (no host sync) end to end against
    the fp32 oracle, with the decode steps in hipGraphs -- on the prefill GEMM kernel's grouped mode (pg) and on the
    tile / weight-streaming grouped kernels."""
    import symmetry_amd.models.moe as moe_mod
    from symmetry_amd.engine.llm_engine import EngineConfig, LLMEngine
    from symmetry_amd.engine.sequence import SamplingParams

    eng = LLMEngine(EngineConfig(model="tiny-mixtral", device="cuda:0", max_num_seqs=4, max_model_len=1024,
                                 num_kv_blocks=64, use_graphs=True))
    assert eng.model.moe.pre, "expected the preshuffled expert copies"
    prompts = [list(range(40 + 7 * i, 40 + 7 * i + 90 + 20 * i)) for i in range(3)]  # 90..130 tokens each
    calls = {"grouped_gemm": [], "pg_grouped": []}
    origs = {n: getattr(ops, n) for n in calls}
    saved = moe_mod.PG_GROUPED
    moe_mod.PG_GROUPED = pg
    for n, f in origs.items():
        setattr(moe_mod.ops, n, lambda *a, _n=n, _f=f, **k: calls[_n].append(a[0].shape[0]) or _f(*a, **k))
    try:
        seqs = [eng.add_request(f"m{i}", p, SamplingParams(max_tokens=6, ignore_eos=True))
                for i, p in enumerate(prompts)]
        while eng.has_unfinished():
            eng.step()
    finally:
        for n, f in origs.items():
            setattr(moe_mod.ops, n, f)
        moe_mod.PG_GROUPED = saved
    used = calls["pg_grouped" if pg else "grouped_gemm"]
    assert used and max(used) > 64, calls
    if pg:
        assert not calls["grouped_gemm"] or max(calls["grouped_gemm"]) <= 64
    for p, s in zip(prompts, seqs):
        assert len(s.output_ids) == 6
        _agree(eng.weights, p, s.output_ids, tol=0.08)

