"""Tensor / expert parallelism on CPU with the gloo backend, world_size 2-8 (SURVEY.md §4.2 'Distributed').

* TP=2 engine (rank 0 schedules, rank 1 mirrors through the metadata broadcast) generates the
  same tokens as TP=1 on the same weights;
* EP=2 MoE in both modes (all-reduce combine, all-to-all dispatch) equals the local MoE block;
* the Comm primitives (all_reduce / all_gather / all_to_all_rows) are exact.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _init(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(0)


def _run(fn, world=2):
    port = _port()
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    procs = [ctx.Process(target=_entry, args=(fn, r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = [q.get() for _ in range(world)]
    for p in procs:
        p.join(60)
    errs = [r for r in results if isinstance(r, str)]
    assert not errs, errs[0]
    return sorted(results, key=lambda r: r[0])


def _entry(fn, rank, world, port, q):
    import traceback

    try:
        _init(rank, world, port)
        q.put((rank, fn(rank, world)))
    except Exception:
        q.put(traceback.format_exc())
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


# ----------------------------------------------------------------------------------------------
def _comm_worker(rank, world):
    from symmetry_amd.parallel.comm import TorchComm

    c = TorchComm()
    t = torch.full((4,), float(rank + 1))
    c.all_reduce(t)
    m = torch.tensor([rank * 10], dtype=torch.int64)
    c.all_reduce(m, op="max")
    g = c.all_gather(torch.tensor([[rank, rank]]))
    send = torch.arange(6, dtype=torch.float32).view(3, 2) + 100 * rank
    sc = [1, 2] if rank == 0 else [2, 1]
    rc = [1, 2] if rank == 0 else [2, 1]
    r = c.all_to_all_rows(send, sc, rc)
    # the host-staged communicator (GPU ranks sharing one device) must agree with the plain one
    from symmetry_amd.parallel.comm import HostStagedComm

    hs = HostStagedComm()
    t2 = torch.full((4,), float(rank + 1))
    hs.all_reduce(t2)
    assert torch.equal(t2, t)
    assert torch.equal(hs.all_gather(torch.tensor([[rank, rank]])), g)
    assert torch.equal(hs.all_to_all_rows(send, sc, rc), r)
    b = torch.tensor([rank + 5])
    hs.broadcast(b, src=1)
    assert int(b) == 6
    # all_reduce_add_prep (the row-parallel decode epilogue; fused on XgmiComm) == all_reduce + add_prep
    from symmetry_amd.ops import reference

    y = torch.randn(3, 64) + rank
    resid = torch.randn(3, 64, generator=torch.Generator().manual_seed(5))
    w = torch.rand(64, generator=torch.Generator().manual_seed(6)).to(torch.bfloat16)
    xw, ss = torch.empty(3, 64, dtype=torch.bfloat16), torch.empty(3, 2)
    ysum = y.clone()
    c.all_reduce(ysum)
    r_ref, xw_ref, ss_ref = resid.clone(), torch.empty_like(xw), torch.empty_like(ss)
    reference.add_prep(ysum, r_ref, w, xw_ref, ss_ref)
    c.all_reduce_add_prep(y, resid, w, xw, ss)
    assert torch.equal(resid, r_ref) and torch.equal(xw, xw_ref) and torch.equal(ss, ss_ref)
    # vocab-parallel argmax combine of packed u64 keys (value bits high, inverted index low); values with
    # the top bit set exercise the unsigned order
    vals = [[0x80000001, 5], [0x7FFFFFFF, 9]][rank]
    idx = [[3, 100], [1000, 2]][rank]
    keys = torch.tensor([(v << 32) | (0xFFFFFFFF - i) for v, i in zip(vals, idx)], dtype=torch.uint64).view(torch.int64)
    ids = torch.zeros(2, dtype=torch.int32)
    c.argmax_keys(keys, ids)
    assert ids.tolist() == [3, 2], ids
    return t.tolist(), int(m), g.tolist(), r.tolist()


def test_comm_primitives():
    (_, a), (_, b) = _run(_comm_worker)
    assert a[0] == [3.0] * 4 and a[1] == 10
    assert a[2] == [[0, 0], [1, 1]]
    # rank 0 sends row0 -> r0, rows1-2 -> r1; rank 1 sends rows 0-1 -> r0, row2 -> r1
    assert a[3] == [[0.0, 1.0], [100.0, 101.0], [102.0, 103.0]]
    assert b[3] == [[2.0, 3.0], [4.0, 5.0], [104.0, 105.0]]


def _xar_vote_worker(rank, world):
    """The fused-path startup check drops the fused launches on EVERY rank when one rank's attach or self-test
    fails (a rank-local fallback would leave the others waiting in a collective that never comes)."""
    from symmetry_amd.parallel import launch

    class FakeSub:
        destroyed = False

        def destroy(self, inner_too=True):
            FakeSub.destroyed = True

    class FakeComm:
        xar = None
        a2a = None

        def __init__(self, fail_attach=False, fail_test=False):
            self.fail_attach, self.fail_test = fail_attach, fail_test

        def attach_xar(self, group, rows, d):
            if self.fail_attach:
                raise RuntimeError("ipc mapping refused")
            self.xar = FakeSub()

        def xar_self_test(self, d, ks=(256,), rows=(4,), layouts=(False,)):
            return not self.fail_test

        def attach_a2a(self, group, cap, row_bytes):
            if self.fail_attach:
                raise RuntimeError("uncached allocation failed")
            self.a2a = FakeSub()

    group = dist.new_group(backend="gloo")
    out = []
    for fail in ((False, False), (rank == 1, False), (False, rank == 0)):
        c = FakeComm(*fail)
        launch._attach_xar_checked(c, group, 64)
        out.append(c.xar is not None)
    # the expert all-to-all communicator: attached on every rank or on none
    cfg = type("M", (), {"top_k": 2, "num_experts": 8, "hidden_size": 64})()
    for fail in (False, rank == 1):
        c = FakeComm(fail)
        launch._attach_a2a_checked(c, group, 4096, cfg, world)
        out.append(c.a2a is not None)
    return out


def test_a2a_capacity():
    from symmetry_amd.parallel.launch import a2a_capacity

    # one pre-combined row per token of the owner's slice
    assert a2a_capacity(8192, 8) == 1024
    assert a2a_capacity(1000, 3) == 334


def test_fused_path_startup_check_is_all_ranks_or_none():
    res = _run(_xar_vote_worker, world=2)
    assert [r[1] for r in res] == [[True, False, False, True, False], [True, False, False, True, False]]


def _tp_worker(rank, world, model="tiny-llama"):
    from symmetry_amd.engine.llm_engine import EngineConfig
    from symmetry_amd.engine.sequence import SamplingParams
    from symmetry_amd.parallel.launch import init_tp_engine

    ecfg = EngineConfig(model=model, device="cpu", max_num_seqs=4, max_model_len=256, block_size=32,
                        weight_init="full")
    eng, r = init_tp_engine(ecfg)
    if r != 0:
        eng.runner.worker_loop()
        return None
    prompts = [list(range(5, 40)), list(range(100, 120)), list(range(7, 9))]
    seqs = [eng.add_request(f"q{i}", p, SamplingParams(max_tokens=8, ignore_eos=True)) for i, p in enumerate(prompts)]
    while eng.has_unfinished():
        eng.step()
    eng.shutdown()
    return [s.output_ids for s in seqs]


def _tp_ep_worker(rank, world):
    return _tp_worker(rank, world, model="tiny-mixtral")


def _tp_kv8_worker(rank, world):
    return _tp_worker(rank, world, model="tiny-llama-kv8")


def _tp_e8_worker(rank, world):
    return _tp_worker(rank, world, model="tiny-mixtral-e8")


def _tp_wide_batch_worker(rank, world):
    """TP=2 with 70 concurrent sequences: decode steps past 64 rows run the general path under TP."""
    from symmetry_amd.engine.llm_engine import EngineConfig
    from symmetry_amd.engine.sequence import SamplingParams
    from symmetry_amd.parallel.launch import init_tp_engine

    ecfg = EngineConfig(model="tiny-llama", device="cpu", max_num_seqs=70, max_model_len=128, block_size=16,
                        weight_init="full", num_kv_blocks=70 * 8 + 8)
    eng, r = init_tp_engine(ecfg)
    if r != 0:
        eng.runner.worker_loop()
        return None
    assert eng.scheduler.cfg.max_num_seqs == 70
    prompts = [list(range(5 + i, 15 + i)) for i in range(70)]
    seqs = [eng.add_request(f"w{i}", p, SamplingParams(max_tokens=4, ignore_eos=True)) for i, p in enumerate(prompts)]
    widest = 0
    while eng.has_unfinished():
        eng.step()
        widest = max(widest, sum(1 for s in seqs if s.output_ids and not s.status.finished))
    eng.shutdown()
    return {"outs": [seqs[i].output_ids for i in (0, 33, 69)], "prompts": [prompts[i] for i in (0, 33, 69)],
            "widest": widest}


def test_tp_decode_past_64_rows():
    res = _run(_tp_wide_batch_worker, world=2)
    r = res[0][1]
    assert r["widest"] > 64
    from symmetry_amd.engine.llm_engine import EngineConfig, LLMEngine
    from symmetry_amd.models import reference_model as rm

    eng = LLMEngine(EngineConfig(model="tiny-llama", device="cpu", max_model_len=128, weight_init="full"))
    for p, out in zip(r["prompts"], r["outs"]):
        assert len(out) == 4
        lg = rm.forward_logits(eng.weights, p + out[:-1])
        for j, t in enumerate(out):
            row = lg[len(p) - 1 + j]
            assert float(row.max() - row[t]) <= 0.05


def _check_against_oracle(model, tp_out):
    from symmetry_amd.engine.llm_engine import EngineConfig, LLMEngine
    from symmetry_amd.models import reference_model as rm

    eng = LLMEngine(EngineConfig(model=model, device="cpu", max_num_seqs=4, max_model_len=256, block_size=32,
                                 weight_init="full"))
    prompts = [list(range(5, 40)), list(range(100, 120)), list(range(7, 9))]
    for p, out in zip(prompts, tp_out):
        assert len(out) == 8
        lg = rm.forward_logits(eng.weights, p + out[:-1])
        for j, t in enumerate(out):
            row = lg[len(p) - 1 + j]
            assert float(row.max() - row[t]) <= 0.05


@pytest.mark.parametrize("world", [4, 8])
def test_tp_wide_matches_oracle(world):
    """TP=4 and TP=8 on a model with 8 KV heads: at TP=8 each rank holds ONE KV head and two q heads (the
    Llama-3-70B TP=8 shard geometry), 1/8 of the MLP and 1/8 of the vocabulary; the pipelined decode loop
    runs over the shared-memory metadata ring."""
    res = _run(_tp_kv8_worker, world=world)
    assert all(r[1] is None for r in res[1:])
    _check_against_oracle("tiny-llama-kv8", res[0][1])


def test_tp_ep8_mixtral_matches_oracle():
    """Attention TP=8 + experts EP=8 (one expert per rank, BASELINE config 5 at full width)."""
    res = _run(_tp_e8_worker, world=8)
    _check_against_oracle("tiny-mixtral-e8", res[0][1])


@pytest.mark.parametrize("model", ["tiny-llama", "tiny-mixtral"])
def test_tp2_matches_tp1(model):
    """tiny-llama: TP=2.  tiny-mixtral: attention TP=2 + experts EP=2 (BASELINE config 5 layout)."""
    from symmetry_amd.engine.llm_engine import EngineConfig, LLMEngine
    from symmetry_amd.models import reference_model as rm

    res = _run(_tp_worker if model == "tiny-llama" else _tp_ep_worker)
    tp_out = res[0][1]
    eng = LLMEngine(EngineConfig(model=model, device="cpu", max_num_seqs=4, max_model_len=256, block_size=32,
                                 weight_init="full"))
    prompts = [list(range(5, 40)), list(range(100, 120)), list(range(7, 9))]
    for p, out in zip(prompts, tp_out):
        # TP partial sums reduce in a different order: check against the fp32 oracle (near-ties may flip)
        lg = rm.forward_logits(eng.weights, p + out[:-1])
        for j, t in enumerate(out):
            row = lg[len(p) - 1 + j]
            assert float(row.max() - row[t]) <= 0.05


def _ep_worker(rank, world, model="tiny-mixtral"):
    from symmetry_amd.models.config import resolve
    from symmetry_amd.models.transformer import TransformerLM
    from symmetry_amd.models.weights import ShardSpec, random_weights
    from symmetry_amd.parallel.comm import TorchComm

    cfg = resolve(model)
    comm = TorchComm()
    outs = {}
    g = torch.Generator().manual_seed(11)
    x_all = torch.randn(world, 6, cfg.hidden_size, generator=g).bfloat16()  # per-rank token sets
    x_long = torch.randn(13, cfg.hidden_size, generator=g).bfloat16()       # T not a multiple of the world
    full = random_weights(cfg, ShardSpec(), seed=3)
    ref_model = TransformerLM(full, "cpu")
    ep_w = random_weights(cfg, ShardSpec(0, 1, rank, world), seed=3)
    ep_model = TransformerLM(ep_w, "cpu", ep_comm=comm)
    # all-reduce combine: identical tokens on every rank
    ref = ref_model.moe.forward(0, x_all[0]).clone()
    ep_model.moe.mode = "allreduce"
    outs["allreduce"] = torch.allclose(ep_model.moe.forward(0, x_all[0]), ref, atol=1e-4)
    # the same with every rank's expert shard held once, MFMA-preshuffled (decode_weights="replace")
    sc_model = TransformerLM(random_weights(cfg, ShardSpec(0, 1, rank, world), seed=3), "cpu", ep_comm=comm,
                             decode_weights="replace")
    sc_model.moe.mode = "allreduce"
    outs["single_copy_allreduce"] = sc_model.moe.single_copy and torch.allclose(
        sc_model.moe.forward(0, x_all[0]), ref, atol=1e-4)
    # owner exchange over token slices: identical tokens, every rank's local-expert partials go to the slice
    # owners, a bf16 all-gather rebuilds the output (within one bf16 rounding of the fp32 local block)
    ep_model.moe.mode = "a2a"
    for name, x in (("a2a", x_all[0]), ("a2a_long", x_long), ("a2a_short", x_long[:max(1, world - 2)])):
        ref_r = ref_model.moe.forward(1, x).clone()
        got = ep_model.moe.forward(1, x)
        outs[name] = got.dtype == torch.bfloat16 and bool(
            ((got.float() - ref_r).abs() <= 1e-5 + ref_r.abs() * 2.0 ** -8).all())
        outs[name + "_err"] = float((got.float() - ref_r).abs().max())
    # bytes per rank of the owner exchange on gloo (counts exchanged, then all_to_all_single with them as splits):
    # exactly one fp32 row (+ its int side word) per token that has a local expert and another owner, the bf16
    # all-gather of the owners' slices -- against the fp32 all-reduce combine and the old whole-block exchange
    import symmetry_amd.models.moe as moe_mod

    moe = ep_model.moe
    T, d, k = x_long.shape[0], cfg.hidden_size, cfg.top_k
    S = -(-T // world)
    ids = moe._route(1, x_long)[0][: T * k].view(T, k)
    local = ((ids >= moe.e_lo) & (ids < moe.e_hi)).any(1)
    leaving = sum(1 for t in range(T) if local[t] and t // S != rank)
    moe_mod.A2A_STATS = True
    try:
        moe._pending, moe.a2a_bytes = [], {key: 0 for key in moe.a2a_bytes}
        moe.forward(1, x_long)
        b = moe.a2a_stats()
        outs["a2a_bytes_exact"] = (b["return"] == leaving * (d * 4 + 4) and b["gather"] == (world - 1) * S * d * 2
                                   and b["dispatch"] == 0)
        outs["a2a_bytes_vs_padded"] = b["return"] <= (world - 1) * S * (d * 4 + 4)
        moe.mode = "allreduce"
        moe._pending, moe.a2a_bytes = [], {key: 0 for key in moe.a2a_bytes}
        moe.forward(1, x_long)
        ar = moe.a2a_stats()["allreduce"]
        outs["allreduce_bytes_exact"] = ar == 2 * (world - 1) * T * d * 4 // world
        outs["a2a_fewer_bytes"] = b["return"] + b["gather"] < ar
        outs["bytes"] = {"a2a": b["return"] + b["gather"], "allreduce": ar, "leaving_rows": leaving}
        moe.mode = "a2a"
    finally:
        moe_mod.A2A_STATS = False
    # expert all-to-all with DIFFERENT tokens per rank (data-parallel attention in front of EP)
    ref_t = ref_model.moe.forward(1, x_all[rank]).clone()
    got_t = ep_model.moe.forward_tokens(1, x_all[rank], 6)
    # (at EP = 8 the 8 x 12 receive slots take the grouped-GEMM path, the local oracle the skinny one:
    # a different fp32 summation order can flip one bf16 rounding of the SwiGLU activations)
    outs["tokens"] = torch.allclose(got_t, ref_t, atol=2e-3, rtol=1e-3)
    return outs


def _ep8_worker(rank, world):
    return _ep_worker(rank, world, model="tiny-mixtral-e8")


@pytest.mark.parametrize("world", [2, 4])
def test_expert_parallel_modes_match_local_moe(world):
    res = _run(_ep_worker, world=world)
    for _, r in res:
        assert all(v for k, v in r.items() if not k.endswith("_err") and k != "bytes"), str(r)


def test_expert_parallel_a2a_world8():
    """EP = 8, one expert per rank (Mixtral's layout at full width): the owner exchange and the dispatch /
    return exchange of different tokens per rank."""
    res = _run(_ep8_worker, world=8)
    for _, r in res:
        assert all(v for k, v in r.items() if not k.endswith("_err") and k != "bytes"), str(r)


def _capture_worker(rank, world):
    from symmetry_amd.engine.llm_engine import EngineConfig
    from symmetry_amd.parallel.launch import init_tp_engine

    ecfg = EngineConfig(model="tiny-llama", device="cpu", max_num_seqs=4, max_model_len=1024, block_size=32,
                        weight_init="full")
    eng, r = init_tp_engine(ecfg)
    runner = eng.runner
    seen = []

    def fake_capture(bucket, max_blocks, filtered=False):  # records what a GPU rank would capture
        seen.append((bucket, max_blocks, filtered))
        runner.graphs[(bucket, max_blocks, filtered)] = None

    runner._capture = fake_capture
    runner.use_graphs = True
    if r != 0:
        runner.worker_loop()
        return seen
    runner.capture_all()
    eng.shutdown()
    return seen


def test_tp_graph_capture_is_mirrored_on_every_rank():
    """Decode graphs hold RCCL collectives: every rank must capture the same (batch, context) graphs in
    the same order, driven by rank 0's capture commands on the metadata plane."""
    (_, a), (_, b) = _run(_capture_worker)
    assert a == b and len(a) == len(set(a)) > 4


def test_graph_safety_follows_comm_capturability():
    """Decode hipGraphs stay on for TP when the communicator is capturable -- including the xGMI
    communicator wrapping RCCL (regression: a type check for RcclComm turned graphs off under it)."""
    from types import SimpleNamespace

    from symmetry_amd.engine.llm_engine import LLMEngine
    from symmetry_amd.parallel.comm import HostStagedComm, RcclComm, TorchComm, XgmiComm

    assert RcclComm.capturable and not TorchComm.capturable and not HostStagedComm.capturable
    fake = SimpleNamespace(model=SimpleNamespace(moe=None))
    xg = XgmiComm.__new__(XgmiComm)  # no GPU here: only the attribute XgmiComm.__init__ copies
    xg.world, xg.capturable = 8, RcclComm.capturable
    assert LLMEngine._graph_safe(fake, xg, None)
    assert not LLMEngine._graph_safe(fake, SimpleNamespace(world=2, capturable=False), None)
    assert LLMEngine._graph_safe(fake, SimpleNamespace(world=1), None)


def test_tp_prefill_reduce_moves_one_summed_partial():
    """General-path row-parallel projections under TP all-reduce ONE fp32 [T, N] partial per rank (the
    split-K slabs summed locally first), not the S slabs: S x fewer bytes per collective."""
    from symmetry_amd.models.config import resolve
    from symmetry_amd.models.transformer import TransformerLM
    from symmetry_amd.models.weights import ShardSpec, random_weights
    from symmetry_amd import ops

    seen = []

    class RecComm:
        rank, world, capturable = 0, 2, False

        def all_reduce(self, t, op="sum"):
            seen.append(tuple(t.shape))

    cfg = resolve("tiny-llama-kv8")
    w = random_weights(cfg, ShardSpec(0, 2), seed=1)
    m = TransformerLM(w, "cpu", tp_comm=RecComm())
    T = 48
    x = torch.randn(T, m.hq * m.D).bfloat16()
    wo = w.layer(0, "wo")
    N, K = wo.shape
    assert ops.choose_splits(N, K) > 1  # the projection really produces several split-K slabs
    y = m._linear("o", x, wo, reduce=True)
    assert seen == [(1, T, N)] and m.tp_reduced_bytes["o"] == T * N * 4
    # the reduced partial equals the plain product (slab order only changes fp32 rounding)
    torch.testing.assert_close(y[0], x.float() @ wo.float().t(), rtol=2e-2, atol=2e-2)


def test_tp_prefill_reduce_is_bf16_past_decode_sizes():
    """Prefill-sized steps (> 64 rows) all-reduce the row-parallel partial in bf16: half the bytes of the fp32
    [T, N] partial per collective; the result is the fp32 product rounded once."""
    from symmetry_amd.models.config import resolve
    from symmetry_amd.models.transformer import TransformerLM
    from symmetry_amd.models.weights import ShardSpec, random_weights

    seen = []

    class RecComm:
        rank, world, capturable = 0, 2, False

        def all_reduce(self, t, op="sum"):
            seen.append((tuple(t.shape), t.dtype))

    cfg = resolve("tiny-llama-kv8")
    w = random_weights(cfg, ShardSpec(0, 2), seed=1)
    m = TransformerLM(w, "cpu", tp_comm=RecComm())
    T = 96
    x = torch.randn(T, m.hq * m.D).bfloat16()
    wo = w.layer(0, "wo")
    N, K = wo.shape
    y = m._linear("o", x, wo, reduce=True)
    assert seen == [((T, N), torch.bfloat16)] and m.tp_reduced_bytes["o"] == T * N * 2
    torch.testing.assert_close(y.float(), x.float() @ wo.float().t(), rtol=2e-2, atol=2e-2)


def _tp_long_worker(rank, world):
    from symmetry_amd.engine.llm_engine import EngineConfig
    from symmetry_amd.engine.sequence import SamplingParams
    from symmetry_amd.parallel.launch import init_tp_engine

    ecfg = EngineConfig(model="tiny-llama-kv8", device="cpu", max_num_seqs=4, max_model_len=512, block_size=32,
                        weight_init="full")
    eng, r = init_tp_engine(ecfg)
    if r != 0:
        eng.runner.worker_loop()
        return None
    seqs = [eng.add_request(f"l{i}", p, SamplingParams(max_tokens=8, ignore_eos=True))
            for i, p in enumerate(LONG_PROMPTS)]
    while eng.has_unfinished():
        eng.step()
    eng.shutdown()
    return [s.output_ids for s in seqs], dict(eng.model.tp_reduced_bytes)


LONG_PROMPTS = [list(range(5, 95)), list(range(100, 170)), list(range(300, 310))]  # one 170-token prefill step


def test_tp2_bf16_prefill_reduce_matches_oracle():
    """TP=2 over gloo with a 170-token prefill step: the row-parallel all-reduces of that step move bf16
    partials (2 B per element) and every generated token still agrees with the fp32 oracle."""
    from symmetry_amd.engine.llm_engine import EngineConfig, LLMEngine
    from symmetry_amd.models import reference_model as rm

    res = _run(_tp_long_worker)
    outs, red = res[0][1]
    eng = LLMEngine(EngineConfig(model="tiny-llama-kv8", device="cpu", max_num_seqs=4, max_model_len=512,
                                 block_size=32, weight_init="full"))
    for p, out in zip(LONG_PROMPTS, outs):
        assert len(out) == 8
        lg = rm.forward_logits(eng.weights, p + out[:-1])
        for j, t in enumerate(out):
            row = lg[len(p) - 1 + j]
            assert float(row.max() - row[t]) <= 0.06, (j, t, float(row.max() - row[t]))


# ---- the bench's streamed-token check: the fp32 oracle sharded over TP ranks ---------------------------------
def _oracle_shard_worker(rank, world):
    from symmetry_amd.models import reference_model as rm
    from symmetry_amd.models.config import resolve
    from symmetry_amd.models.layout import apply_decode_layout
    from symmetry_amd.models.weights import ShardSpec, random_weights

    cfg = resolve("tiny-llama")
    w = random_weights(cfg, ShardSpec(rank, world), seed=5, mode="full")
    apply_decode_layout(w)  # the engine's layout: the oracle must undo it per shard
    return rm.forward_logits(w, list(range(3, 40)), group=dist.group.WORLD)


def test_sharded_oracle_matches_full_oracle():
    """bench.py's check under TP runs the fp32 oracle on each rank's shard and sums / gathers over the group: it
    must give the unsharded model's logits on every rank."""
    from symmetry_amd.models import reference_model as rm
    from symmetry_amd.models.config import resolve
    from symmetry_amd.models.weights import random_weights

    full = rm.forward_logits(random_weights(resolve("tiny-llama"), seed=5, mode="full"), list(range(3, 40)))
    for _, lg in _run(_oracle_shard_worker, world=2):
        torch.testing.assert_close(lg, full, atol=1e-4, rtol=1e-4)


def test_check_tokens_flags_a_wrong_token():
    from symmetry_amd.models import reference_model as rm

    lg = torch.zeros(6, 10)
    lg[2:, 7] = 3.0
    lg[3, 4] = 2.95  # a near-tie: either token passes
    ok = rm.check_tokens(lg, 3, [7, 4, 7])
    assert ok["mismatches"] == 0 and ok["max_gap"] == 0.05
    bad = rm.check_tokens(lg, 3, [7, 7, 1])
    assert bad["mismatches"] == 1 and bad["first_mismatch"] == 2
