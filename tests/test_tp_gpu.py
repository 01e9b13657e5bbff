"""Tensor / expert parallel launches through the HIP kernels on ONE MI355X.

RCCL refuses two ranks on one device, so the ranks share cuda:0 and reduce through the host-staged
gloo communicator (``SYMMETRY_TP_COMM=gloo``, ``symmetry_amd.parallel.comm.HostStagedComm``).  What
this pins on real hardware is everything of a TP/EP launch except the transport: the sharded weight
layouts (column/row splits, one KV head per rank, the K = F / tp down projection that takes the
non-multiple-of-512 decode GEMM path), vocab-parallel sampling, the rank-0 scheduler driving a
worker through the metadata broadcast, and the expert-parallel MoE blocks.  Graph capture of the
RCCL collectives is covered by ``test_engine_gpu.py::test_rccl_single_rank_allreduce_and_capture``.
"""
import os
import socket

import pytest
import torch

pytestmark = pytest.mark.gpu

PROMPTS = [list(range(300, 341)), list(range(100, 123)), list(range(7, 12))]  # inside every vocab


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _entry(model, rank, world, port, q, xgmi="0", prompts=None, graphs=False, moe_mode="auto"):
    import traceback

    prompts = prompts or PROMPTS
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK="0", SYMMETRY_TP_COMM="gloo", SYMMETRY_XGMI=xgmi, SYMMETRY_MOE_A2A_STATS="1",
                      # the fused GEMM + all-reduce launches between the two processes: the small test models' grids
                      # (<= 64 workgroups per rank) are co-resident on the one GPU
                      SYMMETRY_XGMI_FUSED="force", SYMMETRY_MOE_XGMI_A2A="force", SYMMETRY_MOE_MODE=moe_mode,
                      # graphs: decode steps captured and replayed with every collective on the xGMI kernels
                      SYMMETRY_XGMI_GRAPHS="1" if graphs else "0")
    try:
        from symmetry_amd.engine.llm_engine import EngineConfig
        from symmetry_amd.engine.sequence import SamplingParams
        from symmetry_amd.parallel.launch import init_tp_engine

        ecfg = EngineConfig(model=model, device="cuda", max_num_seqs=4, max_model_len=512, num_kv_blocks=64,
                            use_graphs=graphs, weight_init="full")
        eng, r = init_tp_engine(ecfg)
        if xgmi == "1":
            from symmetry_amd.parallel.comm import XgmiComm

            assert isinstance(eng.runner.model.tp, XgmiComm), type(eng.runner.model.tp)
        if r != 0:
            eng.runner.worker_loop()
            q.put((rank, None))
            return
        try:
            seqs = [eng.add_request(f"t{i}", p, SamplingParams(max_tokens=10, ignore_eos=True))
                    for i, p in enumerate(prompts)]
            while eng.has_unfinished():
                eng.step()
        finally:
            eng.shutdown()  # the worker leaves its loop whatever happened here
        if graphs:
            assert eng.runner.use_graphs and eng.runner.graph_replays > 0, "decode steps did not replay graphs"
        if xgmi == "1":
            calls = eng.runner.model.tp.calls
            # decode steps ran the peer-memory all-reduce: fused into the row-parallel GEMMs (one XAR launch each:
            # GEMM + all-reduce + residual) for the dense model, the fused add_prep kernel around the MoE block
            assert calls.get("gemm_ar", 0) + calls["add_prep"] > 0, calls
            if model == "small-llama":  # dense: every row-parallel decode projection ran as ONE fused XAR launch
                assert calls.get("gemm_ar", 0) > 0 and calls["add_prep"] == 0, calls
            assert calls.get("keys", 0) > 0, calls  # and the vocab-parallel sampling combine
            assert eng.runner.model.tp.error() == 0
        extra = {}
        moe = eng.runner.model.moe
        if moe is not None:
            extra = {"moe_calls": dict(moe.calls), "a2a_bytes": moe.a2a_stats(),
                     "xgmi_a2a": eng.runner.model.tp.calls.get("a2a", 0) if xgmi == "1" else 0}
        q.put((rank, ([s.output_ids for s in seqs], extra)))
    except Exception:
        q.put((rank, traceback.format_exc()))
    finally:
        import torch.distributed as dist

        if dist.is_initialized():
            dist.destroy_process_group()


def _run(model, world=2, xgmi="0", prompts=None, extra=False, graphs=False, moe_mode="auto"):
    import torch.multiprocessing as mp

    port = _port()
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    procs = [ctx.Process(target=_entry, args=(model, r, world, port, q, xgmi, prompts, graphs, moe_mode))
             for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get() for _ in range(world))
    for p in procs:
        p.join(60)
    errs = [v for v in res.values() if isinstance(v, str)]
    assert not errs, errs[0]
    return res[0] if extra else res[0][0]


def _check_oracle(model, prompts, outs):
    """Every token within bf16 noise of the fp32 oracle's best logit; MoE: up to the first position whose
    oracle routing has a near-tie (k-th vs (k+1)-th expert margin < 0.005), where bf16 may pick the other
    expert and the sequences legitimately diverge."""
    from symmetry_amd.engine.llm_engine import EngineConfig, LLMEngine
    from symmetry_amd.models import reference_model as rm

    ref = LLMEngine(EngineConfig(model=model, device="cpu", max_num_seqs=4, max_model_len=512, weight_init="full"))
    for p, out in zip(prompts, outs):
        assert len(out) == 10
        gaps = []
        lg = rm.forward_logits(ref.weights, p + out[:-1], router_gaps=gaps)
        tie = None
        if gaps:
            hit = (torch.stack(gaps).min(0).values < 0.005).nonzero()
            tie = int(hit[0]) if hit.numel() else None
        for j, t in enumerate(out):
            pos = len(p) - 1 + j
            if tie is not None and pos >= tie:
                break
            row = lg[pos]
            assert float(row.max() - row[t]) <= 0.08, (j, t, int(row.argmax()), float(row.max() - row[t]))


LONG_PROMPTS = [list(range(300, 420)), list(range(400, 490)), list(range(7, 40))]  # 243 tokens: a2a prefill


def test_tp2_mixtral_unpadded_a2a_on_one_gpu(gpu):
    """tiny-mixtral attention TP=2 + EP=2 with a 243-token prefill step (SYMMETRY_MOE_MODE=a2a): the replicated-token owner
    exchange (models/moe.py forward_a2a) on the xGMI a2a kernel between the two processes (IPC-mapped buffers on
    one GPU) -- no dispatch leg, at most one pre-combined fp32 row per token leaves a rank, the slices come back
    by a bf16 all-gather -- fewer bytes than the fp32 all-reduce combine, and every token agrees with the fp32
    oracle."""
    outs, extra = _run("tiny-mixtral", xgmi="1", prompts=LONG_PROMPTS, extra=True, moe_mode="a2a")
    assert extra["moe_calls"]["a2a"] > 0 and extra["xgmi_a2a"] > 0, extra
    b = extra["a2a_bytes"]
    from symmetry_amd.models.config import resolve

    cfg = resolve("tiny-mixtral")
    d = cfg.hidden_size
    T = sum(len(p) for p in LONG_PROMPTS)
    calls = extra["moe_calls"]["a2a"]
    assert b["dispatch"] == 0 and b["return"] > 0 and b["gather"] > 0, b
    # a token sends at most one row to its (one) other owner: at most T/2 rows per call leave rank 0 at N = 2
    assert b["return"] <= calls * (T // 2 + 1) * d * 4, b
    allreduce = calls * 2 * (2 - 1) / 2 * T * d * 4  # ring all-reduce of the fp32 [T, d] partials, per rank
    assert b["return"] + b["gather"] < allreduce, (b, allreduce)
    _check_oracle("tiny-mixtral", LONG_PROMPTS, outs)


@pytest.mark.parametrize("xgmi", ["0", "1"])
@pytest.mark.parametrize("model", ["small-llama", "tiny-mixtral"])
def test_tp2_on_one_gpu_matches_oracle(gpu, model, xgmi):
    """small-llama: TP=2 (1 KV head per rank, down K = 1792).  tiny-mixtral: attention TP=2 + EP=2.
    xgmi=1: the decode all-reduces (+ fused residual / norm prep) run on the one-shot peer-memory kernel
    between the two processes (IPC-mapped buffers on the one GPU)."""
    from symmetry_amd.engine.llm_engine import EngineConfig, LLMEngine
    from symmetry_amd.models import reference_model as rm

    outs = _run(model, xgmi=xgmi)
    ref = LLMEngine(EngineConfig(model=model, device="cpu", max_num_seqs=4, max_model_len=512, weight_init="full"))
    for p, out in zip(PROMPTS, outs):
        assert len(out) == 10
        lg = rm.forward_logits(ref.weights, p + out[:-1])
        for j, t in enumerate(out):
            row = lg[len(p) - 1 + j]
            # bf16 kernels + a different reduction order than the fp32 oracle: near-ties may flip
            assert float(row.max() - row[t]) <= 0.08, (j, t, int(row.argmax()), float(row.max() - row[t]))


def test_tp2_fused_xar_under_hipgraphs_on_one_gpu(gpu):
    """The default 8-GPU decode path end to end between two processes: small-llama TP=2 with every decode step
    captured into a hipGraph and replayed, the o / down projections as fused GEMM + xGMI all-reduce + residual
    launches (``SYMMETRY_XGMI_FUSED=force``) on the shared per-tile epoch counters, IPC-mapped peer buffers;
    every token within bf16 noise of the fp32 oracle."""
    outs = _run("small-llama", xgmi="1", graphs=True)
    _check_oracle("small-llama", PROMPTS, outs)


