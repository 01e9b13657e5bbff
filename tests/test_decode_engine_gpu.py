"""The decode-step engine (csrc/kernels/decode_layers.hip): every layer of a dense decode step in ONE persistent
launch, against the per-layer fused launches and the fp32 oracle model."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _engine(model="small-llama", graphs=False):
    from symmetry_amd.engine.llm_engine import EngineConfig, LLMEngine

    return LLMEngine(EngineConfig(model=model, device="cuda:0", max_num_seqs=12, max_model_len=1024,
                                  num_kv_blocks=256, use_graphs=graphs, weight_init="full"))


PROMPTS = [list(range(300, 341)), list(range(100, 123)), list(range(7, 12)), list(range(900, 1200))]


def _generate(eng, n=12):
    from symmetry_amd.engine.sequence import SamplingParams

    seqs = [eng.add_request(f"e{i}", p, SamplingParams(max_tokens=n, ignore_eos=True)) for i, p in enumerate(PROMPTS)]
    while eng.has_unfinished():
        eng.step()
    return [s.output_ids for s in seqs]


@pytest.mark.parametrize("graphs", [False, True])
def test_engine_decode_matches_oracle(gpu, monkeypatch, graphs):
    """small-llama on one GPU (shape class (2, 4, 4, 14): QKV in 2 k-slabs, O K = 1024, gate_up K = 1024, down
    K = 3584): every decode step runs the engine (eager and captured into the decode hipGraphs), and every token
    is within bf16 noise of the fp32 oracle's best next token."""
    from symmetry_amd.models import reference_model as rm
    from symmetry_amd.models import transformer as tr

    monkeypatch.setattr(tr, "DECODE_ENGINE", "1")
    eng = _engine(graphs=graphs)
    outs = _generate(eng)
    assert eng.model.engine_steps > 0, "the engine never ran"
    ref = rm
    for p, out in zip(PROMPTS, outs):
        lg = ref.forward_logits(eng.weights.to("cpu"), p + out[:-1])
        for j, t in enumerate(out):
            row = lg[len(p) - 1 + j]
            assert float(row.max() - row[t]) <= 0.08, (j, t, int(row.argmax()), float(row.max() - row[t]))


def test_engine_tokens_match_per_layer_launches(gpu, monkeypatch):
    """Greedy generations with the engine and with the per-layer fused launches agree token for token up to the
    first position where the fp32 oracle's top-2 logits are closer than the bf16 noise (different fp32 summation
    orders may pick either of a near-tie)."""
    from symmetry_amd.models import reference_model as rm
    from symmetry_amd.models import transformer as tr

    outs = {}
    for mode in ("0", "1"):
        monkeypatch.setattr(tr, "DECODE_ENGINE", mode)
        eng = _engine()
        outs[mode] = _generate(eng)
        assert (eng.model.engine_steps > 0) == (mode == "1")
    w = eng.weights.to("cpu")
    for p, a, b in zip(PROMPTS, outs["0"], outs["1"]):
        lg = rm.forward_logits(w, p + a[:-1])
        for j in range(len(a)):
            if a[j] != b[j]:
                top = lg[len(p) - 1 + j].topk(2).values
                assert float(top[0] - top[1]) < 0.05, (j, a, b)
                break


@pytest.mark.parametrize("graphs", [False, True])
@pytest.mark.parametrize("model,tp", [("llama3:70b", 8), ("llama3:8b", 8), ("llama3:8b", 4), ("llama3:8b", 2),
                                      ("llama3:8b", 1)])
def test_engine_shard_matches_per_layer_launches(gpu, monkeypatch, model, tp, graphs):
    """Every built shape class of the real models, on a TP rank-0 shard (2 layers) with a world-1 xGMI
    communicator (bench/tp_shard.py LocalXgmi): 70B TP = 8 (16, 4, 16, 14) -- QKV 2 k-slabs of 4096, gate_up
    K = 8192 as two tile-major 4096-deep units per tile, O / down two rolled units per workgroup, 8 query heads per
    kv head; 8B TP = 8 / 4 / 2 / 1 -- TP = 1 with 3 rolled QKV units, 7 rolled gate_up units, down as 4 tile-major
    k splits.  The first engine decode step picks the same greedy token as the per-layer launches for (nearly)
    every sequence (a shard's logits are not a model's, so no oracle; a broken engine agrees by chance only)."""
    import os
    import sys

    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bench"))
    from tp_shard import LocalXgmi

    from symmetry_amd.engine.llm_engine import EngineConfig, LLMEngine
    from symmetry_amd.engine.sequence import SamplingParams
    from symmetry_amd.models import transformer as tr
    from symmetry_amd.models.config import resolve

    mc = resolve(model).replace(num_layers=2)
    prompts = [[(97 * i + 13 * k) % 100000 + 300 for k in range(40 + 7 * i)] for i in range(8)]
    toks, steps = {}, {}
    for mode in ("0", "1"):
        monkeypatch.setattr(tr, "DECODE_ENGINE", mode)
        dev = torch.device("cuda:0")
        eng = LLMEngine(EngineConfig(model=model, model_config=mc, device="cuda:0", max_num_seqs=8,
                                     max_model_len=512, num_kv_blocks=64, tp_size=tp, tp_rank=0, weight_init="shard",
                                     use_graphs=graphs, seed=3), tp_comm=LocalXgmi(dev, tp))
        seqs = [eng.add_request(f"s{i}", p, SamplingParams(max_tokens=3, ignore_eos=True))
                for i, p in enumerate(prompts)]
        while eng.has_unfinished():
            eng.step()
        toks[mode] = [s.output_ids for s in seqs]
        steps[mode] = eng.model.engine_steps
        del eng
        torch.cuda.empty_cache()
    assert steps["0"] == 0 and steps["1"] > 0, steps
    assert all(a[0] == b[0] for a, b in zip(toks["0"], toks["1"])), toks  # the prefill token: no engine
    same = sum(a[1] == b[1] for a, b in zip(toks["0"], toks["1"]))
    assert same >= 7, (same, toks)
