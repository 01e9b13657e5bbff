"""Top-k / top-p (nucleus) sampling: the reference semantics on CPU, the HIP kernel on the GPU, and the
engine path (K6)."""
import pytest
import torch

from symmetry_amd import ops
from symmetry_amd.ops import reference as ref


def _rows(B=6, V=1000, seed=0, device="cpu"):
    g = torch.Generator().manual_seed(seed)
    logits = (torch.randn(B, V, generator=g) * 3).to(device)
    temps = torch.tensor([0.7, 1.0, 1.3, 0.0, 1.0, 0.9][:B], device=device)
    top_k = torch.tensor([0, 5, 50, 7, 1, 0][:B], dtype=torch.int32, device=device)
    top_p = torch.tensor([0.9, 1.0, 0.5, 0.3, 1.0, 1.0][:B], device=device)
    seeds = torch.arange(B, dtype=torch.int64, device=device) * 977 + 5
    step = torch.tensor([3], dtype=torch.int64, device=device)
    return logits, temps, top_k, top_p, seeds, step


def _kept_sets(logits, temps, top_k, top_p):
    out = []
    for r in range(logits.shape[0]):
        l = logits[r].float()
        srt, idx = torch.sort(l, descending=True)
        keep = torch.ones_like(l, dtype=torch.bool)
        if 0 < int(top_k[r]) < l.numel():
            keep &= l >= srt[int(top_k[r]) - 1]
        if float(top_p[r]) < 1.0 and float(temps[r]) > 0:
            w = torch.softmax(srt / float(temps[r]), 0)
            n = int((torch.cumsum(w, 0) < float(top_p[r])).sum()) + 1
            keep &= l >= srt[n - 1]
        out.append(set(torch.nonzero(keep).flatten().tolist()))
    return out


def test_reference_respects_filters_and_leaves_other_rows():
    logits, temps, top_k, top_p, seeds, step = _rows()
    ids = torch.full((6,), -1, dtype=torch.int32)
    ref.sample_filtered(logits, temps, top_k, top_p, seeds, step, ids)
    kept = _kept_sets(logits, temps, top_k, top_p)
    for r in (0, 1, 2):
        assert int(ids[r]) in kept[r]
    assert int(ids[3]) == -1 and int(ids[5]) == -1  # greedy row / no filter: untouched
    assert int(ids[4]) == int(logits[4].argmax())   # top_k = 1 is argmax


def test_reference_top_p_distribution():
    """Empirical frequencies over seeds follow the renormalised nucleus distribution."""
    l = torch.tensor([[2.0, 1.5, 1.0, 0.0, -1.0, -3.0]])
    t, p = 1.0, 0.8
    probs = torch.softmax(l[0], 0)
    srt, idx = torch.sort(probs, descending=True)
    n = int((torch.cumsum(srt, 0) < p).sum()) + 1
    nucleus = idx[:n]
    target = torch.zeros(6)
    target[nucleus] = probs[nucleus] / probs[nucleus].sum()
    counts = torch.zeros(6)
    for s in range(3000):
        ids = torch.zeros(1, dtype=torch.int32)
        ref.sample_filtered(l, torch.tensor([t]), torch.tensor([0], dtype=torch.int32), torch.tensor([p]),
                            torch.tensor([s * 7919 + 1]), torch.tensor([s]), ids)
        counts[int(ids)] += 1
    freq = counts / counts.sum()
    assert float((freq - target).abs().max()) < 0.04, (freq, target)


def test_engine_top_k_one_equals_greedy_and_top_p_runs():
    from symmetry_amd.engine.llm_engine import EngineConfig, LLMEngine
    from symmetry_amd.engine.sequence import SamplingParams

    eng = LLMEngine(EngineConfig(model="tiny-llama", device="cpu", max_num_seqs=4, max_model_len=128,
                                 num_kv_blocks=32, block_size=16, use_graphs=False))
    prompt = [3, 14, 15, 92, 65, 35]
    greedy = eng.generate(prompt, SamplingParams(max_tokens=6, temperature=0.0, ignore_eos=True))
    k1 = eng.generate(prompt, SamplingParams(max_tokens=6, temperature=1.0, top_k=1, ignore_eos=True))
    assert k1 == greedy
    a = eng.generate(prompt, SamplingParams(max_tokens=6, temperature=0.8, top_p=0.9, seed=11, ignore_eos=True))
    b = eng.generate(prompt, SamplingParams(max_tokens=6, temperature=0.8, top_p=0.9, seed=11, ignore_eos=True))
    assert a == b and len(a) == 6  # seeded => reproducible


@pytest.mark.gpu
def test_sample_filtered_kernel_matches_reference(gpu):
    for V in (1000, 128256):
        logits, temps, top_k, top_p, seeds, step = _rows(V=V, device=gpu, seed=V)
        ids = torch.full((6,), -1, dtype=torch.int32, device=gpu)
        ops.sample_filtered(logits, temps, top_k, top_p, seeds, step, ids)
        ids_r = torch.full((6,), -1, dtype=torch.int32)
        ref.sample_filtered(logits.cpu(), temps.cpu(), top_k.cpu(), top_p.cpu(), seeds.cpu(), step.cpu(), ids_r)
        assert torch.equal(ids.cpu(), ids_r), (ids.cpu(), ids_r)
