"""The full-size model on the serving path: Llama-3-8B (32 layers, real shapes, random init), start-up warmup
(prefill size classes + their hipGraphs) captured BEFORE the decode graphs -- the order in which a replayed
memset node once stopped working -- then a burst of prompts decoded under hipGraphs.  Every streamed token must
be within bf16 noise of the fp32 oracle of the same weights (models/reference_model.py, teacher-forced), the
check bench.py applies to its clients.  Small-model tests cannot see a kernel that is wrong only at the real
shapes (K = 14336, N = 28672, 32 layers of accumulated error)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", params=["auto", "replace"])
def engine8b(request):
    """auto: preshuffled decode copies + row-major weights (library / pgemm prefill); replace: the single
    preshuffled copy, every prefill projection on pgemm / mgemm (the 70B-on-one-GPU layout at 8B shapes)."""
    from symmetry_amd.engine.llm_engine import EngineConfig, LLMEngine

    eng = LLMEngine(EngineConfig(model="llama3:8b", device="cuda:0", max_num_seqs=16, max_model_len=2048,
                                 num_kv_blocks=16 * 2048 // 64 + 16, use_graphs=True,
                                 decode_weights=request.param))
    assert eng.model.single_copy == (request.param == "replace")
    eng.warmup([16, 128, 512, 768])
    yield eng
    del eng
    torch.cuda.empty_cache()


def _burst(eng, prompts, n):
    from symmetry_amd.engine.sequence import SamplingParams

    seqs = [eng.add_request(f"r{i}", p, SamplingParams(max_tokens=n, ignore_eos=True)) for i, p in enumerate(prompts)]
    while eng.has_unfinished():
        eng.step()
    return seqs


@pytest.mark.parametrize("nprompts,plen", [(6, 128), (10, 128), (1, 300)])
def test_llama3_8b_streams_match_fp32_oracle(gpu, engine8b, nprompts, plen):
    from symmetry_amd.models import reference_model as rm

    g = torch.Generator().manual_seed(nprompts * 1000 + plen)
    prompts = [torch.randint(256, 120000, (plen,), generator=g).tolist() for _ in range(nprompts)]
    seqs = _burst(engine8b, prompts, 12)
    assert engine8b.runner.graph_replays > 0, "decode steps did not replay hipGraphs"
    for s in seqs[:3]:
        lg = rm.forward_logits(engine8b.weights, list(s.prompt_ids) + list(s.output_ids)[:-1])
        r = rm.check_tokens(lg, len(s.prompt_ids), list(s.output_ids))
        assert len(s.output_ids) == 12 and r["mismatches"] == 0, r
