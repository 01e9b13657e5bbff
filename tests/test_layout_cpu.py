"""Decode weight layout (models/layout.py) and the fused forward path on CPU references."""
import torch

from symmetry_amd.models.config import resolve as get_config
from symmetry_amd.models.layout import _inverse, apply_decode_layout, gu_perm, natural_tensors, qkv_perm
from symmetry_amd.models.weights import ShardSpec, random_weights
from symmetry_amd.ops import reference as ref


def test_perms_are_permutations_and_pair_rope_halves():
    p = qkv_perm(4, 2, 128)
    assert torch.equal(p.sort().values, torch.arange(p.numel()))
    # tile j of head 0: dims 8j.. then 64+8j..
    assert p[:16].tolist() == list(range(8)) + list(range(64, 72))
    assert p[16:32].tolist() == list(range(8, 16)) + list(range(72, 80))
    # v heads untouched
    assert torch.equal(p[6 * 128:], torch.arange(6 * 128, 8 * 128))
    g = gu_perm(64)
    assert g[:16].tolist() == list(range(8)) + list(range(64, 72))
    assert torch.equal(g[_inverse(g)], torch.arange(128))


def test_layout_roundtrip():
    cfg = get_config("tiny-llama")
    w = random_weights(cfg, ShardSpec(), seed=1)
    orig = {k: v.clone() for k, v in w.tensors.items()}
    apply_decode_layout(w)
    assert w.layout == "decode"
    assert not torch.equal(w.tensors["layers.0.wqkv"], orig["layers.0.wqkv"])
    nat = natural_tensors(w)
    for k in orig:
        assert torch.equal(nat[k], orig[k]), k


def test_permuted_rope_matches_natural():
    T, Hq, Hkv, D, BS = 5, 2, 1, 128, 16
    g = torch.Generator().manual_seed(0)
    qkv = torch.randn(T, (Hq + 2 * Hkv) * D, generator=g)
    qkv_p = qkv[:, qkv_perm(Hq, Hkv, D)]
    cs = ref.rope_table(32, D, 10000.0)
    pos = torch.arange(T, dtype=torch.int32)
    slots = torch.arange(T, dtype=torch.int32)
    outs = []
    for x, perm in ((qkv, False), (qkv_p, True)):
        q = torch.empty(T, Hq, D)
        kc, vc = torch.zeros(1, Hkv, BS, D), torch.zeros(1, Hkv, D, BS)
        ref.rope_cache(x, pos, slots, cs, q, kc, vc, Hq, Hkv, perm=perm)
        outs.append((q, kc, vc))
    for a, b in zip(*outs):
        assert torch.equal(a, b)


def test_deferred_norm_equals_rmsnorm():
    """xw * rsqrt(sum(ss)/d + eps) == RMSNorm(resid) * w (the fused path's invariant)."""
    T, d = 4, 256
    g = torch.Generator().manual_seed(2)
    resid = torch.zeros(T, d)
    delta = torch.randn(T, d, generator=g)
    w = torch.randn(d, generator=g).bfloat16()
    xw, ss = torch.empty(T, d, dtype=torch.bfloat16), torch.empty(T, 1)
    ref.add_prep(delta, resid, w, xw, ss)
    out, out_ref = torch.empty(T, d, dtype=torch.bfloat16), torch.empty(T, d, dtype=torch.bfloat16)
    ref.rownorm(xw, ss, 1e-5, out)
    ref.rms_norm(delta, w, 1e-5, out_ref)
    # two bf16 roundings (xw, out) vs one: within 2 bf16 ulps
    assert ((out.float() - out_ref.float()).abs() <= out_ref.float().abs() * 2 ** -7 + 1e-3).all()


def test_fused_and_general_paths_agree():
    from symmetry_amd.models.transformer import TransformerLM
    from symmetry_amd.engine.llm_engine import EngineConfig, LLMEngine
    from symmetry_amd.engine.sequence import SamplingParams

    outs = []
    for fused in (True, False):
        eng = LLMEngine(EngineConfig(model="tiny-llama", device="cpu", max_num_seqs=4, max_model_len=128,
                                     num_kv_blocks=32, block_size=16, use_graphs=False, seed=0))
        assert isinstance(eng.model, TransformerLM) and eng.model.fused
        eng.model.fused = fused
        outs.append(eng.generate([1, 2, 3, 4, 5, 6, 7], SamplingParams(max_tokens=6, temperature=0.0)))
    assert outs[0] == outs[1]
