"""Checkpoint I/O: HF safetensors round trip, TP/EP sharding at load, engine from a
checkpoint directory.  safetensors only -- nothing is unpickled."""
import json

import pytest
import torch

from symmetry_amd.models.config import resolve
from symmetry_amd.models.layout import natural_tensors
from symmetry_amd.models.weights import ShardSpec, load_hf_weights, random_weights, save_hf_weights, shard_full


@pytest.mark.parametrize("model", ["tiny-llama", "tiny-mixtral"])
def test_safetensors_roundtrip_and_sharded_load(tmp_path, model):
    cfg = resolve(model)
    w = random_weights(cfg, ShardSpec(), seed=5)
    save_hf_weights(w, str(tmp_path))
    back = load_hf_weights(str(tmp_path), cfg)
    for k, v in natural_tensors(w).items():
        assert torch.equal(back[k], v), k
    for rank in range(2):
        spec = ShardSpec(rank, 2, rank if cfg.is_moe else 0, 2 if cfg.is_moe else 1)
        part = load_hf_weights(str(tmp_path), cfg, spec)
        want = shard_full(cfg, spec, natural_tensors(w))
        for k, v in want.items():
            assert torch.equal(part[k], v), (rank, k)


def test_engine_serves_a_checkpoint_directory(tmp_path):
    from symmetry_amd.engine.llm_engine import EngineConfig, LLMEngine
    from symmetry_amd.engine.sequence import SamplingParams

    ref = LLMEngine(EngineConfig(model="tiny-llama", device="cpu", max_num_seqs=2, max_model_len=128,
                                 num_kv_blocks=16, block_size=16, seed=3, weight_init="full"))
    save_hf_weights(ref.weights, str(tmp_path))
    cfg = resolve("tiny-llama")
    (tmp_path / "config.json").write_text(json.dumps({
        "hidden_size": cfg.hidden_size, "num_attention_heads": cfg.num_heads, "num_key_value_heads": cfg.num_kv_heads,
        "intermediate_size": cfg.intermediate_size, "num_hidden_layers": cfg.num_layers, "vocab_size": cfg.vocab_size,
        "rope_theta": cfg.rope_theta, "rms_norm_eps": cfg.rms_eps, "max_position_embeddings": cfg.max_position,
        "head_dim": cfg.head_dim, "model_type": "llama"}))
    eng = LLMEngine(EngineConfig(model="my-checkpoint", weights=str(tmp_path), device="cpu", max_num_seqs=2,
                                 max_model_len=128, num_kv_blocks=16, block_size=16))
    assert eng.model_cfg.hidden_size == cfg.hidden_size and eng.model_cfg.name == "my-checkpoint"
    p = SamplingParams(max_tokens=6, ignore_eos=True)
    assert eng.generate([4, 5, 6, 7], p) == ref.generate([4, 5, 6, 7], p)
