"""Model configurations and the ``modelName`` registry.

``provider.yaml``'s ``modelName`` (REF: read at ``src/provider.ts:313`` and
forwarded to the upstream server) selects the architecture the native engine
runs.  Ollama-style tags (``llama3:8b``) and HF-style ids both resolve here.
Shapes are the public configs of the named models.
"""
from __future__ import annotations

import dataclasses
from dataclasses import dataclass, field


@dataclass(frozen=True)
class ModelConfig:
    name: str
    vocab_size: int
    hidden_size: int
    intermediate_size: int
    num_layers: int
    num_heads: int
    num_kv_heads: int
    head_dim: int = 128
    rope_theta: float = 500000.0
    rms_eps: float = 1e-5
    max_position: int = 8192
    rope_scaling: dict | None = field(default=None, hash=False, compare=False)
    tie_embeddings: bool = False
    # mixture of experts (Mixtral); num_experts == 0 -> dense MLP
    num_experts: int = 0
    top_k: int = 2
    # special tokens of the chat format
    bos_token_id: int = 128000
    eos_token_ids: tuple = (128001, 128009)
    chat_format: str = "llama3"

    @property
    def is_moe(self) -> bool:
        return self.num_experts > 0

    @property
    def q_size(self) -> int:
        return self.num_heads * self.head_dim

    @property
    def kv_size(self) -> int:
        return self.num_kv_heads * self.head_dim

    def num_params(self) -> int:
        d, f, v = self.hidden_size, self.intermediate_size, self.vocab_size
        attn = d * (self.q_size + 2 * self.kv_size) + self.q_size * d
        mlp = 3 * d * f * (self.num_experts if self.is_moe else 1) + (d * self.num_experts if self.is_moe else 0)
        per_layer = attn + mlp + 2 * d
        head = 0 if self.tie_embeddings else v * d
        return v * d + self.num_layers * per_layer + d + head

    def kv_bytes_per_token(self, dtype_bytes: int = 2) -> int:
        return 2 * self.num_layers * self.kv_size * dtype_bytes

    def replace(self, **kw) -> "ModelConfig":
        return dataclasses.replace(self, **kw)


LLAMA31_SCALING = {
    "rope_type": "llama3",
    "factor": 8.0,
    "low_freq_factor": 1.0,
    "high_freq_factor": 4.0,
    "original_max_position_embeddings": 8192,
}

LLAMA3_8B = ModelConfig(
    name="llama3:8b", vocab_size=128256, hidden_size=4096, intermediate_size=14336, num_layers=32, num_heads=32,
    num_kv_heads=8, rope_theta=500000.0, max_position=8192,
)
LLAMA31_8B = LLAMA3_8B.replace(name="llama3.1:8b", max_position=131072, rope_scaling=LLAMA31_SCALING)
LLAMA3_70B = ModelConfig(
    name="llama3:70b", vocab_size=128256, hidden_size=8192, intermediate_size=28672, num_layers=80, num_heads=64,
    num_kv_heads=8, rope_theta=500000.0, max_position=8192,
)
LLAMA31_70B = LLAMA3_70B.replace(name="llama3.1:70b", max_position=131072, rope_scaling=LLAMA31_SCALING)
MIXTRAL_8X7B = ModelConfig(
    name="mixtral:8x7b", vocab_size=32000, hidden_size=4096, intermediate_size=14336, num_layers=32, num_heads=32,
    num_kv_heads=8, rope_theta=1e6, max_position=32768, num_experts=8, top_k=2, bos_token_id=1,
    eos_token_ids=(2,), chat_format="mistral",
)
# Small configs with the same structure, for CPU tests and GPU smoke runs.
TINY_LLAMA = ModelConfig(
    name="tiny-llama", vocab_size=512, hidden_size=256, intermediate_size=512, num_layers=2, num_heads=4,
    num_kv_heads=2, rope_theta=10000.0, max_position=2048, bos_token_id=500, eos_token_ids=(501, 502),
)
TINY_MIXTRAL = TINY_LLAMA.replace(name="tiny-mixtral", num_experts=4, top_k=2)
# 8 KV heads like Llama-3-70B / Mixtral: TP=8 leaves one KV head (and two q heads) per rank, the 70B TP=8
# shard geometry; the MoE variant has 8 experts, one per rank at EP=8
TINY_LLAMA_KV8 = TINY_LLAMA.replace(name="tiny-llama-kv8", num_heads=16, num_kv_heads=8, intermediate_size=2048)
TINY_MIXTRAL_E8 = TINY_LLAMA_KV8.replace(name="tiny-mixtral-e8", num_experts=8, top_k=2)
SMALL_LLAMA = ModelConfig(
    name="small-llama", vocab_size=32768, hidden_size=1024, intermediate_size=3584, num_layers=4, num_heads=8,
    num_kv_heads=2, max_position=8192, bos_token_id=32000, eos_token_ids=(32001, 32002),
)

_REGISTRY = {
    c.name: c
    for c in (LLAMA3_8B, LLAMA31_8B, LLAMA3_70B, LLAMA31_70B, MIXTRAL_8X7B, TINY_LLAMA, TINY_MIXTRAL, SMALL_LLAMA,
              TINY_LLAMA_KV8, TINY_MIXTRAL_E8)
}
_ALIASES = {
    "llama3": "llama3:8b",
    "llama3:latest": "llama3:8b",
    "llama3:8b-instruct": "llama3:8b",
    "llama3.1": "llama3.1:8b",
    "llama3.1:latest": "llama3.1:8b",
    "meta-llama/meta-llama-3-8b": "llama3:8b",
    "meta-llama/meta-llama-3-8b-instruct": "llama3:8b",
    "meta-llama/llama-3.1-8b-instruct": "llama3.1:8b",
    "meta-llama/meta-llama-3-70b-instruct": "llama3:70b",
    "meta-llama/llama-3.1-70b-instruct": "llama3.1:70b",
    "mixtral": "mixtral:8x7b",
    "mixtral:latest": "mixtral:8x7b",
    "mistralai/mixtral-8x7b-instruct-v0.1": "mixtral:8x7b",
}


def resolve(model_name: str) -> ModelConfig:
    key = model_name.strip().lower()
    key = _ALIASES.get(key, key)
    if key not in _REGISTRY:
        raise KeyError(f"unknown modelName {model_name!r}; known: {sorted(_REGISTRY) + sorted(_ALIASES)}")
    return _REGISTRY[key]


def known_models() -> list[str]:
    return sorted(set(_REGISTRY) | set(_ALIASES))


def from_hf_config(cfg: dict, name: str = "hf") -> ModelConfig:
    """Build a ModelConfig from a HuggingFace ``config.json`` dict (Llama / Mixtral)."""
    d = cfg["hidden_size"]
    nh = cfg["num_attention_heads"]
    eos = cfg.get("eos_token_id", 2)
    return ModelConfig(
        name=name,
        vocab_size=cfg["vocab_size"],
        hidden_size=d,
        intermediate_size=cfg["intermediate_size"],
        num_layers=cfg["num_hidden_layers"],
        num_heads=nh,
        num_kv_heads=cfg.get("num_key_value_heads", nh),
        head_dim=cfg.get("head_dim", d // nh),
        rope_theta=float(cfg.get("rope_theta", 10000.0)),
        rms_eps=float(cfg.get("rms_norm_eps", 1e-5)),
        max_position=int(cfg.get("max_position_embeddings", 8192)),
        rope_scaling=cfg.get("rope_scaling"),
        tie_embeddings=bool(cfg.get("tie_word_embeddings", False)),
        num_experts=int(cfg.get("num_local_experts", 0)),
        top_k=int(cfg.get("num_experts_per_tok", 2)),
        bos_token_id=int(cfg.get("bos_token_id", 1)),
        eos_token_ids=tuple(eos) if isinstance(eos, list) else (int(eos),),
        chat_format="mistral" if cfg.get("model_type") == "mixtral" else "llama3",
    )
