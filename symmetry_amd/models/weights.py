"""Model weights: random init (the benchmark mode), safetensors loading, TP/EP sharding.

Weights live in the fused layout the kernels consume:

=================  =======================  ========================================
name               shape (per rank)          notes
=================  =======================  ========================================
embed              [V, d]                    replicated (1 GB for Llama-3-8B)
layers.i.ln1/ln2   [d]
layers.i.wqkv      [(Hq+2Hkv)/tp * D, d]    q|k|v rows of this rank's heads
layers.i.wo        [d, Hq/tp * D]           row-parallel (input columns split)
layers.i.w_gu      [2F/tp, d]               gate rows | up rows of this rank
layers.i.w_down    [d, F/tp]                row-parallel
layers.i.router    [E, d]                   MoE only (replicated)
layers.i.w13       [E/ep, 2F, d]            MoE experts of this rank (gate | up)
layers.i.w2        [E/ep, d, F]
norm               [d]
lm_head            [V/tp, d]                vocab-parallel
=================  =======================  ========================================

``mode="full"`` generates every full tensor from a per-name seed and slices
it, so any TP degree sees the same model (used by the TP-equivalence tests);
``mode="shard"`` generates each rank's shard directly (no full copy: the
70B/TP=8 path), seeded by (name, rank).
"""
from __future__ import annotations

import hashlib
import json
import os
from dataclasses import dataclass, field

import torch

from .config import ModelConfig

INIT_STD = 0.02
# matrices are drawn with std = INIT_GAIN / sqrt(fan_in): 0.02 at d = 4096 (the Llama init),
# and the same activation scale for the small test configs
INIT_GAIN = 1.28


def _std(name: str, shape) -> float:
    if name == "embed":
        return INIT_STD
    return INIT_GAIN / (shape[-1] ** 0.5)


@dataclass
class ShardSpec:
    tp_rank: int = 0
    tp_size: int = 1
    ep_rank: int = 0
    ep_size: int = 1

    def validate(self, cfg: ModelConfig) -> None:
        tp = self.tp_size
        if cfg.num_heads % tp or cfg.num_kv_heads % tp:
            raise ValueError(f"tp={tp} must divide num_heads={cfg.num_heads} and num_kv_heads={cfg.num_kv_heads}")
        if cfg.intermediate_size % tp:
            raise ValueError(f"tp={tp} must divide intermediate_size")
        if cfg.vocab_size % (16 * tp):
            raise ValueError(f"vocab {cfg.vocab_size} must be a multiple of 16*tp")
        if cfg.is_moe and cfg.num_experts % self.ep_size:
            raise ValueError(f"ep={self.ep_size} must divide num_experts={cfg.num_experts}")


@dataclass
class ModelWeights:
    cfg: ModelConfig
    shard: ShardSpec
    tensors: dict = field(default_factory=dict)
    layout: str = "natural"  # "decode" after models.layout.apply_decode_layout
    # names of tensors stored MFMA-preshuffled in place (decode_weights="replace": one copy per weight)
    shuffled: frozenset = frozenset()

    def to(self, device) -> "ModelWeights":
        """Copy on ``device`` (keeps the layout tags)."""
        return ModelWeights(self.cfg, self.shard, {k: v.to(device) for k, v in self.tensors.items()}, self.layout,
                            self.shuffled)

    def __getitem__(self, k):
        return self.tensors[k]

    def layer(self, i: int, name: str) -> torch.Tensor:
        return self.tensors[f"layers.{i}.{name}"]

    def nbytes(self) -> int:
        return sum(t.numel() * t.element_size() for t in self.tensors.values())


def _seed(base: int, name: str, rank: int = -1) -> int:
    h = hashlib.sha256(f"{base}:{name}:{rank}".encode()).digest()
    return int.from_bytes(h[:8], "little") & ((1 << 63) - 1)


def _randn(shape, seed: int, device, dtype, std=INIT_STD) -> torch.Tensor:
    gdev = device if torch.device(device).type != "cpu" else "cpu"
    g = torch.Generator(device=gdev)
    g.manual_seed(seed)
    t = torch.randn(shape, generator=g, device=device, dtype=torch.float32 if gdev == "cpu" else dtype)
    t.mul_(std)
    return t.to(dtype)


def _row_slices(cfg: ModelConfig, shard: ShardSpec):
    tp, r = shard.tp_size, shard.tp_rank
    D = cfg.head_dim
    hq, hkv = cfg.num_heads // tp, cfg.num_kv_heads // tp
    q = slice(r * hq * D, (r + 1) * hq * D)
    k = slice(cfg.q_size + r * hkv * D, cfg.q_size + (r + 1) * hkv * D)
    v = slice(cfg.q_size + cfg.kv_size + r * hkv * D, cfg.q_size + cfg.kv_size + (r + 1) * hkv * D)
    f = cfg.intermediate_size // tp
    return q, k, v, slice(r * f, (r + 1) * f)


def shard_full(cfg: ModelConfig, shard: ShardSpec, full: dict) -> dict:
    """Slice full (unsharded, fused-layout) tensors to one rank's shards."""
    q, k, v, fs = _row_slices(cfg, shard)
    F = cfg.intermediate_size
    out = {}
    vs = cfg.vocab_size // shard.tp_size
    for name, t in full.items():
        if name.endswith(".wqkv"):
            out[name] = torch.cat([t[q], t[k], t[v]], 0).contiguous()
        elif name.endswith(".wo"):
            out[name] = t[:, q].contiguous()
        elif name.endswith(".w_gu"):
            out[name] = torch.cat([t[fs], t[F + fs.start : F + fs.stop]], 0).contiguous()
        elif name.endswith(".w_down"):
            out[name] = t[:, fs].contiguous()
        elif name == "lm_head":
            out[name] = t[shard.tp_rank * vs : (shard.tp_rank + 1) * vs].contiguous()
        elif name.endswith(".w13") or name.endswith(".w2"):
            e = cfg.num_experts // shard.ep_size
            out[name] = t[shard.ep_rank * e : (shard.ep_rank + 1) * e].contiguous()
        else:
            out[name] = t
    return out


def full_shapes(cfg: ModelConfig) -> dict:
    d, F, V, E = cfg.hidden_size, cfg.intermediate_size, cfg.vocab_size, cfg.num_experts
    shapes = {"embed": (V, d), "norm": (d,), "lm_head": (V, d)}
    for i in range(cfg.num_layers):
        p = f"layers.{i}."
        shapes[p + "ln1"] = (d,)
        shapes[p + "ln2"] = (d,)
        shapes[p + "wqkv"] = (cfg.q_size + 2 * cfg.kv_size, d)
        shapes[p + "wo"] = (d, cfg.q_size)
        if cfg.is_moe:
            shapes[p + "router"] = (E, d)
            shapes[p + "w13"] = (E, 2 * F, d)
            shapes[p + "w2"] = (E, d, F)
        else:
            shapes[p + "w_gu"] = (2 * F, d)
            shapes[p + "w_down"] = (d, F)
    return shapes


def shard_shape(cfg: ModelConfig, shard: ShardSpec, name: str, shape: tuple) -> tuple:
    tp = shard.tp_size
    if name.endswith(".wqkv"):
        return ((cfg.q_size + 2 * cfg.kv_size) // tp, shape[1])
    if name.endswith(".wo"):
        return (shape[0], cfg.q_size // tp)
    if name.endswith(".w_gu"):
        return (2 * cfg.intermediate_size // tp, shape[1])
    if name.endswith(".w_down"):
        return (shape[0], cfg.intermediate_size // tp)
    if name == "lm_head":
        return (cfg.vocab_size // tp, shape[1])
    if name.endswith(".w13") or name.endswith(".w2"):
        return (cfg.num_experts // shard.ep_size,) + tuple(shape[1:])
    return shape


def random_weights(cfg: ModelConfig, shard: ShardSpec | None = None, device="cpu", dtype=torch.bfloat16,
                   seed: int = 0, mode: str = "full") -> ModelWeights:
    shard = shard or ShardSpec()
    shard.validate(cfg)
    shapes = full_shapes(cfg)
    tensors = {}
    if mode == "full":
        full = {}
        for name, shape in shapes.items():
            if len(shape) == 1:
                full[name] = torch.ones(shape, dtype=dtype)
            else:
                full[name] = _randn(shape, _seed(seed, name), "cpu", dtype, _std(name, shape))
        if cfg.tie_embeddings:
            full["lm_head"] = full["embed"]
        for name, t in shard_full(cfg, shard, full).items():
            tensors[name] = t.to(device)
    elif mode == "shard":
        for name, shape in shapes.items():
            sshape = shard_shape(cfg, shard, name, shape)
            if len(sshape) == 1:
                tensors[name] = torch.ones(sshape, dtype=dtype, device=device)
            else:
                rank = shard.tp_rank if name not in ("embed",) and not name.endswith("router") else -1
                tensors[name] = _randn(sshape, _seed(seed, name, rank), device, dtype, _std(name, shape))
    else:
        raise ValueError(mode)
    return ModelWeights(cfg, shard, tensors)


# --------------------------------------------------------------------------------------------------
# HuggingFace safetensors checkpoints (Llama / Mixtral naming) -> fused, sharded layout
# --------------------------------------------------------------------------------------------------
def _hf_index(path: str) -> dict:
    idx = os.path.join(path, "model.safetensors.index.json")
    if os.path.exists(idx):
        with open(idx) as f:
            return json.load(f)["weight_map"]
    files = [f for f in os.listdir(path) if f.endswith(".safetensors")]
    from safetensors import safe_open

    wmap = {}
    for fn in files:
        with safe_open(os.path.join(path, fn), framework="pt") as f:
            for k in f.keys():
                wmap[k] = fn
    return wmap


def load_hf_weights(path: str, cfg: ModelConfig, shard: ShardSpec | None = None, device="cpu",
                    dtype=torch.bfloat16) -> ModelWeights:
    """Load a HF safetensors checkpoint directory and fuse/shard it (no pickle anywhere)."""
    from safetensors import safe_open

    shard = shard or ShardSpec()
    shard.validate(cfg)
    wmap = _hf_index(path)
    handles = {}

    def get(name: str) -> torch.Tensor:
        fn = wmap[name]
        if fn not in handles:
            handles[fn] = safe_open(os.path.join(path, fn), framework="pt")
        return handles[fn].get_tensor(name).to(dtype)

    full = {"embed": get("model.embed_tokens.weight"), "norm": get("model.norm.weight")}
    full["lm_head"] = get("lm_head.weight") if "lm_head.weight" in wmap else full["embed"]
    for i in range(cfg.num_layers):
        p, h = f"layers.{i}.", f"model.layers.{i}."
        full[p + "ln1"] = get(h + "input_layernorm.weight")
        full[p + "ln2"] = get(h + "post_attention_layernorm.weight")
        full[p + "wqkv"] = torch.cat([get(h + f"self_attn.{n}_proj.weight") for n in "qkv"], 0)
        full[p + "wo"] = get(h + "self_attn.o_proj.weight")
        if cfg.is_moe:
            m = h + "block_sparse_moe."
            full[p + "router"] = get(m + "gate.weight")
            full[p + "w13"] = torch.stack([
                torch.cat([get(m + f"experts.{e}.w1.weight"), get(m + f"experts.{e}.w3.weight")], 0)
                for e in range(cfg.num_experts)])
            full[p + "w2"] = torch.stack([get(m + f"experts.{e}.w2.weight") for e in range(cfg.num_experts)])
        else:
            full[p + "w_gu"] = torch.cat([get(h + "mlp.gate_proj.weight"), get(h + "mlp.up_proj.weight")], 0)
            full[p + "w_down"] = get(h + "mlp.down_proj.weight")
    tensors = {k: v.to(device) for k, v in shard_full(cfg, shard, full).items()}
    return ModelWeights(cfg, shard, tensors)


def save_hf_weights(weights: ModelWeights, path: str) -> None:
    """Write full (tp=1) fused weights back out in HF naming (used to test the loader)."""
    from safetensors.torch import save_file

    from .layout import natural_tensors

    cfg = weights.cfg
    t = natural_tensors(weights)
    out = {"model.embed_tokens.weight": t["embed"], "model.norm.weight": t["norm"], "lm_head.weight": t["lm_head"]}
    q, kv, F = cfg.q_size, cfg.kv_size, cfg.intermediate_size
    for i in range(cfg.num_layers):
        p, h = f"layers.{i}.", f"model.layers.{i}."
        out[h + "input_layernorm.weight"] = t[p + "ln1"]
        out[h + "post_attention_layernorm.weight"] = t[p + "ln2"]
        w = t[p + "wqkv"]
        out[h + "self_attn.q_proj.weight"] = w[:q]
        out[h + "self_attn.k_proj.weight"] = w[q : q + kv]
        out[h + "self_attn.v_proj.weight"] = w[q + kv :]
        out[h + "self_attn.o_proj.weight"] = t[p + "wo"]
        if cfg.is_moe:
            m = h + "block_sparse_moe."
            out[m + "gate.weight"] = t[p + "router"]
            for e in range(cfg.num_experts):
                out[m + f"experts.{e}.w1.weight"] = t[p + "w13"][e, :F]
                out[m + f"experts.{e}.w3.weight"] = t[p + "w13"][e, F:]
                out[m + f"experts.{e}.w2.weight"] = t[p + "w2"][e]
        else:
            out[h + "mlp.gate_proj.weight"] = t[p + "w_gu"][:F]
            out[h + "mlp.up_proj.weight"] = t[p + "w_gu"][F:]
            out[h + "mlp.down_proj.weight"] = t[p + "w_down"]
    os.makedirs(path, exist_ok=True)
    save_file({k: v.contiguous().cpu() for k, v in out.items()}, os.path.join(path, "model.safetensors"))
