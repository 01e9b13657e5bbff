"""HF ``tokenizer.json`` path (real checkpoints ship one): chat template with the Llama-3 special tokens,
streaming detokenization of byte-level BPE (multi-byte characters split across tokens), and an engine
serving a checkpoint directory that carries its own tokenizer.  The tokenizer is trained here, in
memory, with the ``tokenizers`` library (no network, no downloaded files)."""
import json

import pytest

tokenizers = pytest.importorskip("tokenizers")


def _train(tmp_path, vocab=300):
    from tokenizers import Tokenizer, decoders, models, pre_tokenizers, trainers

    tok = Tokenizer(models.BPE())
    tok.pre_tokenizer = pre_tokenizers.ByteLevel(add_prefix_space=False)
    tok.decoder = decoders.ByteLevel()
    specials = ["<|begin_of_text|>", "<|end_of_text|>", "<|start_header_id|>", "<|end_header_id|>", "<|eot_id|>"]
    trainer = trainers.BpeTrainer(vocab_size=vocab, special_tokens=specials,
                                  initial_alphabet=pre_tokenizers.ByteLevel.alphabet())
    corpus = ["hello world, streaming tokens over the swarm", "héllo wörld ünïcode ✓ 🚀 日本語テキスト",
              "the quick brown fox jumps over the lazy dog"] * 50
    tok.train_from_iterator(corpus, trainer)
    path = tmp_path / "tokenizer.json"
    tok.save(str(path))
    return str(tmp_path), tok


def test_chat_template_and_streaming_detok(tmp_path):
    from symmetry_amd.engine.tokenizer import HFTokenizer, IncrementalDetokenizer
    from symmetry_amd.models.config import resolve

    d, raw = _train(tmp_path)
    cfg = resolve("tiny-llama")
    tok = HFTokenizer(d, cfg)
    ids = tok.apply_chat_template([{"role": "system", "content": "be brief"}, {"role": "user", "content": "hi ✓"}])
    assert ids[0] == raw.token_to_id("<|begin_of_text|>")
    assert ids.count(raw.token_to_id("<|eot_id|>")) == 2 and ids.count(raw.token_to_id("<|start_header_id|>")) == 3
    text = "héllo wörld ✓ 🚀 日本語テキスト and more"
    toks = tok.encode(text)
    det = IncrementalDetokenizer(tok)
    pieces = [det.add(t) for t in toks]
    pieces.append(det.flush())
    assert "".join(pieces) == text == det.text
    assert all("�" not in p for p in pieces)  # never a half character in a streamed event


def test_engine_uses_checkpoint_tokenizer(tmp_path):
    from symmetry_amd.engine.llm_engine import EngineConfig, LLMEngine
    from symmetry_amd.engine.sequence import SamplingParams
    from symmetry_amd.engine.tokenizer import HFTokenizer
    from symmetry_amd.models.config import resolve
    from symmetry_amd.models.weights import ShardSpec, random_weights, save_hf_weights

    d, raw = _train(tmp_path)
    cfg = resolve("tiny-llama")
    save_hf_weights(random_weights(cfg, ShardSpec(), seed=1), d)
    (tmp_path / "config.json").write_text(json.dumps({
        "hidden_size": cfg.hidden_size, "num_attention_heads": cfg.num_heads, "num_key_value_heads": cfg.num_kv_heads,
        "intermediate_size": cfg.intermediate_size, "num_hidden_layers": cfg.num_layers, "vocab_size": cfg.vocab_size,
        "head_dim": cfg.head_dim, "eos_token_id": raw.token_to_id("<|eot_id|>"),
        "bos_token_id": raw.token_to_id("<|begin_of_text|>"), "model_type": "llama"}))
    eng = LLMEngine(EngineConfig(model="ckpt", weights=d, device="cpu", max_num_seqs=2, max_model_len=128,
                                 num_kv_blocks=16, block_size=16))
    assert isinstance(eng.tokenizer, HFTokenizer)
    out = []
    seq = eng.add_chat_request("r", [{"role": "user", "content": "hello"}], SamplingParams(max_tokens=5),
                               callback=lambda o: out.append(o))
    while eng.has_unfinished():
        eng.step()
    assert seq.status.finished and out[-1].finished
    assert "".join(o.text for o in out) == eng.tokenizer.decode(seq.output_ids)
