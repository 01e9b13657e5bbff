"""Host-side hot path of wide decode batches (CPU): the vectorised decode metadata packer writes exactly the
bytes of the generic one, Sequence.token_slice equals slicing token_ids, and the per-token SSE fast path
encodes exactly what the generic chunk encoding does."""
import json
import random

import numpy as np

from symmetry_amd.engine.model_runner import ModelRunner, _Layout
from symmetry_amd.engine.sequence import SamplingParams, Sequence
from symmetry_amd.protocol import sse


class _Runner:
    block_size = 64
    _fill_decode = ModelRunner._fill_decode
    _fill_generic = ModelRunner._fill_generic


def _seqs(n, rng):
    out, prev = [], {}
    for i in range(n):
        prompt = [rng.randrange(1, 1000) for _ in range(rng.randrange(1, 300))]
        s = Sequence(f"r{i}", prompt, SamplingParams(temperature=rng.choice([0.0, 0.7]), top_k=rng.choice([0, 40]),
                                                     top_p=rng.choice([1.0, 0.9])))
        s.output_ids = [rng.randrange(1, 1000) for _ in range(rng.randrange(0, 50))]
        s.sampling_seed = rng.randrange(-(1 << 63), 1 << 63)
        total = len(prompt) + len(s.output_ids)
        # pipelined decode: the newest token may still be in flight (num_computed == total)
        s.num_computed = total - 1 if rng.random() < 0.5 else total
        if s.num_computed == total:
            prev[s.seq_id] = rng.randrange(0, 256)
        s.block_table = rng.sample(range(1, 5000), (s.num_computed + 64) // 64)
        out.append(s)
    return out, prev


def test_decode_fill_matches_generic():
    rng = random.Random(7)
    r = _Runner()
    for n, bucket in ((1, 1), (10, 12), (130, 160), (256, 256)):
        seqs, prev = _seqs(n, rng)
        mb = max(len(s.block_table) for s in seqs) + 2
        lay = _Layout(bucket, bucket, mb, prefill=False)
        a = np.full(lay.size, 77, dtype=np.int32)
        b = np.full(lay.size, 99, dtype=np.int32)
        r._fill_decode(lay, a, seqs, prev)
        r._fill_generic(lay, b, seqs, [1] * n, prev)
        assert np.array_equal(a, b), n


def test_token_slice():
    s = Sequence("x", list(range(10)), SamplingParams())
    s.output_ids = list(range(100, 105))
    for start in range(16):
        for n in range(0, 8):
            assert s.token_slice(start, n) == s.token_ids[start:start + n]


def test_sse_fast_path_bytes():
    def generic(cid, model, content, finish_reason, created):
        obj = {"id": cid, "object": "chat.completion.chunk", "created": created, "model": model,
               "system_fingerprint": "symmetry_amd",
               "choices": [{"index": 0, "delta": {"content": content}, "finish_reason": finish_reason}]}
        return "data: " + json.dumps(obj, separators=(",", ":"), ensure_ascii=False) + "\n\n"

    for content in ("tok", 'q"uote\\', "ü 漢字 \n\t\x01", ""):
        for fr in (None, "stop", "length"):
            assert sse.chunk_event('c"1', "llama3:8b", content, finish_reason=fr, created=7) == \
                generic('c"1', "llama3:8b", content, fr, 7)
