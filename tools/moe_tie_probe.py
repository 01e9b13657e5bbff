"""Why does a MoE engine run leave the fp32 oracle's argmax?  Router near-ties of the oracle per position."""
import sys

import torch

sys.path.insert(0, ".")
from symmetry_amd.engine.llm_engine import EngineConfig, LLMEngine  # noqa: E402
from symmetry_amd.engine.sequence import SamplingParams  # noqa: E402
from symmetry_amd.models import reference_model as rm  # noqa: E402

eng = LLMEngine(EngineConfig(model="tiny-mixtral", device="cuda:0", max_num_seqs=8, max_model_len=1024,
                             num_kv_blocks=64, use_graphs=True))
prompts = [eng.tokenizer.apply_chat_template([{"role": "user", "content": f"question {i} " * (i + 1)}])
           for i in range(5)]
seqs = [eng.add_request(f"g{i}", p, SamplingParams(max_tokens=12, ignore_eos=True)) for i, p in enumerate(prompts)]
while eng.has_unfinished():
    eng.step()
cpu = eng.weights.to("cpu")
gaps = []
orig = rm._moe


def spy(cfg, w, i, h):
    lg = h @ w.layer(i, "router").float().t()
    top = lg.topk(3, dim=-1).values
    gaps.append((i, (top[:, 1] - top[:, 2]).min().item(), int((top[:, 1] - top[:, 2]).argmin())))
    return orig(cfg, w, i, h)


rm._moe = spy
for p, s in zip(prompts, seqs):
    gaps.clear()
    lg = rm.forward_logits(cpu, p + s.output_ids[:-1])
    margins = [float(lg[len(p) - 1 + j].max() - lg[len(p) - 1 + j][t]) for j, t in enumerate(s.output_ids)]
    print(len(p), "max margin", round(max(margins), 4), "at", margins.index(max(margins)),
          "router 2nd-3rd gap min per layer", [(i, round(g, 5), pos) for i, g, pos in gaps], flush=True)
