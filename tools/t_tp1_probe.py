import sys, os, torch
sys.path.insert(0, "/root/repo"); sys.path.insert(0, "/root/repo/bench")
from tp_shard import LocalXgmi
from symmetry_amd.engine.llm_engine import EngineConfig, LLMEngine
from symmetry_amd.engine.sequence import SamplingParams
from symmetry_amd.models import transformer as tr
from symmetry_amd.models.config import resolve
mc = resolve("llama3:8b").replace(num_layers=2)
prompts = [[(97 * i + 13 * k) % 100000 + 300 for k in range(20 + 7 * i)] for i in range(6)]
for graphs in (True,):
    toks = {}
    for mode in ("0", "1"):
        tr.DECODE_ENGINE = mode
        dev = torch.device("cuda:0")
        eng = LLMEngine(EngineConfig(model="llama3:8b", model_config=mc, device="cuda:0", max_num_seqs=8, max_model_len=1024,
                                     num_kv_blocks=64, use_graphs=graphs, weight_init="full", seed=3))
        if graphs:
            eng.warmup([16, 128])
        seqs = [eng.add_request(f"s{i}", p, SamplingParams(max_tokens=4, ignore_eos=True)) for i, p in enumerate(prompts)]
        while eng.has_unfinished():
            eng.step()
        toks[mode] = [s.output_ids for s in seqs]
        fb = eng.model._engine_cache.get("fault")
        print("graphs", graphs, "mode", mode, "engine_steps", eng.model.engine_steps, "fault", None if fb is None else fb.tolist(), toks[mode], flush=True)
        del eng; torch.cuda.empty_cache()
