#!/bin/bash
# Mixtral 8x7B prefill TTFT, 1-4 prompts of 128 tokens: weight-streaming grouped GEMM on preshuffled expert
# copies (auto) vs the tile kernel only -> gpurun_out/mix_ab.jsonl
set -o pipefail
for c in 1 2 3 4; do
  timeout -k 10 300 python3 bench/prefill.py --model mixtral:8x7b --clients $c --prompt-len 128 --reps 5 2>/dev/null | grep ttft | sed 's/}$/, "preshuffled_experts": "auto"}/' >> gpurun_out/mix_ab.jsonl || exit 1
  SYMMETRY_MOE_PRESHUFFLE=0 SYMMETRY_MOE_STREAM_POLICY=0 timeout -k 10 300 python3 bench/prefill.py --model mixtral:8x7b --clients $c --prompt-len 128 --reps 5 2>/dev/null | grep ttft | sed 's/}$/, "preshuffled_experts": "off"}/' >> gpurun_out/mix_ab.jsonl || exit 1
done
