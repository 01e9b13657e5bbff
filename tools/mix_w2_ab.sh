#!/bin/bash
# Mixtral 4 x 128-token prefill: w2 on the tile kernel (default) vs the streaming kernel with 128-row units vs
# its 2x-mean units -> gpurun_out/w2_ab.jsonl
set -o pipefail
for rep in 1 2; do
  timeout -k 10 300 python3 bench/prefill.py --model mixtral:8x7b --clients 4 --prompt-len 128 --reps 5 2>/dev/null | grep ttft | sed 's/}$/, "arm": "default"}/' >> gpurun_out/w2_ab.jsonl || exit 1
  SYMMETRY_MOE_PRE_ROWS=176 SYMMETRY_MOE_STREAM_POLICY=801 timeout -k 10 300 python3 bench/prefill.py --model mixtral:8x7b --clients 4 --prompt-len 128 --reps 5 2>/dev/null | grep ttft | sed 's/}$/, "arm": "w2 stream mt8"}/' >> gpurun_out/w2_ab.jsonl || exit 1
  SYMMETRY_MOE_PRE_ROWS=176 timeout -k 10 300 python3 bench/prefill.py --model mixtral:8x7b --clients 4 --prompt-len 128 --reps 5 2>/dev/null | grep ttft | sed 's/}$/, "arm": "w2 stream auto-mt"}/' >> gpurun_out/w2_ab.jsonl || exit 1
done
