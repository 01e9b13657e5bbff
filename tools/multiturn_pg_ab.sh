#!/bin/bash
# Multi-turn chat TTFT (prefix-cache tails of ~130 tokens over 1.1-1.5K contexts) with prefill graphs on / off
set -o pipefail
mkdir -p gpurun_out
for t in 256 0 256 0; do
  SYMMETRY_PREFILL_GRAPH_TOKENS=$t timeout -k 10 240 python -u bench/multiturn.py 2>>gpurun_out/mt_pg.err | grep '^{' \
    | sed "s/^{/{\"prefill_graph_tokens\": $t, /" >> gpurun_out/mt_pg.jsonl || exit $?
done
