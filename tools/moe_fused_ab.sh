#!/bin/bash
# Mixtral 4-client decode step: one-launch MoE routing + fused combine/prep (1) vs the five routing launches (0),
# alternating runs -> gpurun_out/moe_fused_ab.jsonl
set -o pipefail
mkdir -p gpurun_out
for run in 1 2; do
  for f in 0 1; do
    SYMMETRY_MOE_DECODE_FUSED=$f timeout -k 10 300 python -u bench.py --model mixtral:8x7b --clients 4 --steps 48 \
      --warmup 8 --client-end 0 > gpurun_out/moe_ab_$f.json 2> gpurun_out/moe_ab.err || exit $?
    grep '^{' gpurun_out/moe_ab_$f.json | python3 -c "
import json,sys; d=json.loads(sys.stdin.readline()); print(json.dumps({'fused': $f, 'run': $run, 'ms_per_step': d['ms_per_step'], 'engine_per_client_tokens_per_s': d.get('engine_per_client_tokens_per_s')}))" >> gpurun_out/moe_fused_ab.jsonl
  done
done
