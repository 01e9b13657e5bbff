#!/bin/bash
# 10 clients (headline config): which projections of the fused decode path run better on mgemm + fused
# epilogue (in-launch split-K reduction, all 256 CUs) than on the decode GEMMs.  Alternating arms.
set -o pipefail
out=gpurun_out/mg_proj_10_ab.jsonl
for rep in $(seq 1 ${REPS:-3}); do
  for proj in none qkv qkv,o o; do
    p=$proj; [ "$p" = none ] && p=""
    SYMMETRY_MG_PROJ=$p timeout -k 10 240 python -u bench.py --clients 10 --steps 96 --warmup 8 --client-end 0 \
      --max-model-len 1024 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'clients': 10, 'mg_proj': '$proj', 'rep': $rep, 'ms_per_step': d['ms_per_step']}))" >> $out || exit $?
    tail -1 $out
  done
done
