#!/bin/bash
# TP shard timing (bench/tp_shard.py) with the column-parallel projections on mgemm + fused epilogue
set -o pipefail
out=gpurun_out/tp_shard_mg_ab.jsonl
for tp in 8 4; do
  for rep in $(seq 1 ${REPS:-2}); do
    for proj in none qkv qkv,gu; do
      p=$proj; [ "$p" = none ] && p=""
      SYMMETRY_MG_PROJ=$p timeout -k 10 200 python -u bench/tp_shard.py --tp $tp --clients 10 2>/dev/null | grep "^{" | \
        python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'tp': $tp, 'mg_proj': '$proj', 'rep': $rep, 'ms_per_step': d['ms_per_step']}))" >> $out || exit $?
      tail -1 $out
    done
  done
done
