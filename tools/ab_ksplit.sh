#!/bin/bash
# Split-K x-resident decode GEMMs (SYMMETRY_DG_KSPLIT=1, default) vs whole-K tiles: 10-client bench (QKV 384
# tiles on 256 CUs) and the TP=8 / TP=4 shard timing (QKV 48 / 96 tiles).  Alternating arms.
set -o pipefail
out=gpurun_out/ksplit_ab.jsonl
for rep in $(seq 1 ${REPS:-2}); do
  for ks in 1 0; do
    SYMMETRY_DG_KSPLIT=$ks timeout -k 10 240 python -u bench.py --clients 10 --steps 96 --warmup 8 --client-end 0 \
      --max-model-len 1024 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'bench': '8b_10c', 'ksplit': $ks, 'rep': $rep, 'ms_per_step': d['ms_per_step']}))" >> $out || exit $?
    tail -1 $out
  done
done
for tp in 8 4; do
  for ks in 1 0; do
    SYMMETRY_DG_KSPLIT=$ks timeout -k 10 200 python -u bench/tp_shard.py --tp $tp --clients 10 2>/dev/null | grep "^{" | \
      python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'bench': 'tp_shard', 'tp': $tp, 'ksplit': $ks, 'ms_per_step': d['ms_per_step']}))" >> $out || exit $?
    tail -1 $out
  done
done
