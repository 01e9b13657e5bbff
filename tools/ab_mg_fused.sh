#!/bin/bash
# A/B of the fused general decode path (mgemm + in-launch split-K reduction + decode epilogues) against the
# slab + consumer-kernel path, alternating arms, at wide client counts (bench.py, engine-side timing).
set -o pipefail
out=gpurun_out/mg_fused_ab.jsonl
for c in ${CLIENTS:-64 32 20}; do
  for rep in 1 2; do
    for mg in ${MODES:-all 0}; do
      SYMMETRY_MG_FUSED=$mg timeout -k 10 240 python -u bench.py --clients $c --steps 64 --warmup 8 --client-end 0 \
        --max-model-len 1024 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'clients': $c, 'mg_fused': '$mg', 'rep': $rep, 'ms_per_step': d['ms_per_step'], 'tokens_per_s': d['value'], 'p50_ttft_ms': d['p50_ttft_ms']}))" >> $out || exit $?
      tail -1 $out
    done
  done
done
[ -n "$SKIP10" ] && exit 0
# 10 clients (the headline config): the fused decode kernels vs the fused general path forced from 1 row
out2=gpurun_out/mg_general_10_ab.jsonl
for rep in 1 2; do
  for gr in 20 1; do
    SYMMETRY_GENERAL_ROWS=$gr timeout -k 10 240 python -u bench.py --clients 10 --steps 64 --warmup 8 --client-end 0 \
      --max-model-len 1024 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'clients': 10, 'general_rows': $gr, 'rep': $rep, 'ms_per_step': d['ms_per_step'], 'p50_ttft_ms': d['p50_ttft_ms']}))" >> $out2 || exit $?
    tail -1 $out2
  done
done
