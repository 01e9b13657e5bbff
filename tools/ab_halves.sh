#!/bin/bash
# Row-half remainder tiles of the x-resident decode GEMM: correctness, then end-to-end A/B (1 GPU, 10 clients)
# and the TP=8 / TP=4 shard timings.  Run on the gpurun box: bash tools/ab_halves.sh
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_decode_gemm_gpu.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/halves_test.log 2>&1
rc=$?; tail -3 gpurun_out/halves_test.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python -u tools/ab_bench.py gpurun_out/halves_ab.jsonl --reps 3 \
  --arm whole 'SYMMETRY_DG_HALVES=0' '--client-end 0 --steps 64 --warmup 8' \
  --arm halves 'SYMMETRY_DG_HALVES=1' '--client-end 0 --steps 64 --warmup 8' > gpurun_out/halves_ab.log 2>&1
rc=$?; tail -2 gpurun_out/halves_ab.log; [ $rc -eq 0 ] || exit $rc
for tp in 4 8; do for hv in 0 1; do
  SYMMETRY_DG_HALVES=$hv timeout -k 10 200 python -u bench/tp_shard.py --tp $tp --clients 10 > gpurun_out/tp_h${hv}_$tp.json 2>/dev/null
  rc=$?; echo "tp $tp halves $hv $(tail -1 gpurun_out/tp_h${hv}_$tp.json | cut -c1-120)"; [ $rc -eq 0 ] || exit $rc
done; done
