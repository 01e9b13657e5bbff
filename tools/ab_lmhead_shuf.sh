#!/bin/bash
# Preshuffled lm_head copy in the fused decode path: tests, kernel comparison, bench A/B.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_decode_gemm_gpu.py tests/test_engine_gpu.py -x -q --timeout 120 \
  --timeout-method thread > gpurun_out/lmh_test.log 2>&1
rc=$?; tail -3 gpurun_out/lmh_test.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u bench/kernels/bench_decode_gemm.py --shapes lm_head --m 10 --variants -1 \
  --layouts row shuf --chain 4 > gpurun_out/lmh_kernels.jsonl 2>&1
rc=$?; grep '^{' gpurun_out/lmh_kernels.jsonl | cut -c1-140; [ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python -u tools/ab_bench.py gpurun_out/lmh_ab.jsonl --reps 3 \
  --arm row 'SYMMETRY_LMHEAD_SHUF=0' '--client-end 0 --steps 64 --warmup 8' \
  --arm shuf 'SYMMETRY_LMHEAD_SHUF=1' '--client-end 0 --steps 64 --warmup 8' > gpurun_out/lmh_ab.log 2>&1
rc=$?; tail -2 gpurun_out/lmh_ab.log; exit $rc
