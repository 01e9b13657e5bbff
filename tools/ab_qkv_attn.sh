#!/bin/bash
# Fused QKV + decode attention launch (decode_qkv_attn_kernel): correctness, then end-to-end A/B.
# Run on the gpurun box: bash tools/ab_qkv_attn.sh
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_decode_gemm_gpu.py -k "qkv_attn" -x -q --timeout 120 \
  --timeout-method thread > gpurun_out/qa_test.log 2>&1
rc=$?; tail -3 gpurun_out/qa_test.log; [ $rc -eq 0 ] || exit $rc
SYMMETRY_QKV_ATTN=1 timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 120 \
  --timeout-method thread > gpurun_out/qa_engine.log 2>&1
rc=$?; tail -3 gpurun_out/qa_engine.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python -u tools/ab_bench.py gpurun_out/qa_ab.jsonl --reps 3 \
  --arm launches 'SYMMETRY_QKV_ATTN=0' '--client-end 0 --steps 64 --warmup 8' \
  --arm fused 'SYMMETRY_QKV_ATTN=1' '--client-end 0 --steps 64 --warmup 8' > gpurun_out/qa_ab.log 2>&1
rc=$?; tail -3 gpurun_out/qa_ab.log; exit $rc
