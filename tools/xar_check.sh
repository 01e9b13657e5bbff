#!/bin/bash
# Fused row-parallel GEMM + xGMI all-reduce (XAR): kernel tests, TP tests, TP-shard A/B (fused on / off), 1-GPU bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_xgmi_gpu.py tests/test_tp_gpu.py tests/test_decode_gemm_gpu.py -x -q \
  --timeout 120 --timeout-method thread > gpurun_out/xar_tests.log 2>&1
rc=$?; tail -4 gpurun_out/xar_tests.log; [ $rc -eq 0 ] || exit $rc
for tp in ${TPS:-8 4 2}; do
  for fused in 1 0; do
    SYMMETRY_XGMI_FUSED=$fused timeout -k 10 200 python -u bench/tp_shard.py --tp $tp --clients 10 > gpurun_out/tp_shard_${tp}_f$fused.json 2> gpurun_out/tp_shard_${tp}_f$fused.err
    rc=$?; echo "tp=$tp fused=$fused $(tail -1 gpurun_out/tp_shard_${tp}_f$fused.json)"; [ $rc -eq 0 ] || exit $rc
  done
done
for fused in 1 0; do
  SYMMETRY_XGMI_FUSED=$fused timeout -k 10 300 python -u bench/tp_shard.py --tp 8 --clients 4 --model llama3:70b > gpurun_out/tp_shard_70b_f$fused.json 2>gpurun_out/tp_shard_70b_f$fused.err
  rc=$?; echo "70b fused=$fused $(tail -1 gpurun_out/tp_shard_70b_f$fused.json)"; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 300 python -u bench.py --client-end 0 --steps 64 > gpurun_out/bench_ce0.json 2> gpurun_out/bench_ce0.err
rc=$?; grep '^{' gpurun_out/bench_ce0.json | cut -c1-400; exit $rc
