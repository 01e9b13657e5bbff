#!/bin/bash
# Persistent x-resident MLP launch (decode_mlp_xres_kernel): correctness, per-layer timing + phase stamps.
# Run on the gpurun box: bash tools/ab_persistent_mlp.sh [ab]
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_decode_gemm_gpu.py -k "decode_mlp" -x -q --timeout 120 \
  --timeout-method thread > gpurun_out/mlp_test.log 2>&1
rc=$?; tail -3 gpurun_out/mlp_test.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u bench/kernels/bench_decode_mlp.py --ms 10 16 --stamps --xcfgs 8 16 24 > gpurun_out/mlp_layer.jsonl 2>&1
rc=$?; cat gpurun_out/mlp_layer.jsonl; [ $rc -eq 0 ] || exit $rc
[ "$1" = "ab" ] || exit 0
timeout -k 10 600 python -u tools/ab_bench.py gpurun_out/mlp_ab.jsonl --reps 3 \
  --arm launches '' '--client-end 0 --steps 64 --warmup 8' \
  --arm persistent '' '--client-end 0 --steps 64 --warmup 8 --persistent-mlp' > gpurun_out/mlp_ab.log 2>&1
rc=$?; tail -4 gpurun_out/mlp_ab.log; exit $rc
