#!/bin/bash
# Decode-step engine A/B on one GPU: edge form x control-wave prefetch, phase stamps + TP=8 shard step time
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/engine_ab.jsonl
: > $out
timeout -k 10 200 python -u -m pytest tests/test_decode_engine_gpu.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/engine_tests.log 2>&1 || { tail -20 gpurun_out/engine_tests.log; exit 1; }
for edge in 1 0; do
  for cp in 0 1; do
    echo "{\"edge_mode\": $edge, \"ctl_prefetch\": $cp}" >> $out
    SYMMETRY_ENGINE_EDGE=$edge SYMMETRY_ENGINE_CTL_PREFETCH=$cp timeout -k 10 200 \
      python -u bench/kernels/bench_engine.py --tp ${TP:-8} >> $out 2>> gpurun_out/engine_ab.err || exit $?
    SYMMETRY_ENGINE_EDGE=$edge SYMMETRY_ENGINE_CTL_PREFETCH=$cp timeout -k 10 200 \
      python -u bench/tp_shard.py --tp ${TP:-8} --clients 10 --engine 1 2>> gpurun_out/engine_ab.err | grep '^{' >> $out || exit $?
  done
done
cat $out
